"""CPU pin of the engine's double sin / cos (procgen-1_amd/csrc/pg_sincos.h, the same source the
HIP kernels compile): correctly rounded against 200-bit mpmath, and within 1 ulp of glibc (what
the reference links) with the disagreement rate bounded.  The .so built here is test
infrastructure (gcc, host), never the product."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "procgen-1_amd", "csrc", "pg_sincos.h")


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("sincos")
    src = d / "s.c"
    src.write_text('#include "%s"\n#include <stdint.h>\n'
                   "void run(const double *x, double *s, double *c, int64_t n) {"
                   " for (int64_t i = 0; i < n; i++) pg_sincos_cr(x[i], &s[i], &c[i]); }\n"
                   "void glibc(const double *x, double *s, double *c, int64_t n) {"
                   " for (int64_t i = 0; i < n; i++) { s[i] = sin(x[i]); c[i] = cos(x[i]); } }\n" % HDR)
    so = d / "s.so"
    subprocess.run(["gcc", "-O2", "-march=x86-64", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so), str(src),
                    "-lm"], check=True)
    L = ctypes.CDLL(str(so))
    for f in (L.run, L.glibc):
        f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64]
    return L


def call(f, x):
    s = np.empty_like(x)
    c = np.empty_like(x)
    f(x.ctypes.data, s.ctypes.data, c.ctypes.data, x.size)
    return s, c


def test_correctly_rounded_vs_mpmath(lib):
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 200
    rng = np.random.RandomState(0)
    x = np.concatenate([rng.uniform(-8, 8, 3000), rng.uniform(-1200, 1200, 1000), [1e-9, -3e-5, 0.785398, 1.5707963,
                                                                                     3.14159265, 1e4]])
    s, c = call(lib.run, x)
    for i, v in enumerate(x):
        assert s[i] == float(mpmath.sin(mpmath.mpf(float(v)))), v
        assert c[i] == float(mpmath.cos(mpmath.mpf(float(v)))), v


def test_glibc_agreement(lib):
    pi = np.float32(3.14159265358979323846264338327950288)
    rng = np.random.RandomState(1)
    rot = rng.uniform(-60, 60, 1_000_000).astype(np.float32)
    deg = (rot * np.float32(180) / pi).astype(np.float32).astype(np.float64)
    x = 0.017453292519943295769 * deg
    s, c = call(lib.run, x)
    gs, gc = call(lib.glibc, x)
    for a, b in ((s, gs), (c, gc)):
        ulps = np.abs(a.view(np.int64) - b.view(np.int64))
        assert ulps.max() <= 1
        assert np.count_nonzero(ulps) / ulps.size < 5e-3
