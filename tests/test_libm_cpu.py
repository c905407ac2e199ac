"""CPU pins of the engine's C-library math (procgen-1_amd/csrc/pg_libm.h, the same source the HIP
kernels compile): atan2f bit-identical to glibc's (what the reference links); double sin / cos
correctly rounded against 200-bit mpmath and within 1 ulp of glibc with the disagreement rate
bounded.  The .so built here is test infrastructure (gcc, host), never the product."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "procgen-1_amd", "csrc", "pg_libm.h")


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("sincos")
    src = d / "s.c"
    src.write_text('#include "%s"\n#include <stdint.h>\n'
                   "void run(const double *x, double *s, double *c, int64_t n) {"
                   " for (int64_t i = 0; i < n; i++) pg_sincos_cr(x[i], &s[i], &c[i]); }\n"
                   "void glibc(const double *x, double *s, double *c, int64_t n) {"
                   " for (int64_t i = 0; i < n; i++) { s[i] = sin(x[i]); c[i] = cos(x[i]); } }\n"
                   "void a2(const float *y, const float *x, float *o, int64_t n) {"
                   " for (int64_t i = 0; i < n; i++) o[i] = pg_atan2f(y[i], x[i]); }\n"
                   "void a2g(const float *y, const float *x, float *o, int64_t n) {"
                   " for (int64_t i = 0; i < n; i++) o[i] = atan2f(y[i], x[i]); }\n" % HDR)
    so = d / "s.so"
    subprocess.run(["gcc", "-O2", "-march=x86-64", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so), str(src),
                    "-lm"], check=True)
    L = ctypes.CDLL(str(so))
    for f in (L.run, L.glibc, L.a2, L.a2g):
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


def test_atan2f_bit_identical_to_glibc(lib):
    rng = np.random.RandomState(2)
    n = 4_000_000
    y = (rng.uniform(-30, 30, n) * np.where(rng.rand(n) < 0.3, 1e-3, 1)).astype(np.float32)
    x = rng.uniform(-30, 30, n).astype(np.float32)
    special = np.array([0.0, -0.0, 1.0, -1.0, 0.05, -0.05, 3.0, -2.5, 1e-30, -1e-30, 1e30, -1e30, 0.8, -0.8,
                        -6.99e-8], np.float32)
    yy, xx = np.meshgrid(special, special)
    y = np.concatenate([y, yy.ravel()])
    x = np.concatenate([x, xx.ravel(), ])
    a = np.empty_like(y)
    g = np.empty_like(y)
    lib.a2(y.ctypes.data, x.ctypes.data, a.ctypes.data, y.size)
    lib.a2g(y.ctypes.data, x.ctypes.data, g.ctypes.data, y.size)
    bad = np.nonzero(a.view(np.uint32) != g.view(np.uint32))[0]
    assert bad.size == 0, (y[bad[:4]], x[bad[:4]], a[bad[:4]], g[bad[:4]])
