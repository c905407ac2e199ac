"""Exhaustive check of the only libm call in the game logic built so far: bigfish's fish radius
(FISH_MAX_R - FISH_MIN_R) * pow(rand01(), 1.4) + FISH_MIN_R (bigfish.cpp:84), double pow,
narrowed to float.  rand01() = float(u / 2^32) (randgen.cpp:19-23) takes 2^24 + 2^26 + 1
distinct values: u * 2^-32 for u < 2^24, every float of [2^-8, 1), and 1.0.  The device
result (ROCm's pow) must equal the C library's (glibc, what the reference links) for every
one of them -- then bigfish's physics is bit-exact, not merely within a tolerance."""
import ctypes

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu


def all_rand01_values():
    small = (np.arange(1 << 24, dtype=np.float64) * 2.0 ** -32).astype(np.float32)
    lo = np.float32(2.0 ** -8).view(np.uint32)
    hi = np.float32(1.0).view(np.uint32)
    binades = np.arange(lo, hi, dtype=np.uint32).view(np.float32)
    return np.concatenate([small, binades, np.array([1.0], np.float32)])


def test_bigfish_radius_pow_matches_c_library_exhaustively():
    import torch
    from procgen_amd import _lib
    lib = _lib.load()
    x = all_rand01_values()
    assert x.size == (1 << 24) + (1 << 26) + 1
    ref = np.empty_like(x)
    oracle_lib.load().oracle_bigfish_radius(x.ctypes.data, ref.ctypes.data, x.size)
    dx = torch.from_numpy(x).cuda()
    dout = torch.empty_like(dx)
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.procgen_selftest_libm(0, dx.data_ptr(), dout.data_ptr(), x.size, stream) == 0
    torch.cuda.synchronize()
    got = dout.cpu().numpy()
    bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0]
    assert bad.size == 0, "%d of %d radii differ, first u=%r: device %r vs libm %r" % (
        bad.size, x.size, x[bad[:5]].tolist(), got[bad[:5]].tolist(), ref[bad[:5]].tolist())
