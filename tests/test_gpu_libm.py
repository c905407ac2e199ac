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


def _device(which, x, out_words, out_dtype):
    import torch
    from procgen_amd import _lib
    lib = _lib.load()
    dx = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    dout = torch.zeros(out_words, dtype=out_dtype, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    n = x.size if which != 2 else x.size // 2
    assert lib.procgen_selftest_libm(which, dx.data_ptr(), dout.data_ptr(), n, stream) == 0
    torch.cuda.synchronize()
    return dout.cpu().numpy()


def game_rotations():
    """Entity rotations the games draw at: accumulated vrot sums (Entity::step, entity.cpp:63) of
    dodgeball's balls (PI * 0.23f for 50 steps) and dust clouds (PI / 0.3f), plus a broad sample of
    float angles (continuous steering games)."""
    pi = np.float32(3.14159265358979323846264338327950288)
    out = []
    for vrot in (pi * np.float32(0.23), pi / np.float32(0.3)):
        r = np.float32(0)
        for _ in range(64):
            r = np.float32(r + vrot)
            out.append(r)
    rng = np.random.RandomState(0)
    out = np.concatenate([np.array(out, np.float32), rng.uniform(-60, 60, 2_000_000).astype(np.float32),
                          rng.uniform(-7, 7, 2_000_000).astype(np.float32)])
    return out


def test_qt_rotation_matrix_matches_c_library():
    """QTransform::rotate's sin / cos (draw_image, basic-abstract-game.cpp:912-913) on the device vs
    glibc.  Render-only transcendental (pixel-tolerance class).  The device
    rounds correctly (pg_sincos.h); glibc 2.35 does not in ~0.15% of these arguments, so entries
    may differ by 1 ulp there -- never more (the pixels quantise the matrix; the parity tests
    observe bit-exact frames)."""
    import torch
    x = game_rotations()
    ref = np.empty(4 * x.size, np.float64)
    oracle_lib.load().oracle_qt_rotation(x.ctypes.data, ref.ctypes.data, x.size)
    got = _device(1, x, 4 * x.size, torch.float64)
    ulps = np.abs(got.view(np.int64) - ref.view(np.int64))
    assert ulps.max() <= 1, "rotation matrix differs by %d ulp" % ulps.max()
    frac = np.count_nonzero(ulps) / ulps.size
    print("qt rotation: %d of %d matrix entries differ by 1 ulp (%.2e)" % (np.count_nonzero(ulps), ulps.size, frac))
    assert frac < 5e-3


def test_face_rotation_matches_c_library():
    """Entity::face_direction = -atan2f(dy, dx) (entity.cpp:84-88): the device runs the restated glibc
    atan2f (pg_libm.h), bit-identical for any direction."""
    import torch
    vals = np.array([-1, 0, 1, -0.05, 0.05, -0.075, 0.075, 2.5, -3.0, -0.0], np.float32)
    rng = np.random.RandomState(5)
    dxy = np.concatenate([np.array([(a, b) for a in vals for b in vals if a != 0 or b != 0], np.float32).reshape(-1),
                          rng.uniform(-20, 20, 2_000_000).astype(np.float32)])
    ref = np.empty(dxy.size // 2, np.float32)
    oracle_lib.load().oracle_face_rotation(dxy.ctypes.data, ref.ctypes.data, ref.size)
    got = _device(2, dxy, ref.size, torch.float32)
    pairs = dxy.reshape(-1, 2)
    bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0]
    assert bad.size == 0, "face_direction differs for %r: %r vs %r" % (pairs[bad[:4]], got[bad[:4]], ref[bad[:4]])
