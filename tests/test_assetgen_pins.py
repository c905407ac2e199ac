"""AssetGen pins -- CPU only (`use_generated_assets`).

The oracle's restatement of AssetGen (oracle/procgen_oracle.c, ag_*: assetgen.cpp:3-195 and the
Qt 5.9 raster paths it paints with) against the REFERENCE's own assetgen.cpp + randgen.cpp compiled
with the real Qt 5.9.7 of this image (oracle/ref_qt_harness.cpp -> oracle/_ref/libref_qt.so, built
by `make -C oracle ref` in the build container, where /root/reference exists; the library is
absent on the GPU box (oracle/_ref/ is listed in .gpurunignore), and these tests skip wherever it
was not built):

* whole generated images, bit for bit, plus the generator's position after painting (the next
  randint() must agree): 64x64 ARGB32 sprites (basic-abstract-game.cpp:101-107) in both the
  rect-resource and the shape-resource mode over 200 seeds;
* the primitives one by one: fillRect(QRectF) (opaque, alpha 200 SourceOver, transparent Source),
  drawEllipse(QRectF) with a brush (QRasterizer fill of the flattened outline), with a 1-px pen
  (QCosmeticStroker), on canvases of 64x64 and 500x500, RGB32 and ARGB32;
* 500x500 RGB32 backgrounds (basic-abstract-game.cpp:778-782), 200 cases;
* the cosmetic stroker alone on random closed polylines (every dropout / duplicate / reversal-cap
  rule the ellipse outline exercises).

Every comparison is bit-exact equality.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle_lib

REF_QT = os.path.join(os.path.dirname(oracle_lib.REF_SO), "libref_qt.so")
I, U, D, P, I32 = ctypes.c_int, ctypes.c_uint32, ctypes.c_double, ctypes.c_void_p, ctypes.c_int32
RGB32, ARGB32 = 4, 5


def libs():
    if not os.path.exists(REF_QT):
        pytest.skip("oracle/_ref/libref_qt.so not built (needs /root/reference and Qt at build time)")
    ref = ctypes.CDLL(REF_QT)
    ref.ref_generate_resource.restype = I32
    ref.ref_generate_resource.argtypes = [I32, I, I, I, I, I, I, I, U, P]
    ref.ref_qt_shape.argtypes = [I, I, I, I, D, D, D, D, U, U, I, P]
    ref.ref_qt_polyline.argtypes = [I, I, P, I, U, P]
    orc = oracle_lib.load()
    orc.oracle_generate_resource.argtypes = [I32, I, I, I, I, I, I, I, U, P, P]
    orc.oracle_qt_shape.argtypes = [I, I, I, I, D, D, D, D, U, U, I, P]
    orc.oracle_qt_polyline.argtypes = [I, I, P, I, U, P]
    return ref, orc


def generate(ref, orc, seed, pre, w, h, fmt, num_recurse, blotch_scale, is_rect):
    a = np.zeros((h, w), np.uint32)
    b = np.zeros((h, w), np.uint32)
    nxt = np.zeros(1, np.int32)
    ra = ref.ref_generate_resource(seed, pre, w, h, fmt, num_recurse, blotch_scale, is_rect, 0, a.ctypes.data)
    rc = orc.oracle_generate_resource(seed, pre, w, h, fmt, num_recurse, blotch_scale, is_rect, 0, b.ctypes.data,
                                      nxt.ctypes.data)
    assert rc == 0, "an integral ellipse rect (Qt's midpoint path) was met"
    return a, b, int(ra), int(nxt[0])


@pytest.mark.parametrize("is_rect", [1, 0])
def test_generated_sprites(is_rect):
    """64x64 ARGB32 sprites: AssetGen pgen(&asset_rand_gen); asset_rand_gen.seed(fixed_asset_seed +
    type); generate_resource(asset, 0, 5, use_block_asset(type)) -- 400 seeds, every pixel, and the
    generator position after painting."""
    ref, orc = libs()
    bad = []
    for k in range(400):
        seed = (k * 2654435761) % (1 << 32) - (1 << 31)
        a, b, ra, rb = generate(ref, orc, seed, 0, 64, 64, ARGB32, 0, 5, is_rect)
        assert ra == rb, "generator position differs after painting (seed %d)" % seed
        if not np.array_equal(a, b):
            bad.append((seed, int((a != b).sum())))
    assert not bad, "sprites differ (seed, pixels): %r" % bad[:10]


def _fnv(name):
    h = 0x811c9dc5
    for c in name.encode():
        h = ((h ^ c) * 0x1000193) & 0xffffffff
    return h


def test_game_sprite_seeds():
    """The seeds the games actually use: fixed_asset_seed = FNV-1a(env name) (vecgame.cpp:156-167,
    370-375) + type, types 0..79, both modes: all 2,560 images bit-exact."""
    ref, orc = libs()
    games = ("bigfish bossfight caveflyer chaser climber coinrun dodgeball fruitbot heist jumper leaper maze "
             "miner ninja plunder starpilot").split()
    bad = []
    for g in games:
        for t in range(80):
            seed = ((_fnv(g) + t) % (1 << 32)) - (1 << 31) if (_fnv(g) + t) % (1 << 32) >= (1 << 31) else (_fnv(g) + t) % (1 << 32)
            for is_rect in (0, 1):
                a, b, ra, rb = generate(ref, orc, seed, 0, 64, 64, ARGB32, 0, 5, is_rect)
                assert ra == rb
                if not np.array_equal(a, b):
                    bad.append((g, t, is_rect, int((a != b).sum())))
    assert not bad, bad


def test_generated_backgrounds():
    """500x500 RGB32 backgrounds: generate_resource(bg, 1, 50, true) after the reset's own draws."""
    ref, orc = libs()
    bad = []
    for k in range(200):
        a, b, ra, rb = generate(ref, orc, 7919 * k - 12345, k % 13, 500, 500, RGB32, 1, 50, 1)
        assert ra == rb, "generator position differs after painting (case %d)" % k
        if not np.array_equal(a, b):
            bad.append((k, int((a != b).sum())))
    assert not bad, "backgrounds differ (case, pixels): %r" % bad


def _random_rects(rng, n, W, H, maxsz):
    for _ in range(n):
        w = rng.uniform(0.2, maxsz)
        h = rng.uniform(0.2, maxsz)
        if rng.rand() < 0.2:
            h = rng.uniform(0.2, 3)
        x = rng.uniform(-0.3, W - w + 0.3) if W - w > 0 else 0.0
        y = rng.uniform(-0.3, H - h + 0.3) if H - h > 0 else 0.0
        if rng.rand() < 0.2:
            x, w = 0.0, float(W)  # create_bar's full-width bars touch both borders
        yield x, y, w, h


@pytest.mark.parametrize("kind,fmt,source", [(0, RGB32, 0), (0, ARGB32, 1), (2, RGB32, 0), (2, ARGB32, 1),
                                             (3, RGB32, 0), (1, ARGB32, 0)])
def test_qt_primitives(kind, fmt, source):
    """fillRect / drawEllipse brush / pen / both on 64x64 and 500x500 canvases (opaque colours over a
    non-trivial destination; kind 0 also with the alpha-200 colour of paint_rect_resource's veil)."""
    ref, orc = libs()
    rng = np.random.RandomState(100 + kind * 10 + fmt + source)
    for W, n, maxsz in ((64, 500, 64), (500, 60, 250)):
        for i, (x, y, w, h) in enumerate(_random_rects(rng, n, W, W, maxsz)):
            init = rng.randint(0, 1 << 24, size=(W, W)).astype(np.uint32) | np.uint32(0xff000000)
            c1 = 0xff000000 | int(rng.randint(0, 1 << 24))
            if kind == 0 and i % 3 == 1:
                c1 = (c1 & 0xffffff) | (200 << 24)
            if kind == 0 and source and i % 3 == 2:
                c1 = 0  # paint_shape_resource's transparent clear
            c2 = 0xff000000 | int(rng.randint(0, 1 << 24))
            a, b = init.copy(), init.copy()
            ref.ref_qt_shape(W, W, fmt, kind, x, y, w, h, c1, c2, source, a.ctypes.data)
            assert orc.oracle_qt_shape(W, W, fmt, kind, x, y, w, h, c1, c2, source, b.ctypes.data) == 0
            np.testing.assert_array_equal(b, a, err_msg="kind %d rect (%r, %r, %r, %r) on %d px" % (kind, x, y, w, h, W))


def test_cosmetic_stroker_closed_polylines():
    """The stroker's per-segment rules on closed polylines (caps off, reversal caps and their
    round-back, duplicate and dropout control, segments that cover no pixel centre) -- the rules the
    ellipse outline exercises -- bit-exact on 4,000 random closed polylines."""
    ref, orc = libs()
    rng = np.random.RandomState(11)
    W, n, bad = 40, 4000, 0
    for t in range(n):
        p = [rng.uniform(14, 26, 2)]
        for _ in range(rng.randint(2, 5)):
            p.append(p[-1] + rng.uniform(-4, 4, 2))
        p.append(p[0])
        pts = np.ascontiguousarray(np.array(p, np.float64).ravel())
        a = np.zeros((W, W), np.uint32)
        b = a.copy()
        ref.ref_qt_polyline(W, W, pts.ctypes.data, len(p), 0xff335577, a.ctypes.data)
        orc.oracle_qt_polyline(W, W, pts.ctypes.data, len(p), 0xff335577, b.ctypes.data)
        bad += not np.array_equal(a, b)
    assert bad == 0, "%d of %d closed polylines differ" % (bad, n)
