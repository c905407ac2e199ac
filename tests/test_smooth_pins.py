"""Pins of the oracle's render_mode="rgb_array" primitives -- CPU only.

The 512x512 frame (vecgame.cpp:318-330, 415-423 -> Game::render_to_buf with antialias = true,
game.cpp:97-107) is painted with QPainter::Antialiasing + SmoothPixmapTransform.  The oracle
restates the two primitives the supported games paint with (oracle/procgen_oracle.c qt_smooth_*):
drawImage(QRectF, QImage) -- antialiased rect coverage + bilinear fetch -- and fillRect(QRectF, QColor).
Both are checked here against the REAL Qt 5.9.7 raster engine of this image through
tools/qt_smooth_probe.cpp (oracle/_ref/libqt_probe.so, built by `make -C oracle ref`; absent on the
GPU box, where these tests skip): random rects on 64- and 512-px canvases, up- and downscaling,
clipped at every border, premultiplied sprites with transparent texels, mirrored images, opacity,
RGB32 backgrounds -- bit-exact.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle_lib

PROBE = os.path.join(os.path.dirname(oracle_lib.REF_SO), "libqt_probe.so")
D, I, P, U = ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32


def libs():
    if not os.path.exists(PROBE):
        pytest.skip("oracle/_ref/libqt_probe.so not built (needs Qt at build time)")
    q = ctypes.CDLL(PROBE)
    q.qtp_draw.argtypes = [I, I, P, I, P, I, I, I, I, D, D, D, D, D, D, U, I, I]
    q.qtp_prim.argtypes = [I, I, P, I, D, D, D, D, U, I]
    o = oracle_lib.load()
    o.oracle_qt_smooth.argtypes = [I, I, P, I, P, I, I, I, I, D, D, D, D, D, U]
    o.oracle_qt_smooth_rot.argtypes = [I, I, P, P, I, I, I, I, D, D, D, D, D, D]
    o.oracle_qt_prim.argtypes = [I, I, P, I, D, D, D, D, U, I]
    return q, o


def both(q, o, canvas, kind, img, fmt, mir, x, y, w, h, op=1.0, argb=0):
    a = np.ascontiguousarray(canvas.copy())
    b = np.ascontiguousarray(canvas.copy())
    im = np.ascontiguousarray(img if img is not None else np.zeros((1, 1), np.uint32))
    q.qtp_draw(a.shape[1], a.shape[0], a.ctypes.data, kind, im.ctypes.data, im.shape[1], im.shape[0], fmt, mir,
               x, y, w, h, 0.0, op, argb, 1, 1)
    o.oracle_qt_smooth(b.shape[1], b.shape[0], b.ctypes.data, kind, im.ctypes.data, im.shape[1], im.shape[0], fmt,
                       mir, x, y, w, h, op, argb)
    return a, b


def _canvas(rng, W):
    return rng.randint(0, 1 << 24, (W, W)).astype(np.uint32) | np.uint32(0xff000000)


@pytest.mark.parametrize("W", [64, 512])
def test_smooth_fill_rect(W):
    """fillRect(QRectF, opaque colour) under Antialiasing: thin, sub-pixel, clipped and large rects."""
    q, o = libs()
    rng = np.random.RandomState(W)
    for k in range(600 if W == 64 else 150):
        x, y = rng.uniform(-W * 0.3, W * 0.95, 2)
        w, h = rng.uniform(0.05, W * 0.6, 2)
        if k % 3 == 0:
            w, h = rng.uniform(0.02, 2.5, 2)
        if k % 11 == 0:
            x, y, w, h = 0.0, 0.0, float(W), float(W)  # the black background fill
        col = 0xff000000 | int(rng.randint(0, 1 << 24))
        a, b = both(q, o, _canvas(rng, W), 1, None, 6, 0, x, y, w, h, argb=col)
        np.testing.assert_array_equal(b, a, err_msg="fill (%r, %r, %r, %r) on %d px" % (x, y, w, h, W))


@pytest.mark.parametrize("W", [64, 512])
def test_smooth_draw_image(W):
    """drawImage(QRectF, QImage) with SmoothPixmapTransform + Antialiasing: every fetch helper
    (simple upscale, > 8x vertical upscale, 4-bit SSE2 downscale groups + 8-bit tail), the 256-span
    buffer flushes, clamped edges, transparent texels, mirrored images, opacity, RGB32 sources."""
    q, o = libs()
    rng = np.random.RandomState(100 + W)
    for k in range(160 if W == 64 else 60):
        iw, ih = rng.randint(2, 150, 2)
        img = rng.randint(0, 1 << 24, (ih, iw)).astype(np.uint32) | np.uint32(0xff000000)
        fmt = 6
        if k % 3 == 0:
            img[rng.rand(ih, iw) < 0.4] = 0  # premultiplied sprite with transparent texels
        op = 1.0
        if k % 5 == 0:
            fmt = 4  # RGB32 background
        elif k % 7 == 0:
            op = float(rng.choice([0.5, 0.25, 0.7, 0.3]))
        mir = int(k % 4 == 1)
        x, y = rng.uniform(-W * 0.2, W * 0.95, 2)
        w, h = rng.uniform(1, W * 0.5, 2)
        if k % 9 == 0:
            h = w * rng.uniform(9, 14)  # > 8x vertical upscale helper
        if k % 13 == 0:
            w, h = float(iw), float(ih)  # not stretched: the untransformed texture fill
        a, b = both(q, o, _canvas(rng, W), 0, img, fmt, mir, x, y, w, h, op=op)
        np.testing.assert_array_equal(b, a, err_msg="image %dx%d fmt %d mir %d op %r at (%r, %r, %r, %r) on %d px"
                                      % (iw, ih, fmt, mir, op, x, y, w, h, W))


@pytest.mark.parametrize("W", [64, 512])
def test_smooth_draw_image_rotated(W):
    """translate(center); rotate(deg); drawImage(QRectF(-w/2, -h/2, w, h)) (basic-abstract-game.cpp:908-916)
    with SmoothPixmapTransform + Antialiasing: QRasterizer::rasterizeLine's general branch (corners on
    the 26.6 grid, the four edge slopes, intersectPixelFP), its near-horizontal / near-vertical
    branches (angles within a 64th of a pixel of 0 / 90 / 180 degrees), the rotate fetch helpers (4-bit
    SSE2 groups, 8-bit lead-in / tail, 8-bit positions beyond an 8x zoom), QTransform's fuzzy type
    (rotate(-180) is a scale), clipped at every border, transparent texels, mirroring, opacity."""
    q, o = libs()
    rng = np.random.RandomState(300 + W)
    for k in range(300 if W == 64 else 80):
        iw, ih = rng.randint(2, 150, 2)
        img = rng.randint(0, 1 << 24, (ih, iw)).astype(np.uint32) | np.uint32(0xff000000)
        if k % 3 == 0:
            img[rng.rand(ih, iw) < 0.4] = 0
        op = float(rng.choice([0.5, 0.25, 0.7])) if k % 7 == 0 else 1.0
        mir = int(k % 4 == 1)
        x, y = rng.uniform(-W * 0.2, W * 0.95, 2)
        w, h = rng.uniform(0.5, W * 0.5, 2)
        if k % 5 == 0:
            w = h  # square sprites
        if k % 11 == 0:
            w, h = rng.uniform(0.5, 4, 2) * (iw / 8.0, ih / 8.0)  # > 8x zoom: 8-bit positions
        deg = float(rng.uniform(-360, 360))
        if k % 6 == 0:
            deg = float(rng.choice([90, -90, 180, -180, 270, 0.01, -0.02, 179.99, 90.005, 45, -45]))
        a = _canvas(rng, W)
        b = a.copy()
        q.qtp_draw(W, W, a.ctypes.data, 2, img.ctypes.data, iw, ih, 6, mir, x, y, w, h, deg, op, 0, 1, 1)
        o.oracle_qt_smooth_rot(W, W, b.ctypes.data, img.ctypes.data, iw, ih, 6, mir, x, y, w, h, deg, op)
        np.testing.assert_array_equal(b, a, err_msg="image %dx%d mir %d op %r at (%r, %r, %r, %r) deg %r on %d px"
                                      % (iw, ih, mir, op, x, y, w, h, deg, W))


@pytest.mark.parametrize("kind", [10, 11, 12, 13, 14])
def test_compass_primitives(kind):
    """jumper's compass primitives (jumper.cpp:137-177) under Antialiasing on a 512 canvas against the
    real Qt: drawEllipse(QRectF) brush + 1-px pen (10), pen only (13), brush only (14) -- the gray
    raster fill of the flattened outline and the antialiased cosmetic stroker; the translucent
    drawEllipse(QRect) (12); drawLine(QLine) with a wide square-capped pen (11)."""
    q, o = libs()
    W = 512
    rng = np.random.RandomState(700 + kind)
    for k in range(250):
        c = _canvas(rng, W)
        a, b = c.copy(), c.copy()
        penw = 1
        if kind == 11:
            x, y = rng.randint(-20, W + 20, 2)
            x2, y2 = x + rng.randint(-120, 121), y + rng.randint(-120, 121)
            if k % 7 == 0:
                x2 = x  # vertical / horizontal needles
            if k % 11 == 0:
                y2 = y
            args = (float(x), float(y), float(x2), float(y2))
            penw = int(rng.choice([2, 3, 4, 5, 6, 8]))
        else:
            x, y = rng.uniform(-40, W + 10, 2)
            w, h = rng.uniform(0.5, 160, 2)
            if k % 3 == 0:
                w = h  # the compass dial is round
            if k % 17 == 0:
                w, h = rng.uniform(0.3, 3, 2)  # tiny
            args = (x, y, w, h)
        col = 0x78ffffff if kind == 12 else 0xff000000 | int(rng.randint(0, 1 << 24))
        q.qtp_prim(W, W, a.ctypes.data, kind, *args, col, penw)
        o.oracle_qt_prim(W, W, b.ctypes.data, kind, *args, col, penw)
        np.testing.assert_array_equal(b, a, err_msg="kind %d case %d args %r pen %d" % (kind, k, args, penw))


def replay(q, log, res):
    """The oracle's logged painter commands of one frame through the real Qt, on one canvas."""
    canvas = np.zeros((res, res), np.uint32) | np.uint32(0xff000000)
    for row in log:
        kind = int(row[0])
        x, y, w, h = (float(v) for v in row[1:5])
        if kind == 1:
            canvas = _draw(q, canvas, 1, None, 6, 0, x, y, w, h, 1.0, int(row[5]))
        elif kind >= 10:  # jumper's compass primitives (qtp_prim)
            canvas = np.ascontiguousarray(canvas)
            q.qtp_prim(res, res, canvas.ctypes.data, kind, x, y, w, h, int(row[5]), int(row[6]))
        else:  # 0: drawImage(QRectF); 2: translate(rect centre); rotate(row[9] degrees); drawImage
            ptr, dims, fm, op = int(row[5]), int(row[6]), int(row[7]), float(row[8])
            iw, ih = dims >> 16, dims & 0xffff
            img = np.ctypeslib.as_array((ctypes.c_uint32 * (iw * ih)).from_address(ptr)).reshape(ih, iw).copy()
            canvas = _draw(q, canvas, kind, img, fm >> 1, fm & 1, x, y, w, h, op, 0, float(row[9]))
    return canvas


def _draw(q, canvas, kind, img, fmt, mir, x, y, w, h, op, argb, deg=0.0):
    a = np.ascontiguousarray(canvas)
    im = np.ascontiguousarray(img if img is not None else np.zeros((1, 1), np.uint32))
    q.qtp_draw(a.shape[1], a.shape[0], a.ctypes.data, kind, im.ctypes.data, im.shape[1], im.shape[0], fmt, mir,
               x, y, w, h, deg, op, argb, 1, 1)
    return a


ALL_GAMES = ["coinrun", "bigfish", "maze", "miner", "chaser", "climber", "ninja", "bossfight", "caveflyer", "dodgeball",
             "fruitbot", "heist", "jumper", "leaper", "plunder", "starpilot"]


@pytest.mark.parametrize("game", ALL_GAMES)
def test_rgb_array_frames_replayed_through_qt(game):
    """Whole 512x512 rgb_array frames: the oracle paints the frame of a running env and logs every
    painter call (background fill + image, grid tiles, entities, overlays); the same calls replayed
    through the real Qt with Antialiasing + SmoothPixmapTransform give the same pixels."""
    q, _ = libs()
    orc = oracle_lib.OracleEnv(game, 1, num_levels=0, rand_seed=3, paint_vel_info=1)
    rng = np.random.RandomState(4)
    for t in range(40):
        orc.step(rng.randint(0, 15, 1).astype(np.int32))
        if t % 13 != 12:
            continue
        rgb, log = orc.render_rgb_array(512, log_cap=20000)
        assert len(log) > 3
        qt_frame = replay(q, log, 512)
        ref = np.stack([(qt_frame >> 16) & 255, (qt_frame >> 8) & 255, qt_frame & 255], -1).astype(np.uint8)
        np.testing.assert_array_equal(rgb[0], ref, err_msg="%s step %d" % (game, t))


@pytest.mark.parametrize("opts", [{}, {"distribution_mode": 0}, {"center_agent": 0}])
def test_rgb_array_jumper_compass_frames(opts):
    """jumper's compass at 512 (dial ellipse, wide needle, distance bar, the translucent jump
    ellipse while falling) in whole replayed frames, hard / easy mode and the uncentered view."""
    q, _ = libs()
    orc = oracle_lib.OracleEnv("jumper", 1, num_levels=0, rand_seed=5, **opts)
    rng = np.random.RandomState(6)
    kinds = set()
    for t in range(240):
        # up for 3 steps, then run or wait for 3: a mid-air second jump draws the jump ellipse
        act = 5 if (t // 3) % 2 == 0 else int(rng.choice([1, 4, 7]))
        orc.step(np.array([act], np.int32))
        if t % 12 != 0 or t == 0:
            continue
        rgb, log = orc.render_rgb_array(512, log_cap=20000)
        kinds |= {int(r[0]) for r in log}
        qt_frame = replay(q, log, 512)
        ref = np.stack([(qt_frame >> 16) & 255, (qt_frame >> 8) & 255, qt_frame & 255], -1).astype(np.uint8)
        np.testing.assert_array_equal(rgb[0], ref, err_msg="jumper %r step %d" % (opts, t))
    assert {10, 11, 12}.issubset(kinds), kinds
