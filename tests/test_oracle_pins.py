"""Pins of the CPU oracle (the parity checker) -- CPU only.

* MT19937 / RandGen draws: against the reference's own randgen.cpp compiled from
  /root/reference (oracle/_ref, built by `make -C oracle ref`) and the C++ standard's
  known answer ([rand.predef]: the 10000th output of a default-seeded mt19937 is 4123659995).
* Entity::step: against the reference's entity.cpp (oracle/_ref).
* Qt raster compositing: against canvases produced by the real Qt 5.9.7 raster engine
  (tests/golden/qt_raster_goldens.npz, made by tools/make_raster_goldens.py).
* Oracle trajectories: regression fixture tests/golden/coinrun_oracle_traj.npz
  (tools/make_oracle_goldens.py).
"""
import ctypes
import os
import zlib

import numpy as np
import pytest

import oracle_lib
from golden_io import encode_cmds

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ref_lib():
    if not os.path.exists(oracle_lib.REF_SO):
        pytest.skip("oracle/_ref/libref.so not built (needs /root/reference at build time)")
    lib = ctypes.CDLL(oracle_lib.REF_SO)
    lib.ref_mt_stream.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int]
    lib.ref_randgen_script.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.ref_entity_steps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


def test_mt_known_answer():
    lib = oracle_lib.load()
    out = np.zeros(10000, np.uint32)
    lib.oracle_mt_stream(5489, out.ctypes.data, 10000)
    assert int(out[-1]) == 4123659995


@pytest.mark.parametrize("seed", [0, 1, 5489, 199, 2147483646, -1, -123456])
def test_mt_stream_vs_reference(seed):
    ref = ref_lib()
    lib = oracle_lib.load()
    n = 3000  # crosses several twists
    a = np.zeros(n, np.uint32)
    b = np.zeros(n, np.uint32)
    lib.oracle_mt_stream(seed & 0xFFFFFFFF, a.ctypes.data, n)
    ref.ref_mt_stream(seed, b.ctypes.data, n)
    np.testing.assert_array_equal(a, b)


def random_ops(rng, n):
    ops = np.zeros((n, 3), np.int32)
    for i in range(n):
        k = int(rng.integers(0, 6))
        if k == 0:
            lo = int(rng.integers(-1000, 1000))
            ops[i] = (0, lo, lo + int(rng.integers(1, 1 << 30)))
        elif k == 1:
            ops[i] = (1, int(rng.integers(1, 100000)), 0)
        elif k == 4:
            lo = int(rng.integers(-800, 800))
            ops[i] = (4, lo, lo + int(rng.integers(1, 800)))
        else:
            ops[i] = (k, 0, 0)
    return ops


@pytest.mark.parametrize("seed", [0, 7, 424242])
def test_randgen_helpers_vs_reference(seed):
    ref = ref_lib()
    lib = oracle_lib.load()
    rng = np.random.default_rng(seed)
    ops = random_ops(rng, 4000)
    a = np.zeros(len(ops), np.int32)
    b = np.zeros(len(ops), np.int32)
    lib.oracle_randgen_script(seed, ops.ctypes.data, len(ops), a.ctypes.data)
    ref.ref_randgen_script(seed, ops.ctypes.data, len(ops), b.ctypes.data)
    np.testing.assert_array_equal(a, b)


def oracle_entity_steps(init, etype, smart, friction, vrot, expire, steps):
    """Entity::step restated in numpy float32 with the oracle's operation order."""
    f = np.float32
    x, y, vx, vy, rx, ry = (f(v) for v in init)
    rot = f(0)
    alpha, grow, decay = f(1), f(1), f(1)
    life, erase, img = 0, 0, etype
    if etype == 54:
        grow = f(1.4)
        expire_t = 4
    else:
        expire_t = -1
    if etype == 59:
        grow, decay = f(1.05), f(0.8)
    if expire:
        expire_t = expire
    out = []
    for _ in range(steps):
        if not smart:
            x = f(x + vx)
            y = f(y + vy)
        rot = f(rot + f(vrot))
        vx = f(vx * f(friction))
        vy = f(vy * f(friction))
        life += 1
        if expire_t > 0 and life > expire_t:
            erase = 1
        if etype == 54 and img < 58:
            img += 1
        rx = f(rx * grow)
        ry = f(ry * grow)
        alpha = f(decay * alpha)
        words = np.array([x, y, vx, vy, rx, ry, rot, alpha], np.float32).view(np.uint32).tolist()
        out.append(words + [life, erase, img])
    return np.array(out, np.uint32)


@pytest.mark.parametrize("etype,smart,friction,vrot,expire", [
    (59, 0, 1.0, 0.0, 8), (54, 0, 1.0, 0.1, 0), (5, 1, 1.0, 0.0, 0), (2, 0, 0.9, 0.3, 0), (20, 0, 0.95, -0.2, 30)])
def test_entity_step_vs_reference(etype, smart, friction, vrot, expire):
    ref = ref_lib()
    init = np.array([10.5, 3.25, 0.15, 0.01, 0.3, 0.2], np.float32)
    steps = 40
    b = np.zeros((steps, 11), np.uint32)
    ref.ref_entity_steps(init.ctypes.data, etype, smart, friction, vrot, expire, steps, b.ctypes.data)
    a = oracle_entity_steps(init, etype, smart, friction, vrot, expire, steps)
    np.testing.assert_array_equal(a, b)


def test_qt_raster_goldens():
    """Every painter case replayed through the oracle's Qt restatement equals real Qt 5.9.7."""
    from procgen_amd.assets import atlas_for
    lib = oracle_lib.load()
    z = np.load(os.path.join(GOLDEN, "qt_raster_goldens.npz"), allow_pickle=False)
    cmds, synth, cin, cout = z["cmds"], z["synth"], z["canvas_in"], z["canvas_out"]
    atlas = atlas_for("coinrun")
    bad = []
    for i in range(cin.shape[0]):
        b = encode_cmds(cmds[cmds["case"] == i], synth, atlas)
        canvas = cin[i].copy()
        rc = lib.oracle_qt_replay(b, len(b), canvas.ctypes.data)
        assert rc == len(b)
        if not np.array_equal(canvas, cout[i]):
            bad.append(i)
    assert not bad, "Qt raster mismatch in cases %s" % bad[:10]


def test_qt_raster_rotation_goldens():
    """Rotated drawImage (translate + rotate + drawImage, basic-abstract-game.cpp:908-916) replayed
    through the oracle's qt_transform_image restatement equals real Qt 5.9.7
    (tests/golden/qt_raster_rot_goldens.npz, tools/make_raster_rot_goldens.py)."""
    from procgen_amd.assets import atlas_for
    lib = oracle_lib.load()
    z = np.load(os.path.join(GOLDEN, "qt_raster_rot_goldens.npz"), allow_pickle=False)
    cmds, synth, cin, cout = z["cmds"], z["synth"], z["canvas_in"], z["canvas_out"]
    atlas = atlas_for(str(z["atlas_game"]))
    bad = []
    for i in range(cin.shape[0]):
        b = encode_cmds(cmds[cmds["case"] == i], synth, atlas)
        canvas = cin[i].copy()
        rc = lib.oracle_qt_replay(b, len(b), canvas.ctypes.data)
        assert rc == len(b)
        if not np.array_equal(canvas, cout[i]):
            bad.append(i)
    assert not bad, "Qt rotated raster mismatch in %d cases, first %s" % (len(bad), bad[:10])


def test_oracle_trajectory_fixture():
    """Regression pin of the oracle itself (tests/golden/coinrun_oracle_traj.npz)."""
    path = os.path.join(GOLDEN, "coinrun_oracle_traj.npz")
    z = np.load(path, allow_pickle=False)
    envs = z["envs"]
    steps = int(z["steps"])
    orcs = [oracle_lib.OracleEnv("coinrun", 1, env_offset=int(e), num_levels=200, start_level=0, rand_seed=0)
            for e in envs]
    frames_at = list(z["frame_steps"])
    fi = 0
    for t in range(steps + 1):
        for k, (e, o) in enumerate(zip(envs, orcs)):
            if t:
                o.step(oracle_lib.hashed_actions(int(z["action_seed"]), [e], t))
            ob = o.observe()
            assert ob["rew"][0] == z["rew"][t, k]
            assert ob["first"][0] == z["first"][t, k]
            assert ob["level_seed"][0] == z["level_seed"][t, k]
            assert ob["prev_level_seed"][0] == z["prev_level_seed"][t, k]
            assert zlib.crc32(ob["rgb"][0].tobytes()) == z["rgb_crc32"][t, k], "crc at step %d env %d" % (t, e)
            if t in frames_at:
                np.testing.assert_array_equal(ob["rgb"][0], z["frames"][frames_at.index(t), k])
        fi += 1


MAZE_CASES = [(mode, dim, 0) for mode in (0, 1) for dim in (3, 5, 6, 7, 11, 13, 15, 25)] + \
             [(2, dim, doors) for dim in (5, 7, 9, 11, 13, 23) for doors in (0, 1, 2, 3)]


@pytest.mark.parametrize("mode,dim,doors", MAZE_CASES)
def test_mazegen_vs_reference(mode, dim, doors):
    """MazeGen (Kruskal, no-dead-ends, doors + BFS keys, place_objects) against the reference's own
    mazegen.cpp compiled from /root/reference (oracle/_ref), grid and next RNG draw bit-exact."""
    ref = ref_lib()
    ref.ref_mazegen.argtypes = [ctypes.c_int32, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p, ctypes.c_void_p]
    lib = oracle_lib.load()
    n = (dim + 2) ** 2
    for seed in range(40):
        objs = 1 if mode == 0 else 0
        a, b = np.zeros(n, np.int32), np.zeros(n, np.int32)
        da, db = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        ra = lib.oracle_mazegen(seed * 7919 + dim, dim, mode, doors, 2, objs, a.ctypes.data, da.ctypes.data)
        rb = ref.ref_mazegen(seed * 7919 + dim, dim, mode, doors, 2, objs, b.ctypes.data, db.ctypes.data)
        assert ra == rb == dim + 2
        np.testing.assert_array_equal(a, b, err_msg="seed %d" % seed)
        assert da[0] == db[0]


def test_argument_evaluation_order_pinned():
    """climber.cpp:196 draws two randn(2) inside one call's arguments; C++ leaves their order
    unspecified.  The oracle (and the engine) take g++'s order -- right to left, the vx draw
    first -- pinned here against that call compiled by g++ with the reference's RandGen."""
    ref = ref_lib()
    ref.ref_climber_enemy_args.argtypes = [ctypes.c_int32, ctypes.c_void_p]
    lib = oracle_lib.load()
    for seed in range(64):
        out = np.zeros(2, np.float32)
        ref.ref_climber_enemy_args(seed, out.ctypes.data)
        ops = np.array([[1, 2, 0], [1, 2, 0]], np.int32)  # two randn(2)
        draws = np.zeros(2, np.int32)
        lib.oracle_randgen_script(seed & 0xFFFFFFFF, ops.ctypes.data, 2, draws.ctypes.data)
        vdraw, ydraw = int(draws[0]), int(draws[1])
        assert out[0] == np.float32(0 + ydraw + 2 + .5)
        assert out[1] == np.float32(.15 * (vdraw * 2 - 1))


def test_leaper_operand_order_pinned():
    """leaper.cpp:155 multiplies rand_sign() by randrange(): g++ evaluates the left operand
    first (the sign's rand01 is the first draw); the oracle and engine follow that order."""
    ref = ref_lib()
    ref.ref_leaper_lane_speed.argtypes = [ctypes.c_int32, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
    lib = oracle_lib.load()
    for seed in range(256):
        out = np.zeros(1, np.float32)
        ref.ref_leaper_lane_speed(seed, 0.05, 0.2, out.ctypes.data)
        ops = np.array([[2, 0, 0], [2, 0, 0]], np.int32)
        draws = np.zeros(2, np.int32)
        lib.oracle_randgen_script(seed & 0xFFFFFFFF, ops.ctypes.data, 2, draws.ctypes.data)
        u = draws.view(np.float32)
        sign = np.float32(1.0) if u[0] < 0.5 else np.float32(-1.0)
        spd = np.float32(u[1] * np.float32(np.float32(0.2) - np.float32(0.05)) + np.float32(0.05))
        assert out[0] == sign * spd, seed


def test_caveflyer_operand_order_pinned():
    """caveflyer.cpp:235 multiplies (.1 * rand01() + .1) by (randn(2) * 2 - 1): g++ draws the left
    operand first; the oracle and engine follow that order."""
    ref = ref_lib()
    ref.ref_caveflyer_enemy_vel.argtypes = [ctypes.c_int32, ctypes.c_void_p]
    lib = oracle_lib.load()
    for seed in range(256):
        out = np.zeros(1, np.float32)
        ref.ref_caveflyer_enemy_vel(seed, out.ctypes.data)
        ops = np.array([[2, 0, 0], [1, 2, 0]], np.int32)  # rand01, randn(2)
        draws = np.zeros(2, np.int32)
        lib.oracle_randgen_script(seed & 0xFFFFFFFF, ops.ctypes.data, 2, draws.ctypes.data)
        u = float(draws[:1].view(np.float32)[0])
        want = np.float32((.1 * u + .1) * (int(draws[1]) * 2 - 1))
        assert out[0] == want, seed


def test_qt_raster_fill_goldens():
    """fillRect(QRectF, opaque QColor) (chaser orbs, bars, draw_grid_obj) replayed through the
    oracle's restatement equals real Qt 5.9.7 (tests/golden/qt_raster_fill_goldens.npz,
    tools/make_raster_fill_goldens.py)."""
    from procgen_amd.assets import atlas_for
    lib = oracle_lib.load()
    z = np.load(os.path.join(GOLDEN, "qt_raster_fill_goldens.npz"), allow_pickle=False)
    cmds, synth, cin, cout = z["cmds"], z["synth"], z["canvas_in"], z["canvas_out"]
    atlas = atlas_for("coinrun")
    bad = []
    for i in range(cin.shape[0]):
        b = encode_cmds(cmds[cmds["case"] == i], synth, atlas)
        canvas = cin[i].copy()
        rc = lib.oracle_qt_replay(b, len(b), canvas.ctypes.data)
        assert rc == len(b)
        if not np.array_equal(canvas, cout[i]):
            bad.append(i)
    assert not bad, "Qt fillRect mismatch in %d cases, first %s" % (len(bad), bad[:10])


def test_spawner_sort_vs_libstdcxx(tmp_path):
    """starpilot sorts its spawners with std::sort(spawn_cmp) (starpilot.cpp:28-30, 340); equal spawn
    times are common, so the order among them is libstdc++'s introsort's.  The oracle's restatement
    must leave the same permutation as the real std::sort of this toolchain (g++ / libstdc++, what
    the reference builds with)."""
    import subprocess
    src = tmp_path / "s.cpp"
    src.write_text(
        "#include <algorithm>\n#include <vector>\n#include <cstdint>\n"
        "struct E { int t, i; };\n"
        "extern \"C\" void cxx_sort(const int32_t *key, int32_t *idx, int n) {\n"
        "  std::vector<E> v; for (int i = 0; i < n; i++) v.push_back({key[i], i});\n"
        "  std::sort(v.begin(), v.end(), [](const E &x, const E &y) { return x.t > y.t; });\n"
        "  for (int i = 0; i < n; i++) idx[i] = v[i].i; }\n")
    so = tmp_path / "s.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", str(so), str(src)], check=True)
    cxx = ctypes.CDLL(str(so))
    cxx.cxx_sort.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib = oracle_lib.load()
    rng = np.random.RandomState(0)
    for trial in range(3000):
        n = int(rng.choice([0, 1, 2, 5, 16, 17, 33, 64, 100, 200, 300]))
        kind = trial % 4
        if kind == 0:
            key = rng.randint(0, 20, n)
        elif kind == 1:
            key = np.sort(rng.randint(0, 500, n))
        elif kind == 2:
            key = np.sort(rng.randint(0, 500, n))[::-1]
        else:  # starpilot-like: groups t + 5j with t increasing by 10..30
            ts, t = [], 1 + rng.randint(10, 30)
            while len(ts) < n:
                for j in range(rng.randint(0, 5) + 1):
                    ts.append(t + 5 * j)
                t += rng.randint(10, 30)
            key = np.array(ts[:n])
        key = np.ascontiguousarray(key, dtype=np.int32)
        a = np.zeros(n, np.int32)
        b = np.zeros(n, np.int32)
        lib.oracle_spawn_sort(key.ctypes.data, a.ctypes.data, n)
        cxx.cxx_sort(key.ctypes.data, b.ctypes.data, n)
        np.testing.assert_array_equal(a, b, err_msg="trial %d n %d kind %d" % (trial, n, kind))


def test_jumper_compass_table_pins():
    """jumper's compass overlay is stamped from Qt 5.9.7 raster output (tools/qt_compass_tables.cpp):
    the translucent jump ellipse's SourceOver blend equals premultiplied 0x78787878 + BYTE_MUL(dst, 135)
    on every pixel Qt changed, and the packed table words carry the per-configuration geometry."""
    from procgen_amd.assets import ASSET_DIR, compass_table_words
    z = np.load(os.path.join(ASSET_DIR, "jumper_compass.npz"), allow_pickle=False)
    bg, out = z["blend_bg"].astype(np.uint64), z["blend_out"].astype(np.uint64)

    def byte_mul(x, a):
        t = (x & 0xff00ff) * a
        t = ((t + ((t >> 8) & 0xff00ff) + 0x800080) >> 8) & 0xff00ff
        x = ((x >> 8) & 0xff00ff) * a
        x = (x + ((x >> 8) & 0xff00ff) + 0x800080) & 0xff00ff00
        return x | t

    changed = out != bg
    assert changed.sum() > 500
    pred = (0x78787878 + byte_mul(bg, 135)) & 0xffffffff
    np.testing.assert_array_equal(pred[changed], out[changed])
    w = compass_table_words()
    assert w[0] == 0x434D5053
    geom = z["cfg_geom"]
    for cfg in range(4):
        np.testing.assert_array_equal(w[5 + 9 * cfg:5 + 9 * cfg + 6].view(np.int32), geom[cfg])
    # hard mode, centred: the dial is Qt's midpoint ellipse of QRect(55, 1, 8, 8) with a 1-px pen
    dial = z["dial"][1]
    assert int(dial[1]) != 0 and int(dial[0]) == 0 and all(int(r) == 0 for r in dial[11:])


def test_grid_vs_reference():
    """grid.h: Grid<int>::resize value-initialises, contains / get / to_index / to_xy, and (fork
    buffer.h) serialize writes no bytes -- the oracle's Game grid (grid_contains, get_obj with the
    out-of-bounds object, y * w + x) against the reference's Grid compiled in oracle/_ref."""
    ref = ref_lib()
    orc = oracle_lib.load()
    P = ctypes.c_void_p
    ref.ref_grid_ops.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, P]
    orc.oracle_grid_ops.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P]
    rng = np.random.RandomState(5)
    for w, h in ((1, 1), (13, 13), (64, 64), (20, 35), (35, 20), (100, 7)):
        xy = np.stack([rng.randint(-3, w + 3, 400), rng.randint(-3, h + 3, 400)], 1).astype(np.int32)
        xy = np.ascontiguousarray(np.concatenate([xy, [[0, 0], [w - 1, h - 1], [w, 0], [0, h], [-1, 0]]]).astype(np.int32))
        a = np.zeros((len(xy), 5), np.int32)
        b = a.copy()
        nbytes = np.zeros(1, np.int32)
        za = ref.ref_grid_ops(w, h, xy.ctypes.data, len(xy), a.ctypes.data, nbytes.ctypes.data)
        zb = orc.oracle_grid_ops(w, h, xy.ctypes.data, len(xy), b.ctypes.data)
        assert za == zb == w * h
        assert int(nbytes[0]) == 0
        inside = a[:, 0] == 1
        np.testing.assert_array_equal(b[:, :2], a[:, :2])
        np.testing.assert_array_equal(b[:, 2], a[:, 2])
        # to_xy round trip: defined (and used by the games) for in-grid indices
        np.testing.assert_array_equal(b[inside, 3:], a[inside, 3:])


def test_qt_utils_vs_reference():
    """qt-utils.h: adjust_rect (QRectF arithmetic; coinrun.cpp:66, leaper.cpp:244 and the background
    rect, basic-abstract-game.cpp:1013) and to_shade (the velocity squares, :972-973), against the
    reference header compiled with the real Qt 5.9.7 (oracle/_ref/libref_qt.so)."""
    qt_so = os.path.join(os.path.dirname(oracle_lib.REF_SO), "libref_qt.so")
    if not os.path.exists(qt_so):
        pytest.skip("oracle/_ref/libref_qt.so not built")
    ref = ctypes.CDLL(qt_so)
    orc = oracle_lib.load()
    P, L = ctypes.c_void_p, ctypes.c_int64
    for lib, pre in ((ref, "ref"), (orc, "oracle")):
        getattr(lib, pre + "_adjust_rect").argtypes = [P, P, P, L]
        getattr(lib, pre + "_to_shade").argtypes = [P, P, L]
    rng = np.random.RandomState(9)
    n = 20000
    base = np.ascontiguousarray(rng.uniform(-100, 600, (n, 4)))
    adj = np.ascontiguousarray(rng.uniform(-2, 2, (n, 4)))
    adj[:4] = [[0, -.7415, 1, 1.7415], [0, -.275, 1, 1.55], [-0.3, 0, 1.7, 1], [0, 0, 1, 1]]
    a, b = np.zeros((n, 4)), np.zeros((n, 4))
    ref.ref_adjust_rect(base.ctypes.data, adj.ctypes.data, a.ctypes.data, n)
    orc.oracle_adjust_rect(base.ctypes.data, adj.ctypes.data, b.ctypes.data, n)
    np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))
    f = np.concatenate([rng.uniform(-0.5, 1.5, 200000), np.linspace(-0.01, 1.01, 100001),
                        [0.0, -0.0, 1.0, 1 / 255, 254.5 / 255, 255.5 / 255]]).astype(np.float32)
    f = np.ascontiguousarray(np.concatenate([f, np.nextafter(f, np.float32(2)), np.nextafter(f, np.float32(-2))]))
    sa, sb = np.zeros(len(f), np.int32), np.zeros(len(f), np.int32)
    ref.ref_to_shade(f.ctypes.data, sa.ctypes.data, len(f))
    orc.oracle_to_shade(f.ctypes.data, sb.ctypes.data, len(f))
    np.testing.assert_array_equal(sa, sb)
