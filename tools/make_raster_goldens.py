#!/usr/bin/env python3
"""Generate tests/golden/qt_raster_goldens.npz with the REAL Qt 5.9.7 raster engine.

Build container only (needs /opt/conda Qt).  Each case = a 64x64 RGB32 canvas and a
list of painter commands (drawImage(QRectF, QImage) with optional setOpacity and
mirroring, fillRect); tools/qt_raster_golden.cpp replays them through QPainter and
returns the canvas.  The oracle's qt_* restatement must reproduce every canvas
bit-for-bit (tests/test_oracle_qt_raster.py).

Images come either from a synthetic pixel pool stored in the fixture or from the
committed coinrun asset atlas (referenced by slot, not copied).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from procgen_amd.assets import atlas_for  # noqa: E402
from golden_io import CMD_DTYPE, encode_all  # noqa: E402

QT = "/opt/conda"
OUT = os.path.join(REPO, "tests", "golden", "qt_raster_goldens.npz")


def build_tool(out):
    subprocess.run(["g++", "-O2", "-fPIC", "-std=c++17", os.path.join(HERE, "qt_raster_golden.cpp"),
                    "-I%s/include/qt" % QT, "-I%s/include/qt/QtGui" % QT, "-I%s/include/qt/QtCore" % QT,
                    "-L%s/lib" % QT, "-lQt5Gui", "-lQt5Core", "-Wl,-rpath,%s/lib" % QT, "-o", out],
                   check=True)


def f32(v):
    return float(np.float32(v))


def main():
    rng = np.random.default_rng(12345)
    atlas = atlas_for("coinrun")
    synth = []
    synth_off = 0
    cmds = []
    canvases = []

    def synth_image(iw, ih, fmt):
        nonlocal synth_off
        a = rng.integers(0, 256, size=(ih, iw), dtype=np.uint32)
        a[rng.random((ih, iw)) < 0.3] = 255
        a[rng.random((ih, iw)) < 0.2] = 0
        if fmt == 4:
            a[:] = 255
        c = [np.minimum(rng.integers(0, 256, size=(ih, iw), dtype=np.uint32), a) for _ in range(3)]
        px = (a << 24) | (c[0] << 16) | (c[1] << 8) | c[2]
        synth.append(px.reshape(-1))
        off = synth_off
        synth_off += px.size
        return off

    def add(case, kind, x, y, w, h, opacity=1.0, mirrored=0, fmt=6, src=0, ref=0, iw=0, ih=0, color=0):
        cmds.append((case, kind, x, y, w, h, opacity, mirrored, fmt, src, ref, iw, ih, color))

    case = 0
    # ---- synthetic cases
    for _ in range(400):
        if rng.random() < 0.8:
            canvases.append(np.full(4096, 0xff000000, dtype=np.uint32))
        else:
            canvases.append((rng.integers(0, 2 ** 24, size=4096, dtype=np.uint32) | 0xff000000).astype(np.uint32))
        for _k in range(rng.integers(1, 6)):
            fmt = 6 if rng.random() < 0.85 else 4
            iw, ih = int(rng.integers(2, 24)), int(rng.integers(2, 24))
            off = synth_image(iw, ih, fmt)
            r = rng.random()
            if r < 0.15:  # integral size == image size (non-stretch path)
                x, y, w, h = float(rng.integers(-10, 60)), float(rng.integers(-10, 60)), float(iw), float(ih)
                if rng.random() < 0.5:
                    x += rng.random()
                    y += rng.random()
            elif r < 0.3:  # tiny targets
                x, y = rng.uniform(-5, 66), rng.uniform(-5, 66)
                w, h = rng.uniform(0.05, 2.5), rng.uniform(0.05, 2.5)
            else:
                x, y = rng.uniform(-30, 70), rng.uniform(-30, 70)
                w, h = rng.uniform(0.5, 90), rng.uniform(0.5, 90)
            op = [1.0, 1.0, 1.0, 0.5, 0.4, f32(0.32), f32(0.256), f32(0.2048), rng.random()][rng.integers(0, 9)]
            add(case, 0, x, y, w, h, op, int(rng.random() < 0.3), fmt, 0, off, iw, ih)
        case += 1

    # ---- coinrun-like cases: real atlas images at the engine's geometry
    unit = f32(64 / np.float32(13))
    slots = [i for i in range(1000) if atlas.sprites[i][1] > 0]
    for _ in range(300):
        canvases.append(np.full(4096, 0xff000000, dtype=np.uint32))
        # background with a random offset: adjust_rect(main_rect, QRectF(-offset_x, 0, ar, 1))
        bi = int(rng.integers(0, atlas.backgrounds.shape[0]))
        bw, bh = atlas.backgrounds[bi][1:3]
        cx, cy = f32(rng.uniform(0.5, 63.5)), f32(rng.uniform(0.5, 63.5))
        view_dim = f32(64.0 / unit)
        x_off = f32(unit * f32(cx - view_dim / 2))
        y_off = f32(unit * f32(cy - view_dim / 2))
        mx = f32(f32(0 * unit) - x_off)
        my = f32(f32(f32(view_dim - 64) * unit) + y_off)
        mw = f32(64 * unit)
        bg_ar = f32(np.float32(bw) / np.float32(bh))
        off_x = f32(np.float32(rng.random()) * f32(bg_ar - 1))
        add(case, 0, mx + mw * -off_x, my, mw * f32(bg_ar / 1.0), mw, 1.0, 0, 4, 2, bi)
        for _k in range(int(rng.integers(4, 40))):
            slot = int(slots[rng.integers(0, len(slots))])
            ex, ey = f32(rng.uniform(cx - 8, cx + 8)), f32(rng.uniform(cy - 8, cy + 8))
            kind = rng.random()
            if kind < 0.5:  # grid tile with RENDER_EPS
                gx, gy = float(np.floor(ex)), float(np.floor(ey))
                eps = np.float32(0.02)
                x = f32(f32(f32(np.float32(gx) - eps) * unit) - x_off)
                y = f32(f32(f32(f32(view_dim - np.float32(gy + 1)) - eps) * unit) + y_off)
                w = f32(f32(1 + 2 * eps) * unit)
                add(case, 0, x, y, w, w, 1.0, 0, 6, 1, slot)
            else:  # entity rect (player adjust_rect included sometimes)
                rx = f32(rng.choice([0.5, 0.3, 0.2, 0.35, 0.44]))
                ry = f32(rng.choice([0.5, 0.5787, 0.2, 0.21]))
                x = f32(f32(f32(ex - rx) * unit) - x_off)
                y = f32(f32(f32(view_dim - f32(ey + ry)) * unit) + y_off)
                w = f32(f32(2 * rx) * unit)
                h = f32(f32(2 * ry) * unit)
                if rng.random() < 0.3:
                    y, h = y + h * -.7415, h * 1.7415
                op = 1.0
                if rng.random() < 0.3:
                    op = float(np.float32(0.5) * np.float32(0.8) ** int(rng.integers(0, 9)))
                add(case, 0, x, y, w, h, op, int(rng.random() < 0.4), 6, 1, slot)
        case += 1

    cmds = np.array(cmds, dtype=CMD_DTYPE)
    synth = np.concatenate(synth).astype(np.uint32)
    canvas_in = np.stack(canvases).astype(np.uint32)
    stream = encode_all(canvas_in, cmds, synth, atlas)
    with tempfile.TemporaryDirectory() as td:
        tool = os.path.join(td, "qt_raster_golden")
        build_tool(tool)
        res = subprocess.run([tool], input=stream, stdout=subprocess.PIPE, check=True).stdout
    canvas_out = np.frombuffer(res, dtype="<u4").reshape(case, 4096)
    np.savez_compressed(OUT, cmds=cmds, synth=synth, canvas_in=canvas_in, canvas_out=canvas_out,
                        qt_version=np.array("5.9.7"))
    print("wrote", OUT, case, "cases", len(cmds), "commands", os.path.getsize(OUT) / 1e6, "MB")


if __name__ == "__main__":
    main()
