#!/usr/bin/env python3
"""Generate tests/golden/qt_raster_fill_goldens.npz: QPainter::fillRect(QRectF, QColor) with opaque
colours through the REAL Qt 5.9.7 raster engine (build container only, needs /opt/conda Qt).

The games fill fractional rectangles with opaque colours: chaser's orbs (chaser.cpp:111-117),
the ninja / plunder / jumper bars (ninja.cpp:166-175, plunder.cpp:66-77, jumper.cpp:159-161),
starpilot's backdrop (starpilot.cpp:110-112) and draw_grid_obj (basic-abstract-game.cpp:924-928).
Cases mix random geometry (fractions near .5, negative and off-canvas rects) with chaser-orb
geometry.  The oracle's qt_fill_rectf must reproduce every canvas (tests/test_oracle_pins.py).
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
sys.path.insert(0, HERE)
from procgen_amd.assets import atlas_for  # noqa: E402
from golden_io import CMD_DTYPE, encode_all  # noqa: E402
from make_raster_goldens import build_tool, f32  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "qt_raster_fill_goldens.npz")


def main():
    rng = np.random.default_rng(4242)
    cmds, canvases = [], []

    def add(case, x, y, w, h, color):
        cmds.append((case, 1, x, y, w, h, 1.0, 0, 0, 0, 0, 0, 0, color))

    case = 0
    for _ in range(300):
        canvases.append(np.full(4096, 0xff203040, dtype=np.uint32))
        for _k in range(int(rng.integers(1, 8))):
            r = rng.random()
            if r < 0.3:  # coordinates at / near x.5 (qRound ties)
                x, y = rng.integers(-4, 68) + 0.5, rng.integers(-4, 68) + 0.5
                w, h = rng.integers(0, 20) + rng.choice([0, 0.5, 0.25]), rng.integers(0, 20) + rng.choice([0, 0.5])
                if rng.random() < 0.3:
                    x, y = np.nextafter(x, -1e9), np.nextafter(y, 1e9)
            elif r < 0.45:  # negative extents
                x, y = rng.uniform(-10, 74), rng.uniform(-10, 74)
                w, h = rng.uniform(-20, 20), rng.uniform(-20, 20)
            else:
                x, y = rng.uniform(-10, 74), rng.uniform(-10, 74)
                w, h = rng.uniform(0, 30), rng.uniform(0, 30)
            color = 0xff000000 | int(rng.integers(0, 2 ** 24))
            add(case, float(x), float(y), float(w), float(h), color)
        case += 1
    for md in (11, 13, 19):  # chaser orbs: get_screen_rect of a grid cell, then the ORB_DIM inset
        unit = f32(np.float32(64) / np.float32(md))
        for _ in range(40):
            canvases.append(np.full(4096, 0xff000000, dtype=np.uint32))
            for gx in range(md):
                gy = int(rng.integers(0, md))
                eps = np.float32(0.02)
                rx = f32(f32(np.float32(gx) - eps) * unit)
                ry = f32(f32(f32(np.float32(md) - np.float32(gy + 1)) - eps) * unit)
                rw = f32(f32(1 + 2 * eps) * unit)
                d = 0.3
                x = rx + rw * (1 - np.float32(d)) / 2
                y = ry + rw * (1 - np.float32(d)) / 2
                add(case, float(x), float(y), float(rw * np.float32(d)), float(rw * np.float32(d)), 0xff00ff00)
            case += 1

    cmds = np.array(cmds, dtype=CMD_DTYPE)
    synth = np.zeros(1, np.uint32)
    atlas = atlas_for("coinrun")
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
