#!/usr/bin/env python3
"""Build procgen-1_amd/assets/jumper_compass.npz: the Qt 5.9.7 raster output of jumper's compass
overlay (jumper.cpp:137-177), tabulated by tools/qt_compass_tables.cpp (build container only,
needs /opt/conda Qt).

Arrays (uint64 row bitmaps, bit x of row y = pixel (x, y) painted):
  cfg_geom   int32[4, 6]   x1, y1, bx0, by0, bnx, bny per cfg = hard + 2 * uncentered
  cfg_cf     float32[4, 3] cx, cy, cr (the floats draw_compass derives from compass_rect)
  dial       uint64[4, 64]
  needle     uint64[4, NY, NX, 64] (endpoint (bx0 + i, by0 + j) at [cfg, j, i]; zero padded)
  jump       uint64[MAXW + 1, MAXH + 1, 64] for QRect(20, 20, w, h) (translation invariant)
  blend_bg / blend_out uint32[4096]: QColor(255, 255, 255, 120) ellipse over a random RGB32 canvas
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "procgen-1_amd", "assets", "jumper_compass.npz")
QT = "/opt/conda"


def main():
    with tempfile.TemporaryDirectory() as td:
        tool = os.path.join(td, "qt_compass_tables")
        subprocess.run(["g++", "-O2", "-fPIC", "-std=c++17", os.path.join(HERE, "qt_compass_tables.cpp"),
                        "-I%s/include/qt" % QT, "-I%s/include/qt/QtGui" % QT, "-I%s/include/qt/QtCore" % QT,
                        "-L%s/lib" % QT, "-lQt5Gui", "-lQt5Core", "-Wl,-rpath,%s/lib" % QT, "-o", tool], check=True)
        raw = subprocess.run([tool], check=True, capture_output=True).stdout
    off = 0

    def take(dtype, n):
        nonlocal off
        a = np.frombuffer(raw, dtype=dtype, count=n, offset=off)
        off += a.nbytes
        return a.copy()

    geoms, cfs, dials, needles = [], [], [], []
    for _ in range(4):
        g = take(np.int32, 6)
        cf = take(np.float32, 3)
        dial = take(np.uint64, 64)
        nx, ny = int(g[4]), int(g[5])
        nd = take(np.uint64, nx * ny * 64).reshape(ny, nx, 64)
        geoms.append(g), cfs.append(cf), dials.append(dial), needles.append(nd)
    maxw, maxh = take(np.int32, 2)
    jump = take(np.uint64, (maxw + 1) * (maxh + 1) * 64).reshape(maxw + 1, maxh + 1, 64)
    bg = take(np.uint32, 4096)
    out = take(np.uint32, 4096)
    assert off == len(raw)
    NY = max(n.shape[0] for n in needles)
    NX = max(n.shape[1] for n in needles)
    needle = np.zeros((4, NY, NX, 64), np.uint64)
    for k, n in enumerate(needles):
        needle[k, :n.shape[0], :n.shape[1]] = n
    np.savez_compressed(OUT, cfg_geom=np.stack(geoms), cfg_cf=np.stack(cfs), dial=np.stack(dials), needle=needle,
                        jump=jump, blend_bg=bg, blend_out=out)
    print(OUT, np.stack(geoms).tolist(), needle.shape)


if __name__ == "__main__":
    main()
