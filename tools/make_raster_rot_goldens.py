#!/usr/bin/env python3
"""Generate tests/golden/qt_raster_rot_goldens.npz: rotated drawImage cases through the REAL
Qt 5.9.7 raster engine (build container only, needs /opt/conda Qt).

draw_image with rotation != 0 (reference basic-abstract-game.cpp:908-916) does
save(); translate(center); rotate(rotation * 180 / PI); drawImage(QRectF(-w/2, -h/2, w, h), img).
The cases mix synthetic images at random geometry and angles with the angles the games
produce (heist face_direction: -atan2f(dy, dx) for the 8 move directions, ring keys PI/2;
heist.cpp:186-199, entity.cpp:84-88) at heist-like geometry with the real heist atlas.
The oracle's restatement (qt_draw_image_rotated in oracle/procgen_oracle.c) must reproduce
every canvas bit-for-bit (tests/test_oracle_pins.py).
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
from golden_io import CMD_ROT_DTYPE, encode_all  # noqa: E402
from make_raster_goldens import build_tool, f32  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "qt_raster_rot_goldens.npz")
PI_F = np.float32(3.14159265358979323846264338327950288)


def game_angles():
    out = []
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            if dx == 0 and dy == 0:
                continue
            rot = np.float32(-1) * np.arctan2(np.float32(dy), np.float32(dx))
            if rot != 0:
                out.append(float(np.float32(np.float32(rot * np.float32(180)) / PI_F)))
    out.append(float(np.float32(np.float32(np.float32(PI_F / np.float32(2)) * np.float32(180)) / PI_F)))
    # leaper: frog +-PI/2, 0, PI; cars PI (leaper.cpp:156-158, 240-246) -- and Qt's exact special
    # cases of QTransform::rotate (+-90, 180 = a scale, 270)
    for rot in (PI_F, -PI_F, -PI_F / np.float32(2)):
        out.append(float(np.float32(np.float32(np.float32(rot) * np.float32(180)) / PI_F)))
    out += [90.0, -90.0, 180.0, -180.0, 270.0, -270.0]
    return out


def main():
    rng = np.random.default_rng(777)
    atlas = atlas_for("heist")
    angles = game_angles()
    synth, cmds, canvases = [], [], []
    synth_off = 0

    def synth_image(iw, ih):
        nonlocal synth_off
        a = rng.integers(0, 256, size=(ih, iw), dtype=np.uint32)
        a[rng.random((ih, iw)) < 0.3] = 255
        a[rng.random((ih, iw)) < 0.2] = 0
        c = [np.minimum(rng.integers(0, 256, size=(ih, iw), dtype=np.uint32), a) for _ in range(3)]
        px = (a << 24) | (c[0] << 16) | (c[1] << 8) | c[2]
        synth.append(px.reshape(-1))
        off = synth_off
        synth_off += px.size
        return off

    def add(case, x, y, w, h, deg, opacity=1.0, mirrored=0, src=0, ref=0, iw=0, ih=0):
        cmds.append((case, 3, x, y, w, h, opacity, mirrored, 6, src, ref, iw, ih, 0, deg))

    case = 0
    for _ in range(250):  # synthetic images, random geometry, game and random angles
        if rng.random() < 0.25:
            canvases.append((rng.integers(0, 2 ** 24, size=4096, dtype=np.uint32) | 0xff000000).astype(np.uint32))
        else:
            canvases.append(np.full(4096, 0xff203040, dtype=np.uint32))
        for _k in range(int(rng.integers(1, 5))):
            iw, ih = int(rng.integers(2, 24)), int(rng.integers(2, 24))
            off = synth_image(iw, ih)
            x, y = rng.uniform(-20, 70), rng.uniform(-20, 70)
            w, h = rng.uniform(0.3, 40), rng.uniform(0.3, 40)
            deg = angles[rng.integers(0, len(angles))] if rng.random() < 0.6 else float(rng.uniform(-400, 400))
            op = [1.0, 1.0, 0.5, f32(0.8), rng.random()][rng.integers(0, 5)]
            add(case, x, y, w, h, deg, op, int(rng.random() < 0.4), 0, off, iw, ih)
        case += 1

    unit = f32(np.float32(64) / np.float32(13))
    view_dim = f32(np.float32(64.0) / unit)
    slots = [i for i in range(1000) if atlas.sprites[i][1] > 0]
    for _ in range(200):  # heist geometry: agent-sized entities at world positions, ring keys
        canvases.append(np.full(4096, 0xff000000, dtype=np.uint32))
        for _k in range(int(rng.integers(1, 6))):
            slot = int(slots[rng.integers(0, len(slots))])
            ex, ey = f32(rng.uniform(0, 13)), f32(rng.uniform(0, 13))
            rx = f32(rng.choice([0.375, 0.3, 0.5, 0.03]))
            ry = f32(rx / f32(np.float32(atlas.sprites[slot][1]) / np.float32(atlas.sprites[slot][2])))
            x = f32(f32(ex - rx) * unit)
            y = f32(f32(view_dim - f32(ey + ry)) * unit)
            w, h = f32(f32(2 * rx) * unit), f32(f32(2 * ry) * unit)
            deg = angles[rng.integers(0, len(angles))]
            add(case, x, y, w, h, deg, 1.0, 0, 1, slot)
        case += 1

    cmds = np.array(cmds, dtype=CMD_ROT_DTYPE)
    synth = np.concatenate(synth).astype(np.uint32)
    canvas_in = np.stack(canvases).astype(np.uint32)
    stream = encode_all(canvas_in, cmds, synth, atlas)
    with tempfile.TemporaryDirectory() as td:
        tool = os.path.join(td, "qt_raster_golden")
        build_tool(tool)
        res = subprocess.run([tool], input=stream, stdout=subprocess.PIPE, check=True).stdout
    canvas_out = np.frombuffer(res, dtype="<u4").reshape(case, 4096)
    np.savez_compressed(OUT, cmds=cmds, synth=synth, canvas_in=canvas_in, canvas_out=canvas_out,
                        atlas_game=np.array("heist"), qt_version=np.array("5.9.7"))
    print("wrote", OUT, case, "cases", len(cmds), "commands", os.path.getsize(OUT) / 1e6, "MB")


if __name__ == "__main__":
    main()
