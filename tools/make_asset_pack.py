#!/usr/bin/env python3
"""Build the committed asset packs under procgen-1_amd/assets/.

The reference loads every PNG with Qt (``QImage(path).convertToFormat(fmt)``,
procgen/src/resources.cpp:20-30): sprites as ARGB32_Premultiplied, backgrounds
as RGB32.  This script runs tools/qt_asset_dump.cpp -- linked against the Qt5
present in this image (/opt/conda, Qt 5.9.7) -- so the packed pixels are exactly
what the reference's renderer composites, then stores them zlib-compressed as
``.npz`` (uint32 0xAARRGGBB arrays, loaded with allow_pickle=False).

Run in the build container only (needs /root/reference and /opt/conda Qt):
    python tools/make_asset_pack.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
from procgen_amd import catalog  # noqa: E402

ASSET_ROOT = "/root/reference/procgen/data/assets/"
OUT_DIR = os.path.join(REPO, "procgen-1_amd", "assets")
QT = "/opt/conda"


def build_dumper(out):
    cmd = ["g++", "-O2", "-fPIC", "-std=c++17", os.path.join(HERE, "qt_asset_dump.cpp"),
           "-I%s/include/qt" % QT, "-I%s/include/qt/QtGui" % QT, "-I%s/include/qt/QtCore" % QT,
           "-L%s/lib" % QT, "-lQt5Gui", "-lQt5Core", "-Wl,-rpath,%s/lib" % QT, "-o", out]
    subprocess.run(cmd, check=True)


def dump(tool, items):
    """items: list of (kind, relpath) -> dict relpath -> uint32[h, w]"""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "dump.bin")
        lines = "".join("%s %s\n" % (k, p) for k, p in items)
        subprocess.run([tool, ASSET_ROOT, out], input=lines.encode(), check=True)
        raw = np.fromfile(out, dtype=np.uint32)
    res = {}
    off = 0
    for _, p in items:
        _, w, h = raw[off:off + 3]
        off += 3
        res[p] = raw[off:off + w * h].reshape(h, w).copy()
        off += w * h
    assert off == raw.size
    return res


def key(path):
    return path.replace("/", "|")


def main():
    os.makedirs(OUT_DIR, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        tool = os.path.join(td, "qt_asset_dump")
        build_dumper(tool)
        only = sys.argv[1:]
        for game in catalog.SUPPORTED_GAMES:
            if only and game not in only:
                continue
            names = sorted({n for v in catalog.sprite_table(game).values() for n in v})
            imgs = dump(tool, [("S", n) for n in names])
            np.savez_compressed(os.path.join(OUT_DIR, "sprites_%s.npz" % game),
                                **{key(k): v for k, v in imgs.items()})
            group = catalog.GAMES[game][1]
            group = catalog.BACKGROUND_PACK.get(group, group)  # subset groups share a pack
            bgs = catalog.BACKGROUND_GROUPS[group]
            imgs = dump(tool, [("B", n) for n in dict.fromkeys(bgs)])
            np.savez_compressed(os.path.join(OUT_DIR, "bg_%s.npz" % group),
                                **{key(k): v for k, v in imgs.items()})
            print(game, "ok")


if __name__ == "__main__":
    main()
