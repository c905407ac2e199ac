#!/usr/bin/env python3
"""Write a grid of oracle frames to a PNG (visual sanity check while restating a game).

    python tools/frames_png.py GAME OUT.png [steps] [key=value ...]
"""
import os
import struct
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle_lib import OracleEnv  # noqa: E402


def write_png(path, img):
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def main():
    game, out = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    kw = {k: int(v) for k, v in (a.split("=") for a in sys.argv[4:])}
    n = 8
    env = OracleEnv(game, n, **kw)
    rng = np.random.RandomState(0)
    rows = []
    for t in range(steps + 1):
        if t:
            env.step(rng.randint(0, 15, n).astype(np.int32))
        if t % max(1, steps // 4) == 0:
            rows.append(np.concatenate(list(env.observe()["rgb"]), axis=1))
    img = np.concatenate(rows[:5], axis=0)
    img = img.repeat(2, 0).repeat(2, 1)
    write_png(out, np.ascontiguousarray(img))


if __name__ == "__main__":
    main()
