"""Serialisation of Qt painter command lists (shared by tools/make_raster_goldens.py and
tests/test_oracle_qt_raster.py).

Byte format = tools/qt_raster_golden.cpp's stdin format (little endian)."""
import struct

import numpy as np

CMD_DTYPE = np.dtype([
    ("case", "<i4"), ("kind", "<i4"), ("x", "<f8"), ("y", "<f8"), ("w", "<f8"), ("h", "<f8"),
    ("opacity", "<f8"), ("mirrored", "<i4"), ("fmt", "<i4"),
    # image source: src 0 = synthetic (offset/iw/ih into synth pixel array), 1 = atlas sprite slot,
    # 2 = atlas background index ; for fills `color` holds 0xAARRGGBB
    ("src", "<i4"), ("ref", "<i8"), ("iw", "<i4"), ("ih", "<i4"), ("color", "<u4"),
])
# kind 3 (rotated drawImage) carries its angle in degrees
CMD_ROT_DTYPE = np.dtype(CMD_DTYPE.descr + [("deg", "<f8")])


def image_of(cmd, synth, atlas):
    if cmd["src"] == 0:
        off, iw, ih = int(cmd["ref"]), int(cmd["iw"]), int(cmd["ih"])
        return synth[off:off + iw * ih], iw, ih
    table = atlas.sprites if cmd["src"] == 1 else atlas.backgrounds
    off, iw, ih, _ = (int(v) for v in table[int(cmd["ref"])])
    return atlas.pixels[off:off + iw * ih], iw, ih


def encode_cmds(cmds, synth, atlas):
    """Command list of ONE case -> bytes (u32 ncmds + commands)."""
    out = [struct.pack("<I", len(cmds))]
    for c in cmds:
        out.append(struct.pack("<Iddddd", int(c["kind"]), c["x"], c["y"], c["w"], c["h"], c["opacity"]))
        out.append(struct.pack("<Ii", int(c["mirrored"]), 0))
        if c["kind"] == 3:
            out.append(struct.pack("<d", float(c["deg"])))
        if c["kind"] in (0, 3):
            px, iw, ih = image_of(c, synth, atlas)
            out.append(struct.pack("<III", int(c["fmt"]), iw, ih))
            out.append(np.ascontiguousarray(px, dtype="<u4").tobytes())
        else:
            out.append(struct.pack("<I", int(c["color"])))
    return b"".join(out)


def encode_all(canvas_in, cmds, synth, atlas):
    ncase = canvas_in.shape[0]
    parts = [struct.pack("<I", ncase)]
    for i in range(ncase):
        parts.append(struct.pack("<I", 4))  # QImage::Format_RGB32
        parts.append(np.ascontiguousarray(canvas_in[i], dtype="<u4").tobytes())
        parts.append(encode_cmds(cmds[cmds["case"] == i], synth, atlas))
    return b"".join(parts)
