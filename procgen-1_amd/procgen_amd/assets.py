"""Asset atlas: the committed Qt-decoded packs flattened into one pixel array.

Layout handed to the engine (and, in tests, to the CPU oracle):

* ``pixels``  uint32[P] -- 0xAARRGGBB; sprites premultiplied ARGB32, backgrounds RGB32
  (the formats the reference converts to, procgen/src/resources.cpp:964, 969);
* ``sprites`` int32[1000, 4] -- (offset, w, h, 0) per image slot
  ``type + 100 * theme`` (basic-abstract-game.cpp:896); w = h = 0 for no image;
* ``backgrounds`` int32[B, 4] -- (offset, w, h, 0) in background-group order
  (``randn(B)`` picks one, basic-abstract-game.cpp:776);
* ``num_themes`` int32[100] -- ``asset_num_themes`` (basic-abstract-game.cpp:119).

Mirrored sprites (``QImage::mirrored(true, false)``, basic-abstract-game.cpp:121)
are not stored: the compositor flips the source column instead.
"""
import functools
import os

import numpy as np

from . import catalog

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def _key(path):
    return path.replace("/", "|")


@functools.lru_cache(maxsize=None)
def _load_pack(name):
    path = os.path.join(ASSET_DIR, name)
    if not os.path.exists(path):
        raise FileNotFoundError("asset pack %s missing (run tools/make_asset_pack.py)" % path)
    with np.load(path, allow_pickle=False) as z:
        return {k.replace("|", "/"): np.ascontiguousarray(z[k], dtype=np.uint32) for k in z.files}


class Atlas:
    def __init__(self, game):
        if game not in catalog.GAMES:
            raise ValueError("game %r has no asset table in this build (supported: %s)"
                             % (game, ", ".join(catalog.SUPPORTED_GAMES)))
        table = catalog.sprite_table(game)
        group = catalog.GAMES[game][1]
        sprites = _load_pack("sprites_%s.npz" % game)
        bgs = _load_pack("bg_%s.npz" % group)

        chunks, offset = [], 0
        seen = {}

        def place(img):
            nonlocal offset
            ident = id(img)
            if ident in seen:
                return seen[ident]
            chunks.append(img.reshape(-1))
            seen[ident] = offset
            offset += img.size
            return seen[ident]

        self.sprites = np.zeros((catalog.NUM_IMAGE_SLOTS, 4), dtype=np.int32)
        self.num_themes = np.zeros(catalog.MAX_ASSETS, dtype=np.int32)
        for t, names in table.items():
            self.num_themes[t] = len(names)
            for theme, n in enumerate(names):
                img = sprites[n]
                slot = t + catalog.MAX_ASSETS * theme
                self.sprites[slot] = (place(img), img.shape[1], img.shape[0], 0)

        names = catalog.BACKGROUND_GROUPS[group]
        self.backgrounds = np.zeros((len(names), 4), dtype=np.int32)
        for i, n in enumerate(names):
            img = bgs[n]
            self.backgrounds[i] = (place(img), img.shape[1], img.shape[0], 0)

        self.pixels = np.ascontiguousarray(np.concatenate(chunks)).astype(np.uint32)
        assert self.pixels.size < 2 ** 31
        self.game = game


@functools.lru_cache(maxsize=None)
def atlas_for(game):
    return Atlas(game)
