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

``EngineAtlas`` packs several games for the engine's C ABI (procgen_upload_atlas): one
pixel array, per-game tables indexed by game id (procgen/env.py:15-32 order).
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
        bgs = _load_pack("bg_%s.npz" % catalog.BACKGROUND_PACK.get(group, group))

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
                if theme >= catalog.MAX_IMAGE_THEMES:
                    break  # never drawn: draw_image asserts theme < MAX_IMAGE_THEMES (basic-abstract-game.cpp:897)
                img = sprites[n]
                slot = t + catalog.MAX_ASSETS * theme
                self.sprites[slot] = (place(img), img.shape[1], img.shape[0], 0)

        names = catalog.BACKGROUND_GROUPS[group]
        self.backgrounds = np.zeros((len(names), 4), dtype=np.int32)
        for i, n in enumerate(names):
            img = bgs[n]
            self.backgrounds[i] = (place(img), img.shape[1], img.shape[0], 0)

        if game == "jumper":  # the compass overlay table rides in image slot TABLE_SLOT
            table = compass_table_words()
            self.sprites[catalog.TABLE_SLOT] = (place(table), table.size, 1, 0)

        self.pixels = np.ascontiguousarray(np.concatenate(chunks)).astype(np.uint32)
        assert self.pixels.size < 2 ** 31
        self.game = game


@functools.lru_cache(maxsize=None)
def compass_table_words():
    """jumper_compass.npz flattened to the uint32 words the oracle and the engine read:
    magic, NY, NX, MAXW, MAXH; per cfg (hard + 2 * uncentered) x1, y1, bx0, by0, bnx, bny, cx, cy, cr
    (float bits); dial[4][64] u64; needle[4][NY][NX][64] u64; jump[MAXW + 1][MAXH + 1][64] u64."""
    path = os.path.join(ASSET_DIR, "jumper_compass.npz")
    if not os.path.exists(path):
        raise FileNotFoundError("%s missing (run tools/make_compass_tables.py)" % path)
    with np.load(path, allow_pickle=False) as z:
        geom, cf, dial, needle, jump = z["cfg_geom"], z["cfg_cf"], z["dial"], z["needle"], z["jump"]
    head = np.array([0x434D5053, needle.shape[1], needle.shape[2], jump.shape[0] - 1, jump.shape[1] - 1], np.uint32)
    cfg = np.concatenate([geom.astype(np.int32).view(np.uint32), cf.astype(np.float32).view(np.uint32)], axis=1)
    parts = [head, cfg.reshape(-1)] + [np.ascontiguousarray(a, dtype=np.uint64).view(np.uint32).reshape(-1)
                                       for a in (dial, needle, jump)]
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.uint32)


@functools.lru_cache(maxsize=None)
def atlas_for(game):
    return Atlas(game)


class EngineAtlas:
    """Atlases of every game of a batch in the engine's layout (include/procgen_mi355x.h)."""

    NUM_GAMES = 16
    MAX_BG = 64

    def __init__(self, games):
        games = list(dict.fromkeys(games))
        self.sprites = np.zeros((self.NUM_GAMES, catalog.NUM_IMAGE_SLOTS, 4), dtype=np.int32)
        self.backgrounds = np.zeros((self.NUM_GAMES, self.MAX_BG, 4), dtype=np.int32)
        self.num_backgrounds = np.zeros(self.NUM_GAMES, dtype=np.int32)
        self.num_themes = np.zeros((self.NUM_GAMES, catalog.MAX_ASSETS), dtype=np.int32)
        chunks, base = [], 0
        for g in games:
            a = atlas_for(g)
            gid = catalog.ENV_NAMES.index(g)
            sp = a.sprites.copy()
            sp[:, 0] += np.where(sp[:, 1] > 0, base, 0).astype(np.int32)
            self.sprites[gid] = sp
            nb = a.backgrounds.shape[0]
            assert nb <= self.MAX_BG
            bg = a.backgrounds.copy()
            bg[:, 0] += base
            self.backgrounds[gid, :nb] = bg
            self.num_backgrounds[gid] = nb
            self.num_themes[gid] = a.num_themes
            chunks.append(a.pixels)
            base += a.pixels.size
        self.pixels = np.ascontiguousarray(np.concatenate(chunks)).astype(np.uint32)
        assert self.pixels.size < 2 ** 31
        self.games = games


@functools.lru_cache(maxsize=None)
def engine_atlas_for(names):
    """names: tuple of game names (a batch's env_name list)."""
    return EngineAtlas(names)
