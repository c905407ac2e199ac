"""CPU check of the native asset loader libenv_make runs (csrc/pg_assets.cpp, the reference's
global_init -> images_load, vecgame.cpp:144-153): for every game, every image slot, background
and theme count it builds from the committed packs + manifest equals procgen_amd.assets.Atlas
(the host-side restatement the oracle reads).  No GPU: procgen_atlas_host runs the loader alone."""
import ctypes

import numpy as np
import pytest

from procgen_amd import _lib, catalog
from procgen_amd.assets import atlas_for

NG, SLOTS, MAXBG = 16, 1000, 64


def native_atlas(names, root=None):
    lib = _lib.load()
    sprites = np.zeros((NG, SLOTS, 4), np.int32)
    bgs = np.zeros((NG, MAXBG, 4), np.int32)
    nbg = np.zeros(NG, np.int32)
    themes = np.zeros((NG, 100), np.int32)
    rootb = root.encode() if root else None
    n = lib.procgen_atlas_host(names.encode(), rootb, None, 0, None, None, None, None)
    assert n > 0, lib.procgen_error_string(None)
    pixels = np.zeros(n, np.uint32)
    n2 = lib.procgen_atlas_host(names.encode(), rootb, pixels.ctypes.data, n, sprites.ctypes.data, bgs.ctypes.data,
                                nbg.ctypes.data, themes.ctypes.data)
    assert n2 == n
    return pixels, sprites, bgs, nbg, themes


def image(pixels, rec):
    off, w, h = int(rec[0]), int(rec[1]), int(rec[2])
    return pixels[off:off + w * h]


@pytest.mark.parametrize("game", catalog.ENV_NAMES)
def test_native_atlas_matches_python_atlas(game):
    pixels, sprites, bgs, nbg, themes = native_atlas(game)
    gid = catalog.ENV_NAMES.index(game)
    a = atlas_for(game)
    assert np.array_equal(themes[gid], a.num_themes)
    assert nbg[gid] == a.backgrounds.shape[0]
    for slot in range(SLOTS):
        ref = a.sprites[slot]
        got = sprites[gid, slot]
        assert tuple(got[1:3]) == tuple(ref[1:3]), (game, slot)
        if ref[1] > 0:
            assert np.array_equal(image(pixels, got), image(a.pixels, ref)), (game, slot)
    for i in range(a.backgrounds.shape[0]):
        assert tuple(bgs[gid, i, 1:3]) == tuple(a.backgrounds[i, 1:3])
        assert np.array_equal(image(pixels, bgs[gid, i]), image(a.pixels, a.backgrounds[i])), (game, i)
    other = [g for g in range(NG) if g != gid]
    assert not sprites[other].any() and not nbg[other].any()


def test_mixed_batch_places_each_image_once():
    names = ",".join(catalog.ENV_NAMES)
    pixels, sprites, bgs, nbg, themes = native_atlas(names)
    # coinrun, climber, ninja and jumper share the platform group: one copy of each background
    g = [catalog.ENV_NAMES.index(x) for x in ("coinrun", "climber", "ninja", "jumper")]
    for k in g[1:]:
        assert np.array_equal(bgs[k], bgs[g[0]])
    total = sum(atlas_for(x).pixels.size for x in catalog.ENV_NAMES)
    assert pixels.size < total // 2
    for gid, game in enumerate(catalog.ENV_NAMES):
        a = atlas_for(game)
        assert nbg[gid] == a.backgrounds.shape[0]
        for slot in np.nonzero(a.sprites[:, 1])[0]:
            assert np.array_equal(image(pixels, sprites[gid, slot]), image(a.pixels, a.sprites[slot]))


def test_missing_resource_root_fails_cleanly(tmp_path):
    lib = _lib.load()
    n = lib.procgen_atlas_host(b"coinrun", str(tmp_path).encode(), None, 0, None, None, None, None)
    assert n < 0
    assert b"manifest" in lib.procgen_error_string(None)


def test_manifest_is_current():
    """The committed manifest is what tools/make_asset_manifest.py writes from catalog.py."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(repo, "procgen-1_amd", "assets", "manifest.txt")
    before = open(path).read()
    tool = os.path.join(repo, "tools", "make_asset_manifest.py")
    if not os.path.exists(tool):
        pytest.skip("tools/ not shipped here")
    subprocess.run([sys.executable, tool], check=True, capture_output=True)
    assert open(path).read() == before
