"""CPU tests of host logic: asset catalogue/atlas (the data contract that drives RNG draw
counts) and the synthetic action hash shared by engine and tests."""
import numpy as np

from oracle_lib import hashed_actions, splitmix64


def test_background_groups_match_reference_counts():
    from procgen_amd import catalog
    # SURVEY.md Appendix A (resources.cpp:837-979 incl. the space append and caves)
    counts = {g: len(v) for g, v in catalog.BACKGROUND_GROUPS.items()}
    assert counts == {"platform": 62, "space": 13, "topdown": 9, "topdown_simple": 1, "water": 7,
                      "water_surface": 4, "caves": 3}
    assert catalog.PLATFORM_BACKGROUNDS[:2] == ["platform_backgrounds/alien_bg.png",
                                                "platform_backgrounds/another_world_bg.png"]
    assert catalog.PLATFORM_BACKGROUNDS[49] == "space_backgrounds/deep_space_01.png"


def test_coinrun_theme_counts():
    from procgen_amd import catalog
    nt = catalog.num_themes("coinrun")
    # coinrun.cpp:72-121: PLAYER 5 colours, walking enemies 9, ground themes 6, crates 4
    assert nt[0] == 5 and nt[6] == 9 and nt[7] == 9 and nt[15] == 6 and nt[16] == 6 and nt[20] == 4
    assert nt[1] == nt[2] == nt[3] == nt[17] == nt[18] == 1
    assert nt[59] == 1  # TRAIL reserved sprite


def test_atlas_layout():
    from procgen_amd.assets import atlas_for
    a = atlas_for("coinrun")
    assert a.backgrounds.shape == (62, 4)
    assert a.sprites.shape == (1000, 4)
    # alien sprites are 128x256, tiles 128x128, the trail dot 17x17
    assert tuple(a.sprites[0][1:3]) == (128, 256)
    assert tuple(a.sprites[15][1:3]) == (128, 128)
    assert tuple(a.sprites[59][1:3]) == (17, 17)
    for off, w, h, _ in a.backgrounds:
        assert w > 0 and h > 0 and off + w * h <= a.pixels.size
    # RGB32 backgrounds are opaque
    off, w, h, _ = a.backgrounds[0]
    assert np.all(a.pixels[off:off + w * h] >> 24 == 255)


def test_hashed_actions_vector_matches_scalar():
    ids = np.array([0, 1, 77, 65535, 2 ** 31 + 5])
    v = hashed_actions(0x5EED, ids, 12345)
    s = [splitmix64((0x5EED ^ ((int(g) & 0xFFFFFFFF) << 32) ^ 12345)) % 15 for g in ids]
    assert v.tolist() == s
    assert v.min() >= 0 and v.max() < 15


def test_new_game_theme_counts():
    from procgen_amd import catalog
    bf, mz, hs = catalog.num_themes("bigfish"), catalog.num_themes("maze"), catalog.num_themes("heist")
    assert bf[0] == 1 and bf[2] == 3                      # bigfish.cpp:34-43
    assert mz[51] == 1 and mz[2] == 1 and mz[0] == 1      # maze.cpp:33-41
    assert hs[2] == 3 and hs[1] == 3 and hs[9] == 1       # heist.cpp:46-64


def test_engine_atlas_tables():
    from procgen_amd import catalog
    from procgen_amd.assets import atlas_for, engine_atlas_for
    ea = engine_atlas_for(("bigfish", "coinrun", "heist", "maze"))
    for g in ("bigfish", "coinrun", "heist", "maze"):
        gid = catalog.ENV_NAMES.index(g)
        a = atlas_for(g)
        assert ea.num_backgrounds[gid] == a.backgrounds.shape[0]
        np.testing.assert_array_equal(ea.num_themes[gid], a.num_themes)
        for slot in np.nonzero(a.sprites[:, 1])[0]:
            off, w, h, _ = ea.sprites[gid, slot]
            o2, w2, h2, _ = a.sprites[slot]
            assert (w, h) == (w2, h2)
            np.testing.assert_array_equal(ea.pixels[off:off + w * h], a.pixels[o2:o2 + w * h])
    assert ea.num_backgrounds[catalog.ENV_NAMES.index("maze")] == 9  # topdown group


def test_miner_catalog():
    from procgen_amd import catalog
    mn = catalog.num_themes("miner")
    assert mn[0] == mn[1] == mn[2] == mn[6] == mn[9] == mn[10] == mn[12] == 1  # miner.cpp:50-66
    assert 11 not in catalog.MINER_SPRITES  # mud.png is absent from the reference's assets
    assert len(catalog.BACKGROUND_GROUPS["caves"]) == 3
