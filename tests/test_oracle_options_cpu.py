"""Render options of the CPU oracle (the parity checker) -- CPU only.

* use_monochrome_assets: draw_image -> draw_grid_obj -> fillRect(color_for_type(type, theme))
  (basic-abstract-game.cpp:886-928, 464-490).  Every colour channel of color_for_type is
  chunk * (digit + 1) - 1 with chunk = 64, i.e. one of {63, 127, 191, 255}.
* paint_vel_info: two grey squares QRectF(0, 0, 12.8, 12.8) and QRectF(12.8, 0, 12.8, 12.8)
  shaded by to_shade(.5 * v / max + .5) (:969-977, qt-utils.h:21-28) -> pixel columns [0, 13)
  and [13, 26) of rows [0, 13) after Qt's qRound of the edges.  Games with
  has_useful_vel_info = false (chaser, heist, maze, miner, plunder) draw nothing extra.
No reference fixture covers these options: the colour formula and the fill geometry are pinned
by the Qt fill goldens (tests/golden/qt_raster_fill_goldens.npz) and the properties below.
"""
import numpy as np
import pytest

from oracle_lib import OracleEnv

MONO_LEVELS = {63, 127, 191, 255}


def _frames(game, steps, **kw):
    orc = OracleEnv(game, 4, num_levels=0, rand_seed=1, **kw)
    rng = np.random.RandomState(0)
    out = [orc.observe()["rgb"].copy()]
    for _ in range(steps):
        orc.step(rng.randint(0, 15, size=4).astype(np.int32))
        out.append(orc.observe()["rgb"].copy())
    return np.stack(out)


@pytest.mark.parametrize("game", ["coinrun", "maze", "heist", "bigfish", "climber"])
def test_monochrome_palette(game):
    fr = _frames(game, 30, use_monochrome_assets=1, use_backgrounds=0)
    px = fr.reshape(-1, 3)
    black = (px == 0).all(axis=1)
    levels = np.isin(px, list(MONO_LEVELS)).all(axis=1)
    assert (black | levels).all(), "monochrome frame holds a colour outside the color_for_type palette"
    assert levels.mean() > 0.001  # something is drawn (bigfish: a few small fish on black)


def test_monochrome_restrict_themes_changes_colours_only_for_themed_types():
    a = _frames("coinrun", 10, use_monochrome_assets=1, use_backgrounds=0)
    b = _frames("coinrun", 10, use_monochrome_assets=1, use_backgrounds=0, restrict_themes=1)
    assert a.shape == b.shape
    # same geometry: the set of black (undrawn) pixels does not depend on the theme
    np.testing.assert_array_equal((a == 0).all(axis=-1), (b == 0).all(axis=-1))


@pytest.mark.parametrize("game", ["coinrun", "bigfish", "starpilot"])
def test_vel_info_squares(game):
    fr = _frames(game, 40, paint_vel_info=1)
    base = _frames(game, 40)
    sq1, sq2 = fr[:, :, :13, :13], fr[:, :, :13, 13:26]
    for sq in (sq1, sq2):
        flat = sq.reshape(sq.shape[0], sq.shape[1], -1)
        assert (flat == flat[..., :1]).all(), "velocity square is not one grey level"
    # outside the two squares the frame is the plain render
    mask = np.ones((64, 64), bool)
    mask[:13, :26] = False
    np.testing.assert_array_equal(fr[:, :, mask], base[:, :, mask])
    if game == "coinrun":  # the agent starts at rest: to_shade(.5) = int(127.5) = 127
        assert (sq1[0] == 127).all() and (sq2[0] == 127).all()


@pytest.mark.parametrize("game", ["maze", "chaser", "plunder"])
def test_vel_info_absent_without_useful_velocity(game):
    np.testing.assert_array_equal(_frames(game, 20, paint_vel_info=1), _frames(game, 20))
