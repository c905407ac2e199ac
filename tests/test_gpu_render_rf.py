"""The register-frame render (pg_render.hip pg_render_rf_kernel: no LDS frame, lane = screen column,
8 rows at a time in registers, every (image, row) blended per pixel in draw order) forced on for every
game through PROCGEN_MI355X_RENDER_RF=all, against the oracle frame by frame: the painter's algorithm
of basic-abstract-game.cpp:930-1016 (background, grid tiles x-major / y-minor, z-ordered entities,
velocity squares, game_draw overlays) must come out bit-identical to the stamping kernel's and the
oracle's.  The games where it is the default (pg_capi.cpp RF_DEFAULT) run it in every other GPU test
too; PROCGEN_MI355X_RENDER_RF=0 keeps the LDS-frame kernel, which the uncentered / monochrome /
generated-asset tests exercise for every game."""
import pytest

from test_gpu_games import GAMES, LATENT, run_pair

pytestmark = pytest.mark.gpu

ALL = [g for g in GAMES + ["coinrun"] if g != "bossfight"]  # bossfight stays on the LDS-frame kernel (rf_game)


@pytest.fixture
def rf(monkeypatch):
    monkeypatch.setenv("PROCGEN_MI355X_RENDER_RF", "all")


@pytest.mark.parametrize("game", ALL)
def test_rf_parity_hard(game, rf):
    run_pair(game, 24, 200, seed=41, num_levels=0, rand_seed=2, latent=game in LATENT)


@pytest.mark.parametrize("game", ALL)
def test_rf_parity_easy_options(game, rf):
    kw = dict(distribution_mode="easy", restrict_themes=True, paint_vel_info=True)
    if game in ("coinrun", "heist", "ninja"):
        kw["use_backgrounds"] = False
    run_pair(game, 16, 150, seed=42, num_levels=20, start_level=3, rand_seed=5, latent=game in LATENT, **kw)


@pytest.mark.parametrize("game", ["jumper", "fruitbot", "starpilot", "plunder"])
def test_rf_parity_long(game, rf):
    """Many rotated / tiled images and the compass over long episodes."""
    run_pair(game, 12, 600, seed=43, num_levels=0, rand_seed=9)


def test_rf_off_keeps_lds_kernel(monkeypatch):
    monkeypatch.setenv("PROCGEN_MI355X_RENDER_RF", "0")
    run_pair("coinrun", 16, 100, seed=44, num_levels=0, rand_seed=3)
