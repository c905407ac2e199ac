"""The register-frame render (pg_render.hip pg_render_rf_kernel: no LDS frame, lane = screen column,
4 rows at a time in registers (RF_RB), every (image, row) blended per pixel in draw order) forced on for every
game through PROCGEN_MI355X_RENDER_RF=all, against the oracle frame by frame: the painter's algorithm
of basic-abstract-game.cpp:930-1016 (background, grid tiles x-major / y-minor, z-ordered entities,
velocity squares, game_draw overlays) must come out bit-identical to the stamping kernel's and the
oracle's.  The games where it is the default (pg_capi.cpp RF_DEFAULT) run it in every other GPU test
too; PROCGEN_MI355X_RENDER_RF=0 keeps the LDS-frame kernel, which the uncentered / monochrome /
generated-asset tests exercise for every game."""
import numpy as np
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


@pytest.mark.parametrize("game", ["bigfish", "climber"])
def test_rf_default_long_episodes(game):
    """Two games the register-frame render serves by default (RF_DEFAULT), over long episodes: bigfish's
    fish lists grow for thousands of steps, climber's tall world scrolls; every frame must stay within the
    kernel's descriptor / tile-row caps (an overflow raises PG_ERR_RENDER) and bit-exact."""
    run_pair(game, 8, 2000, seed=45, num_levels=0, rand_seed=13)


@pytest.mark.parametrize("game", ["climber", "coinrun"])
def test_restored_uncentered_state_in_centred_env(game):
    """A state carries its options (game.cpp:266): an uncentered climber state (a 20 x 64 world, 64 tile
    rows) restored into a default (centred) env must leave the register-frame render for that game (its
    window exceeds 63 rows) and draw exactly what the uncentered env draws; restoring a centred state
    back returns the game to the default kernel.  coinrun (64 x 64) the same with the LDS kernel."""
    from procgen_amd import ProcgenGym3Env
    a = ProcgenGym3Env(num=2, env_name=game, num_levels=0, rand_seed=3, center_agent=False)
    b = ProcgenGym3Env(num=2, env_name=game, num_levels=0, rand_seed=8)  # centred: rf for climber
    rng = np.random.RandomState(5)
    for _ in range(20):
        act = rng.randint(0, 15, size=2).astype(np.int32)
        a.act(act)
        b.act(act)
    a.observe()
    b.set_state(a.get_state())
    for t in range(40):
        act = rng.randint(0, 15, size=2).astype(np.int32)
        a.act(act)
        b.act(act)
        ra, oa, fa = a.observe()
        rb, ob, fb = b.observe()
        np.testing.assert_array_equal(ob["rgb"], oa["rgb"], err_msg="step %d" % t)
        np.testing.assert_array_equal(rb, ra)
        np.testing.assert_array_equal(fb, fa)
    c = ProcgenGym3Env(num=2, env_name=game, num_levels=0, rand_seed=9)
    for _ in range(5):
        c.act(np.zeros(2, np.int32))
    c.observe()
    b.set_state(c.get_state())  # centred again: back on the default kernel, still exact
    for t in range(20):
        act = rng.randint(0, 15, size=2).astype(np.int32)
        b.act(act)
        c.act(act)
        _, ob, _ = b.observe()
        _, oc, _ = c.observe()
        np.testing.assert_array_equal(ob["rgb"], oc["rgb"], err_msg="recentred step %d" % t)
    for e in (a, b, c):
        e.close()
