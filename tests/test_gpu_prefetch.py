"""Level prefetch (pg_reset.hip request_spare / swap_spare, PGDev::sp_*): the next level of every env
is generated ahead on a side stream and swapped in when the episode ends.  The result must be what
the in-line reset (Game::reset, game.cpp:109-134) produces, so these runs force the prefetch on for
every game (it is on by default only for caveflyer and jumper) and compare against the oracle step
for step, through many episode ends."""
import numpy as np
import pytest

from test_gpu_coinrun import assert_same, gpu_obs
from test_gpu_games import GAMES, LATENT, make_gpu, run_pair

pytestmark = pytest.mark.gpu

ALL = GAMES + ["coinrun"]


@pytest.fixture
def prefetch(monkeypatch):
    def on(lag=None):
        monkeypatch.setenv("PROCGEN_MI355X_PREFETCH", "1")
        if lag is not None:
            monkeypatch.setenv("PROCGEN_MI355X_PREFETCH_LAG", str(lag))
    return on


@pytest.mark.parametrize("game", ALL)
def test_prefetch_parity(game, prefetch):
    prefetch()
    # the maze games rarely end under random actions: their small easy levels do, now and then
    kw = dict(distribution_mode="easy") if game in ("maze", "heist", "miner") else {}
    episodes, _ = run_pair(game, 32, 300, seed=21, num_levels=0, rand_seed=3, latent=game in LATENT, **kw)
    if game not in ("maze", "heist", "miner"):
        assert episodes > 0


@pytest.mark.parametrize("game,lag", [("caveflyer", 1), ("jumper", 3), ("bigfish", 5), ("miner", 8)])
def test_prefetch_lags(game, lag, prefetch):
    prefetch(lag)
    episodes, _ = run_pair(game, 12, 250, seed=22, num_levels=0, rand_seed=8, latent=game in LATENT)
    assert episodes > 0


@pytest.mark.parametrize("game", ["caveflyer", "heist", "chaser"])
def test_prefetch_bounded_levels_and_modes(game, prefetch):
    prefetch()
    run_pair(game, 8, 200, seed=23, num_levels=50, start_level=7, rand_seed=1, distribution_mode="easy",
             latent=game in LATENT)


@pytest.mark.parametrize("game", ["caveflyer", "jumper"])
def test_prefetch_forced_off(game, monkeypatch):
    monkeypatch.setenv("PROCGEN_MI355X_PREFETCH", "0")
    run_pair(game, 8, 150, seed=24, num_levels=0, rand_seed=2)


@pytest.mark.parametrize("game", ["caveflyer", "bigfish"])
def test_prefetch_after_set_state(game, prefetch):
    """set_state replaces an env's level-seed generator: its spare (made from the old one) must not
    be swapped in.  Env 3 gets env 0's state and must then play exactly env 0's levels."""
    prefetch()
    num = 4
    env = make_gpu(num, game, num_levels=0, start_level=0, rand_seed=4)
    rng = np.random.RandomState(5)
    for _ in range(20):
        env.act(rng.randint(0, 15, size=num).astype(np.int32))
        env.observe()
    st = env.get_state()
    st[3] = st[0]
    env.set_state(st)
    ends = 0
    for t in range(1, 301):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        act[3] = act[0]
        env.act(act)
        g = gpu_obs(env)
        for key in ("rgb", "rew", "first", "level_seed", "prev_level_seed"):
            np.testing.assert_array_equal(g[key][3], g[key][0], err_msg="%s differs at step %d" % (key, t))
        ends += int(g["first"][0])
    env.close()
    assert ends > 0


@pytest.mark.parametrize("mode", ["all", "default", "jumper_caveflyer", "inband"])
def test_prefetch_mixed_batch(mode, prefetch, monkeypatch):
    """A mixed batch with the prefetch forced on for every game ("all": every game's chain requests and
    swaps its own spares, one ring slot per act, cleared once for all games), with the default (off in a
    mixed batch) and with PROCGEN_MI355X_PREFETCH_GAMES=jumper,caveflyer (only those chains use spares,
    the others reset in line), and with PROCGEN_MI355X_PREFETCH_INBAND=1 on top (those chains' level
    generation runs as one job on a chain stream after every chain, not on the prefetch stream); parity per
    env against the oracle."""
    from oracle_lib import OracleEnv
    if mode == "all":
        prefetch()
    elif mode in ("jumper_caveflyer", "inband"):
        monkeypatch.setenv("PROCGEN_MI355X_PREFETCH_GAMES", "jumper,caveflyer")
        if mode == "inband":
            monkeypatch.setenv("PROCGEN_MI355X_PREFETCH_INBAND", "1")
    names = ["caveflyer", "coinrun", "jumper", "maze"]
    num = 8
    env = make_gpu(num, ",".join(names), num_levels=0, rand_seed=6)
    orcs = [OracleEnv(names[n % len(names)], 1, env_offset=n, num_levels=0, rand_seed=6) for n in range(num)]
    rng = np.random.RandomState(7)
    for t in range(1, 241):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        env.act(act)
        g = gpu_obs(env)
        for n, o in enumerate(orcs):
            o.step(act[n:n + 1])
            assert_same(g, o.observe(), t, idx=slice(n, n + 1))
    env.close()
