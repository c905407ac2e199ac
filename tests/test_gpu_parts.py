"""A single-game act split into parts (PROCGEN_MI355X_PARTS, pg_capi.cpp launch_step chains): each
contiguous env range runs its own step -> reset -> render chain on its own stream, with its reset
queue, slow-env list and spare requests in its own PGDev slot.  Envs are independent, so the result
must be exactly the unsplit one: parity against the oracle step for step, uneven part sizes, with and
without the level prefetch, latent info included."""
import numpy as np
import pytest

from test_gpu_games import LATENT, make_gpu, run_pair

pytestmark = pytest.mark.gpu


@pytest.fixture
def parts(monkeypatch):
    def on(n, prio=False):
        monkeypatch.setenv("PROCGEN_MI355X_PARTS", str(n))
        if prio:
            monkeypatch.setenv("PROCGEN_MI355X_PART_PRIO", "1")
    return on


@pytest.mark.parametrize("game,n", [("coinrun", 3), ("caveflyer", 2), ("maze", 4), ("bigfish", 3)])
def test_parts_parity(game, n, parts):
    parts(n)
    kw = dict(distribution_mode="easy") if game == "maze" else {}
    episodes, _ = run_pair(game, 200, 150, seed=31, num_levels=0, rand_seed=5, latent=game in LATENT, **kw)
    if game != "maze":
        assert episodes > 0


def test_parts_priority_and_prefetch(parts, monkeypatch):
    parts(4, prio=True)
    monkeypatch.setenv("PROCGEN_MI355X_PREFETCH", "1")
    run_pair("jumper", 256, 120, seed=32, num_levels=50, start_level=3, rand_seed=2)


def test_parts_reported(parts):
    parts(3)
    env = make_gpu(200, "coinrun", num_levels=0, rand_seed=1)
    assert env.num_parts() == 3
    env.close()
    env = make_gpu(64, "coinrun", num_levels=0, rand_seed=1)  # too few envs: one chain
    assert env.num_parts() == 1
    env.close()


@pytest.mark.parametrize("serial", ["1", "0"])
def test_parts_host_buffers_set_state_before_observe(serial, parts, monkeypatch):
    """Host buffers with 3 parts, PROCGEN_MI355X_HOST_SERIAL on and off: each part's observations leave
    on the copy stream as soon as it rendered (pg_capi.cpp launch_step).  A set_state between act and
    observe re-renders (vecgame.cpp:503): observe must return the restored env's frame and step data,
    not the early copy of the act's -- env 5 takes env 0's state and then plays env 0's game."""
    parts(3)
    monkeypatch.setenv("PROCGEN_MI355X_HOST_SERIAL", serial)
    from test_gpu_coinrun import gpu_obs
    num = 200
    env = make_gpu(num, "coinrun", num_levels=0, rand_seed=6)
    assert env.num_parts() == 3
    rng = np.random.RandomState(7)
    for t in range(1, 41):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        act[5] = act[0]
        env.act(act)
        if t % 10 == 0:
            st = env.get_state()
            st[5] = st[0]
            env.set_state(st)
        g = gpu_obs(env)
        if t >= 10:
            for key in ("rgb", "rew", "first", "level_seed", "prev_level_seed", "prev_level_complete"):
                np.testing.assert_array_equal(g[key][5], g[key][0], err_msg="%s differs at step %d" % (key, t))
    env.close()


def test_parts_two_prefetch_streams(parts, monkeypatch):
    """PROCGEN_MI355X_PREFETCH_STREAMS=2 with parts: acts a and a+1 generate spares on different streams,
    and act a+1's generation must wait for act a's whichever chain is enqueued first (host_serial
    enqueues part 1 before part 0)."""
    parts(3)
    monkeypatch.setenv("PROCGEN_MI355X_PREFETCH", "1")
    monkeypatch.setenv("PROCGEN_MI355X_PREFETCH_STREAMS", "2")
    episodes, _ = run_pair("caveflyer", 192, 150, seed=33, num_levels=0, rand_seed=4)
    assert episodes > 0
