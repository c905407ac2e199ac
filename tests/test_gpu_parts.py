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
