"""GPU parity of WHOLE populations at the BASELINE sizes: every env, every step.

The reference runs every env of a vec env as an independent Game seeded with its own draw
(procgen/src/vecgame.cpp:349-378), so BASELINE configs[1]-[3] are 65,536 separate trajectories each.
The sampled full-size tests (test_gpu_coinrun.py, test_gpu_games.py, test_gpu_c5.py) compare a few
envs; here the engine's reward, first, level seeds and a 64-bit digest of every observation
(procgen_read_outputs) are compared with the oracle's for every env at every step, the oracle leg
running in a host worker pool (tests/population.py) while the GPU leg runs.  Scale-only paths are
covered by construction: the slow-env launch order, the two-part coinrun split, reset-queue pressure,
and -- with PROCGEN_MI355X_HEAVY_US=0 -- every env on the slow list (past PG_HEAVY_CAP) with host
buffers.
"""
import numpy as np
import pytest

from oracle_lib import hashed_actions
from population import KEYS, OraclePopulation, compare, obs_digest

pytestmark = pytest.mark.gpu


def engine_population(names, num, steps, seed, **kw):
    from procgen_amd import ProcgenGym3Env
    env = ProcgenGym3Env(num=num, env_name=",".join(names), device_buffers=True, **kw)
    out = {k: [] for k in KEYS}
    episodes = 0
    for t in range(steps + 1):
        if t:
            env.act_hashed(seed, t)
        r = env.read_outputs()
        for k in KEYS:
            out[k].append(r[k])
        episodes += int(r["first"].sum()) if t else 0
    env.close()
    return {k: np.stack(v) for k, v in out.items()}, episodes


def run_population(names, num, steps, seed, **kw):
    orc = OraclePopulation(names, num, steps, seed, **kw)  # starts the host workers first
    eng, episodes = engine_population(names, num, steps, seed, **kw)
    compare(eng, orc.result(), names)
    return episodes


def test_c2_coinrun_whole_population():
    """configs[1]: coinrun, 65,536 envs, start_level 0, num_levels 200 -- all 65,536 envs x 200 steps
    (the default 2-part split, the slow-env launch order and the crate-pile envs of
    test_gpu_coinrun.CRATE_PILE_ENVS included)."""
    eps = run_population(["coinrun"], 65536, 200, 0xC2, num_levels=200, start_level=0, rand_seed=0)
    assert eps > 1000  # resets at scale: the reset queue and the mode-2 renders


def test_c3_bigfish_whole_population():
    """configs[2]: bigfish (float-position entities, many-entity collisions), 65,536 envs x 100 steps."""
    eps = run_population(["bigfish"], 65536, 100, 0xC3, num_levels=0, rand_seed=0)
    assert eps > 0


def test_c4_maze_heist_whole_population():
    """configs[3]: maze + heist, 32,768 envs each (one batch, env n plays maze / heist by n % 2) x 100 steps."""
    eps = run_population(["maze", "heist"], 65536, 100, 0xC4, num_levels=0, rand_seed=0)
    assert eps > 0


def test_coinrun_every_env_slow_host_buffers(monkeypatch):
    """PROCGEN_MI355X_HEAVY_US=0 lists every env as slow on every act (16,384 envs: the slow list
    overflows PG_HEAVY_CAP = 2,048, so both launch-order paths run), with the default 2-part split and
    gym3's host buffers (libenv_observe copies every part's outputs): every env x 120 steps."""
    from procgen_amd import ProcgenGym3Env
    monkeypatch.setenv("PROCGEN_MI355X_HEAVY_US", "0")
    num, steps, seed = 16384, 120, 0x51
    kw = dict(num_levels=200, start_level=0, rand_seed=3)
    orc = OraclePopulation(["coinrun"], num, steps, seed, **kw)
    env = ProcgenGym3Env(num=num, env_name="coinrun", **kw)
    assert env.num_parts() == 2
    ids = np.arange(num)
    out = {k: [] for k in KEYS}
    for t in range(steps + 1):
        if t:
            env.act(hashed_actions(seed, ids, t))
        rew, ob, first = env.observe()
        info = env.get_info()
        out["obs_digest"].append(obs_digest(ob["rgb"]))
        out["rew"].append(rew.astype(np.float32))
        out["first"].append(first.astype(np.uint8))
        for k in ("prev_level_seed", "prev_level_complete", "level_seed"):
            out[k].append(np.array([i[k] for i in info], np.int32 if "seed" in k else np.uint8))
    env.close()
    compare({k: np.stack(v) for k, v in out.items()}, orc.result(), ["coinrun"])
