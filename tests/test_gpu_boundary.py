"""GPU checks of the drop-in boundary (include/libenv.h), against the CPU oracle:

* gym3 CEnv's exact call sequence with no extension call (tests/gym3_cenv.py) -- libenv_make
  loads the images itself (vecgame.cpp:144-153);
* several act() calls before one observe() keep their own actions (vecgame.cpp:426-444);
* a state of another game is refused by set_state (game.cpp:259 fassert) and leaves the env intact;
* a shard whose env_offset is not a multiple of the number of names plays the games of the same
  global envs (vecgame.cpp:357-358);
* procgen_upload_atlas can still replace the loaded atlas (same frames).
"""
import numpy as np
import pytest

from oracle_lib import OracleEnv
from test_gpu_coinrun import assert_same, gpu_obs

pytestmark = pytest.mark.gpu

BASE = {"num_levels": 200, "start_level": 0, "num_actions": 15, "rand_seed": 0, "center_agent": True,
        "use_backgrounds": True, "distribution_mode": 1}


def cenv_obs(env):
    rew, ob, first = env.observe()
    info = env.info()
    return dict(rgb=ob["rgb"], rew=rew, first=first, prev_level_seed=info["prev_level_seed"],
                prev_level_complete=info["prev_level_complete"], level_seed=info["level_seed"])


@pytest.mark.parametrize("names", ["coinrun", "maze,heist,jumper,starpilot"])
def test_gym3_cenv_sequence_parity(names):
    from procgen_amd import _lib
    from gym3_cenv import LIBENV_SYMBOLS, CEnv, RecordingLib
    lib = RecordingLib(_lib.LIB_PATH)
    num = 8
    env = CEnv(lib, num, dict(BASE, env_name=names))
    gl = names.split(",")
    orcs = [OracleEnv(gl[n % len(gl)], 1, env_offset=n, num_levels=200, start_level=0, rand_seed=0)
            for n in range(num)]
    rng = np.random.RandomState(4)
    for t in range(0, 121):
        if t:
            act = rng.randint(0, 15, size=num).astype(np.int32)
            env.act(act)
            for n, o in enumerate(orcs):
                o.step(act[n:n + 1])
        g = cenv_obs(env)
        for n, o in enumerate(orcs):
            assert_same(g, o.observe(), t, idx=slice(n, n + 1))
    env.close()
    assert set(lib.looked_up) <= set(LIBENV_SYMBOLS)


def test_back_to_back_acts_keep_their_actions():
    """act(a1); act(a2); act(a3); observe(): three steps with three action vectors."""
    from procgen_amd import ProcgenGym3Env
    num = 16
    env = ProcgenGym3Env(num=num, env_name="coinrun", num_levels=200, start_level=0, rand_seed=0)
    orc = OracleEnv("coinrun", num, num_levels=200, start_level=0, rand_seed=0)
    rng = np.random.RandomState(12)
    env.observe()
    for t in range(1, 41):
        acts = [rng.randint(0, 15, size=num).astype(np.int32) for _ in range(3)]
        for a in acts:
            env._ac["action"][:] = a
            env._lib.libenv_act(env._handle)  # no observe in between
            orc.step(a)
        assert_same(gpu_obs(env), orc.observe(), t)
    env.close()


def test_cross_game_set_state_is_refused():
    from procgen_amd import ProcgenGym3Env
    from procgen_amd.env import ProcgenError
    env = ProcgenGym3Env(num=2, env_name="coinrun,miner", num_levels=20, rand_seed=3)
    for _ in range(5):
        env.act(np.array([3, 4]))
        env.observe()
    states = env.get_state()
    with pytest.raises(ProcgenError):
        env.set_state([states[1], states[0]])  # miner's state into coinrun's slot (a sticky error,
        # as the reference's fassert ends the process)
    # nothing was written: both slots still hold their own state
    assert env.get_state() == states
    env.close()
    env = ProcgenGym3Env(num=2, env_name="coinrun,miner", num_levels=20, rand_seed=3)
    bad = bytearray(states[0])
    bad[8 + 27 * 4:8 + 28 * 4] = np.array([-5], np.int32).tobytes()  # PGEnv.num_ents < 0
    with pytest.raises(ProcgenError):
        env.set_state([bytes(bad), states[1]])
    env.close()


def test_shard_offset_not_multiple_of_names():
    """A 6-env shard at global offset 3 of a 3-name vec env plays names[(3 + e) % 3]."""
    from procgen_amd import ProcgenGym3Env
    names = ["coinrun", "maze", "bigfish"]
    off, num = 3 * 5 + 1, 6
    env = ProcgenGym3Env(num=num, env_name=",".join(names), num_levels=0, rand_seed=9, env_offset=off)
    orcs = [OracleEnv(names[(off + e) % 3], 1, env_offset=off + e, num_levels=0, rand_seed=9) for e in range(num)]
    rng = np.random.RandomState(2)
    for t in range(0, 101):
        if t:
            act = rng.randint(0, 15, size=num).astype(np.int32)
            env.act(act)
            for e, o in enumerate(orcs):
                o.step(act[e:e + 1])
        g = gpu_obs(env)
        for e, o in enumerate(orcs):
            assert_same(g, o.observe(), t, idx=slice(e, e + 1))
    env.close()


def test_uploaded_atlas_matches_loaded_atlas():
    from procgen_amd import ProcgenGym3Env
    names = "coinrun,jumper,chaser"
    a = ProcgenGym3Env(num=6, env_name=names, num_levels=0, rand_seed=5)
    b = ProcgenGym3Env(num=6, env_name=names, num_levels=0, rand_seed=5, upload_atlas=True)
    rng = np.random.RandomState(0)
    for t in range(60):
        if t:
            act = rng.randint(0, 15, size=6)
            a.act(act)
            b.act(act)
        np.testing.assert_array_equal(a.observe()[1]["rgb"], b.observe()[1]["rgb"])
    a.close()
    b.close()
