"""ProcgenEnv (baselines VecEnv, procgen/env.py:276-290) and make_env (gym, procgen/
gym_registration.py:6-26) over the HIP engine: same frames, rewards and dones as the oracle."""
import numpy as np
import pytest

from oracle_lib import OracleEnv

pytestmark = pytest.mark.gpu


def test_procgen_env_matches_oracle():
    from procgen_amd import ProcgenEnv
    num, steps = 8, 80
    ve = ProcgenEnv(num_envs=num, env_name="coinrun", num_levels=50, start_level=0, rand_seed=3)
    orc = OracleEnv("coinrun", num, num_levels=50, start_level=0, rand_seed=3)
    ob = ve.reset()
    np.testing.assert_array_equal(ob["rgb"], orc.observe()["rgb"])
    rng = np.random.RandomState(5)
    for _ in range(steps):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        ob, rew, done, infos = ve.step(act)
        orc.step(act)
        o = orc.observe()
        np.testing.assert_array_equal(ob["rgb"], o["rgb"])
        np.testing.assert_array_equal(rew, o["rew"])
        np.testing.assert_array_equal(done.astype(np.uint8), o["first"])
        assert len(infos) == num and "level_seed" in infos[0]
    ve.close()


def test_gym_make_env_matches_oracle():
    from procgen_amd import make_env
    ge = make_env(env_name="bigfish", num_levels=0, rand_seed=7)
    orc = OracleEnv("bigfish", 1, num_levels=0, rand_seed=7)
    np.testing.assert_array_equal(ge.reset(), orc.observe()["rgb"][0])
    rng = np.random.RandomState(6)
    for _ in range(60):
        a = int(rng.randint(0, 15))
        ob, rew, done, info = ge.step(a)
        orc.step(np.array([a], np.int32))
        o = orc.observe()
        np.testing.assert_array_equal(ob, o["rgb"][0])
        assert rew == float(o["rew"][0]) and done == bool(o["first"][0])
    ge.close()
