"""GPU parity at the full per-GPU sizes of BASELINE configs 4 and 5:

* C5: all 16 games mixed, 524,288 envs sharded 8 x 65,536.  One GPU runs a full 65,536-env shard
  at env_offset r * 65,536 (r = 0 and r = 7, the first and last shard): env n plays game
  n % 16 and draws the n-th level-seed-generator seed (vecgame.cpp:349-362), so these are the
  envs of the 8-GPU job;
* C4 combined: maze + heist in one vec env, 2 x 32,768 envs.

Device-resident stepping (procgen_act_hashed: on-device counter-hash actions, the same hash
oracle_lib.hashed_actions computes), sampled envs copied out with procgen_read_envs, compared
bit-exact every step with the oracle running those global envs alone.
"""
import numpy as np
import pytest

from oracle_lib import OracleEnv, hashed_actions
from test_gpu_coinrun import assert_same

pytestmark = pytest.mark.gpu

ENV_NAMES = ["bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot",
             "heist", "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot"]


def run_sampled(names, num, offset, sample, steps, seed, rand_seed=0):
    from procgen_amd import ProcgenGym3Env
    env = ProcgenGym3Env(num=num, env_name=",".join(names), num_levels=0, rand_seed=rand_seed,
                         env_offset=offset, device_buffers=True)
    sample = np.asarray(sample, np.int32)
    glob = offset + sample.astype(np.int64)
    orcs = [OracleEnv(names[int(n) % len(names)], 1, env_offset=int(n), num_levels=0, rand_seed=rand_seed)
            for n in glob]
    g = env.read_envs(sample)
    for k, o in enumerate(orcs):
        assert_same(g, o.observe(), 0, idx=slice(k, k + 1))
    episodes = 0
    for t in range(1, steps + 1):
        env.act_hashed(seed, t)
        g = env.read_envs(sample)
        act = hashed_actions(seed, glob, t)
        for k, o in enumerate(orcs):
            o.step(act[k:k + 1])
            try:
                assert_same(g, o.observe(), t, idx=slice(k, k + 1))
            except AssertionError as e:
                raise AssertionError("%s\n  local env %d = global env %d (%s)" % (
                    e, sample[k], glob[k], names[int(glob[k]) % len(names)]))
        episodes += int(g["first"].sum())
    env.close()
    return episodes


@pytest.mark.parametrize("shard", [0, 7])
def test_c5_all16_mixed_full_shard(shard):
    num = 65536
    # every game at the start, the end and the middle of the shard (48 envs, 3 per game)
    sample = list(range(16)) + list(range(num // 2, num // 2 + 16)) + list(range(num - 16, num))
    eps = run_sampled(ENV_NAMES, num, shard * num, sample, 150, seed=0xC5C5 + shard)
    assert eps > 0


def test_c4_maze_heist_combined():
    num = 65536  # 32,768 of each (env n plays names[n % 2])
    sample = [0, 1, 2, 3, 4095, 4096, 32767, 32768, 50001, 50002, num - 2, num - 1]
    eps = run_sampled(["maze", "heist"], num, 0, sample, 520, seed=0xC4)  # maze times out at 500 (maze.cpp:22)
    assert eps > 0


def test_double_buffered_gather_on_device():
    """procgen_amd.gather.ObsGather with the HIP engine (world 1: the gather is a device copy on
    the communication stream): step t's gathered frames, read after step t+1 was issued, are step
    t's frames (sampled envs vs the oracle), and the engine keeps alternating its render target."""
    import torch
    from procgen_amd import ProcgenGym3Env
    from procgen_amd.gather import ObsGather
    torch.cuda.set_device(0)
    num = 4096
    names = ENV_NAMES
    env = ProcgenGym3Env(num=num, env_name=",".join(names), num_levels=0, rand_seed=5, device_buffers=True)
    dp = env.device_ptrs()
    g = ObsGather(num, engine_stream=torch.cuda.ExternalStream(dp.stream),
                  bind=lambda t: env.set_obs_buffer(None if t is None else t.data_ptr()),
                  alive=env.is_open)
    sample = np.array([0, 1, 2, 3, 17, 33, 1000, 2047, 4095], np.int32)
    orcs = [OracleEnv(names[int(n) % 16], 1, env_offset=int(n), num_levels=0, rand_seed=5) for n in sample]
    seed = 0xD8
    pending = None
    for t in range(1, 82):
        k = g.step(lambda: env.act_hashed(seed, t)) if t <= 80 else None
        if pending is not None:
            tp, kp = pending
            got = g.result(kp)[torch.from_numpy(sample).long().cuda()].cpu().numpy()
            g.release(kp)
            act = hashed_actions(seed, sample, tp)
            for j, o in enumerate(orcs):
                o.step(act[j:j + 1])
                np.testing.assert_array_equal(got[j], o.observe()["rgb"][0], err_msg="step %d env %d" % (tp, sample[j]))
        pending = (t, k) if k is not None else None
    torch.cuda.synchronize()
    g.close()  # unbinds: the engine renders into its own tensor again
    env.act_hashed(seed, 82)
    env.wait()
    env.close()
