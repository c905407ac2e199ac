"""Multi-rank sharding on CPU (gloo, world_size 2).

The GPU path shards envs by contiguous global index range: rank r owns
[r*E, (r+1)*E) and seeds each env's level-seed generator with the global index's draw of
rand_seed's MT (vecgame.cpp:349-362), so results are independent of the rank count.  Here
each rank runs its shard with the oracle (same env_offset contract as libenv_make's
`env_offset` option), the observations are concatenated with an all_gather (the only
collective the north star allows), and rank 0 checks the result against one unsharded
2E-env run.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

E = 3
STEPS = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "procgen-1_amd"))
    from oracle_lib import OracleEnv, hashed_actions
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = OracleEnv("coinrun", E, env_offset=rank * E, num_levels=50, rand_seed=3)
    ids = np.arange(rank * E, (rank + 1) * E)
    frames, rews = [], []
    for t in range(STEPS + 1):
        if t:
            env.step(hashed_actions(99, ids, t))
        o = env.observe()
        local = torch.from_numpy(o["rgb"].copy())
        gathered = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        lr = torch.from_numpy(o["rew"].copy())
        gr = [torch.empty_like(lr) for _ in range(world)]
        dist.all_gather(gr, lr)
        if rank == 0:
            frames.append(torch.cat(gathered).numpy())
            rews.append(torch.cat(gr).numpy())
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put((np.stack(frames), np.stack(rews)))


def test_two_rank_shards_equal_one_unsharded_run():
    from oracle_lib import OracleEnv, hashed_actions
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames, rews = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = OracleEnv("coinrun", world * E, num_levels=50, rand_seed=3)
    ids = np.arange(world * E)
    for t in range(STEPS + 1):
        if t:
            ref.step(hashed_actions(99, ids, t))
        o = ref.observe()
        np.testing.assert_array_equal(frames[t], o["rgb"])
        np.testing.assert_array_equal(rews[t], o["rew"])


def _worker_double_buffered(rank, world, port, q):
    """procgen_amd.gather.ObsGather over gloo: step t renders into local[t % 2] and is gathered
    while step t+1 is issued; step t's gathered frames are read only after step t+1 was issued,
    so a missing double buffer would show step t+1's frames instead."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "procgen-1_amd"))
    from oracle_lib import OracleEnv, hashed_actions
    from procgen_amd.gather import ObsGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = OracleEnv("coinrun", E, env_offset=rank * E, num_levels=50, rand_seed=3)
    ids = np.arange(rank * E, (rank + 1) * E)
    target = {}
    g = ObsGather(E, world=world, dist=dist, device="cpu", bind=lambda t: target.__setitem__("buf", t))

    def act(t):
        def run():
            if t:
                env.step(hashed_actions(99, ids, t))
            target["buf"].copy_(torch.from_numpy(env.observe()["rgb"]))
        return run

    frames = []
    pending = None
    for t in range(STEPS + 2):
        k = g.step(act(t)) if t <= STEPS else None
        if pending is not None:
            frames.append(g.result(pending).numpy().copy())  # step t-1, read after step t was issued
            g.release(pending)
        pending = k
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put(np.stack(frames))


def test_double_buffered_gather_matches_unsharded_run():
    from oracle_lib import OracleEnv, hashed_actions
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_double_buffered, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert frames.shape[0] == STEPS + 1
    ref = OracleEnv("coinrun", world * E, num_levels=50, rand_seed=3)
    ids = np.arange(world * E)
    for t in range(STEPS + 1):
        if t:
            ref.step(hashed_actions(99, ids, t))
        np.testing.assert_array_equal(frames[t], ref.observe()["rgb"], err_msg="step %d" % t)
