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
