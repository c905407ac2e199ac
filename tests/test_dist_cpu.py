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


# ---------------------------------------------------------------- the engine's own shard plan
MIXED = ("bigfish,bossfight,caveflyer,chaser,climber,coinrun,dodgeball,fruitbot,heist,jumper,leaper,maze,"
         "miner,ninja,plunder,starpilot")


def _plan(lib, names, n, offset, seed):
    game = np.zeros(n, np.int32)
    lsg = np.zeros(n, np.uint32)
    lists = np.zeros(n, np.int32)
    ng = lib.procgen_shard_plan(names.encode(), n, offset, seed, game.ctypes.data, lsg.ctypes.data, lists.ctypes.data)
    assert ng > 0
    return ng, game, lsg, lists


def _worker_engine_plan(rank, world, port, q, names, E_):
    """Each rank asks the ENGINE (libprocgen_mi355x.so, procgen_shard_plan: the function libenv_make
    builds every env from -- game, level-seed generator seed, mixed-batch chain lists) for its shard
    at env_offset = rank * E_ and all_gathers it; no GPU is touched."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "procgen-1_amd"))
    from procgen_amd import _lib
    lib = _lib.load()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ng, game, lsg, lists = _plan(lib, names, E_, rank * E_, 12345)
    out = []
    # global env index of every local list entry: the chains of a shard must cover the global
    # envs of each game that fall in the shard, in global order
    glob_lists = lists.astype(np.int64) + rank * E_ if ng > 1 else np.zeros(0, np.int64)
    for a in (torch.from_numpy(game.astype(np.int64)), torch.from_numpy(lsg.astype(np.int64)),
              torch.from_numpy(glob_lists)):
        g = [torch.empty_like(a) for _ in range(world)]
        dist.all_gather(g, a)
        out.append([x.numpy() for x in g])
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put((ng, out))


@pytest.mark.parametrize("names,E_", [("coinrun", 64), (MIXED, 128)])
def test_engine_shard_plan_two_ranks(names, E_):
    """2 gloo ranks, each planning its shard with the engine's host code, concatenate to the plan of
    one unsharded 2E-env vec env (vecgame.cpp:349-362, 357-358): same game per global env, same
    level-seed seeds, and per game the two shards' chain lists (in global indices) are the
    unsharded list split at the shard boundary."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "procgen-1_amd"))
    from procgen_amd import _lib
    lib = _lib.load()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_engine_plan, args=(r, world, port, q, names, E_)) for r in range(world)]
    for p in procs:
        p.start()
    ng, (games, seeds, glists) = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ng1, game1, lsg1, lists1 = _plan(lib, names, world * E_, 0, 12345)
    assert ng == ng1
    np.testing.assert_array_equal(np.concatenate(games), game1)
    np.testing.assert_array_equal(np.concatenate(seeds), lsg1.astype(np.int64))
    # the n-th seed is the n-th draw of mt19937(12345): the same stream numpy's MT19937 legacy seeding gives
    rs = np.random.RandomState(12345)
    np.testing.assert_array_equal(lsg1, rs.randint(0, 1 << 32, size=world * E_, dtype=np.uint64).astype(np.uint32))
    if ng > 1:
        per = E_ // ng
        for k in range(ng):
            full = lists1[k * (world * per):(k + 1) * (world * per)]
            split = np.concatenate([glists[r][k * per:(k + 1) * per] for r in range(world)])
            np.testing.assert_array_equal(split, full, err_msg="game %d" % k)
            assert np.all(game1[full] == game1[full[0]])
