#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the MI355X Procgen engine (BASELINE.json metric).

Workload (BASELINE.json configs[1], the default): coinrun, num_envs = 65,536 per GPU, start_level=0,
num_levels=200, hard, center_agent, backgrounds -- ProcgenGym3Env defaults
(procgen/env.py:229-246) -- with uniform random actions from an on-device counter hash
(splitmix64).  One "step" = one libenv act on every env: game step + auto-reset/level
generation + 64x64 render into the HBM-resident observation tensor.

    python bench.py --gpus N --steps K --warmup W
    python bench.py --env-name bigfish                      (configs[2]; maze / heist: --num-envs 32768)
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Each rank owns the contiguous global env range [rank*E, (rank+1)*E) (level-seed draws of
the global index, vecgame.cpp:349-362); there is no data-path collective (weak scaling).
Rank 0 prints ONE JSON line.  Extra fields: ``roofline`` (render kernel = the obs writer:
12,288 algorithmic bytes per env-step) and ``cpu_baseline`` (the
CPU oracle on this host's cores, bounded sample).
"""
import argparse
import glob
import json
import multiprocessing as mp
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

OBS_BYTES = 64 * 64 * 3
HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md: 8 TB/s spec


def _cpu_worker(args):
    n_envs, steps, seed, game, num_levels = args
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import numpy as np
    from oracle_lib import OracleEnv
    env = OracleEnv(game, n_envs, num_levels=num_levels, start_level=0, rand_seed=seed)
    rng = np.random.RandomState(seed)
    acts = rng.randint(0, 15, size=(steps, n_envs)).astype(np.int32)
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(acts[t])
    return time.perf_counter() - t0


def cpu_baseline(game, num_levels, max_workers=16, steps=12000):
    """The CPU oracle (scalar C restatement of the reference step path, parity-checked)
    on this host: `cores` worker processes, each 64 envs x `steps` random steps (~10 s of
    CPU work per worker for coinrun)."""
    cores = min(len(os.sched_getaffinity(0)), max_workers)
    envs = 64
    with mp.get_context("spawn").Pool(cores) as pool:
        t0 = time.perf_counter()
        times = pool.map(_cpu_worker, [(envs, steps, 1000 + i, game, num_levels) for i in range(cores)])
        wall = time.perf_counter() - t0
    rate = cores * envs * steps / max(times)
    return {"value": round(rate, 1), "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": "%s %d envs x %d random steps per worker, %d worker processes (oracle/procgen_oracle.c, "
                      "-O2 -march=x86-64 -ffp-contract=off); rate = total env-steps / slowest worker "
                      "(%.1f s wall, slowest worker %.1f s)" % (game, envs, steps, cores, wall, max(times))}


def pmc_traffic():
    """HBM bytes per render launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        return d.get("render_hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--env-name", default="coinrun",
                    help="game (or comma list = mixed batch); the headline metric is coinrun (BASELINE configs[1])")
    ap.add_argument("--num-levels", type=int, default=None,
                    help="default: 200 for coinrun (configs[1]), 0 = unbounded otherwise (SURVEY 8d)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="after every step, RCCL all-gather of every rank's uint8[E,64,64,3] obs shard into a "
                         "[N*E,64,64,3] tensor on each rank (north star's obs concatenation; SURVEY 8(e))")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist
    else:
        torch.cuda.set_device(0)

    from procgen_amd import ProcgenGym3Env
    E = args.num_envs
    game = args.env_name
    num_levels = args.num_levels if args.num_levels is not None else (200 if game == "coinrun" else 0)
    env = ProcgenGym3Env(num=E, env_name=game, num_levels=num_levels, start_level=0, rand_seed=0,
                         distribution_mode="hard", device_buffers=True, env_offset=rank * E)
    seed = 0x5EED
    gather = None
    if args.gather:
        # the engine's HBM obs shard as a torch tensor (no copy), gathered on the engine's own stream so
        # the collective is ordered after the render of the same step and before the next step's
        dp = env.device_ptrs()

        class _Shard:
            __cuda_array_interface__ = {"shape": (E, 64, 64, 3), "typestr": "|u1", "data": (dp.rgb, False),
                                        "version": 2}

        local = torch.as_tensor(_Shard(), device="cuda")
        gathered = torch.empty((world * E, 64, 64, 3), dtype=torch.uint8, device="cuda")
        stream = torch.cuda.ExternalStream(dp.stream)

        def gather():
            with torch.cuda.stream(stream):
                if dist is not None:
                    dist.all_gather_into_tensor(gathered, local)
                else:
                    gathered.copy_(local)

    def step(t):
        env.act_hashed(seed, t)
        if gather is not None:
            gather()

    t = 0
    for _ in range(args.warmup):
        t += 1
        step(t)
    env.wait()

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    env.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t += 1
        step(t)
    env.wait()
    barrier()
    elapsed = time.perf_counter() - t0
    n_timed, kt = env.kernel_times()  # ms: step, reset, render, total per step
    env.set_timing(False)

    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    total_steps = world * E * args.steps
    value = total_steps / elapsed
    ms_per_step = elapsed * 1000 / args.steps

    if rank == 0:
        names = ["pg_step_kernel", "pg_reset_kernel", "pg_render_kernel"]
        dom = max(range(3), key=lambda i: kt[i])
        render_ms = kt[2]
        algo_bytes = E * OBS_BYTES  # per render launch: every env's 64x64x3 obs write
        achieved = algo_bytes / (render_ms * 1e-3) if render_ms > 0 else 0.0
        traffic = pmc_traffic()
        roof = {"bound": "hbm", "kernel": names[2], "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 5), "traffic": traffic,
                "algorithmic_bytes_per_launch": algo_bytes,
                "kernel_ms": {"step": round(kt[0], 4), "reset": round(kt[1], 4), "render": round(kt[2], 4)},
                "dominant_kernel": names[dom], "timed_launches": n_timed}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(game.split(",")[0], num_levels)
            except Exception as e:  # the baseline must never hide the GPU number
                cpu = {"error": repr(e)}
        line = {
            "metric": "env-steps/sec at num_envs=65536 (1/2/4/8 GPU) + obs/reward parity vs CPU ref",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
            "config": {"workload": "%s num_envs=%d per GPU, start_level=0 num_levels=%d, hard, "
                                   "center_agent, backgrounds, random actions (device counter hash)"
                                   % (game, E, num_levels),
                       "env_name": game, "num_envs_per_gpu": E, "global_envs": world * E,
                       "parallelism": "env-sharded x%d" % world,
                       "gather": ("rccl all_gather_into_tensor of obs, %d B per rank per step" % (E * OBS_BYTES))
                       if args.gather else None},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    env.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
