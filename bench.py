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
Rank 0 prints ONE JSON line.  Extra fields: ``roofline`` (12,288 algorithmic bytes per env-step,
SURVEY.md section 8(d), over the dominant kernel's average duration; the render kernel -- the obs
writer -- and the whole step beside it) and ``cpu_baseline`` (the CPU oracle on this host's cores,
bounded sample).
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


def pmc_traffic(game, kernel="pg_render_kernel", field="hbm_bytes_per_launch"):
    """HBM bytes (FETCH_SIZE + WRITE_SIZE) per render launch of `game` from the newest committed
    rocprofv3 PMC summary under profiles/ (separate FETCH_SIZE / WRITE_SIZE passes over this same
    bench command: scripts/gpu_counters.sh -> *counters_summary.json, or the older
    scripts/gpu_profile.sh -> *pmc*.json), or (None, None).  "Newest" = last by path name
    (profiles/r01_v1 ... profiles/r02/r02_x ...), not by file time, which a checkout resets."""
    files = glob.glob(os.path.join(REPO, "profiles", "**", "*pmc*.json"), recursive=True)
    files += glob.glob(os.path.join(REPO, "profiles", "**", "*counters_summary.json"), recursive=True)
    for path in sorted(files, key=lambda p: os.path.relpath(p, REPO), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        if (field == "hbm_bytes_per_launch" and kernel == "pg_render_kernel" and d.get("game", "coinrun") == game
                and d.get("render_hbm_bytes_per_launch")):
            return d["render_hbm_bytes_per_launch"], os.path.relpath(path, os.path.join(REPO, "profiles"))
        g = d.get(game)
        if isinstance(g, dict):
            for kname, k in g.items():
                if kname.startswith(kernel) and isinstance(k, dict) and k.get(field):
                    return k[field], os.path.relpath(path, os.path.join(REPO, "profiles"))
    return None, None


def host_path_rate(game, num_levels, E, steps):
    """The reference's own contract: host buffers (libenv_act reads numpy actions, libenv_observe
    fills numpy obs / rew / first / info after a device->host copy), PCIe included.  Reported
    beside `value` (device-resident obs), never as it.  `value`: gym3 CEnv default semantics
    (observe() returns fresh copies); `reuse_arrays`: CEnv(reuse_arrays=True), the live buffers."""
    import numpy as np
    from procgen_amd import ProcgenGym3Env
    out = {}
    for reuse in (False, True):
        env = ProcgenGym3Env(num=E, env_name=game, num_levels=num_levels, start_level=0, rand_seed=0,
                             distribution_mode="hard", reuse_arrays=reuse)
        rng = np.random.RandomState(0)
        acts = rng.randint(0, 15, size=(steps + 4, E)).astype(np.int32)
        for k in range(4):
            env.act(acts[k])
            env.observe()
        t0 = time.perf_counter()
        for k in range(steps):
            env.act(acts[4 + k])
            rew, ob, first = env.observe()
            info = env.get_info_arrays()
        dt = time.perf_counter() - t0
        env.close()
        out[reuse] = E * steps / dt
    # the PCIe ceiling on this box: one obs plane device -> page-locked host, best of 3
    import torch
    dev = torch.empty(E * OBS_BYTES, dtype=torch.uint8, device="cuda")
    host = torch.empty(E * OBS_BYTES, dtype=torch.uint8, pin_memory=True)
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, dev.numel() / (time.perf_counter() - t0))
    del dev, host
    return {"value": round(out[False], 1), "reuse_arrays": round(out[True], 1), "unit": "env-steps/s",
            "steps": steps, "num_envs": E,
            "obs_GBps": round(out[False] * OBS_BYTES / 1e9, 2), "reuse_obs_GBps": round(out[True] * OBS_BYTES / 1e9, 2),
            "pcie_d2h_GBps": round(best / 1e9, 2),
            "what": "ProcgenGym3Env host mode: act(numpy) + observe() -> numpy rgb/rew/first + info arrays "
                    "(libenv_observe: DMA straight into the page-locked caller buffers; reuse_arrays: the live "
                    "buffers, no host copies); pcie_d2h_GBps: a plain 805 MB device -> pinned copy"}


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
    ap.add_argument("--settle", type=int, default=300,
                    help="untimed steps after the warmup so that episodes, resets and entity lists reach "
                         "steady state before the timed window (reported as settle_steps)")
    ap.add_argument("--host-steps", type=int, default=24,
                    help="steps of the host-buffer (libenv observe -> numpy) path reported as host_path; 0 = skip")
    ap.add_argument("--gather", action="store_true",
                    help="after every step, RCCL all-gather of every rank's uint8[E,64,64,3] obs shard into a "
                         "[N*E,64,64,3] tensor on each rank (north star's obs concatenation; SURVEY 8(e))")
    args = ap.parse_args()
    # stdout carries exactly the one JSON line: everything else written to fd 1 (RCCL's version banner
    # at communicator init, library chatter) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    # --gather under a launcher (WORLD_SIZE set) runs RCCL even at world 1, so the single-GPU line
    # times the same all_gather_into_tensor the 8-GPU node runs
    if world > 1 or (args.gather and "WORLD_SIZE" in os.environ):
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
        # double-buffered obs all-gather (procgen_amd/gather.py): step t renders into local[t % 2]
        # and its RCCL all-gather runs on a communication stream while step t+1 computes
        from procgen_amd.gather import ObsGather
        dp = env.device_ptrs()
        gather = ObsGather(E, world=world, dist=dist, engine_stream=torch.cuda.ExternalStream(dp.stream),
                           bind=lambda buf: env.set_obs_buffer(None if buf is None else buf.data_ptr()),
                           alive=env.is_open)

    def step(t):
        if gather is not None:
            gather.step(lambda: env.act_hashed(seed, t))
        else:
            env.act_hashed(seed, t)

    t = 0
    for _ in range(args.warmup + args.settle):
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
    n_timed, kt, kt_games = env.kernel_times()  # ms: step, reset, render (sums over games), wall span
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
        mixed = len(game.split(",")) > 1
        parts = env.num_parts()  # a single game's act split into chains over env ranges (kernel_times: per part)
        algo_bytes = E * OBS_BYTES // parts  # every env's 64x64x3 obs write, per launch (one part's envs)
        if not mixed:
            # 12,288 algorithmic bytes per env-step (the obs write), E env-steps per
            # launch; `achieved` divides them by the DOMINANT kernel's average in-bench duration (HIP
            # events on the engine stream), and the render kernel (the obs writer itself) and the
            # whole step (ms_per_step) are reported beside it
            dom = max(range(3), key=lambda i: kt[i])
            dom_ms = kt[dom]
            achieved = algo_bytes / (dom_ms * 1e-3) if dom_ms > 0 else 0.0
            traffic, traffic_src = pmc_traffic(game, names[dom], "hbm_bytes_per_part_act")
            roof = {"bound": "hbm", "kernel": names[dom], "achieved": round(achieved / 1e9, 2),
                    "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 5),
                    "traffic": traffic, "traffic_source": traffic_src,
                    "traffic_what": "FETCH_SIZE + WRITE_SIZE of the kernel's launches in one part of one act "
                                    "(the step: 1 launch; the render: modes 1 + 2), like kernel_ms",
                    "algorithmic_bytes_per_launch": algo_bytes,
                    "kernel_ms": {"step": round(kt[0], 4), "reset": round(kt[1], 4), "render": round(kt[2], 4),
                                  "step_wall": round(kt[3], 4)},
                    "dominant_kernel": names[dom], "timed_launches": n_timed}
            # per part-act counter bytes (scripts/counter_summary.py hbm_bytes_per_part_act): the step
            # kernel's one launch, the render's two launches (mode 1 + mode 2) -- matching the kernel
            # times, which are per part with the render's two modes summed
            for i, key in ((2, "render_kernel"), (0, "step_kernel"), (1, "reset_kernel")):
                tr, src = pmc_traffic(game, names[i], "hbm_bytes_per_part_act")
                a = algo_bytes / (kt[i] * 1e-3) if kt[i] > 0 else 0.0
                roof[key] = {"ms": round(kt[i], 4), "achieved": round(a / 1e9, 2), "frac": round(a / HBM_PEAK, 5),
                             "traffic_per_part_act": tr, "traffic_source": src,
                             "traffic_GBps": round(tr / (kt[i] * 1e-3) / 1e9, 2) if tr and kt[i] > 0 else None,
                             "traffic_ratio": round(tr / algo_bytes, 3) if tr else None}
            roof["parts"] = parts
            e2e = E * OBS_BYTES / (ms_per_step * 1e-3)
            tr_all, src_all = pmc_traffic(game, "_all_kernels", "hbm_bytes_per_part_act")
            roof["end_to_end"] = {"ms_per_step": round(ms_per_step, 4), "achieved": round(e2e / 1e9, 2),
                                  "frac": round(e2e / HBM_PEAK, 5),
                                  "act_traffic": tr_all * parts if tr_all else None, "traffic_source": src_all,
                                  "act_traffic_ratio": round(tr_all * parts / (E * OBS_BYTES), 3) if tr_all else None}
        else:
            # a mixed batch runs every game's step -> reset -> render chain concurrently on its own
            # stream: no single kernel's duration is attributable, so the roofline is taken over
            # the step's wall span (fork -> join on the env's stream), i.e. all 16 chains together
            achieved = E * OBS_BYTES / (kt[3] * 1e-3) if kt[3] > 0 else 0.0
            roof = {"bound": "hbm", "kernel": "all games' step+reset+render chains (concurrent streams)",
                    "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK, 5), "traffic": None,
                    "algorithmic_bytes_per_launch": E * OBS_BYTES,
                    "kernel_ms": {"step_wall": round(kt[3], 4),
                                  "sum_over_games": {"step": round(kt[0], 4), "reset": round(kt[1], 4),
                                                     "render": round(kt[2], 4)},
                                  "per_game": {g: [round(x, 4) for x in v] for g, v in kt_games.items()}},
                    "timed_launches": n_timed}
        host = None
        if args.host_steps > 0 and world == 1:
            try:
                host = host_path_rate(game, num_levels, E, args.host_steps)
            except Exception as e:
                host = {"error": repr(e)}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(game.split(",")[0], num_levels)
            except Exception as e:  # the baseline must never hide the GPU number
                cpu = {"error": repr(e)}
        line = {
            "metric": "env-steps/sec at num_envs=65536 (1/2/4/8 GPU) + obs/reward parity vs CPU ref",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "settle_steps": args.settle, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
            "config": {"workload": "%s num_envs=%d per GPU, start_level=0 num_levels=%d, hard, "
                                   "center_agent, backgrounds, random actions (device counter hash)"
                                   % (game, E, num_levels),
                       "env_name": game, "num_envs_per_gpu": E, "global_envs": world * E,
                       "parallelism": "env-sharded x%d" % world,
                       "gather": ("double-buffered rccl all_gather_into_tensor of obs on a comm stream, "
                                  "%d B per rank per step" % (E * OBS_BYTES)) if args.gather else None},
            "roofline": roof,
            "host_path": host,
            "cpu_baseline": cpu,
        }
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    if gather is not None:
        gather.close()
    env.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
