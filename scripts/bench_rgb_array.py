#!/usr/bin/env python3
"""render_mode="rgb_array" cost (vecgame.cpp:318-330, 415-423): every observe paints each env's
current state again at 512 x 512 (Game::render_to_buf with antialiasing, game.cpp:97-107) and hands
the 786,432-byte RGB888 frame to the caller in info["rgb"].  Here: pg_render_hires_kernel<G> (one
256-thread workgroup per env, the 1 MB RGB32 frame in HBM, then bgr32_to_rgb888 into a 786 KB
device plane) and the device -> host copy into the info buffers.

Prints one JSON line: act + observe rate of ProcgenGym3Env(render_mode="rgb_array") at --num-envs,
the same without rgb_array (the 64 x 64 observation alone), and the per-observe milliseconds they
differ by.  The kernel's own duration and HBM bytes come from rocprofv3 over this script
(scripts/gpu_r05c.sh: --kernel-trace --stats, FETCH_SIZE, WRITE_SIZE passes).

    python3 scripts/bench_rgb_array.py --env-name coinrun --num-envs 4096 --steps 6
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

FRAME_RGB = 512 * 512 * 3
FRAME_RGB32 = 512 * 512 * 4


def run(game, n, steps, render_mode):
    import numpy as np
    from procgen_amd import ProcgenGym3Env
    kw = dict(render_mode=render_mode) if render_mode else {}
    env = ProcgenGym3Env(num=n, env_name=game, num_levels=0, start_level=0, rand_seed=0, reuse_arrays=True, **kw)
    rng = np.random.RandomState(0)
    acts = rng.randint(0, 15, size=(steps + 2, n)).astype(np.int32)
    for k in range(2):
        env.act(acts[k])
        env.observe()
        env.get_info_arrays()
    t0 = time.perf_counter()
    for k in range(steps):
        env.act(acts[2 + k])
        env.observe()
        info = env.get_info_arrays()
    dt = time.perf_counter() - t0
    if render_mode:
        assert info["rgb"].shape == (n, 512, 512, 3)
    env.close()
    return dt / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env-name", default="coinrun")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    t_rgb = run(args.env_name, args.num_envs, args.steps, "rgb_array")
    t_obs = run(args.env_name, args.num_envs, args.steps, None)
    n = args.num_envs
    extra = t_rgb - t_obs
    print(json.dumps({
        "what": "render_mode=rgb_array: act + observe + get_info of ProcgenGym3Env (host buffers, reuse_arrays)",
        "env_name": args.env_name, "num_envs": n, "steps": args.steps,
        "ms_per_step_rgb_array": round(t_rgb * 1e3, 3), "ms_per_step_obs_only": round(t_obs * 1e3, 3),
        "ms_rgb_array_per_observe": round(extra * 1e3, 3),
        "frames_per_s": round(n / extra, 1) if extra > 0 else None,
        "info_rgb_GBps": round(n * FRAME_RGB / extra / 1e9, 3) if extra > 0 else None,
        "bytes_per_frame": {"rgb32_frame_hbm": FRAME_RGB32, "rgb888_plane": FRAME_RGB, "d2h": FRAME_RGB},
    }), flush=True)


if __name__ == "__main__":
    main()
