#!/usr/bin/env python3
"""Diagnostic: rebuild the 65,536-env engine several times in one process (with small engines
of other options in between, as the GPU test file does) and compare the first steps of the
first envs across trials -- frames and get_state snapshots.  Debug aid, not a test."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
from oracle_lib import hashed_actions  # noqa: E402
from procgen_amd import ProcgenGym3Env  # noqa: E402

WATCH = 16


def small_engines():
    for kw in [dict(num_levels=50, rand_seed=1, distribution_mode="easy", center_agent=False),
               dict(num_levels=10, rand_seed=2, use_backgrounds=False, restrict_themes=True)]:
        e = ProcgenGym3Env(num=8, env_name="coinrun", **kw)
        rng = np.random.RandomState(0)
        for _ in range(50):
            e.act(rng.randint(0, 15, size=8))
            e.observe()
        e.close()


def trial(steps):
    num = 65536
    env = ProcgenGym3Env(num=num, env_name="coinrun", num_levels=200, start_level=0, rand_seed=0)
    ids = np.arange(num)
    frames, states = [], []
    for t in range(steps + 1):
        if t:
            env.act(hashed_actions(0x5EED, ids, t))
        _, ob, _ = env.observe()
        frames.append(ob["rgb"][:WATCH].copy())
        states.append([bytes(env.get_state_one(i)) if hasattr(env, "get_state_one") else None for i in range(2)])
    env.close()
    return frames, states


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ref = None
    for k in range(trials):
        if k % 2 == 1:
            small_engines()
        frames, _ = trial(steps)
        if ref is None:
            ref = frames
            print("trial 0 recorded", flush=True)
            continue
        bad = 0
        for t in range(steps + 1):
            d = np.argwhere(np.any(frames[t] != ref[t], axis=-1))
            if len(d):
                bad += 1
                envs = sorted(set(d[:, 0].tolist()))
                print("trial %d step %d: %d px differ in envs %s; first %s" % (k, t, len(d), envs, d[:6].tolist()))
                for e, r, c in d[:6]:
                    print("   env %d (%d,%d) now %s ref %s" % (e, r, c, frames[t][e, r, c].tolist(), ref[t][e, r, c].tolist()))
        print("trial %d: %s" % (k, "identical" if not bad else "%d frames differ" % bad), flush=True)


if __name__ == "__main__":
    main()
