#!/usr/bin/env python3
"""Write tests/golden/coinrun_oracle_traj.npz: oracle trajectories of sampled envs of the
65,536-env configuration (BASELINE configs[1]: coinrun, start_level=0, num_levels=200,
rand_seed=0, hard), hashed random actions (seed 0x5EED).  Per step: reward, first,
level seeds and the CRC32 of the 12,288-byte observation; full frames at a few steps.

This fixture pins the ORACLE against silent drift (it is produced by it); the oracle's
link to the reference is pinned separately (tests/test_oracle_pins.py)."""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
import oracle_lib  # noqa: E402

ENVS = [0, 1, 2, 3, 4095, 12345, 65535]
STEPS = 1100
FRAMES = [0, 1, 10, 100, 999, 1000, 1001]
SEED = 0x5EED


def main():
    orcs = [oracle_lib.OracleEnv("coinrun", 1, env_offset=e, num_levels=200, start_level=0, rand_seed=0) for e in ENVS]
    k = len(ENVS)
    rew = np.zeros((STEPS + 1, k), np.float32)
    first = np.zeros((STEPS + 1, k), np.uint8)
    ls = np.zeros((STEPS + 1, k), np.int32)
    pls = np.zeros((STEPS + 1, k), np.int32)
    crc = np.zeros((STEPS + 1, k), np.uint32)
    frames = np.zeros((len(FRAMES), k, 64, 64, 3), np.uint8)
    for t in range(STEPS + 1):
        for j, (e, o) in enumerate(zip(ENVS, orcs)):
            if t:
                o.step(oracle_lib.hashed_actions(SEED, [e], t))
            ob = o.observe()
            rew[t, j], first[t, j] = ob["rew"][0], ob["first"][0]
            ls[t, j], pls[t, j] = ob["level_seed"][0], ob["prev_level_seed"][0]
            crc[t, j] = zlib.crc32(ob["rgb"][0].tobytes())
            if t in FRAMES:
                frames[FRAMES.index(t), j] = ob["rgb"][0]
    out = os.path.join(REPO, "tests", "golden", "coinrun_oracle_traj.npz")
    np.savez_compressed(out, envs=np.array(ENVS, np.int32), steps=np.int32(STEPS), action_seed=np.int64(SEED),
                        rew=rew, first=first, level_seed=ls, prev_level_seed=pls, rgb_crc32=crc,
                        frame_steps=np.array(FRAMES, np.int32), frames=frames)
    print("wrote", out, "episodes ended:", int(first[1:].sum()), "rewards:", float(rew.sum()))


if __name__ == "__main__":
    main()
