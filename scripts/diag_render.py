#!/usr/bin/env python3
"""Diagnostic: find frames where the engine's RGB differs from the oracle and print the
differing pixels (engine vs oracle) plus the agent state.  Debug aid, not a test."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
from oracle_lib import OracleEnv, hashed_actions  # noqa: E402
from procgen_amd import ProcgenGym3Env  # noqa: E402


def report(tag, g, o, limit=12):
    diff = np.argwhere(np.any(g != o, axis=-1))
    print("%s: %d pixels differ" % (tag, len(diff)))
    for r, c in diff[:limit]:
        print("   (%2d,%2d) gpu %s oracle %s" % (r, c, g[r, c].tolist(), o[r, c].tolist()))


def main():
    num = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sample = [0, 1, 2, 63, 64, 1000, 4095, 12345, 30000, 32767, 32768, 50001, 65534, 65535]
    sample = [k for k in sample if k < num]
    env = ProcgenGym3Env(num=num, env_name="coinrun", num_levels=200, start_level=0, rand_seed=0)
    orcs = [OracleEnv("coinrun", 1, env_offset=i, num_levels=200, rand_seed=0) for i in sample]
    ids = np.arange(num)
    bad = 0
    for t in range(0, steps + 1):
        if t:
            act = hashed_actions(0x5EED, ids, t)
            env.act(act)
        _, ob, _ = env.observe()
        for k, o in zip(sample, orcs):
            if t:
                o.step(act[k:k + 1])
            orgb = o.observe()["rgb"][0]
            if not np.array_equal(ob["rgb"][k], orgb):
                bad += 1
                report("step %d env %d" % (t, k), ob["rgb"][k], orgb)
                if bad > 6:
                    return
    print("done, %d bad frames" % bad)


if __name__ == "__main__":
    main()
