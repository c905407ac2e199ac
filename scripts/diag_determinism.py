#!/usr/bin/env python3
"""Diagnostic: run two identical 65,536-env engines side by side and report the first step
and envs where their outputs differ (any difference is nondeterminism).  Debug aid."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
from procgen_amd import ProcgenGym3Env  # noqa: E402


def snap(env):
    rew, ob, first = env.observe()
    return rew.copy(), ob["rgb"].copy(), first.copy()


def main():
    num = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    a = ProcgenGym3Env(num=num, env_name="coinrun", num_levels=200, start_level=0, rand_seed=0)
    b = ProcgenGym3Env(num=num, env_name="coinrun", num_levels=200, start_level=0, rand_seed=0)
    rng = np.random.RandomState(1)
    nbad = 0
    for t in range(steps + 1):
        if t:
            act = rng.randint(0, 15, size=num).astype(np.int32)
            a.act(act)
            b.act(act)
        ra, oa, fa = snap(a)
        rb, ob, fb = snap(b)
        bad_env = np.nonzero(np.any(oa.reshape(num, -1) != ob.reshape(num, -1), axis=1) | (ra != rb) | (fa != fb))[0]
        if len(bad_env):
            nbad += len(bad_env)
            print("step %d: %d envs differ, e.g. %s" % (t, len(bad_env), bad_env[:8].tolist()))
            for e in bad_env[:3]:
                d = np.argwhere(np.any(oa[e] != ob[e], axis=-1))
                print("   env %d rew %s/%s first %s/%s, %d px, first px %s" %
                      (e, ra[e], rb[e], fa[e], fb[e], len(d), d[:4].tolist()))
            if nbad > 50:
                break
    print("done: %d env-frames differ" % nbad)


if __name__ == "__main__":
    main()
