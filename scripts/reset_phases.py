#!/usr/bin/env python3
"""Level-generation phases of the reset kernel (diagnostic build, make -C procgen-1_amd/csrc
VARIANT=rprof ONLY=pg_reset.hip EXTRA=-DPG_PROF_RESET): average s_memtime cycles per reset of each
phase that pg_reset.hip's RMARK stamps (caveflyer / jumper / leaper), over the resets of a device-resident
run.  Phase shares only: never quote this build's wall time."""
import json
import os
import sys

os.environ.setdefault("PROCGEN_MI355X_LIB", "rprof")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = {
    "caveflyer": ["preamble", "fill+4 updates", "best room (+free list, picks)", "find_path", "expand+4 updates",
                  "object placement", "tail", "write-back"],
    "leaper": ["preamble+lanes", "build loop (spawn + step)", "-", "-", "-", "-", "entities to HBM+tail", "write-back"],
    "jumper": ["maze (no dead ends)", "fill+2 updates+border", "best room+free list+candidates", "find_path",
               "expand", "ordered scans", "preamble+tail", "write-back"],
}


def main(game, num=4096, steps=200):
    torch.cuda.set_device(0)
    from procgen_amd import ProcgenGym3Env, _lib
    lib = _lib.load()
    env = ProcgenGym3Env(num=num, env_name=game, num_levels=0, start_level=0, rand_seed=0, device_buffers=True)
    for t in range(1, steps + 1):
        env.act_hashed(0x5EED, t)
    env.wait()
    raw = np.zeros((num, 16), np.uint64)
    lib.procgen_profile_raw(env._handle, raw.ctypes.data)
    env.close()
    resets = raw[:, 0].astype(np.float64)
    cyc = raw[:, 8:16].astype(np.float64)
    n = resets.sum()
    per = cyc.sum(0) / n
    out = {"game": game, "num_envs": num, "steps": steps, "resets": int(n),
           "cycles_per_reset": {name: round(float(per[k]), 1) for k, name in enumerate(PHASES[game])},
           "total_cycles_per_reset": round(float(per.sum()), 1),
           "slowest_env_cycles_per_reset": round(float((cyc.sum(1) / np.maximum(resets, 1)).max()), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    for g in (sys.argv[1:] or ["jumper", "caveflyer", "leaper"]):
        main(g)
