#!/usr/bin/env python3
"""Per-phase cycle breakdown of the step and render kernels (diagnostic build).

Runs the bench workload on libprocgen_mi355x_prof.so (make -C procgen-1_amd/csrc PROFILE=1),
whose kernels accumulate s_memtime deltas per phase; prints the average cycles per env-step
of each phase.  Phase shares only -- the stamps themselves cost time (cdna_hip_programming.md
section 7, In-kernel stamps), so never quote this build's wall time."""
import os
import sys
import json

os.environ.setdefault("PROCGEN_MI355X_LIB", "prof")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

STEP = ["rng+action", "set_action+velocity", "step_entities", "collisions", "erase", "trails", "finish", "ilist+nonsmart"]
RENDER = ["setup tables", "bg+fast tiles", "generic tiles", "entity setup", "entity stamping", "overlays", "output",
          "setup env+window"]


def main(game="coinrun", num=65536, warm=20, steps=50):
    torch.cuda.set_device(0)
    from procgen_amd import ProcgenGym3Env, _lib
    lib = _lib.load()
    env = ProcgenGym3Env(num=num, env_name=game, num_levels=200 if game == "coinrun" else 0, start_level=0,
                         rand_seed=0, device_buffers=True)
    for t in range(1, warm + 1):
        env.act_hashed(0x5EED, t)
    env.wait()
    a = np.zeros(16, np.uint64)
    lib.procgen_profile_read(env._handle, a.ctypes.data)
    for t in range(warm + 1, warm + steps + 1):
        env.act_hashed(0x5EED, t)
    env.wait()
    b = np.zeros(16, np.uint64)
    lib.procgen_profile_read(env._handle, b.ctypes.data)
    d = (b - a).astype(np.float64) / (num * steps)
    out = {"game": game, "cycles_per_env_step": {"step": {n: round(d[k], 1) for k, n in enumerate(STEP)},
                                   "render": {n: round(d[8 + k], 1) for k, n in enumerate(RENDER)}}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    for g in (sys.argv[1:] or ["coinrun"]):
        main(g)
