#!/usr/bin/env python3
"""Smart-entity census of the step kernel (diagnostic build, never the product):
  make -C procgen-1_amd/csrc VARIANT=smart EXTRA="-DPG_PROFILE -DPG_PROF_SMART"
then PROCGEN_MI355X_LIB=smart python scripts/smart_census.py [game].  Per env-step: the step phases
(s_memtime cycles, as scripts/phase_profile.py), the smart entities stepped, sub_step calls, cycles of
the agent's basic_step_object and of the other smart entities', push-memo hits and the entity count.
The stamps cost time themselves: shares only, never wall time."""
import json
import os
import sys

os.environ.setdefault("PROCGEN_MI355X_LIB", "smart")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

STEP = ["rng+action", "set_action+velocity", "step_entities (smart)", "collisions", "erase", "tail", "finish",
        "ilist+nonsmart"]
SMART = ["smart entities", "sub_step calls", "agent cycles", "other smart cycles", "memo hits", "num_ents"]


def main(game="coinrun", num=65536, warm=300, steps=50):
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
    out = {"game": game, "per_env_step": {"step_phase_cycles": {k: round(d[i], 1) for i, k in enumerate(STEP)},
                                          "smart": {k: round(d[8 + i], 2) for i, k in enumerate(SMART)}}}
    env.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["coinrun"]))
