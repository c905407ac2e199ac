#!/usr/bin/env python3
"""use_generated_assets diagnostic: per game, make 8 envs, report device errors (with the AssetGen
reason bits) and the first-frame / 60-step pixel mismatch count against the oracle."""
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

from oracle_lib import OracleEnv  # noqa: E402
from procgen_amd import ProcgenGym3Env  # noqa: E402

games = sys.argv[1:] or ["coinrun", "bigfish", "heist", "fruitbot", "starpilot", "maze"]
for g in games:
    try:
        env = ProcgenGym3Env(num=8, env_name=g, num_levels=0, rand_seed=23, use_generated_assets=True)
        orc = OracleEnv(g, 8, num_levels=0, rand_seed=23, use_generated_assets=1)
        rng = np.random.RandomState(0)
        worst = []
        for t in range(61):
            if t:
                a = rng.randint(0, 15, 8).astype(np.int32)
                env.act(a)
                orc.step(a)
            try:
                _, ob, _ = env.observe()
            except Exception as e:  # noqa: BLE001
                errs = [int(env.debug_env(i)[66]) for i in range(8)]
                print(g, "step", t, "ERROR", e, "per-env error", errs, flush=True)
                break
            d = np.any(ob["rgb"] != orc.observe()["rgb"], axis=-1).sum(axis=(1, 2))
            worst.append(int(d.max()))
        print(g, "max mismatching pixels per env per step:", worst[:8], "... max", max(worst) if worst else None, flush=True)
        env.close()
    except Exception:  # noqa: BLE001
        traceback.print_exc()
