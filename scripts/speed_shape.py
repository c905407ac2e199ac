#!/usr/bin/env python3
"""The reference's speed-test shape on the engine (procgen/env_test.py:55-69 test_multi_speed): for each
of the 16 games and num_envs in {1, 2, 16}, ProcgenGym3Env(num=num_envs, env_name=game) with default
options, zero actions, and 1,000 act + observe round trips through the host buffers -- the latency a
small-batch user of the reference sees.  Prints one JSON object: per game and num_envs, ms per
act + observe and env-steps/s (after 50 untimed round trips)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))

import numpy as np  # noqa: E402

GAMES = ["bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot", "heist",
         "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot"]


def rollout(env, actions, n):
    for _ in range(n):
        env.act(actions)
        env.observe()


def main():
    import torch
    torch.cuda.set_device(0)
    from procgen_amd import ProcgenGym3Env
    steps = int(os.environ.get("SPEED_STEPS", "1000"))
    games = sys.argv[1:] or GAMES
    out = {"what": "ProcgenGym3Env act(zeros) + observe() round trips, host buffers (procgen/env_test.py:55-69)",
           "steps": steps, "results": {}}
    for g in games:
        row = {}
        for num in (1, 2, 16):
            env = ProcgenGym3Env(num=num, env_name=g)
            actions = np.zeros([env.num], np.int32)
            rollout(env, actions, 50)
            t0 = time.perf_counter()
            rollout(env, actions, steps)
            dt = time.perf_counter() - t0
            env.close()
            row[str(num)] = {"ms_per_act_observe": round(dt * 1e3 / steps, 4), "env_steps_per_s": round(num * steps / dt, 1)}
        out["results"][g] = row
        print(g, row, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
