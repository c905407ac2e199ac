#!/usr/bin/env python3
"""Per-game CPU baseline table: the CPU oracle (oracle/procgen_oracle.c, the scalar restatement of
the reference step path; test infrastructure, never the product) timed on this host, one process,
for every game at num_envs {1, 8, 64, 512}.  The reference's own speed test
(procgen/env_test.py:55-69) times act + observe of zero actions for 1,000 steps at num_envs 1 / 2 / 16;
this table uses the same zero-action shape (column `zero`) and uniform random actions (column
`random`, the bench's workload), with fewer steps at large num_envs so every cell is ~1 s of CPU work.
The 16 games run in parallel worker processes (one game each, at most 16, the box's CPU share), as
the bench's `cpu_baseline` runs its 16 workers; a cell is the rate of one process on one core.

    python3 scripts/cpu_baseline_table.py > profiles/r05/r05_cpu_baseline_games.json
"""
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

GAMES = ["bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot", "heist",
         "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot"]
SIZES = [1, 8, 64, 512]


def rate(game, n, steps, zero):
    from oracle_lib import OracleEnv
    env = OracleEnv(game, n, num_levels=0, start_level=0, rand_seed=0)
    rng = np.random.RandomState(0)
    acts = np.zeros((steps, n), np.int32) if zero else rng.randint(0, 15, size=(steps, n)).astype(np.int32)
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(acts[t])
        env.observe()  # the observation copy of act + observe
    return n * steps / (time.perf_counter() - t0)


def game_row(g):
    row = {}
    for n in SIZES:
        steps = max(20, min(1000, 60000 // n))
        row[str(n)] = {"zero": round(rate(g, n, steps, True), 1), "random": round(rate(g, n, steps, False), 1),
                       "steps": steps}
    print("%-10s %s" % (g, " ".join("%6d:%9.0f" % (n, row[str(n)]["random"]) for n in SIZES)), file=sys.stderr)
    return g, row


def main():
    import multiprocessing as mp
    games = sys.argv[1].split(",") if len(sys.argv) > 1 else GAMES
    workers = min(len(games), 16, len(os.sched_getaffinity(0)))
    out = {"what": "CPU oracle env-steps/s, one process per game (cores = 1 per cell), act + observe per step",
           "host": platform.processor() or platform.machine(), "cpus_visible": len(os.sched_getaffinity(0)),
           "workers": workers, "sizes": SIZES, "games": {}}
    with mp.get_context("spawn").Pool(workers) as pool:
        for g, row in pool.map(game_row, games):
            out["games"][g] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
