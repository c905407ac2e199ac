"""Writes tests/golden/upstream_states.npz: for every game, the upstream-format get_state bytes of a
1-env batch (rand_seed 7, num_levels 0) after 12 seeded actions.  Run on the GPU box:

    python3 scripts/make_state_golden.py gpurun_out/upstream_states.npz

tests/test_state_golden.py re-parses the file on the CPU against the oracle (so the committed bytes
are pinned to the oracle's objects) and, on the GPU, compares a fresh get_state with it byte for
byte (so later layout changes are caught)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

GAMES = ["bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot", "heist",
         "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot"]
STEPS = 12
SEED = 7


def actions():
    return np.random.RandomState(11).randint(0, 15, size=(STEPS, 1)).astype(np.int32)


def capture(game):
    from procgen_amd import ProcgenGym3Env
    env = ProcgenGym3Env(num=1, env_name=game, num_levels=0, start_level=0, rand_seed=SEED)
    for a in actions():
        env.act(a)
        env.observe()
    b = env.get_state()[0]
    env.close()
    return np.frombuffer(b, np.uint8).copy()


def main(out):
    np.savez_compressed(out, **{g: capture(g) for g in GAMES})
    print("wrote", out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "upstream_states.npz")
