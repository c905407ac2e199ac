"""The reference's own state test (procgen/state_test.py:65-124) on the GPU engine, for all 16 games.

`run_state_test` there drives ProcgenGym3Env(num=2, env_name, rand_seed=0) through one sequence of
uniform random actions (gym3.types_np.sample of Discrete(15), RandomState(0)) and requires:
  * two runs to be identical (observations, rewards, firsts, info);
  * a run that calls get_state after every observe to be identical to one that does not, and two
    such runs to produce identical state bytes;
  * a run that also calls set_state(get_state()) after every observe to change nothing;
  * a state saved halfway, restored into an env built with rand_seed=1, to reproduce the rest of the
    rollout -- first observation (the restored reward / first / info and the re-rendered frame)
    included.
Miner has states the reference itself cannot restore (no PLAYER entity: `restorable`); the port skips
set_state on those and restores the first restorable state from the halfway step on.
The reference runs 10,000 steps per game (:9); here coinrun and bigfish (a float-position game) run
10,000, the other games 2,000 (the whole file runs inside the GPU suite's time budget).  Rollouts are
compared through a 128-bit digest per step of every array the reference compares (and of the state
bytes), so 10,000-step rollouts need no gigabytes of host memory; the state at the restore point is
kept whole.  The reference runs each rollout in a fresh subprocess; here each rollout is a fresh
VecEnv in this process (nothing is shared between two ProcgenGym3Env instances but the immutable
asset atlas)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALL = ["bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot", "heist",
       "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot"]
LONG = {"coinrun", "bigfish"}


def num_steps(game):
    return 10000 if game in LONG else 2000


def actions_for(game):
    # gym3.types_np.sample(Discrete(15), bshape=(2,), rng) draws rng.randint(0, 15, size=(2,))
    rng = np.random.RandomState(0)
    return [rng.randint(0, 15, size=2).astype(np.int32) for _ in range(num_steps(game))]


def _digest(rew, ob, first, info):
    h = hashlib.blake2b(digest_size=16)
    h.update(np.ascontiguousarray(rew).tobytes())
    h.update(np.ascontiguousarray(first).tobytes())
    for k in sorted(ob):
        h.update(k.encode())
        h.update(np.ascontiguousarray(ob[k]).tobytes())
    for d in info:
        for k in sorted(d):
            h.update(k.encode())
            h.update(np.ascontiguousarray(d[k]).tobytes())
    return h.hexdigest()


def _state_digest(states):
    h = hashlib.blake2b(digest_size=16)
    for s in states:
        h.update(len(s).to_bytes(4, "little"))
        h.update(s)
    return h.hexdigest()


def restorable(game, states):
    """Whether the reference's BasicAbstractGame::deserialize accepts the states: it requires a PLAYER
    entity (fassert(agent_idx >= 0), basic-abstract-game.cpp:1238-1240).  Miner has states without
    one: a boulder that falls onto the agent in move_cell's second sweep (above the agent,
    miner.cpp:300-304) erases it after game_step's `died` check (:279-282), so the episode ends one
    step later and the state in between lists no agent.  The reference fasserts on restoring such a
    state; this build refuses it with an error (pg_state.cpp), so set_state is skipped there."""
    if game != "miner":
        return True
    from upstream_state import parse
    return all(any(e["type"] == 0 for e in parse(s, game)["entities"]) for s in states)


def gather(game, actions, state=None, get_state=False, set_state_every_step=False, rand_seed=0, keep_state_at=None):
    """gather_rollouts (state_test.py:12-30): per step the digest of (ob, info) and, with get_state,
    of the state bytes; the state itself at step `keep_state_at`."""
    from procgen_amd import ProcgenGym3Env
    env = ProcgenGym3Env(num=2, env_name=game, rand_seed=rand_seed)
    if state is not None:
        env.callmethod("set_state", state)
    obs, sts, kept = [], [], None

    def record(i):
        nonlocal kept
        rew, ob, first = env.observe()
        obs.append(_digest(rew, ob, first, env.get_info()))
        if get_state:
            st = env.callmethod("get_state")
            sts.append(_state_digest(st))
            if kept is None and keep_state_at is not None and i >= keep_state_at and restorable(game, st):
                kept = (i, st)
            if set_state_every_step and restorable(game, st):
                env.callmethod("set_state", st)

    record(0)
    for i, act in enumerate(actions, 1):
        env.act(act)
        record(i)
    env.close()
    return obs, sts, kept


def first_difference(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i
    return None if len(a) == len(b) else min(len(a), len(b))


def assert_identical(a, b, what):
    assert len(a) == len(b), "%s: %d vs %d steps" % (what, len(a), len(b))
    i = first_difference(a, b)
    assert i is None, "%s: first difference at step %d" % (what, i)


@pytest.fixture(scope="module", params=ALL)
def runs(request):
    """The reference rollout and the get_state rollout of one game (state kept at the restore point).
    Module scope: pytest groups the tests below by game and computes these once per game."""
    game = request.param
    actions = actions_for(game)
    offset = len(actions) // 2
    ref, _, _ = gather(game, actions)
    state_obs, state_sts, kept = gather(game, actions, get_state=True, keep_state_at=offset)
    # the restore point: the halfway step, or the next one the reference can deserialize (restorable)
    offset, kept = kept if kept is not None else (offset, None)
    return dict(game=game, actions=actions, offset=offset, ref=ref, state_obs=state_obs, state_sts=state_sts,
                kept=kept)


def test_state_runs_identical(runs):
    """state_test.py:80-91: a second run, and a run saving states, match the first."""
    assert len(runs["ref"]) == len(runs["actions"]) + 1
    basic, _, _ = gather(runs["game"], runs["actions"])
    assert_identical(runs["ref"], basic, "second run")
    assert_identical(runs["ref"], runs["state_obs"], "run with get_state every step")


def test_state_bytes_identical(runs):
    """state_test.py:93-101: two runs saving states produce the same states."""
    obs2, sts2, _ = gather(runs["game"], runs["actions"], get_state=True)
    assert_identical(runs["ref"], obs2, "second run with get_state")
    assert_identical(runs["state_sts"], sts2, "state bytes of two runs")


def test_state_set_every_step(runs):
    """state_test.py:103-112: set_state(get_state()) after every observe changes nothing."""
    obs3, sts3, _ = gather(runs["game"], runs["actions"], get_state=True, set_state_every_step=True)
    assert_identical(runs["ref"], obs3, "run with set_state every step")
    assert_identical(runs["state_sts"], sts3, "state bytes with set_state every step")


def test_state_restore_into_other_seed(runs):
    """state_test.py:114-124: the state at the halfway step, restored into an env built with
    rand_seed=1, reproduces the remaining rollout from its first observation on."""
    off = runs["offset"]
    assert runs["kept"] is not None
    obs, sts, _ = gather(runs["game"], runs["actions"][off:], state=runs["kept"], get_state=True, rand_seed=1)
    assert_identical(runs["ref"][off:], obs, "restored rollout")
    assert_identical(runs["state_sts"][off:], sts, "restored rollout's state bytes")
