"""Committed upstream-format state bytes, one per game (tests/golden/upstream_states.npz, written by
scripts/make_state_golden.py on the GPU box).

The byte format is reconstructed from upstream procgen's serialize/deserialize (the fork's
WriteBuffer/ReadBuffer are stubs, buffer.h), so it is "parity unpinned" against the reference.
What these tests pin instead:
  * CPU: every committed state parses field by field (tests/upstream_state.py) and its objects equal
    the oracle's after the same seeded actions -- entity words bit for bit, cur_time, step_rand_int,
    level seed, generator position, grid;
  * GPU: a fresh get_state of the same run equals the committed bytes exactly, so any later change
    of the layout or of a serialized member shows up here."""
import os
import struct
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))

from make_state_golden import GAMES, SEED, actions, capture  # noqa: E402

GOLDEN = os.path.join(HERE, "golden", "upstream_states.npz")


def _golden():
    if not os.path.exists(GOLDEN):
        pytest.skip("tests/golden/upstream_states.npz not generated yet")
    return np.load(GOLDEN)


def _fnv(name):
    h = 0x811c9dc5
    for c in name.encode():
        h = ((h ^ c) * 0x1000193) & 0xffffffff
    return h - (1 << 32) if h >= 1 << 31 else h


@pytest.mark.parametrize("game", GAMES)
def test_golden_state_matches_oracle(game):
    from oracle_lib import OracleEnv
    from upstream_state import END_OF_BUFFER, entity_words, parse
    b = bytes(_golden()[game])
    d = parse(b, game)
    assert d["end"] == END_OF_BUFFER and d["consumed"] == len(b)
    assert d["version"] == 0 and d["game_name"] == game and d["fixed_asset_seed"] == _fnv(game)
    orc = OracleEnv(game, 1, rand_seed=SEED)
    for a in actions():
        orc.step(a)
    o = orc.debug(0)
    assert len(d["entities"]) == o[0] and d["cur_time"] == o[1]
    assert d["background_index"] == o[6] and d["step_rand_int"] == o[8] and d["current_level_seed"] == o[10]
    assert d["rand_gen"]["pos"] == o[11] and len(d["rand_gen"]["words"]) == 624
    assert d["grid_size"] == d["main_width"] * d["main_height"] == len(d["grid"]["data"])
    if not o[14]:
        ax, ay = struct.unpack("<ff", struct.pack("<ii", int(o[2]), int(o[3])))
        assert struct.pack("<ff", d["entities"][0]["x"], d["entities"][0]["y"]) == struct.pack("<ff", ax, ay)
    oe = orc.entities(0)
    got = np.array([entity_words(e) for e in d["entities"]], np.int32).reshape(-1, 31)
    assert got.shape == oe.shape
    np.testing.assert_array_equal(got, oe)


@pytest.mark.gpu
@pytest.mark.parametrize("game", GAMES)
def test_get_state_equals_golden(game):
    want = _golden()[game]
    got = capture(game)
    assert got.shape == want.shape, "state length %d, golden %d" % (got.size, want.size)
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, "first differing byte at %d" % diff[0]
