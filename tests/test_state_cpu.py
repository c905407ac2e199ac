"""CPU checks of the oracle's restatement of MinerGame::game_set_state (miner.cpp:423-449), the
checker the GPU test (tests/test_gpu_state.py) holds the engine to: the latent info reflects the
written grid and positions, a DEAD_PLAYER cell removes the agent from the entity list, and the
cases where the reference would crash are refused.  Also: the engine library declares the entry."""
import ctypes
import os

import numpy as np
import pytest

from oracle_lib import OracleEnv

SPACE, DEAD_PLAYER = 100, 12


def test_oracle_miner_set_state_roundtrip():
    orc = OracleEnv("miner", 2, rand_seed=5)
    lat = orc.latent()
    w, h = lat["grid_size"][0]
    grid = lat["grid"][0][: w * h].reshape(h, w).copy()
    free = np.argwhere(grid == SPACE)
    ay, ax = free[0]
    ey, ex = free[-1]
    orc.miner_set_state(0, grid, (ax, ay), (ex, ey))
    lat2 = orc.latent()
    np.testing.assert_array_equal(lat2["grid"][0][: w * h].reshape(h, w), grid)
    assert tuple(lat2["agent_pos"][0]) == (ax, ay)
    assert tuple(lat2["exit_pos"][0]) == (ex, ey)
    n0 = orc.debug(0)[0]
    grid[ay, ax] = DEAD_PLAYER
    orc.miner_set_state(0, grid, (ax, ay), (ex, ey))
    d = orc.debug(0)
    assert d[0] == n0 - 1 and d[14] == 1  # one entity fewer, agent erased
    # env 1 untouched
    np.testing.assert_array_equal(orc.latent()["grid"][1], lat["grid"][1])


def test_oracle_miner_set_state_refusals():
    orc = OracleEnv("miner", 1, rand_seed=5)
    w, h = orc.latent()["grid_size"][0]
    with pytest.raises(ValueError):
        orc.miner_set_state(0, np.full((h + 1, w), SPACE, np.int32), (1, 1), (2, 2))
    maze = OracleEnv("maze", 1, rand_seed=5)
    with pytest.raises(ValueError):
        maze.miner_set_state(0, np.full((2, 2), SPACE, np.int32), (1, 1), (1, 1))


def test_engine_exports_set_latent_state():
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "procgen-1_amd", "procgen_amd",
                      "libprocgen_mi355x.so")
    if not os.path.exists(so):
        pytest.skip("engine not built")
    lib = ctypes.CDLL(so)
    assert hasattr(lib, "procgen_set_latent_state")


# ---------------------------------------------------------------- RandGen text of get_state
def _mt_state(seed, draws):
    """std::mt19937 (seed) after `draws` outputs: (624 words, position) -- the libstdc++ layout."""
    x = [seed & 0xffffffff]
    for i in range(1, 624):
        x.append((1812433253 * (x[-1] ^ (x[-1] >> 30)) + i) & 0xffffffff)
    p = 624
    for _ in range(draws):
        if p >= 624:
            for k in range(624):
                y = (x[k] & 0x80000000) | (x[(k + 1) % 624] & 0x7fffffff)
                x[k] = x[(k + 397) % 624] ^ (y >> 1) ^ (0x9908b0df if y & 1 else 0)
            p = 0
        p += 1
    return np.array(x, np.uint32), p


def test_get_state_randgen_text_matches_reference():
    """get_state writes each RandGen as RandGen::serialize does (randgen.cpp:100-106); the vectors
    are the reference's own serialize output (tools/make_state_goldens.py, oracle/_ref)."""
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "procgen-1_amd", "procgen_amd",
                      "libprocgen_mi355x.so")
    if not os.path.exists(so):
        pytest.skip("engine not built")
    lib = ctypes.CDLL(so)
    lib.procgen_mt_text.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "randgen_text.npz"))
    for seed, draws, text, n in zip(z["seeds"], z["draws"], z["text"], z["length"]):
        words, pos = _mt_state(int(seed), int(draws))
        buf = ctypes.create_string_buffer(1 << 14)
        k = lib.procgen_mt_text(words.ctypes.data, pos, buf, len(buf))
        assert buf.raw[:k] == bytes(text[:n]), (seed, draws)
