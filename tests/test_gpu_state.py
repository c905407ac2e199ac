"""GPU parity for the fork's latent-state setter, MinerGame::game_set_state
(procgen/src/games/miner.cpp:423-449; the JS binding's setState, cheerpgame.cpp:54-56), through the
C ABI (procgen_set_latent_state) against the oracle's restatement (oracle_miner_set_state).

The reference's own tests hold no vectors for this path: the cases are
synthetic edits of live states -- a rearranged grid with the agent and exit moved, a grid holding a
DEAD_PLAYER cell (the agent leaves the entity list), a smaller grid than the world -- each checked
bit-exact (RGB, reward, first, level seeds, latent info) right after the call and for 120 steps.
"""
import numpy as np
import pytest

from oracle_lib import OracleEnv
from test_gpu_coinrun import assert_same, gpu_obs
from test_gpu_games import check_latent, make_gpu

pytestmark = pytest.mark.gpu

SPACE, BOULDER, DIAMOND, DIRT, DEAD_PLAYER = 100, 1, 2, 9, 12


def edited(lat, i, rng, kind):
    w, h = lat["grid_size"][i]
    grid = lat["grid"][i][: w * h].reshape(h, w).copy()
    free = np.argwhere(grid == SPACE)
    agent = free[rng.randint(len(free))][::-1] if len(free) else lat["agent_pos"][i]
    exit_ = free[rng.randint(len(free))][::-1] if len(free) else lat["exit_pos"][i]
    if kind == "rearrange":  # swap dirt / diamonds / boulders around in the interior
        inner = grid[1:-1, 1:-1]
        vals = inner.reshape(-1)
        rng.shuffle(vals)
        grid[1:-1, 1:-1] = vals.reshape(inner.shape)
        grid[agent[1], agent[0]] = SPACE
    elif kind == "dead":
        grid[agent[1], agent[0]] = DEAD_PLAYER
    elif kind == "partial":  # only the first rows are written (w x h smaller than the world)
        grid = grid[: max(1, h // 2)]
        grid[grid == DIRT] = DIAMOND
    return grid, agent, exit_


@pytest.mark.parametrize("kind", ["rearrange", "dead", "partial"])
def test_miner_set_latent_state(kind):
    num = 6
    env = make_gpu(num, "miner", num_levels=0, start_level=0, rand_seed=3)
    orc = OracleEnv("miner", num, rand_seed=3)
    rng = np.random.RandomState(11)
    for t in range(1, 16):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        env.act(act)
        orc.step(act)
    assert_same(gpu_obs(env), orc.observe(), 15)
    lat = orc.latent()
    for i in range(0, num, 2):
        grid, agent, exit_ = edited(lat, i, rng, kind)
        env.set_latent_state(i, grid, agent, exit_)
        orc.miner_set_state(i, grid, agent, exit_)
    g = gpu_obs(env)
    o = orc.observe()
    np.testing.assert_array_equal(g["rgb"], o["rgb"], err_msg="frame after set_latent_state")
    check_latent(env, orc, 0)
    for t in range(1, 121):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        env.act(act)
        orc.step(act)
        assert_same(gpu_obs(env), orc.observe(), t)
        check_latent(env, orc, t)
    env.close()


def test_set_latent_state_rejects_other_games():
    from procgen_amd.env import ProcgenError
    env = make_gpu(2, "maze", num_levels=0, start_level=0, rand_seed=0)
    with pytest.raises(ProcgenError):
        env.set_latent_state(0, np.full((3, 3), SPACE, np.int32), (1, 1), (2, 2))
    env.close()


# ---------------------------------------------------------------- upstream get_state / set_state
ALL = ["bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun", "dodgeball", "fruitbot", "heist",
       "jumper", "leaper", "maze", "miner", "ninja", "plunder", "starpilot"]


def _fnv(name):
    h = 0x811c9dc5
    for c in name.encode():
        h = ((h ^ c) * 0x1000193) & 0xffffffff
    return h - (1 << 32) if h >= 1 << 31 else h


@pytest.mark.parametrize("game", ALL)
def test_upstream_state_fields(game):
    """get_state bytes walked field by field (tests/upstream_state.py) and checked against the
    oracle's own objects after the same steps."""
    import struct
    from upstream_state import END_OF_BUFFER, entity_words, parse
    num = 3
    env = make_gpu(num, game, num_levels=0, start_level=0, rand_seed=9)
    orc = OracleEnv(game, num, rand_seed=9)
    rng = np.random.RandomState(2)
    for _ in range(25):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        env.act(act)
        orc.step(act)
    assert_same(gpu_obs(env), orc.observe(), 25)
    lat = orc.latent()
    for i, b in enumerate(env.get_state()):
        d = parse(b, game)
        o = orc.debug(i)
        assert d["end"] == END_OF_BUFFER and d["consumed"] == len(b), "state does not end at END_OF_BUFFER"
        assert d["version"] == 0 and d["game_name"] == game and d["fixed_asset_seed"] == _fnv(game)
        assert len(d["entities"]) == o[0] and d["cur_time"] == o[1]
        assert d["background_index"] == o[6] and d["step_rand_int"] == o[8] and d["current_level_seed"] == o[10]
        assert d["rand_gen"]["pos"] == o[11] and len(d["rand_gen"]["words"]) == 624
        assert d["grid_size"] == d["main_width"] * d["main_height"] == len(d["grid"]["data"])
        if not o[14]:  # agent listed: entity 0 is the agent
            ax, ay = struct.unpack("<ff", struct.pack("<ii", int(o[2]), int(o[3])))
            assert d["entities"][0]["type"] == 0
            assert struct.pack("<ff", d["entities"][0]["x"], d["entities"][0]["y"]) == struct.pack("<ff", ax, ay)
        if game in ("maze", "miner"):
            w, h = lat["grid_size"][i]
            assert d["grid"]["data"] == list(lat["grid"][i][: w * h])
        # every field of every listed entity, bit for bit, against the oracle's entity list
        oe = orc.entities(i)
        got = np.array([entity_words(e) for e in d["entities"]], np.int32).reshape(-1, 31)
        assert got.shape == oe.shape, "entity count"
        for k in range(len(oe)):
            np.testing.assert_array_equal(got[k], oe[k], err_msg="entity %d of env %d" % (k, i))
    env.close()


@pytest.mark.parametrize("game", ALL)
def test_upstream_state_transfer(game):
    """set_state of env 0's upstream state into env 3: from then on env 3 plays exactly env 0's
    game (same frames, rewards, firsts, level seeds) under the same actions -- the format carries
    everything the step path reads."""
    num = 4
    env = make_gpu(num, game, num_levels=0, start_level=0, rand_seed=4)
    rng = np.random.RandomState(5)
    for _ in range(20):
        env.act(rng.randint(0, 15, size=num).astype(np.int32))
        env.observe()
    st = env.get_state()
    st[3] = st[0]
    env.set_state(st)
    g = gpu_obs(env)
    np.testing.assert_array_equal(g["rgb"][3], g["rgb"][0])
    for t in range(1, 81):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        act[3] = act[0]
        env.act(act)
        g = gpu_obs(env)
        for key in ("rgb", "rew", "first", "level_seed", "prev_level_seed"):
            np.testing.assert_array_equal(g[key][3], g[key][0], err_msg="%s differs at step %d" % (key, t))
    env.close()


def test_upstream_state_rejects_other_game():
    from procgen_amd import ProcgenGym3Env
    from procgen_amd.env import ProcgenError
    env = ProcgenGym3Env(num=2, env_name="maze,heist", num_levels=0, start_level=0, rand_seed=0)
    st = env.get_state()
    with pytest.raises(ProcgenError):
        env.set_state([st[1], st[1]])  # a heist state into the maze slot
    env.close()
