"""GPU parity for bigfish, maze, heist and mixed batches: the HIP engine (through the libenv
C ABI) against the CPU oracle, every step.

Bar (BASELINE.json north_star): bit-exact reward / done(first) / level seeds and RGB for the
integer-coordinate games (maze, heist); bigfish is the "float tolerance" class (its fish
radius goes through the double pow of bigfish.cpp:84) -- the test still demands bit-exact
results and reports any difference with the step and env, so a libm ulp would show up here.
Heist exercises the rotated-sprite path (agent face_direction, ring keys) and MazeGen with
doors; maze exercises MazeGen, grid_step movement and the fork's latent-state info; miner
(fork-modified, miner.cpp) exercises the falling-object passes, agent death and latent state.
"""
import numpy as np
import pytest

from oracle_lib import OracleEnv, hashed_actions
from test_gpu_coinrun import KEYS, assert_same, gpu_obs

pytestmark = pytest.mark.gpu


def make_gpu(num, env_name, **kw):
    from procgen_amd import ProcgenGym3Env
    return ProcgenGym3Env(num=num, env_name=env_name, **kw)


def oracle_kw(gpu_kw):
    kw = dict(gpu_kw)
    dm = kw.pop("distribution_mode", "hard")
    kw["distribution_mode"] = {"easy": 0, "hard": 1, "extreme": 2, "memory": 10}[dm]
    for k in ("center_agent", "use_backgrounds", "restrict_themes", "use_sequential_levels", "use_monochrome_assets",
              "paint_vel_info", "use_generated_assets"):
        if k in kw:
            kw[k] = int(kw[k])
    return kw


def check_latent(env, orc, step):
    info = env.get_info()
    lat = orc.latent()
    for key in ("grid_size", "grid", "agent_pos", "exit_pos"):
        got = np.stack([np.asarray(i[key]) for i in info])
        np.testing.assert_array_equal(got, lat[key], err_msg="latent %s differs at step %d" % (key, step))


def run_pair(game, num, steps, seed=0, latent=False, **gpu_kw):
    env = make_gpu(num, game, **gpu_kw)
    orc = OracleEnv(game, num, **oracle_kw(gpu_kw))
    rng = np.random.RandomState(seed)
    assert_same(gpu_obs(env), orc.observe(), 0)
    if latent:
        check_latent(env, orc, 0)
    episodes = rewards = 0
    for t in range(1, steps + 1):
        act = rng.randint(0, 15, size=num).astype(np.int32)
        env.act(act)
        orc.step(act)
        g = gpu_obs(env)
        assert_same(g, orc.observe(), t)
        if latent:
            check_latent(env, orc, t)
        episodes += int(g["first"].sum())
        rewards += float(g["rew"].sum())
    env.close()
    return episodes, rewards


LATENT = ("maze", "miner")
# every game of this build except coinrun (tests/test_gpu_coinrun.py)
GAMES = ["bigfish", "maze", "heist", "miner", "climber", "leaper", "chaser", "fruitbot", "dodgeball", "plunder",
         "starpilot", "bossfight", "ninja", "caveflyer", "jumper"]


@pytest.mark.parametrize("game", GAMES)
def test_parity_hard_unbounded(game):
    run_pair(game, 16, 300, seed=1, num_levels=0, rand_seed=0, latent=game in LATENT)


@pytest.mark.parametrize("game", GAMES)
def test_parity_200_levels_easy(game):
    run_pair(game, 8, 200, seed=2, num_levels=200, start_level=0, rand_seed=5, distribution_mode="easy",
             latent=game in LATENT)


@pytest.mark.parametrize("game", ["maze", "heist", "miner"])
def test_parity_memory_mode_centered(game):
    # memory mode turns center_agent on in game_reset (maze.cpp:70, heist.cpp:124, miner.cpp:145)
    run_pair(game, 8, 150, seed=3, num_levels=0, rand_seed=9, distribution_mode="memory", latent=game in LATENT)


def test_miner_long_run_deaths():
    """miner: boulders fall on the agent (death leaves DEAD_PLAYER and ends the episode one step
    later, miner.cpp:326-330, 256-259), diamonds, exits -- 32 envs x 600 steps."""
    episodes, rewards = run_pair("miner", 32, 600, seed=8, num_levels=0, rand_seed=4, latent=True)
    assert episodes > 0


@pytest.mark.parametrize("game", GAMES + ["coinrun"])
def test_parity_monochrome_assets(game):
    """use_monochrome_assets: every sprite becomes fillRect(color_for_type) (basic-abstract-game.cpp:
    464-490, 886-928); with and without restrict_themes (mask_theme_if_necessary, :458-462)."""
    run_pair(game, 8, 120, seed=11, num_levels=0, rand_seed=2, use_monochrome_assets=True, latent=game in LATENT)
    run_pair(game, 4, 60, seed=12, num_levels=0, rand_seed=6, use_monochrome_assets=True, restrict_themes=True)


@pytest.mark.parametrize("game", GAMES + ["coinrun"])
def test_parity_paint_vel_info(game):
    """paint_vel_info: two grey velocity squares in the top-left corner (basic-abstract-game.cpp:
    969-977); games with has_useful_vel_info = false draw nothing extra."""
    run_pair(game, 8, 150, seed=13, num_levels=0, rand_seed=7, paint_vel_info=True)


@pytest.mark.parametrize("game", GAMES)
def test_parity_options(game):
    run_pair(game, 8, 150, seed=4, num_levels=20, rand_seed=3, use_backgrounds=False, restrict_themes=True,
             use_sequential_levels=True)


def test_climber_uncentered():
    """climber with center_agent=False: visibility = max(20, 64) (prepare_for_drawing :832-838)."""
    run_pair("climber", 8, 200, seed=11, num_levels=0, rand_seed=6, center_agent=False)


def test_leaper_extreme_and_long():
    """leaper extreme mode (leaper-only, game.cpp:80-81; 20x20 world, fast lanes) and a long
    hard-mode run: cars (rotated PI when driving left), logs carrying the frog, finish line tiles."""
    run_pair("leaper", 16, 300, seed=12, num_levels=0, rand_seed=7, distribution_mode="extreme")
    run_pair("leaper", 32, 500, seed=13, num_levels=0, rand_seed=8)


def test_chaser_extreme_and_long():
    """chaser extreme mode (19x19 maze, 5 enemies), and a long hard run: eggs hatch after 50
    steps, enemies chase / flee at junctions (step_rand_int), large orbs make them edible."""
    run_pair("chaser", 16, 300, seed=14, num_levels=0, rand_seed=3, distribution_mode="extreme")
    run_pair("chaser", 32, 600, seed=15, num_levels=0, rand_seed=4)


def test_fruitbot_long_and_uncentered():
    """fruitbot: key bullets (collides_with_entities) open locked doors, fruit / food rewards,
    vertically tiled background; a long hard run and an uncentered one (visibility = 60)."""
    run_pair("fruitbot", 32, 500, seed=16, num_levels=0, rand_seed=5)
    run_pair("fruitbot", 8, 200, seed=17, num_levels=0, rand_seed=6, center_agent=False)


def test_dodgeball_modes():
    """dodgeball: recursive room split, enemies that reflect off lava walls and fire, player balls
    (collides_with_entities) that kill enemies and leave rotating dust clouds, rotating balls drawn
    through the device QTransform::rotate; extreme (8 splits) and memory (40x40, centred) modes."""
    run_pair("dodgeball", 32, 500, seed=18, num_levels=0, rand_seed=7)
    run_pair("dodgeball", 8, 200, seed=19, num_levels=0, rand_seed=8, distribution_mode="extreme")
    run_pair("dodgeball", 8, 200, seed=20, num_levels=0, rand_seed=9, distribution_mode="memory")


def test_plunder_long():
    """plunder: lanes of ships, cannonballs (collides_with_entities) hit targets / non-targets and leave
    explosions, juice runs out (~670 steps without hits), juice / progress bars (fillRect(QRectF))."""
    episodes, _ = run_pair("plunder", 16, 900, seed=21, num_levels=0, rand_seed=10)
    assert episodes > 0


def test_starpilot_long_and_extreme():
    """starpilot: the spawner list (std::sort order among equal spawn times, popped as cur_time
    reaches them), aimed enemy bullets (sqrt, face_direction through glibc's atan2f), player shots
    both ways (sin / cos of PI), explosions, the finish line at t = 500, the scrolling tiled space
    background; extreme mode (more health, smaller bullets)."""
    run_pair("starpilot", 32, 650, seed=22, num_levels=0, rand_seed=11)
    run_pair("starpilot", 8, 300, seed=23, num_levels=0, rand_seed=12, distribution_mode="extreme")


def test_bossfight_long():
    """bossfight: shields up / down cycles, reflected bullets (type change mid collision walk), boss
    damage rounds with explosions, laser trails, attack modes 0-3 (sin / cos of the fire angles)."""
    run_pair("bossfight", 32, 800, seed=24, num_levels=0, rand_seed=13)


def test_ninja_long_and_easy():
    """ninja: charged jumps, throwing stars (smart entities that stick to walls, blow up bombs: grid
    write-through + explosions), fire / bomb deaths, the jump-charge bar; easy mode (visibility 10)."""
    run_pair("ninja", 32, 600, seed=25, num_levels=0, rand_seed=14)
    run_pair("ninja", 8, 300, seed=26, num_levels=0, rand_seed=15, distribution_mode="easy")


def test_caveflyer_modes():
    """caveflyer: RoomGenerator levels (cellular automaton, best room, BFS goal path, 4x dilation),
    thrust along the heading (sin / cos of the agent's rotation), exhaust, lasers that explode on
    cave walls / targets (3 hits) / meteors, reflecting enemies facing their velocity (atan2f), the
    agent drawn at arbitrary rotations; easy (30x30) and memory (60x60, unpruned) modes."""
    run_pair("caveflyer", 32, 600, seed=27, num_levels=0, rand_seed=16)
    run_pair("caveflyer", 8, 300, seed=28, num_levels=0, rand_seed=17, distribution_mode="easy")
    run_pair("caveflyer", 8, 200, seed=29, num_levels=0, rand_seed=18, distribution_mode="memory")


def test_jumper_modes():
    """jumper: MazeGen + RoomGenerator levels, spikes and long-wall breaking (in-order scans), double
    jumps with a cooldown, trails, the compass overlay (Qt-tabulated dial / needle / jump ellipse,
    double atan2 + sin / cos for the needle, the distance bar); easy, uncentered and memory (45x45,
    no compass, timeout 2000) modes."""
    run_pair("jumper", 32, 600, seed=30, num_levels=0, rand_seed=19)
    run_pair("jumper", 8, 300, seed=31, num_levels=0, rand_seed=20, distribution_mode="easy")
    run_pair("jumper", 8, 200, seed=32, num_levels=0, rand_seed=21, center_agent=False)
    run_pair("jumper", 8, 200, seed=33, num_levels=0, rand_seed=22, distribution_mode="memory")


def test_bigfish_long_episodes():
    """bigfish episodes run up to 6,000 steps (bigfish.cpp:25): many fish spawn, grow, leave."""
    run_pair("bigfish", 8, 1200, seed=6, num_levels=0, rand_seed=12)


def test_mixed_batch_parity():
    """env n plays names[n % 4] (vecgame.cpp:357-358), level seeds from the global index."""
    names = sorted(GAMES + ["coinrun"])
    num = 4 * len(names)
    env = make_gpu(num, ",".join(names), num_levels=0, rand_seed=21)
    orcs = [OracleEnv(names[n % len(names)], 1, env_offset=n, num_levels=0, rand_seed=21) for n in range(num)]
    g = gpu_obs(env)
    for n, o in enumerate(orcs):
        assert_same(g, o.observe(), 0, idx=slice(n, n + 1))
    for t in range(1, 151):
        act = hashed_actions(0xC0FFEE, np.arange(num), t)
        env.act(act)
        g = gpu_obs(env)
        for n, o in enumerate(orcs):
            o.step(act[n:n + 1])
            assert_same(g, o.observe(), t, idx=slice(n, n + 1))
    env.close()


@pytest.mark.parametrize("game", ["bigfish", "maze", "heist"])
def test_full_size_sampled_parity(game):
    """BASELINE configs 3/4 sizes (bigfish 65,536, maze/heist 32,768), sampled envs."""
    num = 65536 if game == "bigfish" else 32768
    env = make_gpu(num, game, num_levels=0, rand_seed=0)
    sample = [0, 1, 63, 64, 4095, 12345, num // 2, num - 1]
    orcs = [OracleEnv(game, 1, env_offset=i, num_levels=0, rand_seed=0) for i in sample]
    ids = np.arange(num)
    g = gpu_obs(env)
    for k, o in zip(sample, orcs):
        assert_same(g, o.observe(), 0, idx=slice(k, k + 1))
    for t in range(1, 101):
        act = hashed_actions(0x5EED, ids, t)
        env.act(act)
        g = gpu_obs(env)
        for k, o in zip(sample, orcs):
            o.step(act[k:k + 1])
            assert_same(g, o.observe(), t, idx=slice(k, k + 1))
    env.close()


@pytest.mark.parametrize("game", GAMES)
def test_state_roundtrip(game):
    env = make_gpu(4, game, num_levels=20, rand_seed=11)
    rng = np.random.RandomState(1)
    for _ in range(30):
        env.act(rng.randint(0, 15, size=4))
        env.observe()
    states = env.get_state()
    acts = [rng.randint(0, 15, size=4) for _ in range(60)]
    a = []
    for ac in acts:
        env.act(ac)
        a.append(gpu_obs(env))
    env.set_state(states)
    for k, ac in enumerate(acts):
        env.act(ac)
        b = gpu_obs(env)
        for key in KEYS + ["rgb"]:
            np.testing.assert_array_equal(a[k][key], b[key])
    env.close()
