"""GPU parity for render_mode="rgb_array" (SURVEY.md section 8(f) row 3): info["rgb"], the 512x512
frame painted with Antialiasing + SmoothPixmapTransform (vecgame.cpp:318-330, 415-423;
game.cpp:97-107), from the device kernel (pg_render.hip pg_render_hires_kernel) against the oracle's
restatement (oracle_render_rgb_array), whose primitives and whole frames are pinned against the
real Qt 5.9.7 (tests/test_smooth_pins.py).  Bar: bit-exact, every checked step."""
import numpy as np
import pytest

from oracle_lib import OracleEnv
from test_gpu_games import make_gpu, oracle_kw

pytestmark = pytest.mark.gpu

GAMES = ["coinrun", "bigfish", "maze", "miner", "chaser", "climber", "ninja", "bossfight", "caveflyer", "dodgeball",
         "fruitbot", "heist", "jumper", "leaper", "plunder", "starpilot"]
ROTATING = ["bossfight", "caveflyer", "dodgeball", "fruitbot", "heist", "leaper", "plunder", "starpilot"]


def run_rgb_array(game, num, steps, every, seed, actions=None, **kw):
    env = make_gpu(num, game, render_mode="rgb_array", **kw)
    orc = OracleEnv(game, num, **oracle_kw(kw))
    rng = np.random.RandomState(seed)
    checked = 0
    for t in range(steps + 1):
        if t:
            act = (rng.randint(0, 15, size=num) if actions is None else rng.choice(actions, size=num)).astype(np.int32)
            env.act(act)
            orc.step(act)
        if t % every:
            continue
        _, ob, _ = env.observe()
        np.testing.assert_array_equal(ob["rgb"], orc.observe()["rgb"], err_msg="64x64 obs at step %d" % t)
        info = env.get_info()
        got = np.stack([np.asarray(i["rgb"]) for i in info])
        assert got.shape == (num, 512, 512, 3) and got.dtype == np.uint8
        exp = orc.render_rgb_array(512)
        if not np.array_equal(got, exp):
            d = np.argwhere(np.any(got != exp, axis=-1))
            raise AssertionError("%s info['rgb'] differs at step %d: %d pixels, first %s: %s vs %s"
                                 % (game, t, len(d), d[0].tolist(), got[tuple(d[0])].tolist(), exp[tuple(d[0])].tolist()))
        checked += 1
    env.close()
    return checked


@pytest.mark.parametrize("game", GAMES)
def test_rgb_array_parity(game):
    assert run_rgb_array(game, 4, 60, 6, seed=50, num_levels=0, rand_seed=31) == 11


@pytest.mark.parametrize("game", ROTATING)
def test_rgb_array_rotated_long(game):
    """longer runs of the games whose entities rotate (the antialiased rotated drawImage, tiles,
    starpilot's scrolling background, plunder's bars), 8 envs, frames every 25 steps."""
    assert run_rgb_array(game, 8, 200, 25, seed=53, num_levels=0, rand_seed=35) == 9


@pytest.mark.parametrize("game", ["coinrun", "maze", "ninja"])
def test_rgb_array_options(game):
    """easy mode, uncentered view, velocity squares, monochrome fills -- still bit-exact."""
    run_rgb_array(game, 2, 30, 10, seed=51, num_levels=0, rand_seed=32, distribution_mode="easy", center_agent=False,
                  paint_vel_info=True)
    run_rgb_array(game, 2, 20, 10, seed=52, num_levels=0, rand_seed=33, use_monochrome_assets=True)


def test_rgb_array_mixed_batch():
    """a mixed batch (coinrun,maze): each game's frames land in its own envs' info."""
    env = make_gpu(4, "coinrun,maze", render_mode="rgb_array", num_levels=0, rand_seed=34)
    _, ob, _ = env.observe()
    info = env.get_info()
    for e in range(4):
        orc = OracleEnv(("coinrun", "maze")[e % 2], 1, env_offset=e, num_levels=0, rand_seed=34)
        np.testing.assert_array_equal(np.asarray(info[e]["rgb"]), orc.render_rgb_array(512)[0])
    env.close()


@pytest.mark.parametrize("kw", [{"distribution_mode": "easy"}, {"distribution_mode": "hard"},
                                {"distribution_mode": "easy", "center_agent": False},
                                {"distribution_mode": "hard", "center_agent": False},
                                {"distribution_mode": "memory"}],
                         ids=["easy", "hard", "easy_uncentered", "hard_uncentered", "memory"])
def test_rgb_array_jumper_compass(kw):
    """jumper's compass at RENDER_RES (jumper.cpp:137-177): the dial (gray-raster ellipse fill + antialiased
    cosmetic pen), the wide square-capped needle, the distance bar and the translucent jump ellipse, in every
    distribution mode (exploration is hard mode's compass) and both views; 8 envs, 150 steps, frames every 10 steps."""
    assert run_rgb_array("jumper", 8, 150, 10, seed=57, num_levels=0, rand_seed=41, **kw) == 16


@pytest.mark.parametrize("kw", [{"distribution_mode": "easy"}, {"distribution_mode": "hard", "center_agent": False}],
                         ids=["easy", "hard_uncentered"])
def test_rgb_array_jumper_jump_ellipse(kw):
    """jump-heavy actions, every frame checked: the translucent ellipse under the agent after a mid-air jump
    (jumper.cpp:163-166; in env 0 of the oracle at steps 9, 20, 38, 47 (easy) / 9, 21, 37, 55 (hard, uncentered))."""
    assert run_rgb_array("jumper", 8, 60, 1, seed=57, actions=[2, 5, 8, 1, 7], num_levels=0, rand_seed=41, **kw) == 61


@pytest.mark.parametrize("chunks", ["1", "3", "64"])
def test_rgb_array_chunks(chunks, monkeypatch):
    """the frames render in PROCGEN_MI355X_HR_CHUNKS chunks, each DMA'd into the caller's page-locked
    info["rgb"] array while the next renders (pg_capi.cpp copy_latent): one chunk, ragged chunks (7 envs in
    3), more chunks than envs (empty ones skipped), single-game and mixed batches."""
    monkeypatch.setenv("PROCGEN_MI355X_HR_CHUNKS", chunks)
    assert run_rgb_array("coinrun", 7, 20, 10, seed=58, num_levels=0, rand_seed=42) == 3
    env = make_gpu(6, "coinrun,maze,heist", render_mode="rgb_array", num_levels=0, rand_seed=43)
    env.observe()
    info = env.get_info()
    for e in range(6):
        orc = OracleEnv(("coinrun", "maze", "heist")[e % 3], 1, env_offset=e, num_levels=0, rand_seed=43)
        np.testing.assert_array_equal(np.asarray(info[e]["rgb"]), orc.render_rgb_array(512)[0])
    env.close()
