"""GPU parity for use_generated_assets: the device AssetGen painter
(procgen-1_amd/csrc/pg_assetgen.h) against the oracle's restatement (oracle/procgen_oracle.c ag_*),
itself pinned to the reference's assetgen.cpp built with the real Qt 5.9.7 (tests/test_assetgen_pins.py).

With the option on, every sprite is a 64x64 ARGB32 image generated at make time from
fixed_asset_seed(env name) + type (basic-abstract-game.cpp:101-107, generated on the device once per
game), and every reset paints a fresh 500x500 RGB32 background with the level's own generator after
background_index = randn(1) (:778-782), generated on the device inside the reset kernel.  Both
painters are the same restated algorithm, so the bar here is bit-exact RGB every step.
"""
import numpy as np
import pytest

from test_gpu_games import GAMES, run_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("game", GAMES + ["coinrun"])
def test_parity_generated_assets(game):
    """Every game: rect- and shape-mode sprites (use_block_asset), scaled / rotated / mirrored /
    tiled draws of 64 x 64 generated images (coinrun, heist and caveflyer leave their 128-px tile
    fast path for the generic tile pass), the generated 500 x 500 background under each game's
    background placement (fruitbot's and starpilot's vertical tiling, coinrun's scroll) -- resets
    happen within the run, so backgrounds are painted at reset time on the device and compared
    pixel for pixel."""
    episodes, _ = run_pair(game, 8, 120, seed=40, num_levels=0, rand_seed=23, use_generated_assets=True)


def test_generated_assets_many_resets():
    """Short episodes (num_levels=3, easy) so many envs reset mid-run: the in-kernel background
    painter's generator position must equal the oracle's after every reset."""
    run_pair("bigfish", 16, 200, seed=41, num_levels=3, start_level=0, rand_seed=24, distribution_mode="easy",
             use_generated_assets=True)


def test_generated_assets_state_refused():
    """get_state of a use_generated_assets env is refused, as BasicAbstractGame::serialize fasserts
    !use_generated_assets (basic-abstract-game.cpp:1185)."""
    from procgen_amd import ProcgenGym3Env
    env = ProcgenGym3Env(num=2, env_name="coinrun", use_generated_assets=True)
    with pytest.raises(Exception):
        env.get_state()
    env.close()
