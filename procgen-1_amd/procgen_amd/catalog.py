"""Asset catalogue: which images each game draws, and in which order.

This is DATA restated from the reference, not code: the order of every list
below drives RNG draw counts (``choose_random_theme`` draws ``randn(#themes)``,
reference ``procgen/src/basic-abstract-game.cpp:1047-1050``) and background
indices (``randn(#backgrounds)``, ``basic-abstract-game.cpp:776``), so it must
match the reference exactly.

Background groups: ``procgen/src/resources.cpp:837-952``; the platform group
gets every space background appended (``resources.cpp:972-975``) and ``caves``
is ``platform[2, 3, 13]`` (``resources.cpp:977-979``).

Per-game sprite tables: ``asset_for_type`` of each game (coinrun:
``procgen/src/games/coinrun.cpp:72-121``, bigfish ``bigfish.cpp:34-43``, maze
``maze.cpp:33-41``, heist ``heist.cpp:46-64``) plus the reserved engine sprites
(``basic-abstract-game.cpp:424-438``).
"""

# Image slot of an (image type, theme) pair, as in the reference
# (``img_idx = img_type + theme * MAX_ASSETS``, basic-abstract-game.cpp:896).
MAX_ASSETS = 100
MAX_IMAGE_THEMES = 10
NUM_IMAGE_SLOTS = MAX_ASSETS * MAX_IMAGE_THEMES

SPACE_BACKGROUNDS = [
    "space_backgrounds/deep_space_01.png",
    "space_backgrounds/spacegen_01.png",
    "space_backgrounds/milky_way_01.png",
    "space_backgrounds/ez_space_lite_01.png",
    "space_backgrounds/meyespace_v1_01.png",
    "space_backgrounds/eye_nebula_01.png",
    "space_backgrounds/deep_sky_01.png",
    "space_backgrounds/space_nebula_01.png",
    "space_backgrounds/Background-1.png",
    "space_backgrounds/Background-2.png",
    "space_backgrounds/Background-3.png",
    "space_backgrounds/Background-4.png",
    "space_backgrounds/parallax-space-backgound.png",
]

_PLATFORM_ONLY = (
    ["platform_backgrounds/%s.png" % n for n in (
        "alien_bg", "another_world_bg", "back_cave", "caverns", "cyberpunk_bg",
        "parallax_forest", "scifi_bg", "scifi2_bg", "living_tissue_bg",
        "airadventurelevel1", "airadventurelevel2", "airadventurelevel3",
        "airadventurelevel4", "cave_background", "blue_desert", "blue_grass",
        "blue_land", "blue_shroom", "colored_desert", "colored_grass",
        "colored_land", "colored_shroom", "landscape1", "landscape2",
        "landscape3", "landscape4")]
    + ["platform_backgrounds/battleback%d.png" % i for i in range(1, 11)]
    + ["platform_backgrounds/sunrise.png"]
    + ["platform_backgrounds_2/%s%d.png" % (n, i)
       for n in ("beach", "fantasy", "candy") for i in range(1, 5)]
)

# resources.cpp:972-975: the space backgrounds are appended to the platform group
PLATFORM_BACKGROUNDS = _PLATFORM_ONLY + SPACE_BACKGROUNDS

TOPDOWN_BACKGROUNDS = ["topdown_backgrounds/floortiles.png"] + [
    "topdown_backgrounds/backgrounddetailed%d.png" % i for i in range(1, 9)]
TOPDOWN_SIMPLE_BACKGROUNDS = ["topdown_backgrounds/floortiles.png"]
WATER_BACKGROUNDS = ["water_backgrounds/water%d.png" % i for i in range(1, 5)] + [
    "water_backgrounds/underwater%d.png" % i for i in range(1, 4)]
WATER_SURFACE_BACKGROUNDS = ["water_backgrounds/water%d.png" % i for i in range(1, 5)]
CAVES = [PLATFORM_BACKGROUNDS[2], PLATFORM_BACKGROUNDS[3], PLATFORM_BACKGROUNDS[13]]

BACKGROUND_GROUPS = {
    "platform": PLATFORM_BACKGROUNDS,
    "space": SPACE_BACKGROUNDS,
    "topdown": TOPDOWN_BACKGROUNDS,
    "topdown_simple": TOPDOWN_SIMPLE_BACKGROUNDS,
    "water": WATER_BACKGROUNDS,
    "water_surface": WATER_SURFACE_BACKGROUNDS,
    "caves": CAVES,
}

# Groups whose images all live in another group's pack (no duplicate pack committed):
# water_surface = water[0:4] (resources.cpp:952-961), space = platform[-13:] (:972-975).
BACKGROUND_PACK = {"water_surface": "water", "space": "platform"}

# ---------------------------------------------------------------- object ids
# procgen/src/object-ids.h:9-27
EXPLOSION, EXPLOSION2, EXPLOSION3, EXPLOSION4, EXPLOSION5, TRAIL = 54, 55, 56, 57, 58, 59

# basic-abstract-game.cpp:424-438 (reserved engine sprites)
RESERVED_SPRITES = {
    EXPLOSION: ["misc_assets/explosion1.png"],
    EXPLOSION2: ["misc_assets/explosion2.png"],
    EXPLOSION3: ["misc_assets/explosion3.png"],
    EXPLOSION4: ["misc_assets/explosion4.png"],
    EXPLOSION5: ["misc_assets/explosion5.png"],
    TRAIL: ["misc_assets/iconCircle_white.png"],
}

# ---------------------------------------------------------------- coinrun
# procgen/src/games/coinrun.cpp:13-34
_WALKING_ENEMIES = ["slimeBlock", "slimePurple", "slimeBlue", "slimeGreen", "mouse",
                    "snail", "ladybug", "wormGreen", "wormPink"]
_PLAYER_COLORS = ["Beige", "Blue", "Green", "Pink", "Yellow"]
_GROUND_THEMES = ["Dirt", "Grass", "Planet", "Sand", "Snow", "Stone"]


def _player(kind):
    return ["kenney/Players/128x256/%s/alien%s_%s.png" % (c, c, kind) for c in _PLAYER_COLORS]


COINRUN_SPRITES = {
    0: _player("stand"),                 # PLAYER
    9: _player("jump"),                  # PLAYER_JUMP
    12: _player("walk1"),                # PLAYER_RIGHT1
    13: _player("walk2"),                # PLAYER_RIGHT2
    6: ["kenney/Enemies/%s.png" % e for e in _WALKING_ENEMIES],       # ENEMY1
    7: ["kenney/Enemies/%s_move.png" % e for e in _WALKING_ENEMIES],  # ENEMY2
    1: ["kenney/Items/coinGold.png"],    # GOAL
    16: ["kenney/Ground/%s/%sMid.png" % (g, g.lower()) for g in _GROUND_THEMES],     # WALL_TOP
    15: ["kenney/Ground/%s/%sCenter.png" % (g, g.lower()) for g in _GROUND_THEMES],  # WALL_MID
    18: ["kenney/Tiles/lavaTop_low.png"],  # LAVA_TOP
    17: ["kenney/Tiles/lava.png"],         # LAVA_MID
    2: ["kenney/Enemies/sawHalf.png"],     # SAW
    3: ["kenney/Enemies/sawHalf_move.png"],  # SAW2
    20: ["kenney/Tiles/boxCrate.png", "kenney/Tiles/boxCrate_double.png",
         "kenney/Tiles/boxCrate_single.png", "kenney/Tiles/boxCrate_warning.png"],  # CRATE
}

# ---------------------------------------------------------------- bigfish
# procgen/src/games/bigfish.cpp:34-43 (PLAYER 0, FISH 2)
BIGFISH_SPRITES = {
    0: ["misc_assets/fishTile_072.png"],
    2: ["misc_assets/fishTile_074.png", "misc_assets/fishTile_078.png", "misc_assets/fishTile_080.png"],
}

# ---------------------------------------------------------------- maze
# procgen/src/games/maze.cpp:33-41 (WALL_OBJ 51, GOAL 2, PLAYER 0)
MAZE_SPRITES = {
    51: ["kenney/Ground/Sand/sandCenter.png"],
    2: ["misc_assets/cheese.png"],
    0: ["kenney/Enemies/mouse_move.png"],
}

# ---------------------------------------------------------------- heist
# procgen/src/games/heist.cpp:46-64 (WALL_OBJ 51, EXIT 9, PLAYER 0, KEY 2, LOCKED_DOOR 1)
HEIST_SPRITES = {
    51: ["kenney/Ground/Dirt/dirtCenter.png"],
    9: ["misc_assets/gemYellow.png"],
    0: ["misc_assets/spaceAstronauts_008.png"],
    2: ["misc_assets/keyBlue.png", "misc_assets/keyGreen.png", "misc_assets/keyRed.png"],
    1: ["misc_assets/lock_blue.png", "misc_assets/lock_green.png", "misc_assets/lock_red.png"],
}

# ---------------------------------------------------------------- miner (fork-modified)
# procgen/src/games/miner.cpp:50-66 (PLAYER 0, DEAD_PLAYER 12, BOULDER 1, DIAMOND 2, EXIT 6,
# DIRT 9, MUD 11, OOB_WALL 10).  misc_assets/mud.png is listed (resources.cpp:511) but absent
# from the reference's asset tree: MUD has no image here (drawn as nothing).
MINER_SPRITES = {
    0: ["misc_assets/robot_greenDrive1.png"],
    12: ["misc_assets/fire_1.png"],
    1: ["misc_assets/elementStone007.png"],
    2: ["misc_assets/gemBlue.png"],
    6: ["misc_assets/window.png"],
    9: ["misc_assets/dirt.png"],
    10: ["misc_assets/tile_bricksGrey.png"],
}

# ---------------------------------------------------------------- climber
# procgen/src/games/climber.cpp:47-89 (PLAYER 0, PLAYER_JUMP 9, PLAYER_RIGHT1 12, PLAYER_RIGHT2 13,
# WALL_TOP 16, WALL_MID 15, ENEMY1 6, ENEMY2 7, COIN 1)
_CL_COLORS = ["Blue", "Green", "Grey", "Red"]
CLIMBER_SPRITES = {
    0: ["platformer/player%s_stand.png" % c for c in _CL_COLORS],
    9: ["platformer/player%s_walk4.png" % c for c in _CL_COLORS],
    12: ["platformer/player%s_walk1.png" % c for c in _CL_COLORS],
    13: ["platformer/player%s_walk2.png" % c for c in _CL_COLORS],
    16: ["platformer/tileBlue_05.png", "platformer/tileGreen_05.png", "platformer/tileYellow_06.png",
         "platformer/tileBrown_06.png"],
    15: ["platformer/tileBlue_08.png", "platformer/tileGreen_08.png", "platformer/tileYellow_09.png",
         "platformer/tileBrown_09.png"],
    6: ["platformer/enemySwimming_1.png"],
    7: ["platformer/enemySwimming_2.png"],
    1: ["platformer/yellowCrystal.png"],
}

# ---------------------------------------------------------------- leaper
# procgen/src/games/leaper.cpp:45-66 (LOG 1, ROAD 2, WATER 3, CAR 4, FINISH_LINE 5, PLAYER 0)
LEAPER_SPRITES = {
    2: ["misc_assets/roadTile6b.png"],
    3: ["misc_assets/terrainTile6.png"],
    4: ["misc_assets/car_%s.png" % c for c in ("yellow_5", "black_1", "blue_2", "green_3", "red_4")],
    1: ["misc_assets/elementWood044.png"],
    0: ["misc_assets/frog%d.png" % i for i in (1, 2, 4, 6, 7)],
    5: ["misc_assets/finish2.png"],
}

# ---------------------------------------------------------------- chaser
# procgen/src/games/chaser.cpp:54-72 (PLAYER 0, ENEMY 6, ENEMY2 7, ENEMY3 8, LARGE_ORB 2, ENEMY_WEAK 3,
# ENEMY_EGG 4, MAZE_WALL 5); ORB (1002) is a grid fill, not an image
CHASER_SPRITES = {
    0: ["misc_assets/enemyFloating_1b.png"],
    6: ["misc_assets/enemyFlying_1.png"],
    7: ["misc_assets/enemyFlying_2.png"],
    8: ["misc_assets/enemyFlying_3.png"],
    2: ["misc_assets/yellowCrystal.png"],
    3: ["misc_assets/enemyWalking_1b.png"],
    4: ["misc_assets/enemySpikey_1b.png"],
    5: ["misc_assets/tileStone_slope.png"],
}

# ---------------------------------------------------------------- fruitbot
# procgen/src/games/fruitbot.cpp:46-76 (PLAYER 0, BARRIER 1, OUT_OF_BOUNDS_WALL 2, PLAYER_BULLET 3,
# BAD_OBJ 4, GOOD_OBJ 7, LOCKED_DOOR 10, LOCK 11, PRESENT 12)
FRUITBOT_SPRITES = {
    0: ["misc_assets/robot_3Dblue.png"],
    1: ["misc_assets/tileStone_slope.png"],
    2: ["misc_assets/tileStone_slope.png"],
    3: ["misc_assets/keyRed2.png"],
    4: ["misc_assets/food%d.png" % i for i in range(1, 7)],
    7: ["misc_assets/fruit%d.png" % i for i in range(1, 7)],
    10: ["misc_assets/fenceYellow.png"],
    11: ["misc_assets/lockRed2.png"],
    12: ["misc_assets/present%d.png" % i for i in range(1, 4)],
}

# ---------------------------------------------------------------- dodgeball
# procgen/src/games/dodgeball.cpp:50-88 (LAVA_WALL 1, PLAYER_BALL 3, ENEMY 4, DOOR 5, ENEMY_BALL 6,
# DOOR_OPEN 7, DUST_CLOUD 8, OOB_WALL 10)
DODGEBALL_SPRITES = {
    0: ["misc_assets/character12.png"],
    3: ["misc_assets/ball_soccer1.png"],
    4: ["misc_assets/character%d.png" % i for i in range(1, 12)],
    5: ["misc_assets/blockRed.png"],
    6: ["misc_assets/ball_soccer2.png"],
    7: ["misc_assets/blockGreen.png"],
    1: ["misc_assets/tileStone_slope2.png"],
    10: ["misc_assets/tileStone_slope2.png"],
    8: ["misc_assets/spaceEffect%d.png" % i for i in range(1, 10)],
}

# ---------------------------------------------------------------- plunder
# procgen/src/games/plunder.cpp:49-64 (PLAYER_BULLET 1, TARGET_LEGEND 2, TARGET_BACKGROUND 3, PANEL 6,
# SHIP 7; the agent and the legend draw SHIP images)
PLUNDER_SPRITES = {
    7: ["misc_assets/ship_%d.png" % i for i in range(1, 7)],
    1: ["misc_assets/cannonBall.png"],
    6: ["misc_assets/panel_wood.png"],
    3: ["misc_assets/target_red2.png"],
}

# ---------------------------------------------------------------- starpilot
# procgen/src/games/starpilot.cpp:60-104 (BULLET_PLAYER 1, BULLET2 2, BULLET3 3, FLYER 4, METEOR 5,
# CLOUD 6, TURRET 7, FAST_FLYER 8, FINISH_LINE 9)
_SP_SHIPS = ["misc_assets/spaceShips_%03d.png" % i for i in range(1, 8)]
STARPILOT_SPRITES = {
    0: ["misc_assets/playerShip2_blue.png"],
    1: ["misc_assets/towerDefense_tile295.png"],
    2: ["misc_assets/towerDefense_tile296.png"],
    3: ["misc_assets/towerDefense_tile297.png"],
    4: _SP_SHIPS,
    8: _SP_SHIPS,
    5: ["misc_assets/spaceMeteors_%03d.png" % i for i in range(1, 5)] +
       ["misc_assets/meteorGrey_big%d.png" % i for i in range(1, 5)],
    6: ["misc_assets/spaceEffect%d.png" % i for i in range(1, 10)],
    7: ["misc_assets/spaceStation_018.png", "misc_assets/spaceStation_019.png"],
    9: ["misc_assets/spaceRockets_%03d.png" % i for i in range(1, 5)],
}

# ---------------------------------------------------------------- bossfight
# procgen/src/games/bossfight.cpp:76-106 (PLAYER_BULLET 1, BOSS 2, SHIELDS 3, ENEMY_BULLET 4,
# LASER_TRAIL 5 and REFLECTED_BULLET 6 draw other types' images, BARRIER 7)
_BF_LASERS = ["misc_assets/laserGreen14.png", "misc_assets/laserRed11.png", "misc_assets/laserBlue09.png"]
BOSSFIGHT_SPRITES = {
    0: ["misc_assets/playerShip1_blue.png", "misc_assets/playerShip1_green.png",
        "misc_assets/playerShip2_orange.png", "misc_assets/playerShip3_red.png"],
    2: ["misc_assets/enemyShipBlack1.png", "misc_assets/enemyShipBlue2.png", "misc_assets/enemyShipGreen3.png",
        "misc_assets/enemyShipRed4.png"],
    4: _BF_LASERS,
    1: _BF_LASERS,
    3: ["misc_assets/shield2.png"],
    7: ["misc_assets/spaceMeteors_%03d.png" % i for i in range(1, 5)] +
       ["misc_assets/meteorGrey_big%d.png" % i for i in range(1, 5)],
}

# ---------------------------------------------------------------- ninja
# procgen/src/games/ninja.cpp:45-74 (GOAL 1, BOMB 6, THROWING_STAR 7, PLAYER_JUMP 9, PLAYER_RIGHT1 12,
# PLAYER_RIGHT2 13, FIRE 14, WALL_MID 20)
NINJA_SPRITES = {
    20: ["misc_assets/tile_bricksGrey.png", "misc_assets/tile_bricksGrown.png", "misc_assets/tile_bricksRed.png"],
    1: ["platformer/shroom%d.png" % i for i in range(1, 7)],
    0: ["platformer/zombie_idle.png"],
    9: ["platformer/zombie_jump.png"],
    12: ["platformer/zombie_walk1.png"],
    13: ["platformer/zombie_walk2.png"],
    6: ["misc_assets/bomb.png"],
    7: ["misc_assets/saw.png"],
    14: ["misc_assets/bomb.png"],
}

# ---------------------------------------------------------------- caveflyer
# procgen/src/games/caveflyer.cpp:36-55 (PLAYER 0, GOAL 1, OBSTACLE 2, TARGET 3, PLAYER_BULLET 4,
# ENEMY 5, CAVEWALL 8, EXHAUST 9)
CAVEFLYER_SPRITES = {
    1: ["misc_assets/ufoGreen2.png"],
    2: ["misc_assets/meteorBrown_big1.png"],
    3: ["misc_assets/ufoRed2.png"],
    4: ["misc_assets/laserBlue02.png"],
    5: ["misc_assets/enemyShipBlue4.png"],
    0: ["misc_assets/playerShip1_red.png"],
    8: ["misc_assets/groundA.png"],
    9: ["misc_assets/towerDefense_tile295.png"],
}

# ---------------------------------------------------------------- jumper
# procgen/src/games/jumper.cpp:52-83 (PLAYER 0, GOAL 1, SPIKE 2, CAVEWALL 6, CAVEWALL_TOP 7,
# PLAYER_JUMP 9, PLAYER_LEFT1 10, PLAYER_LEFT2 11, PLAYER_RIGHT1 12, PLAYER_RIGHT2 13)
JUMPER_SPRITES = {
    0: ["misc_assets/bunny2_ready.png"],
    2: ["misc_assets/spikeMan_stand.png"],
    1: ["misc_assets/carrot.png"],
    9: ["misc_assets/bunny2_jump.png"],
    12: ["misc_assets/bunny2_walk1.png"],
    13: ["misc_assets/bunny2_walk2.png"],
    10: ["misc_assets/bunny2_walk1.png"],
    11: ["misc_assets/bunny2_walk2.png"],
    7: ["platformer/tileBlue_05.png", "platformer/tileGreen_05.png", "platformer/tileYellow_06.png",
        "platformer/tileBrown_06.png"],
    6: ["platformer/tileBlue_08.png", "platformer/tileGreen_08.png", "platformer/tileYellow_09.png",
        "platformer/tileBrown_09.png"],
}

GAMES = {
    # game name -> (sprite table, background group)
    "coinrun": (COINRUN_SPRITES, "platform"),   # coinrun.cpp:60-62
    "bigfish": (BIGFISH_SPRITES, "water"),      # bigfish.cpp:30-32
    "maze": (MAZE_SPRITES, "topdown"),          # maze.cpp:29-31
    "heist": (HEIST_SPRITES, "topdown"),        # heist.cpp:37-39
    "miner": (MINER_SPRITES, "caves"),          # miner.cpp:45-47
    "climber": (CLIMBER_SPRITES, "platform"),   # climber.cpp:43-45
    "leaper": (LEAPER_SPRITES, "topdown"),      # leaper.cpp:41-43
    "chaser": (CHASER_SPRITES, "topdown_simple"),  # chaser.cpp:50-52
    "fruitbot": (FRUITBOT_SPRITES, "topdown"),  # fruitbot.cpp:42-44
    "dodgeball": (DODGEBALL_SPRITES, "topdown"),  # dodgeball.cpp:46-48
    "plunder": (PLUNDER_SPRITES, "water_surface"),  # plunder.cpp:45-47
    "starpilot": (STARPILOT_SPRITES, "space"),  # starpilot.cpp:56-58
    "bossfight": (BOSSFIGHT_SPRITES, "space"),  # bossfight.cpp:72-74
    "ninja": (NINJA_SPRITES, "platform"),       # ninja.cpp:43-45
    "caveflyer": (CAVEFLYER_SPRITES, "space"),  # caveflyer.cpp:31-33
    "jumper": (JUMPER_SPRITES, "platform"),     # jumper.cpp:48-50
}

# Game ids used across the C ABI (procgen/env.py:15-32 ordering).
ENV_NAMES = [
    "bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun",
    "dodgeball", "fruitbot", "heist", "jumper", "leaper", "maze", "miner",
    "ninja", "plunder", "starpilot",
]
SUPPORTED_GAMES = sorted(GAMES)


def sprite_table(game):
    """type -> [names] for a game, engine-reserved sprites included.

    The reserved list only applies where the game itself defines no sprite for
    the type (basic-abstract-game.cpp:94-98)."""
    table = dict(RESERVED_SPRITES)
    table.update(GAMES[game][0])
    return table


def num_themes(game):
    """asset_num_themes[type] for every type with a sprite (basic-abstract-game.cpp:113-119)."""
    return {t: len(v) for t, v in sprite_table(game).items()}


# Image slot that carries a game's Qt-tabulated overlay raster instead of a sprite (never drawn as an
# image): jumper's compass (jumper.cpp:137-177; tools/make_compass_tables.py -> jumper_compass.npz).
TABLE_SLOT = 99
