// pg_engine.h -- HBM layout of the MI355X Procgen engine (shared by kernels and host glue).
//
// One env = one wavefront.  Per-env state lives in HBM, resident across steps:
//   PGEnv        per-env scalars (Game + BasicAbstractGame + per-game members), 512 B
//   entity SoA   [num_envs][PG_NF field planes][PG_CAP] (lane = entity slot; pg_ent_index)
//   grid         int16 [num_envs][PG_GRID_MAX] (row-major y*w+x, reference grid.h:14-79)
//   mt           uint32 [num_envs][2][PG_MT_WORDS] (rand_gen, level_seed_rand_gen)
// Field and member names follow the reference (game.h, basic-abstract-game.h,
// entity.h, games/coinrun.cpp).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define PG_RES 64
#define PG_OBS_BYTES (64 * 64 * 3)
#define PG_CAP 512            // entity slots per env (coinrun worst case < 400)
#define PG_GRID_MAX (64 * 64) // largest world (coinrun, ninja 64x64)
#define PG_MT_N 624
#define PG_MT_WORDS 625       // 624 state words + index
#define PG_NUM_SLOTS 1000     // image slots: type + 100 * theme
#define PG_MAX_BG 64
#define PG_GEN_BG_PX (500 * 500) // use_generated_assets: one env's background (QImage 500 x 500 RGB32)

// game ids = index in the reference's env list (procgen/env.py:15-32)
enum PGGame {
    PG_GAME_BIGFISH = 0, PG_GAME_BOSSFIGHT = 1, PG_GAME_CAVEFLYER = 2, PG_GAME_CHASER = 3, PG_GAME_CLIMBER = 4, PG_GAME_COINRUN = 5, PG_GAME_DODGEBALL = 6, PG_GAME_FRUITBOT = 7, PG_GAME_HEIST = 8, PG_GAME_JUMPER = 9, PG_GAME_LEAPER = 10, PG_GAME_MAZE = 11,
    PG_GAME_MINER = 12, PG_GAME_NINJA = 13, PG_GAME_PLUNDER = 14, PG_GAME_STARPILOT = 15
};
#ifndef PG_NUM_GAMES
#define PG_NUM_GAMES 16
#endif
#define PG_LATENT_GRID (35 * 35) // fork latent-state grid info (vecgame.cpp:280-291)

// error codes (mirrored in include/procgen_mi355x.h)
#ifndef PG_ERR_NONE
#define PG_ERR_NONE 0
#define PG_ERR_ENTITY_OVERFLOW 1
#define PG_ERR_BAD_OPTION 2
#define PG_ERR_NO_ATLAS 3
#define PG_ERR_HIP 4
#define PG_ERR_GRID 5
#define PG_ERR_ASSETGEN 6 // the AssetGen painter met a path it does not restate (reason bits << 16 in error_any)
#define PG_ERR_RENDER 7   // a draw referenced atlas pixels / a case the renderer does not have
#endif

// reference DistributionMode (game.h:34-39)
enum { PG_EASY = 0, PG_HARD = 1, PG_EXTREME = 2, PG_MEMORY = 10 };

// entity flag bits (entity.h bools)
enum {
    EF_WILL_ERASE = 1,
    EF_COLLIDES = 2,
    EF_REFLECTED = 4,
    EF_ABS_COORDS = 8,
    EF_SMART_STEP = 16,
    EF_AVOIDS = 32,
    EF_AUTO_ERASE = 64,
};

// entity field planes
enum {
    F_X, F_Y, F_VX, F_VY, F_RX, F_RY,
    F_ROTATION, F_VROT, F_ALPHA, F_ALPHA_DECAY, F_GROW_RATE, F_FRICTION,
    F_COLLISION_MARGIN, F_HEALTH, F_THETA, F_CLIMBER_SPAWN_X,
    F_TYPE, F_IMAGE_TYPE, F_IMAGE_THEME, F_RENDER_Z,
    F_LIFE_TIME, F_EXPIRE_TIME, F_FIRE_TIME, F_SPAWN_TIME,
    F_FLAGS,
    PG_NF
};

struct PGEnv {
    // ---- Game (game.h:64-134)
    int32_t game_id;
    int32_t action;
    int32_t cur_time;
    int32_t timeout;
    int32_t current_level_seed;
    int32_t prev_level_seed;
    int32_t episodes_remaining;
    int32_t episode_done;
    int32_t last_reward_timer;
    float last_reward;
    int32_t default_action;
    int32_t reset_count;
    float total_reward;
    float sd_reward;          // step_data
    int32_t sd_done;
    int32_t sd_level_complete;
    int32_t level_seed_low;
    int32_t level_seed_high;
    int32_t game_n;
    // ---- options (GameOptions, game.h:47-61)
    int32_t opt_distribution_mode;
    int32_t opt_center_agent;
    int32_t opt_use_backgrounds;
    int32_t opt_restrict_themes;
    int32_t opt_use_sequential_levels;
    int32_t opt_debug_mode;
    int32_t opt_paint_vel_info;
    int32_t opt_use_monochrome_assets;
    // ---- BasicAbstractGame (basic-abstract-game.h:128-176)
    int32_t num_ents;
    int32_t agent_erased;
    int32_t background_index;
    float bg_pct_x;
    float bg_tile_ratio;
    int32_t last_move_action;
    int32_t move_action;
    int32_t special_action;
    float mixrate;
    float maxspeed;
    float max_jump;
    float action_vx;
    float action_vy;
    float action_vrot;
    float visibility;
    float min_visibility;
    int32_t main_width;
    int32_t main_height;
    int32_t out_of_bounds_object;
    int32_t step_rand_int;
    int32_t grid_step;
    int32_t random_agent_start;
    int32_t has_useful_vel_info;
    float char_dim;
    // ghost of the agent after erase_if_needed removed it (shared_ptr keeps it alive in the reference)
    float ghost_x, ghost_y, ghost_vx, ghost_vy, ghost_rx, ghost_ry;
    // ---- coinrun (coinrun.cpp:38-47)
    float last_agent_y;
    int32_t wall_theme;
    int32_t has_support;
    int32_t facing_right;
    int32_t is_on_crate;
    float gravity;
    float air_control;
    // ---- bookkeeping
    int32_t rg_mti;           // rand_gen position (mt words live in the mt plane)
    int32_t lsg_mti;          // level_seed_rand_gen position
    int32_t error;            // PG_ERR_* of this env (sticky)
    int32_t grid8_ok;         // the int8 grid mirror is current (written at reset)
    // ---- bigfish (bigfish.cpp:20-22)
    int32_t fish_eaten;
    float r_inc;
    // ---- maze (maze.cpp:16-18) / heist (heist.cpp:18-21)
    int32_t maze_dim;
    int32_t world_dim;
    int32_t num_keys;
    int32_t has_keys;         // bit k = has_keys[k]
    // ---- miner (miner.cpp:26-28)
    int32_t diamonds_remaining;
    int32_t died;
    int32_t main_area;
    // ---- climber (climber.cpp:30-36; the platformer members are shared with coinrun)
    int32_t coin_quota;
    int32_t coins_collected;
    // ---- leaper (leaper.cpp:27-32): at most 4 + 1 lanes of each kind
    int32_t bottom_road_y;
    int32_t bottom_water_y;
    int32_t goal_y;
    int32_t num_road_lanes;
    int32_t num_water_lanes;
    float road_lane_speeds[5];
    float water_lane_speeds[5];
    // ---- chaser (chaser.cpp:26-35; free_cells / is_space_vec are derived from the grid: the
    //      MAZE_WALL cells never change after the reset)
    int32_t eat_timeout;
    int32_t egg_timeout;
    int32_t eat_time;
    int32_t total_enemies;
    int32_t total_orbs;
    int32_t orbs_collected;
    // ---- fruitbot (fruitbot.cpp:26-28)
    int32_t last_fire_time;   // (also dodgeball, dodgeball.cpp:33)
    // ---- dodgeball (dodgeball.cpp:28-35; the rooms list lives only during the reset)
    float db_min_dim;
    float db_hard_min_dim;
    float db_ball_vscale;
    float db_ball_r;
    int32_t num_enemies;
    int32_t enemy_fire_delay;
    // ---- members of the games added later share one block (an env plays one game)
    union {
        struct { // plunder (plunder.cpp:19-31)
            uint32_t lane_dirs;     // bit i = lane_directions[i]
            uint32_t target_bools;  // bit i = target_bools[i]
            uint32_t perm;          // image_permutation[i] in bits 4i..4i+3
            float lane_vels[5];
            int32_t num_lanes, num_current_ship_types, targets_hit, target_quota;
            float juice_left, r_scale, spawn_prob, legend_r, min_agent_x;
        } pl;
        struct { // bossfight (bossfight.cpp:34-58; the constant members are literals in the kernels)
            uint32_t attack_modes;  // attack_modes[i] in bits 2i..2i+1 (num_rounds <= 5)
            int32_t time_to_swap, invulnerable_duration, num_rounds, round_num, round_health, curr_vel_timeout;
            int32_t attack_mode, player_laser_theme, boss_laser_theme, damaged_until_time, shields_are_up;
            int32_t barriers_moves_right;
            float boss_bullet_vel, rand_pct, rand_fire_pct, rand_pct_x, rand_pct_y;
        } bf;
        struct { // ninja (ninja.cpp:25-33; has_support, facing_right, wall_theme, gravity, air_control,
                 // last_fire_time are the shared members above)
            float jump_charge, jump_charge_inc;
        } nj;
        struct { // jumper (jumper.cpp:31-39; has_support, facing_right, wall_theme are shared; the goal
                 // is entity 1 for the whole episode)
            int32_t jump_count, jump_delta, jump_time;
            float compass_dim;
        } jp;
        int32_t words[20];
    } gs;
    // entity slots reserved at the top of the planes, [PG_CAP - num_tail, PG_CAP): starpilot's
    // spawner list (starpilot.cpp:34), vector index i at slot PG_CAP - 1 - i (pop_back frees the
    // lowest slot)
    int32_t num_tail;
};

// The PGEnv members pg_step_kernel writes back (everything else is read-only there).  One list for
// the step's write-back (pg_step.hip) and for the level prefetch's mask of step-written words that a
// swapped-in spare keeps from the live env (pg_capi.cpp sp_mask): a member added to one is in both.
// `error` is written back too but is not in the lists (a spare never carries the live env's error).
#define PG_STEP_WB_COMMON(X)                                                                          \
    X(action) X(cur_time) X(sd_reward) X(sd_done) X(sd_level_complete) X(total_reward)                 \
    X(last_reward_timer) X(last_reward) X(prev_level_seed) X(episode_done) X(num_ents) X(agent_erased) \
    X(ghost_x) X(ghost_y) X(ghost_vx) X(ghost_vy) X(ghost_rx) X(ghost_ry) X(move_action)               \
    X(special_action) X(last_move_action) X(action_vx) X(action_vy) X(action_vrot) X(step_rand_int)    \
    X(rg_mti)
#define PG_STEP_WB_COINRUN(X) X(has_support) X(facing_right) X(is_on_crate) X(last_agent_y)
#define PG_STEP_WB_BIGFISH(X) X(fish_eaten)
#define PG_STEP_WB_HEIST(X) X(has_keys)
#define PG_STEP_WB_MINER(X) X(diamonds_remaining) X(died)
#define PG_STEP_WB_CLIMBER(X) X(has_support) X(facing_right) X(coins_collected)
#define PG_STEP_WB_CHASER(X) X(eat_time) X(orbs_collected)
#define PG_STEP_WB_FRUITBOT(X) X(last_fire_time)
#define PG_STEP_WB_DODGEBALL(X) X(last_fire_time) X(num_enemies)
#define PG_STEP_WB_PLUNDER(X) X(last_fire_time) X(gs)
#define PG_STEP_WB_STARPILOT(X) X(num_tail)
#define PG_STEP_WB_BOSSFIGHT(X) X(last_fire_time) X(gs)
#define PG_STEP_WB_NINJA(X) X(last_fire_time) X(gs) X(has_support) X(facing_right)
#define PG_STEP_WB_JUMPER(X) X(gs) X(has_support) X(facing_right)
#define PG_STEP_WB_ALL(X)                                                                              \
    PG_STEP_WB_COMMON(X) PG_STEP_WB_COINRUN(X) PG_STEP_WB_BIGFISH(X) PG_STEP_WB_HEIST(X)              \
    PG_STEP_WB_MINER(X) PG_STEP_WB_CLIMBER(X) PG_STEP_WB_CHASER(X) PG_STEP_WB_FRUITBOT(X)              \
    PG_STEP_WB_DODGEBALL(X) PG_STEP_WB_PLUNDER(X) PG_STEP_WB_STARPILOT(X) PG_STEP_WB_BOSSFIGHT(X)      \
    PG_STEP_WB_NINJA(X) PG_STEP_WB_JUMPER(X)

static_assert(sizeof(PGEnv) == 512, "PGEnv must stay 512 B");

// The frames the register-frame render (pg_render.hip pg_render_rf_kernel) draws: atlas colours (not
// monochrome) and a tile window of at most 63 x 63 -- always when centred, else the whole world.  One
// predicate for the kernel's check and the host's selection (make-time options, restored states).
static inline __host__ __device__ bool pg_rf_serves(const PGEnv &s) {
    return !s.opt_use_monochrome_assets && (s.opt_center_agent || (s.main_width <= 63 && s.main_height <= 63));
}

// The largest world of each game (width x height; its level generator's bound, also the set_state check
// of pg_capi.cpp): the step kernel loads that many grid cells before it knows the env's own size.
static inline __host__ __device__ constexpr int pg_game_max_w(int g) {
    return g == 2 ? 60 : g == 3 ? 19 : g == 5 ? 64 : g == 6 ? 40 : g == 8 ? 23 : g == 9 ? 45 : g == 11 ? 31 : g == 12 ? 35 :
           g == 13 ? 64 : g == 15 ? 16 : 20;
}
static inline __host__ __device__ constexpr int pg_game_max_h(int g) {
    return g == 2 ? 60 : g == 3 ? 19 : g == 4 ? 64 : g == 5 ? 64 : g == 6 ? 40 : g == 7 ? 60 : g == 8 ? 23 : g == 9 ? 45 :
           g == 11 ? 31 : g == 12 ? 35 : g == 13 ? 64 : g == 15 ? 16 : 20;
}

// Entity storage: one contiguous block of PG_NF planes x PG_CAP slots per env (51,200 B), so every field
// of an env is a 32-bit byte offset from the env's block (plane f at f * 2,048 B): the kernels address
// an env's entities from one base register instead of 25 plane bases 128 MB apart.
#define PG_ENT_BLOCK (PG_NF * PG_CAP) // words per env
static inline __host__ __device__ size_t pg_ent_index(int env, int f, int slot) {
    return (size_t)env * PG_ENT_BLOCK + (size_t)f * PG_CAP + (size_t)slot;
}

// Everything a kernel needs, passed by value.
struct PGDev {
    int32_t num_envs;
    int32_t env_offset;       // global index of env 0 (multi-GPU shard)
    int32_t num_actions;
    PGEnv *envs;
    float *ents;              // num_envs blocks of PG_NF planes x PG_CAP words (pg_ent_index; int planes reinterpret)
    int16_t *grid;            // num_envs * PG_GRID_MAX
    int8_t *grid8;            // num_envs * PG_GRID_MAX: int8 mirror for the step kernel's LDS copy
    uint32_t *mt;             // num_envs * 2 * PG_MT_WORDS
    int32_t *actions;         // num_envs
    uint8_t *rgb;             // num_envs * PG_OBS_BYTES
    float *rew;
    uint8_t *first;
    int32_t *prev_level_seed;
    uint8_t *prev_level_complete;
    int32_t *level_seed;
    int32_t *reset_queue;     // [num_envs] env ids needing a reset this step
    int32_t *reset_count;     // [1]
    int32_t *error_any;       // [1] OR of all env errors
    uint64_t *prof;           // [num_envs][16] per-phase s_memtime sums (PG_PROFILE builds only)
    // atlas: one pixel array, per-game tables (a kernel of game G sees its own via game_view)
    const uint32_t *pixels;
    uint32_t num_pixels;        // bound of every texel index the stamping paths form
    const int32_t *sprites;   // [PG_NUM_GAMES][PG_NUM_SLOTS][4] (offset, w, h, pad)
    const int32_t *backgrounds; // [PG_NUM_GAMES][PG_MAX_BG][4]
    int32_t num_backgrounds;    // of the viewed game
    const int32_t *num_themes;  // [PG_NUM_GAMES][100]
    int32_t num_bg[PG_NUM_GAMES];
    // rotation transforms of QTransform::rotate for the angles the games draw at (host-built
    // with the C library's sin/cos, exactly as Qt's qSin/qCos; see pg_capi.cpp rot_table)
    const double *rot_table;    // [PG_ROT_N][4] = m11, m12, m21, m22
    const float *rot_angles;    // [PG_ROT_N] entity rotation values (radians, float) of the table
    int32_t *latent;            // [num_envs][PG_LATENT_N] grid_size, grid, agent_pos, exit_pos (maze)
    // use_generated_assets: each env's 500 x 500 RGB32 background, repainted by AssetGen at every
    // reset (basic-abstract-game.cpp:60-63, 778-782); null otherwise
    uint32_t *gen_bg;
    // step launch order (pg_step_kernel): sched = [slow-list length of parity 1 | reset counts
    // (reset_count points here) | slow-list length of parity 0], 16 ints each (one per game), so one
    // 32-int memset clears the reset counts with the length of the parity being written.
    int32_t *sched;
    uint8_t *done8;            // [num_envs] the last step ended the episode (a reset is queued)
    int32_t *heavy;             // [2][PG_NUM_GAMES][PG_HEAVY_CAP] each game's slow envs of a step
    uint8_t *heavy_flag;        // [2][num_envs] env is on its game's slow list
    int64_t heavy_ticks;        // wall-clock ticks (100 MHz) above which a step counts as slow
    int32_t slow_predict;       // also list envs the step predicts slow (pg_step.hip step_env; 0 = off)
    // level prefetch (single-game batches; pg_reset.hip): every env's next level is generated ahead,
    // on a side stream, into a spare state -- the next level depends only on the level-seed
    // generator (game.cpp:109-134) -- and swapped in when the episode ends.  Null when off.
    PGEnv *sp_envs;             // [num_envs] the spare's scalars
    float *sp_ents;             // as ents
    int16_t *sp_grid;           // num_envs * PG_GRID_MAX
    int8_t *sp_grid8;
    uint32_t *sp_mt;            // num_envs * 2 * PG_MT_WORDS (rand_gen, level_seed_rand_gen)
    int32_t *sp_latent;         // num_envs * PG_LATENT_N (maze, miner)
    int32_t *sp_level_seed;     // [num_envs] (the spare reset's level_seed output)
    PGEnv *sp_in;               // [sp_lag][num_envs] inputs of the spare resets, by act mod sp_lag
    uint32_t *sp_in_lsg;        // [sp_lag][num_envs][PG_MT_WORDS] their level-seed generators
    int32_t *sp_gen;            // [num_envs] act whose reset requested the env's spare (PG_SP_NONE: none)
    int32_t *sp_queue;          // [sp_lag][PG_NUM_GAMES][num_envs] envs whose spare to generate
    int32_t *sp_count;          // [sp_lag][PG_NUM_GAMES]
    int32_t sp_lag;             // a spare requested at act a is swapped in from act a + sp_lag
    uint32_t sp_mask[4];        // PGEnv words the step kernel may change: poisoned in the spare input
    int32_t render_rf;          // bit g: game g renders with pg_render_rf_kernel (host: options it serves)
};
#define PG_SP_LAG_MAX 8
#define PG_SP_NONE ((int32_t)0x80808080) // sp_gen of an env without a valid spare (memset 0x80)
#define PG_SP_SENT 0x7f7fbeefu   // poison of a step-changed word the spare reset did not write
#define PG_HEAVY_CAP 2048
#define PG_SCHED_RC 16
#define PG_SCHED_HC(p) ((p) ? 0 : 32)
#define PG_SCHED_CLEAR(p) ((p) ? 0 : 16) // first of the 32 ints to zero before a launch of parity p
#define PG_ROT_N 16
#define PG_TABLE_SLOT 99 // image slot of a game's Qt-tabulated overlay raster (jumper's compass)
#define PG_LATENT_N (2 + PG_LATENT_GRID + 2 + 2)

// The tables of game G (kernels are instantiated per game).
static inline __host__ __device__ PGDev game_view(const PGDev &d, int g) {
    PGDev v = d;
    v.sprites = d.sprites + (size_t)g * PG_NUM_SLOTS * 4;
    v.backgrounds = d.backgrounds + (size_t)g * PG_MAX_BG * 4;
    v.num_themes = d.num_themes + (size_t)g * 100;
    v.num_backgrounds = d.num_bg[g];
    return v;
}
