/*
 * procgen_oracle.c -- scalar CPU restatement of the reference step path.
 *
 * TEST INFRASTRUCTURE ONLY (see procgen_oracle.h): this is the checker the HIP
 * engine is compared against, never the product.  Every function cites the
 * reference file:line it restates (paths relative to /root/reference/procgen/src).
 *
 * Build: oracle/Makefile, -O2 -march=x86-64 -ffp-contract=off (no FMA
 * contraction: the reference's float/double arithmetic must be reproduced
 * operation by operation).
 *
 * Floating point: C promotion rules are kept exactly as the reference C++ has
 * them (e.g. `.9 * vx` is a double multiply then a float store).  libm calls use
 * the precision the reference TU resolves to: double sqrt
 * in basic_step_object, double `sign` in push_obj.
 */
#include "procgen_oracle.h"

#include <math.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ constants */
/* game.h:25-28 */
#define RES_W 64
#define RES_H 64
/* object-ids.h:9-27 */
#define INVALID_OBJ (-1)
#define INVALID_IDX (-2)
#define PLAYER 0
#define SPACE 100
#define WALL_OBJ 51
#define EXIT_OBJ 52
#define AGENT_OBJ 53
#define EXPLOSION 54
#define EXPLOSION5 58
#define TRAIL 59
#define DOOR_OBJ 200
#define KEY_OBJ 300
/* basic-abstract-game.cpp:6-20 */
static const float PI_F = 3.14159265358979323846264338327950288f; /* cpp-utils.h:12 */
#define MIXRATEROT 0.5f
#define POS_EPS (-0.001f)
#define RENDER_EPS 0.02f
#define USE_ASSET_THRESHOLD 100
#define MAX_ASSETS 100
#define MAX_IMAGE_THEMES 10
/* game.h:34-39 */
enum { EasyMode = 0, HardMode = 1, ExtremeMode = 2, MemoryMode = 10 };

#define MAX_ENTS 8192
#define MAX_GRID (64 * 64)
/* MazeGen arrays: array_dim = maze_dim + 2 <= world 31 (memory maze) + 2 */
#define MAZE_MAX_CELLS (33 * 33)

/* game ids: index in the reference's env list (procgen/env.py:15-32) */
enum { GAME_BIGFISH = 0, GAME_BOSSFIGHT = 1, GAME_CAVEFLYER = 2, GAME_CHASER = 3, GAME_CLIMBER = 4, GAME_COINRUN = 5, GAME_DODGEBALL = 6, GAME_FRUITBOT = 7, GAME_HEIST = 8, GAME_JUMPER = 9, GAME_LEAPER = 10, GAME_MAZE = 11,
       GAME_MINER = 12, GAME_NINJA = 13, GAME_PLUNDER = 14, GAME_STARPILOT = 15 };

static void fatal_msg(const char *m) {
    fprintf(stderr, "oracle fatal: %s\n", m);
    abort();
}
#define fassert(c)                                  \
    do {                                            \
        if (!(c)) fatal_msg("fassert failed: " #c); \
    } while (0)

/* ================================================================== MT19937
 * std::mt19937 as libstdc++ implements it (standard-defined; randgen.h:12). */
typedef struct {
    uint32_t mt[624];
    int mti;
    bool is_seeded;
} MT;

static void mt_seed(MT *m, uint32_t s) { /* std::mersenne_twister_engine::seed */
    m->mt[0] = s;
    for (int i = 1; i < 624; i++) m->mt[i] = 1812433253u * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
    m->mti = 624;
    m->is_seeded = true;
}

static void mt_twist(MT *m) {
    for (int i = 0; i < 624; i++) {
        uint32_t y = (m->mt[i] & 0x80000000u) | (m->mt[(i + 1) % 624] & 0x7fffffffu);
        m->mt[i] = m->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m->mti = 0;
}

static uint32_t mt_next(MT *m) {
    if (m->mti >= 624) mt_twist(m);
    uint32_t y = m->mt[m->mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* ================================================================== RandGen (randgen.cpp) */
static int rg_randint(MT *m, int low, int high) { /* randgen.cpp:6-11 */
    fassert(m->is_seeded);
    uint32_t x = mt_next(m);
    uint32_t range = (uint32_t)high - (uint32_t)low;
    return (int)((uint32_t)low + (x % range));
}
static int rg_randn(MT *m, int high) { /* randgen.cpp:13-17 */
    fassert(m->is_seeded);
    uint32_t x = mt_next(m);
    return (int)(x % (uint32_t)high);
}
static float rg_rand01(MT *m) { /* randgen.cpp:19-23 */
    fassert(m->is_seeded);
    uint32_t x = mt_next(m);
    return (float)((double)x / ((double)0xffffffffu + 1));
}
static bool rg_randbool(MT *m) { return (double)rg_rand01(m) > .5; }                          /* :25-27 */
static float rg_randrange(MT *m, float lo, float hi) { return rg_rand01(m) * (hi - lo) + lo; } /* :29-31 */
static int rg_randint0(MT *m) { /* randgen.cpp:90-93 */
    fassert(m->is_seeded);
    return (int)mt_next(m);
}
static void rg_seed(MT *m, int seed) { mt_seed(m, (uint32_t)seed); } /* :95-98 */

/* ================================================================== Entity (entity.h/.cpp) */
typedef struct {
    float x, y, vx, vy, rx, ry;
    int type, image_type, image_theme, render_z;
    bool will_erase, collides_with_entities;
    float collision_margin, rotation, vrot;
    bool is_reflected;
    int fire_time, spawn_time, life_time, expire_time;
    bool use_abs_coords;
    float friction;
    bool smart_step, avoids_collisions, auto_erase;
    float alpha, health, theta, grow_rate, alpha_decay, climber_spawn_x;
} Entity;

static void entity_init(Entity *e, float x, float y, float vx, float vy, float rx, float ry, int type) {
    /* entity.cpp:8-47 */
    memset(e, 0, sizeof(*e));
    e->x = x; e->y = y; e->vx = vx; e->vy = vy; e->rx = rx; e->ry = ry;
    e->type = type; e->image_type = type; e->image_theme = 0;
    e->will_erase = false; e->collides_with_entities = false;
    e->collision_margin = 0.0f; e->rotation = 0.0f; e->is_reflected = false; e->vrot = 0.0f;
    e->alpha = 1.0f; e->grow_rate = 1.0f; e->alpha_decay = 1.0f;
    e->fire_time = -1; e->spawn_time = -1; e->expire_time = -1; e->life_time = 0;
    e->health = 1; e->theta = -100;
    e->friction = 1; e->smart_step = false; e->avoids_collisions = false; e->auto_erase = true;
    e->render_z = 0; e->use_abs_coords = false; e->climber_spawn_x = 0;
    if (type == EXPLOSION) {
        e->grow_rate = 1.4f;
        e->expire_time = 4;
    } else if (type == TRAIL) {
        e->grow_rate = 1.05f;
        e->alpha_decay = 0.8f;
    }
}

static void entity_step(Entity *e) { /* entity.cpp:57-82 */
    if (!e->smart_step) {
        e->x += e->vx;
        e->y += e->vy;
    }
    e->rotation += e->vrot;
    e->vx *= e->friction;
    e->vy *= e->friction;
    e->life_time += 1;
    if (e->expire_time > 0 && e->life_time > e->expire_time) e->will_erase = true;
    if (e->type == EXPLOSION) {
        if (e->image_type < EXPLOSION5) e->image_type++;
    }
    e->rx *= e->grow_rate;
    e->ry *= e->grow_rate;
    e->alpha = e->alpha_decay * e->alpha;
}

/* ================================================================== game state */
typedef struct {
    /* GameOptions (game.h:47-61) */
    bool paint_vel_info, use_generated_assets, use_monochrome_assets, restrict_themes;
    bool use_backgrounds, center_agent, use_sequential_levels;
    int debug_mode, distribution_mode;
} GameOptions;

typedef struct {
    int game_id;
    GameOptions options;
    /* Game (game.h:64-134) */
    bool grid_step;
    int level_seed_low, level_seed_high, game_n;
    MT level_seed_rand_gen, rand_gen;
    float sd_reward;
    bool sd_done, sd_level_complete;
    int action, timeout, current_level_seed, prev_level_seed, episodes_remaining;
    bool episode_done;
    int last_reward_timer;
    float last_reward;
    int default_action, cur_time, reset_count;
    float total_reward;
    /* BasicAbstractGame (basic-abstract-game.h) */
    int grid_size, grid_w, grid_h;
    int grid[MAX_GRID];
    Entity *ents;
    int num_ents;
    bool agent_erased; /* agent removed from `entities` but still referenced by `agent` */
    Entity agent_ghost;
    int background_index;
    float bg_tile_ratio, bg_pct_x, char_dim;
    int last_move_action, move_action, special_action;
    float mixrate, maxspeed, max_jump;
    float action_vx, action_vy, action_vrot;
    float center_x, center_y;
    bool random_agent_start, has_useful_vel_info;
    int step_rand_int;
    int main_width, main_height, out_of_bounds_object;
    float unit, view_dim, x_off, y_off, visibility, min_visibility;
    /* coinrun (coinrun.cpp:38-47) */
    float last_agent_y;
    int wall_theme;
    bool has_support, facing_right, is_on_crate;
    float gravity, air_control;
    /* bigfish (bigfish.cpp:20-22) */
    int fish_eaten;
    float r_inc;
    /* maze (maze.cpp:16-18) / heist (heist.cpp:18-21) */
    int maze_dim, world_dim, num_keys;
    bool has_keys[4];
    /* miner (miner.cpp:26-28) */
    int diamonds_remaining, main_area;
    bool died;
    /* climber (climber.cpp:30-36; has_support, facing_right, wall_theme, gravity, air_control shared
     * with coinrun's members above) */
    int coin_quota, coins_collected;
    /* chaser (chaser.cpp:26-35; free_cells / is_space_vec of the last reset) */
    int eat_timeout, egg_timeout, eat_time, total_enemies, total_orbs, orbs_collected, num_free;
    int last_fire_time; /* fruitbot (fruitbot.cpp:26-28), dodgeball (dodgeball.cpp:33) */
    /* dodgeball (dodgeball.cpp:28-35) */
    float db_min_dim, db_hard_min_dim, db_ball_vscale, db_ball_r;
    int db_num_enemies, db_enemy_fire_delay;
    /* plunder (plunder.cpp:19-31); lane_directions / target_bools / image_permutation / lane_vels */
    bool pl_lane_dirs[5], pl_target_bools[6];
    int pl_perm[6];
    float pl_lane_vels[5];
    int pl_num_lanes, pl_num_current_ship_types, pl_targets_hit, pl_target_quota;
    float pl_juice_left, pl_r_scale, pl_spawn_prob, pl_legend_r, pl_min_agent_x;
    /* starpilot (starpilot.cpp:34-48): the spawner list (sorted by spawn time, popped from the back);
     * the hp_* tables are init_hps() of the distribution mode */
    Entity sp_spawners[512];
    int sp_num_spawners;
    float sp_hp_vs[9], sp_hp_healths[9], sp_hp_bullet_r[9], sp_hp_object_r[9], sp_hp_prob[9];
    float sp_total_prob_weight, sp_hp_slow_v, sp_hp_weapon_bullet_dist, sp_hp_spawn_right_threshold;
    int sp_hp_min_enemy_delta_t, sp_hp_max_group_size, sp_hp_max_enemy_delta_t;
    /* bossfight (bossfight.cpp:34-58); boss / shields are entities 1 and 2 of the list */
    int bf_attack_modes[8], bf_num_attack_modes;
    int bf_time_to_swap, bf_invulnerable_duration, bf_vulnerable_duration, bf_num_rounds, bf_round_num,
        bf_round_health, bf_boss_vel_timeout, bf_curr_vel_timeout, bf_attack_mode, bf_player_laser_theme,
        bf_boss_laser_theme, bf_damaged_until_time;
    bool bf_shields_are_up, bf_barriers_moves_right;
    float bf_base_fire_prob, bf_boss_bullet_vel, bf_barrier_vel, bf_barrier_spawn_prob, bf_rand_pct, bf_rand_fire_pct,
        bf_rand_pct_x, bf_rand_pct_y;
    Entity *bf_boss, *bf_shields;
    /* ninja (ninja.cpp:25-33; has_support / facing_right / wall_theme / gravity / air_control shared) */
    float nj_jump_charge, nj_jump_charge_inc;
    /* jumper (jumper.cpp:31-39; has_support / facing_right / wall_theme shared; goal = entity 1) */
    int jp_jump_count, jp_jump_delta, jp_jump_time;
    float jp_compass_dim;
    int free_list[MAX_GRID];
    bool is_space[MAX_GRID];
    /* leaper (leaper.cpp:27-32) */
    int bottom_road_y, bottom_water_y, goal_y, num_road_lanes, num_water_lanes;
    float road_lane_speeds[8], water_lane_speeds[8];
    /* observation of the last step */
    uint32_t canvas[RES_W * RES_H];
    /* use_generated_assets: the env's 500 x 500 RGB32 background, repainted by AssetGen at every
     * reset (basic-abstract-game.cpp:60-63, 778-782) */
    uint32_t *gen_bg;
} Game;

typedef struct {
    int count, offset;
    Game *games;
    const or_atlas *atlas;
    /* use_generated_assets: the atlas the games draw from (generated sprites, one 500 x 500
     * background slot whose pixels are each env's gen_bg) */
    or_atlas gen_atlas;
    uint32_t *gen_pixels;
    or_image *gen_sprites, *gen_backgrounds;
    int32_t *gen_num_themes;
} Vec;

static Entity *AG(Game *g) { return g->agent_erased ? &g->agent_ghost : &g->ents[0]; }

/* ------------------------------------------------------------------ grid (grid.h) */
static bool grid_contains(Game *g, int x, int y) { return 0 <= y && y < g->grid_h && 0 <= x && x < g->grid_w; }
static void grid_set(Game *g, int x, int y, int v) {
    fassert(grid_contains(g, x, y));
    g->grid[y * g->grid_w + x] = v;
}
static int get_obj(Game *g, int x, int y) { /* basic-abstract-game.cpp:180-185 */
    if (!grid_contains(g, x, y)) return g->out_of_bounds_object;
    return g->grid[y * g->grid_w + x];
}
static void set_obj(Game *g, int x, int y, int v) { grid_set(g, x, y, v); } /* :229-231 */
static int get_obj_from_floats(Game *g, float i, float j) { /* :167-174 */
    if (i < 0) return g->out_of_bounds_object;
    if (j < 0) return g->out_of_bounds_object;
    return get_obj(g, (int)floorf(i), (int)floorf(j));
}
static void fill_elem(Game *g, int x, int y, int dx, int dy, int elem) { /* :125-131 (char elem) */
    signed char c = (signed char)elem;
    for (int j = 0; j < dx; j++)
        for (int k = 0; k < dy; k++) grid_set(g, x + j, y + k, c);
}

/* ------------------------------------------------------------------ entity list */
static int add_entity_rxy(Game *g, float x, float y, float vx, float vy, float rx, float ry, int type) {
    fassert(g->num_ents < MAX_ENTS);
    entity_init(&g->ents[g->num_ents], x, y, vx, vy, rx, ry, type);
    return g->num_ents++;
}
static int add_entity(Game *g, float x, float y, float vx, float vy, float r, int type) { /* :575-579 */
    return add_entity_rxy(g, x, y, vx, vy, r, r, type);
}

static bool is_out_of_bounds(Game *g, const Entity *e) { /* :1077-1093 */
    float x = e->x, y = e->y, rx = e->rx, ry = e->ry;
    if (x + rx < 0) return true;
    if (y + ry < 0) return true;
    if (x - rx > g->main_width) return true;
    if (y - ry > g->main_height) return true;
    return false;
}

static void erase_if_needed(Game *g) { /* :757-765 */
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *e = &g->ents[i];
        if (e->will_erase || (e->auto_erase && is_out_of_bounds(g, e))) {
            if (i == 0 && !g->agent_erased) {
                g->agent_ghost = *e;
                g->agent_erased = true;
            }
            memmove(&g->ents[i], &g->ents[i + 1], sizeof(Entity) * (size_t)(g->num_ents - i - 1));
            g->num_ents--;
        }
    }
}

static bool has_collision(const Entity *e1, const Entity *e2, float margin) { /* :1154-1159 */
    float threshold_x = (e1->rx + e2->rx) + margin;
    float threshold_y = (e1->ry + e2->ry) + margin;
    return (fabsf(e1->x - e2->x) < threshold_x) && (fabsf(e1->y - e2->y) < threshold_y);
}

static bool has_agent_collision(Game *g, const Entity *e1) { /* :1135-1140 */
    if (e1->type == PLAYER) return false;
    return has_collision(e1, AG(g), e1->collision_margin);
}

/* ================================================================== per-game hooks */
/* coinrun object ids, coinrun.cpp:13-30 */
#define CR_GOAL 1
#define CR_SAW 2
#define CR_SAW2 3
#define CR_ENEMY 5
#define CR_ENEMY1 6
#define CR_ENEMY2 7
#define CR_PLAYER_JUMP 9
#define CR_PLAYER_RIGHT1 12
#define CR_PLAYER_RIGHT2 13
#define CR_WALL_MID 15
#define CR_WALL_TOP 16
#define CR_LAVA_MID 17
#define CR_LAVA_TOP 18
#define CR_ENEMY_BARRIER 19
#define CR_CRATE 20
static const float CR_GOAL_REWARD = 10.0f;
static bool cr_is_wall(int t) { return t == CR_WALL_MID || t == CR_WALL_TOP; } /* :175-177 */
static bool cr_is_lava(int t) { return t == CR_LAVA_MID || t == CR_LAVA_TOP; } /* :179-181 */

static bool hook_is_blocked(Game *g, const Entity *src, int target, bool is_horizontal) {
    (void)is_horizontal;
    /* basic-abstract-game.cpp:494-501 */
    bool base = (target == WALL_OBJ) || (target == g->out_of_bounds_object);
    if (g->game_id == GAME_NINJA && target == 20) { /* ninja.cpp:128-141: WALL_MID */
        if (src->type == PLAYER) return true;
        if (src->type == 7) { /* THROWING_STAR: sticks to walls */
            ((Entity *)src)->vx = 0;
            ((Entity *)src)->vy = 0;
            return true;
        }
    }
    if (g->game_id == GAME_JUMPER) /* jumper.cpp:117-124: CAVEWALL 6, CAVEWALL_TOP 7 */
        return base || (src->type == PLAYER && (target == 6 || target == 7));
    if (g->game_id == GAME_COINRUN) { /* coinrun.cpp:204-211 */
        if (base) return true;
        if (src->type == PLAYER && cr_is_wall(target)) return true;
        return false;
    }
    if (g->game_id == GAME_FRUITBOT) /* fruitbot.cpp:83-85: PLAYER vs OUT_OF_BOUNDS_WALL 2 */
        return base || (src->type == PLAYER && target == 2);
    if (g->game_id == GAME_CHASER) { /* chaser.cpp:94-99: MAZE_WALL 5 */
        if (target == 5) return true;
        return base;
    }
    if (g->game_id == GAME_CLIMBER) { /* climber.cpp:147-154: WALL_MID 15, WALL_TOP 16 */
        if (base) return true;
        if (src->type == PLAYER && (target == 15 || target == 16)) return true;
        return false;
    }
    if (g->game_id == GAME_MINER) { /* miner.cpp:68-75: BOULDER 1, MOVING_BOULDER 3, OOB_WALL 10 */
        if (base) return true;
        if (src->type == PLAYER && (target == 1 || target == 3 || target == 10)) return true;
        return false;
    }
    return base;
}

/* bigfish object ids / constants (bigfish.cpp:7-17) */
#define BF_FISH 2
static const int BF_COMPLETION_BONUS = 10;
static const int BF_POSITIVE_REWARD = 1;
static const float BF_FISH_MIN_R = .25f;
static const float BF_FISH_MAX_R = 2;
static const int BF_FISH_QUOTA = 30;
/* maze (maze.cpp:6-12) */
static const float MZ_REWARD = 10.0f;
#define MZ_GOAL 2
/* heist (heist.cpp:10-15) */
static const float HS_COMPLETION_BONUS = 10.0f;
#define HS_LOCKED_DOOR 1
#define HS_KEY 2
#define HS_EXIT 9
#define HS_KEY_ON_RING 11

static bool hook_is_blocked_ents(Game *g, const Entity *src, const Entity *target, bool is_horizontal) {
    if (g->game_id == GAME_HEIST) { /* heist.cpp:66-71 */
        if (target->type == HS_LOCKED_DOOR) return !g->has_keys[target->image_theme];
    }
    if (g->game_id == GAME_COINRUN) { /* coinrun.cpp:187-202 */
        if (target->type == CR_CRATE && !is_horizontal) {
            Entity *agent = AG(g);
            if (agent->vy >= 0) return false;
            if (g->action_vy < 0) return false;
            if (g->last_agent_y < (target->y + target->ry + agent->ry)) return false;
            g->is_on_crate = true;
            return true;
        }
    }
    return hook_is_blocked(g, src, target->type, is_horizontal); /* :503-505 */
}

static bool hook_will_reflect(Game *g, int src, int target) {
    if (g->game_id == GAME_CAVEFLYER) /* caveflyer.cpp:120-122: ENEMY 5 off CAVEWALL 8 / out of bounds */
        return src == 5 && (target == 8 || target == g->out_of_bounds_object);
    if (g->game_id == GAME_COINRUN) /* coinrun.cpp:140-142 */
        return src == CR_ENEMY && (cr_is_wall(target) || target == CR_ENEMY_BARRIER);
    if (g->game_id == GAME_FRUITBOT) /* fruitbot.cpp:79-81: BAD_OBJ 4 off BARRIER 1 / WALL_OBJ */
        return src == 4 && (target == 1 || target == WALL_OBJ);
    if (g->game_id == GAME_DODGEBALL) /* dodgeball.cpp:98-100: ENEMY 4 off LAVA_WALL 1 / OOB_WALL 10 */
        return src == 4 && (target == 1 || target == g->out_of_bounds_object);
    if (g->game_id == GAME_CLIMBER) /* climber.cpp:113-115: ENEMY 5 off walls and ENEMY_BARRIER 19 */
        return src == 5 && (target == 15 || target == 16 || target == 19);
    if (g->game_id == GAME_MINER) /* miner.cpp:77-79: ENEMY 5 off BOULDER, DIAMOND, MOVING_BOULDER/DIAMOND, out of bounds */
        return src == 5 && (target == 1 || target == 2 || target == 3 || target == 4 || target == g->out_of_bounds_object);
    return false;
}

/* handle_collision(src, target) (basic :383-385 is empty) */
static void bf_prepare_boss(Game *g);
static int spawn_child(Game *g, int src_i, int type, float obj_r) { /* basic-abstract-game.cpp:233-239, match_vel false */
    Entity *src = &g->ents[src_i];
    return add_entity(g, src->x, src->y, 0, 0, obj_r, type);
}
static void hook_handle_collision(Game *g, int si, int ti) {
    Entity *src = &g->ents[si], *target = &g->ents[ti];
    if (g->game_id == GAME_CAVEFLYER && target->type == 4) { /* caveflyer.cpp:92-118: PLAYER_BULLET */
        bool erase_bullet = false;
        if (src->type == 3) { /* TARGET */
            src->health -= 1;
            erase_bullet = true;
            if (src->health <= 0 && !src->will_erase) {
                spawn_child(g, si, EXPLOSION, (float)(.5 * src->rx));
                src->will_erase = true;
                g->sd_reward += 3.0f; /* TARGET_REWARD */
            }
        } else if (src->type == 2 || src->type == 5 || src->type == 1) { /* OBSTACLE, ENEMY, GOAL */
            erase_bullet = true;
        }
        if (erase_bullet && !target->will_erase) {
            target->will_erase = true;
            int e = spawn_child(g, ti, EXPLOSION, (float)(.5 * target->rx));
            g->ents[e].vx = src->vx;
            g->ents[e].vy = src->vy;
        }
        return;
    }
    if (g->game_id == GAME_BOSSFIGHT) { /* bossfight.cpp:140-190 */
        if (src->type == 1) { /* PLAYER_BULLET */
            bool will_erase = false;
            if (target->type == 3) { /* SHIELDS */
                if (g->bf_shields_are_up) {
                    src->type = 6; /* REFLECTED_BULLET */
                    float theta = (float)(PI_F * (1.25 + .5 * g->bf_rand_pct));
                    src->vy = (float)(1 * sin((double)theta) * .5); /* PLAYER_BULLET_VEL (const int 1) */
                    src->vx = (float)(1 * cos((double)theta) * .5);
                    src->expire_time = 4;
                    src->life_time = 0;
                    src->alpha_decay = 0.8f;
                }
            } else if (target->type == 2) { /* BOSS */
                if (!g->bf_shields_are_up) {
                    target->health -= 1;
                    will_erase = true;
                    if ((int)target->health % g->bf_round_health == 0) {
                        g->sd_reward += 1; /* POSITIVE_REWARD (const int) */
                        if (target->health == 0) {
                            g->sd_done = true;
                            g->sd_reward += 10; /* COMPLETION_BONUS (const int) */
                            g->sd_level_complete = true;
                        } else {
                            g->bf_round_num++;
                            bf_prepare_boss(g);
                            g->bf_curr_vel_timeout = 40; /* BOSS_DAMAGED_TIMEOUT */
                            g->bf_damaged_until_time = g->cur_time + 40;
                        }
                    }
                }
            }
            if (will_erase && !src->will_erase) {
                src->will_erase = true;
                float tvx = target->vx, tvy = target->vy;
                int e = spawn_child(g, si, EXPLOSION, (float)(.5 * src->rx));
                g->ents[e].vx = tvx;
                g->ents[e].vy = tvy;
            }
        } else if (src->type == 7) { /* BARRIER */
            if (target->type == 4 || target->type == 1) { /* ENEMY_BULLET, PLAYER_BULLET */
                target->will_erase = true;
                spawn_child(g, ti, EXPLOSION, (float)(.5 * target->rx));
            } else if (target->type == 5) { /* LASER_TRAIL */
                target->will_erase = true;
            }
            src = &g->ents[si];
            if (src->health <= 0) {
                if (!src->will_erase) {
                    float svx = src->vx, svy = src->vy;
                    int e = spawn_child(g, si, EXPLOSION, (float)(.5 * src->rx));
                    g->ents[e].vx = svx;
                    g->ents[e].vy = svy;
                }
                g->ents[si].will_erase = true;
            }
        }
        return;
    }
    if (g->game_id == GAME_STARPILOT) { /* starpilot.cpp:138-145: BULLET_PLAYER 1 vs destructible non-CLOUD */
        int tt = target->type;
        bool destructible = tt == 4 || tt == 8 || tt == 7 || tt == 5; /* FLYER, FAST_FLYER, TURRET, METEOR */
        if (src->type == 1 && tt != 6 && destructible) {
            src->will_erase = true;
            target->health -= 1;
            float sx = src->x, sy = src->y, tvx = target->vx, tvy = target->vy, r = (float)(.5 * src->rx);
            add_entity(g, sx, sy, tvx, tvy, r, EXPLOSION);
        }
        return;
    }
    if (g->game_id == GAME_PLUNDER) { /* plunder.cpp:87-108 */
        if (src->type == 1) { /* PLAYER_BULLET */
            if (target->type == 7) { /* SHIP */
                target->will_erase = true;
                src->will_erase = true;
                if (g->pl_target_bools[target->image_theme]) {
                    g->pl_targets_hit += 1;
                    g->sd_reward += 1.0f; /* POSITIVE_REWARD */
                    g->pl_juice_left += 0.1f;
                } else {
                    g->pl_juice_left -= 0.1f;
                }
            } else if (target->type == 6) { /* PANEL */
                src->will_erase = true;
            }
            if (target->will_erase) {
                float tx = target->x, ty = target->y, tvx = target->vx / 2, tvy = target->vy / 2;
                float tr = (float)(.5 * target->rx);
                add_entity(g, tx, ty, tvx, tvy, tr, EXPLOSION);
            }
        }
        return;
    }
    if (g->game_id == GAME_DODGEBALL) { /* dodgeball.cpp:120-151 */
        if (target->type == 3) { /* PLAYER_BALL */
            if (src->type == 1) { /* LAVA_WALL */
                target->will_erase = true;
            } else if (src->type == 4) { /* ENEMY */
                src->health -= 1;
                target->will_erase = true;
                if (src->health <= 0 && !src->will_erase) {
                    src->will_erase = true;
                    g->sd_reward += 2; /* ENEMY_REWARD (const int 2.0f) */
                    int c = spawn_child(g, si, 8, src->rx); /* DUST_CLOUD */
                    Entity *ent = &g->ents[c];
                    ent->vrot = PI_F / 0.3f;
                    ent->grow_rate = 1.0f / 1.2f;
                    ent->expire_time = 4;
                    ent->alpha_decay = 0.9f;
                    ent->image_theme = g->step_rand_int % 9; /* choose_step_random_theme: 9 spaceEffect themes */
                }
            }
        } else if (target->type == 6) { /* ENEMY_BALL */
            if (src->type == 1) target->will_erase = true;
        }
        return;
    }
    if (g->game_id == GAME_FRUITBOT) { /* fruitbot.cpp:117-134 */
        if (src->type == 3) { /* PLAYER_BULLET */
            if (target->type == 1) { /* BARRIER */
                src->will_erase = true;
            } else if (target->type == 11) { /* LOCK */
                src->will_erase = true;
                target->will_erase = true;
                for (int k = 0; k < g->num_ents; k++) { /* the door of this lock */
                    Entity *ent = &g->ents[k];
                    if (ent->type == 10 && fabsf(ent->y - target->y) < 1) {
                        ent->will_erase = true;
                        break;
                    }
                }
            }
        }
    }
}

static void hook_handle_agent_collision(Game *g, Entity *obj) {
    if (g->game_id == GAME_COINRUN) { /* coinrun.cpp:123-131 */
        if (obj->type == CR_ENEMY) g->sd_done = true;
        else if (obj->type == CR_SAW) g->sd_done = true;
    } else if (g->game_id == GAME_BIGFISH) { /* bigfish.cpp:45-59 */
        if (obj->type == BF_FISH) {
            Entity *agent = AG(g);
            if (obj->rx > agent->rx) {
                g->sd_done = true;
            } else {
                g->sd_reward += BF_POSITIVE_REWARD;
                obj->will_erase = true;
                agent->rx += g->r_inc;
                agent->ry += g->r_inc;
                g->fish_eaten += 1;
            }
        }
    } else if (g->game_id == GAME_JUMPER) { /* jumper.cpp:86-96: GOAL 1, SPIKE 2 */
        if (obj->type == 1) {
            g->sd_reward += 10.0f; /* GOAL_REWARD */
            g->sd_level_complete = true;
            g->sd_done = true;
        } else if (obj->type == 2) {
            g->sd_done = true;
        }
    } else if (g->game_id == GAME_CAVEFLYER) { /* caveflyer.cpp:57-71 */
        if (obj->type == 1) { /* GOAL */
            g->sd_reward += 10.0f;
            g->sd_level_complete = true;
            g->sd_done = true;
        } else if (obj->type == 2 || obj->type == 5 || obj->type == 3) { /* OBSTACLE, ENEMY, TARGET */
            g->sd_done = true;
        }
    } else if (g->game_id == GAME_NINJA) { /* ninja.cpp:77-87 */
        if (obj->type == EXPLOSION) {
            g->sd_done = true;
        } else if (obj->type == 1) { /* GOAL */
            g->sd_reward += 10.0f;
            g->sd_level_complete = true;
            g->sd_done = true;
        }
    } else if (g->game_id == GAME_BOSSFIGHT) { /* bossfight.cpp:120-131: BOSS, BARRIER, ENEMY_BULLET */
        if (obj->type == 2 || obj->type == 7 || obj->type == 4) g->sd_done = true;
    } else if (g->game_id == GAME_STARPILOT) { /* starpilot.cpp:126-136 */
        int t = obj->type;
        if (t == 9) { /* FINISH_LINE */
            g->sd_done = true;
            g->sd_reward += 10.0f; /* COMPLETION_BONUS */
            g->sd_level_complete = true;
        } else if (t == 4 || t == 8 || t == 2 || t == 3 || t == 7 || t == 5) { /* is_lethal (:346-350) */
            g->sd_done = true;
        }
    } else if (g->game_id == GAME_DODGEBALL) { /* dodgeball.cpp:102-118 */
        if (obj->type == 4 || obj->type == 6 || obj->type == 1) { /* ENEMY, ENEMY_BALL, LAVA_WALL */
            g->sd_done = true;
        } else if (obj->type == 5) { /* DOOR */
            if (g->db_num_enemies == 0) {
                g->sd_done = true;
                g->sd_reward += 10.0f; /* COMPLETION_BONUS */
                g->sd_level_complete = true;
            }
        }
    } else if (g->game_id == GAME_FRUITBOT) { /* fruitbot.cpp:95-115 */
        if (obj->type == 1) { /* BARRIER */
            g->sd_done = true;
        } else if (obj->type == 4) { /* BAD_OBJ: PENALTY (const int -4) */
            g->sd_reward += -4;
            obj->will_erase = true;
        } else if (obj->type == 10) { /* LOCKED_DOOR */
            g->sd_done = true;
        } else if (obj->type == 7) { /* GOOD_OBJ: POSITIVE_REWARD (const int 1) */
            g->sd_reward += 1;
            obj->will_erase = true;
        } else if (obj->type == 12) { /* PRESENT */
            g->sd_reward += 10.0f; /* COMPLETION_BONUS */
            g->sd_done = true;
            g->sd_level_complete = true;
        }
    } else if (g->game_id == GAME_CHASER) { /* chaser.cpp:119-133: LARGE_ORB 2, ENEMY 6 */
        if (obj->type == 2) {
            g->eat_time = g->cur_time;
            g->sd_reward += 0.04f; /* ORB_REWARD */
            obj->will_erase = true;
        } else if (obj->type == 6) {
            if (g->cur_time - g->eat_time < g->eat_timeout) obj->will_erase = true;
            else g->sd_done = true;
        }
    } else if (g->game_id == GAME_LEAPER) { /* leaper.cpp:69-77: CAR 4, FINISH_LINE 5 */
        Entity *agent = AG(g);
        if (obj->type == 4) {
            g->sd_done = true;
        } else if (obj->type == 5 && agent->vx == 0 && agent->vy == 0) {
            g->sd_reward += 10; /* GOAL_REWARD (const int) */
            g->sd_done = true;
            g->sd_level_complete = true;
        }
    } else if (g->game_id == GAME_CLIMBER) { /* climber.cpp:93-103: ENEMY 5, COIN 1 */
        if (obj->type == 5) {
            g->sd_done = true;
        } else if (obj->type == 1) {
            g->sd_reward += 1.0f; /* COIN_REWARD */
            g->coins_collected += 1;
            obj->will_erase = true;
        }
    } else if (g->game_id == GAME_MINER) { /* miner.cpp:81-93: ENEMY 5, EXIT 6 */
        if (obj->type == 5) {
            g->sd_done = true;
        } else if (obj->type == 6) {
            if (g->diamonds_remaining == 0) {
                g->sd_reward += 10.0f; /* COMPLETION_BONUS */
                g->sd_level_complete = true;
                g->sd_done = true;
            }
        }
    } else if (g->game_id == GAME_HEIST) { /* heist.cpp:80-96 */
        if (obj->type == HS_EXIT) {
            g->sd_done = true;
            g->sd_reward = HS_COMPLETION_BONUS;
            g->sd_level_complete = true;
        } else if (obj->type == HS_KEY) {
            obj->will_erase = true;
            g->has_keys[obj->image_theme] = true;
        } else if (obj->type == HS_LOCKED_DOOR) {
            int door_num = obj->image_theme;
            if (g->has_keys[door_num]) obj->will_erase = true;
        }
    }
}

/* should_preserve_type_themes + mask_theme_if_necessary (basic-abstract-game.cpp:454-462, heist.cpp:42-44) */
static int mask_theme(Game *g, int theme, int type) {
    bool preserve = (g->game_id == GAME_HEIST && (type == HS_KEY || type == HS_LOCKED_DOOR)) ||
                    (g->game_id == GAME_PLUNDER && type == 7) || /* plunder.cpp:83-85: SHIP */
                    (g->game_id == GAME_LEAPER && type == PLAYER); /* leaper.cpp:87-89 */
    if (g->options.restrict_themes && !preserve) return 0;
    return theme;
}

/* should_draw_entity (basic-abstract-game.cpp:1052-1054, heist.cpp:73-78) */
static bool hook_should_draw_entity(Game *g, const Entity *e) {
    if (g->game_id == GAME_BOSSFIGHT && e->type == 3) return g->bf_shields_are_up; /* bossfight.cpp:133-138 */
    if (g->game_id == GAME_HEIST && e->type == HS_KEY_ON_RING) return g->has_keys[e->image_theme];
    return true;
}

static void hook_handle_grid_collision(Game *g, Entity *obj, int type, int i, int j) {
    (void)i; (void)j;
    if (g->game_id == GAME_NINJA) { /* ninja.cpp:89-106 */
        if (obj->type == PLAYER) {
            if (type == 14 || type == 6) g->sd_done = true; /* FIRE, BOMB */
        } else if (obj->type == 7) { /* THROWING_STAR */
            if (type == 6) {
                obj->will_erase = true;
                set_obj(g, i, j, SPACE);
                add_entity(g, (float)(i + .5), (float)(j + .5), 0, 0, .5, EXPLOSION);
            }
            if (type == 20) obj->will_erase = true;
        }
        return;
    }
    if (g->game_id == GAME_COINRUN) { /* coinrun.cpp:144-154 */
        if (obj->type == PLAYER) {
            if (type == CR_GOAL) {
                g->sd_reward += CR_GOAL_REWARD;
                g->sd_done = true;
                g->sd_level_complete = true;
            } else if (cr_is_lava(type)) {
                g->sd_done = true;
            }
        }
    }
}

static int hook_image_for_type(Game *g, int type) {
    if (g->game_id == GAME_COINRUN) { /* coinrun.cpp:213-225 */
        if (type == PLAYER) {
            Entity *agent = AG(g);
            if (fabs((double)agent->vx) < .01 && g->action_vx == 0 && g->has_support) {
                return PLAYER;
            } else {
                return (g->cur_time / 5 % 2 == 0 || !g->has_support) ? CR_PLAYER_RIGHT1 : CR_PLAYER_RIGHT2;
            }
        } else if (type == CR_ENEMY_BARRIER) {
            return -1;
        }
    }
    if (g->game_id == GAME_DODGEBALL && type == 5) /* dodgeball.cpp:90-96: DOOR -> DOOR_OPEN 7 when clear */
        return g->db_num_enemies == 0 ? 7 : 5;
    if (g->game_id == GAME_CHASER && type == 6) { /* chaser.cpp:101-113: ENEMY */
        if (g->cur_time - g->eat_time < g->eat_timeout) return 3; /* ENEMY_WEAK */
        int rem = (g->cur_time / 2) % 4;
        if (rem == 3) rem = 1;
        return 6 + rem;
    }
    if (g->game_id == GAME_CLIMBER) { /* climber.cpp:156-170 */
        if (type == PLAYER) {
            Entity *agent = AG(g);
            if (!g->has_support) return 9; /* PLAYER_JUMP */
            if (fabsf(agent->vx) < .01 && g->action_vx == 0 && g->has_support) return PLAYER;
            return (g->cur_time / 5 % 2 == 0 || !g->has_support) ? 12 : 13;
        } else if (type == 19) {
            return -1;
        }
    }
    if (g->game_id == GAME_JUMPER && type == PLAYER) { /* jumper.cpp:126-135 */
        Entity *agent = AG(g);
        if (fabs((double)agent->vx) < .01 && g->action_vx == 0 && g->has_support) return PLAYER;
        bool first = g->cur_time / 5 % 2 == 0 || !g->has_support;
        if (g->facing_right) return first ? 12 : 13; /* PLAYER_RIGHT1 / 2 */
        return first ? 10 : 11;                      /* PLAYER_LEFT1 / 2 */
    }
    if (g->game_id == GAME_NINJA && type == PLAYER) { /* ninja.cpp:143-153 */
        Entity *agent = AG(g);
        if (fabs((double)agent->vx) < .01 && g->action_vx == 0 && g->has_support) return PLAYER;
        return (g->cur_time / 5 % 2 == 0 || !g->has_support) ? 12 : 13; /* PLAYER_RIGHT1 / 2 */
    }
    if (g->game_id == GAME_MINER) { /* miner.cpp:95-103: MOVING_BOULDER -> BOULDER, MOVING_DIAMOND -> DIAMOND */
        if (type == 3) return 1;
        if (type == 4) return 2;
    }
    return abs(type); /* basic-abstract-game.cpp:446-448 */
}

static int hook_theme_for_grid_obj(Game *g, int type) {
    if (g->game_id == GAME_JUMPER) return (type == 6 || type == 7) ? g->wall_theme : 0; /* jumper.cpp:107-112 */
    if (g->game_id == GAME_NINJA) return type == 20 ? g->wall_theme : 0; /* ninja.cpp:119-124 */
    if (g->game_id == GAME_COINRUN || g->game_id == GAME_CLIMBER) { /* coinrun.cpp:133-138, climber.cpp:106-111 */
        if (type == 15 || type == 16) return g->wall_theme;
        return 0;
    }
    return 0;
}

static bool is_player_image(int t) {
    return t == PLAYER || t == CR_PLAYER_JUMP || t == CR_PLAYER_RIGHT1 || t == CR_PLAYER_RIGHT2;
}

/* ================================================================== physics (basic-abstract-game.cpp) */
static bool sub_step(Game *g, int obj_i, float _vx, float _vy, int depth);

static double dsign(double x) { return x > 0 ? +1 : (x == 0 ? 0 : -1); } /* cpp-utils.h:42-44 */

static bool push_obj(Game *g, int src_i, int target_i, bool is_horizontal, int depth) { /* :248-276 */
    Entity *src = &g->ents[src_i], *target = &g->ents[target_i];
    float rsum = is_horizontal ? (src->rx + target->rx) : (src->ry + target->ry);
    float delx = target->x - src->x;
    float dely = target->y - src->y;
    float t_vx = 0, t_vy = 0;
    if (is_horizontal) {
        t_vx = (float)((double)src->x + dsign(delx) * (double)rsum - (double)target->x);
    } else {
        t_vy = (float)((double)src->y + dsign(dely) * (double)rsum - (double)target->y);
    }
    bool block = false;
    if (depth < 5) block = sub_step(g, target_i, t_vx, t_vy, depth + 1);
    target = &g->ents[target_i];
    if (is_horizontal) target->vx = 0;
    else target->vy = 0;
    return block;
}

/* diagnostic counters of the physics work (scripts only: how many sub_steps / collision-scan
 * iterations one step costs an env) */
static long long g_diag_substeps, g_diag_scans;
void oracle_diag_counters(long long *out, int reset) {
    out[0] = g_diag_substeps;
    out[1] = g_diag_scans;
    if (reset) g_diag_substeps = g_diag_scans = 0;
}

static bool sub_step(Game *g, int obj_i, float _vx, float _vy, int depth) { /* :278-380 */
    g_diag_substeps++;
    Entity *obj = &g->ents[obj_i];
    if (obj->will_erase) return false;
    float ny = obj->y + _vy;
    float nx = obj->x + _vx;
    float margin = 0.98f;
    bool is_horizontal = _vx != 0;
    bool block = false, reflect = false;
    for (int i = 0; i < 2; i++) {
        for (int j = 0; j < 2; j++) {
            int type2 = get_obj_from_floats(g, nx + obj->rx * margin * (float)(2 * i - 1),
                                            ny + obj->ry * margin * (float)(2 * j - 1));
            block = block || hook_is_blocked(g, obj, type2, is_horizontal);
            reflect = reflect || hook_will_reflect(g, obj->type, type2);
        }
    }
    if (reflect) {
        if (is_horizontal) {
            float delta;
            if (_vx < 0) delta = ceilf(nx - obj->rx) - (nx - obj->rx);
            else delta = floorf(nx + obj->rx) - (nx + obj->rx);
            obj->vx = -1 * obj->vx;
            nx = nx + 2 * delta;
        } else {
            float delta;
            if (_vy < 0) delta = ceilf(ny - obj->ry) - (ny - obj->ry);
            else delta = floorf(ny + obj->ry) - (ny + obj->ry);
            obj->vy = -1 * obj->vy;
            ny = ny + 2 * delta;
        }
    } else if (block) {
        if (is_horizontal) {
            if (g->grid_step) nx = obj->x;
            else nx = _vx > 0 ? (floorf(nx + obj->rx) - obj->rx) : (ceilf(nx - obj->rx) + obj->rx);
        } else {
            if (g->grid_step) ny = obj->y;
            else ny = _vy > 0 ? (floorf(ny + obj->ry) - obj->ry) : (ceilf(ny - obj->ry) + obj->ry);
        }
    }
    obj->x = nx;
    obj->y = ny;
    bool block2 = false;
    for (int i = g->num_ents - 1; i >= 0; i--) {
        obj = &g->ents[obj_i];
        Entity *m = &g->ents[i];
        if (i == obj_i || m->will_erase) continue;
        bool curr_block = false;
        if (has_collision(obj, m, POS_EPS)) {
            g_diag_scans++;
            if (hook_is_blocked_ents(g, obj, m, is_horizontal)) {
                curr_block = true;
            } else if (hook_will_reflect(g, obj->type, m->type)) {
                if (is_horizontal) {
                    float delx = m->x - obj->x;
                    float rsum = m->rx + obj->rx;
                    obj->x += _vx > 0 ? -2 * (rsum - delx) : 2 * (rsum + delx);
                    obj->vx = -1 * obj->vx;
                } else {
                    float dely = m->y - obj->y;
                    float rsum = m->ry + obj->ry;
                    obj->y += _vy > 0 ? -2 * (rsum - dely) : 2 * (rsum + dely);
                    obj->vy = -1 * obj->vy;
                }
            }
            if (curr_block) push_obj(g, i, obj_i, is_horizontal, depth);
        }
        block2 = block2 || curr_block;
    }
    return block || block2;
}

static void basic_step_object(Game *g, int obj_i) { /* :602-665 */
    Entity *obj = &g->ents[obj_i];
    if (obj->will_erase) return;
    int num_sub_steps;
    if (g->grid_step) {
        num_sub_steps = 1;
    } else {
        /* double sqrt: the TU resolves the unqualified sqrt to the C double function */
        num_sub_steps = (int)(4 * sqrt((double)(obj->vx * obj->vx + obj->vy * obj->vy)));
        if (num_sub_steps < 4) num_sub_steps = 4;
    }
    float pct = (float)(1.0 / num_sub_steps);
    float cmp = fabsf(obj->vx) - fabsf(obj->vy);
    bool step_x_first = cmp == 0 ? g->step_rand_int % 2 == 0 : (cmp > 0);
    if (obj->type == PLAYER) {
        if (g->action_vx != 0) step_x_first = true;
        if (g->action_vy != 0) step_x_first = false;
    }
    float vx_pct = 0, vy_pct = 0;
    for (int s = 0; s < num_sub_steps; s++) {
        bool block_x = false, block_y = false;
        if (step_x_first) {
            block_x = sub_step(g, obj_i, g->ents[obj_i].vx * pct, 0, 0);
            block_y = sub_step(g, obj_i, 0, g->ents[obj_i].vy * pct, 0);
        } else {
            block_y = sub_step(g, obj_i, 0, g->ents[obj_i].vy * pct, 0);
            block_x = sub_step(g, obj_i, g->ents[obj_i].vx * pct, 0, 0);
        }
        if (!block_x) vx_pct += 1;
        if (!block_y) vy_pct += 1;
        if (block_x && block_y) break;
    }
    vx_pct = vx_pct / (float)num_sub_steps;
    vy_pct = vy_pct / (float)num_sub_steps;
    obj = &g->ents[obj_i];
    obj->vx *= vx_pct;
    obj->vy *= vy_pct;
}

static void check_grid_collisions(Game *g, int ent_i) { /* :145-165 */
    Entity *ent = &g->ents[ent_i];
    float ax = ent->x, ay = ent->y, arx = ent->rx, ary = ent->ry;
    int min_x = (int)(ax - (arx + POS_EPS));
    int max_x = (int)(ax + (arx + POS_EPS));
    int min_y = (int)(ay - (ary + POS_EPS));
    int max_y = (int)(ay + (ary + POS_EPS));
    for (int x = min_x; x <= max_x; x++) {
        for (int y = min_y; y <= max_y; y++) {
            int grid_type = get_obj_from_floats(g, (float)x, (float)y);
            if (grid_type != SPACE) hook_handle_grid_collision(g, &g->ents[ent_i], grid_type, x, y);
        }
    }
}

static void step_entities(Game *g) { /* :1095-1107 */
    int count = g->num_ents;
    for (int i = count - 1; i >= 0; i--) {
        if (g->ents[i].smart_step) basic_step_object(g, i);
        entity_step(&g->ents[i]);
    }
}

/* ------------------------------------------------------------------ agent control */
static void coinrun_set_action_xy(Game *g, int move_action) { /* coinrun.cpp:451-472 */
    g->action_vx = (float)(move_action / 3 - 1);
    g->action_vy = (float)((move_action % 3) - 1);
    if (g->action_vx > 0) g->facing_right = true;
    if (g->action_vx < 0) g->facing_right = false;
    Entity *agent = AG(g);
    int obj_below_1 = get_obj_from_floats(g, (float)((double)agent->x - ((double)agent->rx - .01)),
                                          (float)((double)agent->y - ((double)agent->ry + .01)));
    int obj_below_2 = get_obj_from_floats(g, (float)((double)agent->x + ((double)agent->rx - .01)),
                                          (float)((double)agent->y - ((double)agent->ry + .01)));
#define CAN_SUPPORT(o) (cr_is_wall(o) || (o) == g->out_of_bounds_object) /* coinrun.cpp:447-449 */
    g->has_support = (g->is_on_crate || CAN_SUPPORT(obj_below_1) || CAN_SUPPORT(obj_below_2)) && agent->vy == 0;
#undef CAN_SUPPORT
    g->is_on_crate = false;
    if (g->action_vy == 1) {
        if (!g->has_support) g->action_vy = 0;
    }
}

static void climber_set_action_xy(Game *g, int move_action) { /* climber.cpp:299-318 */
    g->action_vx = (float)(move_action / 3 - 1);
    g->action_vy = (float)((move_action % 3) - 1);
    if (g->action_vy < 0) g->action_vy = 0;
    if (g->action_vx > 0) g->facing_right = true;
    if (g->action_vx < 0) g->facing_right = false;
    Entity *agent = AG(g);
    int obj_below_1 = get_obj_from_floats(g, (float)((double)agent->x - ((double)agent->rx - .01)),
                                          (float)((double)agent->y - ((double)agent->ry + .01)));
    int obj_below_2 = get_obj_from_floats(g, (float)((double)agent->x + ((double)agent->rx - .01)),
                                          (float)((double)agent->y - ((double)agent->ry + .01)));
#define CAN_SUPPORT(o) ((o) == 15 || (o) == 16 || (o) == g->out_of_bounds_object) /* :295-297 */
    g->has_support = CAN_SUPPORT(obj_below_1) || CAN_SUPPORT(obj_below_2);
#undef CAN_SUPPORT
    if (g->has_support && g->action_vy == 1) g->action_vy = 1;
    else g->action_vy = 0;
}

static void caveflyer_set_action_xy(Game *g, int move_action);
static void jumper_set_action_xy(Game *g, int move_action);
static void set_action_xy(Game *g, int move_action) {
    if (g->game_id == GAME_JUMPER) {
        jumper_set_action_xy(g, move_action);
        return;
    }
    if (g->game_id == GAME_CAVEFLYER) {
        caveflyer_set_action_xy(g, move_action);
        return;
    }
    if (g->game_id == GAME_NINJA) { /* ninja.cpp:387-418 */
        g->action_vx = (float)(move_action / 3 - 1);
        g->action_vy = (float)((move_action % 3) - 1);
        if (g->action_vy < 0) g->action_vy = 0;
        if (g->action_vx > 0) g->facing_right = true;
        if (g->action_vx < 0) g->facing_right = false;
        Entity *agent = AG(g);
        int b1 = get_obj_from_floats(g, (float)(agent->x - (agent->rx - .01)), (float)(agent->y - (agent->ry + .01)));
        int b2 = get_obj_from_floats(g, (float)(agent->x + (agent->rx - .01)), (float)(agent->y - (agent->ry + .01)));
        g->has_support = (b1 == 20 || b1 == g->out_of_bounds_object) || (b2 == 20 || b2 == g->out_of_bounds_object);
        if (g->has_support && g->action_vy == 1) {
            g->action_vy = 1;
            g->nj_jump_charge += g->nj_jump_charge_inc;
            if (g->nj_jump_charge > 1) g->nj_jump_charge = 1;
        } else {
            g->action_vy = 0;
        }
        if (!g->has_support) g->nj_jump_charge = 0;
        return;
    }
    if (g->game_id == GAME_PLUNDER) { /* plunder.cpp:110-114 */
        g->action_vx = (float)(move_action / 3 - 1);
        g->action_vy = 0;
        g->action_vrot = 0;
        return;
    }
    if (g->game_id == GAME_FRUITBOT) { /* fruitbot.cpp:154-158 */
        g->action_vx = (float)(move_action / 3 - 1);
        g->action_vy = 0.2f;
        g->action_vrot = 0;
        return;
    }
    if (g->game_id == GAME_COINRUN) {
        coinrun_set_action_xy(g, move_action);
        return;
    }
    if (g->game_id == GAME_CLIMBER) {
        climber_set_action_xy(g, move_action);
        return;
    }
    g->action_vx = (float)(move_action / 3 - 1); /* basic-abstract-game.cpp:667-671 */
    g->action_vy = (float)(move_action % 3 - 1);
    g->action_vrot = 0;
    if (g->game_id == GAME_MAZE || g->game_id == GAME_MINER) { /* maze.cpp:107-111, miner.cpp:105-109 */
        if (g->action_vx != 0) g->action_vy = 0;
    }
}

static float clip_abs(float x, float y) { /* cpp-utils.h:46-52 */
    if (x > y) return y;
    if (x < -y) return -y;
    return x;
}

static void lp_decay_vel(float *vel);
static double cu_sign(double x);
static void update_agent_velocity(Game *g) {
    Entity *agent = AG(g);
    if (g->game_id == GAME_JUMPER) { /* jumper.cpp:98-105 */
        float v_scale = 1.0f;
        agent->vx = (1 - g->mixrate) * agent->vx + g->mixrate * g->maxspeed * g->action_vx * v_scale;
        if (g->action_vy != 0) agent->vy = g->maxspeed * g->action_vy * 2;
        return;
    }
    if (g->game_id == GAME_CAVEFLYER) { /* caveflyer.cpp:73-81: no (1 - mixrate) decay */
        float v_scale = 1.0f;
        agent->vx = (float)((double)agent->vx + (double)(g->mixrate * g->maxspeed * g->action_vx * v_scale) * .2);
        agent->vy = (float)((double)agent->vy + (double)(g->mixrate * g->maxspeed * g->action_vy * v_scale) * .2);
        agent->vx = (float)(.9 * (double)agent->vx);
        agent->vy = (float)(.9 * (double)agent->vy);
        return;
    }
    if (g->game_id == GAME_NINJA) { /* ninja.cpp:108-121 */
        float mixrate_x = g->has_support ? g->mixrate : (g->mixrate * g->air_control);
        agent->vx = (1 - mixrate_x) * agent->vx + mixrate_x * g->maxspeed * g->action_vx;
        if (g->action_vy < 1 && g->nj_jump_charge > 0) {
            agent->vy = g->nj_jump_charge * g->max_jump;
            g->nj_jump_charge = 0;
        }
        if (!g->has_support) {
            if (agent->vy > -2) agent->vy -= g->gravity;
        }
        return;
    }
    if (g->game_id == GAME_COINRUN) { /* coinrun.cpp:156-173 */
        float mixrate_x = g->has_support ? g->mixrate : (g->mixrate * g->air_control);
        agent->vx = (1 - mixrate_x) * agent->vx + mixrate_x * g->maxspeed * g->action_vx;
        if (fabsf(agent->vx) < mixrate_x * g->maxspeed) agent->vx = 0;
        if (g->action_vy > 0) {
            agent->vy = g->max_jump;
        } else {
            if (g->has_support) agent->vy = (float)((double)agent->vy + .2 * (double)g->action_vy);
        }
        if (!(g->has_support && g->action_vy > 0)) {
            agent->vy -= g->gravity;
            agent->vy = clip_abs(agent->vy, g->max_jump);
        }
        return;
    }
    if (g->game_id == GAME_CHASER) { /* chaser.cpp:83-92 (cpp-utils sign, double) */
        if (g->action_vx != 0) agent->vx = g->maxspeed * g->action_vx;
        if (g->action_vy != 0) agent->vy = g->maxspeed * g->action_vy;
        agent->vx = (float)(cu_sign(agent->vx) * g->maxspeed);
        agent->vy = (float)(cu_sign(agent->vy) * g->maxspeed);
        return;
    }
    if (g->game_id == GAME_LEAPER) { /* leaper.cpp:228-244 */
        if (agent->vx == 0 && agent->vy == 0) {
            if (g->action_vx != 0) {
                agent->vx = g->maxspeed * g->action_vx;
                agent->image_theme = 1;
                agent->rotation = (agent->vx > 0 ? 1 : -1) * PI_F / 2;
            } else if (g->action_vy != 0) {
                agent->vy = g->maxspeed * g->action_vy;
                agent->image_theme = 1;
                agent->rotation = agent->vy > 0 ? 0 : PI_F;
            }
        }
        lp_decay_vel(&agent->vx);
        lp_decay_vel(&agent->vy);
        return;
    }
    if (g->game_id == GAME_CLIMBER) { /* climber.cpp:117-128 */
        float mixrate_x = g->has_support ? g->mixrate : (g->mixrate * g->air_control);
        agent->vx = (1 - mixrate_x) * agent->vx + mixrate_x * g->maxspeed * g->action_vx;
        if (g->action_vy > 0) agent->vy = g->max_jump;
        if (!g->has_support) {
            if (agent->vy > -2) agent->vy -= g->gravity;
        }
        return;
    }
    /* basic-abstract-game.cpp:678-693 */
    float v_scale = 1.0f;
    agent->vx = (1 - g->mixrate) * agent->vx;
    agent->vy = (1 - g->mixrate) * agent->vy;
    agent->vx += g->mixrate * g->maxspeed * g->action_vx * v_scale;
    agent->vy += g->mixrate * g->maxspeed * g->action_vy * v_scale;
    agent->vx = (float)(.9 * (double)agent->vx);
    agent->vy = (float)(.9 * (double)agent->vy);
}

/* ------------------------------------------------------------------ base game_step */
static void basic_game_step(Game *g) { /* basic-abstract-game.cpp:695-755 */
    g->step_rand_int = rg_randint(&g->rand_gen, 0, 1000000);
    g->move_action = g->action % 9;
    g->special_action = 0;
    if (g->action >= 9) {
        g->special_action = g->action - 8;
        g->move_action = 4;
    }
    if (g->move_action != 4) g->last_move_action = g->move_action;
    g->action_vrot = 0;
    g->action_vx = 0;
    g->action_vy = 0;
    set_action_xy(g, g->move_action);
    Entity *agent = AG(g);
    if (g->grid_step) {
        agent->vx = g->action_vx;
        agent->vy = g->action_vy;
    } else {
        update_agent_velocity(g);
        agent->vrot = MIXRATEROT * agent->vrot;
        agent->vrot += MIXRATEROT * (15 * PI_F / 180) * g->action_vrot;
    }
    step_entities(g);
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *ent = &g->ents[i];
        if (has_agent_collision(g, ent)) hook_handle_agent_collision(g, ent);
        if (ent->collides_with_entities) { /* :735-744 */
            for (int j = g->num_ents - 1; j >= 0; j--) {
                if (i == j) continue;
                Entity *e1 = &g->ents[i], *e2 = &g->ents[j];
                if (has_collision(e1, e2, e1->collision_margin) && !e1->will_erase && !e2->will_erase)
                    hook_handle_collision(g, i, j);
            }
        }
        if (g->ents[i].smart_step) check_grid_collisions(g, i);
    }
    erase_if_needed(g);
    g->sd_done = g->sd_done || is_out_of_bounds(g, AG(g));
}

/* ------------------------------------------------------------------ coinrun level generation */
static void choose_random_theme(Game *g, Entity *e, const or_atlas *at) { /* :1047-1050 */
    int nt = at->num_themes[e->image_type];
    fassert(nt > 0);
    e->image_theme = rg_randn(&g->rand_gen, nt);
}

static void cr_fill_block_top(Game *g, int x, int y, int dx, int dy, int fill, int top) { /* coinrun.cpp:227-231 */
    fassert(dy > 0);
    fill_elem(g, x, y, dx, dy - 1, fill);
    fill_elem(g, x, y + dy - 1, dx, 1, top);
}
static void cr_fill_ground_block(Game *g, int x, int y, int dx, int dy) {
    cr_fill_block_top(g, x, y, dx, dy, CR_WALL_MID, CR_WALL_TOP);
}
static void cr_fill_lava_block(Game *g, int x, int y, int dx, int dy) {
    cr_fill_block_top(g, x, y, dx, dy, CR_LAVA_MID, CR_LAVA_TOP);
}
static void cr_create_saw_enemy(Game *g, int x, int y) { /* :248-250 */
    add_entity(g, (float)(x + .5), (float)(y + .5), 0, 0, (float).5, CR_SAW);
}
static void cr_create_enemy(Game *g, int x, int y, const or_atlas *at) { /* :252-258 */
    int i = add_entity(g, (float)(x + .5), (float)(y + .5), (float)(.15 * (rg_randn(&g->rand_gen, 2) * 2 - 1)), 0,
                       (float).5, CR_ENEMY);
    Entity *e = &g->ents[i];
    e->smart_step = true;
    e->image_type = CR_ENEMY1;
    e->render_z = 1;
    choose_random_theme(g, e, at);
}
static void cr_create_crate(Game *g, int x, int y, const or_atlas *at) { /* :260-263 */
    int i = add_entity(g, (float)(x + .5), (float)(y + .5), 0, 0, (float).5, CR_CRATE);
    choose_random_theme(g, &g->ents[i], at);
}

static void cr_generate_coin_to_the_right(Game *g, const or_atlas *at) { /* coinrun.cpp:265-414 */
    MT *r = &g->rand_gen;
    int max_difficulty = 3;
    int dif = rg_randn(r, max_difficulty) + 1;
    int num_sections = rg_randn(r, dif) + dif;
    int curr_x = 5;
    int curr_y = 1;
    int pit_threshold = dif;
    int danger_type = rg_randn(r, 3);
    bool allow_pit = (g->options.debug_mode & (1 << 1)) == 0;
    bool allow_crate = (g->options.debug_mode & (1 << 2)) == 0;
    bool allow_dy = (g->options.debug_mode & (1 << 3)) == 0;
    int w = g->main_width;
    float _max_dy = g->max_jump * g->max_jump / (2 * g->gravity);
    float _max_dx = g->maxspeed * 2 * g->max_jump / g->gravity;
    int max_dy = (int)((double)_max_dy - .5);
    int max_dx = (int)((double)_max_dx - .5);
    bool allow_monsters = true;
    if (g->options.distribution_mode == EasyMode) allow_monsters = false;

    for (int section_idx = 0; section_idx < num_sections; section_idx++) {
        if (curr_x + 15 >= w) break;
        int dy = rg_randn(r, 4) + 1 + (int)(dif / 3);
        if (!allow_dy) dy = 0;
        if (dy > max_dy) dy = max_dy;
        if (curr_y >= 20) {
            dy *= -1;
        } else if (curr_y >= 5 && rg_randn(r, 2) == 1) {
            dy *= -1;
        }
        int dx = rg_randn(r, 2 * dif) + 3 + (int)(dif / 3);
        curr_y += dy;
        if (curr_y < 1) curr_y = 1;
        bool use_pit = allow_pit && (dx > 7) && (curr_y > 3) && (rg_randn(r, 20) >= pit_threshold);
        if (use_pit) {
            int x1 = rg_randn(r, 3) + 1;
            int x2 = rg_randn(r, 3) + 1;
            int pit_width = dx - x1 - x2;
            if (pit_width > max_dx) {
                pit_width = max_dx;
                x2 = dx - x1 - pit_width;
            }
            cr_fill_ground_block(g, curr_x, 0, x1, curr_y);
            cr_fill_ground_block(g, curr_x + dx - x2, 0, x2, curr_y);
            int lava_height = rg_randn(r, curr_y - 3) + 1;
            if (danger_type == 0) {
                cr_fill_lava_block(g, curr_x + x1, 1, pit_width, lava_height);
            } else if (danger_type == 1) {
                for (int ei = 0; ei < pit_width; ei++) cr_create_saw_enemy(g, curr_x + x1 + ei, 1);
            } else if (danger_type == 2) {
                for (int ei = 0; ei < pit_width; ei++) cr_create_enemy(g, curr_x + x1 + ei, 1, at);
            }
            if (pit_width > 4) {
                int x3, w1;
                if (pit_width == 5) {
                    x3 = 1 + rg_randn(r, 2);
                    w1 = 1 + rg_randn(r, 2);
                } else if (pit_width == 6) {
                    x3 = 2 + rg_randn(r, 2);
                    w1 = 1 + rg_randn(r, 2);
                } else {
                    x3 = 2 + rg_randn(r, 2);
                    int x4 = 2 + rg_randn(r, 2);
                    w1 = pit_width - x3 - x4;
                }
                cr_fill_ground_block(g, curr_x + x1 + x3, curr_y - 1, w1, 1);
            }
        } else {
            cr_fill_ground_block(g, curr_x, 0, dx, curr_y);
            int ob1_x = -1;
            int ob2_x = -1;
            if (rg_randn(r, 10) < (2 * dif) && dx > 3) {
                ob1_x = curr_x + rg_randn(r, dx - 2) + 1;
                cr_create_saw_enemy(g, ob1_x, curr_y);
            }
            if (rg_randn(r, 10) < dif && dx > 3 && (max_dx >= 4) && allow_monsters) {
                ob2_x = curr_x + rg_randn(r, dx - 2) + 1;
                cr_create_enemy(g, ob2_x, curr_y, at);
            }
            if (allow_crate) {
                for (int i = 0; i < 2; i++) {
                    int crate_x = curr_x + rg_randn(r, dx - 2) + 1;
                    if (rg_randn(r, 2) == 1 && ob1_x != crate_x && ob2_x != crate_x) {
                        int pile_height = rg_randn(r, 3) + 1;
                        for (int j = 0; j < pile_height; j++) cr_create_crate(g, crate_x, curr_y + j, at);
                    }
                }
            }
        }
        if (!cr_is_wall(get_obj(g, curr_x - 1, curr_y))) set_obj(g, curr_x - 1, curr_y, CR_ENEMY_BARRIER);
        curr_x += dx;
        set_obj(g, curr_x, curr_y, CR_ENEMY_BARRIER);
    }
    set_obj(g, curr_x, curr_y, CR_GOAL);
    cr_fill_ground_block(g, curr_x, 0, 1, curr_y);
    fill_elem(g, curr_x + 1, 0, g->main_width - curr_x - 1, g->main_height, CR_WALL_MID);
}

static void gen_paint_background(Game *g);
static void basic_game_reset(Game *g, const or_atlas *at) { /* basic-abstract-game.cpp:767-806 */
    fassert(g->main_width > 0 && g->main_height > 0);
    g->bg_pct_x = rg_rand01(&g->rand_gen);
    g->grid_size = g->main_width * g->main_height;
    fassert(g->grid_size <= MAX_GRID);
    g->grid_w = g->main_width;
    g->grid_h = g->main_height;
    memset(g->grid, 0, sizeof(g->grid));
    g->background_index = rg_randn(&g->rand_gen, at->num_backgrounds);
    if (g->gen_bg) gen_paint_background(g); /* AssetGen bggen(&rand_gen); generate_resource (:778-782) */
    g->num_ents = 0;
    g->agent_erased = false;
    float ax, ay;
    float a_r = 0.4f;
    if (g->random_agent_start) {
        ax = rg_rand01(&g->rand_gen) * (g->main_width - 2 * a_r) + a_r;
        ay = rg_rand01(&g->rand_gen) * (g->main_height - 2 * a_r) + a_r;
    } else {
        ax = a_r;
        ay = a_r;
    }
    int ai = add_entity(g, ax, ay, 0, 0, a_r, PLAYER);
    fassert(ai == 0);
    g->ents[0].smart_step = true;
    g->ents[0].render_z = 1;
    erase_if_needed(g);
    fill_elem(g, 0, 0, g->main_width, g->main_height, SPACE);
}

static void coinrun_game_reset(Game *g, const or_atlas *at) { /* coinrun.cpp:416-445 */
    basic_game_reset(g, at);
    g->gravity = 0.2f;
    g->max_jump = 1.5f;
    g->air_control = 0.15f;
    g->maxspeed = .5f;
    g->has_support = false;
    g->facing_right = true;
    Entity *agent = AG(g);
    if (g->options.distribution_mode == EasyMode) {
        agent->image_theme = 0;
        g->wall_theme = 0;
        g->background_index = 0;
    } else {
        choose_random_theme(g, agent, at);
        g->wall_theme = rg_randn(&g->rand_gen, 6);
    }
    agent->rx = .5f;
    agent->ry = 0.5787f;
    agent->x = 1 + agent->rx;
    agent->y = 1 + agent->ry;
    g->last_agent_y = agent->y;
    g->is_on_crate = false;
    /* init_floor_and_walls, coinrun.cpp:241-246 */
    fill_elem(g, 0, 0, g->main_width, 1, CR_WALL_TOP);
    fill_elem(g, 0, 0, 1, g->main_height, CR_WALL_MID);
    fill_elem(g, g->main_width - 1, 0, 1, g->main_height, CR_WALL_MID);
    fill_elem(g, 0, g->main_height - 1, g->main_width, 1, CR_WALL_MID);
    cr_generate_coin_to_the_right(g, at);
}

static void coinrun_game_step(Game *g) { /* coinrun.cpp:474-498 */
    basic_game_step(g);
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = false;
    if (g->action_vx < 0) agent->is_reflected = true;
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *ent = &g->ents[i];
        if (ent->type == CR_ENEMY) {
            float ex = ent->x, ey = (float)((double)ent->y - (double)ent->ry * .5);
            int ti = add_entity_rxy(g, ex, ey, 0, 0.01f, 0.3f, 0.2f, TRAIL);
            g->ents[ti].expire_time = 8;
            g->ents[ti].alpha = .5f;
            ent = &g->ents[i];
            ent->image_type = g->cur_time / 5 % 2 == 0 ? CR_ENEMY1 : CR_ENEMY2;
            ent->is_reflected = ent->vx > 0;
        } else if (ent->type == CR_SAW) {
            ent->image_type = g->cur_time % 2 == 0 ? CR_SAW : CR_SAW2;
        }
    }
    g->last_agent_y = AG(g)->y;
}

/* ================================================================== spawn helpers (basic-abstract-game.cpp) */
/* asset_aspect_ratios[img_idx] (:79-123): width * 1.0 / height of the image loaded for the slot,
 * after mask_theme_if_necessary picked the theme actually loaded. */
static float asset_aspect_ratio(Game *g, const or_atlas *at, int img_idx) {
    int type = img_idx % MAX_ASSETS, theme = img_idx / MAX_ASSETS;
    theme = mask_theme(g, theme, type);
    const or_image *im = &at->sprites[type + theme * MAX_ASSETS];
    fassert(im->w > 0 && im->h > 0);
    return (float)(im->w * 1.0 / im->h);
}

static void match_aspect_ratio(Game *g, const or_atlas *at, Entity *e) { /* :1023-1033, match_width = true */
    int img_idx = e->image_type + e->image_theme * MAX_ASSETS;
    e->ry = e->rx / asset_aspect_ratio(g, at, img_idx);
}

static float rand_pos(Game *g, float r, float min, float max) { /* :1109-1117 */
    fassert(min <= max);
    if (max - min <= 2 * r) return (max + min) / 2;
    float range = max - min;
    fassert(range >= 2 * r);
    return (range - 2 * r) * rg_rand01(&g->rand_gen) + r + min;
}

static bool has_any_collision(Game *g, const Entity *e1, float margin) { /* :1123-1133 */
    for (int i = g->num_ents - 1; i >= 0; i--) {
        const Entity *ent = &g->ents[i];
        if (!ent->avoids_collisions && has_collision(e1, ent, margin)) return true;
    }
    return false;
}

/* reposition (:548-569); `e` is not in `entities` yet */
static void reposition(Game *g, Entity *e, float x, float y, float w, float h, bool check_collisions) {
    float rx = e->rx, ry = e->ry;
    e->x = rand_pos(g, rx, x, x + w);
    e->y = rand_pos(g, ry, y, y + h);
    int count = 0;
    while ((has_agent_collision(g, e) || (check_collisions && has_any_collision(g, e, 0))) && (count < 100)) {
        e->x = rand_pos(g, rx, x, x + w);
        e->y = rand_pos(g, ry, y, y + h);
        count++;
    }
}

/* spawn_entity / spawn_entity_rxy (:520-527, 571-573) */
static int spawn_entity(Game *g, float r, int type, float x, float y, float w, float h) {
    Entity e;
    entity_init(&e, 0, 0, 0, 0, r, r, type);
    reposition(g, &e, x, y, w, h, true);
    fassert(g->num_ents < MAX_ENTS);
    g->ents[g->num_ents] = e;
    return g->num_ents++;
}

/* ================================================================== MazeGen (mazegen.cpp) */
#define MAZE_OFFSET 1
typedef struct {
    MT *rand_gen;
    int maze_dim, array_dim;
    int grid[MAZE_MAX_CELLS];              /* Grid<int> array_dim x array_dim */
    int cell_sets_idxs[MAZE_MAX_CELLS];    /* set label of maze cell maze_dim*y+x */
    int num_free_cells;
    int free_cells[MAZE_MAX_CELLS];
    bool in_free_set[MAZE_MAX_CELLS];
} MazeGen;

static void mg_init(MazeGen *m, MT *r, int maze_dim) { /* :12-20 */
    memset(m, 0, sizeof(*m));
    m->rand_gen = r;
    m->maze_dim = maze_dim;
    m->array_dim = maze_dim + 2;
    fassert(m->array_dim * m->array_dim <= MAZE_MAX_CELLS);
}
static void mg_set(MazeGen *m, int x, int y, int v) {
    fassert(0 <= x && x < m->array_dim && 0 <= y && y < m->array_dim);
    m->grid[y * m->array_dim + x] = v;
}
static int mg_gridget(MazeGen *m, int x, int y) {
    fassert(0 <= x && x < m->array_dim && 0 <= y && y < m->array_dim);
    return m->grid[y * m->array_dim + x];
}
static void mg_set_index(MazeGen *m, int idx, int v) {
    fassert(0 <= idx && idx < m->array_dim * m->array_dim);
    m->grid[idx] = v;
}
static void mg_set_free_cell(MazeGen *m, int x, int y) { /* :26-34 */
    mg_set(m, x + MAZE_OFFSET, y + MAZE_OFFSET, SPACE);
    int cell = m->maze_dim * y + x;
    if (!m->in_free_set[cell]) {
        m->free_cells[m->num_free_cells] = cell;
        m->in_free_set[cell] = true;
        m->num_free_cells += 1;
    }
}
static int mg_get_obj(MazeGen *m, int idx) { /* :36-47 */
    int x = idx % m->array_dim, y = idx / m->array_dim;
    if (x <= 0 || x >= m->array_dim - 1) return INVALID_OBJ;
    if (y <= 0 || y >= m->array_dim - 1) return INVALID_OBJ;
    return mg_gridget(m, x, y);
}
/* get_neighbors (:49-67): order (-1,0) (0,-1) (0,1) (1,0) */
static int mg_neighbors(MazeGen *m, int idx, int type, int *out) {
    int x = idx % m->array_dim, y = idx / m->array_dim, n = 0;
    for (int dx = -1; dx <= 1; dx++) {
        for (int dy = -1; dy <= 1; dy++) {
            if (dx == 0 && dy == 0) continue;
            if (dx != 0 && dy != 0) continue;
            int n_idx = (y + dy) * m->array_dim + (x + dx);
            if (mg_get_obj(m, n_idx) == type) out[n++] = n_idx;
        }
    }
    return n;
}

/* expand_to_type (:69-98) over ascending std::set<int> iteration, sets as bitmaps */
static int mg_expand_to_type(MazeGen *m, const bool *s0, bool *s1, int type) {
    int cells = m->array_dim * m->array_dim;
    static bool curr[MAZE_MAX_CELLS], next[MAZE_MAX_CELLS];
    memcpy(curr, s0, (size_t)cells);
    bool any = false;
    for (int i = 0; i < cells; i++) any = any || curr[i];
    while (any) {
        memset(next, 0, (size_t)cells);
        for (int elem = 0; elem < cells; elem++) {
            if (!curr[elem]) continue;
            int targets[4], adj[4];
            int nt = mg_neighbors(m, elem, type, targets);
            int na = mg_neighbors(m, elem, SPACE, adj);
            for (int k = 0; k < na; k++) {
                int j = adj[k];
                if (!s0[j] && !s1[j]) {
                    next[j] = true;
                    s1[j] = true;
                }
            }
            if (nt > 0) return targets[0];
        }
        any = false;
        for (int i = 0; i < cells; i++) {
            curr[i] = next[i];
            any = any || next[i];
        }
    }
    return -1;
}

static void mg_generate_maze(MazeGen *m) { /* :112-188 */
    int md = m->maze_dim;
    for (int i = 0; i < m->array_dim; i++)
        for (int j = 0; j < m->array_dim; j++) mg_set(m, i, j, WALL_OBJ);
    mg_set(m, MAZE_OFFSET, MAZE_OFFSET, 0);
    static int walls[2 * MAZE_MAX_CELLS][4];
    int nw = 0;
    m->num_free_cells = 0;
    memset(m->in_free_set, 0, sizeof(m->in_free_set));
    for (int i = 0; i < md * md; i++) m->cell_sets_idxs[i] = i;
    for (int i = 1; i < md; i += 2)
        for (int j = 0; j < md; j += 2)
            if (i > 0 && i < md - 1) {
                walls[nw][0] = i - 1; walls[nw][1] = j; walls[nw][2] = i + 1; walls[nw][3] = j;
                nw++;
            }
    for (int i = 0; i < md; i += 2)
        for (int j = 1; j < md; j += 2)
            if (j > 0 && j < md - 1) {
                walls[nw][0] = i; walls[nw][1] = j - 1; walls[nw][2] = i; walls[nw][3] = j + 1;
                nw++;
            }
    while (nw > 0) {
        int n = rg_randn(m->rand_gen, nw);
        int x1 = walls[n][0], y1 = walls[n][1], x2 = walls[n][2], y2 = walls[n][3];
        int s0_idx = m->cell_sets_idxs[md * y1 + x1];
        int s1_idx = m->cell_sets_idxs[md * y2 + x2];
        int x0 = (x1 + x2) / 2, y0 = (y1 + y2) / 2;
        int center = md * y0 + x0;
        bool can_remove = (mg_gridget(m, x0 + MAZE_OFFSET, y0 + MAZE_OFFSET) == WALL_OBJ) && (s0_idx != s1_idx);
        if (can_remove) {
            mg_set_free_cell(m, x1, y1);
            mg_set_free_cell(m, x0, y0);
            mg_set_free_cell(m, x2, y2);
            /* s1 |= s0 | {center}; every member relabelled s1_idx */
            for (int c = 0; c < md * md; c++)
                if (m->cell_sets_idxs[c] == s0_idx) m->cell_sets_idxs[c] = s1_idx;
            m->cell_sets_idxs[center] = s1_idx;
        }
        memmove(walls[n], walls[n + 1], sizeof(walls[0]) * (size_t)(nw - n - 1));
        nw--;
    }
}

static void mg_generate_maze_with_doors(MazeGen *m, int num_doors) { /* :213-290 */
    mg_generate_maze(m);
    int cells = m->array_dim * m->array_dim;
    static int forks[MAZE_MAX_CELLS], rem[MAZE_MAX_CELLS], chosen[MAZE_MAX_CELLS], space_cells[MAZE_MAX_CELLS];
    int nf = 0;
    for (int i = 0; i < cells; i++) {
        if (mg_get_obj(m, i) == SPACE) {
            int adj[4];
            if (mg_neighbors(m, i, SPACE, adj) > 2) forks[nf++] = i;
        }
    }
    /* RandGen::choose_n (randgen.cpp:49-68) */
    int nc = 0;
    if (num_doors > nf) {
        for (int i = 0; i < nf; i++) chosen[nc++] = forks[i];
    } else {
        int nr = nf;
        memcpy(rem, forks, sizeof(int) * (size_t)nf);
        while (nc < num_doors) {
            int k = rg_randn(m->rand_gen, nr);
            chosen[nc++] = rem[k];
            memmove(&rem[k], &rem[k + 1], sizeof(int) * (size_t)(nr - k - 1));
            nr--;
        }
    }
    num_doors = nc;
    for (int i = 0; i < nc; i++) mg_set_index(m, chosen[i], DOOR_OBJ);
    int agent_cell;
    {
        int ns = 0;
        for (int i = 0; i < cells; i++)
            if (mg_get_obj(m, i) == SPACE) space_cells[ns++] = i;
        int dn[4];
        do {
            fassert(ns > 0);
            agent_cell = space_cells[rg_randn(m->rand_gen, ns)];
        } while (mg_neighbors(m, agent_cell, DOOR_OBJ, dn) > 0);
        mg_set_index(m, agent_cell, AGENT_OBJ);
    }
    static bool s0[MAZE_MAX_CELLS], s1[MAZE_MAX_CELLS];
    memset(s0, 0, sizeof(s0));
    s0[agent_cell] = true;
    for (int door_num = 0; door_num < num_doors + 1; door_num++) {
        memset(s1, 0, sizeof(s1));
        int found_door = -1;
        if (door_num < num_doors) {
            found_door = mg_expand_to_type(m, s0, s1, DOOR_OBJ);
            mg_set_index(m, found_door, DOOR_OBJ + door_num + 1);
            for (int i = 0; i < cells; i++) s0[i] = s0[i] || s1[i];
        }
        mg_expand_to_type(m, s0, s1, -999);
        int ns = 0;
        for (int i = 0; i < cells; i++)
            if (s1[i]) space_cells[ns++] = i;
        fassert(ns > 0);
        int key_cell = space_cells[rg_randn(m->rand_gen, ns)];
        mg_set_index(m, key_cell, door_num == num_doors ? EXIT_OBJ : (KEY_OBJ + door_num + 1));
        for (int i = 0; i < cells; i++) s0[i] = s0[i] || s1[i];
        if (found_door >= 0) s0[found_door] = true;
    }
}

static void mg_generate_maze_no_dead_ends(MazeGen *m) { /* :190-211 */
    mg_generate_maze(m);
    int cells = m->array_dim * m->array_dim;
    for (int i = 0; i < cells; i++) {
        if (mg_get_obj(m, i) == SPACE) {
            int adj_space[4], adj_wall[4];
            if (mg_neighbors(m, i, SPACE, adj_space) == 1) {
                int nw = mg_neighbors(m, i, WALL_OBJ, adj_wall);
                if (nw > 0) mg_set_index(m, adj_wall[rg_randn(m->rand_gen, nw)], SPACE);
            }
        }
    }
}

static void mg_place_objects(MazeGen *m, int start_obj, int num_objs) { /* :292-306 */
    for (int j = 0; j < num_objs; j++) {
        int mm = rg_randn(m->rand_gen, m->num_free_cells);
        while (m->free_cells[mm] == -1 || m->free_cells[mm] == 0) mm = rg_randn(m->rand_gen, m->num_free_cells);
        int coin_cell = m->free_cells[mm];
        m->free_cells[mm] = -1;
        mg_set(m, coin_cell % m->maze_dim + MAZE_OFFSET, coin_cell / m->maze_dim + MAZE_OFFSET, start_obj + j);
    }
}

/* ================================================================== bigfish (games/bigfish.cpp) */
static void bigfish_game_reset(Game *g, const or_atlas *at) { /* :62-78 */
    basic_game_reset(g, at);
    g->options.center_agent = false;
    g->fish_eaten = 0;
    float start_r = .5f;
    if (g->options.distribution_mode == EasyMode) start_r = 1;
    g->r_inc = (BF_FISH_MAX_R - start_r) / BF_FISH_QUOTA;
    Entity *agent = AG(g);
    agent->rx = start_r;
    agent->ry = start_r;
    agent->y = 1 + agent->ry;
}

static void bigfish_game_step(Game *g, const or_atlas *at) { /* :80-106 */
    basic_game_step(g);
    MT *r = &g->rand_gen;
    if (rg_randn(r, 10) == 1) {
        /* pow(float, 1.4) is the double pow */
        float ent_r = (float)((double)(BF_FISH_MAX_R - BF_FISH_MIN_R) * pow((double)rg_rand01(r), 1.4) +
                              (double)BF_FISH_MIN_R);
        float ent_y = rg_rand01(r) * (g->main_height - 2 * ent_r);
        float moves_right = (double)rg_rand01(r) < .5;
        float ent_vx = (float)((.15 + (double)rg_rand01(r) * .25) * (moves_right ? 1 : -1));
        float ent_x = moves_right ? -1 * ent_r : g->main_width + ent_r;
        int i = add_entity(g, ent_x, ent_y, ent_vx, 0, ent_r, BF_FISH);
        Entity *ent = &g->ents[i];
        choose_random_theme(g, ent, at);
        match_aspect_ratio(g, at, ent);
        ent->is_reflected = !moves_right;
    }
    if (g->fish_eaten >= BF_FISH_QUOTA) {
        g->sd_done = true;
        g->sd_reward += BF_COMPLETION_BONUS;
        g->sd_level_complete = true;
    }
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = false;
    if (g->action_vx < 0) agent->is_reflected = true;
}

/* ================================================================== maze (games/maze.cpp) */
static void maze_choose_world_dim(Game *g) { /* :45-58 */
    int d = g->options.distribution_mode;
    if (d == EasyMode) g->world_dim = 15;
    else if (d == HardMode) g->world_dim = 25;
    else if (d == MemoryMode) g->world_dim = 31;
    g->main_width = g->world_dim;
    g->main_height = g->world_dim;
}

static void maze_game_reset(Game *g, const or_atlas *at) { /* :60-105 */
    maze_choose_world_dim(g);
    basic_game_reset(g, at);
    g->grid_step = true;
    g->maze_dim = rg_randn(&g->rand_gen, (g->world_dim - 1) / 2) * 2 + 3;
    int margin = (g->world_dim - g->maze_dim) / 2;
    static MazeGen mg;
    mg_init(&mg, &g->rand_gen, g->maze_dim);
    g->options.center_agent = g->options.distribution_mode == MemoryMode;
    Entity *agent = AG(g);
    agent->rx = .5f;
    agent->ry = .5f;
    agent->x = (float)(margin + .5);
    agent->y = (float)(margin + .5);
    mg_generate_maze(&mg);
    mg_place_objects(&mg, MZ_GOAL, 1);
    for (int i = 0; i < g->grid_size; i++) g->grid[i] = WALL_OBJ;
    for (int i = 0; i < g->maze_dim; i++)
        for (int j = 0; j < g->maze_dim; j++)
            set_obj(g, margin + i, margin + j, mg_gridget(&mg, i + MAZE_OFFSET, j + MAZE_OFFSET));
    if (margin > 0) {
        for (int i = 0; i < g->maze_dim + 2; i++) {
            set_obj(g, margin - 1, margin + i - 1, WALL_OBJ);
            set_obj(g, margin + g->maze_dim, margin + i - 1, WALL_OBJ);
            set_obj(g, margin + i - 1, margin - 1, WALL_OBJ);
            set_obj(g, margin + i - 1, margin + g->maze_dim, WALL_OBJ);
        }
    }
}

static void maze_game_step(Game *g) { /* :113-131 */
    basic_game_step(g);
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = true;
    if (g->action_vx < 0) agent->is_reflected = false;
    int ix = (int)agent->x;
    int iy = (int)agent->y;
    if (get_obj(g, ix, iy) == MZ_GOAL) {
        set_obj(g, ix, iy, SPACE);
        g->sd_reward += MZ_REWARD;
        g->sd_level_complete = true;
    }
    g->sd_done = g->sd_reward > 0;
}

/* ================================================================== heist (games/heist.cpp) */
static void heist_choose_world_dim(Game *g) { /* :98-113 */
    int d = g->options.distribution_mode;
    if (d == EasyMode) g->world_dim = 9;
    else if (d == HardMode) g->world_dim = 13;
    else if (d == MemoryMode) g->world_dim = 23;
    g->maxspeed = .75f;
    g->main_width = g->world_dim;
    g->main_height = g->world_dim;
}

static void heist_game_reset(Game *g, const or_atlas *at) { /* :115-203 */
    heist_choose_world_dim(g);
    basic_game_reset(g, at);
    MT *r = &g->rand_gen;
    int min_maze_dim = 5;
    int max_diff = (g->world_dim - min_maze_dim) / 2;
    int difficulty = rg_randn(r, max_diff + 1);
    g->options.center_agent = g->options.distribution_mode == MemoryMode;
    if (g->options.distribution_mode == MemoryMode) g->num_keys = rg_randn(r, 4);
    else g->num_keys = difficulty + rg_randn(r, 2);
    if (g->num_keys > 3) g->num_keys = 3;
    for (int i = 0; i < 4; i++) g->has_keys[i] = false;
    int maze_dim = difficulty * 2 + min_maze_dim;
    float maze_scale = (float)(g->main_height / (g->world_dim * 1.0));
    Entity *agent = AG(g);
    agent->rx = (float)(.375 * maze_scale);
    agent->ry = (float)(.375 * maze_scale);
    float r_ent = maze_scale / 2;
    static MazeGen mg;
    mg_init(&mg, r, maze_dim);
    mg_generate_maze_with_doors(&mg, g->num_keys);
    agent->x = -1;
    agent->y = -1;
    int off_x = rg_randn(r, g->world_dim - maze_dim + 1);
    int off_y = rg_randn(r, g->world_dim - maze_dim + 1);
    for (int i = 0; i < g->grid_size; i++) g->grid[i] = WALL_OBJ;
    for (int i = 0; i < maze_dim; i++) {
        for (int j = 0; j < maze_dim; j++) {
            int x = off_x + i, y = off_y + j;
            int obj = mg_gridget(&mg, i + MAZE_OFFSET, j + MAZE_OFFSET);
            float obj_x = (float)((x + .5) * maze_scale);
            float obj_y = (float)((y + .5) * maze_scale);
            if (obj != WALL_OBJ) set_obj(g, x, y, SPACE);
            if (obj >= KEY_OBJ) {
                int k = spawn_entity(g, (float)(.375 * maze_scale), HS_KEY, maze_scale * x, maze_scale * y, maze_scale,
                                     maze_scale);
                g->ents[k].image_theme = obj - KEY_OBJ - 1;
                match_aspect_ratio(g, at, &g->ents[k]);
            } else if (obj >= DOOR_OBJ) {
                int k = add_entity(g, obj_x, obj_y, 0, 0, r_ent, HS_LOCKED_DOOR);
                g->ents[k].image_theme = obj - DOOR_OBJ - 1;
            } else if (obj == EXIT_OBJ) {
                int k = spawn_entity(g, (float)(.375 * maze_scale), HS_EXIT, maze_scale * x, maze_scale * y, maze_scale,
                                     maze_scale);
                match_aspect_ratio(g, at, &g->ents[k]);
            } else if (obj == AGENT_OBJ) {
                agent = AG(g);
                agent->x = obj_x;
                agent->y = obj_y;
            }
        }
    }
    float ring_key_r = 0.03f;
    for (int i = 0; i < g->num_keys; i++) {
        int k = add_entity(g, (float)(1 - ring_key_r * (2 * i + 1.25)), (float)(ring_key_r * .75), 0, 0, ring_key_r,
                           HS_KEY_ON_RING);
        Entity *e = &g->ents[k];
        e->image_theme = i;
        e->image_type = HS_KEY;
        e->rotation = PI_F / 2;
        e->render_z = 1;
        e->use_abs_coords = true;
        match_aspect_ratio(g, at, e);
    }
}

static void heist_game_step(Game *g) { /* :205-209 */
    basic_game_step(g);
    Entity *agent = AG(g);
    /* Entity::face_direction (entity.cpp:84-88): entity.cpp includes <math.h>, so atan2 of
     * floats is atan2f */
    float dx = g->action_vx, dy = g->action_vy;
    if (dx != 0 || dy != 0) agent->rotation = -1 * atan2f(dy, dx) + 0.0f;
}

/* ================================================================== miner (games/miner.cpp, fork-modified) */
#define MN_BOULDER 1
#define MN_DIAMOND 2
#define MN_MOVING_BOULDER 3
#define MN_MOVING_DIAMOND 4
#define MN_ENEMY 5
#define MN_EXIT 6
#define MN_DIRT 9
#define MN_OOB_WALL 10
#define MN_MUD 11
#define MN_DEAD_PLAYER 12
static const float MN_DIAMOND_REWARD = 1.0f;

static int get_obj_idx(Game *g, int idx) { /* basic-abstract-game.cpp:194-199 */
    if (!(0 <= idx && idx < g->grid_w * g->grid_h)) return g->out_of_bounds_object;
    return g->grid[idx];
}
static void set_obj_idx(Game *g, int idx, int v) { /* :225-227 */
    fassert(0 <= idx && idx < g->grid_w * g->grid_h);
    g->grid[idx] = v;
}
static int mn_agent_index(Game *g) { /* miner.cpp:98-100 */
    Entity *a = AG(g);
    return (int)a->y * g->main_width + (int)a->x;
}
static int mn_moving_type(int t) { /* :220-227 */
    if (t == MN_DIAMOND) return MN_MOVING_DIAMOND;
    if (t == MN_BOULDER) return MN_MOVING_BOULDER;
    return t;
}
static bool mn_is_moving(int t) { return t == MN_MOVING_BOULDER || t == MN_MOVING_DIAMOND; } /* :229-231 */
static int mn_stationary_type(int t) { /* :233-240 */
    if (t == MN_MOVING_DIAMOND) return MN_DIAMOND;
    if (t == MN_MOVING_BOULDER) return MN_BOULDER;
    return t;
}
static bool mn_is_free(Game *g, int idx) { /* :242-244 */
    return get_obj_idx(g, idx) == SPACE && (mn_agent_index(g) != idx);
}
static bool mn_is_round(int t) { /* :246-248 */
    return t == MN_BOULDER || t == MN_MOVING_BOULDER || t == MN_DIAMOND || t == MN_MOVING_DIAMOND;
}

static void miner_choose_world_dim(Game *g) { /* :119-132 */
    int d = g->options.distribution_mode;
    if (d == EasyMode) { g->main_width = 10; g->main_height = 10; }
    else if (d == HardMode) { g->main_width = 20; g->main_height = 20; }
    else if (d == MemoryMode) { g->main_width = 35; g->main_height = 35; }
    g->main_area = g->main_width * g->main_height;
}

static void miner_game_reset(Game *g, const or_atlas *at) { /* :134-218 */
    miner_choose_world_dim(g);
    basic_game_reset(g, at);
    MT *r = &g->rand_gen;
    g->died = false;
    Entity *agent = AG(g);
    agent->rx = .5f;
    agent->ry = .5f;
    g->options.center_agent = g->options.distribution_mode == MemoryMode;
    g->grid_step = true;
    float diamond_pct = 12 / 400.0f;
    float boulder_pct = 80 / 400.0f;
    float mud_pct = 12 / 400.0f;
    int num_diamonds = (int)(diamond_pct * g->grid_size);
    int num_boulders = (int)(boulder_pct * g->grid_size);
    int num_mud = (int)(mud_pct * g->grid_size);
    /* RandGen::simple_choose(main_area, k) (randgen.cpp:70-88): rejection against a std::set */
    int k = num_diamonds + num_boulders + num_mud + 1;
    static int obj_idxs[MAX_GRID];
    static bool taken[MAX_GRID];
    fassert(k <= g->main_area && g->main_area <= MAX_GRID);
    memset(taken, 0, sizeof(taken));
    for (int i = 0; i < k; i++) {
        int next = rg_randn(r, g->main_area);
        while (taken[next]) next = rg_randn(r, g->main_area);
        obj_idxs[i] = next;
        taken[next] = true;
    }
    int agent_x = obj_idxs[0] % g->main_width;
    int agent_y = obj_idxs[0] / g->main_width;
    agent->x = (float)(agent_x + .5);
    agent->y = (float)(agent_y + .5);
    for (int i = 0; i < g->main_area; ++i) set_obj_idx(g, i, MN_DIRT);
    for (int i = 0; i < num_diamonds; ++i) set_obj_idx(g, obj_idxs[i + 1], MN_DIAMOND);
    for (int i = 0; i < num_boulders; ++i) set_obj_idx(g, obj_idxs[i + 1 + num_diamonds], MN_BOULDER);
    for (int i = 0; i < num_mud; ++i) set_obj_idx(g, obj_idxs[i + 1 + num_diamonds + num_boulders], MN_MUD);
    static int dirt_cells[MAX_GRID]; /* get_cells_with_type(DIRT) (:203-213): ascending */
    int nd = 0;
    for (int i = 0; i < g->grid_size; i++)
        if (g->grid[i] == MN_DIRT) dirt_cells[nd++] = i;
    set_obj(g, (int)agent->x, (int)agent->y, SPACE);
    for (int i = -1; i <= 1; ++i) {
        for (int j = -1; j <= 1; ++j) {
            int ox = agent_x + i, oy = agent_y + j;
            if (get_obj(g, ox, oy) == MN_BOULDER) set_obj(g, ox, oy, MN_DIRT);
        }
    }
    static int exit_candidates[MAX_GRID];
    int ne = 0;
    for (int c = 0; c < nd; c++) {
        int cell = dirt_cells[c];
        int above_obj = get_obj_idx(g, cell + g->main_width);
        if (above_obj == MN_DIRT || above_obj == g->out_of_bounds_object) exit_candidates[ne++] = cell;
    }
    fassert(ne > 0);
    int exit_cell = exit_candidates[rg_randn(r, ne)];
    set_obj_idx(g, exit_cell, SPACE);
    int e = add_entity(g, (float)((exit_cell % g->main_width) + .5), (float)((exit_cell / g->main_width) + .5), 0, 0,
                       .5f, MN_EXIT);
    g->ents[e].render_z = -1;
}

static void mn_move_cell(Game *g, int x, int y, bool *has_moved) { /* :310-346 */
    int w = g->main_width;
    int idx = x + w * y;
    bool current_moved = has_moved[idx];
    int obj = get_obj_idx(g, idx);
    int obj_x = idx % w;
    int stat_type = mn_stationary_type(obj);
    int agent_idx = mn_agent_index(g);
    /* `BOULDER || DIAMOND && !moved`: && binds tighter */
    if (stat_type == MN_BOULDER || (stat_type == MN_DIAMOND && !current_moved)) {
        int below_idx = idx - w;
        int below_object = get_obj_idx(g, below_idx);
        bool agent_is_below = agent_idx == below_idx;
        if (below_object == SPACE && !agent_is_below) {
            set_obj_idx(g, idx, SPACE);
            int two_below_obj = get_obj_idx(g, below_idx - w);
            int obj_type = two_below_obj == SPACE ? mn_moving_type(obj) : stat_type;
            set_obj_idx(g, below_idx, obj_type);
            has_moved[below_idx] = true;
        } else if (agent_is_below && mn_is_moving(obj)) {
            g->died = true;
            /* entities.erase(entities.begin()): entities[0] is the agent */
            fassert(!g->agent_erased && g->num_ents > 0);
            g->agent_ghost = g->ents[0];
            g->agent_erased = true;
            memmove(&g->ents[0], &g->ents[1], sizeof(Entity) * (size_t)(g->num_ents - 1));
            g->num_ents--;
            set_obj_idx(g, below_idx, MN_DEAD_PLAYER);
        } else if (mn_is_round(below_object) && obj_x > 0 && mn_is_free(g, idx - 1) && mn_is_free(g, idx - w - 1)) {
            set_obj_idx(g, idx, SPACE);
            set_obj_idx(g, idx - 1, stat_type);
            has_moved[idx - 1] = true;
        } else if (mn_is_round(below_object) && obj_x < w - 1 && mn_is_free(g, idx + 1) && mn_is_free(g, idx - w + 1)) {
            set_obj_idx(g, idx, SPACE);
            set_obj_idx(g, idx + 1, stat_type);
            has_moved[idx + 1] = true;
        } else {
            set_obj_idx(g, idx, stat_type);
        }
    }
}

static void miner_game_step(Game *g) { /* :250-308 */
    static bool has_moved[MAX_GRID];
    memset(has_moved, 0, sizeof(has_moved));
    int w = g->main_width, h = g->main_height;
    for (int y = 0; (float)y <= AG(g)->y; ++y)
        for (int x = 0; x < w; ++x) mn_move_cell(g, x, y, has_moved);
    basic_game_step(g);
    if (g->died) {
        g->sd_done = true;
        return;
    }
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = false;
    if (g->action_vx < 0) agent->is_reflected = true;
    /* handle_push (:262-281) */
    int agent_idx = mn_agent_index(g);
    int agentx = agent_idx % w;
    if (g->action_vx == 1 && (agent->vx == 0) && (agentx < w - 2) && get_obj_idx(g, agent_idx + 1) == MN_BOULDER &&
        get_obj_idx(g, agent_idx + 2) == SPACE) {
        set_obj_idx(g, agent_idx + 1, SPACE);
        set_obj_idx(g, agent_idx + 2, MN_BOULDER);
        has_moved[agent_idx + 2] = true;
        agent->x += 1;
    } else if (g->action_vx == -1 && (agent->vx == 0) && (agentx > 1) && get_obj_idx(g, agent_idx - 1) == MN_BOULDER &&
               get_obj_idx(g, agent_idx - 2) == SPACE) {
        set_obj_idx(g, agent_idx - 1, SPACE);
        set_obj_idx(g, agent_idx - 2, MN_BOULDER);
        has_moved[agent_idx - 2] = true;
        agent->x -= 1;
    }
    int agent_obj = mn_stationary_type(get_obj(g, (int)agent->x, (int)agent->y));
    if (agent_obj == MN_DIAMOND) g->sd_reward += MN_DIAMOND_REWARD;
    if (agent_obj == MN_DIRT || agent_obj == MN_MUD || agent_obj == MN_DIAMOND) set_obj(g, (int)agent->x, (int)agent->y, SPACE);
    for (int y = (int)(AG(g)->y + 1); y < h; ++y)
        for (int x = 0; x < w; ++x) mn_move_cell(g, x, y, has_moved);
    int diamonds = 0; /* count_diamonds (:348-356) */
    for (int idx = 0; idx < g->main_area; ++idx)
        if (mn_stationary_type(get_obj_idx(g, idx)) == MN_DIAMOND) ++diamonds;
    g->diamonds_remaining = diamonds;
}

/* ================================================================== climber (games/climber.cpp) */
#define CL_COIN 1
#define CL_ENEMY 5
#define CL_ENEMY1 6
#define CL_ENEMY2 7
#define CL_PLAYER_JUMP 9
#define CL_PLAYER_RIGHT1 12
#define CL_PLAYER_RIGHT2 13
#define CL_WALL_MID 15
#define CL_WALL_TOP 16
#define CL_ENEMY_BARRIER 19
static const float CL_PATROL_RANGE = 4;
static bool cl_is_wall(int t) { return t == CL_WALL_MID || t == CL_WALL_TOP; } /* :139-141 */

static void climber_choose_world_dim(Game *g) { /* :263-266 */
    g->main_width = g->options.distribution_mode == EasyMode ? 16 : 20;
    g->main_height = 64;
}

static int cl_choose_delta_y(Game *g) { /* :171-176 */
    int max_dy = (int)(g->max_jump * g->max_jump / (2 * g->gravity));
    int min_dy = 3;
    return rg_randn(&g->rand_gen, max_dy - min_dy + 1) + min_dy;
}

static void cl_generate_platforms(Game *g, const or_atlas *at) { /* :178-232 */
    MT *r = &g->rand_gen;
    int difficulty = rg_randn(r, 3);
    int min_platforms = difficulty * difficulty + 1;
    int max_platforms = (difficulty + 1) * (difficulty + 1) + 1;
    int num_platforms = rg_randn(r, max_platforms - min_platforms + 1) + min_platforms;
    g->coin_quota = 0;
    g->coins_collected = 0;
    int curr_x = rg_randn(r, g->main_width - 4) + 2;
    int curr_y = 0;
    int margin_x = 3;
    float enemy_prob = g->options.distribution_mode == EasyMode ? .2f : .5f;
    for (int i = 0; i < num_platforms; i++) {
        int delta_y = cl_choose_delta_y(g);
        bool can_spawn_enemy = (curr_x >= margin_x) && (curr_x <= g->main_width - margin_x);
        if (can_spawn_enemy && ((double)rg_rand01(r) < (double)enemy_prob)) {
            /* add_entity(curr_x + .5, curr_y + randn(2) + 2 + .5, .15 * (randn(2) * 2 - 1), ...): g++
             * evaluates the arguments right to left, so the vx draw comes first (pinned by
             * oracle/ref_harness.cpp ref_climber_enemy_args) */
            int vdraw = rg_randn(r, 2);
            int ydraw = rg_randn(r, 2);
            int e = add_entity(g, (float)(curr_x + .5), (float)(curr_y + ydraw + 2 + .5), (float)(.15 * (vdraw * 2 - 1)), 0,
                               .5f, CL_ENEMY);
            Entity *ent = &g->ents[e];
            ent->image_type = CL_ENEMY1;
            ent->smart_step = true;
            ent->climber_spawn_x = (float)(curr_x + .5);
            match_aspect_ratio(g, at, ent);
        }
        curr_y += delta_y;
        int plat_len = 2 + rg_randn(r, 10);
        int vx = rg_randn(r, 2) * 2 - 1;
        if (curr_x < margin_x) vx = 1;
        if (curr_x > g->main_width - margin_x) vx = -1;
        int candidates[16], nc = 0;
        for (int j = 0; j < plat_len; j++) {
            int nx = curr_x + (j + 1) * vx;
            if (nx <= 0 || nx >= g->main_width - 1) break;
            candidates[nc++] = nx;
            set_obj(g, nx, curr_y, CL_WALL_TOP);
        }
        fassert(nc > 0);
        if ((double)rg_rand01(r) < .5 || i == num_platforms - 1) {
            int coin_x = candidates[rg_randn(r, nc)];
            add_entity(g, (float)(coin_x + .5), (float)(curr_y + 1.5), 0, 0, 0.3f, CL_COIN);
            g->coin_quota += 1;
        }
        curr_x = candidates[rg_randn(r, nc)];
    }
}

static void climber_game_reset(Game *g, const or_atlas *at) { /* :268-288 */
    climber_choose_world_dim(g);
    basic_game_reset(g, at);
    g->gravity = 0.2f;
    g->max_jump = 1.5f;
    g->air_control = 0.15f;
    g->maxspeed = .5f;
    g->has_support = false;
    g->facing_right = true;
    Entity *agent = AG(g);
    agent->rx = .5f;
    agent->ry = .5f;
    agent->x = 1 + agent->rx;
    agent->y = 1 + agent->ry;
    choose_random_theme(g, agent, at);
    g->wall_theme = rg_randn(&g->rand_gen, 4); /* NUM_WALL_THEMES */
    /* init_floor_and_walls (:164-169) */
    fill_elem(g, 0, 0, g->main_width, 1, CL_WALL_TOP);
    fill_elem(g, 0, 0, 1, g->main_height, CL_WALL_MID);
    fill_elem(g, g->main_width - 1, 0, 1, g->main_height, CL_WALL_MID);
    fill_elem(g, 0, g->main_height - 1, g->main_width, 1, CL_WALL_MID);
    cl_generate_platforms(g, at);
}

static void climber_game_step(Game *g) { /* :320-346 */
    basic_game_step(g);
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = false;
    if (g->action_vx < 0) agent->is_reflected = true;
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *ent = &g->ents[i];
        if (ent->type == CL_ENEMY) {
            if (ent->x > ent->climber_spawn_x + CL_PATROL_RANGE) ent->vx = -1 * fabsf(ent->vx);
            else if (ent->x < ent->climber_spawn_x - CL_PATROL_RANGE) ent->vx = fabsf(ent->vx);
            ent->image_type = g->cur_time / 5 % 2 == 0 ? CL_ENEMY1 : CL_ENEMY2;
            ent->is_reflected = ent->vx < 0;
        }
    }
    if (g->coin_quota == g->coins_collected) {
        g->sd_done = true;
        g->sd_reward += 10.0f; /* COMPLETION_BONUS */
        g->sd_level_complete = true;
    }
}

/* ================================================================== chaser (games/chaser.cpp) */
static const float CH_ORB_REWARD = 0.04f;
static const float CH_COMPLETION_BONUS = 10.0f;
static const float CH_ORB_DIM = 0.3f;
#define CH_LARGE_ORB 2
#define CH_ENEMY_WEAK 3
#define CH_ENEMY_EGG 4
#define CH_MAZE_WALL 5
#define CH_ENEMY 6
#define CH_MARKER 1001
#define CH_ORB 1002

static double cu_sign(double x) { return x > 0 ? 1 : (x == 0 ? 0 : -1); } /* cpp-utils.h:43-45 */

/* RandGen::simple_choose (randgen.cpp:70-88): rejection against a std::set */
static void rg_simple_choose(MT *r, int n, int k, int *out) {
    fassert(k <= n);
    for (int i = 0; i < k; i++) {
        int next = rg_randn(r, n);
        for (;;) {
            bool seen = false;
            for (int j = 0; j < i; j++)
                if (out[j] == next) seen = true;
            if (!seen) break;
            next = rg_randn(r, n);
        }
        out[i] = next;
    }
}

static bool ch_can_eat_enemies(Game *g) { return g->cur_time - g->eat_time < g->eat_timeout; } /* :255-257 */

static int ch_to_grid_idx(Game *g, int x, int y) { /* basic-abstract-game.cpp:187-192 */
    if (!grid_contains(g, x, y)) return -2; /* INVALID_IDX */
    return y * g->main_width + x;
}

static void ch_spawn_egg(Game *g, int enemy_cell) { /* :259-262 */
    int e = add_entity(g, (float)((enemy_cell % g->maze_dim) + .5), (float)((enemy_cell / g->maze_dim) + .5), 0, 0, .5f,
                       CH_ENEMY_EGG);
    g->ents[e].health = (float)g->egg_timeout;
}

static void chaser_game_reset(Game *g, const or_atlas *at) { /* :147-252 */
    MT *r = &g->rand_gen;
    int extra_orb_sign = 1;
    if (g->options.distribution_mode == EasyMode) {
        g->maze_dim = 11; g->total_enemies = 3; extra_orb_sign = 0;
    } else if (g->options.distribution_mode == HardMode) {
        g->maze_dim = 13; g->total_enemies = 3; extra_orb_sign = -1;
    } else if (g->options.distribution_mode == ExtremeMode) {
        g->maze_dim = 19; g->total_enemies = 5; extra_orb_sign = 1;
    } else {
        fatal_msg("chaser: bad distribution mode");
    }
    g->main_width = g->maze_dim; /* choose_world_dim (:141-144) */
    g->main_height = g->maze_dim;
    basic_game_reset(g, at);
    g->options.center_agent = false;
    Entity *agent = AG(g);
    agent->rx = .5f;
    agent->ry = .5f;
    g->eat_time = -1 * g->eat_timeout;
    fill_elem(g, 0, 0, g->main_width, g->main_height, CH_MAZE_WALL);
    static MazeGen mg;
    mg_init(&mg, r, g->maze_dim);
    mg_generate_maze_no_dead_ends(&mg);
    const int md = g->maze_dim;
    static int quad[4][MAX_GRID];
    int qn[4] = {0, 0, 0, 0}, orbs_for_quadrant[4];
    int extra_quad = rg_randn(r, 4);
    for (int i = 0; i < 4; i++) orbs_for_quadrant[i] = 1 + (i == extra_quad ? extra_orb_sign : 0);
    for (int i = 0; i < md; i++) {
        for (int j = 0; j < md; j++) {
            int obj = mg_gridget(&mg, i + MAZE_OFFSET, j + MAZE_OFFSET);
            set_obj(g, i, j, obj == WALL_OBJ ? CH_MAZE_WALL : obj);
            if (obj == SPACE) {
                int idx = j * md + i;
                int quad_idx = (i >= md / 2.0 ? 1 : 0) * 2 + (j >= md / 2.0 ? 1 : 0);
                quad[quad_idx][qn[quad_idx]++] = idx;
            }
        }
    }
    for (int i = 0; i < 4; i++) {
        int sel[8];
        fassert(orbs_for_quadrant[i] <= 8);
        rg_simple_choose(r, qn[i], orbs_for_quadrant[i], sel);
        for (int j = 0; j < orbs_for_quadrant[i]; j++) {
            int cell = quad[i][sel[j]];
            add_entity(g, (float)((cell % g->main_width) + .5), (float)((cell / g->main_width) + .5), 0, 0, 0.4f,
                       CH_LARGE_ORB); /* spawn_entity_at_idx (:587-594) */
            set_obj_idx(g, cell, CH_MARKER);
        }
    }
    static int free_cells[MAX_GRID];
    int nfree = 0;
    for (int i = 0; i < g->grid_size; i++)
        if (g->grid[i] == SPACE) free_cells[nfree++] = i; /* get_cells_with_type (:205-215) */
    int sel[8];
    fassert(1 + g->total_enemies <= 8);
    rg_simple_choose(r, nfree, 1 + g->total_enemies, sel);
    int start = free_cells[sel[0]];
    agent->x = (float)((start % md) + .5);
    agent->y = (float)((start / md) + .5);
    for (int i = 0; i < g->total_enemies; i++) {
        int cell = free_cells[sel[i + 1]];
        set_obj_idx(g, cell, CH_MARKER);
        ch_spawn_egg(g, cell);
    }
    for (int k = 0; k < nfree; k++) set_obj_idx(g, free_cells[k], CH_ORB);
    g->total_orbs = nfree;
    g->orbs_collected = 0;
    for (int i = 0; i < g->grid_size; i++)
        if (g->grid[i] == CH_MARKER) g->grid[i] = SPACE;
    g->num_free = 0;
    for (int i = 0; i < g->grid_size; i++) {
        bool is_space = g->grid[i] != CH_MAZE_WALL;
        if (is_space) g->free_list[g->num_free++] = i;
        g->is_space[i] = is_space;
    }
}

static void chaser_game_step(Game *g) { /* :286-376 */
    basic_game_step(g);
    int num_enemies = 0;
    float default_enemy_speed = .5;
    float vscale = ch_can_eat_enemies(g) ? (default_enemy_speed * .5f) : default_enemy_speed;
    Entity *agent = AG(g);
    for (int j = g->num_ents - 1; j >= 0; j--) {
        Entity *ent = &g->ents[j];
        if (ent->type == CH_ENEMY_EGG) {
            num_enemies++;
            ent->health -= 1;
            if (ent->health == 0) {
                ent->will_erase = true;
                fassert(g->num_ents < MAX_ENTS); /* spawn_child (:233-239) */
                Entity child;
                entity_init(&child, ent->x, ent->y, 0, 0, .5f, .5f, CH_ENEMY);
                child.smart_step = true;
                g->ents[g->num_ents++] = child;
                ent = &g->ents[j];
                agent = AG(g);
            }
        } else if (ent->type == CH_ENEMY) {
            num_enemies++;
            float x = (float)(ent->x - .5);
            float y = (float)(ent->y - .5);
            int dist_scale = ch_can_eat_enemies(g) ? -1 : 1;
            int enemy_idx = ch_to_grid_idx(g, (int)x, (int)y);
            int agent_idx = ch_to_grid_idx(g, (int)agent->x, (int)agent->y);
            bool is_at_junction = fabs(x - round(x)) + fabs(y - round(y)) < .01;
            bool be_agressive = g->step_rand_int % 2 == 0;
            if ((ent->vx == 0 && ent->vy == 0) || is_at_junction) {
                int adj[4], nadj = 0, sn[4], nsn = 0;
                int prev_idx = ch_to_grid_idx(g, (int)(x - cu_sign(ent->vx)), (int)(y - cu_sign(ent->vy)));
                int ex = enemy_idx % g->main_width, ey = enemy_idx / g->main_width; /* get_adjacent (:269-284) */
                for (int i = -1; i <= 1; i++)
                    for (int jj = -1; jj <= 1; jj++) {
                        if (i == 0 && jj == 0) continue;
                        if (i != 0 && jj != 0) continue;
                        int nb = ch_to_grid_idx(g, ex + i, ey + jj);
                        if (nb != -2) adj[nadj++] = nb;
                    }
                int min_dist = 2 * g->main_width;
                for (int k = 0; k < nadj; k++) {
                    int a = adj[k];
                    if (g->is_space[a] && a != prev_idx) {
                        int md = (abs((a % g->main_width) - (agent_idx % g->main_width)) +
                                  abs((a / g->main_width) - (agent_idx / g->main_width))) * dist_scale;
                        if (be_agressive) {
                            if (md < min_dist) {
                                min_dist = md;
                                nsn = 0;
                                sn[nsn++] = a;
                            } else if (md == min_dist) {
                                sn[nsn++] = a;
                            }
                        } else {
                            sn[nsn++] = a;
                        }
                    }
                }
                fassert(nsn > 0);
                int neighbor = sn[(unsigned long)g->step_rand_int % (unsigned long)nsn];
                int nx = neighbor % g->main_width;
                int ny = neighbor / g->main_width;
                ent->vx = (nx - x) * vscale;
                ent->vy = (ny - y) * vscale;
            }
        }
    }
    if (num_enemies < g->total_enemies) {
        int selected_idx = (int)((unsigned long)g->step_rand_int % (unsigned long)g->num_free);
        ch_spawn_egg(g, g->free_list[selected_idx]);
    }
    agent = AG(g);
    int agent_idx = (int)agent->y * g->main_width + (int)agent->x; /* get_agent_index (:176-178) */
    if (get_obj_idx(g, agent_idx) == CH_ORB) {
        set_obj_idx(g, agent_idx, SPACE);
        g->sd_reward += CH_ORB_REWARD;
        g->orbs_collected += 1;
    }
    if (g->orbs_collected == g->total_orbs) {
        g->sd_reward += CH_COMPLETION_BONUS;
        g->sd_level_complete = true;
        g->sd_done = true;
    }
}

/* ================================================================== fruitbot (games/fruitbot.cpp) */
#define FB_BARRIER 1
#define FB_OUT_OF_BOUNDS_WALL 2
#define FB_PLAYER_BULLET 3
#define FB_BAD_OBJ 4
#define FB_GOOD_OBJ 7
#define FB_LOCKED_DOOR 10
#define FB_LOCK 11
#define FB_PRESENT 12
#define FB_KEY_DURATION 8
static const float FB_DOOR_ASPECT_RATIO = 3.25f;

static void fit_aspect_ratio(Game *g, const or_atlas *at, Entity *e) { /* basic-abstract-game.cpp:1034-1045 */
    float ar = asset_aspect_ratio(g, at, e->image_type + e->image_theme * MAX_ASSETS);
    if (ar > 1) e->ry = e->rx / ar;
    else e->rx = e->ry * ar;
}

static void fb_add_walls(Game *g, float ry, bool use_door, float min_pct) { /* :157-189 */
    MT *r = &g->rand_gen;
    float rw = (float)g->main_width;
    float wall_ry = 0.3f;
    float lock_rx = .25;
    float lock_ry = 0.45f;
    float pct = (float)(min_pct + .2 * rg_rand01(r));
    if (use_door) {
        pct += 0.1f;
        float lock_pct_w = 2 * lock_rx / g->main_width;
        float door_pct_w = (wall_ry * 2 * FB_DOOR_ASPECT_RATIO) / g->main_width;
        int num_doors = (int)ceilf((pct - 2 * lock_pct_w) / door_pct_w);
        pct = 2 * lock_pct_w + door_pct_w * num_doors;
    }
    float gapw = pct * rw;
    float w1 = rg_rand01(r) * (rw - gapw);
    float w2 = rw - w1 - gapw;
    add_entity_rxy(g, w1 / 2, ry, 0, 0, w1 / 2, wall_ry, FB_BARRIER);
    add_entity_rxy(g, rw - w2 / 2, ry, 0, 0, w2 / 2, wall_ry, FB_BARRIER);
    if (use_door) {
        int is_on_right = rg_randn(r, 2);
        float lock_x = w1 + lock_rx + is_on_right * (gapw - 2 * lock_rx);
        float door_x = w1 + gapw / 2 - (is_on_right * 2 - 1) * lock_rx;
        add_entity_rxy(g, door_x, ry, 0, 0, gapw / 2 - lock_rx, wall_ry, FB_LOCKED_DOOR);
        add_entity_rxy(g, lock_x, ry - lock_ry + wall_ry, 0, 0, lock_rx, lock_ry, FB_LOCK);
    }
}

static void fruitbot_game_reset(Game *g, const or_atlas *at) { /* :191-245 */
    MT *r = &g->rand_gen;
    g->main_width = g->options.distribution_mode == EasyMode ? 10 : 20; /* choose_world_dim (:144-152) */
    g->main_height = 60;
    basic_game_reset(g, at);
    g->last_fire_time = 0;
    int min_sep = 4, num_walls = 10, object_group_size = 6, buf_h = 4;
    float door_prob = .125;
    float min_pct = .1f;
    if (g->options.distribution_mode == EasyMode) {
        num_walls = 5; object_group_size = 2; door_prob = 0; min_pct = .2f;
    }
    int partition[16] = {0};
    fassert(num_walls <= 16);
    int px = g->main_height - min_sep * num_walls - buf_h; /* RandGen::partition (randgen.cpp:33-41) */
    for (int i = 0; i < px; i++) partition[rg_randn(r, num_walls)] += 1;
    int curr_h = 0;
    for (int k = 0; k < num_walls; k++) {
        int dy = min_sep + partition[k];
        curr_h += dy;
        bool use_door = (dy > 5) && rg_rand01(r) < door_prob;
        fb_add_walls(g, (float)curr_h, use_door, min_pct);
    }
    Entity *agent = AG(g);
    agent->y = agent->ry;
    int num_good = rg_randn(r, 10) + 10;
    int num_bad = rg_randn(r, 10) + 10;
    for (int i = 0; i < g->main_width; i++) {
        int e = add_entity_rxy(g, (float)(i + .5), (float)(g->main_height - .5), 0, 0, .5f, .5f, FB_PRESENT);
        choose_random_theme(g, &g->ents[e], at);
    }
    for (int i = 0; i < num_good; i++) spawn_entity(g, .5f, FB_GOOD_OBJ, 0, 0, (float)g->main_width, (float)g->main_height);
    for (int i = 0; i < num_bad; i++) spawn_entity(g, .5f, FB_BAD_OBJ, 0, 0, (float)g->main_width, (float)g->main_height);
    for (int i = 0; i < g->num_ents; i++) {
        Entity *e = &g->ents[i];
        if (e->type == FB_GOOD_OBJ || e->type == FB_BAD_OBJ) {
            e->image_theme = rg_randn(r, object_group_size);
            fit_aspect_ratio(g, at, e);
        }
    }
    AG(g)->rotation = -1 * PI_F / 2;
}

static void fruitbot_game_step(Game *g) { /* :247-258 */
    basic_game_step(g);
    if (g->special_action == 1 && (g->cur_time - g->last_fire_time) >= FB_KEY_DURATION) {
        float vx = 0, vy = 1;
        Entity *agent = AG(g);
        float bullet_vscale = .5;
        int e = add_entity(g, agent->x, agent->y, vx * bullet_vscale, vy * bullet_vscale, .25f, FB_PLAYER_BULLET);
        g->ents[e].expire_time = FB_KEY_DURATION;
        g->ents[e].collides_with_entities = true;
        g->last_fire_time = g->cur_time;
    }
}

/* ================================================================== dodgeball (games/dodgeball.cpp) */
#define DB_LAVA_WALL 1
#define DB_PLAYER_BALL 3
#define DB_ENEMY 4
#define DB_DOOR 5
#define DB_ENEMY_BALL 6
#define DB_DUST_CLOUD 8
static const float DB_ENEMY_VEL = 0.05f;

static void entity_face_direction(Entity *e, float dx, float dy) { /* entity.cpp:84-88, rotation_offset 0 */
    if (dx != 0 || dy != 0) e->rotation = -1 * atan2f(dy, dx) + 0.0f;
}

typedef struct { float x, y, w, h; } DbRoom; /* QRectF of float-valued corners */

static void db_add_room(Game *g, DbRoom *rooms, int *n, DbRoom room) { /* :157-164 */
    float rw = room.w, rh = room.h;
    if ((rw >= g->db_min_dim || rh >= g->db_min_dim) && (rw >= g->db_hard_min_dim) && (rh >= g->db_hard_min_dim)) {
        fassert(*n < 64);
        rooms[(*n)++] = room;
    }
}

static void db_split_room(Game *g, DbRoom *rooms, int *n, DbRoom room, float thickness) { /* :166-224 */
    MT *r = &g->rand_gen;
    bool will_split_width = rg_rand01(r) < .5;
    bool choice2 = rg_rand01(r) < .5;
    if (room.w < g->db_min_dim) will_split_width = false;
    if (room.h < g->db_min_dim) will_split_width = true;
    float rx = room.x, ry = room.y, rw = room.w, rh = room.h;
    float gap = (float)(.25 * (rg_randn(r, 3) + 1));
    float pct = 1 - gap;
    if (!will_split_width) {
        float wy, wh, remy;
        if (choice2) {
            wy = ry;
            remy = ry + pct * rh;
            wh = pct * rh;
        } else {
            wy = ry + (1 - pct) * rh;
            remy = ry;
            wh = pct * rh;
        }
        add_entity_rxy(g, rx + rw / 2, wy + wh / 2, 0, 0, thickness, wh / 2, DB_LAVA_WALL);
        float nextw = rw / 2 - thickness;
        db_add_room(g, rooms, n, (DbRoom){rx, wy, nextw, wh});
        db_add_room(g, rooms, n, (DbRoom){rx + rw / 2 + thickness, wy, nextw, wh});
        db_add_room(g, rooms, n, (DbRoom){rx, remy, rw, rh - wh});
    } else {
        float wx, ww, remx;
        if (choice2) {
            wx = rx;
            remx = rx + pct * rw;
            ww = pct * rw;
        } else {
            wx = rx + (1 - pct) * rw;
            remx = rx;
            ww = pct * rw;
        }
        add_entity_rxy(g, wx + ww / 2, ry + rh / 2, 0, 0, ww / 2, thickness, DB_LAVA_WALL);
        float nexth = rh / 2 - thickness;
        db_add_room(g, rooms, n, (DbRoom){wx, ry, ww, nexth});
        db_add_room(g, rooms, n, (DbRoom){wx, ry + rh / 2 + thickness, ww, nexth});
        db_add_room(g, rooms, n, (DbRoom){remx, ry, rw - ww, rh});
    }
}

static void db_choose_vel(Game *g, Entity *e) { /* :226-238 */
    MT *r = &g->rand_gen;
    float vel = DB_ENEMY_VEL * (rg_randn(r, 2) * 2 - 1);
    if (rg_randn(r, 2) == 0) {
        e->vx = vel;
        e->vy = 0;
    } else {
        e->vy = vel;
        e->vx = 0;
    }
    e->spawn_time = rg_randn(r, 50) + 25;
}

static int spawn_entity_rxy(Game *g, float rx, float ry, int type, float x, float y, float w, float h) { /* :520-527 */
    Entity e;
    entity_init(&e, 0, 0, 0, 0, rx, ry, type);
    reposition(g, &e, x, y, w, h, true);
    fassert(g->num_ents < MAX_ENTS);
    g->ents[g->num_ents] = e;
    return g->num_ents++;
}

static bool agent_has_collision(Game *g) { /* :529-538 */
    for (int i = 0; i < g->num_ents; i++)
        if (has_agent_collision(g, &g->ents[i])) return true;
    return false;
}

static void reposition_agent(Game *g) { /* :540-546 */
    Entity *agent = AG(g);
    int count = 0;
    do {
        agent->x = rg_rand01(&g->rand_gen) * (g->main_width - 2 * agent->rx) + agent->rx;
        agent->y = rg_rand01(&g->rand_gen) * (g->main_height - 2 * agent->ry) + agent->ry;
        count++;
    } while (agent_has_collision(g) && (count < 100));
}

static void dodgeball_game_reset(Game *g, const or_atlas *at) { /* :259-369 */
    MT *r = &g->rand_gen;
    int world_dim = g->options.distribution_mode == MemoryMode ? 40 : 20; /* choose_world_dim (:248-257) */
    g->main_width = world_dim;
    g->main_height = world_dim;
    basic_game_reset(g, at);
    g->options.center_agent = g->options.distribution_mode == MemoryMode;
    g->last_fire_time = 0;
    DbRoom rooms[64];
    int nrooms = 0;
    rooms[nrooms++] = (DbRoom){0, 0, (float)g->main_width, (float)g->main_height};
    int dm = g->options.distribution_mode;
    float thickness = 0.3f, enemy_r = .5, exit_r = .75;
    g->db_ball_r = .25;
    g->db_ball_vscale = .25;
    int num_iterations = 0, max_extra_enemies = 3;
    Entity *agent = AG(g);
    if (dm == EasyMode) {
        num_iterations = 2;
        thickness *= 2; enemy_r *= 2; g->db_ball_r *= 2; g->db_ball_vscale *= 2;
        g->maxspeed = .75;
        agent->rx = 1; agent->ry = 1;
        exit_r *= 2;
    } else if (dm == HardMode) {
        num_iterations = 4;
        thickness *= 1.5; enemy_r *= 1.5; g->db_ball_r *= 1.5; g->db_ball_vscale *= 1.5;
        g->maxspeed = .5;
        agent->rx = .75; agent->ry = .75;
    } else if (dm == ExtremeMode) {
        num_iterations = 8;
        g->maxspeed = .25;
    } else if (dm == MemoryMode) {
        num_iterations = 16;
        thickness *= 1.5; enemy_r *= 1.5; g->db_ball_r *= 1.5; g->db_ball_vscale *= 1.5;
        g->maxspeed = .5;
        agent->rx = .75; agent->ry = .75;
        max_extra_enemies = 16;
    } else {
        fatal_msg("dodgeball: bad distribution mode");
    }
    g->db_hard_min_dim = 4 * agent->rx + 2 * thickness + .5;
    g->db_min_dim = agent->rx * 8 + .5;
    for (int it = 0; it < num_iterations; it++) {
        if (nrooms == 0) break;
        int idx = rg_randn(r, nrooms);
        DbRoom room = rooms[idx];
        memmove(&rooms[idx], &rooms[idx + 1], sizeof(DbRoom) * (size_t)(nrooms - idx - 1));
        nrooms--;
        db_split_room(g, rooms, &nrooms, room, thickness);
    }
    float border_r = 0;
    float doorlen = 2 * exit_r;
    int exit_wall_choice = rg_randn(r, 4);
    float mw = (float)g->main_width, mh = (float)g->main_height;
    if (exit_wall_choice == 0)
        spawn_entity_rxy(g, doorlen / 2, exit_r, DB_DOOR, 2 * border_r, 2 * border_r, mw - 4 * border_r, 2 * exit_r);
    else if (exit_wall_choice == 1)
        spawn_entity_rxy(g, doorlen / 2, exit_r, DB_DOOR, 2 * border_r, mh - 2 * border_r - 2 * exit_r, mw - 4 * border_r,
                         2 * exit_r);
    else if (exit_wall_choice == 2)
        spawn_entity_rxy(g, exit_r, doorlen / 2, DB_DOOR, 2 * border_r, 2 * border_r, 2 * exit_r, mh - 4 * border_r);
    else
        spawn_entity_rxy(g, exit_r, doorlen / 2, DB_DOOR, mw - 2 * border_r - 2 * exit_r, 2 * border_r, 2 * exit_r,
                         mh - 4 * border_r);
    reposition_agent(g);
    g->db_num_enemies = rg_randn(r, max_extra_enemies + 1) + 3;
    for (int i = 0; i < g->db_num_enemies; i++) spawn_entity(g, enemy_r, DB_ENEMY, 0, 0, mw, mh);
    int enemy_theme = rg_randn(r, 7); /* NUM_ENEMY_THEMES */
    for (int i = 0; i < g->num_ents; i++) {
        Entity *e = &g->ents[i];
        if (e->type == DB_ENEMY) {
            e->image_theme = enemy_theme;
            e->health = 1;
            e->spawn_time = 0;
            e->fire_time = 10;
            e->collides_with_entities = true;
            e->smart_step = true;
            db_choose_vel(g, e);
            entity_face_direction(e, e->vx, e->vy);
        } else if (e->type == DB_LAVA_WALL) {
            e->collides_with_entities = true;
        }
    }
    entity_face_direction(AG(g), 1, 0);
}

static void db_fire_ball(Game *g, int ei, float vx, float vy) { /* :371-376 */
    Entity *ent = &g->ents[ei];
    float ex = ent->x, ey = ent->y;
    int b = add_entity(g, ex, ey, vx * g->db_ball_vscale, vy * g->db_ball_vscale, g->db_ball_r, DB_ENEMY_BALL);
    g->ents[ei].fire_time = g->cur_time + rg_randn(&g->rand_gen, 4);
    g->ents[b].vrot = PI_F * 0.23f; /* BALL_V_ROT */
    g->ents[b].expire_time = 50;
}

static void dodgeball_game_step(Game *g) { /* :378-444 */
    basic_game_step(g);
    float vx = (float)(g->last_move_action / 3 - 1);
    float vy = (float)(g->last_move_action % 3 - 1);
    entity_face_direction(AG(g), vx, vy);
    if (g->special_action == 1 && (g->cur_time - g->last_fire_time) >= 7) {
        Entity *agent = AG(g);
        int b = add_entity(g, agent->x, agent->y, vx * g->db_ball_vscale, vy * g->db_ball_vscale, g->db_ball_r,
                           DB_PLAYER_BALL);
        g->ents[b].collides_with_entities = true;
        g->ents[b].expire_time = 50;
        g->ents[b].vrot = PI_F * 0.23f;
        g->last_fire_time = g->cur_time;
    }
    g->db_num_enemies = 0;
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *ent = &g->ents[i];
        if (ent->type == DB_ENEMY) {
            g->db_num_enemies++;
            if (ent->spawn_time == 0) db_choose_vel(g, ent);
            else ent->spawn_time -= 1;
            bool can_fire = (g->cur_time - ent->fire_time) >= g->db_enemy_fire_delay;
            if (can_fire) {
                Entity *agent = AG(g);
                float dx = ent->x - agent->x;
                float dy = ent->y - agent->y;
                float bvelx = (float)(ent->x < agent->x ? 1 : -1);
                float bvely = (float)(ent->y < agent->y ? 1 : -1);
                if (fabs((double)dx) < 1) {
                    db_fire_ball(g, i, 0, bvely);
                    ent = &g->ents[i];
                    ent->vx = 0;
                    ent->vy = bvely * DB_ENEMY_VEL;
                } else if (fabs((double)dy) < 1) {
                    db_fire_ball(g, i, bvelx, 0);
                    ent = &g->ents[i];
                    ent->vx = bvelx * DB_ENEMY_VEL;
                    ent->vy = 0;
                }
            }
            entity_face_direction(ent, ent->vx, ent->vy);
        } else if (ent->type == DB_PLAYER_BALL || ent->type == DB_ENEMY_BALL) {
            if (ent->x < ent->rx || ent->x > (g->main_width - ent->rx)) ent->will_erase = true;
            else if (ent->y < ent->ry || ent->y > (g->main_height - ent->ry)) ent->will_erase = true;
        }
    }
    erase_if_needed(g);
}

/* ================================================================== plunder (games/plunder.cpp) */
#define PL_PLAYER_BULLET 1
#define PL_TARGET_LEGEND 2
#define PL_TARGET_BACKGROUND 3
#define PL_PANEL 6
#define PL_SHIP 7

static void rg_choose_n(MT *r, const int *elems, int count, int n, int *out) { /* randgen.cpp:49-68 */
    int rem[64];
    fassert(count <= 64);
    memcpy(rem, elems, sizeof(int) * (size_t)count);
    int nrem = count;
    if (n > count) {
        memcpy(out, rem, sizeof(int) * (size_t)count);
        return;
    }
    for (int k = 0; k < n; k++) {
        int idx = rg_randn(r, nrem);
        out[k] = rem[idx];
        memmove(&rem[idx], &rem[idx + 1], sizeof(int) * (size_t)(nrem - idx - 1));
        nrem--;
    }
}

static void plunder_game_reset(Game *g, const or_atlas *at) { /* :116-192 */
    MT *r = &g->rand_gen;
    basic_game_reset(g, at);
    Entity *agent = AG(g);
    agent->image_type = PL_SHIP;
    g->pl_juice_left = 1;
    g->pl_targets_hit = 0;
    g->pl_target_quota = 20;
    g->pl_spawn_prob = 0.06f;
    g->pl_r_scale = g->options.distribution_mode == EasyMode ? 1.5f : 1.0f;
    int num_total_ship_types = 6;
    g->pl_num_lanes = 5;
    int image_idxs[6];
    for (int i = 0; i < num_total_ship_types; i++) image_idxs[i] = i;
    rg_choose_n(r, image_idxs, num_total_ship_types, num_total_ship_types, g->pl_perm);
    g->pl_num_current_ship_types = 2;
    for (int i = 0; i < num_total_ship_types; i++) g->pl_target_bools[i] = false;
    for (int i = 0; i < g->pl_num_current_ship_types / 2; i++) g->pl_target_bools[g->pl_perm[i]] = true;
    for (int i = 0; i < g->pl_num_lanes; i++) {
        g->pl_lane_dirs[i] = rg_rand01(r) < .5;
        g->pl_lane_vels[i] = (float)(.15 + .1 * rg_rand01(r));
    }
    int num_panels = g->options.distribution_mode == EasyMode ? 0 : rg_randn(r, 4);
    float panel_width = 1.2f;
    for (int i = 0; i < num_panels; i++)
        spawn_entity_rxy(g, panel_width, .5, PL_PANEL, 0, (float)(.25 * g->main_height), (float)g->main_width,
                         (float)(.25 * g->main_height));
    float key_scale = 1.5;
    g->pl_legend_r = 2;
    add_entity(g, g->pl_legend_r, g->pl_legend_r, 0, 0, g->pl_legend_r, PL_TARGET_BACKGROUND);
    int e = add_entity(g, g->pl_legend_r, g->pl_legend_r, 0, 0, g->pl_r_scale * key_scale, PL_TARGET_LEGEND);
    g->ents[e].image_theme = g->pl_perm[0];
    g->ents[e].image_type = PL_SHIP;
    match_aspect_ratio(g, at, &g->ents[e]);
    g->ents[e].rotation = PI_F / 2;
    g->last_fire_time = 0;
    g->options.center_agent = false;
    agent = AG(g);
    agent->rx = g->pl_r_scale;
    agent->rotation = -1 * PI_F / 2;
    agent->image_theme = g->pl_perm[rg_randn(r, g->pl_num_current_ship_types / 2) + g->pl_num_current_ship_types / 2];
    match_aspect_ratio(g, at, agent);
    reposition_agent(g);
    agent->y = 1 + agent->ry;
    g->pl_min_agent_x = 2 * g->pl_legend_r + agent->rx;
    if (agent->x < g->pl_min_agent_x) agent->x = g->pl_min_agent_x;
}

static void plunder_game_step(Game *g, const or_atlas *at) { /* :194-241 */
    MT *r = &g->rand_gen;
    basic_game_step(g);
    g->pl_juice_left -= 0.0015f;
    if (rg_rand01(r) < g->pl_spawn_prob) {
        float ent_r = g->pl_r_scale;
        int lane = rg_randn(r, g->pl_num_lanes);
        float ent_y = (float)((lane * .11 + .4) * (g->main_height / 2 - ent_r) + g->main_height / 2);
        float moves_right = g->pl_lane_dirs[lane];
        float ent_vx = g->pl_lane_vels[lane] * (moves_right != 0 ? 1 : -1);
        Entity ent;
        entity_init(&ent, 0, ent_y, ent_vx, 0, ent_r, ent_r, PL_SHIP);
        ent.image_type = PL_SHIP;
        ent.image_theme = g->pl_perm[rg_randn(r, g->pl_num_current_ship_types)];
        match_aspect_ratio(g, at, &ent);
        ent.x = moves_right != 0 ? -1 * ent_r : (g->main_width + ent_r);
        ent.is_reflected = !(moves_right != 0);
        if (!has_any_collision(g, &ent, 0)) {
            fassert(g->num_ents < MAX_ENTS);
            g->ents[g->num_ents++] = ent;
        }
    }
    if (g->special_action == 1 && (g->cur_time - g->last_fire_time) >= 3) {
        Entity *agent = AG(g);
        int b = add_entity(g, agent->x, agent->y, 0, 1, .25, PL_PLAYER_BULLET);
        g->ents[b].collides_with_entities = true;
        g->ents[b].expire_time = 50;
        g->last_fire_time = g->cur_time;
        g->pl_juice_left -= 0.02f;
    }
    if (g->pl_juice_left <= 0) g->sd_done = true;
    else if (g->pl_juice_left >= 1) g->pl_juice_left = 1;
    if (g->pl_targets_hit >= g->pl_target_quota) {
        g->sd_done = true;
        g->sd_reward += 10.0f; /* COMPLETION_BONUS */
        g->sd_level_complete = true;
    }
    Entity *agent = AG(g);
    if (agent->x < g->pl_min_agent_x) agent->x = g->pl_min_agent_x;
}

/* ================================================================== starpilot (games/starpilot.cpp) */
#define SP_BULLET_PLAYER 1
#define SP_BULLET2 2
#define SP_BULLET3 3
#define SP_FLYER 4
#define SP_METEOR 5
#define SP_CLOUD 6
#define SP_TURRET 7
#define SP_FAST_FLYER 8
#define SP_FINISH_LINE 9
#define SP_SHOOTER_WIN_TIME 500
#define SP_NUM_BASIC_OBJECTS 9
static const float SP_V_SCALE = 2.0f / 5.0f;

/* std::sort(first, last, comp) of libstdc++ (g++ 11, bits/stl_algo.h: introsort with median-of-3
 * pivots, threshold 16, heapsort fallback, final insertion sort) over spawner indices with
 * spawn_cmp (starpilot.cpp:28-30): a before b iff a.spawn_time > b.spawn_time.  Equal spawn times
 * are common, so the reference's order among them is this algorithm's; pinned against the real
 * std::sort in tests/test_oracle_pins.py. */
typedef struct { const int *key; } SortCtx;
static bool ls_cmp(const SortCtx *c, int a, int b) { return c->key[a] > c->key[b]; }
static void ls_swap(int *x, int i, int j) { int t = x[i]; x[i] = x[j]; x[j] = t; }
static void ls_push_heap(const SortCtx *c, int *f, int hole, int top, int value) {
    int parent = (hole - 1) / 2;
    while (hole > top && ls_cmp(c, f[parent], value)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = value;
}
static void ls_adjust_heap(const SortCtx *c, int *f, int hole, int len, int value) {
    int top = hole, second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (ls_cmp(c, f[second], f[second - 1])) second--;
        f[hole] = f[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        f[hole] = f[second - 1];
        hole = second - 1;
    }
    ls_push_heap(c, f, hole, top, value);
}
static void ls_make_heap(const SortCtx *c, int *f, int len) {
    if (len < 2) return;
    for (int parent = (len - 2) / 2;; parent--) {
        ls_adjust_heap(c, f, parent, len, f[parent]);
        if (parent == 0) return;
    }
}
static void ls_heap_sort(const SortCtx *c, int *f, int len) { /* __partial_sort(first, last, last) */
    ls_make_heap(c, f, len);
    for (int last = len; last > 1;) {
        last--;
        int value = f[last];
        f[last] = f[0];
        ls_adjust_heap(c, f, 0, last, value);
    }
}
static int ls_partition_pivot(const SortCtx *c, int *f, int first, int last) {
    int mid = first + (last - first) / 2;
    int a = first + 1, b = mid, cc = last - 1; /* __move_median_to_first(first, a, b, c) */
    if (ls_cmp(c, f[a], f[b])) {
        if (ls_cmp(c, f[b], f[cc])) ls_swap(f, first, b);
        else if (ls_cmp(c, f[a], f[cc])) ls_swap(f, first, cc);
        else ls_swap(f, first, a);
    } else if (ls_cmp(c, f[a], f[cc])) ls_swap(f, first, a);
    else if (ls_cmp(c, f[b], f[cc])) ls_swap(f, first, cc);
    else ls_swap(f, first, b);
    int lo = first + 1, hi = last, pivot = first; /* __unguarded_partition */
    while (true) {
        while (ls_cmp(c, f[lo], f[pivot])) lo++;
        hi--;
        while (ls_cmp(c, f[pivot], f[hi])) hi--;
        if (!(lo < hi)) return lo;
        ls_swap(f, lo, hi);
        lo++;
    }
}
static void ls_introsort_loop(const SortCtx *c, int *f, int first, int last, int depth) {
    while (last - first > 16) {
        if (depth == 0) {
            ls_heap_sort(c, f + first, last - first);
            return;
        }
        depth--;
        int cut = ls_partition_pivot(c, f, first, last);
        ls_introsort_loop(c, f, cut, last, depth);
        last = cut;
    }
}
static void ls_linear_insert(const SortCtx *c, int *f, int last) {
    int val = f[last], next = last - 1;
    while (ls_cmp(c, val, f[next])) {
        f[last] = f[next];
        last = next;
        next--;
    }
    f[last] = val;
}
static void ls_insertion_sort(const SortCtx *c, int *f, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; i++) {
        if (ls_cmp(c, f[i], f[first])) {
            int val = f[i];
            memmove(&f[first + 1], &f[first], sizeof(int) * (size_t)(i - first));
            f[first] = val;
        } else {
            ls_linear_insert(c, f, i);
        }
    }
}
static void libstdcxx_sort(const int *key, int *idx, int n) {
    SortCtx c = {key};
    if (n <= 1) return;
    int lg = 0;
    while ((1 << (lg + 1)) <= n) lg++; /* std::__lg */
    ls_introsort_loop(&c, idx, 0, n, 2 * lg);
    if (n > 16) {
        ls_insertion_sort(&c, idx, 0, 16);
        for (int i = 16; i < n; i++) ls_linear_insert(&c, idx, i);
    } else {
        ls_insertion_sort(&c, idx, 0, n);
    }
}

/* test hook: the permutation std::sort(spawn_cmp) leaves */
void oracle_spawn_sort(const int32_t *spawn_times, int32_t *idx, int n) {
    for (int i = 0; i < n; i++) idx[i] = i;
    libstdcxx_sort(spawn_times, idx, n);
}

static void sp_init_hps(Game *g) { /* :147-224 */
    float scale = 1;
    for (int i = 0; i < SP_NUM_BASIC_OBJECTS; i++) {
        g->sp_hp_vs[i] = 1;
        g->sp_hp_healths[i] = 0;
        g->sp_hp_prob[i] = 1;
        g->sp_hp_object_r[i] = scale / 2;
    }
    float default_bullet_r = (float)(scale / 2.5);
    int dm = g->options.distribution_mode;
    if (dm == EasyMode) {
        g->sp_hp_prob[SP_METEOR] = 0; g->sp_hp_prob[SP_CLOUD] = 0; g->sp_hp_prob[SP_TURRET] = 0;
        g->sp_hp_prob[SP_FAST_FLYER] = 0;
        g->sp_hp_vs[SP_FLYER] = .75; g->sp_hp_vs[SP_BULLET2] = 1.25;
        g->sp_hp_healths[SP_TURRET] = 5; g->sp_hp_healths[SP_FLYER] = 2; g->sp_hp_healths[SP_FAST_FLYER] = 1;
        g->maxspeed = 0.75;
    } else if (dm == HardMode) {
        g->sp_hp_vs[SP_BULLET2] = 2;
        g->sp_hp_healths[SP_TURRET] = 5; g->sp_hp_healths[SP_FLYER] = 2; g->sp_hp_healths[SP_FAST_FLYER] = 1;
        g->maxspeed = 0.75;
    } else if (dm == ExtremeMode) {
        g->sp_hp_vs[SP_BULLET2] = 2;
        g->sp_hp_healths[SP_TURRET] = 10; g->sp_hp_healths[SP_FLYER] = 5; g->sp_hp_healths[SP_FAST_FLYER] = 2;
        g->maxspeed = 0.5;
        default_bullet_r = scale / 5;
    } else {
        fatal_msg("starpilot: bad distribution mode");
    }
    for (int i = 0; i < SP_NUM_BASIC_OBJECTS; i++) g->sp_hp_bullet_r[i] = default_bullet_r;
    g->sp_hp_healths[SP_METEOR] = 500;
    g->sp_hp_vs[SP_FAST_FLYER] = 1.5;
    g->sp_hp_vs[SP_BULLET_PLAYER] = 2;
    g->sp_hp_vs[SP_BULLET3] = 2;
    g->sp_hp_object_r[SP_TURRET] = scale * 2;
    g->sp_hp_object_r[SP_METEOR] = scale * 2;
    g->sp_hp_object_r[SP_CLOUD] = scale * 2;
    g->sp_hp_prob[SP_FLYER] = 3;
    g->sp_hp_slow_v = .5;
    g->sp_hp_max_group_size = 5;
    g->sp_hp_weapon_bullet_dist = 3;
    g->sp_hp_min_enemy_delta_t = 10;
    g->sp_hp_max_enemy_delta_t = g->sp_hp_min_enemy_delta_t + 20;
    g->sp_hp_spawn_right_threshold = 0.9f;
    g->sp_hp_prob[SP_BULLET_PLAYER] = 0; g->sp_hp_prob[SP_BULLET2] = 0; g->sp_hp_prob[SP_BULLET3] = 0;
    g->sp_total_prob_weight = 0;
    for (int i = 2; i < SP_NUM_BASIC_OBJECTS; i++) g->sp_total_prob_weight += g->sp_hp_prob[i];
}

static float rand_pos(Game *g, float r, float min, float max);

static void sp_add_spawners(Game *g, const or_atlas *at, Entity *out, int *count) { /* :226-327 */
    MT *r = &g->rand_gen;
    int t = 1 + rg_randint(r, g->sp_hp_min_enemy_delta_t, g->sp_hp_max_enemy_delta_t);
    bool can_spawn_left = g->options.distribution_mode != EasyMode;
    *count = 0;
    for (int i = 0; t <= SP_SHOOTER_WIN_TIME; i++) {
        int group_size = 1;
        float start_weight = rg_rand01(r) * g->sp_total_prob_weight;
        float curr_weight = start_weight;
        int type;
        for (type = 2; type < SP_NUM_BASIC_OBJECTS; type++) {
            curr_weight -= g->sp_hp_prob[type];
            if (curr_weight <= 0) break;
        }
        if (type >= SP_NUM_BASIC_OBJECTS) type = SP_NUM_BASIC_OBJECTS - 1;
        float rr = g->sp_hp_object_r[type];
        int flyer_theme = 0;
        if (type == SP_FLYER || type == SP_FAST_FLYER) {
            group_size = rg_randint(r, 0, g->sp_hp_max_group_size) + 1;
            flyer_theme = rg_randn(r, 7); /* NUM_SHIP_THEMES */
        }
        float y_pos = rand_pos(g, rr, 0, (float)g->main_height);
        for (int j = 0; j < group_size; j++) {
            int spawn_time = t + j * 5;
            int fire_time = rg_randint(r, 10, 100);
            float k = 2 * PI_F / 4;
            float theta = (float)((rg_rand01(r) - .5) * k);
            float v_scale = g->sp_hp_vs[type];
            if (rg_randint(r, 0, 2) == 1) theta = 0;
            float health = g->sp_hp_healths[type];
            if (type == SP_METEOR || type == SP_CLOUD) {
                theta = 0;
                v_scale = g->sp_hp_slow_v;
                fire_time = -1;
            } else if (type == SP_TURRET) {
                theta = 0;
                v_scale = g->sp_hp_slow_v;
                fire_time = rg_randint(r, 20, 30);
            }
            v_scale *= SP_V_SCALE;
            float vx = (float)(-1 * cos((double)theta) * v_scale);
            float vy = (float)(sin((double)theta) * v_scale);
            bool spawn_right = true;
            float x_pos;
            if (type == SP_FLYER || type == SP_FAST_FLYER) {
                if (rg_rand01(r) > g->sp_hp_spawn_right_threshold && can_spawn_left) spawn_right = false;
            }
            if (spawn_right) {
                x_pos = g->main_width + rr;
            } else {
                x_pos = -rr;
                vx *= -1;
            }
            fassert(*count < 512);
            Entity *sp = &out[(*count)++];
            entity_init(sp, x_pos, y_pos, vx, vy, rr, rr, type);
            sp->fire_time = fire_time;
            sp->spawn_time = spawn_time;
            sp->health = health;
            if (type == SP_CLOUD) {
                sp->render_z = 1;
                choose_random_theme(g, sp, at);
            } else if (type == SP_METEOR) {
                choose_random_theme(g, sp, at);
            } else if (type == SP_FLYER || type == SP_FAST_FLYER) {
                sp->image_theme = flyer_theme;
                sp->rotation = ((vx > 0) ? -1 : 1) * PI_F / 2;
            } else if (type == SP_TURRET) {
                choose_random_theme(g, sp, at);
                match_aspect_ratio(g, at, sp);
            }
        }
        t += rg_randint(r, g->sp_hp_min_enemy_delta_t, g->sp_hp_max_enemy_delta_t);
    }
}

static void starpilot_game_reset(Game *g, const or_atlas *at) { /* :329-344 */
    basic_game_reset(g, at);
    g->options.center_agent = false;
    sp_init_hps(g);
    static Entity gen[512];
    int n = 0;
    sp_add_spawners(g, at, gen, &n);
    int key[512], idx[512];
    for (int i = 0; i < n; i++) key[i] = gen[i].spawn_time;
    for (int i = 0; i < n; i++) idx[i] = i;
    libstdcxx_sort(key, idx, n);
    for (int i = 0; i < n; i++) g->sp_spawners[i] = gen[idx[i]];
    g->sp_num_spawners = n;
    Entity *agent = AG(g);
    agent->rotation = PI_F / 2;
    choose_random_theme(g, agent, at);
}

static void starpilot_game_step(Game *g, const or_atlas *at) { /* :368-430 */
    basic_game_step(g);
    bool is_firing = g->special_action != 0;
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *m = &g->ents[i];
        if (m->type == PLAYER) continue;
        bool fire;
        if (m->fire_time <= 0) fire = false; /* should_fire (:356-366) */
        else if (m->type == SP_TURRET) fire = (g->cur_time - m->spawn_time) % m->fire_time == 0;
        else fire = g->cur_time - m->spawn_time == m->fire_time;
        if (fire) {
            Entity *agent = AG(g);
            int bullet_type = m->type == SP_TURRET ? SP_BULLET3 : SP_BULLET2;
            float bullet_r = g->sp_hp_bullet_r[m->type];
            float b_vx = agent->x - m->x;
            float b_vy = agent->y - m->y;
            float bv_scale = (float)(g->sp_hp_vs[bullet_type] * SP_V_SCALE / sqrt((double)(b_vx * b_vx + b_vy * b_vy)));
            b_vx = b_vx * bv_scale;
            b_vy = b_vy * bv_scale;
            float mx = m->x, my = m->y;
            int b = add_entity(g, mx, my, b_vx, b_vy, bullet_r, bullet_type);
            if (b_vx != 0 || b_vy != 0) g->ents[b].rotation = -1 * atan2f(b_vy, b_vx) + -1 * PI_F / 2;
            m = &g->ents[i];
        }
        bool destructible = m->type == SP_FLYER || m->type == SP_FAST_FLYER || m->type == SP_TURRET || m->type == SP_METEOR;
        if (m->health <= 0 && destructible && !m->will_erase) {
            float mx = m->x, my = m->y, mvx = m->vx, mvy = m->vy, cr = (float)(.5 * m->rx);
            add_entity(g, mx, my, mvx, mvy, cr, EXPLOSION); /* spawn_child(m, EXPLOSION, .5 * rx, true) */
            g->sd_reward += 1.0f; /* ENEMY_REWARD */
            g->ents[i].will_erase = true;
        }
    }
    while (g->sp_num_spawners > 0 && g->cur_time == g->sp_spawners[g->sp_num_spawners - 1].spawn_time) {
        fassert(g->num_ents < MAX_ENTS);
        g->ents[g->num_ents++] = g->sp_spawners[--g->sp_num_spawners];
    }
    float bullet_r = g->sp_hp_bullet_r[PLAYER];
    if (is_firing) {
        Entity *agent = AG(g);
        float theta = g->special_action == 2 ? PI_F : 0;
        float v_scale = g->sp_hp_vs[SP_BULLET_PLAYER] * SP_V_SCALE;
        float vx = (float)(cos((double)theta) * v_scale);
        float vy = (float)(sin((double)theta) * v_scale);
        float x_off = (float)(agent->rx * cos((double)theta));
        int b = add_entity(g, agent->x + x_off, agent->y, vx, vy, bullet_r, SP_BULLET_PLAYER);
        Entity *bl = &g->ents[b];
        bl->collides_with_entities = true;
        if (vx != 0 || vy != 0) bl->rotation = -1 * atan2f(vy, vx) + 0.0f;
        bl->rotation -= PI_F / 2;
    }
    if (g->cur_time == SP_SHOOTER_WIN_TIME) {
        Entity fin;
        entity_init(&fin, (float)g->main_width, (float)(g->main_height / 2), -1 * g->sp_hp_slow_v * SP_V_SCALE, 0, 2,
                    (float)(g->main_height / 2), SP_FINISH_LINE);
        choose_random_theme(g, &fin, at);
        float ar = asset_aspect_ratio(g, at, fin.image_type + fin.image_theme * MAX_ASSETS); /* match_aspect_ratio(finish, false) */
        fin.rx = fin.ry * ar;
        fin.x = g->main_width + fin.rx;
        fassert(g->num_ents < MAX_ENTS);
        g->ents[g->num_ents++] = fin;
    }
}

/* ================================================================== bossfight (games/bossfight.cpp) */
#define BF_PLAYER_BULLET 1
#define BF_BOSS 2
#define BF_SHIELDS 3
#define BF_ENEMY_BULLET 4
#define BF_LASER_TRAIL 5
#define BF_BARRIER 7
static const float BF_BOSS_R = 3;
#define BF_BOTTOM_MARGIN 6

static void bf_prepare_boss(Game *g) { /* :192-199 */
    g->bf_shields_are_up = true;
    g->bf_curr_vel_timeout = g->bf_boss_vel_timeout;
    g->bf_time_to_swap = g->bf_invulnerable_duration;
    g->bf_attack_mode = g->bf_attack_modes[g->bf_round_num % g->bf_num_attack_modes];
    g->bf_boss->vx = 0;
    g->bf_boss->vy = 0;
}

static void bf_spawn_barriers(Game *g, const or_atlas *at) { /* :310-329 */
    MT *r = &g->rand_gen;
    int num_barriers = rg_randn(r, 3) + 1;
    for (int i = 0; i < num_barriers; i++) {
        float barrier_r = 0.6f;
        float min_barrier_y = (float)(2 * AG(g)->ry + barrier_r + .5);
        float ent_y = rg_rand01(r) * (BF_BOTTOM_MARGIN - min_barrier_y - barrier_r) + min_barrier_y;
        float ent_x = rg_rand01(r) * (g->main_width - 2 * barrier_r) + barrier_r;
        Entity ent;
        entity_init(&ent, ent_x, ent_y, 0, 0, barrier_r, barrier_r, BF_BARRIER);
        choose_random_theme(g, &ent, at);
        match_aspect_ratio(g, at, &ent);
        ent.health = 3;
        ent.collides_with_entities = true;
        if (!has_any_collision(g, &ent, 0)) {
            fassert(g->num_ents < MAX_ENTS);
            g->ents[g->num_ents++] = ent;
        }
    }
}

static void bossfight_game_reset(Game *g, const or_atlas *at) { /* :201-250 */
    MT *r = &g->rand_gen;
    basic_game_reset(g, at);
    g->bf_damaged_until_time = 0;
    g->last_fire_time = 0;
    g->bf_boss_bullet_vel = (float)(g->options.distribution_mode == EasyMode ? .5 : .75);
    int max_extra_invulnerable = g->options.distribution_mode == EasyMode ? 1 : 3;
    g->options.center_agent = false;
    int b = add_entity(g, (float)(g->main_width / 2), (float)(g->main_height / 2), 0, 0, BF_BOSS_R, BF_BOSS);
    choose_random_theme(g, &g->ents[b], at);
    match_aspect_ratio(g, at, &g->ents[b]);
    Entity *boss = &g->ents[b];
    add_entity_rxy(g, boss->x, boss->y, 0, 0, (float)(1.2 * boss->rx), (float)(1.2 * boss->ry), BF_SHIELDS);
    fassert(b == 1);
    g->bf_boss = &g->ents[1];
    g->bf_shields = &g->ents[2];
    g->bf_boss_vel_timeout = 20; /* BOSS_VEL_TIMEOUT */
    g->bf_base_fire_prob = 0.1f;
    g->bf_round_health = rg_randn(r, 9) + 1;
    g->bf_num_rounds = 1 + rg_randn(r, 5);
    g->bf_invulnerable_duration = 2 + rg_randn(r, max_extra_invulnerable + 1);
    g->bf_vulnerable_duration = 500;
    g->bf_boss->health = (float)(g->bf_round_health * g->bf_num_rounds);
    choose_random_theme(g, AG(g), at);
    g->bf_player_laser_theme = rg_randn(r, 3); /* NUM_LASER_THEMES */
    g->bf_boss_laser_theme = rg_randn(r, 3);
    g->bf_num_attack_modes = 0;
    for (int i = 0; i < g->bf_num_rounds; i++) g->bf_attack_modes[g->bf_num_attack_modes++] = rg_randn(r, 4);
    g->bf_round_num = 0;
    bf_prepare_boss(g);
    Entity *agent = AG(g);
    agent->rx = .75;
    match_aspect_ratio(g, at, agent);
    reposition_agent(g);
    agent->y = agent->ry;
    g->bf_barrier_vel = 0.1f;
    g->bf_barriers_moves_right = rg_randbool(r);
    g->bf_barrier_spawn_prob = 0.025f;
    bf_spawn_barriers(g, at);
}

static void bf_boss_fire(Game *g, float bullet_r, float vel, float theta) { /* :252-257 */
    Entity *boss = g->bf_boss;
    float bx = boss->x, by = boss->y;
    int e = add_entity(g, bx, by, (float)(vel * cos((double)theta)), (float)(vel * sin((double)theta)), bullet_r,
                       BF_ENEMY_BULLET);
    g->ents[e].image_theme = g->bf_boss_laser_theme;
    g->ents[e].expire_time = 50;
    g->ents[e].vrot = PI_F / 8;
}

static void bossfight_game_step(Game *g) { /* :331-392 */
    MT *r = &g->rand_gen;
    basic_game_step(g);
    /* erase_if_needed may have moved the boss / shields down one slot (only the agent can go) */
    for (int i = 0; i < g->num_ents; i++) {
        if (g->ents[i].type == BF_BOSS) g->bf_boss = &g->ents[i];
        if (g->ents[i].type == BF_SHIELDS) g->bf_shields = &g->ents[i];
    }
    Entity *boss = g->bf_boss;
    g->bf_shields->x = boss->x;
    g->bf_shields->y = boss->y;
    g->bf_rand_pct = rg_rand01(r);
    g->bf_rand_fire_pct = rg_rand01(r);
    g->bf_rand_pct_x = rg_rand01(r);
    g->bf_rand_pct_y = rg_rand01(r);
    if (g->bf_curr_vel_timeout <= 0) {
        float dest_x = g->bf_rand_pct_x * (g->main_width - 2 * BF_BOSS_R) + BF_BOSS_R;
        float dest_y = g->bf_rand_pct_y * (g->main_height - 2 * BF_BOSS_R - BF_BOTTOM_MARGIN) + BF_BOSS_R + BF_BOTTOM_MARGIN;
        boss->vx = (dest_x - boss->x) / g->bf_boss_vel_timeout;
        boss->vy = (dest_y - boss->y) / g->bf_boss_vel_timeout;
        g->bf_curr_vel_timeout = g->bf_boss_vel_timeout;
        if (g->bf_time_to_swap > 0) {
            g->bf_time_to_swap -= 1;
        } else {
            g->bf_time_to_swap = g->bf_shields_are_up ? g->bf_vulnerable_duration : g->bf_invulnerable_duration;
            g->bf_shields_are_up = !g->bf_shields_are_up;
        }
    } else {
        g->bf_curr_vel_timeout -= 1;
    }
    if (g->special_action == 1 && (g->cur_time - g->last_fire_time) >= 3) {
        Entity *agent = AG(g);
        int e = add_entity(g, agent->x, agent->y, 0, 1, .25, BF_PLAYER_BULLET);
        g->ents[e].image_theme = g->bf_player_laser_theme;
        g->ents[e].collides_with_entities = true;
        g->ents[e].expire_time = 25;
        g->last_fire_time = g->cur_time;
    }
    int ct = g->cur_time;
    float bv = g->bf_boss_bullet_vel, rp = g->bf_rand_pct;
    if (g->bf_damaged_until_time >= ct) { /* damaged_mode (:299-305) */
        if (ct % 3 == 0) {
            boss = g->bf_boss;
            float pos_x = boss->x + (2 * g->bf_rand_pct_x - 1) * boss->rx;
            float pos_y = boss->y + (2 * g->bf_rand_pct_y - 1) * boss->ry;
            add_entity(g, pos_x, pos_y, 0, 0, .75, EXPLOSION);
        }
    } else if (g->bf_shields_are_up) { /* active_attack (:307-317) */
        int am = g->bf_attack_mode;
        if (am == 0) { /* :265-271 */
            if (ct % 8 == 0)
                for (int i = 0; i < 5; i++) bf_boss_fire(g, .5, bv, (float)(PI_F * 1.5 + (i - 2) * PI_F / 8));
        } else if (am == 1) { /* :273-282 */
            int dt = 5;
            if (ct % dt == 0) {
                int k = ct / dt;
                k = abs(8 - (k % 16));
                for (int i = 0; i < 4; i++) bf_boss_fire(g, .5, bv, (float)(PI_F * (1.25 + .5 * k / 8.0) + i * PI_F / 2));
            }
        } else if (am == 2) { /* :284-293 */
            if (ct % 10 == 0) {
                int num_bullets = 8;
                float offset = rp * 2 * PI_F;
                for (int i = 0; i < num_bullets; i++) {
                    float theta = 2 * PI_F / num_bullets * i + offset;
                    bf_boss_fire(g, .5, bv, theta);
                }
            }
        } else if (am == 3) { /* :295-299 */
            if (ct % 4 == 0) bf_boss_fire(g, .5, bv, PI_F * (1 + rp));
        }
    } else { /* passive_attack_mode (:259-263) */
        if (g->bf_rand_fire_pct < g->bf_base_fire_prob) bf_boss_fire(g, .5, bv, PI_F * (1 + rp));
    }
    for (int i = g->num_ents - 1; i >= 0; i--) {
        Entity *ent = &g->ents[i];
        if (ent->type == BF_ENEMY_BULLET) {
            float v_trail = .5;
            float ex = ent->x, ey = ent->y, evx = ent->vx * v_trail, evy = ent->vy * v_trail, erx = ent->rx, ery = ent->ry;
            float evrot = ent->vrot, erot = ent->rotation;
            int t = add_entity_rxy(g, ex, ey, evx, evy, erx, ery, BF_LASER_TRAIL);
            Entity *tr = &g->ents[t];
            tr->alpha_decay = 0.7f;
            tr->image_type = BF_ENEMY_BULLET;
            tr->image_theme = g->bf_boss_laser_theme;
            tr->vrot = evrot;
            tr->rotation = erot;
            tr->expire_time = 8;
        }
    }
}

/* ================================================================== ninja (games/ninja.cpp) */
#define NJ_GOAL 1
#define NJ_BOMB 6
#define NJ_THROWING_STAR 7
#define NJ_FIRE 14
#define NJ_WALL_MID 20

static void nj_fill_block_top(Game *g, int x, int y, int dx, int dy, int fill, int top) { /* :162-167 */
    if (dy <= 0) return;
    fill_elem(g, x, y, dx, dy - 1, fill);
    fill_elem(g, x, y + dy - 1, dx, 1, top);
}
static void nj_fill_ground_block(Game *g, int x, int y, int dx, int dy) {
    nj_fill_block_top(g, x, y, dx, dy, NJ_WALL_MID, NJ_WALL_MID);
}

static void nj_generate(Game *g, const or_atlas *at, int difficulty) { /* generate_coin_to_the_right :180-297 */
    MT *r = &g->rand_gen;
    int min_gap = difficulty - 1, min_plat_w = 1, inc_dy = 4;
    if (g->options.distribution_mode == EasyMode) {
        min_gap -= 1;
        if (min_gap < 0) min_gap = 0;
        min_plat_w = 3;
        inc_dy = 2;
    }
    float bomb_prob = (float)(.25 * (difficulty - 1));
    int max_gap_inc = difficulty == 1 ? 1 : 2;
    int num_sections = rg_randn(r, difficulty) + difficulty;
    int start_x = 5, curr_x = start_x, curr_y = g->main_height / 2, min_y = curr_y;
    int w = g->main_width;
    float _max_dy = g->max_jump * g->max_jump / (2 * g->gravity);
    int max_dy = (int)(_max_dy - .5);
    int prev_x, prev_y;
    nj_fill_ground_block(g, 0, 0, start_x, curr_y);
    fill_elem(g, 0, curr_y + 8, start_x, g->main_height - curr_y - 8, NJ_WALL_MID);
    for (int i = 0; i < num_sections; i++) {
        prev_x = curr_x;
        prev_y = curr_y;
        int num_edges = rg_randn(r, 2) + 1;
        int max_y = -1, last_edge_y = -1;
        for (int j = 0; j < num_edges; j++) {
            curr_x = prev_x + j;
            if (curr_x + 15 >= w) break;
            curr_y = prev_y;
            int dy = rg_randn(r, inc_dy) + 1 + (int)(difficulty / 3);
            if (dy > max_dy) dy = max_dy;
            if (curr_y >= g->main_height - 15) dy *= -1;
            else if (curr_y >= 5 && rg_rand01(r) < .4) dy *= -1;
            curr_y += dy;
            if (curr_y < 3) curr_y = 3;
            if (abs(curr_y - last_edge_y) <= 1) curr_y = last_edge_y + 2;
            int dx = min_plat_w + rg_randn(r, 3);
            nj_fill_ground_block(g, curr_x, curr_y - 1, dx, 1);
            curr_x += dx;
            curr_x += min_gap + rg_randn(r, max_gap_inc + 1);
            if (curr_y > max_y) max_y = curr_y;
            if (curr_y < min_y) min_y = curr_y;
            last_edge_y = curr_y;
        }
        if (rg_rand01(r) < bomb_prob) {
            int bx = rg_randn(r, curr_x - prev_x + 1) + prev_x;
            set_obj(g, bx, max_y + 2, NJ_BOMB);
        }
        int ceiling_height = 11;
        int ceiling_start = max_y - 1 + ceiling_height;
        nj_fill_ground_block(g, prev_x, ceiling_start, curr_x - prev_x, g->main_height - ceiling_start);
    }
    int e = add_entity(g, (float)(curr_x + .5), (float)(curr_y + .5), 0, 0, .5, NJ_GOAL);
    choose_random_theme(g, &g->ents[e], at);
    nj_fill_ground_block(g, curr_x, curr_y - 1, 1, 1);
    fill_elem(g, curr_x, curr_y + 6, 1, g->main_height - curr_y - 6, NJ_WALL_MID);
    int fire_y = min_y - 2;
    if (fire_y < 1) fire_y = 1;
    nj_fill_ground_block(g, start_x, 0, g->main_width - start_x, fire_y);
    fill_elem(g, start_x, fire_y, g->main_width - start_x, 1, NJ_FIRE);
    fill_elem(g, curr_x + 1, 0, g->main_width - curr_x - 1, g->main_height, NJ_WALL_MID);
}

static void ninja_game_reset(Game *g, const or_atlas *at) { /* :299-331 */
    basic_game_reset(g, at);
    g->gravity = 0.2f;
    g->max_jump = 1.5;
    g->air_control = 0.15f;
    g->maxspeed = .5;
    g->has_support = false;
    g->facing_right = true;
    g->nj_jump_charge = 0;
    g->nj_jump_charge_inc = .25;
    g->visibility = 16;
    Entity *agent = AG(g);
    agent->rx = .5;
    agent->ry = .5;
    agent->x = 1 + agent->rx;
    agent->y = g->main_height / 2 + agent->ry;
    if (g->options.distribution_mode == EasyMode) {
        g->max_jump = 1.25;
        g->nj_jump_charge_inc = 1;
        g->visibility = 10;
    }
    int difficulty = rg_randn(&g->rand_gen, 3) + 1;
    g->last_fire_time = 0;
    g->wall_theme = rg_randn(&g->rand_gen, 3); /* NUM_WALL_THEMES */
    /* init_floor_and_walls (:169-174) */
    fill_elem(g, 0, 0, g->main_width, 1, NJ_WALL_MID);
    fill_elem(g, 0, 0, 1, g->main_height, NJ_WALL_MID);
    fill_elem(g, g->main_width - 1, 0, 1, g->main_height, NJ_WALL_MID);
    fill_elem(g, 0, g->main_height - 1, g->main_width, 1, NJ_WALL_MID);
    nj_generate(g, at, difficulty);
}

static void ninja_game_step(Game *g) { /* :420-450 */
    basic_game_step(g);
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = false;
    if (g->action_vx < 0) agent->is_reflected = true;
    if (g->special_action > 0 && (g->cur_time - g->last_fire_time) >= 3) {
        float theta = 0, bullet_vel = 1;
        if (g->special_action == 1) theta = 0;
        else if (g->special_action == 2) theta = PI_F / 4;
        else if (g->special_action == 3) theta = PI_F / 2;
        else if (g->special_action == 4) theta = -1 * PI_F / 4;
        if (agent->is_reflected) theta = PI_F - theta;
        int b = add_entity(g, agent->x, agent->y, (float)(bullet_vel * cos((double)theta)),
                           (float)(bullet_vel * sin((double)theta)), .25, NJ_THROWING_STAR);
        g->ents[b].collides_with_entities = true;
        g->ents[b].expire_time = 15;
        g->ents[b].smart_step = true;
        g->last_fire_time = g->cur_time;
    }
}

/* ================================================================== caveflyer (games/caveflyer.cpp) */
#define CF_GOAL 1
#define CF_OBSTACLE 2
#define CF_TARGET 3
#define CF_PLAYER_BULLET 4
#define CF_ENEMY 5
#define CF_CAVEWALL 8
#define CF_EXHAUST 9
#define CF_MARKER 1003

/* RoomGenerator (roomgen.cpp) over the game grid; get_obj(idx) / to_grid_idx follow
 * basic-abstract-game.cpp:187-203 (out-of-grid -> INVALID_IDX -> out_of_bounds_object) */
static int rm_to_grid_idx(Game *g, int x, int y) { return grid_contains(g, x, y) ? y * g->grid_w + x : INVALID_IDX; }
static int rm_get_obj_idx(Game *g, int idx) {
    if (idx < 0 || idx >= g->grid_w * g->grid_h) return g->out_of_bounds_object;
    return g->grid[idx];
}
static void rm_update(Game *g) { /* roomgen.cpp:3-37: count_neighbors(i, WALL_OBJ) >= 5 over the 3x3 block */
    static int next_cells[MAX_GRID];
    for (int i = 0; i < g->grid_size; i++) {
        int x = i % g->grid_w, y = i / g->grid_w, n = 0;
        for (int a = -1; a <= 1; a++)
            for (int b = -1; b <= 1; b++)
                if (get_obj(g, x + a, y + b) == WALL_OBJ) n++;
        next_cells[i] = n >= 5 ? WALL_OBJ : SPACE;
    }
    for (int i = 0; i < g->grid_size; i++) g->grid[i] = next_cells[i];
}
/* build_room (roomgen.cpp:39-70): the start cell joins its own room only when a neighbour
 * rediscovers it, so an isolated SPACE cell yields an empty room.  Fills `room` (bool per cell),
 * returns its size. */
static int rm_build_room(Game *g, int idx, bool *room) {
    static int queue[MAX_GRID * 4 + 1];
    int head = 0, tail = 0, size = 0;
    if (rm_get_obj_idx(g, idx) != SPACE) return 0;
    queue[tail++] = idx;
    while (head < tail) {
        int cur = queue[head++];
        if (rm_get_obj_idx(g, cur) != SPACE) continue;
        int x = cur % g->grid_w, y = cur / g->grid_w;
        for (int i = -1; i <= 1; i++)
            for (int j = -1; j <= 1; j++)
                if ((i == 0 || j == 0) && (i + j != 0)) {
                    int nx = rm_to_grid_idx(g, x + i, y + j);
                    if (nx >= 0 && !room[nx] && rm_get_obj_idx(g, nx) == SPACE) {
                        queue[tail++] = nx;
                        room[nx] = true;
                        size++;
                    }
                }
    }
    return size;
}
/* find_best_room (roomgen.cpp:116-136): first room (scan order) of strictly largest size */
static int rm_find_best_room(Game *g, bool *best) {
    static bool all_rooms[MAX_GRID], next_room[MAX_GRID];
    int best_size = -1;
    memset(all_rooms, 0, sizeof(all_rooms));
    memset(best, 0, MAX_GRID);
    for (int i = 0; i < g->grid_size; i++) {
        if (rm_get_obj_idx(g, i) == SPACE && !all_rooms[i]) {
            memset(next_room, 0, sizeof(next_room));
            int sz = rm_build_room(g, i, next_room);
            for (int k = 0; k < g->grid_size; k++) all_rooms[k] = all_rooms[k] || next_room[k];
            if (sz > best_size) {
                best_size = sz;
                memcpy(best, next_room, MAX_GRID);
            }
        }
    }
    return best_size;
}
/* find_path (roomgen.cpp:72-114): BFS whose `covered` set never holds the source */
static int rm_find_path(Game *g, int src, int dst, int *path) {
    static int expanded[MAX_GRID + 2], parents[MAX_GRID + 2], tmp[MAX_GRID + 2];
    static bool covered[MAX_GRID];
    int n = 0, search_idx = 0;
    if (rm_get_obj_idx(g, src) != SPACE) return 0;
    memset(covered, 0, sizeof(covered));
    expanded[n] = src;
    parents[n++] = -1;
    while (search_idx < n) {
        int cur = expanded[search_idx];
        if (cur == dst) break;
        fassert(rm_get_obj_idx(g, cur) == SPACE);
        int x = cur % g->grid_w, y = cur / g->grid_w;
        for (int i = -1; i <= 1; i++)
            for (int j = -1; j <= 1; j++)
                if ((i == 0 || j == 0) && (i + j != 0)) {
                    int nx = rm_to_grid_idx(g, x + i, y + j);
                    if (nx >= 0 && !covered[nx] && rm_get_obj_idx(g, nx) == SPACE) {
                        fassert(n < MAX_GRID + 2);
                        expanded[n] = nx;
                        parents[n++] = search_idx;
                        covered[nx] = true;
                    }
                }
        search_idx++;
    }
    fassert(search_idx < n && expanded[search_idx] == dst);
    int t = 0;
    while (search_idx >= 0) {
        tmp[t++] = expanded[search_idx];
        search_idx = parents[search_idx];
    }
    for (int j = t - 1; j >= 0; j--) path[t - 1 - j] = tmp[j];
    return t;
}
/* expand_room (roomgen.cpp:138-177): n rounds of 8-neighbour growth through SPACE cells */
static void rm_expand_room(Game *g, bool *set, int n) {
    static bool curr[MAX_GRID], next[MAX_GRID];
    memcpy(curr, set, MAX_GRID);
    for (int loop = 0; loop < n; loop++) {
        memset(next, 0, sizeof(next));
        for (int cur = 0; cur < g->grid_size; cur++) {
            if (!curr[cur] || rm_get_obj_idx(g, cur) != SPACE) continue;
            int x = cur % g->grid_w, y = cur / g->grid_w;
            for (int i = -1; i <= 1; i++)
                for (int j = -1; j <= 1; j++)
                    if (i != 0 || j != 0) {
                        int nx = rm_to_grid_idx(g, x + i, y + j);
                        if (nx >= 0 && !set[nx] && rm_get_obj_idx(g, nx) == SPACE) {
                            set[nx] = true;
                            next[nx] = true;
                        }
                    }
        }
        memcpy(curr, next, MAX_GRID);
    }
}

static void caveflyer_ctor(Game *g) { g->mixrate = 0.9f; } /* caveflyer.cpp:25-29 */

static void caveflyer_choose_world_dim(Game *g) { /* :128-143 */
    int d = g->options.distribution_mode, world_dim = 20;
    if (d == EasyMode) world_dim = 30;
    else if (d == HardMode) world_dim = 40;
    else if (d == MemoryMode) world_dim = 60;
    g->main_width = world_dim;
    g->main_height = world_dim;
}

static void caveflyer_game_reset(Game *g, const or_atlas *at) { /* :145-265 */
    static bool best_room[MAX_GRID], wide_path[MAX_GRID];
    static int free_cells[MAX_GRID], goal_path[MAX_GRID + 2], sel[MAX_GRID];
    MT *r = &g->rand_gen;
    caveflyer_choose_world_dim(g);
    basic_game_reset(g, at);
    g->out_of_bounds_object = WALL_OBJ;
    for (int i = 0; i < g->grid_size; i++) g->grid[i] = rg_rand01(r) < .5 ? WALL_OBJ : SPACE;
    for (int it = 0; it < 4; it++) rm_update(g);
    int best = rm_find_best_room(g, best_room);
    fassert(best > 0);
    for (int i = 0; i < g->grid_size; i++) g->grid[i] = WALL_OBJ;
    int nfree = 0;
    for (int i = 0; i < g->grid_size; i++)
        if (best_room[i]) {
            g->grid[i] = SPACE;
            free_cells[nfree++] = i;
        }
    rg_simple_choose(r, nfree, 2, sel);
    int agent_cell = free_cells[sel[0]], goal_cell = free_cells[sel[1]];
    Entity *agent = AG(g);
    agent->x = (float)((agent_cell % g->main_width) + .5);
    agent->y = (float)((agent_cell / g->main_width) + .5);
    int ge = add_entity(g, (float)((goal_cell % g->main_width) + .5), (float)((goal_cell / g->main_width) + .5), 0, 0,
                        .5, CF_GOAL); /* spawn_entity_at_idx (:587-594) */
    g->ents[ge].collides_with_entities = true;
    int npath = rm_find_path(g, agent_cell, goal_cell, goal_path);
    if (g->options.distribution_mode != MemoryMode) { /* should_prune */
        memset(wide_path, 0, sizeof(wide_path));
        for (int k = 0; k < npath; k++) wide_path[goal_path[k]] = true;
        rm_expand_room(g, wide_path, 4);
        for (int i = 0; i < g->grid_size; i++) g->grid[i] = wide_path[i] ? SPACE : WALL_OBJ;
    }
    for (int it = 0; it < 4; it++) {
        rm_update(g);
        for (int k = 0; k < npath; k++) g->grid[goal_path[k]] = SPACE;
    }
    for (int k = 0; k < npath; k++) g->grid[goal_path[k]] = CF_MARKER;
    nfree = 0;
    for (int i = 0; i < g->grid_size; i++) {
        if (g->grid[i] == SPACE) free_cells[nfree++] = i;
        else if (g->grid[i] == WALL_OBJ) g->grid[i] = CF_CAVEWALL;
    }
    int chunk_size = nfree / 80, num_objs = 3 * chunk_size;
    rg_simple_choose(r, nfree, num_objs, sel);
    for (int i = 0; i < num_objs; i++) {
        int val = free_cells[sel[i]];
        float x = (float)((val % g->main_width) + .5), y = (float)((val / g->main_width) + .5);
        if (i < chunk_size) {
            int e = add_entity(g, x, y, 0, 0, .5, CF_OBSTACLE);
            g->ents[e].collides_with_entities = true;
        } else if (i < 2 * chunk_size) {
            int e = add_entity(g, x, y, 0, 0, .5, CF_TARGET);
            g->ents[e].health = 5;
            g->ents[e].collides_with_entities = true;
        } else {
            int e = add_entity(g, x, y, 0, 0, .5, CF_ENEMY);
            /* (.1 * rand01() + .1) * (randn(2) * 2 - 1): left operand drawn first (pinned,
             * oracle/ref_harness.cpp ref_caveflyer_enemy_vel) */
            double mag = .1 * (double)rg_rand01(r) + .1;
            int sgn = rg_randn(r, 2) * 2 - 1;
            float vel = (float)(mag * sgn);
            if (rg_rand01(r) < .5) g->ents[e].vx = vel;
            else g->ents[e].vy = vel;
            g->ents[e].smart_step = true;
            g->ents[e].collides_with_entities = true;
        }
    }
    for (int i = 0; i < g->grid_size; i++)
        if (g->grid[i] == CF_MARKER) g->grid[i] = SPACE;
    g->out_of_bounds_object = CF_CAVEWALL;
    g->visibility = g->options.distribution_mode == EasyMode ? 10 : 16;
}

static void caveflyer_set_action_xy(Game *g, int move_action) { /* :267-287 */
    float acceleration = (float)(move_action % 3 - 1);
    if (acceleration < 0) acceleration *= 0.33f;
    Entity *agent = AG(g);
    float theta = -1 * agent->rotation + PI_F / 2;
    if (acceleration > 0) {
        int e = add_entity(g, (float)(agent->x - agent->rx * cos((double)theta)),
                           (float)(agent->y - agent->ry * sin((double)theta)), 0, 0, (float)(.5 * agent->rx), CF_EXHAUST);
        agent = AG(g);
        g->ents[e].expire_time = 4;
        g->ents[e].rotation = -1 * theta - PI_F / 2;
        g->ents[e].grow_rate = 1.25;
        g->ents[e].alpha_decay = 0.8f;
    }
    g->action_vy = (float)(acceleration * sin((double)theta));
    g->action_vx = (float)(acceleration * cos((double)theta));
    g->action_vrot = (float)(move_action / 3 - 1);
}

static void caveflyer_game_step(Game *g) { /* :289-324 */
    basic_game_step(g);
    Entity *agent = AG(g);
    if (g->special_action == 1) {
        float theta = -1 * agent->rotation + PI_F / 2;
        float vx = (float)cos((double)theta), vy = (float)sin((double)theta);
        float ax = agent->x, ay = agent->y, arot = agent->rotation;
        int b = add_entity_rxy(g, ax, ay, vx, vy, 0.1f, 0.25f, CF_PLAYER_BULLET);
        g->ents[b].expire_time = 10;
        g->ents[b].rotation = arot;
    }
    for (int ei = g->num_ents - 1; ei >= 0; ei--) {
        Entity *ent = &g->ents[ei];
        if (ent->type == CF_ENEMY) { /* face_direction(vx, vy, -PI / 2) (entity.cpp:84-88) */
            if (ent->vx != 0 || ent->vy != 0) ent->rotation = -1 * atan2f(ent->vy, ent->vx) + (-1 * PI_F / 2);
        }
        if (ent->type != CF_PLAYER_BULLET) continue;
        bool found_wall = false;
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++) {
                int t2 = get_obj_from_floats(g, ent->x + ent->rx * (float)(2 * i - 1), ent->y + ent->ry * (float)(2 * j - 1));
                found_wall = found_wall || t2 == CF_CAVEWALL;
            }
        if (found_wall) {
            ent->will_erase = true;
            spawn_child(g, ei, EXPLOSION, (float)(.5 * ent->rx));
        }
    }
    erase_if_needed(g);
}

/* ================================================================== jumper (games/jumper.cpp) */
#define JP_GOAL 1
#define JP_SPIKE 2
#define JP_CAVEWALL 6
#define JP_CAVEWALL_TOP 7
#define JP_MAZE_SCALE 3
#define JP_JUMP_COOLDOWN 3

static bool jp_is_wall(int t) { return t == JP_CAVEWALL || t == JP_CAVEWALL_TOP; } /* :381-383 */
static bool jp_is_space_on_ground(Game *g, int x, int y) { /* :182-189 */
    if (get_obj(g, x, y) != SPACE) return false;
    if (get_obj(g, x, y + 1) != SPACE) return false;
    int below = get_obj(g, x, y - 1);
    return below == JP_CAVEWALL || below == g->out_of_bounds_object;
}
static bool jp_is_top_wall(Game *g, int x, int y) { return get_obj(g, x, y) == JP_CAVEWALL && get_obj(g, x, y + 1) == SPACE; }
static bool jp_is_left_wall(Game *g, int x, int y) { return get_obj(g, x, y) == JP_CAVEWALL && get_obj(g, x + 1, y) == SPACE; }
static bool jp_is_right_wall(Game *g, int x, int y) { return get_obj(g, x, y) == JP_CAVEWALL && get_obj(g, x - 1, y) == SPACE; }

static void jumper_game_reset(Game *g, const or_atlas *at) { /* :221-379 */
    static bool best_room[MAX_GRID], wide_path[MAX_GRID];
    static int free_cells[MAX_GRID], cands[MAX_GRID], goal_path[MAX_GRID + 2];
    static MazeGen mg;
    MT *r = &g->rand_gen;
    int dm = g->options.distribution_mode;
    if (dm == EasyMode) {
        g->visibility = 12;
        g->jp_compass_dim = 3;
    } else {
        g->visibility = 16;
        g->jp_compass_dim = 2;
    }
    if (dm == MemoryMode) g->timeout = 2000;
    int world_dim = 20; /* choose_world_dim (:204-219) */
    if (dm == EasyMode) world_dim = 20;
    else if (dm == HardMode) world_dim = 40;
    else if (dm == MemoryMode) world_dim = 45;
    g->main_width = world_dim;
    g->main_height = world_dim;
    basic_game_reset(g, at);
    int W = g->main_width, H = g->main_height;
    g->out_of_bounds_object = WALL_OBJ;
    g->wall_theme = rg_randn(r, 4); /* NUM_WALL_THEMES */
    g->jp_jump_count = 0;
    g->jp_jump_delta = 0;
    g->jp_jump_time = 0;
    g->has_support = false;
    g->facing_right = true;
    int maze_dim = W / JP_MAZE_SCALE;
    mg_init(&mg, r, maze_dim);
    mg_generate_maze_no_dead_ends(&mg);
    for (int i = 0; i < g->grid_size; i++) {
        int obj = mg_gridget(&mg, (i % W) / JP_MAZE_SCALE + 1, (i / W) / JP_MAZE_SCALE + 1);
        float prob = obj == WALL_OBJ ? .8f : .2f;
        g->grid[i] = rg_rand01(r) < prob ? WALL_OBJ : SPACE;
    }
    for (int it = 0; it < 2; it++) rm_update(g);
    for (int i = 0; i < W; i++) { /* border cells */
        set_obj(g, i, 0, JP_CAVEWALL);
        set_obj(g, i, H - 1, JP_CAVEWALL);
    }
    for (int i = 0; i < H; i++) {
        set_obj(g, 0, i, JP_CAVEWALL);
        set_obj(g, W - 1, i, JP_CAVEWALL);
    }
    int best = rm_find_best_room(g, best_room);
    fassert(best > 0);
    int nfree = 0;
    for (int i = 0; i < g->grid_size; i++) {
        g->grid[i] = best_room[i] ? SPACE : JP_CAVEWALL;
        if (best_room[i]) free_cells[nfree++] = i;
    }
    int goal_cell = free_cells[rg_randn(r, nfree)]; /* choose_one (randgen.cpp:43-47) */
    int ncand = 0;
    for (int i = 0; i < g->grid_size; i++)
        if (jp_is_space_on_ground(g, i % W, i / W)) cands[ncand++] = i;
    fassert(ncand > 0);
    int agent_cell = cands[rg_randn(r, ncand)];
    int npath = rm_find_path(g, agent_cell, goal_cell, goal_path);
    if (dm != MemoryMode) { /* should_prune */
        memset(wide_path, 0, sizeof(wide_path));
        for (int k = 0; k < npath; k++) wide_path[goal_path[k]] = true;
        rm_expand_room(g, wide_path, 4);
        for (int i = 0; i < g->grid_size; i++) g->grid[i] = wide_path[i] ? SPACE : JP_CAVEWALL;
    }
    int ge = add_entity(g, (float)((goal_cell % W) + .5), (float)((goal_cell / W) + .5), 0, 0, .5, JP_GOAL);
    fassert(ge == 1);
    float spike_prob = dm == MemoryMode ? 0 : .2f;
    for (int i = 0; i < g->grid_size; i++) {
        int x = i % W, y = i / W;
        if (jp_is_space_on_ground(g, x, y) && (jp_is_space_on_ground(g, x - 1, y) && jp_is_space_on_ground(g, x + 1, y))) {
            if (rg_rand01(r) < spike_prob) set_obj(g, x, y, JP_SPIKE);
        }
    }
    for (int i = 0; i < g->grid_size; i++) { /* no long vertical walls (:325-337) */
        int x = i % W, y = i / W;
        if (jp_is_left_wall(g, x, y) && jp_is_left_wall(g, x, y + 1) && jp_is_left_wall(g, x, y + 2))
            set_obj(g, x, y + rg_randn(r, 3), SPACE);
        if (jp_is_right_wall(g, x, y) && jp_is_right_wall(g, x, y + 1) && jp_is_right_wall(g, x, y + 2))
            set_obj(g, x, y + rg_randn(r, 3), SPACE);
    }
    Entity *agent = AG(g);
    agent->x = (float)((agent_cell % W) + .5);
    agent->y = (agent_cell / W) + agent->ry;
    for (int i = 0; i < g->grid_size; i++) { /* get_cells_with_type(SPIKE), ascending */
        if (g->grid[i] != JP_SPIKE) continue;
        g->grid[i] = SPACE;
        float spike_ry = 0.4f, spike_rx = 0.23f;
        add_entity_rxy(g, (float)((i % W) + .5), (i / W) + spike_ry, 0, 0, spike_rx, spike_ry, JP_SPIKE);
    }
    for (int i = 0; i < g->grid_size; i++)
        if (jp_is_top_wall(g, i % W, i / W)) g->grid[i] = JP_CAVEWALL_TOP;
    agent = AG(g);
    agent->rx = 0.254f;
    agent->ry = 0.4f;
    g->out_of_bounds_object = JP_CAVEWALL;
}

static void jumper_set_action_xy(Game *g, int move_action) { /* :389-422 */
    g->action_vx = (float)(move_action / 3 - 1);
    g->action_vy = (float)((move_action % 3) - 1);
    if (g->action_vy < 0) g->action_vy = 0;
    if (g->action_vx > 0) g->facing_right = true;
    if (g->action_vx < 0) g->facing_right = false;
    Entity *agent = AG(g);
    int b1 = get_obj_from_floats(g, (float)(agent->x - (agent->rx - .01)), (float)(agent->y - (agent->ry + .01)));
    int b2 = get_obj_from_floats(g, (float)(agent->x + (agent->rx - .01)), (float)(agent->y - (agent->ry + .01)));
    g->jp_jump_delta = 0;
    g->has_support = (jp_is_wall(b1) || b1 == g->out_of_bounds_object) || (jp_is_wall(b2) || b2 == g->out_of_bounds_object);
    if (g->has_support) g->jp_jump_count = 2;
    if (g->action_vy == 1 && g->jp_jump_count > 0 && (g->cur_time - g->jp_jump_time > JP_JUMP_COOLDOWN)) {
        g->jp_jump_count -= 1;
        g->jp_jump_delta = -1;
    } else {
        g->action_vy = 0;
    }
    if (g->action_vy > 0) g->jp_jump_time = g->cur_time;
    g->action_vrot = 0;
}

static void jumper_game_step(Game *g) { /* :424-441 */
    basic_game_step(g);
    Entity *agent = AG(g);
    if (g->action_vx > 0) agent->is_reflected = false;
    if (g->action_vx < 0) agent->is_reflected = true;
    if (fabs((double)agent->vx) + fabs((double)agent->vy) > .05) {
        float ax = agent->x, ty = (float)(agent->y - agent->ry * .5);
        int t = add_entity_rxy(g, ax, ty, 0, 0.01f, 0.3f, 0.2f, TRAIL);
        g->ents[t].expire_time = 8;
        g->ents[t].alpha = .5;
    }
    agent = AG(g);
    if (agent->vy > -2) agent->vy -= 0.15f;
}

/* ================================================================== leaper (games/leaper.cpp) */
#define LP_LOG 1
#define LP_ROAD 2
#define LP_WATER 3
#define LP_CAR 4
#define LP_FINISH_LINE 5
static const float LP_MONSTER_RADIUS = 0.25f;
static const float LP_LOG_RADIUS = 0.45f;
#define LP_NSTEP 5
static const float LP_MAX_SPEED = (float)(2 / (LP_NSTEP - 1.0));
static const float LP_VEL_DECAY = (float)(2 / (LP_NSTEP - 1.0)) / LP_NSTEP;

static float lp_sign(float x) { return x > 0 ? +1 : (x == 0 ? 0 : -1); } /* leaper.cpp:21-23 */

static float lp_rand_sign(Game *g) { /* :91-97 */
    if ((double)rg_rand01(&g->rand_gen) < 0.5) return 1.0f;
    return -1.0f;
}

static void leaper_choose_world_dim(Game *g) { /* :99-113 */
    int world_dim = 20;
    if (g->options.distribution_mode == EasyMode) world_dim = 9;
    else if (g->options.distribution_mode == HardMode) world_dim = 15;
    g->main_width = world_dim;
    g->main_height = world_dim;
}

static int lp_choose_extra_space(Game *g) { /* :115-117 */
    return g->options.distribution_mode == EasyMode ? 0 : rg_randn(&g->rand_gen, 2);
}

static void lp_spawn_entities(Game *g, const or_atlas *at) { /* :184-218 */
    for (int lane = 0; lane < g->num_road_lanes; lane++) {
        float speed = g->road_lane_speeds[lane];
        float spawn_prob = (float)(fabs(speed) / 6.0);
        if (rg_rand01(&g->rand_gen) < spawn_prob) {
            float x = speed > 0 ? (-1 * LP_MONSTER_RADIUS) : (g->main_width + LP_MONSTER_RADIUS);
            Entity m;
            entity_init(&m, x, (float)(g->bottom_road_y + lane + 0.5), speed, 0, 2 * LP_MONSTER_RADIUS, LP_MONSTER_RADIUS,
                        LP_CAR);
            choose_random_theme(g, &m, at);
            if (speed < 0) m.rotation = PI_F;
            if (!has_any_collision(g, &m, 0)) {
                fassert(g->num_ents < MAX_ENTS);
                g->ents[g->num_ents++] = m;
            }
        }
    }
    for (int lane = 0; lane < g->num_water_lanes; lane++) {
        float speed = g->water_lane_speeds[lane];
        float spawn_prob = (float)(fabs(speed) / 2.0);
        if (rg_rand01(&g->rand_gen) < spawn_prob) {
            float x = speed > 0 ? (-1 * LP_LOG_RADIUS) : (g->main_width + LP_LOG_RADIUS);
            Entity m;
            entity_init(&m, x, (float)(g->bottom_water_y + lane + 0.5), speed, 0, LP_LOG_RADIUS, LP_LOG_RADIUS, LP_LOG);
            if (!has_any_collision(g, &m, 0)) {
                fassert(g->num_ents < MAX_ENTS);
                g->ents[g->num_ents++] = m;
            }
        }
    }
}

static void leaper_game_reset(Game *g, const or_atlas *at) { /* :119-182 */
    leaper_choose_world_dim(g);
    basic_game_reset(g, at);
    MT *r = &g->rand_gen;
    g->options.center_agent = false;
    Entity *agent = AG(g);
    agent->y = agent->ry;
    float min_car_speed = 0.05f, max_car_speed = 0.2f, min_log_speed = 0.05f, max_log_speed = 0.1f;
    if (g->options.distribution_mode == EasyMode) {
        min_car_speed = 0.03f; max_car_speed = 0.12f; min_log_speed = 0.025f; max_log_speed = 0.075f;
    } else if (g->options.distribution_mode == ExtremeMode) {
        min_car_speed = 0.1f; max_car_speed = 0.3f; min_log_speed = 0.1f; max_log_speed = 0.2f;
    }
    g->bottom_road_y = lp_choose_extra_space(g) + 1;
    int max_diff = g->options.distribution_mode == EasyMode ? 3 : 4;
    int difficulty = rg_randn(r, max_diff + 1);
    int extra_lane_option = g->options.distribution_mode == EasyMode ? 0 : rg_randn(r, 4);
    g->num_road_lanes = difficulty + (extra_lane_option == 2 ? 1 : 0);
    for (int lane = 0; lane < g->num_road_lanes; lane++) {
        /* rand_sign() * randrange(...): g++ evaluates the left operand first (pinned,
         * oracle/ref_harness.cpp ref_leaper_lane_speed) */
        float sgn = lp_rand_sign(g);
        float spd = rg_randrange(r, min_car_speed, max_car_speed);
        g->road_lane_speeds[lane] = sgn * spd;
        fill_elem(g, 0, g->bottom_road_y + lane, g->main_width, 1, LP_ROAD);
    }
    g->bottom_water_y = g->bottom_road_y + g->num_road_lanes + lp_choose_extra_space(g) + 1;
    g->num_water_lanes = difficulty + (extra_lane_option == 3 ? 1 : 0);
    int curr_sign = (int)lp_rand_sign(g);
    for (int lane = 0; lane < g->num_water_lanes; lane++) {
        g->water_lane_speeds[lane] = curr_sign * rg_randrange(r, min_log_speed, max_log_speed);
        curr_sign *= -1;
        fill_elem(g, 0, g->bottom_water_y + lane, g->main_width, 1, LP_WATER);
    }
    g->goal_y = g->bottom_water_y + g->num_water_lanes + 1;
    float mn = min_car_speed < min_log_speed ? min_car_speed : min_log_speed; /* std::min */
    for (int i = 0; (float)i < g->main_width / mn; i++) {
        lp_spawn_entities(g, at);
        step_entities(g);
    }
    add_entity_rxy(g, (float)(g->main_width / 2.0), (float)(g->goal_y - .5), 0, 0, (float)(g->main_width / 2.0), .5f,
                   LP_FINISH_LINE);
}

static void lp_decay_vel(float *vel) { /* :220-226 */
    float vel_sign = lp_sign((float)(1.0 * *vel));
    *vel = (fabsf(*vel) - LP_VEL_DECAY);
    if (*vel < 0) *vel = 0;
    *vel = *vel * vel_sign;
}

static void leaper_game_step(Game *g, const or_atlas *at) { /* :252-288 */
    Entity *agent = AG(g);
    if (agent->image_theme >= 1) agent->image_theme = (agent->image_theme + 1) % LP_NSTEP;
    basic_game_step(g);
    lp_spawn_entities(g, at);
    agent = AG(g);
    bool standing_on_log = false;
    float log_vx = 0.0f;
    float margin = -1 * agent->rx;
    for (int i = 0; i < g->num_ents; i++) {
        Entity *m = &g->ents[i];
        if (m->type == LP_LOG && has_collision(agent, m, margin)) {
            standing_on_log = true;
            log_vx = m->vx;
        }
    }
    if (get_obj(g, (int)agent->x, (int)agent->y) == LP_WATER) {
        if (!standing_on_log && agent->vx == 0 && agent->vy == 0) g->sd_done = true;
    }
    if (standing_on_log) agent->x += log_vx;
    if (is_out_of_bounds(g, agent)) g->sd_done = true;
}

/* ================================================================== Game (game.cpp) */
static void game_reset_dispatch(Game *g, const or_atlas *at) {
    if (g->game_id == GAME_COINRUN) coinrun_game_reset(g, at);
    else if (g->game_id == GAME_BIGFISH) bigfish_game_reset(g, at);
    else if (g->game_id == GAME_MAZE) maze_game_reset(g, at);
    else if (g->game_id == GAME_HEIST) heist_game_reset(g, at);
    else if (g->game_id == GAME_MINER) miner_game_reset(g, at);
    else if (g->game_id == GAME_CLIMBER) climber_game_reset(g, at);
    else if (g->game_id == GAME_LEAPER) leaper_game_reset(g, at);
    else if (g->game_id == GAME_CHASER) chaser_game_reset(g, at);
    else if (g->game_id == GAME_FRUITBOT) fruitbot_game_reset(g, at);
    else if (g->game_id == GAME_DODGEBALL) dodgeball_game_reset(g, at);
    else if (g->game_id == GAME_PLUNDER) plunder_game_reset(g, at);
    else if (g->game_id == GAME_STARPILOT) starpilot_game_reset(g, at);
    else if (g->game_id == GAME_BOSSFIGHT) bossfight_game_reset(g, at);
    else if (g->game_id == GAME_NINJA) ninja_game_reset(g, at);
    else if (g->game_id == GAME_CAVEFLYER) caveflyer_game_reset(g, at);
    else if (g->game_id == GAME_JUMPER) jumper_game_reset(g, at);
    else fatal_msg("game not restated");
}
static void game_step_dispatch(Game *g, const or_atlas *at) {
    if (g->game_id == GAME_COINRUN) coinrun_game_step(g);
    else if (g->game_id == GAME_BIGFISH) bigfish_game_step(g, at);
    else if (g->game_id == GAME_MAZE) maze_game_step(g);
    else if (g->game_id == GAME_HEIST) heist_game_step(g);
    else if (g->game_id == GAME_MINER) miner_game_step(g);
    else if (g->game_id == GAME_CLIMBER) climber_game_step(g);
    else if (g->game_id == GAME_LEAPER) leaper_game_step(g, at);
    else if (g->game_id == GAME_CHASER) chaser_game_step(g);
    else if (g->game_id == GAME_FRUITBOT) fruitbot_game_step(g);
    else if (g->game_id == GAME_DODGEBALL) dodgeball_game_step(g);
    else if (g->game_id == GAME_PLUNDER) plunder_game_step(g, at);
    else if (g->game_id == GAME_STARPILOT) starpilot_game_step(g, at);
    else if (g->game_id == GAME_BOSSFIGHT) bossfight_game_step(g);
    else if (g->game_id == GAME_NINJA) ninja_game_step(g);
    else if (g->game_id == GAME_CAVEFLYER) caveflyer_game_step(g);
    else if (g->game_id == GAME_JUMPER) jumper_game_step(g);
    else fatal_msg("game not restated");
}

static void game_reset(Game *g, const or_atlas *at) { /* game.cpp:109-134 */
    g->reset_count++;
    if (g->episodes_remaining == 0) {
        if (g->options.use_sequential_levels && g->sd_level_complete) {
            g->current_level_seed = (int32_t)((uint32_t)g->current_level_seed + 997u);
        } else {
            g->current_level_seed = rg_randint(&g->level_seed_rand_gen, g->level_seed_low, g->level_seed_high);
        }
        g->episodes_remaining = 1;
    } else {
        g->sd_reward = 0;
        g->sd_done = false;
        g->sd_level_complete = false;
    }
    rg_seed(&g->rand_gen, g->current_level_seed);
    game_reset_dispatch(g, at);
    g->cur_time = 0;
    g->total_reward = 0;
    g->episodes_remaining -= 1;
    g->action = g->default_action;
}

static void render(Game *g, const or_atlas *at);

static void game_step(Game *g, const or_atlas *at) { /* game.cpp:136-171 */
    g->cur_time += 1;
    bool will_force_reset = false;
    if (g->action == -1) {
        g->action = g->default_action;
        will_force_reset = true;
    }
    g->sd_reward = 0;
    g->sd_done = false;
    g->sd_level_complete = false;
    game_step_dispatch(g, at);
    g->sd_done = g->sd_done || will_force_reset || (g->cur_time >= g->timeout);
    g->total_reward += g->sd_reward;
    if (g->sd_reward != 0) {
        g->last_reward_timer = 10;
        g->last_reward = g->sd_reward;
    }
    g->prev_level_seed = g->current_level_seed;
    if (g->sd_done) game_reset(g, at);
    if (g->options.use_sequential_levels && g->sd_level_complete) g->sd_done = false;
    g->episode_done = g->sd_done;
    render(g, at); /* observe(), game.cpp:173-191 */
}

/* ================================================================== Qt raster restatement
 * Qt 5 raster engine semantics for the painter calls the games make
 * (QPainter::fillRect, QPainter::drawImage(QRectF, QImage) with and without
 * setOpacity) onto a 64x64 Format_RGB32 image.  Pinned by tests/golden/qt_raster_*.npz
 * produced by the real Qt 5.9.7 (tools/qt_raster_golden.cpp). */
static int qRound(double d) {
    return d >= 0.0 ? (int)(d + 0.5) : (int)(d - (double)((int)(d - 1)) + 0.5) + (int)(d - 1);
}
static int qFloor(double v) { return (int)floor(v); }
static int qCeil(double v) { return (int)ceil(v); }

static inline uint32_t BYTE_MUL(uint32_t x, uint32_t a) {
    uint32_t t = (x & 0xff00ffu) * a;
    t = (t + ((t >> 8) & 0xff00ffu) + 0x800080u) >> 8;
    t &= 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a;
    x = (x + ((x >> 8) & 0xff00ffu) + 0x800080u);
    x &= 0xff00ff00u;
    return x | t;
}
static inline uint32_t INTERPOLATE_PIXEL_255(uint32_t x, uint32_t a, uint32_t y, uint32_t b) {
    uint32_t t = (x & 0xff00ffu) * a + (y & 0xff00ffu) * b;
    t = (t + ((t >> 8) & 0xff00ffu) + 0x800080u) >> 8;
    t &= 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a + ((y >> 8) & 0xff00ffu) * b;
    x = (x + ((x >> 8) & 0xff00ffu) + 0x800080u);
    x &= 0xff00ff00u;
    return x | t;
}

enum { QFMT_RGB32 = 4, QFMT_ARGB32_PM = 6 };

/* intOpacity of the raster paint state for QPainter::setOpacity(o) */
static int qt_int_opacity(double opacity) {
    if (opacity < 0) opacity = 0;
    if (opacity > 1) opacity = 1;
    return (int)(opacity * 256);
}

/* one pixel write of the scale blit's blender */
static inline void qt_blend(uint32_t *dst, uint32_t src, int fmt, int const_alpha) {
    if (fmt == QFMT_RGB32) {
        if (const_alpha == 256) {
            *dst = src;
        } else {
            uint32_t a = (uint32_t)(const_alpha * 255) >> 8;
            *dst = INTERPOLATE_PIXEL_255(src, a, *dst, 255 - a);
        }
    } else {
        if (const_alpha == 256) {
            *dst = src + BYTE_MUL(*dst, (~src) >> 24);
        } else {
            uint32_t a = (uint32_t)(const_alpha * 255) >> 8;
            uint32_t s = BYTE_MUL(src, a);
            *dst = s + BYTE_MUL(*dst, (~s) >> 24);
        }
    }
}

/* Render target of the painter calls: the 64x64 observation (aliased, the canvas argument the
 * primitives get), or -- render_mode="rgb_array" -- a w x h frame painted with Antialiasing +
 * SmoothPixmapTransform (game.cpp:97-107), where the primitives below switch to qt_smooth_*. */
typedef struct {
    uint32_t *px;
    int w, h;
    bool smooth;
    double *log; /* optional command log (tests replay it through the real Qt) */
    int log_n, log_cap;
} QtTarget;
static QtTarget RT = {NULL, 64, 64, false, NULL, 0, 0};
static void qt_smooth_draw_image(double x, double y, double w, double h, const uint32_t *px, int iw, int ih, int fmt,
                                 bool mirrored, double opacity);
static void qt_smooth_fill_rectf(double x, double y, double w, double h, uint32_t argb);
static void qt_smooth_draw_image_rot(double x, double y, double w, double h, double deg, const uint32_t *px, int iw,
                                     int ih, int fmt, bool mirrored, double opacity);

/* QPainter::drawImage(QRectF target, QImage img) with identity transform
 * (qpaintengine_raster.cpp drawImage -> qt_scale_image_32bit). */
static void qt_scale_image(uint32_t *canvas, double rx, double ry, double rw, double rh, const uint32_t *px, int iw,
                           int ih, int fmt, bool mirrored, double opacity);
static void qt_draw_image(uint32_t *canvas, double rx, double ry, double rw, double rh, const uint32_t *px, int iw,
                          int ih, int fmt, bool mirrored, double opacity) {
    if (rw <= 0 || rh <= 0) return; /* QRectF::isEmpty */
    if (RT.smooth) {
        qt_smooth_draw_image(rx, ry, rw, rh, px, iw, ih, fmt, mirrored, opacity);
        return;
    }
    qt_scale_image(canvas, rx, ry, rw, rh, px, iw, ih, fmt, mirrored, opacity);
}
/* qt_scale_image_32bit on the already-mapped target rect (width/height may be negative) */
static void qt_scale_image(uint32_t *canvas, double rx, double ry, double rw, double rh, const uint32_t *px, int iw,
                           int ih, int fmt, bool mirrored, double opacity) {
    if (iw <= 0 || ih <= 0) return;
    int const_alpha = qt_int_opacity(opacity);
    /* qt_mapRect_non_normalizing(r, identity): QRectF(topLeft, bottomRight) */
    double tl_x = rx, tl_y = ry;
    double br_x = rx + rw, br_y = ry + rh;
    double t_left = tl_x, t_top = tl_y;
    double t_w = br_x - tl_x, t_h = br_y - tl_y;
    double t_right = t_left + t_w, t_bottom = t_top + t_h;
    double sx = t_w / (double)iw;
    double sy = t_h / (double)ih;
    int ix = (int)(65536.0 / sx);
    int iy = (int)(65536.0 / sy);
    int cx1 = 0, cx2 = RES_W, cy1 = 0, cy2 = RES_H;
    int tx1 = qRound(t_left), tx2 = qRound(t_right);
    int ty1 = qRound(t_top), ty2 = qRound(t_bottom);
    if (tx2 < tx1) { int t = tx2; tx2 = tx1; tx1 = t; }
    if (ty2 < ty1) { int t = ty2; ty2 = ty1; ty1 = t; }
    if (tx1 < cx1) tx1 = cx1;
    if (tx2 >= cx2) tx2 = cx2;
    if (tx1 >= tx2) return;
    if (ty1 < cy1) ty1 = cy1;
    if (ty2 >= cy2) ty2 = cy2;
    if (ty1 >= ty2) return;
    int h = ty2 - ty1;
    int w = tx2 - tx1;
    uint32_t basex, srcy;
    /* source rect QRectF(0, 0, iw, ih): a negative scale (a mapped TxScale rect) steps back from
     * its right / bottom edge */
    if (sx < 0) {
        int dstx = qFloor((tx1 + 0.5 - t_right) * ix) + 1;
        basex = (uint32_t)((double)iw * 65536) + (uint32_t)dstx;
    } else {
        int dstx = qCeil((tx1 + 0.5 - t_left) * ix) - 1;
        basex = (uint32_t)(0.0 * 65536) + (uint32_t)dstx;
    }
    if (sy < 0) {
        int dsty = qFloor((ty1 + 0.5 - t_bottom) * iy) + 1;
        srcy = (uint32_t)((double)ih * 65536) + (uint32_t)dsty;
    } else {
        int dsty = qCeil((ty1 + 0.5 - t_top) * iy) - 1;
        srcy = (uint32_t)(0.0 * 65536) + (uint32_t)dsty;
    }
    const int ystart = (int)(srcy >> 16);
    if (ystart >= ih && iy < 0) {
        srcy += iy;
        --h;
    }
    const int xstart = (int)(basex >> 16);
    if (xstart >= iw && ix < 0) {
        basex += ix;
        --w;
    }
    int yend = (int)((srcy + (uint32_t)(iy * (h - 1))) >> 16);
    if (yend < 0 || yend >= ih) --h;
    int xend = (int)((basex + (uint32_t)(ix * (w - 1))) >> 16);
    if (xend < 0 || xend >= iw) --w;
    for (int yy = 0; yy < h; yy++) {
        int srow = (int)(srcy >> 16);
        uint32_t *drow = canvas + (ty1 + yy) * RES_W + tx1;
        uint32_t srcx = basex;
        for (int xx = 0; xx < w; xx++) {
            int scol = (int)(srcx >> 16);
            if (mirrored) scol = iw - 1 - scol;
            qt_blend(&drow[xx], px[srow * iw + scol], fmt, const_alpha);
            srcx += (uint32_t)ix;
        }
        srcy += (uint32_t)iy;
    }
}

/* QTransform::rotate(a) applied to translate(tx, ty) (qtransform.cpp): exact special cases for
 * +-90 / 180 / 270, otherwise qSin/qCos (glibc sin/cos) of deg2rad * a. */
typedef struct { double m11, m12, m21, m22, dx, dy; } QtXform;
static QtXform qt_translate_rotate(double tx, double ty, double a) {
    QtXform t = {1, 0, 0, 1, tx, ty};
    if (a == 0) return t;
    double sina = 0, cosa = 0;
    if (a == 90. || a == -270.) sina = 1;
    else if (a == 270. || a == -90.) sina = -1;
    else if (a == 180.) cosa = -1;
    else {
        const double deg2rad = 0.017453292519943295769;
        double b = deg2rad * a;
        sina = sin(b);
        cosa = cos(b);
    }
    t.m11 = cosa; t.m12 = sina; t.m21 = -sina; t.m22 = cosa;
    return t;
}
static void qt_map(const QtXform *t, double x, double y, double *nx, double *ny) {
    *nx = t->m11 * x + t->m21 * y + t->dx;
    *ny = t->m12 * x + t->m22 * y + t->dy;
}

typedef struct { double x, y, u, v; } QtVtx; /* QTransformImageVertex */

/* qt_transform_image_rasterize (qblendfunctions_p.h) for 32-bit source/destination */
static void qt_xform_rasterize(uint32_t *canvas, const uint32_t *px, int iw, bool mirrored, QtVtx tl, QtVtx bl,
                               QtVtx tr, QtVtx br, int sl, int st, int sw, int sh, double topY, double bottomY,
                               int dudx, int dvdx, int dudy, int dvdy, int u0, int v0, int const_alpha) {
    int fromY = qRound(topY);
    if (fromY < 0) fromY = 0;
    int toY = qRound(bottomY);
    if (toY > RES_H) toY = RES_H;
    if (fromY >= toY) return;
    double leftSlope = (bl.x - tl.x) / (bl.y - tl.y);
    double rightSlope = (br.x - tr.x) / (br.y - tr.y);
    int dx_l = (int)(leftSlope * 0x10000);
    int dx_r = (int)(rightSlope * 0x10000);
    int x_l = (int)((tl.x + (0.5 + fromY - tl.y) * leftSlope + 0.5) * 0x10000);
    int x_r = (int)((tr.x + (0.5 + fromY - tr.y) * rightSlope + 0.5) * 0x10000);
#define SRC_AT(uu, vv) px[(vv) * iw + (mirrored ? iw - 1 - (uu) : (uu))]
    for (int y = fromY; y < toY; ++y) {
        uint32_t *line = canvas + y * RES_W;
        int fromX = x_l >> 16;
        if (fromX < 0) fromX = 0;
        int toX = x_r >> 16;
        if (toX > RES_W) toX = RES_W;
        if (fromX < toX) {
            int x1 = fromX;
            int u = x1 * dudx + y * dudy + u0;
            int v = x1 * dvdx + y * dvdy + v0;
            for (; x1 < toX; ++x1) {
                int uu = u >> 16, vv = v >> 16;
                if (uu >= sl && uu < sl + sw && vv >= st && vv < st + sh) break;
                u += dudx;
                v += dvdx;
            }
            int x2 = toX;
            u = (x2 - 1) * dudx + y * dudy + u0;
            v = (x2 - 1) * dvdx + y * dvdy + v0;
            for (; x2 > x1; --x2) {
                int uu = u >> 16, vv = v >> 16;
                if (uu >= sl && uu < sl + sw && vv >= st && vv < st + sh) break;
                u -= dudx;
                v -= dvdx;
            }
            u = fromX * dudx + y * dudy + u0;
            v = fromX * dvdx + y * dvdy + v0;
            for (int x = fromX; x < toX; ++x) {
                int uu = u >> 16, vv = v >> 16;
                if (x < x1 || x >= x2) { /* clamped ends of the scan line */
                    if (uu < sl) uu = sl;
                    if (uu > sl + sw - 1) uu = sl + sw - 1;
                    if (vv < st) vv = st;
                    if (vv > st + sh - 1) vv = st + sh - 1;
                }
                qt_blend(&line[x], SRC_AT(uu, vv), QFMT_ARGB32_PM, const_alpha);
                u += dudx;
                v += dvdx;
            }
        }
        x_l += dx_l;
        x_r += dx_r;
    }
#undef SRC_AT
}

/* QPainter::drawImage(QRectF target, QImage img) under a rotation (qpaintengine_raster.cpp drawImage ->
 * qTransformFunctions[RGB32][ARGB32PM] -> qt_transform_image, qblendfunctions_p.h) */
static void qt_draw_image_xform(uint32_t *canvas, const QtXform *t, double rx, double ry, double rw, double rh,
                                const uint32_t *px, int iw, int ih, bool mirrored, double opacity) {
    if (iw <= 0 || ih <= 0) return;
    int const_alpha = qt_int_opacity(opacity);
    enum { TopLeft, TopRight, BottomRight, BottomLeft };
    QtVtx v[4];
    double sl = 0, st = 0, sr = iw, sb = ih; /* sourceRect QRectF(0, 0, iw, ih) */
    v[TopLeft].u = v[BottomLeft].u = sl;
    v[TopLeft].v = v[TopRight].v = st;
    v[TopRight].u = v[BottomRight].u = sr;
    v[BottomLeft].v = v[BottomRight].v = sb;
    double right = rx + rw, bottom = ry + rh;
    qt_map(t, rx, ry, &v[TopLeft].x, &v[TopLeft].y);
    qt_map(t, right, ry, &v[TopRight].x, &v[TopRight].y);
    qt_map(t, rx, bottom, &v[BottomLeft].x, &v[BottomLeft].y);
    qt_map(t, right, bottom, &v[BottomRight].x, &v[BottomRight].y);
    int topmost = 0;
    for (int i = 1; i < 4; ++i)
        if (v[i].y < v[topmost].y) topmost = i;
    QtVtx tmp;
    switch (topmost) {
    case 1:
        tmp = v[0];
        for (int i = 0; i < 3; ++i) v[i] = v[i + 1];
        v[3] = tmp;
        break;
    case 2:
        tmp = v[0]; v[0] = v[2]; v[2] = tmp;
        tmp = v[1]; v[1] = v[3]; v[3] = tmp;
        break;
    case 3:
        tmp = v[3];
        for (int i = 3; i > 0; --i) v[i] = v[i - 1];
        v[0] = tmp;
        break;
    }
    double dx1 = v[1].x - v[0].x, dy1 = v[1].y - v[0].y;
    double dx2 = v[3].x - v[0].x, dy2 = v[3].y - v[0].y;
    if (dx1 * dy2 - dx2 * dy1 > 0) {
        tmp = v[1]; v[1] = v[3]; v[3] = tmp;
    }
    QtVtx u = {v[1].x - v[0].x, v[1].y - v[0].y, v[1].u - v[0].u, v[1].v - v[0].v};
    QtVtx w = {v[2].x - v[0].x, v[2].y - v[0].y, v[2].u - v[0].u, v[2].v - v[0].v};
    double det = u.x * w.y - u.y * w.x;
    if (det == 0) return;
    double invDet = 1.0 / det;
    double m11 = (u.u * w.y - u.y * w.u) * invDet;
    double m12 = (u.x * w.u - u.u * w.x) * invDet;
    double m21 = (u.v * w.y - u.y * w.v) * invDet;
    double m22 = (u.x * w.v - u.v * w.x) * invDet;
    double mdx = v[0].u - m11 * v[0].x - m12 * v[0].y;
    double mdy = v[0].v - m21 * v[0].x - m22 * v[0].y;
    int dudx = (int)(m11 * 0x10000), dvdx = (int)(m21 * 0x10000);
    int dudy = (int)(m12 * 0x10000), dvdy = (int)(m22 * 0x10000);
    int u0 = qCeil((0.5 * m11 + 0.5 * m12 + mdx) * 0x10000) - 1;
    int v0 = qCeil((0.5 * m21 + 0.5 * m22 + mdy) * 0x10000) - 1;
    int x1 = qFloor(sl), y1 = qFloor(st), x2 = qCeil(sr), y2 = qCeil(sb);
    int sw = x2 - x1, sh = y2 - y1;
    if (v[1].y < v[3].y) {
        qt_xform_rasterize(canvas, px, iw, mirrored, v[0], v[1], v[0], v[3], x1, y1, sw, sh, v[0].y, v[1].y, dudx, dvdx, dudy, dvdy, u0, v0, const_alpha);
        qt_xform_rasterize(canvas, px, iw, mirrored, v[1], v[2], v[0], v[3], x1, y1, sw, sh, v[1].y, v[3].y, dudx, dvdx, dudy, dvdy, u0, v0, const_alpha);
        qt_xform_rasterize(canvas, px, iw, mirrored, v[1], v[2], v[3], v[2], x1, y1, sw, sh, v[3].y, v[2].y, dudx, dvdx, dudy, dvdy, u0, v0, const_alpha);
    } else {
        qt_xform_rasterize(canvas, px, iw, mirrored, v[0], v[1], v[0], v[3], x1, y1, sw, sh, v[0].y, v[3].y, dudx, dvdx, dudy, dvdy, u0, v0, const_alpha);
        qt_xform_rasterize(canvas, px, iw, mirrored, v[0], v[1], v[3], v[2], x1, y1, sw, sh, v[3].y, v[1].y, dudx, dvdx, dudy, dvdy, u0, v0, const_alpha);
        qt_xform_rasterize(canvas, px, iw, mirrored, v[1], v[2], v[3], v[2], x1, y1, sw, sh, v[1].y, v[2].y, dudx, dvdx, dudy, dvdy, u0, v0, const_alpha);
    }
}

/* qFuzzyIsNull(double) (qglobal.h) */
static bool qt_fuzzy_null(double d) { return fabs(d) <= 0.000000000001; }

/* basic-abstract-game.cpp:908-916: save; translate(center); rotate(deg); drawImage(QRectF(-w/2, -h/2, w, h)).
 * QTransform::type() classifies the matrix with qFuzzyIsNull: a rotation whose sine is within 1e-12
 * of 0 (e.g. rotate(-180) = cos -1, sin -1.2e-16) is a TxScale (or TxTranslate), drawn by
 * qt_scale_image_32bit on qt_mapRect_non_normalizing(r, matrix), whose TxScale map ignores m12/m21. */
static void qt_draw_image_rotated(uint32_t *canvas, double x, double y, double w, double h, double deg,
                                  const uint32_t *px, int iw, int ih, bool mirrored, double opacity) {
    if (RT.smooth) {
        qt_smooth_draw_image_rot(x, y, w, h, deg, px, iw, ih, QFMT_ARGB32_PM, mirrored, opacity);
        return;
    }
    QtXform t = qt_translate_rotate(x + w / 2, y + h / 2, deg);
    double rx = -w / 2, ry = -h / 2;
    if (w <= 0 || h <= 0) return; /* QRectF::isEmpty */
    if (qt_fuzzy_null(t.m12) && qt_fuzzy_null(t.m21)) { /* TxScale / TxTranslate */
        double ax = t.m11 * rx + t.dx, ay = t.m22 * ry + t.dy;
        double bx = t.m11 * (rx + w) + t.dx, by = t.m22 * (ry + h) + t.dy;
        qt_scale_image(canvas, ax, ay, bx - ax, by - ay, px, iw, ih, QFMT_ARGB32_PM, mirrored, opacity);
        return;
    }
    qt_draw_image_xform(canvas, &t, rx, ry, w, h, px, iw, ih, mirrored, opacity);
}

/* QPainter::fillRect(QRect, QColor) with an opaque color on RGB32 */
static void qt_fill_rect_int(uint32_t *canvas, int x, int y, int w, int h, uint32_t argb) {
    if (RT.smooth) { /* QPainter::fillRect(QRect) goes through the QRectF overload */
        qt_smooth_fill_rectf(x, y, w, h, argb);
        return;
    }
    int x1 = x < 0 ? 0 : x, y1 = y < 0 ? 0 : y;
    int x2 = x + w > RES_W ? RES_W : x + w, y2 = y + h > RES_H ? RES_H : y + h;
    for (int yy = y1; yy < y2; yy++)
        for (int xx = x1; xx < x2; xx++) canvas[yy * RES_W + xx] = argb | 0xff000000u;
}

/* QPainter::fillRect(QRectF, QColor) with an opaque colour, no antialiasing, identity transform:
 * the raster engine fills toNormalizedFillRect(r) = qRound of the four edges, normalised
 * (qpaintengine_raster.cpp).  Pinned against Qt 5.9.7 (tests/golden/qt_raster_fill_goldens.npz). */
static void qt_fill_rectf(uint32_t *canvas, double x, double y, double w, double h, uint32_t argb) {
    if (RT.smooth) {
        qt_smooth_fill_rectf(x, y, w, h, argb);
        return;
    }
    int x1 = qRound(x), y1 = qRound(y);
    int x2 = qRound(x + w), y2 = qRound(y + h);
    if (x2 < x1) { int t = x1; x1 = x2; x2 = t; }
    if (y2 < y1) { int t = y1; y1 = y2; y2 = t; }
    qt_fill_rect_int(canvas, x1, y1, x2 - x1, y2 - y1, argb);
}

typedef struct { double x, y, w, h; } RectD;

/* ------------------------------------------------------------------ Antialiasing + SmoothPixmapTransform
 * (render_mode="rgb_array": the 512x512 frame, game.cpp:97-107).  Pinned against the real Qt 5.9.7
 * (tests/test_smooth_pins.py).
 *
 * drawImage(QRectF r, img) and fillRect(QRectF r, colour) both rasterise r as a thick line through
 * QRasterizer::rasterizeLine(mid-left, mid-right, h / w) with antialiasing: the line is clipped
 * to the device grown by half its width, turned into a vertical line, and emitted as <= 3 spans
 * per row (left partial column, full columns, right partial column) with 8-bit coverage
 * (rowHeight x columnCoverage x 255 in 16.16, truncated to a byte -- Qt 5.9 does not subtract a
 * pixel when both edges fall in one column, so such coverages wrap).  Spans go through a
 * 256-span buffer; each flush is one blend call whose adjacent spans share one texture fetch.
 * The fetch is fetchTransformedBilinearARGB32PM for the inverse of translate(1/65536) x scale x
 * translate(r.topLeft): simple / > 8x vertical upscale -> 8-bit bilinear (top/bottom first);
 * downscale -> groups of 4 pixels with 4-bit weights (the SSE2 helper), the rest 8-bit. */
#define QT_SPANBUF 256
typedef struct { int x, len, y, cov; } QtSpan;
static int qt_c_int(double v) { return (int)v; }

/* Qt 5.9.7 qrasterizer.cpp helpers: Q16Dot16 arithmetic, qSafeDivide, qSafeFloatToQ16Dot16 and
 * snapTo26Dot6Grid (read off the library's own machine code: the general branch below matches it
 * bit for bit, tests/test_smooth_pins.py) */
static int qt_fp_safe(double x) { /* qSafeFloatToQ16Dot16 */
    const double v = x * 65536.;
    if (v > 2147483647.0) return 0x7fffffff;
    if (v < -2147483648.0) return -2147483647;
    return (int)v;
}
static double qt_safe_div(double x, double y) { return y == 0 ? (x > 0 ? 1e20 : -1e20) : x / y; }
static int qt_fp_mul(int x, int y) { return (int)(((int64_t)x * (int64_t)y) >> 16); } /* Q16Dot16Multiply */
static void qt_snap26(double *x, double *y) {
    const double ny = floor(*y * 64) * 0.015625, nx = floor(*x * 64) * 0.015625;
    *x = nx;
    *y = ny;
}
/* intersectPixelFP: the area of pixel column x in rows [top, bottom) on the outer side of an edge */
static int qt_intersect_pixel(int x, int top, int bottom, int leftIntersectX, int rightIntersectX, int slope, int invSlope) {
    const int leftX = x << 16, rightX = leftX + 65536;
    const int leftIntersectY = top + qt_fp_mul(slope > 0 ? leftX - leftIntersectX : leftX - rightIntersectX, invSlope);
    const int rightIntersectY = leftIntersectY + invSlope;
    if (leftIntersectX >= leftX && rightIntersectX <= rightX)
        return qt_fp_mul(bottom - top, leftIntersectX - leftX + ((rightIntersectX - leftIntersectX) >> 1));
    if (leftIntersectX >= rightX) return bottom - top;
    if (leftIntersectX >= leftX)
        return (bottom - top) -
               ((((rightX - leftIntersectX) >> 1) * (slope > 0 ? rightIntersectY - top : bottom - rightIntersectY)) >> 16);
    if (rightIntersectX <= leftX) return 0;
    if (rightIntersectX <= rightX)
        return (((rightIntersectX - leftX) >> 1) * (slope > 0 ? bottom - leftIntersectY : leftIntersectY - top)) >> 16;
    if (slope > 0) return (bottom - rightIntersectY) + ((rightIntersectY - leftIntersectY) >> 1);
    return (rightIntersectY - top) + ((leftIntersectY - rightIntersectY) >> 1);
}
static void qt_span_add(QtSpan *out, int *k, int cap, int x, int len, int y, int cov) {
    if (cov && len && *k < cap) {
        QtSpan sp = {x, len, y, cov};
        out[(*k)++] = sp;
    }
}
/* the general (neither horizontal nor vertical) antialiased branch: the line's rectangle (corners
 * snapped to the 26.6 grid) scanned row by row, each row's covered columns as single-pixel spans at
 * the four edges and one full-coverage run between them */
static int qt_aa_general_spans(double pax, double pay, double pbx, double pby, double width, int cw, int ch, QtSpan *out,
                               int cap) {
    if (pay > pby) {
        double t = pax; pax = pbx; pbx = t;
        t = pay; pay = pby; pby = t;
    }
    const double hw = 0.5f * width;
    const double dlx = (pbx - pax) * hw, dly = (pby - pay) * hw;
    const double prx = dly, pry = -dlx; /* perp */
    double tx, ty, lx, ly, rx, ry, bx, by;
    if (pax < pbx) {
        tx = pax + prx; ty = pay + pry; lx = pax - prx; ly = pay - pry;
        rx = pbx + prx; ry = pby + pry; bx = pbx - prx; by = pby - pry;
    } else {
        tx = pax - prx; ty = pay - pry; lx = pbx - prx; ly = pby - pry;
        rx = pax + prx; ry = pay + pry; bx = pbx + prx; by = pby + pry;
    }
    qt_snap26(&tx, &ty);
    qt_snap26(&bx, &by);
    qt_snap26(&lx, &ly);
    qt_snap26(&rx, &ry);
    const double topBound = ty < 0 ? 0 : (ty > ch - 1 ? ch - 1 : ty);
    const double bottomBound = by < 0 ? 0 : (by > ch - 1 ? ch - 1 : by);
    const double tlSlopeInv = qt_safe_div(lx - tx, ly - ty), blSlopeInv = qt_safe_div(bx - lx, by - ly);
    const double trSlopeInv = qt_safe_div(rx - tx, ry - ty), brSlopeInv = qt_safe_div(bx - rx, by - ry);
    const int tlS = qt_fp_safe(tlSlopeInv), trS = qt_fp_safe(trSlopeInv), blS = qt_fp_safe(blSlopeInv), brS = qt_fp_safe(brSlopeInv);
    const int itlS = qt_fp_safe(qt_safe_div(1, tlSlopeInv)), itrS = qt_fp_safe(qt_safe_div(1, trSlopeInv));
    const int iblS = qt_fp_safe(qt_safe_div(1, blSlopeInv)), ibrS = qt_fp_safe(qt_safe_div(1, brSlopeInv));
    const int iTop = (int)topBound, iTopFP = iTop << 16, iLeftFP = ((int)ly) << 16, iRightFP = ((int)ry) << 16;
    const int iBottomFP = ((int)bottomBound) << 16;
    int leftAf = qt_fp_safe(tx + (iTop - ty) * tlSlopeInv), rightAf = qt_fp_safe(tx + (iTop - ty) * trSlopeInv);
    int leftBf = 0, rightBf = 0;
    if (iLeftFP < iTopFP) leftBf = qt_fp_safe(lx + (iTop - ly) * blSlopeInv);
    if (iRightFP < iTopFP) rightBf = qt_fp_safe(rx + (iTop - ry) * brSlopeInv);
    const int yTopFP = qt_fp_safe(ty), yLeftFP = qt_fp_safe(ly), yRightFP = qt_fp_safe(ry), yBottomFP = qt_fp_safe(by);
    int rowTop = iTopFP > yTopFP ? iTopFP : yTopFP;
    int tlAf = leftAf + qt_fp_mul(tlS, rowTop - iTopFP), trAf = rightAf + qt_fp_mul(trS, rowTop - iTopFP);
    int k = 0;
    for (int yFP = iTopFP; yFP <= iBottomFP; yFP += 65536, rowTop = yFP) {
        const int rowBottomLeft = yFP + 65536 < yLeftFP ? yFP + 65536 : yLeftFP;
        const int rowBottomRight = yFP + 65536 < yRightFP ? yFP + 65536 : yRightFP;
        const int rowTopLeft = yFP > yLeftFP ? yFP : yLeftFP, rowTopRight = yFP > yRightFP ? yFP : yRightFP;
        const int rowBottom = yFP + 65536 < yBottomFP ? yFP + 65536 : yBottomFP;
        int tlBf, blAf, trBf, brAf, blBf, brBf;
        if (yFP == iLeftFP) {
            leftBf = qt_fp_safe(lx + ((yFP >> 16) - ly) * blSlopeInv);
            tlBf = leftBf + qt_fp_mul(blS, rowTopLeft - yFP);
            blAf = leftAf + qt_fp_mul(tlS, rowBottomLeft - yFP);
        } else {
            tlBf = leftBf;
            blAf = leftAf + tlS;
        }
        if (yFP == iRightFP) {
            rightBf = qt_fp_safe(rx + ((yFP >> 16) - ry) * brSlopeInv);
            trBf = rightBf + qt_fp_mul(brS, rowTopRight - yFP);
            brAf = rightAf + qt_fp_mul(trS, rowBottomRight - yFP);
        } else {
            trBf = rightBf;
            brAf = rightAf + trS;
        }
        if (yFP == iBottomFP) {
            blBf = leftBf + qt_fp_mul(blS, rowBottom - yFP);
            brBf = rightBf + qt_fp_mul(brS, rowBottom - yFP);
        } else {
            blBf = leftBf + blS;
            brBf = rightBf + brS;
        }
        int leftMin, leftMax, rightMin, rightMax;
        if (yFP < iLeftFP) {
            leftMin = blAf >> 16; leftMax = tlAf >> 16;
        } else if (yFP == iLeftFP) {
            leftMin = (blAf > tlBf ? blAf : tlBf) >> 16; leftMax = (tlAf > blBf ? tlAf : blBf) >> 16;
        } else {
            leftMin = tlBf >> 16; leftMax = blBf >> 16;
        }
        leftMin = leftMin < 0 ? 0 : (leftMin > cw - 1 ? cw - 1 : leftMin);
        leftMax = leftMax < 0 ? 0 : (leftMax > cw - 1 ? cw - 1 : leftMax);
        if (yFP < iRightFP) {
            rightMin = trAf >> 16; rightMax = brAf >> 16;
        } else if (yFP == iRightFP) {
            rightMin = (trAf < brBf ? trAf : brBf) >> 16; rightMax = (brAf < trBf ? brAf : trBf) >> 16;
        } else {
            rightMin = brBf >> 16; rightMax = trBf >> 16;
        }
        rightMin = rightMin < 0 ? 0 : (rightMin > cw - 1 ? cw - 1 : rightMin);
        rightMax = rightMax < 0 ? 0 : (rightMax > cw - 1 ? cw - 1 : rightMax);
        if (leftMax > rightMax) leftMax = rightMax;
        if (rightMin < leftMin) rightMin = leftMin;
        const int rowHeight = rowBottom - rowTop, yi = yFP >> 16;
        int x = leftMin;
        for (; x <= leftMax; x++) {
            int ex = 0;
            if (yFP <= iLeftFP) ex += qt_intersect_pixel(x, rowTop, rowBottomLeft, blAf, tlAf, tlS, itlS);
            if (yFP >= iLeftFP) ex += qt_intersect_pixel(x, rowTopLeft, rowBottom, tlBf, blBf, blS, iblS);
            if (x >= rightMin) {
                if (yFP <= iRightFP) ex += (rowBottomRight - rowTop) - qt_intersect_pixel(x, rowTop, rowBottomRight, trAf, brAf, trS, itrS);
                if (yFP >= iRightFP) ex += (rowBottom - rowTopRight) - qt_intersect_pixel(x, rowTopRight, rowBottom, brBf, trBf, brS, ibrS);
            }
            qt_span_add(out, &k, cap, x, 1, yi, ((255 * (rowHeight - ex)) >> 16) & 0xff);
        }
        if (x < rightMin) {
            qt_span_add(out, &k, cap, x, rightMin - x, yi, ((255 * rowHeight) >> 16) & 0xff);
            x = rightMin;
        }
        for (; x <= rightMax; x++) {
            int ex = 0;
            if (yFP <= iRightFP) ex += (rowBottomRight - rowTop) - qt_intersect_pixel(x, rowTop, rowBottomRight, trAf, brAf, trS, itrS);
            if (yFP >= iRightFP) ex += (rowBottom - rowTopRight) - qt_intersect_pixel(x, rowTopRight, rowBottom, brBf, trBf, brS, ibrS);
            qt_span_add(out, &k, cap, x, 1, yi, ((255 * (rowHeight - ex)) >> 16) & 0xff);
        }
        leftAf += tlS;
        leftBf += blS;
        rightAf += trS;
        rightBf += brS;
        tlAf = leftAf;
        trAf = rightAf;
    }
    return k;
}

/* QRasterizer::rasterizeLine(a, b, width) antialiased (squareCap off); clip = [0, cw) x [0, ch) */
static int qt_aa_line_spans_cap(double ax, double ay, double bx, double by, double width, bool squareCap, int cw, int ch,
                                QtSpan *out, int cap) {
    double pax = ax, pay = ay, pbx = bx, pby = by;
    if ((qt_fuzzy_null(ax - bx) && qt_fuzzy_null(ay - by)) || width == 0) return 0; /* QPointF == is fuzzy */
    if (squareCap) { /* the line grows by half its (absolute) width at both ends */
        const double c = 0.5f * width, dx = pbx - pax, dy = pby - pay;
        pax -= dx * c;
        pay -= dy * c;
        pbx += dx * c;
        pby += dy * c;
    }
    {
        const double offx = fabs(by - ay) * width * 0.5, offy = fabs(bx - ax) * width * 0.5;
        const double cl = 0 - offx, ct = 0 - offy;
        const double cr = cl + ((cw - 1 + 1 + offx) - cl), cb = ct + ((ch - 1 + 1 + offy) - ct);
        const bool in_a = cl <= pax && pax <= cr && ct <= pay && pay <= cb;
        const bool in_b = cl <= pbx && pbx <= cr && ct <= pby && pby <= cb;
        if (!in_a || !in_b) {
            double t1 = 0, t2 = 1;
            const double o[2] = {pax, pay}, d[2] = {pbx - pax, pby - pay};
            const double low[2] = {cl, ct}, high[2] = {cr, cb};
            for (int i = 0; i < 2; i++) {
                if (d[i] == 0) {
                    if (o[i] <= low[i] || o[i] >= high[i]) return 0;
                    continue;
                }
                const double dinv = 1 / d[i];
                double tl = (low[i] - o[i]) * dinv, th = (high[i] - o[i]) * dinv;
                if (tl > th) { const double t = tl; tl = th; th = t; }
                if (t1 < tl) t1 = tl;
                if (t2 > th) t2 = th;
                if (t1 >= t2) return 0;
            }
            const double nax = pax + (pbx - pax) * t1, nay = pay + (pby - pay) * t1;
            const double nbx = pax + (pbx - pax) * t2, nby = pay + (pby - pay) * t2;
            pax = nax; pay = nay; pbx = nbx; pby = nby;
        }
    }
    {
        const double d0x = ax - bx, d0y = ay - by, w0 = d0x * d0x + d0y * d0y;
        const double dx = pax - pbx, dy = pay - pby, ww = dx * dx + dy * dy;
        if (ww == 0) return 0;
        width *= sqrt(w0 / ww);
    }
    if ((int)((pby - pay) * 64.) == 0) { /* horizontal (q26Dot6Compare) -> vertical */
        const double xm = (pax + pbx) * 0.5f, dx = fabs(pbx - pax) * 0.5f, yy = pay, dy = width * dx;
        pax = xm; pay = yy - dy;
        pbx = xm; pby = yy + dy;
        width = 1 / width;
    }
    if ((int)((pbx - pax) * 64.) != 0) return qt_aa_general_spans(pax, pay, pbx, pby, width, cw, ch, out, cap);
    if (pay > pby) {
        double t = pay; pay = pby; pby = t;
        t = pax; pax = pbx; pbx = t;
    }
    const double dy = pby - pay, half = 0.5f * width * dy;
    double left = pax - half, right = pax + half;
    left = left < 0 ? 0 : (left > cw ? cw : left);
    right = right < 0 ? 0 : (right > cw ? cw : right);
    pay = pay < 0 ? 0 : (pay > ch ? ch : pay);
    pby = pby < 0 ? 0 : (pby > ch ? ch : pby);
    if (qt_c_int(left * 64) == qt_c_int(right * 64) || qt_c_int(pay * 64) == qt_c_int(pby * 64)) return 0;
    const int iL = qt_c_int(left), iR = qt_c_int(right);
    const int lw = ((iL + 1) << 16) - qt_c_int(left * 65536.), rw = qt_c_int(right * 65536.) - (iR << 16);
    int cov[3], xs[3], lens[3], n = 1;
    if (iL == iR) {
        cov[0] = lw + rw; /* (sic) */
        xs[0] = iL;
        lens[0] = 1;
    } else {
        cov[0] = lw; xs[0] = iL; lens[0] = 1;
        if (lw == 65536) {
            lens[0] = iR - iL;
        } else if (iR - iL > 1) {
            cov[1] = 65536; xs[1] = iL + 1; lens[1] = iR - iL - 1;
            n++;
        }
        if (rw) {
            cov[n] = rw; xs[n] = iR; lens[n] = 1;
            n++;
        }
    }
    const int iTop = qt_c_int(pay) << 16, iBot = qt_c_int(pby) << 16;
    const int yPa = qt_c_int(pay * 65536.), yPb = qt_c_int(pby * 65536.);
    int k = 0;
    for (int yFP = iTop; yFP <= iBot; yFP += 65536) {
        const int rh = (yFP + 65536 < yPb ? yFP + 65536 : yPb) - (yFP > yPa ? yFP : yPa);
        const int yi = yFP >> 16;
        if (yi > ch - 1) break;
        for (int i = 0; i < n; i++) {
            const int c = (int)((((int64_t)rh * (int64_t)(255 * cov[i])) >> 16) >> 16) & 0xff;
            if (c && lens[i] && k < cap) {
                QtSpan sp = {xs[i], lens[i], yi, c};
                out[k++] = sp;
            }
        }
    }
    return k;
}
static int qt_aa_line_spans(double ax, double ay, double bx, double by, double width, int cw, int ch, QtSpan *out,
                            int cap) {
    return qt_aa_line_spans_cap(ax, ay, bx, by, width, false, cw, ch, out, cap);
}
/* the rect's mid line with width h / w (QRasterPaintEngine::drawImage / fillRect, identity matrix) */
static int qt_aa_rect_spans(double x, double y, double w, double h, int cw, int ch, QtSpan *out, int cap) {
    return qt_aa_line_spans((x + x) * 0.5, (y + (y + h)) * 0.5, ((x + w) + (x + w)) * 0.5, (y + (y + h)) * 0.5, h / w, cw,
                            ch, out, cap);
}

static uint32_t qt_interp_256(uint32_t x, uint32_t a, uint32_t y, uint32_t b) { /* INTERPOLATE_PIXEL_256 */
    uint32_t t = (x & 0xff00ffu) * a + (y & 0xff00ffu) * b;
    t = (t >> 8) & 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a + ((y >> 8) & 0xff00ffu) * b;
    return (x & 0xff00ff00u) | t;
}
/* interpolate_4_pixels (SSE2 form): top/bottom with disty first, then left/right with distx */
static uint32_t qt_interp4_8(uint32_t tl, uint32_t tr, uint32_t bl, uint32_t br, uint32_t dx, uint32_t dy) {
    const uint32_t l = qt_interp_256(tl, 256 - dy, bl, dy), r = qt_interp_256(tr, 256 - dy, br, dy);
    return qt_interp_256(l, 256 - dx, r, dx);
}
/* interpolate_4_pixels_16: 4-bit weights, one rounding */
static uint32_t qt_interp4_4(uint32_t tl, uint32_t tr, uint32_t bl, uint32_t br, uint32_t dx, uint32_t dy) {
    const uint32_t dxy = dx * dy;
    const uint32_t wtl = 16 * 16 - 16 * dx - 16 * dy + dxy, wtr = dx * 16 - dxy, wbl = dy * 16 - dxy, wbr = dxy;
    const uint32_t rb = (tl & 0xff00ffu) * wtl + (tr & 0xff00ffu) * wtr + (bl & 0xff00ffu) * wbl + (br & 0xff00ffu) * wbr;
    const uint32_t ag = ((tl >> 8) & 0xff00ffu) * wtl + ((tr >> 8) & 0xff00ffu) * wtr + ((bl >> 8) & 0xff00ffu) * wbl +
                        ((br >> 8) & 0xff00ffu) * wbr;
    return ((rb >> 8) & 0xff00ffu) | (ag & 0xff00ff00u);
}

/* fetchTransformedBilinearARGB32PM (not tiled) of `len` device pixels from (x, y) for a TxScale
 * inverse (m11, m22, mdx, mdy); `mirrored` reads the horizontally mirrored image */
static void qt_fetch_rotate(uint32_t *out, int len, const uint32_t *px, int iw, int ih, bool mirrored, int fx, int fy,
                            int fdx, int fdy, bool fast);
static void qt_fetch_bilinear_x(uint32_t *out, int x, int y, int len, const uint32_t *px, int iw, int ih, bool mirrored,
                                double m11, double m12, double m21, double m22, double mdx, double mdy) {
#define QT_TEX(r, c) px[(size_t)(r) * iw + (mirrored ? iw - 1 - (c) : (c))]
    const double cx = x + 0.5, cy = y + 0.5;
    const int fdx = (int)(m11 * 65536), fdy = (int)(m12 * 65536);
    int fx = (int)((m21 * cy + m11 * cx + mdx) * 65536) - 32768;
    const int fy = (int)((m22 * cy + m12 * cx + mdy) * 65536) - 32768;
    if (fdy != 0) { /* rotation or shear: 8-bit positions beyond an 8x zoom, else the 4-bit SSE2 helper */
        qt_fetch_rotate(out, len, px, iw, ih, mirrored, fx, fy, fdx, fdy, !(fabs(m11) < 1. / 8. || fabs(m22) < 1. / 8.));
        return;
    }
    int y1 = fy >> 16, y2;
    if (y1 < 0) y1 = y2 = 0;
    else if (y1 >= ih - 1) y1 = y2 = ih - 1;
    else y2 = y1 + 1;
    const uint32_t dy8 = (uint32_t)(fy & 0xffff) >> 8, dy4 = (dy8 + 8) >> 4;
    /* simple upscale on x without mirroring; the 8-bit upscale helper beyond 8x (on y, or on x mirrored); else
     * the downscale helper (also a mirrored upscale on x of less than 8x) */
    const bool down = !(fdx > 0 && fdx <= 65536) && !(fdx < 0 && fdx > -8192) && !(fabs(m22) < 1. / 8.);
    int n = 0;
    while (n < len) { /* leading pixels on a clamped column: vertical interpolation only */
        const int c = fx >> 16;
        if (!(c < 0 || c >= iw - 1)) break;
        const int cc = c < 0 ? 0 : iw - 1;
        out[n++] = qt_interp_256(QT_TEX(y1, cc), 256 - dy8, QT_TEX(y2, cc), dy8);
        fx += fdx;
    }
    int bend = len; /* end of the part that needs no column clamp */
    const int64_t max_fx = (int64_t)(iw - 1) * 65536;
    if (fdx > 0) {
        const int64_t b = n + (max_fx - fx) / fdx;
        if (b < bend) bend = (int)b;
    } else if (fdx < 0) {
        const int64_t b = n + (0 - (int64_t)fx) / fdx;
        if (b < bend) bend = (int)b;
    }
    if (down) { /* the SSE2 loop: 4 pixels at a time, 4-bit weights */
        while (n < bend - 3) {
            for (int q = 0; q < 4; q++, n++) {
                const int c = fx >> 16;
                const uint32_t dx4 = (((uint32_t)(fx & 0xffff) >> 8) + 8) >> 4;
                out[n] = qt_interp4_4(QT_TEX(y1, c), QT_TEX(y1, c + 1), QT_TEX(y2, c), QT_TEX(y2, c + 1), dx4, dy4);
                fx += fdx;
            }
        }
    }
    for (; n < len; n++) { /* 8-bit weights; columns clamped past `bend` */
        int c1 = fx >> 16, c2;
        if (c1 < 0) c1 = c2 = 0;
        else if (c1 >= iw - 1) c1 = c2 = iw - 1;
        else c2 = c1 + 1;
        const uint32_t dx8 = (uint32_t)(fx & 0xffff) >> 8;
        out[n] = qt_interp4_8(QT_TEX(y1, c1), QT_TEX(y1, c2), QT_TEX(y2, c1), QT_TEX(y2, c2), dx8, dy8);
        fx += fdx;
    }
#undef QT_TEX
}
static void qt_fetch_bilinear(uint32_t *out, int x, int y, int len, const uint32_t *px, int iw, int ih, bool mirrored,
                              double m11, double m22, double mdx, double mdy) {
    qt_fetch_bilinear_x(out, x, y, len, px, iw, ih, mirrored, m11, 0.0, 0.0, m22, mdx, mdy);
}
/* fetchTransformedBilinearARGB32PM_rotate_helper (8-bit positions) and _fast_rotate_helper: its
 * possibly clamped lead-in pixels and its tail with 8-bit weights, the unclamped middle in groups of
 * 4 with 4-bit weights (the SSE2 loop), the scalar rest of the middle with 8-bit weights */
static void qt_fetch_rotate(uint32_t *out, int len, const uint32_t *px, int iw, int ih, bool mirrored, int fx, int fy,
                            int fdx, int fdy, bool fast) {
#define QT_TEX(r, c) px[(size_t)(r) * iw + (mirrored ? iw - 1 - (c) : (c))]
#define QT_BOUNDS(n, v1, v2) do { if ((v1) < 0) (v2) = (v1) = 0; else if ((v1) >= (n) - 1) (v2) = (v1) = (n) - 1; else (v2) = (v1) + 1; } while (0)
    int n = 0;
    if (fast) {
        for (; n < len; n++) {
            int x1 = fx >> 16, x2, y1 = fy >> 16, y2;
            QT_BOUNDS(iw, x1, x2);
            QT_BOUNDS(ih, y1, y2);
            if (x1 != x2 && y1 != y2) break;
            out[n] = qt_interp4_8(QT_TEX(y1, x1), QT_TEX(y1, x2), QT_TEX(y2, x1), QT_TEX(y2, x2), (uint32_t)(fx & 0xffff) >> 8,
                                  (uint32_t)(fy & 0xffff) >> 8);
            fx += fdx;
            fy += fdy;
        }
        int64_t bend = len;
        const int64_t max_fx = (int64_t)(iw - 1) * 65536, max_fy = (int64_t)(ih - 1) * 65536;
        if (fdx > 0) { const int64_t b = n + (max_fx - fx) / fdx; if (b < bend) bend = b; }
        else if (fdx < 0) { const int64_t b = n + (0 - (int64_t)fx) / fdx; if (b < bend) bend = b; }
        if (fdy > 0) { const int64_t b = n + (max_fy - fy) / fdy; if (b < bend) bend = b; }
        else if (fdy < 0) { const int64_t b = n + (0 - (int64_t)fy) / fdy; if (b < bend) bend = b; }
        while (n < bend - 3) {
            for (int q = 0; q < 4; q++, n++) {
                const int c = fx >> 16, r = fy >> 16;
                const uint32_t dx4 = (((uint32_t)(fx & 0xffff) >> 8) + 8) >> 4, dy4 = (((uint32_t)(fy & 0xffff) >> 8) + 8) >> 4;
                out[n] = qt_interp4_4(QT_TEX(r, c), QT_TEX(r, c + 1), QT_TEX(r + 1, c), QT_TEX(r + 1, c + 1), dx4, dy4);
                fx += fdx;
                fy += fdy;
            }
        }
        for (; n < bend; n++) {
            const int c = fx >> 16, r = fy >> 16;
            out[n] = qt_interp4_8(QT_TEX(r, c), QT_TEX(r, c + 1), QT_TEX(r + 1, c), QT_TEX(r + 1, c + 1),
                                  (uint32_t)(fx & 0xffff) >> 8, (uint32_t)(fy & 0xffff) >> 8);
            fx += fdx;
            fy += fdy;
        }
    }
    for (; n < len; n++) {
        int x1 = fx >> 16, x2, y1 = fy >> 16, y2;
        QT_BOUNDS(iw, x1, x2);
        QT_BOUNDS(ih, y1, y2);
        out[n] = qt_interp4_8(QT_TEX(y1, x1), QT_TEX(y1, x2), QT_TEX(y2, x1), QT_TEX(y2, x2), (uint32_t)(fx & 0xffff) >> 8,
                              (uint32_t)(fy & 0xffff) >> 8);
        fx += fdx;
        fy += fdy;
    }
#undef QT_BOUNDS
#undef QT_TEX
}

static void qt_log10(double kind, double a, double b, double c, double d, double e, double f, double g, double h, double i) {
    if (!RT.log || RT.log_n + 10 > RT.log_cap) return;
    double *q = RT.log + RT.log_n;
    q[9] = i;
    q[0] = kind; q[1] = a; q[2] = b; q[3] = c; q[4] = d; q[5] = e; q[6] = f; q[7] = g; q[8] = h;
    RT.log_n += 10;
}
static void qt_log(double kind, double a, double b, double c, double d, double e, double f, double g, double h) {
    qt_log10(kind, a, b, c, d, e, f, g, h, 0);
}

/* QPainter::drawImage(QRectF(x, y, w, h), img) under Antialiasing + SmoothPixmapTransform on RT */
static void qt_smooth_draw_image(double x, double y, double w, double h, const uint32_t *px, int iw, int ih, int fmt,
                                 bool mirrored, double opacity) {
    if (iw <= 0 || ih <= 0) return;
    qt_log(0, x, y, w, h, (double)(uintptr_t)px, iw * 65536.0 + ih, fmt * 2 + (mirrored ? 1 : 0), opacity);
    const int ca = qt_int_opacity(opacity);
    if (fmt == QFMT_RGB32 && ca != 256) fatal_msg("rgb_array: translucent RGB32 image");
    if (w == (double)iw && h == (double)ih) {
        /* not stretched (and no transform): the untransformed texture fill of the qRound'ed rect,
         * aliased (QRasterPaintEngine::drawImage -> fillRect_normalized -> blend_untransformed_argb) */
        int x1 = qRound(x), y1 = qRound(y), x2 = qRound(x + w), y2 = qRound(y + h);
        const int xoff = -x1, yoff = -y1; /* -qRound(-dx) with dx = -x */
        const int cov = (255 * ca) >> 8;
        if (x1 < 0) x1 = 0;
        if (y1 < 0) y1 = 0;
        if (x2 > RT.w) x2 = RT.w;
        if (y2 > RT.h) y2 = RT.h;
        if (cov == 0) return;
        for (int yy = y1; yy < y2; yy++) {
            const int sy = yoff + yy;
            if (sy < 0 || sy >= ih) continue;
            for (int xx = x1; xx < x2; xx++) {
                const int sx = xoff + xx;
                if (sx < 0 || sx >= iw) continue;
                uint32_t s = px[(size_t)sy * iw + (mirrored ? iw - 1 - sx : sx)], *dp = RT.px + (size_t)yy * RT.w + xx;
                if (fmt == QFMT_RGB32) {
                    *dp = cov == 255 ? s : INTERPOLATE_PIXEL_255(s, (uint32_t)cov, *dp, 255 - (uint32_t)cov);
                } else if (cov == 255) {
                    if (s >= 0xff000000u) *dp = s;
                    else if (s != 0) *dp = s + BYTE_MUL(*dp, (~s) >> 24);
                } else {
                    s = BYTE_MUL(s, (uint32_t)cov);
                    *dp = s + BYTE_MUL(*dp, (~s) >> 24);
                }
            }
        }
        return;
    }
    /* inverse of (translate(1/65536) * QTransform(sx, 0, 0, sy, x, y)) (QSpanData::setupMatrix) */
    const double sx = w / iw, sy = h / ih;
    const double tdx = (1.0 / 65536) * sx + x, tdy = (1.0 / 65536) * sy + y;
    const double m11 = 1. / sx, m22 = 1. / sy, mdx = -tdx * m11, mdy = -tdy * m22;
    static QtSpan spans[4096];
    static uint32_t src[4096];
    const int ns = qt_aa_rect_spans(x, y, w, h, RT.w, RT.h, spans, 4096);
    for (int i = 0; i < ns;) {
        const int x0 = spans[i].x, yy = spans[i].y;
        int j = i, right = x0 + spans[i].len;
        while (j + 1 < ns && (j + 1) % QT_SPANBUF != 0 && spans[j + 1].y == yy && spans[j + 1].x == right) right += spans[++j].len;
        qt_fetch_bilinear(src, x0, yy, right - x0, px, iw, ih, mirrored, m11, m22, mdx, mdy);
        for (int k = i; k <= j; k++) {
            const int cov = (spans[k].cov * ca) >> 8;
            uint32_t *row = RT.px + (size_t)yy * RT.w;
            for (int xx = spans[k].x; xx < spans[k].x + spans[k].len; xx++) {
                uint32_t s = src[xx - x0], *dp = &row[xx];
                if (fmt == QFMT_RGB32) { /* SourceOver of an opaque image = Source (comp_func_Source) */
                    *dp = cov == 255 ? s : INTERPOLATE_PIXEL_255(s, (uint32_t)cov, *dp, 255 - (uint32_t)cov);
                } else if (cov == 255) { /* comp_func_SourceOver */
                    if (s >= 0xff000000u) *dp = s;
                    else if (s != 0) *dp = s + BYTE_MUL(*dp, (~s) >> 24);
                } else {
                    s = BYTE_MUL(s, (uint32_t)cov);
                    *dp = s + BYTE_MUL(*dp, (~s) >> 24);
                }
            }
        }
        i = j + 1;
    }
}

/* QTransform as the raster engine uses it for a rotated drawImage: the type (QTransform::type()'s
 * qFuzzyIsNull classification), translate / scale / operator* / inverted per type, map per type */
enum { QTX_NONE = 0, QTX_TRANSLATE = 1, QTX_SCALE = 2, QTX_ROTATE = 4, QTX_SHEAR = 8 };
typedef struct { double m11, m12, m21, m22, dx, dy; int type; } QtXf;
static int qtx_classify(const QtXf *t) {
    if (!qt_fuzzy_null(t->m12) || !qt_fuzzy_null(t->m21))
        return qt_fuzzy_null(t->m11 * t->m12 + t->m21 * t->m22) ? QTX_ROTATE : QTX_SHEAR;
    if (!qt_fuzzy_null(t->m11 - 1) || !qt_fuzzy_null(t->m22 - 1)) return QTX_SCALE;
    if (!qt_fuzzy_null(t->dx) || !qt_fuzzy_null(t->dy)) return QTX_TRANSLATE;
    return QTX_NONE;
}
static void qtx_translate(QtXf *t, double dx, double dy) {
    if (dx == 0 && dy == 0) return;
    switch (t->type) {
    case QTX_NONE: t->dx = dx; t->dy = dy; t->type = QTX_TRANSLATE; break;
    case QTX_TRANSLATE: t->dx += dx; t->dy += dy; break;
    case QTX_SCALE: t->dx += dx * t->m11; t->dy += dy * t->m22; break;
    default: t->dx += dx * t->m11 + dy * t->m21; t->dy += dy * t->m22 + dx * t->m12; break;
    }
    t->type = qtx_classify(t);
}
static void qtx_scale(QtXf *t, double sx, double sy) {
    if (sx == 1 && sy == 1) return;
    switch (t->type) {
    case QTX_NONE:
    case QTX_TRANSLATE: t->m11 = sx; t->m22 = sy; break;
    case QTX_ROTATE:
    case QTX_SHEAR: t->m12 *= sx; t->m21 *= sy; /* fall through */
    default: t->m11 *= sx; t->m22 *= sy; break;
    }
    t->type = qtx_classify(t);
}
/* translate(1/65536, 1/65536) * m */
static QtXf qtx_delta_times(const QtXf *o) {
    const double d = 1.0 / 65536;
    QtXf r = {1, 0, 0, 1, 0, 0, QTX_NONE};
    const int type = o->type > QTX_TRANSLATE ? o->type : QTX_TRANSLATE;
    if (type == QTX_TRANSLATE) {
        r.dx = d + o->dx; r.dy = d + o->dy;
    } else if (type == QTX_SCALE) {
        r.m11 = 1 * o->m11; r.m22 = 1 * o->m22;
        r.dx = d * o->m11 + o->dx; r.dy = d * o->m22 + o->dy;
    } else {
        r.m11 = 1 * o->m11 + 0 * o->m21; r.m12 = 1 * o->m12 + 0 * o->m22;
        r.m21 = 0 * o->m11 + 1 * o->m21; r.m22 = 0 * o->m12 + 1 * o->m22;
        r.dx = d * o->m11 + d * o->m21 + o->dx; r.dy = d * o->m12 + d * o->m22 + o->dy;
    }
    r.type = qtx_classify(&r);
    return r;
}
static QtXf qtx_inverted(const QtXf *t) {
    QtXf r = {1, 0, 0, 1, 0, 0, QTX_NONE};
    switch (t->type) {
    case QTX_NONE: break;
    case QTX_TRANSLATE: r.dx = -t->dx; r.dy = -t->dy; break;
    case QTX_SCALE:
        r.m11 = 1. / t->m11; r.m22 = 1. / t->m22;
        r.dx = -t->dx * r.m11; r.dy = -t->dy * r.m22;
        break;
    default: { /* QMatrix::inverted */
        const double dtr = t->m11 * t->m22 - t->m12 * t->m21, dinv = 1.0 / dtr;
        r.m11 = t->m22 * dinv; r.m12 = -t->m12 * dinv; r.m21 = -t->m21 * dinv; r.m22 = t->m11 * dinv;
        r.dx = (t->m21 * t->dy - t->m22 * t->dx) * dinv; r.dy = (t->m12 * t->dx - t->m11 * t->dy) * dinv;
        break;
    }
    }
    r.type = qtx_classify(&r);
    return r;
}
static void qtx_map(const QtXf *t, double x, double y, double *nx, double *ny) {
    switch (t->type) {
    case QTX_NONE: *nx = x; *ny = y; break;
    case QTX_TRANSLATE: *nx = x + t->dx; *ny = y + t->dy; break;
    case QTX_SCALE: *nx = t->m11 * x + t->dx; *ny = t->m22 * y + t->dy; break;
    default: *nx = t->m11 * x + t->m21 * y + t->dx; *ny = t->m12 * x + t->m22 * y + t->dy; break;
    }
}

/* fetchTransformedBilinearARGB32PM's floating-point path (an affine matrix outside fast_matrix) */
static void qt_fetch_bilinear_float(uint32_t *out, int x, int y, int len, const uint32_t *px, int iw, int ih, bool mirrored,
                                    const QtXf *m) {
#define QT_TEX(r, c) px[(size_t)(r) * iw + (mirrored ? iw - 1 - (c) : (c))]
    const double cx = x + 0.5, cy = y + 0.5;
    double fx = m->m21 * cy + m->m11 * cx + m->dx, fy = m->m22 * cy + m->m12 * cx + m->dy;
    double fw = 0 * cy + 0 * cx + 1;
    for (int n = 0; n < len; n++) {
        const double iwv = fw == 0 ? 1 : 1 / fw;
        const double pxv = fx * iwv - 0.5, pyv = fy * iwv - 0.5;
        int x1 = (int)pxv - (pxv < 0), x2, y1 = (int)pyv - (pyv < 0), y2;
        const int distx = (int)((pxv - x1) * 256), disty = (int)((pyv - y1) * 256);
        if (x1 < 0) x1 = x2 = 0;
        else if (x1 >= iw - 1) x1 = x2 = iw - 1;
        else x2 = x1 + 1;
        if (y1 < 0) y1 = y2 = 0;
        else if (y1 >= ih - 1) y1 = y2 = ih - 1;
        else y2 = y1 + 1;
        out[n] = qt_interp4_8(QT_TEX(y1, x1), QT_TEX(y1, x2), QT_TEX(y2, x1), QT_TEX(y2, x2), (uint32_t)distx, (uint32_t)disty);
        fx += m->m11;
        fy += m->m12;
        fw += 0;
        if (!fw) fw += 0;
    }
#undef QT_TEX
}

/* QPainter::translate(tx, ty); rotate(deg); drawImage(QRectF(rx, ry, w, h), img) under Antialiasing +
 * SmoothPixmapTransform (basic-abstract-game.cpp:908-916 at RENDER_RES): QRasterPaintEngine::drawImage's
 * transformed branch -- the rect's mid line mapped by the matrix and rasterised with width h / w
 * (tx_noshear), filled with the bilinear texture of the inverse of translate(1/65536) * (matrix *
 * translate(rx, ry) * scale(w / iw, h / ih)) */
static void qt_smooth_draw_image_rot(double x, double y, double w, double h, double deg, const uint32_t *px, int iw,
                                     int ih, int fmt, bool mirrored, double opacity) {
    if (iw <= 0 || ih <= 0 || w <= 0 || h <= 0) return;
    qt_log10(2, x, y, w, h, (double)(uintptr_t)px, iw * 65536.0 + ih, fmt * 2 + (mirrored ? 1 : 0), opacity, deg);
    const double tx = x + w / 2, ty = y + h / 2, rx = -w / 2, ry = -h / 2;
    const int ca = qt_int_opacity(opacity);
    if (fmt == QFMT_RGB32 && ca != 256) fatal_msg("rgb_array: translucent RGB32 image");
    const QtXform r0 = qt_translate_rotate(tx, ty, deg);
    QtXf m = {r0.m11, r0.m12, r0.m21, r0.m22, r0.dx, r0.dy, 0};
    m.type = qtx_classify(&m);
    double ax, ay, bx, by;
    qtx_map(&m, (rx + rx) * 0.5f, (ry + (ry + h)) * 0.5f, &ax, &ay);
    qtx_map(&m, ((rx + w) + (rx + w)) * 0.5f, (ry + (ry + h)) * 0.5f, &bx, &by);
    QtXf copy = m;
    qtx_translate(&copy, rx, ry);
    qtx_scale(&copy, w / iw, h / ih);
    const QtXf dm = qtx_delta_times(&copy);
    const QtXf inv = qtx_inverted(&dm);
    /* QSpanData::setupMatrix: fixed-point stepping only while it cannot overflow */
    const bool fast = inv.m11 * inv.m11 + inv.m21 * inv.m21 < 1e4 && inv.m12 * inv.m12 + inv.m22 * inv.m22 < 1e4 &&
                      fabs(inv.dx) < 1e4 && fabs(inv.dy) < 1e4;
    static QtSpan spans[8192];
    static uint32_t src[4096];
    const int ns = qt_aa_line_spans(ax, ay, bx, by, h / w, RT.w, RT.h, spans, 8192);
    for (int i = 0; i < ns;) {
        const int x0 = spans[i].x, yy = spans[i].y;
        int j = i, right = x0 + spans[i].len;
        while (j + 1 < ns && (j + 1) % QT_SPANBUF != 0 && spans[j + 1].y == yy && spans[j + 1].x == right) right += spans[++j].len;
        if (fast) qt_fetch_bilinear_x(src, x0, yy, right - x0, px, iw, ih, mirrored, inv.m11, inv.m12, inv.m21, inv.m22, inv.dx, inv.dy);
        else qt_fetch_bilinear_float(src, x0, yy, right - x0, px, iw, ih, mirrored, &inv);
        for (int k = i; k <= j; k++) {
            const int cov = (spans[k].cov * ca) >> 8;
            uint32_t *row = RT.px + (size_t)yy * RT.w;
            for (int xx = spans[k].x; xx < spans[k].x + spans[k].len; xx++) {
                uint32_t s = src[xx - x0], *dp = &row[xx];
                if (fmt == QFMT_RGB32) {
                    *dp = cov == 255 ? s : INTERPOLATE_PIXEL_255(s, (uint32_t)cov, *dp, 255 - (uint32_t)cov);
                } else if (cov == 255) {
                    if (s >= 0xff000000u) *dp = s;
                    else if (s != 0) *dp = s + BYTE_MUL(*dp, (~s) >> 24);
                } else {
                    s = BYTE_MUL(s, (uint32_t)cov);
                    *dp = s + BYTE_MUL(*dp, (~s) >> 24);
                }
            }
        }
        i = j + 1;
    }
}

/* QPainter::fillRect(QRectF, QColor) with an opaque colour under Antialiasing on RT (blend_color_argb,
 * SourceOver of an opaque colour = Source) */
static void qt_smooth_fill_rectf(double x, double y, double w, double h, uint32_t argb) {
    if ((argb >> 24) != 255) fatal_msg("rgb_array: translucent fill");
    if (w < 0) { x += w; w = -w; } /* QRectF::normalized */
    if (h < 0) { y += h; h = -h; }
    if (w <= 0 || h <= 0) return;
    qt_log(1, x, y, w, h, (double)argb, 0, 0, 1);
    static QtSpan spans[4096];
    const int ns = qt_aa_rect_spans(x, y, w, h, RT.w, RT.h, spans, 4096);
    for (int k = 0; k < ns; k++) {
        uint32_t *row = RT.px + (size_t)spans[k].y * RT.w;
        const uint32_t cov = (uint32_t)spans[k].cov;
        const uint32_t c = cov == 255 ? argb : BYTE_MUL(argb, cov);
        for (int xx = spans[k].x; xx < spans[k].x + spans[k].len; xx++)
            row[xx] = cov == 255 ? c : c + BYTE_MUL(row[xx], 255 - cov);
    }
}

/* ================================================================== AssetGen (assetgen.cpp) and the
 * Qt 5.9 raster paths it paints with, on a canvas of any size: fillRect(QRectF, QColor) (opaque,
 * alpha 200 SourceOver, transparent Source), drawEllipse(QRectF) with a solid brush (the
 * non-antialiased path filler: QBezier flattening -> QOutlineMapper 26.6 outline -> QRasterizer's
 * scan converter) and a 1-px pen (QCosmeticStroker, aliased).  Pinned against the reference's own
 * assetgen.cpp compiled with the real Qt 5.9.7 of this image (oracle/_ref/libref_qt.so,
 * tests/test_assetgen_pins.py). */
typedef struct {
    uint32_t *px;
    int w, h;
    int fmt;    /* QFMT_RGB32 (backgrounds) or QFMT_ARGB32 (generated sprites, not premultiplied) */
    int source; /* CompositionMode_Source (paint_shape_resource) instead of SourceOver */
} AgCanvas;
enum { QFMT_ARGB32 = 5 };

static uint32_t qt_div_65535(uint32_t x) { return (x + (x >> 16) + 0x8000u) >> 16; }
static uint32_t qt_div_257(uint32_t x) { x += 128u; return (x - (x >> 8)) >> 8; } /* QRgba64::div_257 */
/* qPremultiply(QColor::rgba64()).toArgb32(): the raster engine's solid colour (QSpanData::setup) */
static uint32_t qt_solid_premul(uint32_t argb) {
    const uint32_t a = (argb >> 24) * 257u;
    uint32_t out = qt_div_257(a) << 24;
    for (int s = 16; s >= 0; s -= 8) out |= qt_div_257(qt_div_65535(((argb >> s) & 255u) * 257u * a)) << s;
    return out;
}
/* qUnpremultiply (qrgb.h / qdrawhelper: ARGB32PM -> ARGB32 store) */
static uint32_t qt_unpremultiply(uint32_t p) {
    const uint32_t a = p >> 24;
    if (a == 255) return p;
    if (a == 0) return 0;
    const uint32_t inv = (255u * 0x10000u + a / 2) / a; /* qt_inv_premul_factor */
    uint32_t r = (((p >> 16) & 255u) * inv + 0x8000u) >> 16;
    uint32_t g = (((p >> 8) & 255u) * inv + 0x8000u) >> 16;
    uint32_t b = ((p & 255u) * inv + 0x8000u) >> 16;
    return (a << 24) | (r << 16) | (g << 8) | b;
}

/* one coverage-255 span [x0, x1) of row y in the solid colour `pm` (premultiplied) */
static void ag_span(AgCanvas *c, int y, int x0, int x1, uint32_t pm) {
    if (y < 0 || y >= c->h) return;
    if (x0 < 0) x0 = 0;
    if (x1 > c->w) x1 = c->w;
    uint32_t *row = c->px + (size_t)y * c->w;
    const uint32_t a = pm >> 24;
    for (int x = x0; x < x1; x++) {
        if (c->source || a == 255) {
            row[x] = c->fmt == QFMT_ARGB32 ? qt_unpremultiply(pm) : (pm | 0xff000000u);
        } else {
            /* comp_func_solid_SourceOver on the premultiplied destination (ARGB32 is fetched
             * premultiplied and stored back unpremultiplied) */
            uint32_t d = row[x];
            if (c->fmt == QFMT_ARGB32) {
                const uint32_t da = d >> 24;
                d = da == 255 ? d : (da == 0 ? 0 : BYTE_MUL(d | 0xff000000u, da) & 0x00ffffffu) | (da << 24);
            }
            d = pm + BYTE_MUL(d, 255u - a);
            row[x] = c->fmt == QFMT_ARGB32 ? qt_unpremultiply(d) : d;
        }
    }
}

/* QPainter::fillRect(QRectF, QColor): QRasterPaintEngine::fillRect -> fillRect_normalized of
 * toNormalizedFillRect (qRound of the edges); a fully transparent colour under SourceOver paints
 * nothing */
static void ag_fill_rectf(AgCanvas *c, double x, double y, double w, double h, uint32_t argb) {
    const uint32_t pm = qt_solid_premul(argb);
    if ((pm >> 24) == 0 && !c->source) return;
    int x1 = qRound(x), y1 = qRound(y), x2 = qRound(x + w), y2 = qRound(y + h);
    if (x2 < x1) { int t = x1; x1 = x2; x2 = t; }
    if (y2 < y1) { int t = y1; y1 = y2; y2 = t; }
    if (y1 < 0) y1 = 0;
    if (y2 > c->h) y2 = c->h;
    if (c->fmt == QFMT_ARGB32 && (c->source || (pm >> 24) == 255)) {
        /* qt_rectfill_nonpremul_argb32: the premultiplied QRgba64 unpremultiplied at 16 bits */
        const uint32_t a16 = (argb >> 24) * 257u;
        uint32_t v = argb;
        if (a16 != 0 && a16 != 65535) {
            v = (argb >> 24) << 24;
            for (int sh = 16; sh >= 0; sh -= 8) {
                const uint32_t p16 = qt_div_65535(((argb >> sh) & 255u) * 257u * a16);
                v |= qt_div_257((p16 * 65535u + a16 / 2) / a16) << sh;
            }
        } else if (a16 == 0) {
            v = 0;
        }
        if (x1 < 0) x1 = 0;
        if (x2 > c->w) x2 = c->w;
        for (int yy = y1; yy < y2; yy++)
            for (int xx = x1; xx < x2; xx++) c->px[(size_t)yy * c->w + xx] = v;
        return;
    }
    for (int yy = y1; yy < y2; yy++) ag_span(c, yy, x1, x2, pm);
}

/* ---- drawEllipse(QRectF): QPaintEngineEx::drawEllipse -> qt_curves_for_arc(rect, 0, -360) */
#define QT_PATH_KAPPA 0.5522847498
typedef struct { double x, y; } PtD;
static void qt_ellipse_points(double x, double y, double w, double h, PtD pts[13]) {
    const double w2 = w / 2, w2k = w2 * QT_PATH_KAPPA, h2 = h / 2, h2k = h2 * QT_PATH_KAPPA;
    const PtD p[13] = {{x + w, y + h2},
                       {x + w, y + h2 + h2k}, {x + w2 + w2k, y + h}, {x + w2, y + h},
                       {x + w2 - w2k, y + h}, {x, y + h2 + h2k}, {x, y + h2},
                       {x, y + h2 - h2k}, {x + w2 - w2k, y}, {x + w2, y},
                       {x + w2 + w2k, y}, {x + w, y + h2 - h2k}, {x + w, y + h2}};
    memcpy(pts, p, sizeof(p));
}

/* QBezier::split (qbezier_p.h), alias-safe in the order Qt writes */
typedef struct { double x1, y1, x2, y2, x3, y3, x4, y4; } QBez;
static void qbez_split(const QBez *b, QBez *first, QBez *second) {
    const QBez s = *b;
    double c = (s.x2 + s.x3) * .5;
    first->x2 = (s.x1 + s.x2) * .5;
    second->x3 = (s.x3 + s.x4) * .5;
    first->x1 = s.x1;
    second->x4 = s.x4;
    first->x3 = (first->x2 + c) * .5;
    second->x2 = (second->x3 + c) * .5;
    first->x4 = second->x1 = (first->x3 + second->x2) * .5;
    c = (s.y2 + s.y3) * .5;
    first->y2 = (s.y1 + s.y2) * .5;
    second->y3 = (s.y3 + s.y4) * .5;
    first->y1 = s.y1;
    second->y4 = s.y4;
    first->y3 = (first->y2 + c) * .5;
    second->y2 = (second->y3 + c) * .5;
    first->y4 = second->y1 = (first->y3 + second->y2) * .5;
}
/* QBezier::addToPolygon(threshold): appends the end points of the flattened pieces */
static int qbez_flatten(QBez b0, double threshold, PtD *out, int n) {
    QBez st[10];
    int lv[10];
    st[0] = b0;
    lv[0] = 9;
    int top = 0;
    while (top >= 0) {
        QBez *b = &st[top];
        double y4y1 = b->y4 - b->y1, x4x1 = b->x4 - b->x1;
        double l = fabs(x4x1) + fabs(y4y1), d;
        if (l > 1.) {
            d = fabs((x4x1) * (b->y1 - b->y2) - (y4y1) * (b->x1 - b->x2)) +
                fabs((x4x1) * (b->y1 - b->y3) - (y4y1) * (b->x1 - b->x3));
        } else {
            d = fabs(b->x1 - b->x2) + fabs(b->y1 - b->y2) + fabs(b->x1 - b->x3) + fabs(b->y1 - b->y3);
            l = 1.;
        }
        if (d < threshold * l || lv[top] == 0) {
            out[n].x = b->x4;
            out[n].y = b->y4;
            n++;
            top--;
        } else {
            QBez first, second;
            qbez_split(b, &first, &second);
            st[top] = second;
            st[top + 1] = first;
            lv[top + 1] = --lv[top];
            top++;
        }
    }
    return n;
}

/* QRasterizer / QScanConverter (non-antialiased fill of a 26.6 outline, no legacy rounding) */
typedef struct { int x, delta, top, bottom, winding; } ScanLine;
static int64_t q16mul(int64_t a, int64_t b) { return (a * b) >> 16; }
#define AG_MAX_LINES 512
typedef struct {
    int top, bottom, leftFP, rightFP;
    ScanLine lines[AG_MAX_LINES];
    int n;
} ScanConv;
static void sc_add(ScanConv *s, int x, int delta, int top, int bottom, int winding) {
    if (s->n < AG_MAX_LINES) {
        ScanLine l = {x, delta, top, bottom, winding};
        s->lines[s->n++] = l;
    }
}
/* QScanConverter::clip: true when the whole line was replaced by edge lines */
static bool sc_clip(ScanConv *s, int *xFP, int *iTop, int *iBottom, int slopeFP, int edgeFP, int winding) {
    const bool right = edgeFP == s->rightFP;
    if (*xFP == edgeFP) {
        if ((slopeFP > 0) ^ right) return false;
        sc_add(s, edgeFP, 0, *iTop, *iBottom, winding);
        return true;
    }
    const int lastFP = *xFP + slopeFP * (*iBottom - *iTop);
    if (lastFP == edgeFP) {
        if ((slopeFP < 0) ^ right) return false;
        sc_add(s, edgeFP, 0, *iTop, *iBottom, winding);
        return true;
    }
    if ((lastFP < edgeFP) ^ (*xFP < edgeFP)) {
        const int deltaY = (int)((edgeFP - *xFP) / (slopeFP / 65536.));
        if ((*xFP < edgeFP) ^ right) {
            const int iHeight = (deltaY + 1) >> 16;
            const int iMiddle = *iTop + iHeight;
            sc_add(s, edgeFP, 0, *iTop, iMiddle, winding);
            if (iMiddle != *iBottom) {
                *xFP += slopeFP * (iHeight + 1);
                *iTop = iMiddle + 1;
            } else {
                return true;
            }
        } else {
            const int iHeight = deltaY >> 16;
            const int iMiddle = *iTop + iHeight;
            if (iMiddle != *iBottom) {
                sc_add(s, edgeFP, 0, iMiddle + 1, *iBottom, winding);
                *iBottom = iMiddle;
            }
        }
        return false;
    } else if ((*xFP < edgeFP) ^ right) {
        sc_add(s, edgeFP, 0, *iTop, *iBottom, winding);
        return true;
    }
    return false;
}
static void sc_merge_line(ScanConv *s, int ax, int ay, int bx, int by) {
    int winding = 1;
    if (ay > by) {
        int t = ax; ax = bx; bx = t;
        t = ay; ay = by; by = t;
        winding = -1;
    }
    int iTop = (ay + 32) >> 6, iBottom = (by - 32) >> 6;
    if (iTop < s->top) iTop = s->top;
    if (iBottom > s->bottom) iBottom = s->bottom;
    if (iTop > iBottom) return;
    const int aFP = 65536 / 2 + ax * 1024;
    if (bx == ax) {
        int x = aFP < s->leftFP ? s->leftFP : (aFP > s->rightFP ? s->rightFP : aFP);
        sc_add(s, x, 0, iTop, iBottom, winding);
        return;
    }
    const double slope = (double)(bx - ax) / (double)(by - ay);
    const int slopeFP = (int)(slope * 65536.);
    int xFP = aFP + (int)q16mul(slopeFP, (int64_t)iTop * 65536 + 65536 / 2 - (int64_t)ay * 1024);
    if (sc_clip(s, &xFP, &iTop, &iBottom, slopeFP, s->leftFP, winding)) return;
    if (sc_clip(s, &xFP, &iTop, &iBottom, slopeFP, s->rightFP, winding)) return;
    sc_add(s, xFP, slopeFP, iTop, iBottom, winding);
}
/* emit the spans of every row (winding fill of the ellipse's single convex contour: the rows'
 * crossings sorted by x, spans where the winding is non-zero) */
static void sc_end(ScanConv *s, AgCanvas *c, uint32_t pm) {
    for (int y = s->top; y <= s->bottom; y++) {
        int xs[AG_MAX_LINES], ws[AG_MAX_LINES], k = 0;
        for (int i = 0; i < s->n; i++) {
            const ScanLine *l = &s->lines[i];
            if (y < l->top || y > l->bottom) continue;
            const int x = (int)(((int64_t)l->x + (int64_t)l->delta * (y - l->top)) >> 16);
            int j = k++;
            while (j > 0 && xs[j - 1] > x) { xs[j] = xs[j - 1]; ws[j] = ws[j - 1]; j--; }
            xs[j] = x;
            ws[j] = l->winding;
        }
        int x = 0, wind = 0;
        for (int i = 0; i < k; i++) {
            if (wind != 0 && xs[i] > x) ag_span(c, y, x, xs[i], pm);
            x = xs[i];
            wind += ws[i];
        }
    }
}
/* QOutlineMapper's qreal_to_fixed_26_6 rounds (pinned: truncating here mismatches Qt) */
static int qt_fixed_26_6(double v) { return qRound(v * 64); }

static void ag_fill_ellipse(AgCanvas *c, const PtD pts[13], uint32_t pm) {
    PtD poly[4 * 1100];
    int n = 0;
    poly[n++] = pts[0];
    for (int k = 0; k < 4; k++) {
        QBez b = {poly[n - 1].x, poly[n - 1].y, pts[3 * k + 1].x, pts[3 * k + 1].y, pts[3 * k + 2].x, pts[3 * k + 2].y,
                  pts[3 * k + 3].x, pts[3 * k + 3].y};
        n = qbez_flatten(b, 0.25, poly, n);
    }
    /* closeSubpath: the end point equals the start, nothing added */
    int fx[4 * 1100], fy[4 * 1100];
    int miny = 0x7fffffff, maxy = -0x7fffffff;
    for (int i = 0; i < n; i++) {
        fx[i] = qt_fixed_26_6(poly[i].x);
        fy[i] = qt_fixed_26_6(poly[i].y);
        if (fy[i] < miny) miny = fy[i];
        if (fy[i] > maxy) maxy = fy[i];
    }
    ScanConv *s = (ScanConv *)malloc(sizeof(ScanConv));
    s->top = (miny + 32) >> 6;
    if (s->top < 0) s->top = 0;
    s->bottom = (maxy - 32) >> 6;
    if (s->bottom > c->h - 1) s->bottom = c->h - 1;
    s->leftFP = 0;
    s->rightFP = c->w * 65536; /* IntToQ16Dot16(clip right + 1) */
    s->n = 0;
    if (s->top <= s->bottom) {
        for (int i = 0; i + 1 < n; i++) sc_merge_line(s, fx[i], fy[i], fx[i + 1], fy[i + 1]);
        sc_end(s, c, pm);
    }
    free(s);
}

/* ---- QCosmeticStroker (aliased, solid, no dash) for a 1-px pen (qcosmeticstroker.cpp) */
enum { CS_T2B = 1, CS_B2T = 2, CS_L2R = 4, CS_R2L = 8, CS_VMASK = 3, CS_HMASK = 12 };
enum { CS_NOCAPS = 0, CS_CAPBEGIN = 1, CS_CAPEND = 2 };
#define CS_MAXSUB 6 /* renderCubic's maxSubDivisions */
typedef struct {
    AgCanvas *c;
    uint32_t pm;
    double xmin, xmax, ymin, ymax;
    int lastx, lasty, lastDir;
    bool lastAxisAligned;
} CStroker;
#define CS_INT_MIN (-2147483647 - 1)
static int toF26Dot6(double v) { return (int)(v * 64.); } /* the stroker truncates */
static int F16Dot16FixedDiv(int x, int y) {
    if (abs(x) > 0x7fff) return (int)(((int64_t)x * 65536) / y);
    return x * 65536 / y;
}
static int swapCaps(int caps) { return ((caps & 1) << 1) | ((caps & 2) >> 1); }
static void capAdjust(int caps, int *x1, int *x2, int *y, int yinc) {
    if (caps & CS_CAPBEGIN) {
        *x1 -= 32;
        *y -= yinc >> 1;
    }
    if (caps & CS_CAPEND) *x2 += 32;
}
static void cs_pixel(CStroker *s, int x, int y) {
    if (x < 0 || x >= s->c->w || y < 0 || y >= s->c->h) return;
    ag_span(s->c, y, x, x + 1, s->pm);
}
/* QCosmeticStroker::clipLine: true = completely outside */
static bool cs_clip(CStroker *s, double *x1, double *y1, double *x2, double *y2) {
    if (*x1 < s->xmin) {
        if (*x2 <= s->xmin) goto clipped;
        *y1 += (*y2 - *y1) / (*x2 - *x1) * (s->xmin - *x1);
        *x1 = s->xmin;
    } else if (*x1 > s->xmax) {
        if (*x2 >= s->xmax) goto clipped;
        *y1 += (*y2 - *y1) / (*x2 - *x1) * (s->xmax - *x1);
        *x1 = s->xmax;
    }
    if (*x2 < s->xmin) {
        s->lastx = CS_INT_MIN;
        *y2 += (*y2 - *y1) / (*x2 - *x1) * (s->xmin - *x2);
        *x2 = s->xmin;
    } else if (*x2 > s->xmax) {
        s->lastx = CS_INT_MIN;
        *y2 += (*y2 - *y1) / (*x2 - *x1) * (s->xmax - *x2);
        *x2 = s->xmax;
    }
    if (*y1 < s->ymin) {
        if (*y2 <= s->ymin) goto clipped;
        *x1 += (*x2 - *x1) / (*y2 - *y1) * (s->ymin - *y1);
        *y1 = s->ymin;
    } else if (*y1 > s->ymax) {
        if (*y2 >= s->ymax) goto clipped;
        *x1 += (*x2 - *x1) / (*y2 - *y1) * (s->ymax - *y1);
        *y1 = s->ymax;
    }
    if (*y2 < s->ymin) {
        s->lastx = CS_INT_MIN;
        *x2 += (*x2 - *x1) / (*y2 - *y1) * (s->ymin - *y2);
        *y2 = s->ymin;
    } else if (*y2 > s->ymax) {
        s->lastx = CS_INT_MIN;
        *x2 += (*x2 - *x1) / (*y2 - *y1) * (s->ymax - *y2);
        *y2 = s->ymax;
    }
    return false;
clipped:
    s->lastx = CS_INT_MIN;
    return true;
}
/* drawLine<drawPixel, NoDasher>, both branches in one routine: `vert` = major axis y.  a1 / a2 are
 * the major coordinates (26.6), b1 / b2 the minor ones.  A direction reversal (lastDir ^ mask == dir)
 * caps the path-start end of the new segment -- CapEnd when it is drawn swapped, CapBegin otherwise --
 * and a CapBegin whose rounding lands one major pixel before lastPixel is rounded back; the
 * same-direction dropout test reads |dx| <= 1 && |dy| > 1 in both branches.  Checked bit-exact against
 * Qt 5.9.7 on 200,000 random closed polylines and 200,000 ellipses (tests/test_assetgen_pins.py). */
static void cs_run(CStroker *s, bool vert, int a1, int b1, int a2, int b2, int caps) {
    int dir = vert ? CS_T2B : CS_L2R;
    bool swapped = false;
    if (a1 > a2) {
        swapped = true;
        int t = a1; a1 = a2; a2 = t;
        t = b1; b1 = b2; b2 = t;
        caps = swapCaps(caps);
        dir = vert ? CS_B2T : CS_R2L;
    }
    const int binc = F16Dot16FixedDiv(b2 - b1, a2 - a1);
    int b = b1 * 1024;
    const int mask = vert ? CS_VMASK : CS_HMASK;
    /* a reversal caps the segment's path-start end (CapEnd when drawn swapped, CapBegin otherwise) */
    if ((s->lastDir ^ mask) == dir) caps |= swapped ? CS_CAPEND : CS_CAPBEGIN;
    const int round = (binc > 0) ? 32 : 0;
    capAdjust(caps, &a1, &a2, &b, binc);
    int a = (a1 + 32) >> 6;
    int as = (a2 + 32) >> 6;
    /* "if capAdjust made us round away from what calculateLastPoint gave us, round back": a CapBegin
     * that moved the first major pixel one before the last pixel's is undone */
    if ((caps & CS_CAPBEGIN) && (vert ? s->lasty : s->lastx) == a + 1) a++;
    int lasta = s->lastx, lastb = s->lasty; /* in (x, y) terms below */
    if (a != as) {
        b += ((a * 64) + round - a1) * binc >> 6;
        int fa = a, fb = b >> 16;
        int la = as - 1, lb = (b + (as - a - 1) * binc) >> 16;
        if (swapped) {
            int t = fa; fa = la; la = t;
            t = fb; fb = lb; lb = t;
        }
        (void)fa;
        /* pixels in (x, y) */
        const int fx = vert ? fb : fa, fy = vert ? fa : fb;
        int lx = vert ? lb : la, ly = vert ? la : lb;
        const bool axisAligned = abs(binc) < (1 << 14);
        if (s->lastx > -1) {
            if (fx == s->lastx && fy == s->lasty) { /* remove duplicated pixel */
                if (swapped) {
                    --as;
                } else {
                    ++a;
                    b += binc;
                }
            } else if (s->lastDir != dir &&
                       (((axisAligned && s->lastAxisAligned) && s->lastx != fx && s->lasty != fy) ||
                        (abs(s->lastx - fx) > 1 || abs(s->lasty - fy) > 1))) { /* missing pixel: insert */
                if (swapped) {
                    ++as;
                } else {
                    --a;
                    b -= binc;
                }
            } else if (s->lastDir == dir && abs(s->lastx - fx) <= 1 && abs(s->lasty - fy) > 1) {
                b += binc >> 1;
                const int nl = swapped ? (b >> 16) : ((b + (as - a - 1) * binc) >> 16);
                if (vert) lx = nl;
                else ly = nl;
            }
        }
        s->lastDir = dir;
        s->lastAxisAligned = axisAligned;
        do {
            if (vert) cs_pixel(s, b >> 16, a);
            else cs_pixel(s, a, b >> 16);
            b += binc;
        } while (++a < as);
        lasta = lx;
        lastb = ly;
    }
    s->lastx = lasta;
    s->lasty = lastb;
}
static void cs_line(CStroker *s, double rx1, double ry1, double rx2, double ry2, int caps) {
    if (cs_clip(s, &rx1, &ry1, &rx2, &ry2)) return;
    const int x1 = toF26Dot6(rx1), y1 = toF26Dot6(ry1), x2 = toF26Dot6(rx2), y2 = toF26Dot6(ry2);
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    if (dx < dy) cs_run(s, true, y1, x1, y2, x2, caps);
    else if (dx) cs_run(s, false, x1, y1, x2, y2, caps);
}
/* QCosmeticStroker::calculateLastPoint: the closing segment's last pixel and direction */
static void cs_last_point(CStroker *s, double rx1, double ry1, double rx2, double ry2) {
    /* Qt 5.9 has no NoDirection: lastDir keeps its value when the closing segment has no pixel */
    s->lastx = CS_INT_MIN;
    s->lasty = CS_INT_MIN;
    if (cs_clip(s, &rx1, &ry1, &rx2, &ry2)) return;
    int x1 = toF26Dot6(rx1), y1 = toF26Dot6(ry1), x2 = toF26Dot6(rx2), y2 = toF26Dot6(ry2);
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    if (dx < dy) {
        bool swapped = false;
        if (y1 > y2) {
            swapped = true;
            int t = y1; y1 = y2; y2 = t;
            t = x1; x1 = x2; x2 = t;
        }
        const int xinc = F16Dot16FixedDiv(x2 - x1, y2 - y1);
        int x = x1 * 1024;
        const int y = (y1 + 32) >> 6, ys = (y2 + 32) >> 6;
        const int round = (xinc > 0) ? 32 : 0;
        if (y != ys) {
            x += ((y * 64) + round - y1) * xinc >> 6;
            if (swapped) {
                s->lastx = x >> 16;
                s->lasty = y;
                s->lastDir = CS_B2T;
            } else {
                s->lastx = (x + (ys - y - 1) * xinc) >> 16;
                s->lasty = ys - 1;
                s->lastDir = CS_T2B;
            }
            s->lastAxisAligned = abs(xinc) < (1 << 14);
        }
    } else {
        if (!dx) return;
        bool swapped = false;
        if (x1 > x2) {
            swapped = true;
            int t = x1; x1 = x2; x2 = t;
            t = y1; y1 = y2; y2 = t;
        }
        const int yinc = F16Dot16FixedDiv(y2 - y1, x2 - x1);
        int y = y1 * 1024;
        const int x = (x1 + 32) >> 6, xs = (x2 + 32) >> 6;
        const int round = (yinc > 0) ? 32 : 0;
        if (x != xs) {
            y += ((x * 64) + round - x1) * yinc >> 6;
            if (swapped) {
                s->lastx = x;
                s->lasty = y >> 16;
                s->lastDir = CS_R2L;
            } else {
                s->lastx = xs - 1;
                s->lasty = (y + (xs - x - 1) * yinc) >> 16;
                s->lastDir = CS_L2R;
            }
            s->lastAxisAligned = abs(yinc) < (1 << 14);
        }
    }
}
/* renderCubic / renderCubicSubdivision / splitCubic; points[3] is the start, points[0] the end */
static void cs_split_cubic(PtD *p) {
    const double half = .5;
    double a, b, c, d;
    p[6].x = p[3].x;
    c = p[1].x;
    d = p[2].x;
    p[1].x = a = (p[0].x + c) * half;
    p[5].x = b = (p[3].x + d) * half;
    c = (c + d) * half;
    p[2].x = a = (a + c) * half;
    p[4].x = b = (b + c) * half;
    p[3].x = (a + b) * half;
    p[6].y = p[3].y;
    c = p[1].y;
    d = p[2].y;
    p[1].y = a = (p[0].y + c) * half;
    p[5].y = b = (p[3].y + d) * half;
    c = (c + d) * half;
    p[2].y = a = (a + c) * half;
    p[4].y = b = (b + c) * half;
    p[3].y = (a + b) * half;
}
static void cs_cubic_sub(CStroker *s, PtD *p, int level, int caps) {
    if (level) {
        const double dx = p[3].x - p[0].x, dy = p[3].y - p[0].y;
        const double len = ((double).25) * (fabs(dx) + fabs(dy));
        if (fabs(dx * (p[0].y - p[2].y) - dy * (p[0].x - p[2].x)) >= len ||
            fabs(dx * (p[0].y - p[1].y) - dy * (p[0].x - p[1].x)) >= len) {
            cs_split_cubic(p);
            --level;
            cs_cubic_sub(s, p + 3, level, caps);
            cs_cubic_sub(s, p, level, caps);
            return;
        }
    }
    cs_line(s, p[3].x, p[3].y, p[0].x, p[0].y, caps);
}
/* QCosmeticStroker::drawPath of the ellipse's closed subpath: caps off (closed), the last point of
 * the closing segment (cp2 -> end of the last curve) primes the duplicate / dropout checks */
static void ag_stroke_ellipse(AgCanvas *c, const PtD pts[13], uint32_t pm) {
    CStroker s;
    s.c = c;
    s.pm = pm;
    s.xmin = -1;
    s.xmax = c->w + 1; /* deviceRect.right() + 2 */
    s.ymin = -1;
    s.ymax = c->h + 1;
    s.lastAxisAligned = false;
    s.lastDir = CS_L2R; /* QCosmeticStroker ctor */
    s.lastx = CS_INT_MIN;
    s.lasty = CS_INT_MIN;
    cs_last_point(&s, pts[11].x, pts[11].y, pts[12].x, pts[12].y);
    for (int k = 0; k < 4; k++) {
        PtD p[3 * CS_MAXSUB + 4];
        p[3] = pts[3 * k];
        p[2] = pts[3 * k + 1];
        p[1] = pts[3 * k + 2];
        p[0] = pts[3 * k + 3];
        cs_cubic_sub(&s, p, CS_MAXSUB, CS_NOCAPS);
    }
}

/* QPainter::drawEllipse(QRectF) with setBrush(QBrush(c1)), setPen(QPen(c2)) (assetgen.cpp:95-99):
 * the brush fill, then the pen.  Returns -1 for an integral rect, which Qt draws with its own
 * midpoint-ellipse path instead (QRasterPaintEngine::drawEllipse; not restated: a random float
 * rect is integral with probability ~1e-10) */
static int ag_draw_ellipse(AgCanvas *c, double x, double y, double w, double h, uint32_t brush, uint32_t pen, int parts) {
    if (w <= 0 || h <= 0) return 0; /* QRectF::isNull / empty: qt_curves_for_arc returns nothing */
    if (x == (int)x && y == (int)y && w == (int)w && h == (int)h) return -1;
    PtD pts[13];
    qt_ellipse_points(x, y, w, h, pts);
    if (parts & 1) ag_fill_ellipse(c, pts, qt_solid_premul(brush));
    if (parts & 2) ag_stroke_ellipse(c, pts, qt_solid_premul(pen));
    return 0;
}

/* ================================================================== jumper's compass at RENDER_RES
 * (jumper.cpp:137-177 under Antialiasing, render_mode="rgb_array"): the painter calls are
 *   drawEllipse(QRectF) with QBrush(c) + QPen(c, 1)  -> QPaintEngineEx::drawEllipse: the path of
 *       qt_curves_for_arc filled by the antialiased gray raster (qgrayraster.c, a FreeType
 *       "smooth" rasterizer fork) on QOutlineMapper's flattened 26.6 outline, then stroked by the
 *       antialiased QCosmeticStroker (a width-1 pen under a translation is a fast pen);
 *   drawLine(QLine) with QPen(c, thickness > 1) -> QRasterPaintEngine::stroke;
 *   fillRect(QRectF) (qt_smooth_fill_rectf);
 *   drawEllipse(QRect) with a translucent brush and no pen -> the gray raster fill.
 * Pinned primitive by primitive against the real Qt 5.9.7 (tests/test_smooth_pins.py). */

/* solid colour blend of one antialiased span pixel: blend_color_argb (Source for an opaque colour)
 * / comp_func_solid_SourceOver with const_alpha = coverage, on an RGB32 canvas */
static void qt_aa_blend_solid(uint32_t *d, uint32_t pm, int cov) {
    if (cov <= 0) return;
    const uint32_t c = cov == 255 ? pm : BYTE_MUL(pm, (uint32_t)cov);
    const uint32_t a = c >> 24;
    *d = a == 255 ? c : c + BYTE_MUL(*d, 255u - a);
}

/* ---- qgrayraster.c: PIXEL_BITS 8 cells (area, cover) accumulated along the outline's lines in
 * 24.8, clipped to the clip box [0, cw) x [0, ch) (cells left of it pile up in column -1, cells right
 * of it are dropped), then swept row by row into coverages (area >> 9, nonzero or even-odd) */
#define GR_PB 8
#define GR_ONE (1 << GR_PB)
typedef struct {
    int min_ex, max_ex, min_ey, max_ey, count_ex, count_ey;
    int ex, ey, invalid;     /* current cell (relative; ex -1 = left of the clip) */
    int area, cover;          /* its accumulators (TArea / TCoord: int) */
    int x, y, last_ey;        /* pen position (24.8) and the current row's top */
    int *carea, *ccover;      /* dense cells: (count_ey) x (count_ex + 1), column 0 = ex -1 */
} GrRas;
static void gr_record(GrRas *r) {
    if (!r->invalid && (r->area | r->cover)) {
        const size_t k = (size_t)r->ey * (r->count_ex + 1) + (r->ex + 1);
        r->carea[k] += r->area;
        r->ccover[k] += r->cover;
    }
}
static void gr_set_cell(GrRas *r, int ex, int ey) {
    ey -= r->min_ey;
    if (ex > r->max_ex) ex = r->max_ex;
    ex -= r->min_ex;
    if (ex < 0) ex = -1;
    if (ex != r->ex || ey != r->ey) {
        gr_record(r);
        r->area = 0;
        r->cover = 0;
    }
    r->ex = ex;
    r->ey = ey;
    r->invalid = ((unsigned)ey >= (unsigned)r->count_ey || ex >= r->count_ex);
}
static void gr_start_cell(GrRas *r, int ex, int ey) {
    if (ex > r->max_ex) ex = r->max_ex;
    if (ex < r->min_ex) ex = r->min_ex - 1;
    r->area = 0;
    r->cover = 0;
    r->ex = ex - r->min_ex;
    r->ey = ey - r->min_ey;
    r->last_ey = ey << GR_PB;
    r->invalid = 0;
    gr_set_cell(r, ex, ey);
}
static int gr_trunc(long x) { return (int)(x >> GR_PB); }
static void gr_scanline(GrRas *r, int ey, long x1, int y1, long x2, int y2) {
    long dx = x2 - x1;
    int ex1 = gr_trunc(x1), ex2 = gr_trunc(x2);
    const int fx1 = (int)(x1 - ((long)ex1 << GR_PB)), fx2 = (int)(x2 - ((long)ex2 << GR_PB));
    if (y1 == y2) {
        gr_set_cell(r, ex2, ey);
        return;
    }
    if (ex1 == ex2) {
        const int delta = y2 - y1;
        r->area += (fx1 + fx2) * delta;
        r->cover += delta;
        return;
    }
    long p = (long)(GR_ONE - fx1) * (y2 - y1);
    int first = GR_ONE, incr = 1;
    if (dx < 0) {
        p = (long)fx1 * (y2 - y1);
        first = 0;
        incr = -1;
        dx = -dx;
    }
    int delta = (int)(p / dx), mod = (int)(p % dx);
    if (mod < 0) {
        delta--;
        mod += (int)dx;
    }
    r->area += (fx1 + first) * delta;
    r->cover += delta;
    ex1 += incr;
    gr_set_cell(r, ex1, ey);
    y1 += delta;
    if (ex1 != ex2) {
        p = (long)GR_ONE * (y2 - y1 + delta);
        int lift = (int)(p / dx), rem = (int)(p % dx);
        if (rem < 0) {
            lift--;
            rem += (int)dx;
        }
        mod -= (int)dx;
        while (ex1 != ex2) {
            delta = lift;
            mod += rem;
            if (mod >= 0) {
                mod -= (int)dx;
                delta++;
            }
            r->area += GR_ONE * delta;
            r->cover += delta;
            y1 += delta;
            ex1 += incr;
            gr_set_cell(r, ex1, ey);
        }
    }
    delta = y2 - y1;
    r->area += (fx2 + GR_ONE - first) * delta;
    r->cover += delta;
}
static void gr_line(GrRas *r, long to_x, long to_y) {
    int ey1 = gr_trunc(r->last_ey), ey2 = gr_trunc(to_y);
    const int fy1 = (int)(r->y - r->last_ey), fy2 = (int)(to_y - ((long)ey2 << GR_PB));
    long dx = to_x - r->x, dy = to_y - r->y;
    {
        const int mn = ey1 < ey2 ? ey1 : ey2, mx = ey1 < ey2 ? ey2 : ey1;
        if (mn >= r->max_ey || mx < r->min_ey) goto end;
    }
    if (ey1 == ey2) {
        gr_scanline(r, ey1, r->x, fy1, to_x, fy2);
        goto end;
    }
    {
        int incr = 1;
        if (dx == 0) {
            const int ex = gr_trunc(r->x);
            const int two_fx = (int)((r->x - ((long)ex << GR_PB)) << 1);
            int first = GR_ONE;
            if (dy < 0) {
                first = 0;
                incr = -1;
            }
            int delta = first - fy1;
            r->area += two_fx * delta;
            r->cover += delta;
            ey1 += incr;
            gr_set_cell(r, ex, ey1);
            delta = first + first - GR_ONE;
            const int area = two_fx * delta;
            while (ey1 != ey2) {
                r->area += area;
                r->cover += delta;
                ey1 += incr;
                gr_set_cell(r, ex, ey1);
            }
            delta = fy2 - GR_ONE + first;
            r->area += two_fx * delta;
            r->cover += delta;
            goto end;
        }
        long p = (long)(GR_ONE - fy1) * dx;
        int first = GR_ONE;
        if (dy < 0) {
            p = (long)fy1 * dx;
            first = 0;
            incr = -1;
            dy = -dy;
        }
        int delta = (int)(p / dy), mod = (int)(p % dy);
        if (mod < 0) {
            delta--;
            mod += (int)dy;
        }
        long x = r->x + delta;
        gr_scanline(r, ey1, r->x, fy1, x, first);
        ey1 += incr;
        gr_set_cell(r, gr_trunc(x), ey1);
        if (ey1 != ey2) {
            p = (long)GR_ONE * dx;
            int lift = (int)(p / dy), rem = (int)(p % dy);
            if (rem < 0) {
                lift--;
                rem += (int)dy;
            }
            mod -= (int)dy;
            while (ey1 != ey2) {
                delta = lift;
                mod += rem;
                if (mod >= 0) {
                    mod -= (int)dy;
                    delta++;
                }
                const long x2 = x + delta;
                gr_scanline(r, ey1, x, GR_ONE - first, x2, first);
                x = x2;
                ey1 += incr;
                gr_set_cell(r, gr_trunc(x), ey1);
            }
        }
        gr_scanline(r, ey1, x, GR_ONE - first, to_x, fy2);
    }
end:
    r->x = (int)to_x;
    r->y = (int)to_y;
    r->last_ey = ey2 << GR_PB;
}
static int gr_coverage(int area, bool even_odd) { /* gray_hline */
    int c = area >> (GR_PB * 2 + 1 - 8);
    if (c < 0) c = -c;
    if (even_odd) {
        c &= 511;
        if (c > 256) c = 512 - c;
        else if (c == 256) c = 255;
    } else if (c >= 256) {
        c = 255;
    }
    return c;
}
/* fill one closed contour of 26.6 points (QT_FT_Outline: the decomposer closes it) in `pm` */
static void qt_gray_fill(const int *fx, const int *fy, int n, bool even_odd, uint32_t pm, uint32_t *canvas, int cw, int ch) {
    if (n <= 0) return;
    GrRas r;
    int xmn = fx[0], xmx = fx[0], ymn = fy[0], ymx = fy[0];
    for (int i = 1; i < n; i++) {
        if (fx[i] < xmn) xmn = fx[i];
        if (fx[i] > xmx) xmx = fx[i];
        if (fy[i] < ymn) ymn = fy[i];
        if (fy[i] > ymx) ymx = fy[i];
    }
    r.min_ex = xmn >> 6; r.min_ey = ymn >> 6; r.max_ex = (xmx + 63) >> 6; r.max_ey = (ymx + 63) >> 6;
    if (r.max_ex <= 0 || r.min_ex >= cw || r.max_ey <= 0 || r.min_ey >= ch) return;
    if (r.min_ex < 0) r.min_ex = 0;
    if (r.min_ey < 0) r.min_ey = 0;
    if (r.max_ex > cw) r.max_ex = cw;
    if (r.max_ey > ch) r.max_ey = ch;
    r.count_ex = r.max_ex - r.min_ex;
    r.count_ey = r.max_ey - r.min_ey;
    const size_t ncell = (size_t)r.count_ey * (r.count_ex + 1);
    r.carea = (int *)calloc(ncell, sizeof(int));
    r.ccover = (int *)calloc(ncell, sizeof(int));
    r.invalid = 1;
    r.ex = r.ey = 0;
    r.area = r.cover = 0;
    /* gray_move_to(first) then gray_line_to each point, and back to the first (contour close) */
    {
        const long x0 = (long)fx[0] << (GR_PB - 6), y0 = (long)fy[0] << (GR_PB - 6);
        gr_record(&r);
        gr_start_cell(&r, gr_trunc(x0), gr_trunc(y0));
        r.x = (int)x0;
        r.y = (int)y0;
        for (int i = 1; i <= n; i++) {
            const int k = i < n ? i : 0;
            gr_line(&r, (long)fx[k] << (GR_PB - 6), (long)fy[k] << (GR_PB - 6));
        }
        gr_record(&r);
    }
    /* gray_sweep */
    for (int yi = 0; yi < r.count_ey; yi++) {
        uint32_t *row = canvas + (size_t)(yi + r.min_ey) * cw + r.min_ex;
        const int *ca = r.carea + (size_t)yi * (r.count_ex + 1), *cc = r.ccover + (size_t)yi * (r.count_ex + 1);
        int cover = 0, x = 0;
        for (int cx = -1; cx < r.count_ex; cx++) {
            if (ca[cx + 1] == 0 && cc[cx + 1] == 0) continue; /* no cell here */
            if (cx > x && cover != 0) {
                const int c = gr_coverage(cover * (GR_ONE * 2), even_odd);
                for (int k = x; k < cx; k++) qt_aa_blend_solid(&row[k], pm, c);
            }
            cover += cc[cx + 1];
            const int area = cover * (GR_ONE * 2) - ca[cx + 1];
            if (area != 0 && cx >= 0) qt_aa_blend_solid(&row[cx], pm, gr_coverage(area, even_odd));
            x = cx + 1;
        }
        if (r.count_ex > x && cover != 0) {
            const int c = gr_coverage(cover * (GR_ONE * 2), even_odd);
            for (int k = x; k < r.count_ex; k++) qt_aa_blend_solid(&row[k], pm, c);
        }
    }
    free(r.carea);
    free(r.ccover);
}
/* the ellipse path filled by the gray raster: QOutlineMapper flattens the four curves (threshold
 * 0.25) and rounds to 26.6; QVectorPath::EllipseHint carries no WindingFill -> odd-even */
static void qt_aa_fill_ellipse(const PtD pts[13], uint32_t pm, uint32_t *canvas, int cw, int ch) {
    static PtD poly[4 * 1100];
    static int fx[4 * 1100], fy[4 * 1100];
    int n = 0;
    poly[n++] = pts[0];
    for (int k = 0; k < 4; k++) {
        QBez b = {poly[n - 1].x, poly[n - 1].y, pts[3 * k + 1].x, pts[3 * k + 1].y, pts[3 * k + 2].x, pts[3 * k + 2].y,
                  pts[3 * k + 3].x, pts[3 * k + 3].y};
        n = qbez_flatten(b, 0.25, poly, n);
    }
    for (int i = 0; i < n; i++) {
        fx[i] = qt_fixed_26_6(poly[i].x);
        fy[i] = qt_fixed_26_6(poly[i].y);
    }
    qt_gray_fill(fx, fy, n, true, pm, canvas, cw, ch);
}

/* ---- QCosmeticStroker, antialiased (drawLineAntialiased<drawPixel, NoDasher>): two pixels per
 * major step weighted by the minor position's fraction, the end pixels by their 26.6 coverage */
typedef struct {
    uint32_t *canvas;
    int cw, ch;
    uint32_t pm;
    double xmin, xmax, ymin, ymax;
    int lastx, lasty; /* clipLine writes them (unused antialiased) */
} CStrokerAA;
static void csa_pixel(CStrokerAA *s, int x, int y, int cov) {
    if (x < 0 || x > s->cw - 1 || y < 0 || y > s->ch - 1) return;
    qt_aa_blend_solid(&s->canvas[(size_t)y * s->cw + x], s->pm, (cov * 256) >> 8);
}
static bool csa_clip(CStrokerAA *s, double *x1, double *y1, double *x2, double *y2) {
    CStroker t;
    t.xmin = s->xmin; t.xmax = s->xmax; t.ymin = s->ymin; t.ymax = s->ymax;
    t.lastx = s->lastx;
    const bool out = cs_clip(&t, x1, y1, x2, y2);
    s->lastx = t.lastx;
    return out;
}
static void csa_line(CStrokerAA *s, double rx1, double ry1, double rx2, double ry2, int caps) {
    if (csa_clip(s, &rx1, &ry1, &rx2, &ry2)) return;
    int x1 = toF26Dot6(rx1), y1 = toF26Dot6(ry1), x2 = toF26Dot6(rx2), y2 = toF26Dot6(ry2);
    const int dx = x2 - x1, dy = y2 - y1;
    if (abs(dx) < abs(dy)) { /* vertical */
        const int xinc = F16Dot16FixedDiv(dx, dy);
        if (y1 > y2) {
            int t = y1; y1 = y2; y2 = t;
            t = x1; x1 = x2; x2 = t;
            caps = swapCaps(caps);
        }
        int x = (x1 - 32) * 1024;
        x -= (((y1 & 63) - 32) * xinc) >> 6;
        capAdjust(caps, &y1, &y2, &x, xinc);
        int y = y1 >> 6;
        const int ys = y2 >> 6;
        int aS, aE;
        if (y == ys) {
            aS = y2 - y1;
            aE = 0;
        } else {
            aS = 64 - (y1 & 63);
            aE = y2 & 63;
        }
        {
            const unsigned al = (uint8_t)(x >> 8);
            csa_pixel(s, x >> 16, y, (int)((255 - al) * aS) >> 6);
            csa_pixel(s, (x >> 16) + 1, y, (int)(al * aS) >> 6);
        }
        x += xinc;
        ++y;
        if (y < ys) {
            do {
                const unsigned al = (uint8_t)(x >> 8);
                csa_pixel(s, x >> 16, y, (int)(255 - al));
                csa_pixel(s, (x >> 16) + 1, y, (int)al);
                x += xinc;
            } while (++y < ys);
        }
        if (aE) {
            const unsigned al = (uint8_t)(x >> 8);
            csa_pixel(s, x >> 16, y, (int)((255 - al) * aE) >> 6);
            csa_pixel(s, (x >> 16) + 1, y, (int)(al * aE) >> 6);
        }
    } else { /* horizontal */
        if (!dx) return;
        const int yinc = F16Dot16FixedDiv(dy, dx);
        if (x1 > x2) {
            int t = x1; x1 = x2; x2 = t;
            t = y1; y1 = y2; y2 = t;
            caps = swapCaps(caps);
        }
        int y = (y1 - 32) * 1024;
        y -= (((x1 & 63) - 32) * yinc) >> 6;
        capAdjust(caps, &x1, &x2, &y, yinc);
        int x = x1 >> 6;
        const int xs = x2 >> 6;
        int aS, aE;
        if (x == xs) {
            aS = x2 - x1;
            aE = 0;
        } else {
            aS = 64 - (x1 & 63);
            aE = x2 & 63;
        }
        {
            const unsigned al = (uint8_t)(y >> 8);
            csa_pixel(s, x, y >> 16, (int)((255 - al) * aS) >> 6);
            csa_pixel(s, x, (y >> 16) + 1, (int)(al * aS) >> 6);
        }
        y += yinc;
        ++x;
        if (x < xs) {
            do {
                const unsigned al = (uint8_t)(y >> 8);
                csa_pixel(s, x, y >> 16, (int)(255 - al));
                csa_pixel(s, x, (y >> 16) + 1, (int)al);
                y += yinc;
            } while (++x < xs);
        }
        if (aE) {
            const unsigned al = (uint8_t)(y >> 8);
            csa_pixel(s, x, y >> 16, (int)((255 - al) * aE) >> 6);
            csa_pixel(s, x, (y >> 16) + 1, (int)(al * aE) >> 6);
        }
    }
}
static void csa_cubic_sub(CStrokerAA *s, PtD *p, int level, int caps) {
    if (level) {
        const double dx = p[3].x - p[0].x, dy = p[3].y - p[0].y;
        const double len = ((double).25) * (fabs(dx) + fabs(dy));
        if (fabs(dx * (p[0].y - p[2].y) - dy * (p[0].x - p[2].x)) >= len ||
            fabs(dx * (p[0].y - p[1].y) - dy * (p[0].x - p[1].x)) >= len) {
            cs_split_cubic(p);
            --level;
            csa_cubic_sub(s, p + 3, level, caps);
            csa_cubic_sub(s, p, level, caps);
            return;
        }
    }
    csa_line(s, p[3].x, p[3].y, p[0].x, p[0].y, caps);
}
static void qt_aa_stroke_ellipse(const PtD pts[13], uint32_t pm, uint32_t *canvas, int cw, int ch) {
    CStrokerAA s;
    s.canvas = canvas; s.cw = cw; s.ch = ch; s.pm = pm;
    s.xmin = -1; s.xmax = cw + 1; s.ymin = -1; s.ymax = ch + 1;
    s.lastx = s.lasty = CS_INT_MIN;
    for (int k = 0; k < 4; k++) {
        PtD p[3 * CS_MAXSUB + 4];
        p[3] = pts[3 * k];
        p[2] = pts[3 * k + 1];
        p[1] = pts[3 * k + 2];
        p[0] = pts[3 * k + 3];
        csa_cubic_sub(&s, p, CS_MAXSUB, CS_NOCAPS);
    }
}

/* QRasterPaintEngine::fill's early out: the path's control-point rect, toRect() (qRound of x, y, w,
 * h), must intersect the device rect (QRect::intersects) */
static bool qt_path_on_device(const PtD *p, int n, int cw, int ch) {
    double x0 = p[0].x, x1 = p[0].x, y0 = p[0].y, y1 = p[0].y;
    for (int i = 1; i < n; i++) {
        if (p[i].x < x0) x0 = p[i].x;
        if (p[i].x > x1) x1 = p[i].x;
        if (p[i].y < y0) y0 = p[i].y;
        if (p[i].y > y1) y1 = p[i].y;
    }
    const int rx = qRound(x0), ry = qRound(y0), rw = qRound(x1 - x0), rh = qRound(y1 - y0);
    if (rw == 0 && rh == 0) return false; /* QRect::isNull */
    const int ax2 = rx + rw - 1, ay2 = ry + rh - 1;
    int l1 = rx, r1 = rx, t1 = ry, b1 = ry;
    if (ax2 - rx + 1 < 0) l1 = ax2; else r1 = ax2;
    if (ay2 - ry + 1 < 0) t1 = ay2; else b1 = ay2;
    return !(l1 > cw - 1 || 0 > r1 || t1 > ch - 1 || 0 > b1);
}
/* drawEllipse(QRectF(x, y, w, h)) under Antialiasing: brush `brush` (0 = none) filled, then pen `pen`
 * (0 = none, width 1) stroked; colours non-premultiplied ARGB */
static void qt_aa_draw_ellipse(double x, double y, double w, double h, uint32_t brush, uint32_t pen, uint32_t *canvas,
                               int cw, int ch) {
    if (w <= 0 || h <= 0) return;
    PtD pts[13];
    qt_ellipse_points(x, y, w, h, pts);
    if (brush >> 24 && qt_path_on_device(pts, 13, cw, ch)) qt_aa_fill_ellipse(pts, qt_solid_premul(brush), canvas, cw, ch);
    if (pen >> 24) qt_aa_stroke_ellipse(pts, qt_solid_premul(pen), canvas, cw, ch);
}
/* drawLine(QLine(x1, y1, x2, y2)) with QPen(colour, width > 1), SquareCap, under Antialiasing:
 * QRasterPaintEngine::stroke's rasterizeLine branch (width / length, square caps) */
static void qt_aa_wide_line(int x1, int y1, int x2, int y2, int width, uint32_t argb, uint32_t *canvas, int cw, int ch) {
    const double dx = (double)x2 - x1, dy = (double)y2 - y1, len = sqrt(dx * dx + dy * dy);
    static QtSpan spans[8192];
    int ns;
    if (len == 0) /* a point: the square cap alone, as a horizontal line of the pen's width and relative width 1 */
        ns = qt_aa_line_spans_cap(x1 - width * 0.5, y1, x1 + width * 0.5, y1, 1, false, cw, ch, spans, 8192);
    else
        ns = qt_aa_line_spans_cap(x1, y1, x2, y2, width / len, true, cw, ch, spans, 8192);
    const uint32_t pm = qt_solid_premul(argb);
    for (int k = 0; k < ns; k++)
        for (int xx = spans[k].x; xx < spans[k].x + spans[k].len; xx++)
            qt_aa_blend_solid(&canvas[(size_t)spans[k].y * cw + xx], pm, spans[k].cov);
}

/* one compass primitive on a cw x ch RGB32 canvas (tests/test_smooth_pins.py against
 * tools/qt_smooth_probe.cpp qtp_prim): kind 10 drawEllipse(QRectF) brush + 1-px pen, 13 pen only,
 * 14 brush only, 12 drawEllipse(QRect(int x, y, w, h)) brush only, 11 drawLine(QLine) pen width `penw` */
void oracle_qt_prim(int cw, int ch, uint32_t *inout, int kind, double x, double y, double w, double h, uint32_t argb,
                    int penw) {
    switch (kind) {
    case 10: qt_aa_draw_ellipse(x, y, w, h, argb, argb, inout, cw, ch); break;
    case 13: qt_aa_draw_ellipse(x, y, w, h, 0, argb, inout, cw, ch); break;
    case 14: qt_aa_draw_ellipse(x, y, w, h, argb, 0, inout, cw, ch); break;
    case 12: qt_aa_draw_ellipse((int)x, (int)y, (int)w, (int)h, argb, 0, inout, cw, ch); break;
    case 11: qt_aa_wide_line((int)x, (int)y, (int)w, (int)h, penw, argb, inout, cw, ch); break;
    default: break;
    }
}

/* ---- AssetGen (assetgen.cpp:3-195); float / double promotion as the C++ source has it */
typedef struct {
    MT *rg;
    float rgb_start[3], rgb_len[3];
    int rgb_choice[3];
    float p_rect;
} ColorGen;
static void cg_roll(ColorGen *g) { /* :10-20 */
    for (int i = 0; i < 3; i++) g->rgb_len[i] = rg_rand01(g->rg);
    for (int i = 0; i < 3; i++) g->rgb_start[i] = rg_rand01(g->rg) * (1 - g->rgb_len[i]);
    g->p_rect = rg_rand01(g->rg);
}
static uint32_t cg_rand_color(ColorGen *g) { /* :22-28, QColor(r, g, b) */
    for (int i = 0; i < 3; i++) g->rgb_choice[i] = (int)(255 * (rg_rand01(g->rg) * g->rgb_len[i] + g->rgb_start[i]));
    return 0xff000000u | ((uint32_t)g->rgb_choice[0] << 16) | ((uint32_t)g->rgb_choice[1] << 8) | (uint32_t)g->rgb_choice[2];
}
typedef struct {
    MT *rg;
    AgCanvas *c;
    int err; /* an integral ellipse rect (Qt's midpoint path, not restated) */
} AssetGen;
static RectD ag_choose_sub_rect(AssetGen *a, RectD rect, float min_dim, float max_dim) { /* :35-51 */
    const int w = (int)rect.w, h = (int)rect.h;
    const int smaller = (w > h) ? h : w;
    const float del_dim = max_dim - min_dim;
    const float rdx = (rg_rand01(a->rg) * del_dim + min_dim) * smaller;
    const float rdy = (rg_rand01(a->rg) * del_dim + min_dim) * smaller;
    const float rx_off = rg_rand01(a->rg) * (w - rdx);
    const float ry_off = rg_rand01(a->rg) * (h - rdy);
    RectD r = {rx_off + rect.x, ry_off + rect.y, rdx, rdy};
    return r;
}
static void ag_paint_shape(AssetGen *a, RectD main_rect, ColorGen *cg) { /* :75-102 (split_rect :53-73) */
    const int k = rg_randn(a->rg, 10);
    const int num_splits = (k * k) / 50 + 1;
    const bool is_horizontal = rg_randbool(a->rg);
    const float x = (float)main_rect.x, y = (float)main_rect.y, w = (float)main_rect.w, h = (float)main_rect.h;
    const float dw = w / num_splits, dh = h / num_splits;
    const bool use_rect = rg_randbool(a->rg);
    const bool regen_colors = rg_randbool(a->rg);
    uint32_t c1 = cg_rand_color(cg);
    uint32_t c2 = cg_rand_color(cg);
    for (int i = 0; i < num_splits; i++) {
        RectD r;
        if (is_horizontal) {
            r.x = x + i * dw; r.y = y; r.w = dw; r.h = h;
        } else {
            r.x = x; r.y = y + i * dh; r.w = w; r.h = dh;
        }
        if (regen_colors) {
            c1 = cg_rand_color(cg);
            c2 = cg_rand_color(cg);
        }
        if (use_rect) {
            ag_fill_rectf(a->c, r.x, r.y, r.w, r.h, c1);
        } else if (ag_draw_ellipse(a->c, r.x, r.y, r.w, r.h, c1, c2, 3) < 0) {
            a->err = 1;
        }
    }
}
static void ag_paint_rect_resource(AssetGen *a, RectD rect, int num_recurse, int blotch_scale) { /* :104-132 */
    ColorGen cg = {a->rg, {0}, {0}, {0}, 0};
    cg_roll(&cg);
    const uint32_t bgcolor = cg_rand_color(&cg);
    ag_fill_rectf(a->c, rect.x, rect.y, rect.w, rect.h, bgcolor);
    const float scale = (float)(.3 + .7 * (double)rg_rand01(a->rg));
    const float max_rand_dim = (float)(.5 * (double)scale);
    const float min_rand_dim = (float)(.05 * (double)scale);
    const int num_blotches = rg_randint(a->rg, blotch_scale, 2 * blotch_scale);
    const float p_recurse = (float)((double)rg_rand01(a->rg) * .75);
    for (int j = 0; j < num_blotches; j++) {
        const RectD dst3 = ag_choose_sub_rect(a, rect, min_rand_dim, max_rand_dim);
        if ((num_recurse > 0) && (rg_rand01(a->rg) < p_recurse)) ag_paint_rect_resource(a, dst3, num_recurse - 1, 10);
        else ag_paint_shape(a, dst3, &cg);
    }
    ag_fill_rectf(a->c, rect.x, rect.y, rect.w, rect.h, (bgcolor & 0x00ffffffu) | (200u << 24)); /* setAlpha(200) */
}
static RectD ag_create_bar(AssetGen *a, RectD rect, bool is_horizontal) { /* :134-149 */
    const float k1 = (float)(.45 + (double)rg_rand01(a->rg) * .4);
    const float k2 = (float)(.45 + (double)rg_rand01(a->rg) * .4);
    const float w = (float)(rect.w * k1 * k1);
    const float h = (float)(rect.h * k2 * k2);
    const float pct = rg_rand01(a->rg);
    RectD r;
    if (is_horizontal == 0) {
        r.x = 0; r.y = (rect.h - h) * pct; r.w = rect.w; r.h = h;
    } else {
        r.x = (rect.h - w) * pct; r.y = 0; r.w = w; r.h = rect.h; /* the reference uses height() for x */
    }
    return r;
}
static void ag_paint_shape_resource(AssetGen *a, RectD rect) { /* :151-184 */
    ColorGen cg = {a->rg, {0}, {0}, {0}, 0};
    cg_roll(&cg);
    const bool horizontal_first = rg_randbool(a->rg);
    const int nbar1 = rg_randn(a->rg, 3) / 2 + 1;
    const int nbar2 = rg_randn(a->rg, 3) / 2 + 1;
    const int saved = a->c->source;
    a->c->source = 1; /* save(); setCompositionMode(CompositionMode_Source) */
    ag_fill_rectf(a->c, rect.x, rect.y, rect.w, rect.h, 0x00000000u);
    for (int i = 0; i < nbar1; i++) ag_paint_shape(a, ag_create_bar(a, rect, horizontal_first), &cg);
    for (int i = 0; i < nbar2; i++) ag_paint_shape(a, ag_create_bar(a, rect, !horizontal_first), &cg);
    const int num_blotches = rg_randint(a->rg, 1, 5);
    for (int j = 0; j < num_blotches; j++) ag_paint_shape(a, ag_choose_sub_rect(a, rect, 0.1f, 0.6f), &cg);
    a->c->source = saved; /* restore() */
}
/* AssetGen::generate_resource (:186-195) on the canvas; returns 0, or -1 when an integral ellipse rect
 * was met */
static int ag_generate_resource(MT *rg, AgCanvas *c, int num_recurse, int blotch_scale, bool is_rect) {
    AssetGen a = {rg, c, 0};
    RectD rect = {0, 0, (double)c->w, (double)c->h};
    if (is_rect) ag_paint_rect_resource(&a, rect, num_recurse, blotch_scale);
    else ag_paint_shape_resource(&a, rect);
    return a.err ? -1 : 0;
}

#define GEN_BG_DIM 500   /* QImage(500, 500, Format_RGB32) (basic-abstract-game.cpp:61) */
#define GEN_SPRITE_DIM 64 /* QImage(64, 64, Format_ARGB32) (:105) */
static void gen_paint_background(Game *g) {
    AgCanvas c = {g->gen_bg, GEN_BG_DIM, GEN_BG_DIM, QFMT_RGB32, 0};
    fassert(ag_generate_resource(&g->rand_gen, &c, 1, 50, true) == 0);
}
/* use_block_asset(type) of each game (basic-abstract-game.cpp:412-414 and the overrides: caveflyer.cpp:81,
 * chaser.cpp:74, climber.cpp:128, coinrun.cpp:183, dodgeball.cpp:153, fruitbot.cpp:137, heist.cpp:62,
 * jumper.cpp:107, leaper.cpp:87, ninja.cpp:135) */
static bool gen_use_block_asset(int gid, int t) {
    switch (gid) {
    case GAME_CAVEFLYER: return t == 8;                      /* CAVEWALL */
    case GAME_CHASER: return t == 5;                         /* MAZE_WALL */
    case GAME_CLIMBER: case GAME_COINRUN: return t == 15 || t == 16; /* WALL_MID, WALL_TOP */
    case GAME_DODGEBALL: return t == 1 || t == 5 || t == 7;  /* LAVA_WALL, DOOR, DOOR_OPEN */
    case GAME_FRUITBOT: return t == 1 || t == 10 || t == 12; /* BARRIER, LOCKED_DOOR, PRESENT */
    case GAME_HEIST: return t == WALL_OBJ || t == 1;         /* WALL_OBJ, LOCKED_DOOR */
    case 9 /* jumper */: return t == 6 || t == 7;            /* CAVEWALL, CAVEWALL_TOP */
    case GAME_LEAPER: return t == 3 || t == 2;               /* WATER, ROAD */
    case GAME_NINJA: return t == 20;                         /* WALL_MID */
    default: return false;
    }
}
static uint32_t fnv1a(const char *s) { /* hash_str_uint32 (vecgame.cpp:156-167) */
    uint32_t h = 0x811c9dc5u;
    for (; *s; s++) h = (h ^ (uint8_t)*s) * 0x1000193u;
    return h;
}
#define GEN_TYPES 99 /* image types 0..98 (slot 99 holds jumper's Qt-tabulated compass raster) */
/* The atlas of a use_generated_assets vec (initialize_asset_if_necessary, :79-123): every type's image
 * is generate_resource(64 x 64 ARGB32, 0, 5, use_block_asset(type)) with asset_rand_gen seeded
 * fixed_asset_seed + type, fixed_asset_seed = int(FNV-1a(env name)) (vecgame.cpp:370-375); one theme,
 * aspect ratio 1, the same image for every theme index (the seed ignores the theme); one background
 * slot, 500 x 500, whose pixels are each env's gen_bg.  Drawn premultiplied (Qt converts an ARGB32
 * source when blitting; its pixels are opaque or fully transparent, so that is the pixel or 0). */
static void gen_build_atlas(Vec *v, const char *env_name, int gid, const or_atlas *src) {
    const or_image *tab = &src->sprites[99];
    const size_t tab_px = (size_t)(tab->w > 0 ? tab->w * tab->h : 0);
    v->gen_pixels = (uint32_t *)calloc((size_t)GEN_TYPES * 4096 + tab_px + 1, sizeof(uint32_t));
    v->gen_sprites = (or_image *)calloc(1000, sizeof(or_image));
    v->gen_backgrounds = (or_image *)calloc(1, sizeof(or_image));
    v->gen_num_themes = (int32_t *)calloc(100, sizeof(int32_t));
    const uint32_t seed0 = fnv1a(env_name);
    uint32_t img[64 * 64];
    for (int t = 0; t < GEN_TYPES; t++) {
        MT m;
        rg_seed(&m, (int)(seed0 + (uint32_t)t));
        AgCanvas c = {img, GEN_SPRITE_DIM, GEN_SPRITE_DIM, QFMT_ARGB32, 0};
        fassert(ag_generate_resource(&m, &c, 0, 5, gen_use_block_asset(gid, t)) == 0);
        uint32_t *dst = v->gen_pixels + (size_t)t * 4096;
        for (int k = 0; k < 4096; k++) dst[k] = (img[k] >> 24) == 255 ? img[k] : 0u;
        for (int th = 0; th < 10; th++) {
            or_image im = {(uint32_t)(t * 4096), GEN_SPRITE_DIM, GEN_SPRITE_DIM, 0};
            v->gen_sprites[t + 100 * th] = im;
        }
        v->gen_num_themes[t] = 1;
    }
    if (tab_px) {
        memcpy(v->gen_pixels + (size_t)GEN_TYPES * 4096, src->pixels + tab->offset, tab_px * 4);
        or_image im = {(uint32_t)(GEN_TYPES * 4096), tab->w, tab->h, 0};
        v->gen_sprites[99] = im;
        v->gen_num_themes[99] = src->num_themes[99];
    }
    or_image bg = {0, GEN_BG_DIM, GEN_BG_DIM, 0};
    v->gen_backgrounds[0] = bg;
    or_atlas a = {v->gen_pixels, v->gen_sprites, v->gen_backgrounds, 1, v->gen_num_themes};
    v->gen_atlas = a;
    v->atlas = &v->gen_atlas;
}

/* ================================================================== render (basic-abstract-game.cpp) */

static void prepare_for_drawing(Game *g, float rect_height) { /* :828-847 */
    g->center_x = (float)(g->main_width * .5);
    g->center_y = (float)(g->main_height * .5);
    if (g->options.center_agent) {
        Entity *agent = AG(g); /* choose_center, :673-676 */
        if (g->game_id == GAME_CLIMBER) { /* climber.cpp:291-295 */
            g->center_x = (float)(g->main_width / 2.0);
            g->center_y = (float)((double)agent->y + g->main_width / 2.0 - (double)(5 * agent->ry));
            g->visibility = (float)g->main_width;
        } else if (g->game_id == GAME_FRUITBOT) { /* fruitbot.cpp:138-142 */
            g->center_x = (float)(g->main_width / 2.0);
            g->center_y = (float)((double)agent->y + g->main_width / 2.0 - (double)(2 * agent->ry));
            g->visibility = (float)g->main_width;
        } else {
            g->center_x = agent->x;
            g->center_y = agent->y;
        }
    } else {
        g->visibility = (float)(g->main_width > g->main_height ? g->main_width : g->main_height);
        if (g->visibility < g->min_visibility) g->visibility = g->min_visibility;
    }
    float raw_unit = 64 / g->visibility;
    g->unit = (float)((double)raw_unit * ((double)rect_height / 64.0));
    g->view_dim = (float)(64.0 / (double)raw_unit);
    g->x_off = g->unit * (g->center_x - g->view_dim / 2);
    g->y_off = g->unit * (g->center_y - g->view_dim / 2);
}

static RectD get_screen_rect(Game *g, float x, float y, float dx, float dy, float render_eps) { /* :808-810 */
    RectD r;
    r.x = (double)((x - render_eps) * g->unit - g->x_off);
    r.y = (double)((g->view_dim - y - render_eps) * g->unit + g->y_off);
    r.w = (double)((dx + 2 * render_eps) * g->unit);
    r.h = (double)((dy + 2 * render_eps) * g->unit);
    return r;
}

static RectD adjust_rect(RectD b, RectD a) { /* qt-utils.h:12-19 */
    RectD r;
    r.x = b.x + b.w * a.x;
    r.y = b.y + b.h * a.y;
    r.w = b.w * a.w;
    r.h = b.h * a.h;
    return r;
}

static void tile_image_fmt(Game *g, const uint32_t *px, int iw, int ih, int fmt, bool refl, double opacity, RectD rect,
                           float tile_ratio) { /* basic-abstract-game.cpp:849-877 */
    if (tile_ratio != 0) {
        if (tile_ratio < 0) {
            tile_ratio = -1 * tile_ratio;
            int num_tiles = (int)(rect.h / (rect.w * tile_ratio));
            if (num_tiles < 1) num_tiles = 1;
            float tile_height = (float)(rect.h / num_tiles);
            float tile_width = (float)rect.w;
            for (int i = 0; i < num_tiles; i++)
                qt_draw_image(g->canvas, rect.x, rect.y + tile_height * i, tile_width, tile_height, px, iw, ih, fmt,
                              refl, opacity);
        } else {
            int num_tiles = (int)(rect.w / (rect.h * tile_ratio));
            if (num_tiles < 1) num_tiles = 1;
            float tile_width = (float)(rect.w / num_tiles);
            float tile_height = (float)rect.h;
            for (int i = 0; i < num_tiles; i++)
                qt_draw_image(g->canvas, rect.x + tile_width * i, rect.y, tile_width, tile_height, px, iw, ih, fmt,
                              refl, opacity);
        }
    } else {
        qt_draw_image(g->canvas, rect.x, rect.y, rect.w, rect.h, px, iw, ih, fmt, refl, opacity);
    }
}
static void tile_image(Game *g, const uint32_t *px, int iw, int ih, bool refl, double opacity, RectD rect,
                       float tile_ratio) {
    tile_image_fmt(g, px, iw, ih, QFMT_ARGB32_PM, refl, opacity, rect, tile_ratio);
}

static float hook_tile_aspect_ratio(Game *g, const Entity *e) {
    if (g->game_id == GAME_LEAPER && e->type == LP_FINISH_LINE) return 1; /* leaper.cpp:68-74 */
    if (g->game_id == GAME_DODGEBALL && e->type == 1) return e->rx > e->ry ? 1 : -1; /* dodgeball.cpp:240-246 */
    if (g->game_id == GAME_FRUITBOT) { /* fruitbot.cpp:87-93 */
        if (e->type == 1) return 1;
        if (e->type == 10) return 3.25f;
    }
    return 0;                                                            /* :417-419 */
}

/* color_for_type (basic-abstract-game.cpp:464-490): monochrome colour of (type, theme), k = 4 */
static uint32_t color_for_type(Game *g, int type, int theme) {
    theme = mask_theme(g, theme, type);
    int new_type = (29 * (type + 1)) % 64;
    new_type = (new_type + 19 * theme) % 64;
    uint32_t r = 64 * (new_type / 16 + 1) - 1, gg = 64 * ((new_type / 4) % 4 + 1) - 1, b = 64 * (new_type % 4 + 1) - 1;
    return 0xff000000u | (r << 16) | (gg << 8) | b;
}

/* to_shade (qt-utils.h:21-28) */
static int to_shade(float f) {
    int shade = (int)(f * 255);
    return shade < 0 ? 0 : (shade > 255 ? 255 : shade);
}

static void draw_image(Game *g, const or_atlas *at, RectD base, float rotation, bool is_reflected, int base_type,
                       int theme, float alpha, float tile_ratio) { /* :886-922 */
    int img_type = hook_image_for_type(g, base_type);
    if (img_type < 0) return;
    if (g->options.use_monochrome_assets || img_type >= USE_ASSET_THRESHOLD) {
        /* draw_grid_obj: SPACE draws nothing; monochrome fills are restated in a later round */
        if (img_type == SPACE) return;
        if (g->game_id == GAME_CHASER && img_type == CH_ORB) { /* chaser.cpp:111-117 */
            float k = 1 - CH_ORB_DIM;
            qt_fill_rectf(g->canvas, base.x + base.w * k / 2, base.y + base.h * k / 2, base.w * CH_ORB_DIM,
                          base.h * CH_ORB_DIM, 0xff00ff00u);
            return;
        }
        if (!g->options.use_monochrome_assets || img_type >= 64) /* color_for_type fasserts (:464-490) */
            fatal_msg("draw_grid_obj: no colour for this type");
        qt_fill_rectf(g->canvas, base.x, base.y, base.w, base.h, color_for_type(g, img_type, theme));
        return;
    }
    fassert(theme < MAX_IMAGE_THEMES);
    theme = mask_theme(g, theme, img_type); /* the image initialize_asset_if_necessary loaded, :79-123 */
    int img_idx = img_type + theme * MAX_ASSETS;
    RectD r = base;
    if (g->game_id == GAME_COINRUN && is_player_image(img_type)) { /* coinrun.cpp:64-70 */
        RectD adj = {0, -.7415, 1, 1.7415};
        r = adjust_rect(base, adj);
    } else if (g->game_id == GAME_LEAPER && img_type == PLAYER) { /* leaper.cpp:244-250 */
        RectD adj = {0, -.275, 1, 1.55};
        r = adjust_rect(base, adj);
    }
    const or_image *im = &at->sprites[img_idx];
    /* miner's MUD image (misc_assets/mud.png, resources.cpp:511) is absent from the reference's
     * asset tree -- the reference cannot draw it at all (load_resource_ptr fatals); this restatement
     * and the engine both draw nothing for it (parity unpinned for MUD tiles) */
    if (im->w <= 0 && g->game_id == GAME_MINER && img_type == MN_MUD) return;
    if (im->w <= 0) fatal_msg("missing sprite (generated assets are not restated yet)");
    double opacity = alpha != 1 ? (double)alpha : 1.0;
    if (rotation == 0) {
        tile_image(g, at->pixels + im->offset, im->w, im->h, is_reflected, opacity, r, tile_ratio);
    } else { /* :908-916: p.rotate(rotation * 180 / PI) */
        float deg = rotation * 180 / PI_F;
        qt_draw_image_rotated(g->canvas, r.x, r.y, r.w, r.h, (double)deg, at->pixels + im->offset, im->w, im->h,
                              is_reflected, opacity);
    }
}

static void draw_entities(Game *g, const or_atlas *at, int render_z) { /* :1061-1075 */
    for (int i = 0; i < g->num_ents; i++) {
        Entity *e = &g->ents[i];
        if (e->render_z != render_z) continue;
        if (!hook_should_draw_entity(g, e)) continue;
        RectD r1;
        if (e->use_abs_coords) { /* get_abs_rect (:812-814) via get_object_rect (:820-826) */
            float vd = g->view_dim;
            float ax = vd * (e->x - e->rx), ay = vd * (e->y + e->ry), aw = 2 * vd * e->rx, ah = 2 * vd * e->ry;
            r1.x = (double)(ax * g->unit);
            r1.y = (double)(ay * g->unit);
            r1.w = (double)(aw * g->unit);
            r1.h = (double)(ah * g->unit);
        } else {
            r1 = get_screen_rect(g, e->x - e->rx, e->y + e->ry, 2 * e->rx, 2 * e->ry, 0); /* :820-826 */
        }
        draw_image(g, at, r1, e->rotation, e->is_reflected, e->image_type, e->image_theme, e->alpha,
                   hook_tile_aspect_ratio(g, e));
    }
}

static void draw_background(Game *g, const or_atlas *at) { /* :988-1016 */
    qt_fill_rect_int(g->canvas, 0, 0, RT.w, RT.h, 0xff000000u);
    prepare_for_drawing(g, (float)RT.h);
    if (!g->options.use_backgrounds) return;
    RectD main_rect = get_screen_rect(g, 0, (float)g->main_height, (float)g->main_width, (float)g->main_height, 0);
    const or_image *bg = &at->backgrounds[g->background_index];
    const uint32_t *bgpx = g->gen_bg ? g->gen_bg : at->pixels + bg->offset; /* procedurally generated */
    if (g->bg_tile_ratio < 0) { /* :1003-1004 */
        tile_image_fmt(g, bgpx, bg->w, bg->h, QFMT_RGB32, false, 1.0, main_rect, g->bg_tile_ratio);
        return;
    }
    float bgw = (float)bg->w;
    float bgh = (float)bg->h;
    float bg_ar = bgw / bgh;
    float world_ar = (float)(g->main_width * 1.0 / g->main_height);
    float extra_w = bg_ar - world_ar;
    float offset_x = g->bg_pct_x * extra_w;
    RectD adj = {(double)(-offset_x), 0, (double)(bg_ar / world_ar), 1};
    RectD r = adjust_rect(main_rect, adj);
    qt_draw_image(g->canvas, r.x, r.y, r.w, r.h, bgpx, bg->w, bg->h, QFMT_RGB32, false, 1.0);
}

static void draw_foreground(Game *g, const or_atlas *at) { /* :930-979 */
    prepare_for_drawing(g, (float)RT.h);
    draw_entities(g, at, -1);
    int low_x, high_x, low_y, high_y;
    if (g->options.center_agent) {
        double margin = (double)g->visibility / 2.0 + 1;
        low_x = (int)((double)g->center_x - margin);
        high_x = (int)((double)g->center_x + margin);
        low_y = (int)((double)g->center_y - margin);
        high_y = (int)((double)g->center_y + margin);
    } else {
        low_x = 0;
        high_x = g->main_width - 1;
        low_y = 0;
        high_y = g->main_height - 1;
    }
    for (int x = low_x; x <= high_x; x++) {
        for (int y = low_y; y <= high_y; y++) {
            int type = get_obj(g, x, y);
            if (type == INVALID_OBJ) continue;
            int theme = hook_theme_for_grid_obj(g, type);
            RectD r2 = get_screen_rect(g, (float)x, (float)(y + 1), 1, 1, RENDER_EPS);
            draw_image(g, at, r2, 0, false, type, theme, 1.0f, 0);
        }
    }
    draw_entities(g, at, 0);
    draw_entities(g, at, 1);
    if (g->has_useful_vel_info && g->options.paint_vel_info) { /* :969-977 */
        Entity *agent = AG(g);
        float infodim = (float)(RT.h * .2);
        int s1 = to_shade((float)(.5 * (double)agent->vx / (double)g->maxspeed + .5));
        int s2 = to_shade((float)(.5 * (double)agent->vy / (double)g->max_jump + .5));
        qt_fill_rectf(g->canvas, 0, 0, infodim, infodim, 0xff000000u | (uint32_t)(s1 * 0x010101));
        qt_fill_rectf(g->canvas, infodim, 0, infodim, infodim, 0xff000000u | (uint32_t)(s2 * 0x010101));
    }
}

/* jumper's draw_compass (jumper.cpp:137-177).  The dial ellipse, the cosmetic needle line and the
 * translucent jump ellipse are the Qt 5.9.7 raster output tabulated by tools/qt_compass_tables.cpp
 * (the atlas image slot JP_TABLE_SLOT carries the table, procgen_amd/assets.py); the distance bar
 * is fillRect(QRectF) (qt_fill_rectf, pinned by qt_raster_fill_goldens). */
#define JP_TABLE_SLOT 99
static void jp_stamp(uint32_t *canvas, const uint32_t *rows64, int dx, int dy, uint32_t argb, bool blend) {
    for (int y = 0; y < RES_H; y++) {
        int sy = y - dy;
        if (sy < 0 || sy >= RES_H) continue;
        uint64_t m = (uint64_t)rows64[2 * sy] | ((uint64_t)rows64[2 * sy + 1] << 32);
        for (int x = 0; x < RES_W; x++) {
            int sx = x - dx;
            if (sx < 0 || sx >= 64 || !((m >> sx) & 1)) continue;
            uint32_t *d = &canvas[y * RES_W + x];
            *d = blend ? argb + BYTE_MUL(*d, (~argb) >> 24) : argb;
        }
    }
}
static void qt_aa_draw_ellipse(double x, double y, double w, double h, uint32_t brush, uint32_t pen, uint32_t *canvas,
                               int cw, int ch);
static void qt_aa_wide_line(int x1, int y1, int x2, int y2, int width, uint32_t argb, uint32_t *canvas, int cw, int ch);
/* the compass at RENDER_RES: the painter calls themselves, restated antialiased (qt_aa_*; each
 * logged as kind 10 / 11 / 12 for the replay through the real Qt) */
static void jp_draw_compass_smooth(Game *g) {
    const float u = g->unit, vd = g->view_dim, cd = g->jp_compass_dim;
    const float ax = (float)(vd - cd - .25), ay = .25f; /* get_abs_rect (:812-814) */
    const double rx = (double)(ax * u), ry = (double)(ay * u), rw = (double)(cd * u), rh = (double)(cd * u);
    qt_log(10, rx, ry, rw, rh, (double)0xffa8a69eu, 1, 0, 1);
    qt_aa_draw_ellipse(rx, ry, rw, rh, 0xffa8a69eu, 0xffa8a69eu, RT.px, RT.w, RT.h); /* QColor(168, 166, 158) */
    const float pen_thickness = (float)(RT.w / (256.0 / cd));
    const float cx = (float)(rx + rw / 2), cy = (float)(ry + rh / 2); /* QRectF::center */
    const float cr = (float)(rw / 2 * .95);
    Entity *agent = AG(g), *goal = &g->ents[1];
    const float theta = (float)atan2((double)(goal->y - agent->y), (double)(goal->x - agent->x)); /* get_theta */
    const int x1 = (int)cx, y1 = (int)cy; /* QPainter::drawLine(int, int, int, int) */
    const int x2 = (int)(cx + cr * cos((double)theta)), y2 = (int)(cy - cr * sin((double)theta));
    qt_log(11, x1, y1, x2, y2, (double)0xfffcba03u, (int)pen_thickness, 0, 1);
    qt_aa_wide_line(x1, y1, x2, y2, (int)pen_thickness, 0xfffcba03u, RT.px, RT.w, RT.h); /* QColor(252, 186, 3) */
    float ddx = agent->x - goal->x, ddy = agent->y - goal->y; /* get_distance (:133-143) */
    float dist = (float)sqrt((double)(ddx * ddx + ddy * ddy));
    float dist_pct = (float)(dist / (g->main_width * sqrt(2)));
    float bar_thickness = cd / 8;
    qt_fill_rectf(g->canvas, (double)((float)(vd - cd - .25) * u), (double)((float)(.25 + cd) * u),
                  (double)(cd * dist_pct * u), (double)(bar_thickness * u), 0xfffcba03u);
    if (g->jp_jump_delta < 0 && !g->has_support) { /* drawEllipse(QRect(...)), QColor(255, 255, 255, 120) */
        RectD r1 = get_screen_rect(g, agent->x - agent->rx, agent->y + agent->ry, 2 * agent->rx, 2 * agent->ry, 0);
        const int qx = (int)r1.x, qy = (int)(r1.y + r1.h * (5.0 / 6)), qw = (int)r1.w, qh = (int)(r1.h / 3);
        qt_log(12, qx, qy, qw, qh, (double)0x78ffffffu, 0, 0, 1);
        qt_aa_draw_ellipse(qx, qy, qw, qh, 0x78ffffffu, 0, RT.px, RT.w, RT.h);
    }
}
static void jp_draw_compass(Game *g, const or_atlas *at) {
    if (RT.smooth) {
        jp_draw_compass_smooth(g);
        return;
    }
    const or_image *ti = &at->sprites[JP_TABLE_SLOT];
    fassert(ti->w > 0);
    const uint32_t *t = at->pixels + ti->offset;
    const int NY = (int)t[1], NX = (int)t[2], MAXW = (int)t[3], MAXH = (int)t[4];
    const int cfg = (g->options.distribution_mode == EasyMode ? 0 : 1) + (g->options.center_agent ? 0 : 2);
    const uint32_t *cg = t + 5 + 9 * cfg;
    const int x1 = (int)cg[0], y1 = (int)cg[1], bx0 = (int)cg[2], by0 = (int)cg[3], bnx = (int)cg[4], bny = (int)cg[5];
    float cx, cy, cr;
    memcpy(&cx, &cg[6], 4);
    memcpy(&cy, &cg[7], 4);
    memcpy(&cr, &cg[8], 4);
    const uint32_t *dial = t + 5 + 36;
    const uint32_t *needle = dial + 4 * 128;
    const uint32_t *jump = needle + (size_t)4 * NY * NX * 128;
    float u = g->unit, vd = g->view_dim, cd = g->jp_compass_dim;
    /* the table geometry must be the frame's: compass_rect = get_abs_rect(vd - cd - .25, .25, cd, cd) */
    double rx = (double)((float)(vd - cd - .25) * u), rw = (double)(cd * u);
    fassert((float)(rx + rw / 2) == cx);
    jp_stamp(g->canvas, dial + 128 * cfg, 0, 0, 0xffa8a69eu, false); /* QColor(168, 166, 158) */
    Entity *agent = AG(g), *goal = &g->ents[1];
    float theta = (float)atan2((double)(goal->y - agent->y), (double)(goal->x - agent->x)); /* get_theta (:241-246) */
    int x2 = (int)(cx + cr * cos((double)theta)), y2 = (int)(cy - cr * sin((double)theta));
    (void)x1; (void)y1;
    fassert(bx0 <= x2 && x2 < bx0 + bnx && by0 <= y2 && y2 < by0 + bny);
    jp_stamp(g->canvas, needle + ((size_t)(cfg * NY + (y2 - by0)) * NX + (x2 - bx0)) * 128, 0, 0, 0xfffcba03u, false);
    float ddx = agent->x - goal->x, ddy = agent->y - goal->y; /* get_distance (:133-143) */
    float dist = (float)sqrt((double)(ddx * ddx + ddy * ddy));
    float dist_pct = (float)(dist / (g->main_width * sqrt(2)));
    float bar_thickness = cd / 8;
    qt_fill_rectf(g->canvas, (double)((float)(vd - cd - .25) * u), (double)((float)(.25 + cd) * u),
                  (double)(cd * dist_pct * u), (double)(bar_thickness * u), 0xfffcba03u);
    if (g->jp_jump_delta < 0 && !g->has_support) { /* get_object_rect(agent) -> QRect(int, ...) */
        RectD r1 = get_screen_rect(g, agent->x - agent->rx, agent->y + agent->ry, 2 * agent->rx, 2 * agent->ry, 0);
        int qx = (int)r1.x, qy = (int)(r1.y + r1.h * (5.0 / 6)), qw = (int)r1.w, qh = (int)(r1.h / 3);
        fassert(0 <= qw && qw <= MAXW && 0 <= qh && qh <= MAXH);
        jp_stamp(g->canvas, jump + (size_t)(qw * (MAXH + 1) + qh) * 128, qx - 20, qy - 20, 0x78787878u, true);
    }
}

static void render(Game *g, const or_atlas *at) { /* game.cpp:97-107 -> game_draw, :1018-1021 */
    if (g->game_id == GAME_STARPILOT) { /* starpilot.cpp:107-124: scrolling tiled background */
        /* `rect` is the render target's: 64 x 64, or RENDER_RES for render_mode="rgb_array" */
        const int rw = RT.smooth ? RT.w : RES_W, rh = RT.smooth ? RT.h : RES_H;
        float scale = (float)(rh / g->main_height); /* int / int */
        qt_fill_rect_int(g->canvas, 0, 0, rw, rh, 0xff000000u);
        if (g->options.use_backgrounds) {
            float bg_k = 3;
            float t = (float)g->cur_time;
            float x_off = -t * scale * g->sp_hp_slow_v * 2 / g->char_dim;
            const float BG_RATIO = 18;
            RectD r_bg = {(double)x_off, (double)(-rh * (bg_k - 1) / 2), (double)(rh * bg_k * BG_RATIO),
                          (double)(rh * bg_k)};
            const or_image *bg = &at->backgrounds[g->background_index];
            tile_image_fmt(g, g->gen_bg ? g->gen_bg : at->pixels + bg->offset, bg->w, bg->h, QFMT_RGB32, false, 1.0, r_bg, 1);
        }
        draw_foreground(g, at);
        return;
    }
    draw_background(g, at);
    draw_foreground(g, at);
    if (g->game_id == GAME_JUMPER && g->options.distribution_mode != MemoryMode) jp_draw_compass(g, at);
    if (g->game_id == GAME_NINJA) { /* ninja.cpp:155-164: jump charge bar, get_abs_rect (:812-814) */
        float u = g->unit;
        float bar_height = 3 * g->nj_jump_charge;
        float vis = g->visibility;
        qt_fill_rectf(g->canvas, (double)(.25f * u), (double)((float)(vis - .5 - bar_height) * u), (double)(.5f * u),
                      (double)(bar_height * u), 0xff42f587u);
    }
    if (g->game_id == GAME_PLUNDER) { /* plunder.cpp:66-77: juice and progress bars, get_abs_rect (:812-814) */
        float u = g->unit;
        qt_fill_rectf(g->canvas, (double)(.25f * u), (double)(.25f * u), (double)(g->main_width * g->pl_juice_left * u),
                      (double)(.5f * u), 0xff42f587u);
        float prog = (float)(g->main_width * (g->pl_targets_hit * 1.0 / g->pl_target_quota));
        qt_fill_rectf(g->canvas, (double)(.25f * u), (double)(.75f * u), (double)(prog * u), (double)(.5f * u),
                      0xfff54290u);
    }
}

/* ================================================================== construction (vecgame.cpp) */
static int game_id_of(const char *name) {
    if (strcmp(name, "coinrun") == 0) return GAME_COINRUN;
    if (strcmp(name, "bigfish") == 0) return GAME_BIGFISH;
    if (strcmp(name, "maze") == 0) return GAME_MAZE;
    if (strcmp(name, "heist") == 0) return GAME_HEIST;
    if (strcmp(name, "miner") == 0) return GAME_MINER;
    if (strcmp(name, "climber") == 0) return GAME_CLIMBER;
    if (strcmp(name, "leaper") == 0) return GAME_LEAPER;
    if (strcmp(name, "chaser") == 0) return GAME_CHASER;
    if (strcmp(name, "fruitbot") == 0) return GAME_FRUITBOT;
    if (strcmp(name, "dodgeball") == 0) return GAME_DODGEBALL;
    if (strcmp(name, "plunder") == 0) return GAME_PLUNDER;
    if (strcmp(name, "starpilot") == 0) return GAME_STARPILOT;
    if (strcmp(name, "bossfight") == 0) return GAME_BOSSFIGHT;
    if (strcmp(name, "ninja") == 0) return GAME_NINJA;
    if (strcmp(name, "caveflyer") == 0) return GAME_CAVEFLYER;
    if (strcmp(name, "jumper") == 0) return GAME_JUMPER;
    return -1;
}

static void basic_ctor(Game *g) { /* Game ctor game.cpp:25-39 + BasicAbstractGame ctor :22-46 */
    g->timeout = 1000;
    g->episodes_remaining = 0;
    g->last_reward = -1;
    g->default_action = 0;
    g->reset_count = 0;
    g->current_level_seed = 0;
    g->sd_reward = 0;
    g->sd_done = true;
    g->sd_level_complete = false;
    g->char_dim = 5;
    g->main_width = 0;
    g->main_height = 0;
    g->visibility = 16;
    g->min_visibility = 0;
    g->mixrate = 0.5f;
    g->maxspeed = 0.5f;
    g->max_jump = g->maxspeed;
    g->default_action = 4;
    g->last_move_action = 7;
    g->bg_tile_ratio = 0;
    g->out_of_bounds_object = INVALID_OBJ;
    g->has_useful_vel_info = true;
    g->random_agent_start = true;
}

static void coinrun_ctor(Game *g) { /* coinrun.cpp:49-58 */
    g->visibility = 13;
    g->mixrate = 0.2f;
    g->main_width = 64;
    g->main_height = 64;
    g->out_of_bounds_object = CR_WALL_MID;
}
static void bigfish_ctor(Game *g) { /* bigfish.cpp:24-29 */
    g->timeout = 6000;
    g->main_width = 20;
    g->main_height = 20;
}
static void maze_ctor(Game *g) { /* maze.cpp:20-28 */
    g->timeout = 500;
    g->random_agent_start = false;
    g->has_useful_vel_info = false;
    g->out_of_bounds_object = WALL_OBJ;
    g->visibility = 8.0f;
}
static void fruitbot_ctor(Game *g) { /* fruitbot.cpp:30-40 */
    g->mixrate = .5f;
    g->maxspeed = 0.85f;
    g->bg_tile_ratio = -1;
    g->out_of_bounds_object = 2; /* OUT_OF_BOUNDS_WALL */
}
static void ninja_ctor(Game *g) { /* ninja.cpp:35-41 */
    g->main_width = 64;
    g->main_height = 64;
    g->out_of_bounds_object = 20; /* WALL_MID */
}
static void bossfight_ctor(Game *g) { /* bossfight.cpp:60-68 */
    g->timeout = 4000;
    g->main_width = 20;
    g->main_height = 20;
    g->mixrate = .5;
    g->maxspeed = 0.85f;
}
static void starpilot_ctor(Game *g) { /* starpilot.cpp:50-54 */
    g->main_width = 16;
    g->main_height = 16;
}
static void plunder_ctor(Game *g) { /* plunder.cpp:33-43 */
    g->timeout = 4000;
    g->main_width = 20;
    g->main_height = 20;
    g->mixrate = .5;
    g->maxspeed = 0.85f;
    g->has_useful_vel_info = false;
}
static void dodgeball_ctor(Game *g) { /* dodgeball.cpp:37-44 */
    g->mixrate = .5;
    g->db_enemy_fire_delay = 50;
    g->out_of_bounds_object = 10; /* OOB_WALL */
}
static void chaser_ctor(Game *g) { /* chaser.cpp:37-47 */
    g->mixrate = 1;
    g->maxspeed = .5f;
    g->eat_timeout = 75;
    g->egg_timeout = 50;
    g->has_useful_vel_info = false;
}
static void leaper_ctor(Game *g) { /* leaper.cpp:34-38 */
    g->maxspeed = LP_MAX_SPEED;
    g->timeout = 500;
}
static void climber_ctor(Game *g) { /* climber.cpp:38-41 */
    g->out_of_bounds_object = CL_WALL_MID;
}
static void miner_ctor(Game *g) { /* miner.cpp:30-43 */
    g->main_width = 20;
    g->main_height = 20;
    g->main_area = g->main_width * g->main_height;
    g->mixrate = .5f;
    g->maxspeed = .5f;
    g->has_useful_vel_info = false;
    g->out_of_bounds_object = MN_OOB_WALL;
    g->visibility = 8.0f;
    g->diamonds_remaining = -1;
}
static void heist_ctor(Game *g) { /* heist.cpp:23-35 */
    g->has_useful_vel_info = false;
    g->main_width = 20;
    g->main_height = 20;
    g->out_of_bounds_object = WALL_OBJ;
    g->visibility = 8.0f;
}

/* Envs with global indices env_offset + n * stride (n < count) of a vec env: a mixed batch plays name
 * n % #names at env n (vecgame.cpp:357-358), so one game's envs of it are a strided range. */
void *oracle_make(const char *env_name, int count, int env_offset, const or_options *opt, const or_atlas *atlas) {
    return oracle_make_strided(env_name, count, env_offset, 1, opt, atlas);
}
void *oracle_make_strided(const char *env_name, int count, int env_offset, int stride, const or_options *opt,
                          const or_atlas *atlas) {
    int gid = game_id_of(env_name);
    if (stride < 1) return NULL;
    if (gid < 0 || count <= 0) return NULL;
    int dm = opt->distribution_mode;
    /* game.cpp:76-86: easy and hard for every game; extreme for chaser, dodgeball, leaper, starpilot;
     * memory for caveflyer, dodgeball, heist, jumper, maze, miner (game ids: procgen/env.py:15-32) */
    bool dm_ok = dm == EasyMode || dm == HardMode ||
                 (dm == ExtremeMode && (gid == GAME_CHASER || gid == GAME_DODGEBALL || gid == GAME_LEAPER || gid == 15)) ||
                 (dm == MemoryMode && (gid == 2 || gid == GAME_DODGEBALL || gid == GAME_HEIST || gid == 9 ||
                                       gid == GAME_MAZE || gid == GAME_MINER));
    if (!dm_ok) return NULL;
    Vec *v = (Vec *)calloc(1, sizeof(Vec));
    v->count = count;
    v->offset = env_offset;
    v->atlas = atlas;
    v->games = (Game *)calloc((size_t)count, sizeof(Game));
    if (opt->use_generated_assets) gen_build_atlas(v, env_name, gid, atlas);
    int level_seed_low = 0, level_seed_high = 0; /* vecgame.cpp:332-341 */
    if (opt->num_levels == 0) {
        level_seed_low = 0;
        level_seed_high = 2147483647;
    } else if (opt->num_levels > 0) {
        level_seed_low = opt->start_level;
        level_seed_high = opt->start_level + opt->num_levels;
    }
    MT seed_gen; /* vecgame.cpp:349-350 */
    rg_seed(&seed_gen, opt->rand_seed);
    for (int n = 0; n < env_offset; n++) (void)rg_randint0(&seed_gen);
    for (int n = 0; n < count; n++) {
        if (n > 0)
            for (int k = 1; k < stride; k++) (void)rg_randint0(&seed_gen); /* the other names' envs */
        Game *g = &v->games[n];
        g->game_id = gid;
        g->ents = (Entity *)calloc(MAX_ENTS, sizeof(Entity));
        basic_ctor(g);
        if (gid == GAME_COINRUN) coinrun_ctor(g);
        else if (gid == GAME_BIGFISH) bigfish_ctor(g);
        else if (gid == GAME_MAZE) maze_ctor(g);
        else if (gid == GAME_HEIST) heist_ctor(g);
        else if (gid == GAME_MINER) miner_ctor(g);
        else if (gid == GAME_CLIMBER) climber_ctor(g);
        else if (gid == GAME_LEAPER) leaper_ctor(g);
        else if (gid == GAME_CHASER) chaser_ctor(g);
        else if (gid == GAME_FRUITBOT) fruitbot_ctor(g);
        else if (gid == GAME_DODGEBALL) dodgeball_ctor(g);
        else if (gid == GAME_PLUNDER) plunder_ctor(g);
        else if (gid == GAME_STARPILOT) starpilot_ctor(g);
        else if (gid == GAME_BOSSFIGHT) bossfight_ctor(g);
        else if (gid == GAME_NINJA) ninja_ctor(g);
        else if (gid == GAME_CAVEFLYER) caveflyer_ctor(g);
        rg_seed(&g->level_seed_rand_gen, rg_randint0(&seed_gen)); /* vecgame.cpp:362 */
        g->level_seed_high = level_seed_high;
        g->level_seed_low = level_seed_low;
        g->game_n = env_offset + n * stride;
        /* parse_options, game.cpp:62-95 */
        g->options.paint_vel_info = opt->paint_vel_info;
        g->options.use_generated_assets = opt->use_generated_assets != 0;
        if (g->options.use_generated_assets) g->gen_bg = (uint32_t *)calloc((size_t)GEN_BG_DIM * GEN_BG_DIM, 4);
        g->options.use_monochrome_assets = opt->use_monochrome_assets;
        g->options.restrict_themes = opt->restrict_themes;
        g->options.use_backgrounds = opt->use_backgrounds;
        g->options.center_agent = opt->center_agent;
        g->options.use_sequential_levels = opt->use_sequential_levels;
        g->options.distribution_mode = dm;
        g->options.debug_mode = opt->debug_mode;
    }
    return v;
}

void oracle_close(void *h) {
    Vec *v = (Vec *)h;
    if (!v) return;
    for (int n = 0; n < v->count; n++) {
        free(v->games[n].ents);
        free(v->games[n].gen_bg);
    }
    free(v->games);
    free(v->gen_pixels);
    free(v->gen_sprites);
    free(v->gen_backgrounds);
    free(v->gen_num_themes);
    free(v);
}

void oracle_start(void *h) { /* vecgame.cpp:126-131 (initial reset + observe) */
    Vec *v = (Vec *)h;
    for (int n = 0; n < v->count; n++) {
        game_reset(&v->games[n], v->atlas);
        render(&v->games[n], v->atlas);
    }
}

void oracle_step(void *h, const int32_t *actions) {
    Vec *v = (Vec *)h;
    for (int n = 0; n < v->count; n++) {
        v->games[n].action = actions[n];
        game_step(&v->games[n], v->atlas);
    }
}

/* render_mode="rgb_array": info["rgb"] of every env, its current state painted at res x res with
 * Antialiasing + SmoothPixmapTransform (vecgame.cpp:415-423, Game::render_to_buf(buf, RENDER_RES,
 * RENDER_RES, true), game.cpp:97-107) and converted by bgr32_to_rgb888.  The games whose draws are
 * all axis-aligned images and fills are restated (bigfish, chaser, climber, coinrun, maze, miner,
 * ninja); the others return -1.  `log` (optional, `cap` doubles) receives env 0's painter
 * commands for replay through the real Qt (tests).  Render-time members (unit, view_dim, offsets)
 * are left as the 64-px observe sets them, as the step path reads them from there. */
int oracle_render_rgb_array(void *h, uint8_t *rgb, int res, double *log, int cap) {
    Vec *v = (Vec *)h;
    uint32_t *frame = (uint32_t *)malloc((size_t)res * res * 4);
    int rc = 0;
    for (int n = 0; n < v->count && rc == 0; n++) {
        Game *g = &v->games[n];
        Game saved = *g;
        RT.px = frame; RT.w = res; RT.h = res; RT.smooth = true;
        RT.log = n == 0 ? log : NULL; RT.log_n = 0; RT.log_cap = cap;
        render(g, v->atlas);
        RT.px = NULL; RT.w = RES_W; RT.h = RES_H; RT.smooth = false; RT.log = NULL;
        *g = saved; /* the 64-px render-time members */
        uint8_t *d = rgb + (size_t)n * res * res * 3;
        for (size_t p = 0; p < (size_t)res * res; p++) {
            const uint32_t c = frame[p];
            d[3 * p + 0] = (uint8_t)(c >> 16);
            d[3 * p + 1] = (uint8_t)(c >> 8);
            d[3 * p + 2] = (uint8_t)c;
        }
    }
    free(frame);
    return rc;
}

void oracle_observe(void *h, uint8_t *rgb, float *rew, uint8_t *first, int32_t *prev_level_seed,
                    uint8_t *prev_level_complete, int32_t *level_seed) {
    Vec *v = (Vec *)h;
    for (int n = 0; n < v->count; n++) {
        Game *g = &v->games[n];
        if (rgb) { /* bgr32_to_rgb888, game.cpp:8-23 */
            uint8_t *d = rgb + (size_t)n * RES_W * RES_H * 3;
            for (int p = 0; p < RES_W * RES_H; p++) {
                uint32_t c = g->canvas[p];
                d[3 * p + 0] = (uint8_t)(c >> 16);
                d[3 * p + 1] = (uint8_t)(c >> 8);
                d[3 * p + 2] = (uint8_t)c;
            }
        }
        if (rew) rew[n] = g->sd_reward;
        if (first) first[n] = (uint8_t)g->sd_done;
        if (prev_level_seed) prev_level_seed[n] = g->prev_level_seed;
        if (prev_level_complete) prev_level_complete[n] = (uint8_t)g->sd_level_complete;
        if (level_seed) level_seed[n] = g->current_level_seed;
    }
}

/* Fork latent-state info (vecgame.cpp:270-316; maze.cpp:152-165): grid_size, the grid row-major
 * (zero padded to 35*35), agent_pos = int(agent->x), int(agent->y); exit_pos is miner-only.
 * Games without a latent state leave everything zero. */
void oracle_latent(void *h, int32_t *grid_size, int32_t *grid, int32_t *agent_pos, int32_t *exit_pos) {
    Vec *v = (Vec *)h;
    for (int n = 0; n < v->count; n++) {
        Game *g = &v->games[n];
        int32_t *gs = grid_size + 2 * n, *gr = grid + 35 * 35 * n, *ap = agent_pos + 2 * n, *ep = exit_pos + 2 * n;
        memset(gs, 0, 8);
        memset(gr, 0, 35 * 35 * 4);
        memset(ap, 0, 8);
        memset(ep, 0, 8);
        if (g->game_id == GAME_MAZE || g->game_id == GAME_MINER) {
            gs[0] = g->grid_w;
            gs[1] = g->grid_h;
            for (int i = 0; i < g->grid_w * g->grid_h && i < 35 * 35; i++) gr[i] = g->grid[i];
            Entity *a = AG(g);
            ap[0] = (int)a->x;
            ap[1] = (int)a->y;
        }
        if (g->game_id == GAME_MINER) { /* miner.cpp:378-396: the first EXIT entity */
            for (int i = 0; i < g->num_ents; i++)
                if (g->ents[i].type == MN_EXIT) {
                    ep[0] = (int)g->ents[i].x;
                    ep[1] = (int)g->ents[i].y;
                    break;
                }
        }
    }
}

/* MinerGame::game_set_state (miner.cpp:423-449): write the grid (a DEAD_PLAYER cell sets `died`),
 * then erase the PLAYER entity if died, else put the agent at (agent_x + .5, agent_y + .5); the
 * first EXIT entity goes to (exit_x + .5, exit_y + .5).  Re-renders the frame, as libenv's
 * set_state re-observes (vecgame.cpp:503).  Returns 0, or -1 when the reference would crash
 * (not miner, grid larger than the world, no EXIT entity). */
int oracle_miner_set_state(void *h, int i, const int32_t *grid, int grid_width, int grid_height, int agent_x,
                           int agent_y, int exit_x, int exit_y) {
    Vec *v = (Vec *)h;
    if (i < 0 || i >= v->count) return -1;
    Game *g = &v->games[i];
    if (g->game_id != GAME_MINER || grid_width < 0 || grid_height < 0 ||
        grid_width * grid_height > g->grid_w * g->grid_h)
        return -1;
    int exit_i = -1;
    for (int k = 0; k < g->num_ents; k++)
        if (g->ents[k].type == MN_EXIT) { exit_i = k; break; }
    if (exit_i < 0) return -1;
    for (int idx = 0; idx < grid_width * grid_height; ++idx) {
        int obj = grid[idx];
        set_obj_idx(g, idx, obj);
        if (obj == MN_DEAD_PLAYER) g->died = true;
    }
    if (g->died) {
        /* std::find_if(PLAYER) + entities.erase: entities[0] is the agent while it is listed */
        if (!g->agent_erased && g->num_ents > 0 && g->ents[0].type == PLAYER) {
            g->agent_ghost = g->ents[0];
            g->agent_erased = true;
            memmove(&g->ents[0], &g->ents[1], sizeof(Entity) * (size_t)(g->num_ents - 1));
            g->num_ents--;
        }
    } else {
        Entity *a = AG(g);
        a->x = agent_x + 0.5f;
        a->y = agent_y + 0.5f;
    }
    for (int k = 0; k < g->num_ents; k++)
        if (g->ents[k].type == MN_EXIT) {
            g->ents[k].x = exit_x + 0.5f;
            g->ents[k].y = exit_y + 0.5f;
            break;
        }
    render(g, v->atlas);
    return 0;
}

int oracle_debug(void *h, int i, int32_t *out, int n) {
    Vec *v = (Vec *)h;
    Game *g = &v->games[i];
    Entity *a = AG(g);
    int32_t vals[16];
    float fv[4] = {a->x, a->y, a->vx, a->vy};
    vals[0] = g->num_ents;
    vals[1] = g->cur_time;
    memcpy(&vals[2], fv, sizeof(fv));
    vals[6] = g->background_index;
    vals[7] = g->wall_theme;
    vals[8] = g->step_rand_int;
    vals[9] = g->has_support;
    vals[10] = g->current_level_seed;
    vals[11] = g->rand_gen.mti;
    memcpy(&vals[12], &g->bg_pct_x, 4);
    vals[13] = a->image_theme;
    vals[14] = g->agent_erased;
    vals[15] = g->reset_count;
    int k = n < 16 ? n : 16;
    memcpy(out, vals, (size_t)k * 4);
    return 16;
}

/* env i's entity list, 31 words per entity in Entity::serialize's order (entity.cpp:90-134: the
 * struct's member order above), floats as their bits, bools as 0 / 1; returns the entity count
 * (the caller's buffer holds cap entities) */
int oracle_entity_words(void *h, int i, int32_t *out, int cap) {
    Vec *v = (Vec *)h;
    Game *g = &v->games[i];
    for (int k = 0; k < g->num_ents && k < cap; k++) {
        const Entity *e = &g->ents[k];
        int32_t *o = out + (size_t)k * 31;
        float f6[6] = {e->x, e->y, e->vx, e->vy, e->rx, e->ry};
        memcpy(o, f6, sizeof(f6));
        o[6] = e->type; o[7] = e->image_type; o[8] = e->image_theme; o[9] = e->render_z;
        o[10] = e->will_erase; o[11] = e->collides_with_entities;
        float f3[3] = {e->collision_margin, e->rotation, e->vrot};
        memcpy(o + 12, f3, sizeof(f3));
        o[15] = e->is_reflected; o[16] = e->fire_time; o[17] = e->spawn_time; o[18] = e->life_time;
        o[19] = e->expire_time; o[20] = e->use_abs_coords;
        memcpy(o + 21, &e->friction, 4);
        o[22] = e->smart_step; o[23] = e->avoids_collisions; o[24] = e->auto_erase;
        float f7[6] = {e->alpha, e->health, e->theta, e->grow_rate, e->alpha_decay, e->climber_spawn_x};
        memcpy(o + 25, f7, sizeof(f7));
    }
    return g->num_ents;
}

/* ================================================================== pinning helpers */
void oracle_mt_stream(uint32_t seed, uint32_t *out, int n) {
    MT m;
    mt_seed(&m, seed);
    for (int i = 0; i < n; i++) out[i] = mt_next(&m);
}

/* ops: kind 0 randint(a,b) 1 randn(a) 2 rand01 (float bits) 3 randbool 4 randrange(a/8, b/8) 5 randint() */
void oracle_randgen_script(uint32_t seed, const int32_t *ops, int nops, int32_t *out) {
    MT m;
    rg_seed(&m, (int)seed);
    for (int i = 0; i < nops; i++) {
        int k = ops[3 * i], a = ops[3 * i + 1], b = ops[3 * i + 2];
        float f;
        switch (k) {
        case 0: out[i] = rg_randint(&m, a, b); break;
        case 1: out[i] = rg_randn(&m, a); break;
        case 2: f = rg_rand01(&m); memcpy(&out[i], &f, 4); break;
        case 3: out[i] = rg_randbool(&m); break;
        case 4: f = rg_randrange(&m, a / 8.0f, b / 8.0f); memcpy(&out[i], &f, 4); break;
        default: out[i] = rg_randint0(&m); break;
        }
    }
}

typedef struct {
    const uint8_t *p, *end;
} Rd;
static uint32_t rd_u32(Rd *r) {
    uint32_t v;
    if (r->p + 4 > r->end) fatal_msg("replay: short");
    memcpy(&v, r->p, 4);
    r->p += 4;
    return v;
}
static double rd_f64(Rd *r) {
    double v;
    if (r->p + 8 > r->end) fatal_msg("replay: short");
    memcpy(&v, r->p, 8);
    r->p += 8;
    return v;
}

/* replays ONE case body (after the canvas words) of tools/qt_raster_golden.cpp's format */
/* one Antialiasing + SmoothPixmapTransform primitive on a cw x ch RGB32 canvas (tests/test_smooth_pins.py,
 * against tools/qt_smooth_probe.cpp on the real Qt): kind 0 drawImage(QRectF, img [mirrored]) with
 * opacity, kind 1 fillRect(QRectF, opaque colour) */
static double rot_deg;
void oracle_qt_smooth_rot(int cw, int ch, uint32_t *inout, const uint32_t *img, int iw, int ih, int fmt, int mirrored,
                          double x, double y, double w, double h, double deg, double opacity);
void oracle_qt_smooth(int cw, int ch, uint32_t *inout, int kind, const uint32_t *img, int iw, int ih, int fmt,
                      int mirrored, double x, double y, double w, double h, double opacity, uint32_t argb) {
    QtTarget saved = RT;
    RT.px = inout; RT.w = cw; RT.h = ch; RT.smooth = true; RT.log = NULL;
    if (kind == 0) qt_draw_image(inout, x, y, w, h, img, iw, ih, fmt, mirrored != 0, opacity);
    else if (kind == 2) /* translate(x + w/2, y + h/2); rotate(degrees = argb as float bits); drawImage(-w/2, -h/2, w, h) */
        qt_smooth_draw_image_rot(x, y, w, h, rot_deg, img, iw, ih, fmt, mirrored != 0, opacity);
    else qt_fill_rectf(inout, x, y, w, h, argb);
    RT = saved;
}

/* kind 2 of tools/qt_smooth_probe.cpp: translate(x + w/2, y + h/2); rotate(deg); drawImage(QRectF(-w/2, -h/2, w, h)) */
void oracle_qt_smooth_rot(int cw, int ch, uint32_t *inout, const uint32_t *img, int iw, int ih, int fmt, int mirrored,
                          double x, double y, double w, double h, double deg, double opacity) {
    rot_deg = deg;
    oracle_qt_smooth(cw, ch, inout, 2, img, iw, ih, fmt, mirrored, x, y, w, h, opacity, 0);
}

/* qt-utils.h / grid.h pins (tests/test_oracle_pins.py, against the reference headers compiled in
 * oracle/_ref): adjust_rect over (x, y, w, h) quadruples, to_shade of floats, and the Grid
 * operations the oracle's Game grid restates (contains, get_obj's in-range read / out-of-bounds
 * object, y * w + x indexing and its inverse) */
void oracle_adjust_rect(const double *base, const double *adj, double *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        RectD b = {base[4 * i], base[4 * i + 1], base[4 * i + 2], base[4 * i + 3]};
        RectD a = {adj[4 * i], adj[4 * i + 1], adj[4 * i + 2], adj[4 * i + 3]};
        RectD r = adjust_rect(b, a);
        out[4 * i] = r.x; out[4 * i + 1] = r.y; out[4 * i + 2] = r.w; out[4 * i + 3] = r.h;
    }
}
void oracle_to_shade(const float *f, int32_t *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = to_shade(f[i]);
}
int oracle_grid_ops(int w, int h, const int32_t *xy, int n, int32_t *out) {
    if (w <= 0 || h <= 0 || w * h > MAX_GRID) return -1;
    Game *g = (Game *)calloc(1, sizeof(Game));
    g->grid_w = w;
    g->grid_h = h;
    g->out_of_bounds_object = -7;
    for (int i = 0; i < w * h; i++) g->grid[i] = 0; /* Grid::resize: value-initialised */
    int zeros = 0;
    for (int i = 0; i < w * h; i++) zeros += g->grid[i] == 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) set_obj(g, x, y, 3 * (y * w + x) + 1);
    for (int k = 0; k < n; k++) {
        const int x = xy[2 * k], y = xy[2 * k + 1];
        const int idx = y * w + x;
        out[5 * k + 0] = grid_contains(g, x, y);
        out[5 * k + 1] = get_obj(g, x, y);
        out[5 * k + 2] = idx;
        out[5 * k + 3] = idx % w; /* to_xy */
        out[5 * k + 4] = idx / w;
    }
    free(g);
    return zeros;
}

/* bigfish.cpp:84 fish radius through the C library's pow (the checker of the device pow) */
void oracle_bigfish_radius(const float *u, float *out, int64_t n) {
    for (int64_t i = 0; i < n; i++)
        out[i] = (float)((double)(BF_FISH_MAX_R - BF_FISH_MIN_R) * pow((double)u[i], 1.4) + (double)BF_FISH_MIN_R);
}

/* libm pins of the device's rotation math (tests/test_gpu_libm.py): the QTransform::rotate matrix of
 * draw_image (m11, m12, m21, m22 before the qFuzzyIsNull clean-up) for each entity rotation, and
 * -atan2f(dy, dx) of Entity::face_direction */
void oracle_qt_rotation(const float *rot, double *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        float deg = rot[i] * 180 / PI_F;
        QtXform t = qt_translate_rotate(0, 0, (double)deg);
        out[4 * i + 0] = t.m11; out[4 * i + 1] = t.m12; out[4 * i + 2] = t.m21; out[4 * i + 3] = t.m22;
    }
}
void oracle_face_rotation(const float *dxy, float *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = -1 * atan2f(dxy[2 * i + 1], dxy[2 * i]) + 0.0f;
}

/* MazeGen pin, same contract as oracle/ref_harness.cpp ref_mazegen */
int oracle_mazegen(int32_t seed, int maze_dim, int mode, int num_doors, int start_obj, int num_objs, int32_t *out,
                   uint32_t *next_draw) {
    static MazeGen m;
    MT r;
    rg_seed(&r, seed);
    mg_init(&m, &r, maze_dim);
    if (mode == 0) mg_generate_maze(&m);
    else if (mode == 1) mg_generate_maze_no_dead_ends(&m);
    else mg_generate_maze_with_doors(&m, num_doors);
    if (num_objs > 0) mg_place_objects(&m, start_obj, num_objs);
    int n = m.array_dim;
    for (int i = 0; i < n * n; i++) out[i] = m.grid[i];
    *next_draw = mt_next(&r);
    return n;
}

int oracle_qt_replay(const uint8_t *cmds, int64_t nbytes, uint32_t *canvas) {
    Rd r = {cmds, cmds + nbytes};
    uint32_t ncmds = rd_u32(&r);
    for (uint32_t k = 0; k < ncmds; k++) {
        uint32_t kind = rd_u32(&r);
        double x = rd_f64(&r), y = rd_f64(&r), w = rd_f64(&r), h = rd_f64(&r);
        double opacity = rd_f64(&r);
        uint32_t mirrored = rd_u32(&r);
        int32_t rot = (int32_t)rd_u32(&r);
        if (kind == 0) {
            uint32_t fmt = rd_u32(&r), iw = rd_u32(&r), ih = rd_u32(&r);
            const uint32_t *px = (const uint32_t *)r.p;
            r.p += 4 * (size_t)iw * ih;
            if (rot != 0) return -1;
            qt_draw_image(canvas, x, y, w, h, px, (int)iw, (int)ih, (int)fmt, mirrored != 0, opacity);
        } else if (kind == 3) { /* drawImage under translate(x + w/2, y + h/2) + rotate(deg) */
            double deg = rd_f64(&r);
            uint32_t fmt = rd_u32(&r), iw = rd_u32(&r), ih = rd_u32(&r);
            const uint32_t *px = (const uint32_t *)r.p;
            r.p += 4 * (size_t)iw * ih;
            if (fmt != QFMT_ARGB32_PM) return -3;
            qt_draw_image_rotated(canvas, x, y, w, h, deg, px, (int)iw, (int)ih, mirrored != 0, opacity);
        } else {
            uint32_t col = rd_u32(&r);
            if (kind == 2) qt_fill_rect_int(canvas, (int)x, (int)y, (int)w, (int)h, col);
            else if (kind == 1 && (col >> 24) == 0xff && opacity == 1.0) qt_fill_rectf(canvas, x, y, w, h, col);
            else return -2;
        }
    }
    return (int)(r.p - cmds);
}

/* diagnostic: type, image_type, rotation bits, rx bits, alpha bits of env i's entities (5 words each);
 * returns the entity count */
int oracle_entities(void *h, int i, int32_t *out, int max_ents) {
    Vec *v = (Vec *)h;
    Game *g = &v->games[i];
    int n = g->num_ents < max_ents ? g->num_ents : max_ents;
    for (int k = 0; k < n; k++) {
        Entity *e = &g->ents[k];
        out[5 * k] = e->type;
        out[5 * k + 1] = e->image_type;
        memcpy(&out[5 * k + 2], &e->rotation, 4);
        memcpy(&out[5 * k + 3], &e->rx, 4);
        memcpy(&out[5 * k + 4], &e->alpha, 4);
    }
    return g->num_ents;
}

/* ---- AssetGen pins (tests/test_assetgen_pins.py) */
/* mirror of ref_qt_shape (oracle/ref_qt_harness.cpp): kind 0 fillRect, 1 ellipse brush + pen,
 * 2 brush only, 3 pen only */
int oracle_qt_shape(int w, int h, int fmt, int kind, double x, double y, double rw, double rh, uint32_t c1, uint32_t c2,
                    int source, uint32_t *inout) {
    AgCanvas c = {inout, w, h, fmt, source};
    if (kind == 0) {
        ag_fill_rectf(&c, x, y, rw, rh, c1);
        return 0;
    }
    return ag_draw_ellipse(&c, x, y, rw, rh, c1, c2, kind == 1 ? 3 : (kind == 2 ? 1 : 2));
}
/* mirror of ref_qt_polyline: QCosmeticStroker::drawPath of a polyline (caps on an open path's ends) */
void oracle_qt_polyline(int w, int h, const double *pts, int n, uint32_t color, uint32_t *inout) {
    AgCanvas c = {inout, w, h, QFMT_RGB32, 0};
    CStroker s;
    s.c = &c;
    s.pm = qt_solid_premul(color);
    s.xmin = -1; s.xmax = w + 1; s.ymin = -1; s.ymax = h + 1;
    s.lastAxisAligned = false;
    s.lastDir = CS_L2R;
    s.lastx = CS_INT_MIN;
    s.lasty = CS_INT_MIN;
    const bool closed = pts[0] == pts[2 * (n - 1)] && pts[1] == pts[2 * (n - 1) + 1];
    if (closed) cs_last_point(&s, pts[2 * (n - 2)], pts[2 * (n - 2) + 1], pts[2 * (n - 1)], pts[2 * (n - 1) + 1]);
    int caps = closed ? CS_NOCAPS : CS_CAPBEGIN;
    for (int i = 1; i < n; i++) {
        if (!closed && i == n - 1) caps |= CS_CAPEND;
        cs_line(&s, pts[2 * (i - 1)], pts[2 * (i - 1) + 1], pts[2 * i], pts[2 * i + 1], caps);
        caps = CS_NOCAPS;
    }
}
/* mirror of ref_generate_resource: returns the generator's next randint() after painting, via *next */
int oracle_generate_resource(int32_t seed, int pre_draws, int w, int h, int fmt, int num_recurse, int blotch_scale,
                             int is_rect, uint32_t init, uint32_t *out, int32_t *next) {
    MT m;
    rg_seed(&m, seed);
    for (int i = 0; i < pre_draws; i++) rg_randint0(&m);
    for (size_t i = 0; i < (size_t)w * h; i++) out[i] = init;
    AgCanvas c = {out, w, h, fmt, 0};
    int rc = ag_generate_resource(&m, &c, num_recurse, blotch_scale, is_rect != 0);
    *next = rg_randint0(&m);
    return rc;
}
