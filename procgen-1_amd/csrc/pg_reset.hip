// pg_reset.hip -- Game::reset + level generation for the envs the step kernel queued
// (reference game.cpp:109-134, basic-abstract-game.cpp:767-806, games/coinrun.cpp:227-445).
//
// Persistent grid of 64-lane workgroups pulling env ids from the queue.  The
// freshly seeded rand_gen lives in LDS for the whole level build (hundreds of
// serial draws at LDS latency), the world grid is assembled in LDS with
// lane-parallel rectangle fills and written to HBM once.
#include "pg_device.h"

namespace {

struct RCtx {
    PGDev d;
    int env;
    PGEnv s;
    float *E;
    size_t plane, eb;
    uint32_t *mt;    // LDS rand_gen words
    int32_t mti;
    int16_t *grid;   // LDS grid
};

DEV float &EF(RCtx &c, int f, int slot) { return c.E[(size_t)f * c.plane + c.eb + slot]; }
DEV int &EI(RCtx &c, int f, int slot) { return reinterpret_cast<int *>(c.E)[(size_t)f * c.plane + c.eb + slot]; }

DEV uint32_t draw(RCtx &c) { return mt_next_lds(c.mt, c.mti); }
DEV int randn(RCtx &c, int n) { return rg_randn_of(draw(c), n); }
DEV float rand01(RCtx &c) { return rg_rand01_of(draw(c)); }

// Entity(x, y, vx, vy, rx, ry, type) (entity.cpp:8-47), appended to `entities`
DEV int add_entity_rxy(RCtx &c, float x, float y, float vx, float vy, float rx, float ry, int type) {
    int i = c.s.num_ents;
    if (i >= PG_CAP) {
        c.s.error = PG_ERR_ENTITY_OVERFLOW;
        return PG_CAP - 1;
    }
    c.s.num_ents = i + 1;
    float grow = 1.0f, decay = 1.0f;
    int expire = -1;
    if (type == EXPLOSION) {
        grow = 1.4f;
        expire = 4;
    } else if (type == TRAIL) {
        grow = 1.05f;
        decay = 0.8f;
    }
    EF(c, F_X, i) = x; EF(c, F_Y, i) = y; EF(c, F_VX, i) = vx; EF(c, F_VY, i) = vy;
    EF(c, F_RX, i) = rx; EF(c, F_RY, i) = ry; EF(c, F_ROTATION, i) = 0; EF(c, F_VROT, i) = 0;
    EF(c, F_ALPHA, i) = 1.0f; EF(c, F_ALPHA_DECAY, i) = decay; EF(c, F_GROW_RATE, i) = grow;
    EF(c, F_FRICTION, i) = 1; EF(c, F_COLLISION_MARGIN, i) = 0; EF(c, F_HEALTH, i) = 1;
    EF(c, F_THETA, i) = -100; EF(c, F_CLIMBER_SPAWN_X, i) = 0;
    EI(c, F_TYPE, i) = type; EI(c, F_IMAGE_TYPE, i) = type; EI(c, F_IMAGE_THEME, i) = 0;
    EI(c, F_RENDER_Z, i) = 0; EI(c, F_LIFE_TIME, i) = 0; EI(c, F_EXPIRE_TIME, i) = expire;
    EI(c, F_FIRE_TIME, i) = -1; EI(c, F_SPAWN_TIME, i) = -1; EI(c, F_FLAGS, i) = EF_AUTO_ERASE;
    return i;
}
DEV int add_entity(RCtx &c, float x, float y, float vx, float vy, float r, int type) {
    return add_entity_rxy(c, x, y, vx, vy, r, r, type);
}

// choose_random_theme (basic-abstract-game.cpp:1047-1050)
DEV void choose_random_theme(RCtx &c, int i) {
    int nt = c.d.num_themes[EI(c, F_IMAGE_TYPE, i)];
    EI(c, F_IMAGE_THEME, i) = randn(c, nt);
}

// grid (grid.h / basic-abstract-game.cpp:125-131, 180-185, 229-231) on the LDS copy
DEV int get_obj(RCtx &c, int x, int y) {
    if (!(0 <= y && y < c.s.main_height && 0 <= x && x < c.s.main_width)) return c.s.out_of_bounds_object;
    return c.grid[y * c.s.main_width + x];
}
DEV void set_obj(RCtx &c, int x, int y, int v) {
    if (!(0 <= y && y < c.s.main_height && 0 <= x && x < c.s.main_width)) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    if (LANE == 0) c.grid[y * c.s.main_width + x] = (int16_t)v;
    wave_sync();
}
DEV void fill_elem(RCtx &c, int x, int y, int dx, int dy, int elem) {
    int16_t v = (int16_t)(signed char)elem; // `char elem` narrowing (basic-abstract-game.cpp:125)
    int n = dx * dy;
    bool bad = false;
    for (int k = LANE; k < n; k += 64) {
        int j = k / dy, l = k % dy;
        int gx = x + j, gy = y + l;
        if (0 <= gy && gy < c.s.main_height && 0 <= gx && gx < c.s.main_width) c.grid[gy * c.s.main_width + gx] = v;
        else bad = true;
    }
    if (ballot(bad)) c.s.error = PG_ERR_GRID;
    wave_sync();
}

// ------------------------------------------------------------------ coinrun level generation
DEV void cr_fill_block_top(RCtx &c, int x, int y, int dx, int dy, int fill, int top) { // coinrun.cpp:227-231
    if (!(dy > 0)) c.s.error = PG_ERR_GRID;
    fill_elem(c, x, y, dx, dy - 1, fill);
    fill_elem(c, x, y + dy - 1, dx, 1, top);
}
DEV void cr_fill_ground_block(RCtx &c, int x, int y, int dx, int dy) { cr_fill_block_top(c, x, y, dx, dy, CR_WALL_MID, CR_WALL_TOP); }
DEV void cr_fill_lava_block(RCtx &c, int x, int y, int dx, int dy) { cr_fill_block_top(c, x, y, dx, dy, CR_LAVA_MID, CR_LAVA_TOP); }
DEV void cr_create_saw_enemy(RCtx &c, int x, int y) { // :248-250
    add_entity(c, (float)(x + .5), (float)(y + .5), 0, 0, (float).5, CR_SAW);
}
DEV void cr_create_enemy(RCtx &c, int x, int y) { // :252-258
    float vx = (float)(.15 * (randn(c, 2) * 2 - 1));
    int i = add_entity(c, (float)(x + .5), (float)(y + .5), vx, 0, (float).5, CR_ENEMY);
    EI(c, F_FLAGS, i) = EF_AUTO_ERASE | EF_SMART_STEP;
    EI(c, F_IMAGE_TYPE, i) = CR_ENEMY1;
    EI(c, F_RENDER_Z, i) = 1;
    choose_random_theme(c, i);
}
DEV void cr_create_crate(RCtx &c, int x, int y) { // :260-263
    int i = add_entity(c, (float)(x + .5), (float)(y + .5), 0, 0, (float).5, CR_CRATE);
    choose_random_theme(c, i);
}

DEV void cr_generate_coin_to_the_right(RCtx &c) { // coinrun.cpp:265-414
    int max_difficulty = 3;
    int dif = randn(c, max_difficulty) + 1;
    int num_sections = randn(c, dif) + dif;
    int curr_x = 5;
    int curr_y = 1;
    int pit_threshold = dif;
    int danger_type = randn(c, 3);
    bool allow_pit = (c.s.opt_debug_mode & (1 << 1)) == 0;
    bool allow_crate = (c.s.opt_debug_mode & (1 << 2)) == 0;
    bool allow_dy = (c.s.opt_debug_mode & (1 << 3)) == 0;
    int w = c.s.main_width;
    float _max_dy = c.s.max_jump * c.s.max_jump / (2 * c.s.gravity);
    float _max_dx = c.s.maxspeed * 2 * c.s.max_jump / c.s.gravity;
    int max_dy = (int)((double)_max_dy - .5);
    int max_dx = (int)((double)_max_dx - .5);
    bool allow_monsters = c.s.opt_distribution_mode != PG_EASY;

    for (int section_idx = 0; section_idx < num_sections; section_idx++) {
        if (curr_x + 15 >= w) break;
        int dy = randn(c, 4) + 1 + (int)(dif / 3);
        if (!allow_dy) dy = 0;
        if (dy > max_dy) dy = max_dy;
        if (curr_y >= 20) {
            dy *= -1;
        } else if (curr_y >= 5 && randn(c, 2) == 1) {
            dy *= -1;
        }
        int dx = randn(c, 2 * dif) + 3 + (int)(dif / 3);
        curr_y += dy;
        if (curr_y < 1) curr_y = 1;
        bool use_pit = allow_pit && (dx > 7) && (curr_y > 3) && (randn(c, 20) >= pit_threshold);
        if (use_pit) {
            int x1 = randn(c, 3) + 1;
            int x2 = randn(c, 3) + 1;
            int pit_width = dx - x1 - x2;
            if (pit_width > max_dx) {
                pit_width = max_dx;
                x2 = dx - x1 - pit_width;
            }
            cr_fill_ground_block(c, curr_x, 0, x1, curr_y);
            cr_fill_ground_block(c, curr_x + dx - x2, 0, x2, curr_y);
            int lava_height = randn(c, curr_y - 3) + 1;
            if (danger_type == 0) {
                cr_fill_lava_block(c, curr_x + x1, 1, pit_width, lava_height);
            } else if (danger_type == 1) {
                for (int ei = 0; ei < pit_width; ei++) cr_create_saw_enemy(c, curr_x + x1 + ei, 1);
            } else if (danger_type == 2) {
                for (int ei = 0; ei < pit_width; ei++) cr_create_enemy(c, curr_x + x1 + ei, 1);
            }
            if (pit_width > 4) {
                int x3, w1;
                if (pit_width == 5) {
                    x3 = 1 + randn(c, 2);
                    w1 = 1 + randn(c, 2);
                } else if (pit_width == 6) {
                    x3 = 2 + randn(c, 2);
                    w1 = 1 + randn(c, 2);
                } else {
                    x3 = 2 + randn(c, 2);
                    int x4 = 2 + randn(c, 2);
                    w1 = pit_width - x3 - x4;
                }
                cr_fill_ground_block(c, curr_x + x1 + x3, curr_y - 1, w1, 1);
            }
        } else {
            cr_fill_ground_block(c, curr_x, 0, dx, curr_y);
            int ob1_x = -1;
            int ob2_x = -1;
            if (randn(c, 10) < (2 * dif) && dx > 3) {
                ob1_x = curr_x + randn(c, dx - 2) + 1;
                cr_create_saw_enemy(c, ob1_x, curr_y);
            }
            if (randn(c, 10) < dif && dx > 3 && (max_dx >= 4) && allow_monsters) {
                ob2_x = curr_x + randn(c, dx - 2) + 1;
                cr_create_enemy(c, ob2_x, curr_y);
            }
            if (allow_crate) {
                for (int i = 0; i < 2; i++) {
                    int crate_x = curr_x + randn(c, dx - 2) + 1;
                    if (randn(c, 2) == 1 && ob1_x != crate_x && ob2_x != crate_x) {
                        int pile_height = randn(c, 3) + 1;
                        for (int j = 0; j < pile_height; j++) cr_create_crate(c, crate_x, curr_y + j);
                    }
                }
            }
        }
        if (!cr_is_wall(get_obj(c, curr_x - 1, curr_y))) set_obj(c, curr_x - 1, curr_y, CR_ENEMY_BARRIER);
        curr_x += dx;
        set_obj(c, curr_x, curr_y, CR_ENEMY_BARRIER);
    }
    set_obj(c, curr_x, curr_y, CR_GOAL);
    cr_fill_ground_block(c, curr_x, 0, 1, curr_y);
    fill_elem(c, curr_x + 1, 0, c.s.main_width - curr_x - 1, c.s.main_height, CR_WALL_MID);
}

DEV void coinrun_game_reset(RCtx &c) {
    // ---- BasicAbstractGame::game_reset (basic-abstract-game.cpp:767-806)
    c.s.bg_pct_x = rand01(c);
    if (c.s.main_width * c.s.main_height > PG_GRID_MAX) c.s.error = PG_ERR_GRID;
    fill_elem(c, 0, 0, c.s.main_width, c.s.main_height, 0); // grid.resize -> zeros
    c.s.background_index = randn(c, c.d.num_backgrounds);
    c.s.num_ents = 0;
    c.s.agent_erased = 0;
    float ax, ay;
    float a_r = 0.4f;
    if (c.s.random_agent_start) {
        ax = rand01(c) * (c.s.main_width - 2 * a_r) + a_r;
        ay = rand01(c) * (c.s.main_height - 2 * a_r) + a_r;
    } else {
        ax = a_r;
        ay = a_r;
    }
    int a = add_entity(c, ax, ay, 0, 0, a_r, PLAYER);
    EI(c, F_FLAGS, a) = EF_AUTO_ERASE | EF_SMART_STEP;
    EI(c, F_RENDER_Z, a) = 1;
    // erase_if_needed(): the agent spawns inside the world, nothing to erase
    fill_elem(c, 0, 0, c.s.main_width, c.s.main_height, SPACE);

    // ---- coinrun (coinrun.cpp:416-445)
    c.s.gravity = 0.2f;
    c.s.max_jump = 1.5f;
    c.s.air_control = 0.15f;
    c.s.maxspeed = .5f;
    c.s.has_support = 0;
    c.s.facing_right = 1;
    if (c.s.opt_distribution_mode == PG_EASY) {
        EI(c, F_IMAGE_THEME, 0) = 0;
        c.s.wall_theme = 0;
        c.s.background_index = 0;
    } else {
        choose_random_theme(c, 0);
        c.s.wall_theme = randn(c, 6);
    }
    float arx = .5f, ary = 0.5787f;
    EF(c, F_RX, 0) = arx;
    EF(c, F_RY, 0) = ary;
    EF(c, F_X, 0) = 1 + arx;
    float agent_y = 1 + ary;
    EF(c, F_Y, 0) = agent_y;
    c.s.last_agent_y = agent_y;
    c.s.is_on_crate = 0;
    // init_floor_and_walls (coinrun.cpp:241-246)
    fill_elem(c, 0, 0, c.s.main_width, 1, CR_WALL_TOP);
    fill_elem(c, 0, 0, 1, c.s.main_height, CR_WALL_MID);
    fill_elem(c, c.s.main_width - 1, 0, 1, c.s.main_height, CR_WALL_MID);
    fill_elem(c, 0, c.s.main_height - 1, c.s.main_width, 1, CR_WALL_MID);
    cr_generate_coin_to_the_right(c);
}

DEV void reset_env(PGDev &d, int env, uint32_t *lds_mt, int16_t *lds_grid, bool initial) {
    RCtx c;
    c.d = d;
    c.env = env;
    c.s = d.envs[env];
    c.E = d.ents;
    c.plane = (size_t)d.num_envs * PG_CAP;
    c.eb = (size_t)env * PG_CAP;
    c.mt = lds_mt;
    c.grid = lds_grid;
    uint32_t *rg = d.mt + (size_t)env * 2 * PG_MT_WORDS;
    uint32_t *lsg = rg + PG_MT_WORDS;

    // ---- Game::reset (game.cpp:109-134)
    c.s.reset_count++;
    if (c.s.episodes_remaining == 0) {
        if (c.s.opt_use_sequential_levels && c.s.sd_level_complete) {
            c.s.current_level_seed = (int32_t)((uint32_t)c.s.current_level_seed + 997u);
        } else {
            uint32_t x = mt_next_global(lsg, c.s.lsg_mti, lds_mt);
            c.s.current_level_seed = rg_randint_of(x, c.s.level_seed_low, c.s.level_seed_high);
        }
        c.s.episodes_remaining = 1;
    } else {
        c.s.sd_reward = 0;
        c.s.sd_done = 0;
        c.s.sd_level_complete = 0;
    }
    wave_sync();
    mt_seed_lds(lds_mt, (uint32_t)c.s.current_level_seed);
    c.mti = PG_MT_N;
    coinrun_game_reset(c);
    c.s.cur_time = 0;
    c.s.total_reward = 0;
    c.s.episodes_remaining -= 1;
    c.s.action = c.s.default_action;
    c.s.rg_mti = c.mti;

    // write the generator, the grid and the scalars back to HBM
    wave_sync();
    for (int i = LANE; i < PG_MT_N; i += 64) rg[i] = lds_mt[i];
    int cells = c.s.main_width * c.s.main_height;
    int16_t *g = d.grid + (size_t)env * PG_GRID_MAX;
    const uint4 *src = reinterpret_cast<const uint4 *>(lds_grid);
    uint4 *dst = reinterpret_cast<uint4 *>(g);
    for (int i = LANE; i < (cells + 7) / 8; i += 64) dst[i] = src[i];
    // int8 mirror for the step kernel (valid when every cell fits, always for coinrun)
    bool fits = true;
    int8_t *g8 = d.grid8 + (size_t)env * PG_GRID_MAX;
    for (int i = LANE; i < (cells + 15) / 16; i += 64) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t word = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                int cell = i * 16 + q * 4 + b;
                int v = cell < cells ? (int)lds_grid[cell] : 0;
                if (v < -128 || v > 127) fits = false;
                word |= (uint32_t)(uint8_t)v << (8 * b);
            }
            w[q] = word;
        }
        reinterpret_cast<uint4 *>(g8)[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    c.s.grid8_ok = ballot(!fits) == 0;
    if (LANE == 0) {
        d.level_seed[env] = c.s.current_level_seed;
        if (initial) { // first observation of set_buffers (vecgame.cpp:381-409): step_data from the ctor
            d.rew[env] = c.s.sd_reward;
            d.first[env] = (uint8_t)c.s.sd_done;
            d.prev_level_seed[env] = c.s.prev_level_seed;
            d.prev_level_complete[env] = (uint8_t)c.s.sd_level_complete;
        }
        if (c.s.error) atomicOr(d.error_any, 1 << c.s.error);
        d.envs[env] = c.s;
    }
    wave_sync();
}

} // namespace

// all_envs != 0: reset every env (initial reset of set_buffers); else drain the step kernel's queue.
extern "C" __global__ __launch_bounds__(64) void pg_reset_kernel(PGDev d, int all_envs) {
    __shared__ uint32_t lds_mt[PG_MT_N];
    __shared__ __attribute__((aligned(16))) int16_t lds_grid[PG_GRID_MAX];
    int count = all_envs ? d.num_envs : *d.reset_count;
    for (int q = blockIdx.x; q < count; q += gridDim.x) {
        int env = all_envs ? q : d.reset_queue[q];
        reset_env(d, env, lds_mt, lds_grid, all_envs != 0);
    }
}

extern "C" void pg_launch_reset(const PGDev *d, hipStream_t s, int all_envs, int grid) {
    int g = grid > 0 ? grid : (d->num_envs < 4096 ? d->num_envs : 4096);
    hipLaunchKernelGGL(pg_reset_kernel, dim3(g), dim3(64), 0, s, *d, all_envs);
}
