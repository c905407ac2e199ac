// pg_reset.hip -- Game::reset + level generation for the envs the step kernel queued
// (reference game.cpp:109-134, basic-abstract-game.cpp:767-806; games/coinrun.cpp:227-445,
// bigfish.cpp:62-78, maze.cpp:45-105, heist.cpp:98-203; mazegen.cpp:12-306).
//
// Persistent grid of 64-lane workgroups pulling env ids from the game's queue.  The
// freshly seeded rand_gen lives in LDS for the whole level build (hundreds of serial draws
// at LDS latency), the world grid is assembled in LDS with lane-parallel rectangle fills and
// written to HBM once.  MazeGen runs in LDS too: Kruskal's order-preserving wall erase is a
// select-the-n-th-live-bit over a wall bitmap, set union a lane-parallel relabel, and the
// std::set BFS of expand_to_type a lane-parallel frontier over cell bytes that honours the
// reference's ascending visiting order and early return.
#include "pg_device.h"
#include "pg_assetgen.h"

namespace {

// LDS scratch for MazeGen (maze / heist): array_dim <= 33 (memory-mode maze, world 31)
#define MG_MAX_DIM 33
#define MG_MAX_CELLS (MG_MAX_DIM * MG_MAX_DIM)
#define MG_MAX_WALLS 512
struct MGScratch {
    int16_t grid[MG_MAX_CELLS];        // Grid<int> array_dim x array_dim
    int16_t labels[MG_MAX_CELLS];      // cell_sets_idxs (maze cell maze_dim*y+x)
    int16_t free_cells[MG_MAX_CELLS];  // free_cells, in insertion order
    int16_t list[MG_MAX_CELLS];        // forks / space cells / choose_n scratch
    uint8_t in_free[MG_MAX_CELLS];     // free_cell_set
    uint8_t s0[MG_MAX_CELLS], s1[MG_MAX_CELLS], curr[MG_MAX_CELLS], next[MG_MAX_CELLS];
    uint32_t walls[MG_MAX_WALLS];      // x1 | y1 << 8 | x2 << 16 | y2 << 24, reference push order
    unsigned long long alive[MG_MAX_WALLS / 64];
};
struct MinerScratch {
    int16_t obj_idxs[35 * 35];  // simple_choose result
    int16_t dirt[35 * 35];      // dirt cells, then exit candidates
    uint8_t taken[35 * 35];     // simple_choose's std::set
};
// leaper's level build steps every entity ~300 times before the first frame (leaper.cpp:174-177):
// the entity list lives in LDS for those steps (slot 0 = the agent) and goes to HBM once
struct LeaperScratch {
    float x[PG_CAP], y[PG_CAP], vx[PG_CAP], rx[PG_CAP], ry[PG_CAP];
    int16_t born[PG_CAP];
    int8_t theme[PG_CAP], type[PG_CAP];
    float road[8], water[8]; // lane speeds (copied into PGEnv with static indices)
};
struct ChaserScratch {
    MGScratch mg;
    int16_t sel[8]; // simple_choose picks
};
template <int G> struct Scratch { uint32_t dummy[1]; };
template <> struct Scratch<PG_GAME_CHASER> { ChaserScratch ch; };
template <> struct Scratch<PG_GAME_FRUITBOT> { int16_t part[16]; };
template <> struct Scratch<PG_GAME_DODGEBALL> { float4 rooms[64]; }; // QRectF x, y, w, h
// starpilot's spawners in generation order (at most 49 groups x 6, starpilot.cpp:226-327), then the
// std::sort permutation and its explicit introsort stack
#define SP_MAX_SPAWNERS 320
struct SpawnerScratch {
    float x[SP_MAX_SPAWNERS], y[SP_MAX_SPAWNERS], vx[SP_MAX_SPAWNERS], vy[SP_MAX_SPAWNERS];
    float r[SP_MAX_SPAWNERS], ry[SP_MAX_SPAWNERS], rot[SP_MAX_SPAWNERS], health[SP_MAX_SPAWNERS];
    int16_t type[SP_MAX_SPAWNERS], theme[SP_MAX_SPAWNERS], fire[SP_MAX_SPAWNERS], spawn[SP_MAX_SPAWNERS];
    int8_t rz[SP_MAX_SPAWNERS];
    int16_t idx[SP_MAX_SPAWNERS];
    int16_t stack[3 * 64];
};
template <> struct Scratch<PG_GAME_STARPILOT> { SpawnerScratch sp; };
// caveflyer's RoomGenerator (roomgen.cpp) over the LDS grid (world up to 60 x 60, memory mode)
struct CaveScratch {
    int16_t a[PG_GRID_MAX];         // CA next cells, then component labels, then BFS parent cells
    int32_t b[PG_GRID_MAX];         // component sizes, then BFS discovery keys, then picks
    int16_t list[PG_GRID_MAX + 1];  // BFS frontier, then free cells
    int16_t list2[PG_GRID_MAX + 1]; // next frontier, then the goal path
    uint8_t f[PG_GRID_MAX];         // CF_* bits per cell
    uint32_t pm[2 * 64];            // the goal path as row masks (cf_rows_of_path)
};
template <> struct Scratch<PG_GAME_CAVEFLYER> { CaveScratch cf; };
// jumper: MazeGen first (its grid is read by the random fill), then the RoomGenerator
template <> struct Scratch<PG_GAME_JUMPER> { union { MGScratch mg; CaveScratch cf; }; };
template <> struct Scratch<PG_GAME_LEAPER> { LeaperScratch lp; };
template <> struct Scratch<PG_GAME_MINER> { MinerScratch mn; };
template <> struct Scratch<PG_GAME_MAZE> { MGScratch mg; };
template <> struct Scratch<PG_GAME_HEIST> { MGScratch mg; };

struct RCtx {
    PGDev d;
    int env;
    PGEnv &s;        // the env's scalars, staged in LDS for the whole reset (wave-uniform: keeping
                     // the 512-B struct in VGPRs cost ~128 registers and scratch spills)
    char *Eb;        // this env's entity block (pg_ent_index)
    uint32_t *mt;    // LDS rand_gen words
    int32_t mti;
    // the next draws, tempered, one per lane: lane k holds mt[wbase + k] (draw() reads it with readlane;
    // a sweep that reads mt words itself and twists must call mt_window_reset)
    uint32_t win;
    int32_t wbase;
    int16_t *grid;   // LDS grid
    AgLds *ag;       // AssetGen scratch (use_generated_assets kernels only, else null)
#ifdef PG_PROF_RESET
    uint64_t last;   // diagnostic build (VARIANT=rprof EXTRA=-DPG_PROF_RESET): level-generation phases
#endif
};

// Diagnostic phase stamps of a level generation (scripts/reset_phases.py): cycles since the previous
// stamp added to prof[env][8 + k]; prof[env][0] counts the resets.  Nothing in the product build.
#ifdef PG_PROF_RESET
#define RMARK(c, k)                                                                          \
    do {                                                                                     \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                    \
        if (LANE == 0) (c).d.prof[(size_t)(c).env * 16 + 8 + (k)] += t_ - (c).last;          \
        (c).last = t_;                                                                       \
    } while (0)
#else
#define RMARK(c, k) ((void)0)
#endif

DEV uint32_t ent_off(int f, int slot) { return (uint32_t)(f * PG_CAP + slot) * 4u; }
DEV float &EF(RCtx &c, int f, int slot) { return *reinterpret_cast<float *>(c.Eb + ent_off(f, slot)); }
DEV int &EI(RCtx &c, int f, int slot) { return *reinterpret_cast<int *>(c.Eb + ent_off(f, slot)); }

#define MT_WIN_NONE (-(1 << 20))
DEV void mt_window_reset(RCtx &c) { c.wbase = MT_WIN_NONE; }
// mt_next_lds with a register window: one LDS read + temper per 64 draws instead of a dependent LDS
// read per draw (level generators draw serially: leaper's build loop, the maze generators, simple_choose)
DEV uint32_t draw(RCtx &c) {
    if (c.mti >= PG_MT_N) {
        mt_twist_lds(c.mt);
        c.mti = 0;
        c.wbase = MT_WIN_NONE;
    }
    int k = c.mti - c.wbase;
    if (k < 0 || k >= 64) {
        c.wbase = c.mti;
        k = 0;
        c.win = c.mti + LANE < PG_MT_N ? mt_temper(c.mt[c.mti + LANE]) : 0u;
    }
    c.mti += 1;
    return (uint32_t)__builtin_amdgcn_readlane((int)c.win, k);
}
struct RCtxRng { // the env's rand_gen as AssetGen's generator (AssetGen bggen(&rand_gen))
    RCtx *c;
    DEV uint32_t next() { return draw(*c); }
};
DEV int randn(RCtx &c, int n) { return rg_randn_of(draw(c), n); }
DEV float rand01(RCtx &c) { return rg_rand01_of(draw(c)); }

// Entity(x, y, vx, vy, rx, ry, type) (entity.cpp:8-47), appended to `entities`
DEV int add_entity_rxy(RCtx &c, float x, float y, float vx, float vy, float rx, float ry, int type) {
    int i = c.s.num_ents;
    if (i >= PG_CAP) {
        c.s.error = PG_ERR_ENTITY_OVERFLOW;
        return PG_CAP - 1;
    }
    if (i >= PG_CAP - c.s.num_tail) {
        c.s.error = PG_ERR_ENTITY_OVERFLOW;
        return PG_CAP - c.s.num_tail - 1;
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

// match_aspect_ratio (basic-abstract-game.cpp:1023-1033, match_width): ry = rx / aspect ratio of
// the image loaded for the slot (mask_theme_if_necessary, :454-462; heist keeps KEY / LOCKED_DOOR
// themes, heist.cpp:42-44)
template <int G>
DEV void match_aspect_ratio(RCtx &c, int i) {
    int type = EI(c, F_IMAGE_TYPE, i), theme = EI(c, F_IMAGE_THEME, i);
    bool preserve = (G == PG_GAME_HEIST && (type == HS_KEY || type == HS_LOCKED_DOOR)) ||
                    (G == PG_GAME_PLUNDER && type == PL_SHIP); // plunder.cpp:83-85
    if (c.s.opt_restrict_themes && !preserve) theme = 0;
    int4 sp = reinterpret_cast<const int4 *>(c.d.sprites)[type + theme * MAX_ASSETS];
    if (sp.y <= 0 || sp.z <= 0) {
        c.s.error = PG_ERR_BAD_OPTION;
        return;
    }
    float ar = (float)(sp.y * 1.0 / sp.z);
    EF(c, F_RY, i) = EF(c, F_RX, i) / ar;
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
    int n = (dx > 0 && dy > 0) ? dx * dy : 0; // the reference loops run dx x dy times
    if (x == 0 && y == 0 && dx == c.s.main_width && dy == c.s.main_height) { // the whole grid: no index math
        for (int k = LANE; k < n && k < PG_GRID_MAX; k += 64) c.grid[k] = v;
        wave_sync();
        return;
    }
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

// ------------------------------------------------------------------ BasicAbstractGame::game_reset
template <int G>
DEV void choose_world_dim(RCtx &c) {
    if constexpr (G == PG_GAME_MAZE) { // maze.cpp:45-58
        int d = c.s.opt_distribution_mode;
        if (d == PG_EASY) c.s.world_dim = 15;
        else if (d == PG_HARD) c.s.world_dim = 25;
        else if (d == PG_MEMORY) c.s.world_dim = 31;
        c.s.main_width = c.s.world_dim;
        c.s.main_height = c.s.world_dim;
    }
    if constexpr (G == PG_GAME_CLIMBER) { // climber.cpp:263-266
        c.s.main_width = c.s.opt_distribution_mode == PG_EASY ? 16 : 20;
        c.s.main_height = 64;
    }
    if constexpr (G == PG_GAME_MINER) { // miner.cpp:119-132
        int d = c.s.opt_distribution_mode;
        if (d == PG_EASY) { c.s.main_width = 10; c.s.main_height = 10; }
        else if (d == PG_HARD) { c.s.main_width = 20; c.s.main_height = 20; }
        else if (d == PG_MEMORY) { c.s.main_width = 35; c.s.main_height = 35; }
        c.s.main_area = c.s.main_width * c.s.main_height;
    }
    if constexpr (G == PG_GAME_DODGEBALL) { // dodgeball.cpp:248-257
        const int world_dim = c.s.opt_distribution_mode == PG_MEMORY ? 40 : 20;
        c.s.main_width = world_dim;
        c.s.main_height = world_dim;
    }
    if constexpr (G == PG_GAME_FRUITBOT) { // fruitbot.cpp:144-152
        c.s.main_width = c.s.opt_distribution_mode == PG_EASY ? 10 : 20;
        c.s.main_height = 60;
    }
    if constexpr (G == PG_GAME_LEAPER) { // leaper.cpp:103-113
        int d = c.s.opt_distribution_mode;
        int world_dim = 20;
        if (d == PG_EASY) world_dim = 9;
        else if (d == PG_HARD) world_dim = 15;
        c.s.main_width = world_dim;
        c.s.main_height = world_dim;
    }
    if constexpr (G == PG_GAME_CAVEFLYER) { // caveflyer.cpp:128-143
        int d = c.s.opt_distribution_mode, world_dim = 20;
        if (d == PG_EASY) world_dim = 30;
        else if (d == PG_HARD) world_dim = 40;
        else if (d == PG_MEMORY) world_dim = 60;
        c.s.main_width = world_dim;
        c.s.main_height = world_dim;
    }
    if constexpr (G == PG_GAME_HEIST) { // heist.cpp:98-113
        int d = c.s.opt_distribution_mode;
        if (d == PG_EASY) c.s.world_dim = 9;
        else if (d == PG_HARD) c.s.world_dim = 13;
        else if (d == PG_MEMORY) c.s.world_dim = 23;
        c.s.maxspeed = .75f;
        c.s.main_width = c.s.world_dim;
        c.s.main_height = c.s.world_dim;
    }
}

template <int G>
DEV void base_game_reset(RCtx &c) { // basic-abstract-game.cpp:767-806
    choose_world_dim<G>(c);
    c.s.bg_pct_x = rand01(c);
    if (c.s.main_width * c.s.main_height > PG_GRID_MAX || c.s.main_width <= 0 || c.s.main_height <= 0)
        c.s.error = PG_ERR_GRID;
    fill_elem(c, 0, 0, c.s.main_width, c.s.main_height, 0); // grid.resize -> zeros
    c.s.background_index = randn(c, c.d.num_backgrounds);
    if (c.ag) { // use_procgen_background: bggen.generate_resource(bg) with rand_gen (:778-782)
        wave_sync();
        AgPainter<RCtxRng> p{c.d.gen_bg + (size_t)c.env * AG_BG_DIM * AG_BG_DIM, AG_BG_DIM, AG_BG_DIM, AG_FMT_RGB32, 0,
                             c.ag, RCtxRng{&c}, 0};
        ag_generate_resource(p, 1, 50, true);
        if (p.err) {
            c.s.error = PG_ERR_ASSETGEN;
            if (LANE == 0) atomicOr(c.d.error_any, p.err << 16);
        }
        wave_sync();
    }
    c.s.num_ents = 0;
    c.s.num_tail = 0;
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


DEV void coinrun_game_reset(RCtx &c) { // coinrun.cpp:416-445
    base_game_reset<PG_GAME_COINRUN>(c);
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

// ------------------------------------------------------------------ bigfish (bigfish.cpp:62-78)
DEV void bigfish_game_reset(RCtx &c) {
    base_game_reset<PG_GAME_BIGFISH>(c);
    c.s.opt_center_agent = 0;
    c.s.fish_eaten = 0;
    float start_r = .5f;
    if (c.s.opt_distribution_mode == PG_EASY) start_r = 1;
    c.s.r_inc = (BF_FISH_MAX_R - start_r) / BF_FISH_QUOTA;
    EF(c, F_RX, 0) = start_r;
    EF(c, F_RY, 0) = start_r;
    EF(c, F_Y, 0) = 1 + start_r;
}

// ------------------------------------------------------------------ MazeGen (mazegen.cpp)
struct MG {
    MGScratch *m;
    int md, ad; // maze_dim, array_dim
    int num_free;
};

DEV int mg_get_obj(const MG &g, int idx) { // :36-47
    int x = idx % g.ad, y = idx / g.ad;
    if (x <= 0 || x >= g.ad - 1) return INVALID_OBJ;
    if (y <= 0 || y >= g.ad - 1) return INVALID_OBJ;
    return g.m->grid[idx];
}
// get_neighbors (:49-67) in the reference's order: (-1,0) (0,-1) (0,1) (1,0)
DEV int mg_first_neighbor(const MG &g, int idx, int type) {
    const int nb[4] = {idx - 1, idx - g.ad, idx + g.ad, idx + 1};
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (mg_get_obj(g, nb[k]) == type) return nb[k];
    return -1;
}
DEV int mg_count_neighbors(const MG &g, int idx, int type) {
    return (mg_get_obj(g, idx - 1) == type) + (mg_get_obj(g, idx - g.ad) == type) + (mg_get_obj(g, idx + g.ad) == type) +
           (mg_get_obj(g, idx + 1) == type);
}
DEV int mg_nth_neighbor(const MG &g, int idx, int type, int n) {
    const int nb[4] = {idx - 1, idx - g.ad, idx + g.ad, idx + 1};
    for (int k = 0; k < 4; k++)
        if (mg_get_obj(g, nb[k]) == type && n-- == 0) return nb[k];
    return -1;
}
DEV void mg_set_index(const MG &g, int idx, int v) {
    if (LANE == 0) g.m->grid[idx] = (int16_t)v;
    wave_sync();
}

DEV void mg_set_free_cell(MG &g, int x, int y) { // :26-34 (uniform; lane 0 writes)
    int cell = g.md * y + x;
    bool was = g.m->in_free[cell] != 0;
    wave_sync();
    if (LANE == 0) {
        g.m->grid[(y + 1) * g.ad + (x + 1)] = SPACE;
        if (!was) {
            g.m->free_cells[g.num_free] = (int16_t)cell;
            g.m->in_free[cell] = 1;
        }
    }
    if (!was) g.num_free += 1;
    wave_sync();
}

// index of the n-th (0-based) set bit of the `words`-word bitmap `alive` (uniform)
DEV int nth_alive(const unsigned long long *alive, int words, int n) {
    for (int w = 0; w < words; w++) {
        unsigned long long a = alive[w];
        int cnt = __popcll(a);
        if (n < cnt) {
            bool mine = ((a >> LANE) & 1ull) && __popcll(a & ((1ull << LANE) - 1ull)) == n;
            return w * 64 + (__ffsll((long long)ballot(mine)) - 1);
        }
        n -= cnt;
    }
    return -1;
}

DEV void mg_generate_maze(RCtx &c, MG &g) { // :112-188
    const int md = g.md, ad = g.ad;
    MGScratch *m = g.m;
    for (int i = LANE; i < ad * ad; i += 64) m->grid[i] = WALL_OBJ;
    for (int i = LANE; i < md * md; i += 64) {
        m->labels[i] = (int16_t)i;
        m->in_free[i] = 0;
    }
    wave_sync();
    if (LANE == 0) m->grid[1 * ad + 1] = 0; // grid.set(MAZE_OFFSET, MAZE_OFFSET, 0)
    g.num_free = 0;
    // wall list in push order: first i odd in [1, md - 2] (x), j even; then i even, j odd in [1, md - 2]
    const int A = (md - 1) / 2, B = (md + 1) / 2;
    const int nw1 = A * B, nw = 2 * A * B;
    if (nw > MG_MAX_WALLS) c.s.error = PG_ERR_GRID; // also right for an even maze_dim (jumper easy: 6)
    for (int k = LANE; k < nw; k += 64) {
        int x1, y1, x2, y2;
        if (k < nw1) {
            int i = 2 * (k / B) + 1, j = 2 * (k % B);
            x1 = i - 1; y1 = j; x2 = i + 1; y2 = j;
        } else {
            int q = k - nw1;
            int i = 2 * (q / A), j = 2 * (q % A) + 1;
            x1 = i; y1 = j - 1; x2 = i; y2 = j + 1;
        }
        m->walls[k] = (uint32_t)x1 | ((uint32_t)y1 << 8) | ((uint32_t)x2 << 16) | ((uint32_t)y2 << 24);
    }
    // The loop below keeps its state in registers (one dependent LDS read per wall instead of ~10):
    //   the live-wall bitmap: lane w holds word w (walls.erase = clearing the bit, the n-th live wall =
    //   the n-th set bit, which is what the reference's vector erase leaves at position n);
    //   the set labels of the room cells (x, y even; the only cells whose labels are compared): room
    //   cell r = (y / 2) * R + x / 2 in lane r % 64, register r / 64, labels = room-cell numbers (the
    //   reference's cell indices, renamed: only their equality matters); merging s0 into s1 relabels
    //   every member.  The wall list itself is the push-order formula above.
    const int words = (nw + 63) / 64;
    uint64_t aw = 0;
    if (LANE < words) {
        const int left = nw - LANE * 64;
        aw = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
    }
    const int R = (md + 1) / 2;
    constexpr int LS = (((MG_MAX_DIM + 1) / 2) * ((MG_MAX_DIM + 1) / 2) + 63) / 64;
    int lab[LS];
#pragma unroll
    for (int j = 0; j < LS; j++) lab[j] = j * 64 + LANE;
    auto label_of = [&](int r) { // uniform room cell -> its label
        int v = lab[0];
#pragma unroll
        for (int j = 1; j < LS; j++)
            if ((r >> 6) == j) v = lab[j];
        return __builtin_amdgcn_readlane(v, r & 63);
    };
    // the packed wall list (x1 | y1 << 8 | x2 << 16 | y2 << 24) in registers: wall k in lane k % 64
    constexpr int WS = MG_MAX_WALLS / 64;
    uint32_t wreg[WS];
#pragma unroll
    for (int j = 0; j < WS; j++) wreg[j] = j * 64 + LANE < nw ? m->walls[j * 64 + LANE] : 0u;
    int freed = 0; // bit j: room cell j * 64 + LANE is in free_cell_set
    auto freed_of = [&](int r) { return (__builtin_amdgcn_readlane(freed, r & 63) >> (r >> 6)) & 1; };
    int nfree = g.num_free;
    for (int rem = nw; rem > 0; rem--) {
        int n = randn(c, rem), k = -1;
        for (int w = 0; w < words; w++) { // nth_alive over the register words
            const uint64_t a = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)aw, w) |
                               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(aw >> 32), w) << 32);
            const int cnt = __popcll(a);
            if (n < cnt) {
                const bool mine = ((a >> LANE) & 1ull) && __popcll(a & ((1ull << LANE) - 1ull)) == n;
                k = w * 64 + (__ffsll((long long)ballot(mine)) - 1);
                break;
            }
            n -= cnt;
        }
        if (LANE == (k >> 6)) aw &= ~(1ull << (k & 63)); // walls.erase(walls.begin() + n)
        uint32_t wv = wreg[0];
#pragma unroll
        for (int j = 1; j < WS; j++)
            if ((k >> 6) == j) wv = wreg[j];
        wv = (uint32_t)__builtin_amdgcn_readlane((int)wv, k & 63);
        const int x1 = wv & 255, y1 = (wv >> 8) & 255, x2 = (wv >> 16) & 255, y2 = wv >> 24;
        const int r1 = (y1 / 2) * R + x1 / 2, r2 = (y2 / 2) * R + x2 / 2;
        const int s0 = label_of(r1), s1 = label_of(r2);
        const int x0 = (x1 + x2) / 2, y0 = (y1 + y2) / 2;
        // the reference also requires the wall cell to be WALL_OBJ: it always is here (a wall cell is
        // only ever opened by its own wall, which is erased when picked)
        if (s0 != s1) {
            // set_free_cell (:26-34) of (x1, y1), (x0, y0), (x2, y2) in that order: the wall cell is
            // never in the set yet, the room cells' membership is the `freed` bits
            const bool new1 = !freed_of(r1), new2 = !freed_of(r2);
            if (LANE == 0) {
                m->grid[(y1 + 1) * ad + (x1 + 1)] = SPACE;
                m->grid[(y0 + 1) * ad + (x0 + 1)] = SPACE;
                m->grid[(y2 + 1) * ad + (x2 + 1)] = SPACE;
                int q = nfree;
                if (new1) m->free_cells[q++] = (int16_t)(md * y1 + x1);
                m->free_cells[q++] = (int16_t)(md * y0 + x0);
                if (new2) m->free_cells[q] = (int16_t)(md * y2 + x2);
            }
            nfree += (int)new1 + 1 + (int)new2;
            if (LANE == (r1 & 63)) freed |= 1 << (r1 >> 6);
            if (LANE == (r2 & 63)) freed |= 1 << (r2 >> 6);
#pragma unroll
            for (int j = 0; j < LS; j++) lab[j] = lab[j] == s0 ? s1 : lab[j]; // s1 |= s0
            wave_sync();
        }
    }
    g.num_free = nfree;
}

DEV void mg_place_objects(RCtx &c, MG &g, int start_obj, int num_objs) { // :292-306
    for (int j = 0; j < num_objs; j++) {
        int mm = randn(c, g.num_free);
        while (g.m->free_cells[mm] == -1 || g.m->free_cells[mm] == 0) mm = randn(c, g.num_free);
        int coin_cell = g.m->free_cells[mm];
        wave_sync();
        if (LANE == 0) {
            g.m->free_cells[mm] = -1;
            g.m->grid[(coin_cell / g.md + 1) * g.ad + (coin_cell % g.md + 1)] = (int16_t)(start_obj + j);
        }
        wave_sync();
    }
}

// Compact the ascending indices i < n with pred(i) into g.m->list; returns the count.
template <typename P>
DEV int mg_compact(const MG &g, int n, P pred) {
    int cnt = 0;
    for (int base = 0; base < n; base += 64) {
        int i = base + LANE;
        bool in = i < n && pred(i);
        unsigned long long b = ballot(in);
        if (in) g.m->list[cnt + __popcll(b & ((1ull << LANE) - 1ull))] = (int16_t)i;
        cnt += __popcll(b);
    }
    wave_sync();
    return cnt;
}

// expand_to_type (:69-98).  The reference walks `curr` (a std::set) in ascending order, adds
// every unseen SPACE neighbour to next/s1, and returns the first `type` neighbour of the first
// element that has one -- after that element's own additions.  So one BFS layer = (1) the
// smallest curr element e* with a `type` neighbour, (2) s1/next |= unseen SPACE neighbours of
// curr elements <= e*, computed per cell.  Every curr / s1 element is an interior cell.
DEV int mg_expand_to_type(MG &g, int type) {
    MGScratch *m = g.m;
    const int cells = g.ad * g.ad;
    for (int i = LANE; i < cells; i += 64) m->curr[i] = m->s0[i];
    wave_sync();
    bool any = true;
    while (any) {
        int estar = 0x7fffffff;
        for (int base = 0; base < cells; base += 64) {
            int i = base + LANE;
            bool has = i < cells && m->curr[i] && mg_first_neighbor(g, i, type) >= 0;
            unsigned long long b = ballot(has);
            if (b) {
                estar = base + __ffsll((long long)b) - 1;
                break;
            }
        }
        bool nonempty = false;
        for (int base = 0; base < cells; base += 64) {
            int j = base + LANE;
            bool add = false;
            if (j < cells) {
                m->next[j] = 0;
                if (mg_get_obj(g, j) == SPACE && !m->s0[j] && !m->s1[j]) {
                    const int nb[4] = {j - 1, j - g.ad, j + g.ad, j + 1};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        int e = nb[k];
                        if (e >= 0 && e < cells && e <= estar && m->curr[e]) add = true;
                    }
                }
                if (add) {
                    m->next[j] = 1;
                    m->s1[j] = 1;
                }
            }
            nonempty = nonempty || ballot(add) != 0;
        }
        wave_sync();
        if (estar != 0x7fffffff) return mg_first_neighbor(g, estar, type);
        for (int i = LANE; i < cells; i += 64) m->curr[i] = m->next[i];
        wave_sync();
        any = nonempty;
    }
    return -1;
}

DEV void mg_generate_maze_with_doors(RCtx &c, MG &g, int num_doors) { // :213-290
    mg_generate_maze(c, g);
    MGScratch *m = g.m;
    const int cells = g.ad * g.ad;
    int nf = mg_compact(g, cells, [&](int i) { return mg_get_obj(g, i) == SPACE && mg_count_neighbors(g, i, SPACE) > 2; });
    // choose_n (randgen.cpp:49-68): order-preserving erase from the fork list = n-th live bit
    int chosen[4];
    int nc = 0;
    if (num_doors > nf) {
        for (int i = 0; i < nf && i < 4; i++) chosen[nc++] = m->list[i];
        if (nf > 4) c.s.error = PG_ERR_GRID;
    } else {
        const int words = (nf + 63) / 64;
        for (int w = LANE; w < words; w += 64) {
            int left = nf - w * 64;
            m->alive[w] = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
        }
        wave_sync();
        for (int rem = nf; nc < num_doors; rem--) {
            int k = nth_alive(m->alive, words, randn(c, rem));
            chosen[nc++] = m->list[k];
            wave_sync();
            if (LANE == 0) m->alive[k >> 6] &= ~(1ull << (k & 63));
            wave_sync();
        }
    }
    num_doors = nc;
    for (int i = 0; i < nc; i++) mg_set_index(g, chosen[i], DOOR_OBJ);
    int ns = mg_compact(g, cells, [&](int i) { return mg_get_obj(g, i) == SPACE; });
    int agent_cell;
    do {
        if (ns <= 0) {
            c.s.error = PG_ERR_GRID;
            return;
        }
        agent_cell = m->list[randn(c, ns)];
    } while (mg_first_neighbor(g, agent_cell, DOOR_OBJ) >= 0);
    mg_set_index(g, agent_cell, AGENT_OBJ);
    for (int i = LANE; i < cells; i += 64) m->s0[i] = i == agent_cell;
    wave_sync();
    for (int door_num = 0; door_num < num_doors + 1; door_num++) {
        for (int i = LANE; i < cells; i += 64) m->s1[i] = 0;
        wave_sync();
        int found_door = -1;
        if (door_num < num_doors) {
            found_door = mg_expand_to_type(g, DOOR_OBJ);
            if (found_door < 0) {
                c.s.error = PG_ERR_GRID;
                return;
            }
            mg_set_index(g, found_door, DOOR_OBJ + door_num + 1);
            for (int i = LANE; i < cells; i += 64) m->s0[i] |= m->s1[i];
            wave_sync();
        }
        mg_expand_to_type(g, -999);
        int nsp = mg_compact(g, cells, [&](int i) { return m->s1[i] != 0; });
        if (nsp <= 0) {
            c.s.error = PG_ERR_GRID;
            return;
        }
        int key_cell = m->list[randn(c, nsp)];
        mg_set_index(g, key_cell, door_num == num_doors ? EXIT_OBJ : (KEY_OBJ + door_num + 1));
        for (int i = LANE; i < cells; i += 64) m->s0[i] |= m->s1[i];
        wave_sync();
        if (found_door >= 0) {
            if (LANE == 0) m->s0[found_door] = 1;
            wave_sync();
        }
    }
}

// ------------------------------------------------------------------ maze (maze.cpp:60-105)
DEV void maze_game_reset(RCtx &c, MGScratch *scratch) {
    base_game_reset<PG_GAME_MAZE>(c);
    c.s.grid_step = 1;
    c.s.maze_dim = randn(c, (c.s.world_dim - 1) / 2) * 2 + 3;
    int margin = (c.s.world_dim - c.s.maze_dim) / 2;
    MG g;
    g.m = scratch;
    g.md = c.s.maze_dim;
    g.ad = g.md + 2;
    if (g.ad > MG_MAX_DIM) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    c.s.opt_center_agent = c.s.opt_distribution_mode == PG_MEMORY;
    EF(c, F_RX, 0) = .5f;
    EF(c, F_RY, 0) = .5f;
    EF(c, F_X, 0) = (float)(margin + .5);
    EF(c, F_Y, 0) = (float)(margin + .5);
    mg_generate_maze(c, g);
    mg_place_objects(c, g, MZ_GOAL, 1);
    const int w = c.s.main_width;
    for (int i = LANE; i < w * c.s.main_height; i += 64) c.grid[i] = WALL_OBJ;
    wave_sync();
    for (int k = LANE; k < g.md * g.md; k += 64) { // set_obj(margin + i, margin + j, maze grid (i + 1, j + 1))
        int i = k / g.md, j = k % g.md;
        c.grid[(margin + j) * w + margin + i] = scratch->grid[(j + 1) * g.ad + (i + 1)];
    }
    wave_sync();
    if (margin > 0) { // border walls (all WALL_OBJ already; kept for the bounds check of set_obj)
        if (margin - 1 < 0 || margin + g.md >= w) c.s.error = PG_ERR_GRID;
    }
}

// ------------------------------------------------------------------ heist (heist.cpp:115-203)
DEV float rand_pos(RCtx &c, float r, float min, float max) { // basic-abstract-game.cpp:1109-1117
    if (max - min <= 2 * r) return (max + min) / 2;
    float range = max - min;
    return (range - 2 * r) * rand01(c) + r + min;
}

// has_agent_collision(e) || has_any_collision(e) for a not-yet-added entity (reposition, :548-569)
DEV bool spawn_collides(RCtx &c, float x, float y, float rx, float ry) {
    bool hit = false;
    for (int base = 0; base < c.s.num_ents; base += 64) {
        int i = base + LANE;
        if (i < c.s.num_ents && !(EI(c, F_FLAGS, i) & EF_AVOIDS)) {
            float tx = (rx + EF(c, F_RX, i)) + 0.0f, ty = (ry + EF(c, F_RY, i)) + 0.0f;
            if ((fabsf(x - EF(c, F_X, i)) < tx) && (fabsf(y - EF(c, F_Y, i)) < ty)) hit = true;
        }
    }
    // the agent is entities[0]: has_agent_collision adds nothing beyond has_any_collision
    return ballot(hit) != 0;
}

// spawn_entity_rxy(rx, ry, type, x, y, w, h) (:520-527): Entity(0, 0, 0, 0, rx, ry, type), reposition, push_back
DEV int spawn_entity_rxy(RCtx &c, float rx, float ry, int type, float x, float y, float w, float h) {
    float ex = rand_pos(c, rx, x, x + w);
    float ey = rand_pos(c, ry, y, y + h);
    int count = 0;
    while (spawn_collides(c, ex, ey, rx, ry) && count < 100) {
        ex = rand_pos(c, rx, x, x + w);
        ey = rand_pos(c, ry, y, y + h);
        count++;
    }
    return add_entity_rxy(c, ex, ey, 0, 0, rx, ry, type);
}
// spawn_entity(r, type, x, y, w, h) (:571-573)
DEV int spawn_entity(RCtx &c, float r, int type, float x, float y, float w, float h) {
    return spawn_entity_rxy(c, r, r, type, x, y, w, h);
}

// reposition_agent (:540-546): agent_has_collision() = has_agent_collision(ent) over `entities`
// (has_collision(ent, agent, ent->collision_margin); PLAYER entities excluded, :1135-1140)
DEV void reposition_agent(RCtx &c) {
    const float arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
    int count = 0;
    bool hit;
    do {
        const float ax = rand01(c) * (c.s.main_width - 2 * arx) + arx;
        const float ay = rand01(c) * (c.s.main_height - 2 * ary) + ary;
        EF(c, F_X, 0) = ax;
        EF(c, F_Y, 0) = ay;
        count++;
        bool h = false;
        for (int base = 0; base < c.s.num_ents; base += 64) {
            const int i = base + LANE;
            if (i < c.s.num_ents && EI(c, F_TYPE, i) != PLAYER) {
                const float tx = (EF(c, F_RX, i) + arx) + EF(c, F_COLLISION_MARGIN, i);
                const float ty = (EF(c, F_RY, i) + ary) + EF(c, F_COLLISION_MARGIN, i);
                if ((fabsf(EF(c, F_X, i) - ax) < tx) && (fabsf(EF(c, F_Y, i) - ay) < ty)) h = true;
            }
        }
        hit = ballot(h) != 0;
    } while (hit && count < 100);
    wave_sync();
}

DEV void heist_game_reset(RCtx &c, MGScratch *scratch) {
    base_game_reset<PG_GAME_HEIST>(c);
    int min_maze_dim = 5;
    int max_diff = (c.s.world_dim - min_maze_dim) / 2;
    int difficulty = randn(c, max_diff + 1);
    c.s.opt_center_agent = c.s.opt_distribution_mode == PG_MEMORY;
    if (c.s.opt_distribution_mode == PG_MEMORY) c.s.num_keys = randn(c, 4);
    else c.s.num_keys = difficulty + randn(c, 2);
    if (c.s.num_keys > 3) c.s.num_keys = 3;
    c.s.has_keys = 0;
    int maze_dim = difficulty * 2 + min_maze_dim;
    float maze_scale = (float)(c.s.main_height / (c.s.world_dim * 1.0));
    EF(c, F_RX, 0) = (float)(.375 * maze_scale);
    EF(c, F_RY, 0) = (float)(.375 * maze_scale);
    float r_ent = maze_scale / 2;
    MG g;
    g.m = scratch;
    g.md = maze_dim;
    g.ad = maze_dim + 2;
    if (g.ad > MG_MAX_DIM) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    mg_generate_maze_with_doors(c, g, c.s.num_keys);
    EF(c, F_X, 0) = -1; // move agent out of the way for maze generation
    EF(c, F_Y, 0) = -1;
    int off_x = randn(c, c.s.world_dim - maze_dim + 1);
    int off_y = randn(c, c.s.world_dim - maze_dim + 1);
    const int w = c.s.main_width;
    for (int i = LANE; i < w * c.s.main_height; i += 64) c.grid[i] = WALL_OBJ;
    wave_sync();
    // the grid writes are order-free; the entity spawns follow the reference's x-major loop
    for (int k = LANE; k < maze_dim * maze_dim; k += 64) {
        int i = k / maze_dim, j = k % maze_dim;
        int obj = scratch->grid[(j + 1) * g.ad + (i + 1)];
        int x = off_x + i, y = off_y + j;
        if (obj != WALL_OBJ && 0 <= x && x < w && 0 <= y && y < c.s.main_height) c.grid[y * w + x] = SPACE;
    }
    wave_sync();
    for (int k = 0; k < maze_dim * maze_dim; k++) {
        int i = k / maze_dim, j = k % maze_dim;
        int obj = scratch->grid[(j + 1) * g.ad + (i + 1)];
        if (obj == WALL_OBJ || obj == SPACE) continue;
        int x = off_x + i, y = off_y + j;
        float obj_x = (float)((x + .5) * maze_scale);
        float obj_y = (float)((y + .5) * maze_scale);
        if (obj >= KEY_OBJ) {
            int e = spawn_entity(c, (float)(.375 * maze_scale), HS_KEY, maze_scale * x, maze_scale * y, maze_scale, maze_scale);
            EI(c, F_IMAGE_THEME, e) = obj - KEY_OBJ - 1;
            match_aspect_ratio<PG_GAME_HEIST>(c, e);
        } else if (obj >= DOOR_OBJ) {
            int e = add_entity(c, obj_x, obj_y, 0, 0, r_ent, HS_LOCKED_DOOR);
            EI(c, F_IMAGE_THEME, e) = obj - DOOR_OBJ - 1;
        } else if (obj == EXIT_OBJ) {
            int e = spawn_entity(c, (float)(.375 * maze_scale), HS_EXIT, maze_scale * x, maze_scale * y, maze_scale, maze_scale);
            match_aspect_ratio<PG_GAME_HEIST>(c, e);
        } else if (obj == AGENT_OBJ) {
            EF(c, F_X, 0) = obj_x;
            EF(c, F_Y, 0) = obj_y;
        }
    }
    float ring_key_r = 0.03f;
    for (int i = 0; i < c.s.num_keys; i++) {
        int e = add_entity(c, (float)(1 - ring_key_r * (2 * i + 1.25)), (float)(ring_key_r * .75), 0, 0, ring_key_r,
                           HS_KEY_ON_RING);
        EI(c, F_IMAGE_THEME, e) = i;
        EI(c, F_IMAGE_TYPE, e) = HS_KEY;
        EF(c, F_ROTATION, e) = PI_F / 2;
        EI(c, F_RENDER_Z, e) = 1;
        EI(c, F_FLAGS, e) = EI(c, F_FLAGS, e) | EF_ABS_COORDS;
        match_aspect_ratio<PG_GAME_HEIST>(c, e);
    }
}

// ------------------------------------------------------------------ miner (miner.cpp:134-218)
DEV void miner_game_reset(RCtx &c, MinerScratch *m) {
    base_game_reset<PG_GAME_MINER>(c);
    c.s.died = 0;
    EF(c, F_RX, 0) = .5f;
    EF(c, F_RY, 0) = .5f;
    c.s.opt_center_agent = c.s.opt_distribution_mode == PG_MEMORY;
    c.s.grid_step = 1;
    const int w = c.s.main_width, area = c.s.main_area, grid_size = c.s.main_width * c.s.main_height;
    float diamond_pct = 12 / 400.0f;
    float boulder_pct = 80 / 400.0f;
    float mud_pct = 12 / 400.0f;
    int num_diamonds = (int)(diamond_pct * grid_size);
    int num_boulders = (int)(boulder_pct * grid_size);
    int num_mud = (int)(mud_pct * grid_size);
    const int k = num_diamonds + num_boulders + num_mud + 1;
    if (area > 35 * 35 || k > area) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    // RandGen::simple_choose(main_area, k) (randgen.cpp:70-88): rejection against a set
    for (int i = LANE; i < area; i += 64) m->taken[i] = 0;
    wave_sync();
    for (int i = 0; i < k; i++) {
        int next = randn(c, area);
        while (m->taken[next]) next = randn(c, area);
        wave_sync();
        if (LANE == 0) {
            m->obj_idxs[i] = (int16_t)next;
            m->taken[next] = 1;
        }
        wave_sync();
    }
    const int agent_x = m->obj_idxs[0] % w, agent_y = m->obj_idxs[0] / w;
    EF(c, F_X, 0) = (float)(agent_x + .5);
    EF(c, F_Y, 0) = (float)(agent_y + .5);
    for (int i = LANE; i < area; i += 64) c.grid[i] = MN_DIRT;
    wave_sync();
    for (int i = LANE; i < k - 1; i += 64) { // distinct cells: order-free
        int v = i < num_diamonds ? MN_DIAMOND : (i < num_diamonds + num_boulders ? MN_BOULDER : MN_MUD);
        c.grid[m->obj_idxs[i + 1]] = (int16_t)v;
    }
    wave_sync();
    // get_cells_with_type(DIRT) (basic-abstract-game.cpp:203-213), ascending
    int nd = 0;
    for (int base = 0; base < grid_size; base += 64) {
        int i = base + LANE;
        bool in = i < grid_size && c.grid[i] == MN_DIRT;
        unsigned long long b = ballot(in);
        if (in) m->dirt[nd + __popcll(b & ((1ull << LANE) - 1ull))] = (int16_t)i;
        nd += __popcll(b);
    }
    wave_sync();
    set_obj(c, agent_x, agent_y, SPACE);
    for (int i = -1; i <= 1; ++i)
        for (int j = -1; j <= 1; ++j)
            if (get_obj(c, agent_x + i, agent_y + j) == MN_BOULDER) set_obj(c, agent_x + i, agent_y + j, MN_DIRT);
    // exit candidates: dirt cells whose cell above is DIRT or out of bounds (idx-based get_obj)
    int ne = 0;
    for (int base = 0; base < nd; base += 64) {
        int q = base + LANE;
        bool in = false;
        int cell = 0;
        if (q < nd) {
            cell = m->dirt[q];
            int above = cell + w;
            int above_obj = (0 <= above && above < grid_size) ? c.grid[above] : c.s.out_of_bounds_object;
            in = above_obj == MN_DIRT || above_obj == c.s.out_of_bounds_object;
        }
        unsigned long long b = ballot(in);
        wave_sync(); // compaction writes into the list being read (positions <= reads)
        if (in) m->dirt[ne + __popcll(b & ((1ull << LANE) - 1ull))] = (int16_t)cell;
        ne += __popcll(b);
        wave_sync();
    }
    if (ne <= 0) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    const int exit_cell = m->dirt[randn(c, ne)];
    if (LANE == 0) c.grid[exit_cell] = SPACE;
    wave_sync();
    int e = add_entity(c, (float)((exit_cell % w) + .5), (float)((exit_cell / w) + .5), 0, 0, .5f, MN_EXIT);
    EI(c, F_RENDER_Z, e) = -1;
}

// ------------------------------------------------------------------ climber (climber.cpp:164-288)
DEV void climber_game_reset(RCtx &c) {
    base_game_reset<PG_GAME_CLIMBER>(c);
    c.s.gravity = 0.2f;
    c.s.max_jump = 1.5f;
    c.s.air_control = 0.15f;
    c.s.maxspeed = .5f;
    c.s.has_support = 0;
    c.s.facing_right = 1;
    EF(c, F_RX, 0) = .5f;
    EF(c, F_RY, 0) = .5f;
    EF(c, F_X, 0) = 1 + .5f;
    EF(c, F_Y, 0) = 1 + .5f;
    choose_random_theme(c, 0);
    c.s.wall_theme = randn(c, 4); // NUM_WALL_THEMES
    const int w = c.s.main_width, h = c.s.main_height;
    fill_elem(c, 0, 0, w, 1, CL_WALL_TOP); // init_floor_and_walls (:164-169)
    fill_elem(c, 0, 0, 1, h, CL_WALL_MID);
    fill_elem(c, w - 1, 0, 1, h, CL_WALL_MID);
    fill_elem(c, 0, h - 1, w, 1, CL_WALL_MID);
    // generate_platforms (:178-232)
    int difficulty = randn(c, 3);
    int min_platforms = difficulty * difficulty + 1;
    int max_platforms = (difficulty + 1) * (difficulty + 1) + 1;
    int num_platforms = randn(c, max_platforms - min_platforms + 1) + min_platforms;
    c.s.coin_quota = 0;
    c.s.coins_collected = 0;
    int curr_x = randn(c, w - 4) + 2;
    int curr_y = 0;
    const int margin_x = 3;
    float enemy_prob = c.s.opt_distribution_mode == PG_EASY ? .2f : .5f;
    for (int i = 0; i < num_platforms; i++) {
        int max_dy = (int)(c.s.max_jump * c.s.max_jump / (2 * c.s.gravity)); // choose_delta_y (:171-176)
        int delta_y = randn(c, max_dy - 3 + 1) + 3;
        bool can_spawn_enemy = (curr_x >= margin_x) && (curr_x <= w - margin_x);
        if (can_spawn_enemy && (rand01(c) < enemy_prob)) {
            // g++ evaluates add_entity's arguments right to left: the vx draw comes first
            // (pinned, tests/test_oracle_pins.py::test_argument_evaluation_order_pinned)
            int vdraw = randn(c, 2);
            int ydraw = randn(c, 2);
            int e = add_entity(c, (float)(curr_x + .5), (float)(curr_y + ydraw + 2 + .5), (float)(.15 * (vdraw * 2 - 1)), 0,
                               .5f, CL_ENEMY);
            EI(c, F_IMAGE_TYPE, e) = CL_ENEMY1;
            EI(c, F_FLAGS, e) = EF_AUTO_ERASE | EF_SMART_STEP;
            EF(c, F_CLIMBER_SPAWN_X, e) = (float)(curr_x + .5);
            match_aspect_ratio<PG_GAME_CLIMBER>(c, e);
        }
        curr_y += delta_y;
        int plat_len = 2 + randn(c, 10);
        int vx = randn(c, 2) * 2 - 1;
        if (curr_x < margin_x) vx = 1;
        if (curr_x > w - margin_x) vx = -1;
        int nc = 0;
        for (int j = 0; j < plat_len; j++) {
            int nx = curr_x + (j + 1) * vx;
            if (nx <= 0 || nx >= w - 1) break;
            nc++;
            set_obj(c, nx, curr_y, CL_WALL_TOP);
        }
        if (nc <= 0) {
            c.s.error = PG_ERR_GRID;
            return;
        }
        // candidates[k] = curr_x + (k + 1) * vx
        if ((double)rand01(c) < .5 || i == num_platforms - 1) {
            int coin_x = curr_x + (randn(c, nc) + 1) * vx;
            add_entity(c, (float)(coin_x + .5), (float)(curr_y + 1.5), 0, 0, 0.3f, CL_COIN);
            c.s.coin_quota += 1;
        }
        curr_x = curr_x + (randn(c, nc) + 1) * vx;
    }
}

// ------------------------------------------------------------------ fruitbot (fruitbot.cpp:157-245)
// fit_aspect_ratio (basic-abstract-game.cpp:1034-1045) of an entity with no preserved themes
DEV void fit_aspect_ratio(RCtx &c, int i) {
    int type = EI(c, F_IMAGE_TYPE, i), theme = EI(c, F_IMAGE_THEME, i);
    if (c.s.opt_restrict_themes) theme = 0;
    int4 sp = reinterpret_cast<const int4 *>(c.d.sprites)[type + theme * MAX_ASSETS];
    if (sp.y <= 0 || sp.z <= 0) {
        c.s.error = PG_ERR_BAD_OPTION;
        return;
    }
    float ar = (float)(sp.y * 1.0 / sp.z);
    if (ar > 1) EF(c, F_RY, i) = EF(c, F_RX, i) / ar;
    else EF(c, F_RX, i) = EF(c, F_RY, i) * ar;
}

DEV void fb_add_walls(RCtx &c, float ry, bool use_door, float min_pct) {
    const float rw = (float)c.s.main_width;
    const float wall_ry = 0.3f, lock_rx = .25, lock_ry = 0.45f;
    float pct = (float)(min_pct + .2 * rand01(c));
    if (use_door) {
        pct += 0.1f;
        float lock_pct_w = 2 * lock_rx / c.s.main_width;
        float door_pct_w = (wall_ry * 2 * 3.25f) / c.s.main_width; // DOOR_ASPECT_RATIO
        int num_doors = (int)ceilf((pct - 2 * lock_pct_w) / door_pct_w);
        pct = 2 * lock_pct_w + door_pct_w * num_doors;
    }
    float gapw = pct * rw;
    float w1 = rand01(c) * (rw - gapw);
    float w2 = rw - w1 - gapw;
    add_entity_rxy(c, w1 / 2, ry, 0, 0, w1 / 2, wall_ry, FB_BARRIER);
    add_entity_rxy(c, rw - w2 / 2, ry, 0, 0, w2 / 2, wall_ry, FB_BARRIER);
    if (use_door) {
        int is_on_right = randn(c, 2);
        float lock_x = w1 + lock_rx + is_on_right * (gapw - 2 * lock_rx);
        float door_x = w1 + gapw / 2 - (is_on_right * 2 - 1) * lock_rx;
        add_entity_rxy(c, door_x, ry, 0, 0, gapw / 2 - lock_rx, wall_ry, FB_LOCKED_DOOR);
        add_entity_rxy(c, lock_x, ry - lock_ry + wall_ry, 0, 0, lock_rx, lock_ry, FB_LOCK);
    }
}

DEV void fruitbot_game_reset(RCtx &c, int16_t *part) {
    base_game_reset<PG_GAME_FRUITBOT>(c);
    c.s.last_fire_time = 0;
    int min_sep = 4, num_walls = 10, object_group_size = 6, buf_h = 4;
    float door_prob = .125, min_pct = .1f;
    if (c.s.opt_distribution_mode == PG_EASY) {
        num_walls = 5; object_group_size = 2; door_prob = 0; min_pct = .2f;
    }
    // RandGen::partition (randgen.cpp:33-41)
    for (int k = LANE; k < num_walls; k += 64) part[k] = 0;
    wave_sync();
    const int px = c.s.main_height - min_sep * num_walls - buf_h;
    for (int i = 0; i < px; i++) {
        int k = randn(c, num_walls);
        if (LANE == 0) part[k] += 1;
    }
    wave_sync();
    int curr_h = 0;
    for (int k = 0; k < num_walls; k++) {
        int dy = min_sep + part[k];
        curr_h += dy;
        bool use_door = (dy > 5) && rand01(c) < door_prob;
        fb_add_walls(c, (float)curr_h, use_door, min_pct);
    }
    EF(c, F_Y, 0) = EF(c, F_RY, 0);
    const int num_good = randn(c, 10) + 10;
    const int num_bad = randn(c, 10) + 10;
    for (int i = 0; i < c.s.main_width; i++) {
        int e = add_entity_rxy(c, (float)(i + .5), (float)(c.s.main_height - .5), 0, 0, .5f, .5f, FB_PRESENT);
        choose_random_theme(c, e);
    }
    wave_sync();
    for (int i = 0; i < num_good; i++) {
        spawn_entity(c, .5f, FB_GOOD_OBJ, 0, 0, (float)c.s.main_width, (float)c.s.main_height);
        wave_sync();
    }
    for (int i = 0; i < num_bad; i++) {
        spawn_entity(c, .5f, FB_BAD_OBJ, 0, 0, (float)c.s.main_width, (float)c.s.main_height);
        wave_sync();
    }
    for (int i = 0; i < c.s.num_ents; i++) {
        int t = EI(c, F_TYPE, i);
        if (t == FB_GOOD_OBJ || t == FB_BAD_OBJ) {
            int theme = randn(c, object_group_size);
            wave_sync();
            EI(c, F_IMAGE_THEME, i) = theme;
            fit_aspect_ratio(c, i);
            wave_sync();
        }
    }
    EF(c, F_ROTATION, 0) = -1 * PI_F / 2;
}

// ------------------------------------------------------------------ dodgeball (dodgeball.cpp:157-369)
DEV void db_add_room(RCtx &c, float4 *rooms, int &n, float x, float y, float w, float h) { // :157-164
    if ((w >= c.s.db_min_dim || h >= c.s.db_min_dim) && (w >= c.s.db_hard_min_dim) && (h >= c.s.db_hard_min_dim)) {
        if (n >= 64) {
            c.s.error = PG_ERR_GRID;
            return;
        }
        if (LANE == 0) rooms[n] = make_float4(x, y, w, h);
        n++;
    }
}

DEV void db_split_room(RCtx &c, float4 *rooms, int &n, float4 room, float thickness) { // :166-224
    bool will_split_width = rand01(c) < .5;
    const bool choice2 = rand01(c) < .5;
    if (room.z < c.s.db_min_dim) will_split_width = false;
    if (room.w < c.s.db_min_dim) will_split_width = true;
    const float rx = room.x, ry = room.y, rw = room.z, rh = room.w;
    const float gap = (float)(.25 * (randn(c, 3) + 1));
    const float pct = 1 - gap;
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
        add_entity_rxy(c, rx + rw / 2, wy + wh / 2, 0, 0, thickness, wh / 2, DB_LAVA_WALL);
        const float nextw = rw / 2 - thickness;
        db_add_room(c, rooms, n, rx, wy, nextw, wh);
        db_add_room(c, rooms, n, rx + rw / 2 + thickness, wy, nextw, wh);
        db_add_room(c, rooms, n, rx, remy, rw, rh - wh);
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
        add_entity_rxy(c, wx + ww / 2, ry + rh / 2, 0, 0, ww / 2, thickness, DB_LAVA_WALL);
        const float nexth = rh / 2 - thickness;
        db_add_room(c, rooms, n, wx, ry, ww, nexth);
        db_add_room(c, rooms, n, wx, ry + rh / 2 + thickness, ww, nexth);
        db_add_room(c, rooms, n, remx, ry, rw - ww, rh);
    }
    wave_sync();
}

DEV void db_choose_vel(RCtx &c, int i) { // :226-238
    const float vel = DB_ENEMY_VEL * (randn(c, 2) * 2 - 1);
    if (randn(c, 2) == 0) {
        EF(c, F_VX, i) = vel;
        EF(c, F_VY, i) = 0;
    } else {
        EF(c, F_VY, i) = vel;
        EF(c, F_VX, i) = 0;
    }
    EI(c, F_SPAWN_TIME, i) = randn(c, 50) + 25;
}

DEV void dodgeball_game_reset(RCtx &c, float4 *rooms) { // :259-369
    base_game_reset<PG_GAME_DODGEBALL>(c);
    c.s.opt_center_agent = c.s.opt_distribution_mode == PG_MEMORY;
    c.s.last_fire_time = 0;
    int n = 0;
    if (LANE == 0) rooms[0] = make_float4(0, 0, (float)c.s.main_width, (float)c.s.main_height);
    n = 1;
    const int dm = c.s.opt_distribution_mode;
    float thickness = 0.3f, enemy_r = .5, exit_r = .75;
    float ball_r = .25, ball_vscale = .25;
    int num_iterations = 0, max_extra_enemies = 3;
    if (dm == PG_EASY) {
        num_iterations = 2;
        thickness *= 2; enemy_r *= 2; ball_r *= 2; ball_vscale *= 2;
        c.s.maxspeed = .75;
        EF(c, F_RX, 0) = 1; EF(c, F_RY, 0) = 1;
        exit_r *= 2;
    } else if (dm == PG_HARD) {
        num_iterations = 4;
        thickness *= 1.5; enemy_r *= 1.5; ball_r *= 1.5; ball_vscale *= 1.5;
        c.s.maxspeed = .5;
        EF(c, F_RX, 0) = .75; EF(c, F_RY, 0) = .75;
    } else if (dm == PG_EXTREME) {
        num_iterations = 8;
        c.s.maxspeed = .25;
    } else { // PG_MEMORY
        num_iterations = 16;
        thickness *= 1.5; enemy_r *= 1.5; ball_r *= 1.5; ball_vscale *= 1.5;
        c.s.maxspeed = .5;
        EF(c, F_RX, 0) = .75; EF(c, F_RY, 0) = .75;
        max_extra_enemies = 16;
    }
    c.s.db_ball_r = ball_r;
    c.s.db_ball_vscale = ball_vscale;
    const float arx = EF(c, F_RX, 0);
    c.s.db_hard_min_dim = (float)(4 * arx + 2 * thickness + .5);
    c.s.db_min_dim = (float)(arx * 8 + .5);
    wave_sync();
    for (int it = 0; it < num_iterations; it++) {
        if (n == 0) break;
        const int idx = randn(c, n);
        const float4 room = rooms[idx];
        wave_sync();
        // rooms.erase(idx): order-preserving shift
        float4 mv = make_float4(0, 0, 0, 0);
        const int k = idx + 1 + LANE;
        if (k < n) mv = rooms[k];
        wave_sync();
        if (k < n) rooms[k - 1] = mv;
        wave_sync();
        n--;
        db_split_room(c, rooms, n, room, thickness);
    }
    const float border_r = 0;
    const float doorlen = 2 * exit_r;
    const int exit_wall_choice = randn(c, 4);
    const float mw = (float)c.s.main_width, mh = (float)c.s.main_height;
    if (exit_wall_choice == 0)
        spawn_entity_rxy(c, doorlen / 2, exit_r, DB_DOOR, 2 * border_r, 2 * border_r, mw - 4 * border_r, 2 * exit_r);
    else if (exit_wall_choice == 1)
        spawn_entity_rxy(c, doorlen / 2, exit_r, DB_DOOR, 2 * border_r, mh - 2 * border_r - 2 * exit_r, mw - 4 * border_r,
                         2 * exit_r);
    else if (exit_wall_choice == 2)
        spawn_entity_rxy(c, exit_r, doorlen / 2, DB_DOOR, 2 * border_r, 2 * border_r, 2 * exit_r, mh - 4 * border_r);
    else
        spawn_entity_rxy(c, exit_r, doorlen / 2, DB_DOOR, mw - 2 * border_r - 2 * exit_r, 2 * border_r, 2 * exit_r,
                         mh - 4 * border_r);
    wave_sync();
    reposition_agent(c);
    c.s.num_enemies = randn(c, max_extra_enemies + 1) + 3;
    for (int i = 0; i < c.s.num_enemies; i++) {
        spawn_entity(c, enemy_r, DB_ENEMY, 0, 0, mw, mh);
        wave_sync();
    }
    const int enemy_theme = randn(c, 7); // NUM_ENEMY_THEMES
    for (int i = 0; i < c.s.num_ents; i++) {
        const int t = EI(c, F_TYPE, i);
        if (t == DB_ENEMY) {
            EI(c, F_IMAGE_THEME, i) = enemy_theme;
            EF(c, F_HEALTH, i) = 1;
            EI(c, F_SPAWN_TIME, i) = 0;
            EI(c, F_FIRE_TIME, i) = 10;
            EI(c, F_FLAGS, i) = EF_AUTO_ERASE | EF_COLLIDES | EF_SMART_STEP;
            db_choose_vel(c, i);
            EF(c, F_ROTATION, i) = face_rotation(EF(c, F_VX, i), EF(c, F_VY, i), EF(c, F_ROTATION, i));
        } else if (t == DB_LAVA_WALL) {
            EI(c, F_FLAGS, i) = EF_AUTO_ERASE | EF_COLLIDES;
        }
        wave_sync();
    }
    EF(c, F_ROTATION, 0) = face_rotation(1, 0, EF(c, F_ROTATION, 0));
    wave_sync();
}

// ------------------------------------------------------------------ plunder (plunder.cpp:116-192)
DEV int pl_perm_at(const PGEnv &s, int i) { return (int)((s.gs.pl.perm >> (4 * i)) & 15u); }

DEV void plunder_game_reset(RCtx &c) {
    base_game_reset<PG_GAME_PLUNDER>(c);
    auto &P = c.s.gs.pl;
    EI(c, F_IMAGE_TYPE, 0) = PL_SHIP;
    P.juice_left = 1;
    P.targets_hit = 0;
    P.target_quota = 20;
    P.spawn_prob = 0.06f;
    P.r_scale = c.s.opt_distribution_mode == PG_EASY ? 1.5f : 1.0f;
    const int num_total_ship_types = 6;
    P.num_lanes = 5;
    // RandGen::choose_n(0..5, 6) (randgen.cpp:49-68): draw from the remaining list, erase
    uint32_t rem = 0x543210u, perm = 0;
    for (int k = 0; k < num_total_ship_types; k++) {
        const int idx = randn(c, num_total_ship_types - k);
        const uint32_t v = (rem >> (4 * idx)) & 15u;
        perm |= v << (4 * k);
        const uint32_t low = rem & ((1u << (4 * idx)) - 1u);
        rem = low | ((rem >> (4 * (idx + 1))) << (4 * idx));
    }
    P.perm = perm;
    P.num_current_ship_types = 2;
    P.target_bools = 0;
    for (int i = 0; i < P.num_current_ship_types / 2; i++) P.target_bools |= 1u << pl_perm_at(c.s, i);
    P.lane_dirs = 0;
    for (int i = 0; i < P.num_lanes; i++) {
        if (rand01(c) < .5) P.lane_dirs |= 1u << i;
        const float v = (float)(.15 + .1 * rand01(c));
        if (i == 0) P.lane_vels[0] = v;
        else if (i == 1) P.lane_vels[1] = v;
        else if (i == 2) P.lane_vels[2] = v;
        else if (i == 3) P.lane_vels[3] = v;
        else P.lane_vels[4] = v;
    }
    const int num_panels = c.s.opt_distribution_mode == PG_EASY ? 0 : randn(c, 4);
    const float panel_width = 1.2f;
    for (int i = 0; i < num_panels; i++) {
        spawn_entity_rxy(c, panel_width, .5, PL_PANEL, 0, (float)(.25 * c.s.main_height), (float)c.s.main_width,
                         (float)(.25 * c.s.main_height));
        wave_sync();
    }
    const float key_scale = 1.5;
    P.legend_r = 2;
    add_entity(c, P.legend_r, P.legend_r, 0, 0, P.legend_r, PL_TARGET_BACKGROUND);
    const int e = add_entity(c, P.legend_r, P.legend_r, 0, 0, P.r_scale * key_scale, PL_TARGET_LEGEND);
    EI(c, F_IMAGE_THEME, e) = pl_perm_at(c.s, 0);
    EI(c, F_IMAGE_TYPE, e) = PL_SHIP;
    match_aspect_ratio<PG_GAME_PLUNDER>(c, e);
    EF(c, F_ROTATION, e) = PI_F / 2;
    c.s.last_fire_time = 0;
    c.s.opt_center_agent = 0;
    EF(c, F_RX, 0) = P.r_scale;
    EF(c, F_ROTATION, 0) = -1 * PI_F / 2;
    EI(c, F_IMAGE_THEME, 0) = pl_perm_at(c.s, randn(c, P.num_current_ship_types / 2) + P.num_current_ship_types / 2);
    match_aspect_ratio<PG_GAME_PLUNDER>(c, 0);
    wave_sync();
    reposition_agent(c);
    EF(c, F_Y, 0) = 1 + EF(c, F_RY, 0);
    P.min_agent_x = 2 * P.legend_r + EF(c, F_RX, 0);
    if (EF(c, F_X, 0) < P.min_agent_x) EF(c, F_X, 0) = P.min_agent_x;
    wave_sync();
}

// ------------------------------------------------------------------ starpilot (starpilot.cpp:226-344)
// std::sort(spawners, spawn_cmp) of libstdc++ (bits/stl_algo.h), run by lane 0 over the LDS index
// array: introsort (median-of-3 pivot, unguarded partition, threshold 16, depth 2 * lg n with a
// heapsort fallback) + final insertion sort -- the same steps as oracle/procgen_oracle.c
// libstdcxx_sort, whose permutation is pinned against the real std::sort.  The recursion on the
// right part becomes an explicit stack (the parts are disjoint, the order they are sorted in does
// not change the result).
struct SpSort {
    const int16_t *key;
    int16_t *f;
    DEV bool cmp(int a, int b) const { return key[a] > key[b]; } // spawn_cmp (:28-30)
    DEV void swp(int i, int j) { int16_t t = f[i]; f[i] = f[j]; f[j] = t; }
    DEV void push_heap(int base, int hole, int top, int value) {
        int parent = (hole - 1) / 2;
        while (hole > top && cmp(f[base + parent], value)) {
            f[base + hole] = f[base + parent];
            hole = parent;
            parent = (hole - 1) / 2;
        }
        f[base + hole] = (int16_t)value;
    }
    DEV void adjust_heap(int base, int hole, int len, int value) {
        int top = hole, second = hole;
        while (second < (len - 1) / 2) {
            second = 2 * (second + 1);
            if (cmp(f[base + second], f[base + second - 1])) second--;
            f[base + hole] = f[base + second];
            hole = second;
        }
        if ((len & 1) == 0 && second == (len - 2) / 2) {
            second = 2 * (second + 1);
            f[base + hole] = f[base + second - 1];
            hole = second - 1;
        }
        push_heap(base, hole, top, value);
    }
    DEV void heap_sort(int base, int len) {
        if (len >= 2)
            for (int parent = (len - 2) / 2;; parent--) {
                adjust_heap(base, parent, len, f[base + parent]);
                if (parent == 0) break;
            }
        for (int last = len; last > 1;) {
            last--;
            int value = f[base + last];
            f[base + last] = f[base];
            adjust_heap(base, 0, last, value);
        }
    }
    DEV int partition_pivot(int first, int last) {
        int mid = first + (last - first) / 2, a = first + 1, b = mid, cc = last - 1;
        if (cmp(f[a], f[b])) {
            if (cmp(f[b], f[cc])) swp(first, b);
            else if (cmp(f[a], f[cc])) swp(first, cc);
            else swp(first, a);
        } else if (cmp(f[a], f[cc])) swp(first, a);
        else if (cmp(f[b], f[cc])) swp(first, cc);
        else swp(first, b);
        int lo = first + 1, hi = last;
        while (true) {
            while (cmp(f[lo], f[first])) lo++;
            hi--;
            while (cmp(f[first], f[hi])) hi--;
            if (!(lo < hi)) return lo;
            swp(lo, hi);
            lo++;
        }
    }
    DEV void linear_insert(int last) {
        int val = f[last], next = last - 1;
        while (cmp(val, f[next])) {
            f[last] = f[next];
            last = next;
            next--;
        }
        f[last] = (int16_t)val;
    }
    DEV void sort(int n, int16_t *stack) {
        if (n <= 1) return;
        int lg = 0;
        while ((1 << (lg + 1)) <= n) lg++;
        int sp = 0;
        int first = 0, last = n, depth = 2 * lg;
        while (true) {
            while (last - first > 16) {
                if (depth == 0) {
                    heap_sort(first, last - first);
                    break;
                }
                depth--;
                int cut = partition_pivot(first, last);
                stack[3 * sp] = (int16_t)cut; stack[3 * sp + 1] = (int16_t)last; stack[3 * sp + 2] = (int16_t)depth;
                sp++;
                last = cut;
            }
            if (sp == 0) break;
            sp--;
            first = stack[3 * sp]; last = stack[3 * sp + 1]; depth = stack[3 * sp + 2];
        }
        // __final_insertion_sort
        const int head = n > 16 ? 16 : n;
        for (int i = 1; i < head; i++) {
            if (cmp(f[i], f[0])) {
                int16_t val = f[i];
                for (int k = i; k > 0; k--) f[k] = f[k - 1];
                f[0] = val;
            } else {
                linear_insert(i);
            }
        }
        for (int i = head; i < n; i++) linear_insert(i);
    }
};

DEV void starpilot_game_reset(RCtx &c, SpawnerScratch *S) {
    base_game_reset<PG_GAME_STARPILOT>(c);
    c.s.opt_center_agent = 0;
    const int mode = c.s.opt_distribution_mode;
    // init_hps (:147-224): maxspeed per mode; the tables are sp_hp_* (pg_device.h)
    c.s.maxspeed = mode == PG_EXTREME ? 0.5f : 0.75f;
    float total = 0;
    for (int i = 2; i < 9; i++) total += sp_hp_prob(mode, i);
    // add_spawners (:226-327)
    const int dmin = 10, dmax = 10 + 20, max_group = 5;
    int t = 1 + dmin + randn(c, dmax - dmin); // randint(lo, hi) = lo + x % (hi - lo)
    const bool can_spawn_left = mode != PG_EASY;
    int n = 0;
    while (t <= SP_SHOOTER_WIN_TIME) {
        int group_size = 1;
        const float start_weight = rand01(c) * total;
        float curr_weight = start_weight;
        int type;
        for (type = 2; type < 9; type++) {
            curr_weight -= sp_hp_prob(mode, type);
            if (curr_weight <= 0) break;
        }
        if (type >= 9) type = 8;
        const float r = sp_hp_object_r(type);
        int flyer_theme = 0;
        if (type == SP_FLYER || type == SP_FAST_FLYER) {
            group_size = randn(c, max_group) + 1; // randint(0, 5) + 1
            flyer_theme = randn(c, 7);            // NUM_SHIP_THEMES
        }
        const float y_pos = rand_pos(c, r, 0, (float)c.s.main_height);
        for (int j = 0; j < group_size; j++) {
            const int spawn_time = t + j * 5;
            int fire_time = 10 + randn(c, 90); // randint(10, 100)
            const float k = 2 * PI_F / 4;
            float theta = (float)((rand01(c) - .5) * k);
            float v_scale = sp_hp_vs(mode, type);
            if (randn(c, 2) == 1) theta = 0; // randint(0, 2)
            const float health = sp_hp_health(mode, type);
            if (type == SP_METEOR || type == SP_CLOUD) {
                theta = 0;
                v_scale = SP_HP_SLOW_V;
                fire_time = -1;
            } else if (type == SP_TURRET) {
                theta = 0;
                v_scale = SP_HP_SLOW_V;
                fire_time = 20 + randn(c, 10); // randint(20, 30)
            }
            v_scale *= SP_V_SCALE;
            double st, ct;
            pg_sincos_cr((double)theta, &st, &ct); // ::cos / ::sin (double) of the float theta
            float vx = (float)(-1 * ct * v_scale);
            const float vy = (float)(st * v_scale);
            bool spawn_right = true;
            float x_pos;
            if (type == SP_FLYER || type == SP_FAST_FLYER)
                if (rand01(c) > 0.9f && can_spawn_left) spawn_right = false; // hp_spawn_right_threshold
            if (spawn_right) {
                x_pos = c.s.main_width + r;
            } else {
                x_pos = -r;
                vx *= -1;
            }
            int theme = 0, rz = 0;
            float ry = r, rot = 0;
            if (type == SP_CLOUD) {
                rz = 1;
                theme = randn(c, c.d.num_themes[SP_CLOUD]);
            } else if (type == SP_METEOR) {
                theme = randn(c, c.d.num_themes[SP_METEOR]);
            } else if (type == SP_FLYER || type == SP_FAST_FLYER) {
                theme = flyer_theme;
                rot = ((vx > 0) ? -1 : 1) * PI_F / 2;
            } else if (type == SP_TURRET) {
                theme = randn(c, c.d.num_themes[SP_TURRET]);
                int th = c.s.opt_restrict_themes ? 0 : theme; // match_aspect_ratio
                int4 sp = reinterpret_cast<const int4 *>(c.d.sprites)[type + th * MAX_ASSETS];
                if (sp.y <= 0 || sp.z <= 0) c.s.error = PG_ERR_BAD_OPTION;
                else ry = r / (float)(sp.y * 1.0 / sp.z);
            }
            if (n >= SP_MAX_SPAWNERS) {
                c.s.error = PG_ERR_ENTITY_OVERFLOW;
            } else if (LANE == 0) {
                S->x[n] = x_pos; S->y[n] = y_pos; S->vx[n] = vx; S->vy[n] = vy; S->r[n] = r; S->ry[n] = ry;
                S->rot[n] = rot; S->health[n] = health; S->type[n] = (int16_t)type; S->theme[n] = (int16_t)theme;
                S->fire[n] = (int16_t)fire_time; S->spawn[n] = (int16_t)spawn_time; S->rz[n] = (int8_t)rz;
                S->idx[n] = (int16_t)n;
            }
            if (n < SP_MAX_SPAWNERS) n++;
        }
        t += dmin + randn(c, dmax - dmin);
    }
    wave_sync();
    if (LANE == 0) {
        SpSort so;
        so.key = S->spawn;
        so.f = S->idx;
        so.sort(n, S->stack);
    }
    wave_sync();
    // spawners[i] -> slot PG_CAP - 1 - i
    if (c.s.num_ents + n > PG_CAP) c.s.error = PG_ERR_ENTITY_OVERFLOW;
    for (int i = LANE; i < n && c.s.num_ents + n <= PG_CAP; i += 64) {
        const int g = S->idx[i], slot = PG_CAP - 1 - i;
        EF(c, F_X, slot) = S->x[g]; EF(c, F_Y, slot) = S->y[g]; EF(c, F_VX, slot) = S->vx[g]; EF(c, F_VY, slot) = S->vy[g];
        EF(c, F_RX, slot) = S->r[g]; EF(c, F_RY, slot) = S->ry[g]; EF(c, F_ROTATION, slot) = S->rot[g];
        EF(c, F_VROT, slot) = 0; EF(c, F_ALPHA, slot) = 1.0f; EF(c, F_ALPHA_DECAY, slot) = 1.0f;
        EF(c, F_GROW_RATE, slot) = 1.0f; EF(c, F_FRICTION, slot) = 1; EF(c, F_COLLISION_MARGIN, slot) = 0;
        EF(c, F_HEALTH, slot) = S->health[g]; EF(c, F_THETA, slot) = -100; EF(c, F_CLIMBER_SPAWN_X, slot) = 0;
        EI(c, F_TYPE, slot) = S->type[g]; EI(c, F_IMAGE_TYPE, slot) = S->type[g]; EI(c, F_IMAGE_THEME, slot) = S->theme[g];
        EI(c, F_RENDER_Z, slot) = S->rz[g]; EI(c, F_LIFE_TIME, slot) = 0; EI(c, F_EXPIRE_TIME, slot) = -1;
        EI(c, F_FIRE_TIME, slot) = S->fire[g]; EI(c, F_SPAWN_TIME, slot) = S->spawn[g]; EI(c, F_FLAGS, slot) = EF_AUTO_ERASE;
    }
    c.s.num_tail = n;
    EF(c, F_ROTATION, 0) = PI_F / 2;
    EI(c, F_IMAGE_THEME, 0) = randn(c, c.d.num_themes[PLAYER]); // choose_random_theme(agent)
    wave_sync();
}

// ------------------------------------------------------------------ bossfight (bossfight.cpp:192-250, 310-329)
DEV void bf_prepare_boss(RCtx &c, int boss) { // :192-199
    auto &B = c.s.gs.bf;
    B.shields_are_up = 1;
    B.curr_vel_timeout = BF_BOSS_VEL_TIMEOUT;
    B.time_to_swap = B.invulnerable_duration;
    B.attack_mode = (int)((B.attack_modes >> (2 * (B.round_num % B.num_rounds))) & 3u);
    EF(c, F_VX, boss) = 0;
    EF(c, F_VY, boss) = 0;
}

DEV void bossfight_game_reset(RCtx &c) {
    base_game_reset<PG_GAME_BOSSFIGHT>(c);
    auto &B = c.s.gs.bf;
    B.damaged_until_time = 0;
    c.s.last_fire_time = 0;
    B.boss_bullet_vel = (float)(c.s.opt_distribution_mode == PG_EASY ? .5 : .75);
    const int max_extra_invulnerable = c.s.opt_distribution_mode == PG_EASY ? 1 : 3;
    c.s.opt_center_agent = 0;
    const int boss = add_entity(c, (float)(c.s.main_width / 2), (float)(c.s.main_height / 2), 0, 0, BF_BOSS_R, BF_BOSS);
    choose_random_theme(c, boss);
    match_aspect_ratio<PG_GAME_BOSSFIGHT>(c, boss);
    add_entity_rxy(c, EF(c, F_X, boss), EF(c, F_Y, boss), 0, 0, (float)(1.2 * EF(c, F_RX, boss)),
                   (float)(1.2 * EF(c, F_RY, boss)), BF_SHIELDS);
    B.round_health = randn(c, 9) + 1;
    B.num_rounds = 1 + randn(c, 5);
    B.invulnerable_duration = 2 + randn(c, max_extra_invulnerable + 1);
    EF(c, F_HEALTH, boss) = (float)(B.round_health * B.num_rounds);
    EI(c, F_IMAGE_THEME, 0) = randn(c, c.d.num_themes[PLAYER]); // choose_random_theme(agent)
    B.player_laser_theme = randn(c, 3); // NUM_LASER_THEMES
    B.boss_laser_theme = randn(c, 3);
    B.attack_modes = 0;
    for (int i = 0; i < B.num_rounds; i++) B.attack_modes |= (uint32_t)randn(c, 4) << (2 * i);
    B.round_num = 0;
    bf_prepare_boss(c, boss);
    EF(c, F_RX, 0) = .75;
    match_aspect_ratio<PG_GAME_BOSSFIGHT>(c, 0);
    wave_sync();
    reposition_agent(c);
    EF(c, F_Y, 0) = EF(c, F_RY, 0);
    B.barriers_moves_right = (double)rand01(c) > .5; // randbool (randgen.cpp:25-27)
    wave_sync();
    // spawn_barriers (:310-329)
    const int num_barriers = randn(c, 3) + 1;
    for (int i = 0; i < num_barriers; i++) {
        const float barrier_r = 0.6f;
        const float min_barrier_y = (float)(2 * EF(c, F_RY, 0) + barrier_r + .5);
        const float ent_y = rand01(c) * (BF_BOTTOM_MARGIN - min_barrier_y - barrier_r) + min_barrier_y;
        const float ent_x = rand01(c) * (c.s.main_width - 2 * barrier_r) + barrier_r;
        const int theme = randn(c, c.d.num_themes[BF_BARRIER]); // choose_random_theme
        const int th = c.s.opt_restrict_themes ? 0 : theme;    // match_aspect_ratio
        const int4 sp = reinterpret_cast<const int4 *>(c.d.sprites)[BF_BARRIER + th * MAX_ASSETS];
        float ry = barrier_r;
        if (sp.y <= 0 || sp.z <= 0) c.s.error = PG_ERR_BAD_OPTION;
        else ry = barrier_r / (float)(sp.y * 1.0 / sp.z);
        if (!spawn_collides(c, ent_x, ent_y, barrier_r, ry)) { // has_any_collision
            const int e = add_entity_rxy(c, ent_x, ent_y, 0, 0, barrier_r, ry, BF_BARRIER);
            EI(c, F_IMAGE_THEME, e) = theme;
            EF(c, F_HEALTH, e) = 3;
            EI(c, F_FLAGS, e) = EF_AUTO_ERASE | EF_COLLIDES;
        }
        wave_sync();
    }
}

// ------------------------------------------------------------------ ninja (ninja.cpp:162-331)
DEV void nj_fill_ground_block(RCtx &c, int x, int y, int dx, int dy) { // fill_block_top(.., WALL_MID, WALL_MID)
    if (dy <= 0) return;
    fill_elem(c, x, y, dx, dy - 1, NJ_WALL_MID);
    fill_elem(c, x, y + dy - 1, dx, 1, NJ_WALL_MID);
}

DEV void ninja_game_reset(RCtx &c) {
    base_game_reset<PG_GAME_NINJA>(c);
    auto &N = c.s.gs.nj;
    c.s.gravity = 0.2f;
    c.s.max_jump = 1.5;
    c.s.air_control = 0.15f;
    c.s.maxspeed = .5;
    c.s.has_support = 0;
    c.s.facing_right = 1;
    N.jump_charge = 0;
    N.jump_charge_inc = .25;
    c.s.visibility = 16;
    EF(c, F_RX, 0) = .5;
    EF(c, F_RY, 0) = .5;
    EF(c, F_X, 0) = 1 + EF(c, F_RX, 0);
    EF(c, F_Y, 0) = c.s.main_height / 2 + EF(c, F_RY, 0);
    if (c.s.opt_distribution_mode == PG_EASY) {
        c.s.max_jump = 1.25;
        N.jump_charge_inc = 1;
        c.s.visibility = 10;
    }
    const int difficulty = randn(c, 3) + 1;
    c.s.last_fire_time = 0;
    c.s.wall_theme = randn(c, 3); // NUM_WALL_THEMES
    const int W = c.s.main_width, H = c.s.main_height;
    fill_elem(c, 0, 0, W, 1, NJ_WALL_MID); // init_floor_and_walls (:169-174)
    fill_elem(c, 0, 0, 1, H, NJ_WALL_MID);
    fill_elem(c, W - 1, 0, 1, H, NJ_WALL_MID);
    fill_elem(c, 0, H - 1, W, 1, NJ_WALL_MID);
    // generate_coin_to_the_right (:180-297)
    int min_gap = difficulty - 1, min_plat_w = 1, inc_dy = 4;
    if (c.s.opt_distribution_mode == PG_EASY) {
        min_gap -= 1;
        if (min_gap < 0) min_gap = 0;
        min_plat_w = 3;
        inc_dy = 2;
    }
    const float bomb_prob = (float)(.25 * (difficulty - 1));
    const int max_gap_inc = difficulty == 1 ? 1 : 2;
    const int num_sections = randn(c, difficulty) + difficulty;
    const int start_x = 5;
    int curr_x = start_x, curr_y = H / 2, min_y = curr_y;
    const float _max_dy = c.s.max_jump * c.s.max_jump / (2 * c.s.gravity);
    const int max_dy = (int)(_max_dy - .5);
    nj_fill_ground_block(c, 0, 0, start_x, curr_y);
    fill_elem(c, 0, curr_y + 8, start_x, H - curr_y - 8, NJ_WALL_MID);
    for (int i = 0; i < num_sections; i++) {
        const int prev_x = curr_x, prev_y = curr_y;
        const int num_edges = randn(c, 2) + 1;
        int max_y = -1, last_edge_y = -1;
        for (int j = 0; j < num_edges; j++) {
            curr_x = prev_x + j;
            if (curr_x + 15 >= W) break;
            curr_y = prev_y;
            int dy = randn(c, inc_dy) + 1 + (int)(difficulty / 3);
            if (dy > max_dy) dy = max_dy;
            if (curr_y >= H - 15) dy *= -1;
            else if (curr_y >= 5 && rand01(c) < .4) dy *= -1;
            curr_y += dy;
            if (curr_y < 3) curr_y = 3;
            if (abs(curr_y - last_edge_y) <= 1) curr_y = last_edge_y + 2;
            const int dx = min_plat_w + randn(c, 3);
            nj_fill_ground_block(c, curr_x, curr_y - 1, dx, 1);
            curr_x += dx;
            curr_x += min_gap + randn(c, max_gap_inc + 1);
            if (curr_y > max_y) max_y = curr_y;
            if (curr_y < min_y) min_y = curr_y;
            last_edge_y = curr_y;
        }
        if (rand01(c) < bomb_prob) {
            const int bx = randn(c, curr_x - prev_x + 1) + prev_x;
            set_obj(c, bx, max_y + 2, NJ_BOMB);
        }
        const int ceiling_start = max_y - 1 + 11; // ceiling_height
        nj_fill_ground_block(c, prev_x, ceiling_start, curr_x - prev_x, H - ceiling_start);
    }
    const int e = add_entity(c, (float)(curr_x + .5), (float)(curr_y + .5), 0, 0, .5, NJ_GOAL);
    choose_random_theme(c, e);
    nj_fill_ground_block(c, curr_x, curr_y - 1, 1, 1);
    fill_elem(c, curr_x, curr_y + 6, 1, H - curr_y - 6, NJ_WALL_MID);
    int fire_y = min_y - 2;
    if (fire_y < 1) fire_y = 1;
    nj_fill_ground_block(c, start_x, 0, W - start_x, fire_y);
    fill_elem(c, start_x, fire_y, W - start_x, 1, NJ_FIRE);
    fill_elem(c, curr_x + 1, 0, W - curr_x - 1, H, NJ_WALL_MID);
    wave_sync();
}

// ------------------------------------------------------------------ caveflyer (caveflyer.cpp:145-265)
// RoomGenerator (roomgen.cpp) restated lane-parallel on the LDS grid:
//  * update(): the cellular automaton reads the whole grid before writing (next_cells), so it is a
//    pull over cells into a scratch copy;
//  * find_best_room(): rooms are the 4-connected SPACE components, labelled with their smallest
//    cell index by min-propagation + pointer jumping; build_room() leaves an isolated cell's room
//    empty (the start cell only joins when a neighbour rediscovers it), so a room's size is its
//    cell count when >= 2, else 0, and the first room in scan order of strictly largest size wins;
//  * find_path(): a level-synchronous BFS that reproduces the FIFO's discovery order: a cell's
//    parent is the frontier entry (frontier order, then neighbour order (-1,0), (0,-1), (0,1),
//    (1,0)) with the smallest key p * 4 + k, and the next frontier is written in key order.  The
//    source never enters `covered`, so it is rediscovered once at depth 2 and expands nothing;
//    the path follows parents from the goal back to the source;
//  * expand_room(set, 4): four pull rounds of 8-neighbour growth through SPACE cells.
#define CF_ROOM 1
#define CF_COVERED 2
#define CF_SET 4
#define CF_CURR 8
#define CF_NEW 16
#define CF_TAKEN 32

DEV void cf_random_fill(RCtx &c) { // rand01() < .5 ? WALL_OBJ : SPACE per cell, draws in cell order
    const int n = c.s.main_width * c.s.main_height;
    for (int base = 0; base < n;) {
        if (c.mti >= PG_MT_N) {
            mt_twist_lds(c.mt);
            c.mti = 0;
            mt_window_reset(c);
        }
        int m = PG_MT_N - c.mti;
        if (m > 64) m = 64;
        if (m > n - base) m = n - base;
        if (LANE < m) c.grid[base + LANE] = rg_rand01_of(mt_temper(c.mt[c.mti + LANE])) < .5 ? WALL_OBJ : SPACE;
        c.mti += m;
        base += m;
        wave_sync();
    }
}

// The room generator's grid sweeps on row masks: lane y holds row y of the grid as a 64-bit mask
// (bit x = cell (x, y); worlds are at most 60 x 60), neighbours come from shifts and from the rows of
// lanes y -/+ 1.  Each sweep is then a few dozen ALU instructions per wave instead of a pass of
// dependent LDS reads per 64 cells (r05 reset phase stamps: the per-cell sweeps and the labelling were
// 2/3 of a caveflyer / jumper level generation).
DEV uint64_t cf_shfl64(uint64_t v, int src) {
    const int lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(uint32_t)(v >> 32), src);
    return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}
DEV uint64_t cf_row_full(int W) { return W >= 64 ? ~0ull : (1ull << W) - 1ull; }
// row LANE of the grid: bit x set where pred(cell) (lanes >= H: 0)
template <typename P>
DEV uint64_t cf_row_of(RCtx &c, P pred) {
    const int W = c.s.main_width, H = c.s.main_height;
    uint64_t r = 0;
    if (LANE < H)
        for (int x = 0; x < W; x++) r |= (uint64_t)(pred(c.grid[LANE * W + x]) ? 1 : 0) << x;
    return r;
}
// grid row LANE from a mask: bit set -> on, clear -> off
DEV void cf_write_row(RCtx &c, uint64_t r, int on, int off) {
    const int W = c.s.main_width, H = c.s.main_height;
    if (LANE < H)
        for (int x = 0; x < W; x++) c.grid[LANE * W + x] = (int16_t)(((r >> x) & 1) ? on : off);
    wave_sync();
}
// the first npath cells of S->list2 as row masks (row LANE returned)
DEV uint64_t cf_rows_of_path(RCtx &c, CaveScratch *S, int npath) {
    const int W = c.s.main_width;
    S->pm[LANE] = 0;
    S->pm[64 + LANE] = 0;
    wave_sync();
    for (int q = LANE; q < npath; q += 64) {
        const int cell = S->list2[q], x = cell % W, y = cell / W;
        atomicOr(&S->pm[2 * y + (x >> 5)], 1u << (x & 31));
    }
    wave_sync();
    const uint64_t r = (uint64_t)S->pm[2 * LANE] | ((uint64_t)S->pm[2 * LANE + 1] << 32);
    wave_sync();
    return LANE < c.s.main_height ? r : 0;
}

// `iters` rounds of roomgen.cpp:3-37 (a cell becomes WALL_OBJ when count_neighbors(i, WALL_OBJ) >= 5
// over its 3 x 3 block, out-of-bounds cells counting as out_of_bounds_object), every cell from the
// previous grid; after each round the cells of `path` (row masks, may be 0) are reset to SPACE.  The
// grid holds only WALL_OBJ / SPACE before and after.
DEV void cf_update(RCtx &c, int iters, uint64_t path) {
    const int W = c.s.main_width, H = c.s.main_height;
    const uint64_t full = cf_row_full(W), ob = c.s.out_of_bounds_object == WALL_OBJ ? ~0ull : 0ull;
    const uint64_t ob_lo = ob & 1ull, ob_hi = ob & (1ull << (W - 1));
    uint64_t row = cf_row_of(c, [](int v) { return v == WALL_OBJ; });
    for (int it = 0; it < iters; it++) {
        uint64_t up = cf_shfl64(row, LANE > 0 ? LANE - 1 : 0), dn = cf_shfl64(row, LANE < 63 ? LANE + 1 : 63);
        if (LANE == 0) up = ob & full;
        if (LANE >= H - 1) dn = ob & full;
        // per source row: sum of (x-1, x, x+1) as a bit-sliced 2-bit number (s + 2 c)
        uint64_t sr[3], cr[3];
        const uint64_t rows3[3] = {up, row, dn};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint64_t m = rows3[k], l = (m << 1) | ob_lo, r = (m >> 1) | ob_hi;
            sr[k] = l ^ m ^ r;
            cr[k] = (l & m) | (l & r) | (m & r);
        }
        const uint64_t t0 = sr[0] ^ sr[1] ^ sr[2], t1 = (sr[0] & sr[1]) | (sr[0] & sr[2]) | (sr[1] & sr[2]);
        const uint64_t u0 = cr[0] ^ cr[1] ^ cr[2], u1 = (cr[0] & cr[1]) | (cr[0] & cr[2]) | (cr[1] & cr[2]);
        // count = t0 + 2 (t1 + u0) + 4 u1 >= 5
        row = ((u1 & (t0 | t1 | u0)) | (t0 & t1 & u0)) & full & ~path;
        if (LANE >= H) row = 0;
    }
    cf_write_row(c, row, WALL_OBJ, SPACE);
}

// find_best_room (roomgen.cpp:116-136) -> label of the best room (cells with a[i] == label), or -1
// find_best_room (roomgen.cpp:116-136) on row masks: the rooms (4-connected SPACE components) are
// flood-filled one at a time from their lowest-index cell (row masks, one dilation step per round,
// until a round adds nothing); the largest room wins, ties to the one first in scan order (lowest
// first cell), rooms of one cell never (fassert(best_room.size() > 0) -> -1).  The winner's rows go
// to S->pm (cf_in_best); returns its first cell.
DEV uint64_t cf_rl64(uint64_t v, int lane) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane) << 32);
}
DEV int cf_find_best_room(RCtx &c, CaveScratch *S) {
    const int W = c.s.main_width, H = c.s.main_height;
    const uint64_t sp = cf_row_of(c, [](int v) { return v == SPACE; });
    uint64_t left = sp, best = 0;
    int best_key = -1;
    for (;;) {
        const unsigned long long nz = ballot(left != 0);
        if (!nz) break;
        const int y0 = __ffsll((long long)nz) - 1, x0 = __builtin_ctzll(cf_rl64(left, y0)), seed = y0 * W + x0;
        uint64_t f = LANE == y0 ? 1ull << x0 : 0ull;
        for (;;) {
            uint64_t up = cf_shfl64(f, LANE > 0 ? LANE - 1 : 0), dn = cf_shfl64(f, LANE < 63 ? LANE + 1 : 63);
            if (LANE == 0) up = 0;
            if (LANE >= H - 1) dn = 0;
            const uint64_t nf = (f | (f << 1) | (f >> 1) | up | dn) & sp;
            if (!ballot(nf != f)) break;
            f = nf;
        }
        int cnt = __popcll(f);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
        const int key = (cnt >= 2 ? cnt : 0) * 4096 + (4095 - seed);
        if (key > best_key) {
            best_key = key;
            best = f;
        }
        left &= ~f;
    }
    S->pm[2 * LANE] = (uint32_t)best;
    S->pm[2 * LANE + 1] = (uint32_t)(best >> 32);
    wave_sync();
    if (best_key < 4096) return -1;
    return 4095 - (best_key & 4095);
}
DEV bool cf_in_best(const CaveScratch *S, int W, int i) {
    const int x = i % W, y = i / W;
    return (S->pm[2 * y + (x >> 5)] >> (x & 31)) & 1u;
}

// find_path (roomgen.cpp:72-114): writes the path's cells (any order) to S->list2, returns its length
DEV int cf_find_path(RCtx &c, CaveScratch *S, int src, int dst) {
    const int W = c.s.main_width, H = c.s.main_height, n = W * H;
    for (int i = LANE; i < n; i += 64) {
        S->b[i] = 0x7fffffff;
        S->f[i] &= (uint8_t)~CF_COVERED;
    }
    if (LANE == 0) S->list[0] = (int16_t)src;
    wave_sync();
    int16_t *fr = S->list, *nx = S->list2;
    int nf = 1;
    bool found = false;
    while (nf > 0 && !found) {
        for (int p = LANE; p < nf; p += 64) { // discovery keys
            const int u = fr[p], x = u % W, y = u / W;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int xx = x + (k == 0 ? -1 : (k == 3 ? 1 : 0)), yy = y + (k == 1 ? -1 : (k == 2 ? 1 : 0));
                if (0 <= xx && xx < W && 0 <= yy && yy < H) {
                    const int v = yy * W + xx;
                    if (c.grid[v] == SPACE && !(S->f[v] & CF_COVERED)) atomicMin(&S->b[v], p * 4 + k);
                }
            }
        }
        wave_sync();
        int cnt = 0;
        bool hit = false;
        for (int base = 0; base < nf; base += 64) { // winners, written in key order (and covered)
            const int p = base + LANE;
            int wm = 0, u = 0;
            if (p < nf) {
                u = fr[p];
                const int x = u % W, y = u / W;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int xx = x + (k == 0 ? -1 : (k == 3 ? 1 : 0)), yy = y + (k == 1 ? -1 : (k == 2 ? 1 : 0));
                    if (0 <= xx && xx < W && 0 <= yy && yy < H) {
                        const int v = yy * W + xx;
                        if (!(S->f[v] & CF_COVERED) && S->b[v] == p * 4 + k) wm |= 1 << k;
                    }
                }
            }
            const int nw = __popc(wm);
            const unsigned long long lt = (1ull << LANE) - 1ull;
            const unsigned long long b0 = ballot(nw & 1), b1 = ballot(nw & 2), b2 = ballot(nw & 4);
            int o = cnt + __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
            const int x = u % W, y = u / W;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (wm & (1 << k)) {
                    const int v = (y + (k == 1 ? -1 : (k == 2 ? 1 : 0))) * W + x + (k == 0 ? -1 : (k == 3 ? 1 : 0));
                    nx[o++] = (int16_t)v;
                    S->a[v] = (int16_t)u;
                    // exactly one (p, k) holds v's key, so marking it covered here cannot hide it from
                    // its own winner; a later 64-entry chunk that also neighbours v fails the key test
                    S->f[v] |= CF_COVERED;
                    hit = hit || v == dst;
                }
            }
            cnt += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        }
        found = ballot(hit) != 0;
        wave_sync();
        int16_t *t = fr;
        fr = nx;
        nx = t;
        nf = cnt;
    }
    if (!found) {
        c.s.error = PG_ERR_GRID;
        return 0;
    }
    // parent chain dst -> src (serial; the path is a set for every later use)
    int len = 0;
    if (LANE == 0) {
        int v = dst;
        for (;;) {
            S->list2[len++] = (int16_t)v;
            if (v == src || len > n) break;
            v = S->a[v];
        }
    }
    len = __shfl(len, 0);
    wave_sync();
    return len;
}

// expand_room (roomgen.cpp:138-177) from the path cells (row masks): each round every SPACE cell not yet
// in the set with an 8-neighbour added in the previous round joins; then the grid becomes SPACE on the
// set and `wall` elsewhere
DEV void cf_expand_room(RCtx &c, uint64_t path, int rounds, int wall) {
    const int W = c.s.main_width, H = c.s.main_height;
    const uint64_t full = cf_row_full(W);
    const uint64_t sp = cf_row_of(c, [](int v) { return v == SPACE; });
    uint64_t set = path, cur = path;
    for (int r = 0; r < rounds; r++) {
        const uint64_t a = cur & sp, h = a | (a << 1) | (a >> 1);
        uint64_t up = cf_shfl64(h, LANE > 0 ? LANE - 1 : 0), dn = cf_shfl64(h, LANE < 63 ? LANE + 1 : 63);
        if (LANE == 0) up = 0;
        if (LANE >= H - 1) dn = 0;
        cur = (h | up | dn) & sp & ~set & full;
        if (LANE >= H) cur = 0;
        set |= cur;
    }
    wave_sync(); // every lane read its row before any is rewritten
    cf_write_row(c, set, SPACE, wall);
}

DEV void caveflyer_game_reset(RCtx &c, CaveScratch *S) {
    base_game_reset<PG_GAME_CAVEFLYER>(c);
    const int W = c.s.main_width, n = W * c.s.main_height;
    c.s.out_of_bounds_object = WALL_OBJ;
    RMARK(c, 0);
    cf_random_fill(c);
    cf_update(c, 4, 0);
    RMARK(c, 1);
    const int best = cf_find_best_room(c, S);
    RMARK(c, 2);
    if (best < 0) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    // the best room stays SPACE, its cells (ascending) are the free cells
    int nfree = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + LANE;
        const bool in = i < n && cf_in_best(S, W, i);
        if (i < n) {
            c.grid[i] = in ? SPACE : WALL_OBJ;
            S->f[i] = 0;
        }
        const unsigned long long m = ballot(in);
        if (in) S->list[nfree + __popcll(m & ((1ull << LANE) - 1ull))] = (int16_t)i;
        nfree += __popcll(m);
    }
    wave_sync();
    // simple_choose(free_cells.size(), 2) (fassert(k <= n), randgen.cpp:74)
    if (nfree < 2) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    int pick0 = randn(c, nfree), pick1 = randn(c, nfree);
    while (pick1 == pick0) pick1 = randn(c, nfree);
    const int agent_cell = S->list[pick0], goal_cell = S->list[pick1];
    EF(c, F_X, 0) = (float)((agent_cell % W) + .5);
    EF(c, F_Y, 0) = (float)((agent_cell / W) + .5);
    wave_sync();
    int ge = add_entity(c, (float)((goal_cell % W) + .5), (float)((goal_cell / W) + .5), 0, 0, .5f, CF_GOAL);
    EI(c, F_FLAGS, ge) = EF_AUTO_ERASE | EF_COLLIDES;
    RMARK(c, 2);
    const int npath = cf_find_path(c, S, agent_cell, goal_cell);
    RMARK(c, 3);
    const uint64_t path = cf_rows_of_path(c, S, npath);
    if (c.s.opt_distribution_mode != PG_MEMORY) cf_expand_room(c, path, 4, WALL_OBJ); // should_prune: path grown 4 times
    cf_update(c, 4, path); // the path cells stay SPACE after every round
    for (int q = LANE; q < npath; q += 64) c.grid[S->list2[q]] = CF_MARKER;
    wave_sync();
    nfree = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + LANE;
        int v = i < n ? c.grid[i] : -1;
        const bool sp = v == SPACE;
        if (v == WALL_OBJ) c.grid[i] = CF_CAVEWALL;
        if (i < n) S->f[i] = 0;
        const unsigned long long m = ballot(sp);
        if (sp) S->list[nfree + __popcll(m & ((1ull << LANE) - 1ull))] = (int16_t)i;
        nfree += __popcll(m);
    }
    wave_sync();
    RMARK(c, 4);
    const int chunk_size = nfree / 80, num_objs = 3 * chunk_size;
    // simple_choose(free_cells.size(), num_objs): rejection against the picks so far
    for (int i = 0; i < num_objs; i++) {
        int next = randn(c, nfree);
        while (S->f[next] & CF_TAKEN) next = randn(c, nfree);
        wave_sync();
        if (LANE == 0) {
            S->f[next] |= CF_TAKEN;
            S->b[i] = next;
        }
        wave_sync();
    }
    for (int i = 0; i < num_objs; i++) {
        const int val = S->list[S->b[i]];
        const float x = (float)((val % W) + .5), y = (float)((val / W) + .5);
        if (i < chunk_size) {
            const int e = add_entity(c, x, y, 0, 0, .5f, CF_OBSTACLE);
            EI(c, F_FLAGS, e) = EF_AUTO_ERASE | EF_COLLIDES;
        } else if (i < 2 * chunk_size) {
            const int e = add_entity(c, x, y, 0, 0, .5f, CF_TARGET);
            EF(c, F_HEALTH, e) = 5;
            EI(c, F_FLAGS, e) = EF_AUTO_ERASE | EF_COLLIDES;
        } else {
            const int e = add_entity(c, x, y, 0, 0, .5f, CF_ENEMY);
            // (.1 * rand01() + .1) * (randn(2) * 2 - 1): left operand first (g++, pinned in
            // tests/test_oracle_pins.py)
            const double mag = .1 * (double)rand01(c) + .1;
            const int sgn = randn(c, 2) * 2 - 1;
            const float vel = (float)(mag * sgn);
            if (rand01(c) < .5) EF(c, F_VX, e) = vel;
            else EF(c, F_VY, e) = vel;
            EI(c, F_FLAGS, e) = EF_AUTO_ERASE | EF_COLLIDES | EF_SMART_STEP;
        }
    }
    RMARK(c, 5);
    for (int i = LANE; i < n; i += 64)
        if (c.grid[i] == CF_MARKER) c.grid[i] = SPACE;
    wave_sync();
    c.s.out_of_bounds_object = CF_CAVEWALL;
    c.s.visibility = c.s.opt_distribution_mode == PG_EASY ? 10 : 16;
}

// ------------------------------------------------------------------ jumper (jumper.cpp:182-379)
DEV void mg_generate_maze_no_dead_ends(RCtx &c, MG &g);
DEV int jp_get(RCtx &c, int x, int y) { return get_obj(c, x, y); }
DEV bool jp_space_on_ground(RCtx &c, int x, int y) { // is_space_on_ground (:182-189)
    if (jp_get(c, x, y) != SPACE) return false;
    if (jp_get(c, x, y + 1) != SPACE) return false;
    const int below = jp_get(c, x, y - 1);
    return below == JP_CAVEWALL || below == c.s.out_of_bounds_object;
}
DEV bool jp_left_wall(RCtx &c, int x, int y) { return jp_get(c, x, y) == JP_CAVEWALL && jp_get(c, x + 1, y) == SPACE; }
DEV bool jp_right_wall(RCtx &c, int x, int y) { return jp_get(c, x, y) == JP_CAVEWALL && jp_get(c, x - 1, y) == SPACE; }
DEV bool jp_spike_site(RCtx &c, int x, int y) {
    return jp_space_on_ground(c, x, y) && jp_space_on_ground(c, x - 1, y) && jp_space_on_ground(c, x + 1, y);
}
DEV bool jp_left_run(RCtx &c, int x, int y) { return jp_left_wall(c, x, y) && jp_left_wall(c, x, y + 1) && jp_left_wall(c, x, y + 2); }
DEV bool jp_right_run(RCtx &c, int x, int y) {
    return jp_right_wall(c, x, y) && jp_right_wall(c, x, y + 1) && jp_right_wall(c, x, y + 2);
}

// The reference's in-order scans whose actions change the predicate of later cells (spike
// placement, long-wall breaking) run speculatively: 64 cells are tested at once against the
// current grid, the first hit is acted on (uniformly, with its RNG draws), and the scan resumes
// after it -- every cell is tested against exactly the grid the serial loop would show it.
template <typename P, typename A>
DEV void jp_ordered_scan(RCtx &c, int n, P pred, A act) {
    const int W = c.s.main_width;
    for (int start = 0; start < n;) {
        const int i = start + LANE;
        const unsigned long long m = ballot(i < n && pred(i % W, i / W));
        if (!m) {
            start += 64;
            continue;
        }
        const int first = start + __ffsll((long long)m) - 1;
        act(first % W, first / W);
        start = first + 1;
    }
}

// The two in-order scans of jumper.cpp:305-337 on row masks (lane y = row y, cf_row_of): the predicate
// of every cell is a mask expression, re-evaluated after each change, and the scan walks its set bits
// in index order (row-major), so every cell is tested against the grid the serial loop would show it.
//   spikes: is_space_on_ground at x - 1, x, x + 1 (space here and above, below CAVEWALL or out of bounds);
//           one rand01 per site, SPIKE placed below spike_prob
//   walls:  a 3-high left / right wall run at (x, y): one randn(3) per hit, cell (x, y + r) opened (once
//           a left run is broken the right run through the same cells is gone, so the reference's second
//           test is false whenever the first was true)
DEV uint64_t jp_rl64(uint64_t v, int lane) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane) << 32);
}
DEV void jp_scans(RCtx &c, float spike_prob) {
    const int W = c.s.main_width, H = c.s.main_height, oob = c.s.out_of_bounds_object;
    const uint64_t full = cf_row_full(W);
    uint64_t sp = cf_row_of(c, [](int v) { return v == SPACE; });
    uint64_t cw = cf_row_of(c, [](int v) { return v == JP_CAVEWALL; });
    const uint64_t ground = cf_row_of(c, [oob](int v) { return v == JP_CAVEWALL || v == oob; });
    const bool oob_space = oob == SPACE; // below row 0 is out of bounds: ground by definition
    auto row_at = [&](uint64_t v, int dy, uint64_t outside) { // row LANE + dy, `outside` beyond the grid
        const int src = LANE + dy;
        const uint64_t r = cf_shfl64(v, src < 0 ? 0 : (src > 63 ? 63 : src));
        return (src < 0 || src >= H) ? outside : r;
    };
    auto sites = [&]() {
        const uint64_t sog = sp & row_at(sp, 1, oob_space ? full : 0) & row_at(ground, -1, full);
        const uint64_t edge_l = oob_space ? 1ull : 0ull, edge_r = oob_space ? 1ull << (W - 1) : 0ull; // never: oob is a wall
        return LANE < H ? sog & ((sog << 1) | edge_l) & ((sog >> 1) | edge_r) & full : 0ull;
    };
    // scan 1: spikes.  A SPIKE leaves the SPACE mask (ground is unchanged: the cell was SPACE)
    uint64_t pm = sites();
    for (int y = 0, from = 0; y < H;) {
        const uint64_t m = jp_rl64(pm, y) & (from >= 64 ? 0ull : ~0ull << from);
        if (!m) {
            y++;
            from = 0;
            continue;
        }
        const int x = __builtin_ctzll(m);
        if (rand01(c) < spike_prob) {
            set_obj(c, x, y, JP_SPIKE);
            if (LANE == y) sp &= ~(1ull << x);
            pm = sites();
        }
        from = x + 1;
    }
    // scan 2: long walls
    auto runs = [&]() {
        const uint64_t spo = oob_space ? 1ull << (W - 1) : 0ull;
        const uint64_t lw = cw & ((sp >> 1) | spo), rw = cw & ((sp << 1) | (oob_space ? 1ull : 0ull)) & full;
        const uint64_t cwo = oob == JP_CAVEWALL ? full : 0ull; // rows beyond the grid: walls only if oob is
        const uint64_t lwo = cwo & (oob_space ? full : 0ull);  // (never a run: oob is not both wall and space)
        const uint64_t lr = lw & row_at(lw, 1, lwo) & row_at(lw, 2, lwo);
        const uint64_t rr = rw & row_at(rw, 1, lwo) & row_at(rw, 2, lwo);
        return LANE < H ? lr | rr : 0ull;
    };
    uint64_t pr = runs();
    for (int y = 0, from = 0; y < H;) {
        const uint64_t m = jp_rl64(pr, y) & (from >= 64 ? 0ull : ~0ull << from);
        if (!m) {
            y++;
            from = 0;
            continue;
        }
        const int x = __builtin_ctzll(m);
        const int yy = y + randn(c, 3); // left run, else right run: one opening either way
        set_obj(c, x, yy, SPACE);
        if (LANE == yy) {
            sp |= 1ull << x;
            cw &= ~(1ull << x);
        }
        pr = runs();
        from = x + 1;
    }
}

DEV void jumper_game_reset(RCtx &c, Scratch<PG_GAME_JUMPER> *X) {
    const int dm = c.s.opt_distribution_mode;
    auto &J = c.s.gs.jp;
    if (dm == PG_EASY) {
        c.s.visibility = 12;
        J.compass_dim = 3;
    } else {
        c.s.visibility = 16;
        J.compass_dim = 2;
    }
    if (dm == PG_MEMORY) c.s.timeout = 2000;
    int world_dim = 20; // choose_world_dim (:204-219)
    if (dm == PG_HARD) world_dim = 40;
    else if (dm == PG_MEMORY) world_dim = 45;
    c.s.main_width = world_dim;
    c.s.main_height = world_dim;
    base_game_reset<PG_GAME_JUMPER>(c);
    const int W = c.s.main_width, H = c.s.main_height, n = W * H;
    c.s.out_of_bounds_object = WALL_OBJ;
    c.s.wall_theme = randn(c, 4); // NUM_WALL_THEMES
    J.jump_count = 0;
    J.jump_delta = 0;
    J.jump_time = 0;
    c.s.has_support = 0;
    c.s.facing_right = 1;
    // MazeGen(maze_dim = W / MAZE_SCALE).generate_maze_no_dead_ends(), then each cell draws against
    // .8 (maze wall) or .2 (maze space) of its 3x3 maze block
    MG g;
    g.m = &X->mg;
    g.md = W / 3;
    g.ad = g.md + 2;
    if (g.ad > MG_MAX_DIM) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    RMARK(c, 6);
    mg_generate_maze_no_dead_ends(c, g);
    RMARK(c, 0);
    for (int base = 0; base < n;) {
        if (c.mti >= PG_MT_N) {
            mt_twist_lds(c.mt);
            c.mti = 0;
            mt_window_reset(c);
        }
        int m = PG_MT_N - c.mti;
        if (m > 64) m = 64;
        if (m > n - base) m = n - base;
        if (LANE < m) {
            const int i = base + LANE;
            const int obj = X->mg.grid[((i / W) / 3 + 1) * g.ad + (i % W) / 3 + 1];
            const float prob = obj == WALL_OBJ ? .8f : .2f;
            c.grid[i] = rg_rand01_of(mt_temper(c.mt[c.mti + LANE])) < prob ? WALL_OBJ : SPACE;
        }
        c.mti += m;
        base += m;
        wave_sync();
    }
    CaveScratch *S = &X->cf; // the maze is dead from here on
    cf_update(c, 2, 0);
    for (int i = LANE; i < n; i += 64) { // border cells
        const int x = i % W, y = i / W;
        if (x == 0 || y == 0 || x == W - 1 || y == H - 1) c.grid[i] = JP_CAVEWALL;
    }
    wave_sync();
    RMARK(c, 1);
    const int best = cf_find_best_room(c, S);
    if (best < 0) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    int nfree = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + LANE;
        const bool in = i < n && cf_in_best(S, W, i);
        if (i < n) {
            c.grid[i] = in ? SPACE : JP_CAVEWALL;
            S->f[i] = 0;
        }
        const unsigned long long m = ballot(in);
        if (in) S->list[nfree + __popcll(m & ((1ull << LANE) - 1ull))] = (int16_t)i;
        nfree += __popcll(m);
    }
    wave_sync();
    const int goal_cell = S->list[randn(c, nfree)]; // choose_one (randgen.cpp:43-47)
    int ncand = 0; // agent candidates: SPACE on ground, ascending
    for (int base = 0; base < n; base += 64) {
        const int i = base + LANE;
        const bool in = i < n && jp_space_on_ground(c, i % W, i / W);
        const unsigned long long m = ballot(in);
        if (in) S->list2[ncand + __popcll(m & ((1ull << LANE) - 1ull))] = (int16_t)i;
        ncand += __popcll(m);
    }
    wave_sync();
    if (ncand == 0) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    const int agent_cell = S->list2[randn(c, ncand)];
    wave_sync();
    RMARK(c, 2);
    const int npath = cf_find_path(c, S, agent_cell, goal_cell);
    RMARK(c, 3);
    if (dm != PG_MEMORY) cf_expand_room(c, cf_rows_of_path(c, S, npath), 4, JP_CAVEWALL); // should_prune
    RMARK(c, 4);
    add_entity(c, (float)((goal_cell % W) + .5), (float)((goal_cell / W) + .5), 0, 0, .5f, JP_GOAL); // entity 1
    const float spike_prob = dm == PG_MEMORY ? 0 : .2f;
    jp_scans(c, spike_prob);
    RMARK(c, 5);
    EF(c, F_X, 0) = (float)((agent_cell % W) + .5);
    EF(c, F_Y, 0) = (float)(agent_cell / W) + EF(c, F_RY, 0);
    wave_sync();
    // spike cells (get_cells_with_type, ascending) become SPIKE entities
    int nsp = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + LANE;
        const bool in = i < n && c.grid[i] == JP_SPIKE;
        const unsigned long long m = ballot(in);
        if (in) {
            S->list[nsp + __popcll(m & ((1ull << LANE) - 1ull))] = (int16_t)i;
            c.grid[i] = SPACE;
        }
        nsp += __popcll(m);
    }
    wave_sync();
    for (int k = 0; k < nsp; k++) {
        const int cell = S->list[k];
        const float spike_ry = 0.4f, spike_rx = 0.23f;
        add_entity_rxy(c, (float)((cell % W) + .5), (float)(cell / W) + spike_ry, 0, 0, spike_rx, spike_ry, JP_SPIKE);
    }
    for (int i = LANE; i < n; i += 64) // is_top_wall -> CAVEWALL_TOP (order-independent)
        if (c.grid[i] == JP_CAVEWALL && jp_get(c, i % W, i / W + 1) == SPACE) c.grid[i] = JP_CAVEWALL_TOP;
    wave_sync();
    EF(c, F_RX, 0) = 0.254f;
    EF(c, F_RY, 0) = 0.4f;
    c.s.out_of_bounds_object = JP_CAVEWALL;
}

// ------------------------------------------------------------------ chaser (chaser.cpp:146-252)
// MazeGen::generate_maze_no_dead_ends (mazegen.cpp:190-211): the scan visits cells in index
// order and may open a wall next to a later cell, so each step finds the first dead end at or
// after the scan position in the current grid (ballot), opens one of its walls, and resumes.
DEV void mg_generate_maze_no_dead_ends(RCtx &c, MG &g) {
    mg_generate_maze(c, g);
    // On row masks of the maze grid (lane y = row y, array_dim <= 33): mg_get_obj is INVALID_OBJ on
    // the border, so only interior cells count as SPACE / WALL neighbours.  A dead end is an interior
    // SPACE cell with exactly one SPACE neighbour; the scan walks them in index order against the
    // current grid (the masks are re-derived after every opened wall), opening the randn(nw)-th WALL
    // neighbour in get_neighbors order (-1, 0) (0, -1) (0, 1) (1, 0).
    const int ad = g.ad;
    const uint64_t inner = LANE >= 1 && LANE < ad - 1 ? ((1ull << (ad - 1)) - 1ull) & ~1ull : 0ull;
    uint64_t sp = 0, wl = 0;
    if (LANE < ad)
        for (int x = 0; x < ad; x++) {
            const int v = g.m->grid[LANE * ad + x];
            sp |= (uint64_t)(v == SPACE) << x;
            wl |= (uint64_t)(v == WALL_OBJ) << x;
        }
    sp &= inner;
    wl &= inner;
    auto row_of = [&](uint64_t v, int dy) {
        const int src = LANE + dy;
        const uint64_t r = cf_shfl64(v, src < 0 ? 0 : (src > 63 ? 63 : src));
        return (src < 0 || src >= ad) ? 0ull : r;
    };
    auto dead_ends = [&]() {
        const uint64_t a = sp << 1, b = row_of(sp, -1), d = row_of(sp, 1), e = sp >> 1;
        const uint64_t odd = a ^ b ^ d ^ e, two = (a & b) | (d & e) | ((a | b) & (d | e));
        return sp & odd & ~two;
    };
    uint64_t de = dead_ends();
    for (int y = 0, from = 0; y < ad;) {
        const uint64_t m = cf_rl64(de, y) & (from >= 64 ? 0ull : ~0ull << from);
        if (!m) {
            y++;
            from = 0;
            continue;
        }
        const int x = __builtin_ctzll(m);
        const uint64_t wr = cf_rl64(wl, y), wu = y > 0 ? cf_rl64(wl, y - 1) : 0ull, wd = cf_rl64(wl, y + 1);
        const bool nb[4] = {((wr >> (x - 1)) & 1) != 0, ((wu >> x) & 1) != 0, ((wd >> x) & 1) != 0, ((wr >> (x + 1)) & 1) != 0};
        const int nw = nb[0] + nb[1] + nb[2] + nb[3];
        if (nw > 0) {
            int n = randn(c, nw), k = 0;
            for (; k < 4; k++)
                if (nb[k] && n-- == 0) break;
            const int ox = x + (k == 0 ? -1 : (k == 3 ? 1 : 0)), oy = y + (k == 1 ? -1 : (k == 2 ? 1 : 0));
            mg_set_index(g, oy * ad + ox, SPACE);
            if (LANE == oy) {
                sp |= 1ull << ox;
                wl &= ~(1ull << ox);
            }
            de = dead_ends();
        }
        from = x + 1;
    }
}

// RandGen::simple_choose(n, k) (randgen.cpp:70-88), k <= 8, picks in LDS
DEV void simple_choose_small(RCtx &c, int n, int k, int16_t *sel) {
    if (k > 8 || k > n) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    for (int i = 0; i < k; i++) {
        int next = randn(c, n);
        for (;;) {
            bool seen = false;
            for (int j = 0; j < i; j++)
                if (sel[j] == next) seen = true;
            if (!seen) break;
            next = randn(c, n);
        }
        wave_sync();
        if (LANE == 0) sel[i] = (int16_t)next;
        wave_sync();
    }
}

// index of the n-th (0-based) position p in [0, count) with pred(p) true, in ascending p
template <typename P>
DEV int nth_where(int count, int n, P pred) {
    int seen = 0;
    for (int base = 0; base < count; base += 64) {
        int p = base + LANE;
        bool f = p < count && pred(p);
        unsigned long long b = ballot(f);
        int cnt = __popcll(b);
        if (n < seen + cnt) {
            bool mine = f && __popcll(b & ((1ull << LANE) - 1ull)) == n - seen;
            return base + __ffsll((long long)ballot(mine)) - 1;
        }
        seen += cnt;
    }
    return -1;
}
template <typename P>
DEV int count_where(int count, P pred) {
    int cnt = 0;
    for (int base = 0; base < count; base += 64) {
        int p = base + LANE;
        cnt += __popcll(ballot(p < count && pred(p)));
    }
    return cnt;
}

DEV void chaser_game_reset(RCtx &c, ChaserScratch *S) {
    int extra_orb_sign = 1;
    const int dm = c.s.opt_distribution_mode;
    if (dm == PG_EASY) { c.s.maze_dim = 11; c.s.total_enemies = 3; extra_orb_sign = 0; }
    else if (dm == PG_HARD) { c.s.maze_dim = 13; c.s.total_enemies = 3; extra_orb_sign = -1; }
    else { c.s.maze_dim = 19; c.s.total_enemies = 5; extra_orb_sign = 1; }
    const int md = c.s.maze_dim;
    c.s.main_width = md; // choose_world_dim (:141-144)
    c.s.main_height = md;
    base_game_reset<PG_GAME_CHASER>(c);
    c.s.opt_center_agent = 0;
    EF(c, F_RX, 0) = .5f;
    EF(c, F_RY, 0) = .5f;
    c.s.eat_time = -1 * c.s.eat_timeout;
    MG g;
    g.m = &S->mg;
    g.md = md;
    g.ad = md + 2;
    if (g.ad > MG_MAX_DIM) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    mg_generate_maze_no_dead_ends(c, g);
    const int extra_quad = randn(c, 4);
    // set_obj(i, j, maze (i + 1, j + 1) with WALL_OBJ -> MAZE_WALL)
    int16_t *mgrid = S->mg.grid;
    for (int k = LANE; k < md * md; k += 64) {
        int x = k % md, y = k / md;
        int obj = mgrid[(y + 1) * g.ad + (x + 1)];
        c.grid[y * md + x] = (int16_t)(obj == WALL_OBJ ? CH_MAZE_WALL : obj);
    }
    wave_sync();
    // quadrant lists: SPACE cells in the reference's x-major visiting order (i = x outer)
    for (int q = 0; q < 4; q++) {
        auto in_q = [&](int k) { // k = i * md + j (x-major)
            int i = k / md, j = k % md;
            int qi = ((double)i >= md / 2.0 ? 1 : 0) * 2 + ((double)j >= md / 2.0 ? 1 : 0);
            return qi == q && mgrid[(j + 1) * g.ad + (i + 1)] == SPACE;
        };
        const int qn = count_where(md * md, in_q);
        const int num_orbs = 1 + (q == extra_quad ? extra_orb_sign : 0);
        simple_choose_small(c, qn, num_orbs, S->sel);
        for (int j = 0; j < num_orbs; j++) {
            const int k = nth_where(md * md, S->sel[j], in_q);
            const int cell = (k % md) * md + k / md; // idx = j * maze_dim + i
            add_entity(c, (float)((cell % md) + .5), (float)((cell / md) + .5), 0, 0, 0.4f, CH_LARGE_ORB);
            wave_sync();
            if (LANE == 0) c.grid[cell] = CH_MARKER;
            wave_sync();
        }
    }
    // free_cells = get_cells_with_type(SPACE) (ascending)
    const int cells = md * md;
    auto is_free = [&](int i) { return c.grid[i] == SPACE; };
    const int nfree = count_where(cells, is_free);
    simple_choose_small(c, nfree, 1 + c.s.total_enemies, S->sel);
    int cell_of[8];
#pragma unroll
    for (int k = 0; k < 8; k++) cell_of[k] = k < 1 + c.s.total_enemies ? nth_where(cells, S->sel[k], is_free) : -1;
    EF(c, F_X, 0) = (float)((cell_of[0] % md) + .5);
    EF(c, F_Y, 0) = (float)((cell_of[0] / md) + .5);
    wave_sync();
#pragma unroll
    for (int k = 1; k < 8; k++) {
        if (k < 1 + c.s.total_enemies) {
            const int cell = cell_of[k];
            int e = add_entity(c, (float)((cell % md) + .5), (float)((cell / md) + .5), 0, 0, .5f, CH_ENEMY_EGG);
            EF(c, F_HEALTH, e) = (float)c.s.egg_timeout;
            wave_sync();
        }
    }
    // every free cell (enemy cells included) becomes an ORB; the LARGE_ORB markers become SPACE
    for (int i = LANE; i < cells; i += 64) {
        int v = c.grid[i];
        if (v == SPACE) c.grid[i] = CH_ORB;
        else if (v == CH_MARKER) c.grid[i] = SPACE;
    }
    c.s.total_orbs = nfree;
    c.s.orbs_collected = 0;
    wave_sync();
}

// ------------------------------------------------------------------ leaper (leaper.cpp:115-218)
DEV float lp_rand_sign(RCtx &c) { return (double)rand01(c) < 0.5 ? 1.0f : -1.0f; } // :91-97
DEV int lp_extra_space(RCtx &c) { return c.s.opt_distribution_mode == PG_EASY ? 0 : randn(c, 2); }

// has_any_collision over the LDS entity list (no leaper entity avoids collisions)
DEV bool lp_collides(const LeaperScratch *L, int n, float x, float y, float rx, float ry) {
    bool hit = false;
    for (int k = LANE; k < n; k += 64) {
        float tx = (rx + L->rx[k]) + 0.0f, ty = (ry + L->ry[k]) + 0.0f;
        if ((fabsf(x - L->x[k]) < tx) && (fabsf(y - L->y[k]) < ty)) hit = true;
    }
    return ballot(hit) != 0;
}

DEV void lp_push(LeaperScratch *L, int &n, int cap, float x, float y, float vx, float rx, float ry, int type, int theme,
                 int born, bool &overflow) {
    if (n >= cap) {
        overflow = true;
        return;
    }
    if (LANE == 0) {
        L->x[n] = x; L->y[n] = y; L->vx[n] = vx; L->rx[n] = rx; L->ry[n] = ry;
        L->type[n] = (int8_t)type; L->theme[n] = (int8_t)theme; L->born[n] = (int16_t)born;
    }
    wave_sync();
    n++;
}

DEV void leaper_game_reset(RCtx &c, LeaperScratch *L) {
    base_game_reset<PG_GAME_LEAPER>(c);
    c.s.opt_center_agent = 0;
    EF(c, F_Y, 0) = EF(c, F_RY, 0);
    const int dm = c.s.opt_distribution_mode;
    float min_car_speed = 0.05f, max_car_speed = 0.2f, min_log_speed = 0.05f, max_log_speed = 0.1f;
    if (dm == PG_EASY) {
        min_car_speed = 0.03f; max_car_speed = 0.12f; min_log_speed = 0.025f; max_log_speed = 0.075f;
    } else if (dm == PG_EXTREME) {
        min_car_speed = 0.1f; max_car_speed = 0.3f; min_log_speed = 0.1f; max_log_speed = 0.2f;
    }
    const int w = c.s.main_width;
    c.s.bottom_road_y = lp_extra_space(c) + 1;
    const int max_diff = dm == PG_EASY ? 3 : 4;
    const int difficulty = randn(c, max_diff + 1);
    const int extra_lane_option = dm == PG_EASY ? 0 : randn(c, 4);
    c.s.num_road_lanes = difficulty + (extra_lane_option == 2 ? 1 : 0);
    for (int lane = 0; lane < c.s.num_road_lanes; lane++) {
        // rand_sign() * randrange(): g++ evaluates the left operand first (pinned,
        // tests/test_oracle_pins.py::test_leaper_operand_order_pinned)
        const float sgn = lp_rand_sign(c);
        const float spd = rand01(c) * (max_car_speed - min_car_speed) + min_car_speed;
        if (LANE == 0) L->road[lane] = sgn * spd;
        fill_elem(c, 0, c.s.bottom_road_y + lane, w, 1, LP_ROAD);
    }
    c.s.bottom_water_y = c.s.bottom_road_y + c.s.num_road_lanes + lp_extra_space(c) + 1;
    c.s.num_water_lanes = difficulty + (extra_lane_option == 3 ? 1 : 0);
    int curr_sign = (int)lp_rand_sign(c);
    for (int lane = 0; lane < c.s.num_water_lanes; lane++) {
        const float spd = rand01(c) * (max_log_speed - min_log_speed) + min_log_speed;
        if (LANE == 0) L->water[lane] = curr_sign * spd;
        curr_sign *= -1;
        fill_elem(c, 0, c.s.bottom_water_y + lane, w, 1, LP_WATER);
    }
    c.s.goal_y = c.s.bottom_water_y + c.s.num_water_lanes + 1;
    wave_sync();
#pragma unroll
    for (int k = 0; k < 5; k++) {
        c.s.road_lane_speeds[k] = k < c.s.num_road_lanes ? L->road[k] : 0.0f;
        c.s.water_lane_speeds[k] = k < c.s.num_water_lanes ? L->water[k] : 0.0f;
    }

    RMARK(c, 0);
    // initial entities: spawn_entities + step_entities (no erase) while i < main_width / min(speed).
    // The loop runs ~400 times with a draw per lane: the entities' x / vx / y / rx / ry live in registers
    // (entity k in lane k % 64, slot k / 64), the lane speeds in scalars, so an iteration touches no LDS;
    // a push also records the entity in the LDS lists for the write-out below
    constexpr int NS = PG_CAP / 64;
    float ex[NS], evx[NS], ey[NS], erx[NS], ery[NS];
#pragma unroll
    for (int j = 0; j < NS; j++) ex[j] = evx[j] = ey[j] = erx[j] = ery[j] = 0.0f;
    int n = 0;
    bool overflow = false;
    auto push = [&](float x, float y, float vx, float rx, float ry, int type, int theme, int born) {
        if (n >= PG_CAP - 1) {
            overflow = true;
            return;
        }
#pragma unroll
        for (int j = 0; j < NS; j++)
            if (j == (n >> 6) && LANE == (n & 63)) {
                ex[j] = x; evx[j] = vx; ey[j] = y; erx[j] = rx; ery[j] = ry;
            }
        if (LANE == 0) {
            L->x[n] = x; L->y[n] = y; L->vx[n] = vx; L->rx[n] = rx; L->ry[n] = ry;
            L->type[n] = (int8_t)type; L->theme[n] = (int8_t)theme; L->born[n] = (int16_t)born;
        }
        n++;
    };
    auto collides = [&](float x, float y, float rx, float ry) { // has_any_collision (no entity avoids it)
        bool hit = false;
#pragma unroll
        for (int j = 0; j < NS; j++)
            if (j * 64 < n && j * 64 + LANE < n) {
                const float tx = (rx + erx[j]) + 0.0f, ty = (ry + ery[j]) + 0.0f;
                if ((fabsf(x - ex[j]) < tx) && (fabsf(y - ey[j]) < ty)) hit = true;
            }
        return ballot(hit) != 0;
    };
    push(EF(c, F_X, 0), EF(c, F_Y, 0), 0, EF(c, F_RX, 0), EF(c, F_RY, 0), PLAYER, 0, 0);
    const float mn = min_car_speed < min_log_speed ? min_car_speed : min_log_speed;
    const int ncar_themes = c.d.num_themes[LP_CAR];
    // c.s is the LDS copy of the env: everything the loop reads from it goes to registers first
    const int nroad = c.s.num_road_lanes, nwater = c.s.num_water_lanes;
    const int road_y = c.s.bottom_road_y, water_y = c.s.bottom_water_y;
    float rsp[5], wsp[5], rpr[5], wpr[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        rsp[k] = c.s.road_lane_speeds[k];
        wsp[k] = c.s.water_lane_speeds[k];
        rpr[k] = (float)(fabs((double)rsp[k]) / 6.0);
        wpr[k] = (float)(fabs((double)wsp[k]) / 2.0);
    }
    // lane j's spawn probability (road lanes, then water lanes) for the speculative pass below
    float pj = 0.0f;
#pragma unroll
    for (int q = 0; q < 5; q++) {
        if (LANE == q && q < nroad) pj = rpr[q];
        if (LANE == nroad + q && q < nwater) pj = wpr[q];
    }
    const int m = nroad + nwater;
    int iters = 0;
    for (int i = 0; (float)i < w / mn; i++) {
        // Speculative pass: an iteration draws one rand01 per lane in lane order, plus a theme draw
        // after each car spawn.  Lane j tests draw mti + j from the register window at once; when no
        // lane spawns (most iterations) that is exactly the serial outcome and the m draws are consumed;
        // otherwise the iteration runs serially below from the same mti.
        if (c.mti + m <= PG_MT_N) {
            if (c.mti - c.wbase < 0 || c.mti - c.wbase + m > 64) {
                c.wbase = c.mti;
                c.win = c.mti + LANE < PG_MT_N ? mt_temper(c.mt[c.mti + LANE]) : 0u;
            }
            const int src = c.mti - c.wbase + LANE;
            const uint32_t wj = (uint32_t)__shfl((int)c.win, src < 64 ? src : 63);
            if (!ballot(LANE < m && rg_rand01_of(wj) < pj)) {
                c.mti += m;
#pragma unroll
                for (int j = 0; j < NS; j++)
                    if (j * 64 < n && j * 64 + LANE < n && j * 64 + LANE >= 1) ex[j] = ex[j] + evx[j];
                iters++;
                continue;
            }
        }
#pragma unroll
        for (int lane = 0; lane < 5; lane++) {
            if (lane >= nroad) break;
            const float speed = rsp[lane], spawn_prob = rpr[lane];
            if (rand01(c) < spawn_prob) {
                const float x = speed > 0 ? (-1 * LP_MONSTER_RADIUS) : (w + LP_MONSTER_RADIUS);
                const float y = (float)(road_y + lane + 0.5);
                const int theme = randn(c, ncar_themes); // choose_random_theme before the check
                if (!collides(x, y, 2 * LP_MONSTER_RADIUS, LP_MONSTER_RADIUS))
                    push(x, y, speed, 2 * LP_MONSTER_RADIUS, LP_MONSTER_RADIUS, LP_CAR, theme, i);
            }
        }
#pragma unroll
        for (int lane = 0; lane < 5; lane++) {
            if (lane >= nwater) break;
            const float speed = wsp[lane], spawn_prob = wpr[lane];
            if (rand01(c) < spawn_prob) {
                const float x = speed > 0 ? (-1 * LP_LOG_RADIUS) : (w + LP_LOG_RADIUS);
                const float y = (float)(water_y + lane + 0.5);
                if (!collides(x, y, LP_LOG_RADIUS, LP_LOG_RADIUS))
                    push(x, y, speed, LP_LOG_RADIUS, LP_LOG_RADIUS, LP_LOG, 0, i);
            }
        }
        // Entity::step of every non-smart entity: x += vx (vy = 0); the agent (smart, at rest) stays
#pragma unroll
        for (int j = 0; j < NS; j++)
            if (j * 64 < n && j * 64 + LANE < n && j * 64 + LANE >= 1) ex[j] = ex[j] + evx[j];
        iters++;
    }
    wave_sync(); // the pushes' LDS records
#pragma unroll
    for (int j = 0; j < NS; j++)
        if (j * 64 + LANE < n) L->x[j * 64 + LANE] = ex[j];
    wave_sync();
    RMARK(c, 1);
    if (overflow) c.s.error = PG_ERR_ENTITY_OVERFLOW;
    // the list to HBM: Entity ctor defaults (entity.cpp:8-47) + what the build set
    for (int k = 1 + LANE; k < n; k += 64) {
        const int type = L->type[k];
        const float vx = L->vx[k];
        EF(c, F_X, k) = L->x[k]; EF(c, F_Y, k) = L->y[k]; EF(c, F_VX, k) = vx; EF(c, F_VY, k) = 0;
        EF(c, F_RX, k) = L->rx[k]; EF(c, F_RY, k) = L->ry[k];
        EF(c, F_ROTATION, k) = (type == LP_CAR && vx < 0) ? PI_F : 0.0f;
        EF(c, F_VROT, k) = 0;
        EF(c, F_ALPHA, k) = 1.0f; EF(c, F_ALPHA_DECAY, k) = 1.0f; EF(c, F_GROW_RATE, k) = 1.0f;
        EF(c, F_FRICTION, k) = 1; EF(c, F_COLLISION_MARGIN, k) = 0; EF(c, F_HEALTH, k) = 1;
        EF(c, F_THETA, k) = -100; EF(c, F_CLIMBER_SPAWN_X, k) = 0;
        EI(c, F_TYPE, k) = type; EI(c, F_IMAGE_TYPE, k) = type; EI(c, F_IMAGE_THEME, k) = L->theme[k];
        EI(c, F_RENDER_Z, k) = 0; EI(c, F_LIFE_TIME, k) = iters - L->born[k]; EI(c, F_EXPIRE_TIME, k) = -1;
        EI(c, F_FIRE_TIME, k) = -1; EI(c, F_SPAWN_TIME, k) = -1; EI(c, F_FLAGS, k) = EF_AUTO_ERASE;
    }
    if (LANE == 0) EI(c, F_LIFE_TIME, 0) = iters;
    wave_sync();
    c.s.num_ents = n;
    add_entity_rxy(c, (float)(w / 2.0), (float)(c.s.goal_y - .5), 0, 0, (float)(w / 2.0), .5f, LP_FINISH_LINE);
}

// ------------------------------------------------------------------ Game::reset
template <int G>
DEV void reset_env(PGDev &d, int env, uint32_t *lds_mt, int16_t *lds_grid, Scratch<G> *scratch, bool initial,
                   PGEnv *lds_env, AgLds *ag) {
    {
        const uint2 *src = reinterpret_cast<const uint2 *>(d.envs + env);
        reinterpret_cast<uint2 *>(lds_env)[LANE] = src[LANE]; // 64 lanes x 8 B = the 512-B PGEnv
    }
    wave_sync();
    RCtx c{d, env, *lds_env};
    c.Eb = reinterpret_cast<char *>(d.ents + pg_ent_index(env, 0, 0));
    c.ag = ag;
    c.mt = lds_mt;
    c.grid = lds_grid;
#ifdef PG_PROF_RESET
    c.last = __builtin_amdgcn_s_memtime();
    if (LANE == 0) d.prof[(size_t)env * 16] += 1; // the reset count (the step phases are off here)
#endif
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
    mt_window_reset(c);
    if constexpr (G == PG_GAME_COINRUN) coinrun_game_reset(c);
    if constexpr (G == PG_GAME_BIGFISH) bigfish_game_reset(c);
    if constexpr (G == PG_GAME_MAZE) maze_game_reset(c, &scratch->mg);
    if constexpr (G == PG_GAME_HEIST) heist_game_reset(c, &scratch->mg);
    if constexpr (G == PG_GAME_MINER) miner_game_reset(c, &scratch->mn);
    if constexpr (G == PG_GAME_CLIMBER) climber_game_reset(c);
    if constexpr (G == PG_GAME_LEAPER) leaper_game_reset(c, &scratch->lp);
    if constexpr (G == PG_GAME_CHASER) chaser_game_reset(c, &scratch->ch);
    if constexpr (G == PG_GAME_FRUITBOT) fruitbot_game_reset(c, scratch->part);
    if constexpr (G == PG_GAME_DODGEBALL) dodgeball_game_reset(c, scratch->rooms);
    if constexpr (G == PG_GAME_PLUNDER) plunder_game_reset(c);
    if constexpr (G == PG_GAME_STARPILOT) starpilot_game_reset(c, &scratch->sp);
    if constexpr (G == PG_GAME_BOSSFIGHT) bossfight_game_reset(c);
    if constexpr (G == PG_GAME_NINJA) ninja_game_reset(c);
    if constexpr (G == PG_GAME_CAVEFLYER) caveflyer_game_reset(c, &scratch->cf);
    if constexpr (G == PG_GAME_JUMPER) jumper_game_reset(c, scratch);
    c.s.cur_time = 0;
    c.s.total_reward = 0;
    c.s.episodes_remaining -= 1;
    c.s.action = c.s.default_action;
    c.s.rg_mti = c.mti;
    RMARK(c, 6);

    // write the generator, the grid and the scalars back to HBM
    wave_sync();
    for (int i = LANE; i < PG_MT_N; i += 64) rg[i] = lds_mt[i];
    int cells = c.s.main_width * c.s.main_height;
    if (cells > PG_GRID_MAX) cells = PG_GRID_MAX;
    int16_t *g = d.grid + (size_t)env * PG_GRID_MAX;
    const uint4 *src = reinterpret_cast<const uint4 *>(lds_grid);
    uint4 *dst = reinterpret_cast<uint4 *>(g);
    for (int i = LANE; i < (cells + 7) / 8; i += 64) dst[i] = src[i];
    // int8 mirror for the step kernel (valid when every cell fits)
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
                if (v < -127 || v > 127) fits = false; // -128 marks an unstaged LDS cell in the step kernel
                word |= (uint32_t)(uint8_t)v << (8 * b);
            }
            w[q] = word;
        }
        reinterpret_cast<uint4 *>(g8)[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    c.s.grid8_ok = ballot(!fits) == 0;
    if constexpr (G == PG_GAME_MAZE || G == PG_GAME_MINER) {
        // fork latent state (maze.cpp:134-165, miner.cpp:363-396): grid_size, grid (zero padded),
        // agent_pos, exit_pos (miner: the exit entity); the step kernel keeps them current
        int32_t *lat = d.latent + (size_t)env * PG_LATENT_N;
        for (int i = LANE; i < PG_LATENT_GRID; i += 64) lat[2 + i] = i < cells ? (int32_t)lds_grid[i] : 0;
        if (LANE == 0) {
            lat[0] = c.s.main_width;
            lat[1] = c.s.main_height;
            lat[2 + PG_LATENT_GRID] = (int)EF(c, F_X, 0);
            lat[3 + PG_LATENT_GRID] = (int)EF(c, F_Y, 0);
            lat[4 + PG_LATENT_GRID] = 0;
            lat[5 + PG_LATENT_GRID] = 0;
            if constexpr (G == PG_GAME_MINER) { // the exit is the entity after the agent
                lat[4 + PG_LATENT_GRID] = (int)EF(c, F_X, 1);
                lat[5 + PG_LATENT_GRID] = (int)EF(c, F_Y, 1);
            }
        }
    }
    if (LANE == 0) {
        d.level_seed[env] = c.s.current_level_seed;
        if (initial) { // first observation of set_buffers (vecgame.cpp:381-409): step_data from the ctor
            d.rew[env] = c.s.sd_reward;
            d.first[env] = (uint8_t)c.s.sd_done;
            d.prev_level_seed[env] = c.s.prev_level_seed;
            d.prev_level_complete[env] = (uint8_t)c.s.sd_level_complete;
        }
        if (c.s.error) atomicOr(d.error_any, 1 << c.s.error);
    }
    wave_sync();
    reinterpret_cast<uint2 *>(d.envs + env)[LANE] = reinterpret_cast<const uint2 *>(lds_env)[LANE];
    wave_sync();
    RMARK(c, 7);
}

// ------------------------------------------------------------------ level prefetch
// The spare's view of the device state: the arrays a reset writes, redirected to the spare
DEV PGDev spare_view(const PGDev &d) {
    PGDev v = d;
    v.envs = d.sp_envs;
    v.ents = d.sp_ents;
    v.grid = d.sp_grid;
    v.grid8 = d.sp_grid8;
    v.mt = d.sp_mt;
    v.latent = d.sp_latent;
    v.level_seed = d.sp_level_seed;
    return v;
}
DEV int sp_slot(const PGDev &d, int act) { return ((act % d.sp_lag) + d.sp_lag) % d.sp_lag; }
// constant indices only: a dynamic index into the by-value kernel argument made the compiler keep a
// private copy of the whole PGDev in scratch (464 B per lane, written by every wave of the persistent
// grid: 4,096 waves x 64 lanes x 464 B = the 121.6 MB of the round-3 reset WRITE_SIZE)
DEV bool sp_masked(const PGDev &d, int w) {
    // readfirstlane: selects of the four values, not a load through a selected address into the copy
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(d.sp_mask[0]), m1 = __builtin_amdgcn_readfirstlane(d.sp_mask[1]);
    const uint32_t m2 = __builtin_amdgcn_readfirstlane(d.sp_mask[2]), m3 = __builtin_amdgcn_readfirstlane(d.sp_mask[3]);
    const int q = w >> 5;
    const uint32_t m = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
    return (m >> (w & 31)) & 1;
}

// After the reset (or swap) of `env` at act `act`: its next level's input -- the post-reset scalars
// (in LDS) with every step-changeable word poisoned, and the level-seed generator -- is queued for
// the prefetch kernel.  The spare then equals a reset at the end of the coming episode: that reset
// reads only members the episode does not change (options, counters, the level-seed generator);
// the step-changed members it does not write keep the live values at the swap.
template <int G>
DEV void request_spare(PGDev &d, int env, int act, const PGEnv *lds_env, int slot) {
    const int par = sp_slot(d, act);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(lds_env);
    uint32_t *dst = reinterpret_cast<uint32_t *>(d.sp_in + (size_t)par * d.num_envs + env);
    for (int w = LANE; w < (int)(sizeof(PGEnv) / 4); w += 64) dst[w] = sp_masked(d, w) ? PG_SP_SENT : src[w];
    __threadfence(); // this wave's level-seed generator writes, before reading them back
    const uint32_t *lsg = d.mt + (size_t)env * 2 * PG_MT_WORDS + PG_MT_WORDS;
    uint32_t *lo = d.sp_in_lsg + ((size_t)par * d.num_envs + env) * PG_MT_WORDS;
    for (int i = LANE; i < PG_MT_WORDS; i += 64) lo[i] = __hip_atomic_load(lsg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (LANE == 0) {
        d.sp_gen[env] = act;
        const int q = atomicAdd(d.sp_count + par * PG_NUM_GAMES + slot, 1);
        d.sp_queue[((size_t)par * PG_NUM_GAMES + slot) * d.num_envs + q] = env;
    }
    wave_sync();
}

// The episode of `env` ended and its spare is complete: the spare becomes the live state (what
// reset_env would have produced), the step-changed members the reset does not write keep their
// live values.  Leaves the new scalars in lds_env too.
template <int G>
DEV void swap_spare(PGDev &d, int env, PGEnv *lds_env) {
    const uint32_t *sp = reinterpret_cast<const uint32_t *>(d.sp_envs + env);
    const uint32_t *lv = reinterpret_cast<const uint32_t *>(d.envs + env);
    uint32_t *out = reinterpret_cast<uint32_t *>(lds_env);
    for (int w = LANE; w < (int)(sizeof(PGEnv) / 4); w += 64) {
        uint32_t a = sp[w];
        if (sp_masked(d, w) && a == PG_SP_SENT) a = lv[w];
        out[w] = a;
    }
    wave_sync();
    const int ne = G == PG_GAME_STARPILOT ? PG_CAP : min(max(lds_env->num_ents, 0), PG_CAP);
    for (int f = 0; f < PG_NF; f++)
        for (int i = LANE; i < ne; i += 64) d.ents[pg_ent_index(env, f, i)] = d.sp_ents[pg_ent_index(env, f, i)];
    int cells = lds_env->main_width * lds_env->main_height;
    if (cells > PG_GRID_MAX || cells < 0) cells = PG_GRID_MAX;
    const uint4 *g16 = reinterpret_cast<const uint4 *>(d.sp_grid + (size_t)env * PG_GRID_MAX);
    uint4 *o16 = reinterpret_cast<uint4 *>(d.grid + (size_t)env * PG_GRID_MAX);
    for (int i = LANE; i < (cells + 7) / 8; i += 64) o16[i] = g16[i];
    const uint4 *g8 = reinterpret_cast<const uint4 *>(d.sp_grid8 + (size_t)env * PG_GRID_MAX);
    uint4 *o8 = reinterpret_cast<uint4 *>(d.grid8 + (size_t)env * PG_GRID_MAX);
    for (int i = LANE; i < (cells + 15) / 16; i += 64) o8[i] = g8[i];
    const uint32_t *m = d.sp_mt + (size_t)env * 2 * PG_MT_WORDS;
    uint32_t *mo = d.mt + (size_t)env * 2 * PG_MT_WORDS;
    for (int i = LANE; i < 2 * PG_MT_WORDS; i += 64) mo[i] = m[i];
    if constexpr (G == PG_GAME_MAZE || G == PG_GAME_MINER) {
        const int32_t *l = d.sp_latent + (size_t)env * PG_LATENT_N;
        int32_t *lo = d.latent + (size_t)env * PG_LATENT_N;
        for (int i = LANE; i < PG_LATENT_N; i += 64) lo[i] = l[i];
    }
    if (LANE == 0) {
        d.level_seed[env] = lds_env->current_level_seed;
        if (lds_env->error) atomicOr(d.error_any, 1 << lds_env->error);
    }
    wave_sync();
    reinterpret_cast<uint2 *>(d.envs + env)[LANE] = reinterpret_cast<const uint2 *>(lds_env)[LANE];
    wave_sync();
}

// mode 1: reset every env in env_list / 0..count-1 (initial reset of set_buffers); mode 0: drain
// this game's queue filled by the step kernel (swapping in complete spares); mode 2: generate the
// spares requested at act `act`.  With prefetch on (d.sp_envs), modes 0 and 1 request the next
// spare of every env they reset; a spare requested at act a is complete once the prefetch launch
// of act a is (the host orders the reset of act a + sp_lag after it).  GEN: use_generated_assets (the
// AssetGen scratch is allocated only in these instances).
template <int G, bool GEN>
__global__ __launch_bounds__(64) void pg_reset_kernel(PGDev d, const int32_t *env_list, int count, int mode, int act, int slot) {
    __shared__ uint32_t lds_mt[PG_MT_N];
    __shared__ __attribute__((aligned(16))) int16_t lds_grid[PG_GRID_MAX];
    __shared__ Scratch<G> scratch;
    __shared__ __attribute__((aligned(16))) PGEnv lds_env;
    AgLds *ag = nullptr;
    if constexpr (GEN) {
        __shared__ AgLds ag_lds;
        ag = &ag_lds;
    }
    PGDev dv = game_view(d, G);
    if (mode == 2) {
        const int par = sp_slot(d, act);
        const int n = d.sp_count[par * PG_NUM_GAMES + slot];
        const int32_t *queue = d.sp_queue + ((size_t)par * PG_NUM_GAMES + slot) * d.num_envs;
        PGDev sv = spare_view(dv);
        for (int q = blockIdx.x; q < n; q += gridDim.x) {
            const int env = queue[q];
            reinterpret_cast<uint2 *>(d.sp_envs + env)[LANE] =
                reinterpret_cast<const uint2 *>(d.sp_in + (size_t)par * d.num_envs + env)[LANE];
            const uint32_t *li = d.sp_in_lsg + ((size_t)par * d.num_envs + env) * PG_MT_WORDS;
            uint32_t *lo = d.sp_mt + (size_t)env * 2 * PG_MT_WORDS + PG_MT_WORDS;
            for (int i = LANE; i < PG_MT_WORDS; i += 64) lo[i] = li[i];
            __threadfence();
            wave_sync();
            reset_env<G>(sv, env, lds_mt, lds_grid, &scratch, false, &lds_env, ag);
        }
        return;
    }
    const int n = mode == 1 ? count : d.reset_count[slot];
    const int32_t *queue = d.reset_queue + (size_t)slot * d.num_envs;
    for (int q = blockIdx.x; q < n; q += gridDim.x) {
        const int env = mode == 1 ? (env_list ? env_list[q] : q) : queue[q];
        const int gen = d.sp_envs ? d.sp_gen[env] : PG_SP_NONE;
        if (mode == 0 && gen != PG_SP_NONE && gen <= act - d.sp_lag) swap_spare<G>(dv, env, &lds_env);
        else reset_env<G>(dv, env, lds_mt, lds_grid, &scratch, mode == 1, &lds_env, ag);
        if (d.sp_envs) request_spare<G>(dv, env, act, &lds_env, slot);
    }
}

// The use_generated_assets sprites of one game (initialize_asset_if_necessary,
// basic-abstract-game.cpp:79-123): workgroup t paints image type t -- asset_rand_gen.seed(
// fixed_asset_seed + t); generate_resource(QImage(64, 64, ARGB32), 0, 5, use_block_asset(t)) -- into
// out[t][64][64], stored premultiplied as the compositor reads it (the pixels are opaque or clear).
__global__ __launch_bounds__(64) void pg_assetgen_sprites_kernel(int game, uint32_t seed0, uint32_t *out) {
    __shared__ uint32_t lds_mt[PG_MT_N];
    __shared__ AgLds ag_lds;
    const int t = blockIdx.x;
    mt_seed_lds(lds_mt, seed0 + (uint32_t)t);
    struct LdsRng {
        uint32_t *mt;
        int32_t mti;
        DEV uint32_t next() { return mt_next_lds(mt, mti); }
    };
    uint32_t *img = out + (size_t)t * AG_SPRITE_DIM * AG_SPRITE_DIM;
    AgPainter<LdsRng> p{img, AG_SPRITE_DIM, AG_SPRITE_DIM, AG_FMT_ARGB32, 0, &ag_lds, LdsRng{lds_mt, PG_MT_N}, 0};
    ag_generate_resource(p, 0, 5, ag_use_block_asset(game, t));
    wave_sync();
    for (int i = LANE; i < AG_SPRITE_DIM * AG_SPRITE_DIM; i += 64) {
        const uint32_t v = img[i];
        img[i] = (v >> 24) == 255 ? v : 0u;
    }
    if (p.err && LANE == 0) img[0] = 0xdeadbeefu; // flagged to the host (never a valid premultiplied texel)
}

} // namespace

extern "C" void pg_launch_reset(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s,
                                int mode, int grid, int act, int slot) {
    if (count <= 0) return;
    int g = grid > 0 ? grid : (count < 4096 ? count : 4096);
#define PG_CASE(G)                                                                                              \
    case G:                                                                                                     \
        if (d->gen_bg) hipLaunchKernelGGL((pg_reset_kernel<G, true>), dim3(g), dim3(64), 0, s, *d, env_list, count, mode, act, slot); \
        else hipLaunchKernelGGL((pg_reset_kernel<G, false>), dim3(g), dim3(64), 0, s, *d, env_list, count, mode, act, slot); \
        break;
    switch (game) {
        PG_CASE(PG_GAME_COINRUN)
        PG_CASE(PG_GAME_BIGFISH)
        PG_CASE(PG_GAME_MAZE)
        PG_CASE(PG_GAME_HEIST)
        PG_CASE(PG_GAME_MINER)
        PG_CASE(PG_GAME_CLIMBER)
        PG_CASE(PG_GAME_LEAPER)
        PG_CASE(PG_GAME_CHASER)
        PG_CASE(PG_GAME_FRUITBOT)
        PG_CASE(PG_GAME_DODGEBALL)
        PG_CASE(PG_GAME_PLUNDER)
        PG_CASE(PG_GAME_STARPILOT)
        PG_CASE(PG_GAME_BOSSFIGHT)
        PG_CASE(PG_GAME_NINJA)
        PG_CASE(PG_GAME_CAVEFLYER)
        PG_CASE(PG_GAME_JUMPER)
    default: break;
    }
#undef PG_CASE
}

extern "C" int pg_launch_assetgen_sprites(int game, uint32_t seed0, uint32_t *d_out, int types, hipStream_t s) {
    if (types <= 0) return 0;
    hipLaunchKernelGGL(pg_assetgen_sprites_kernel, dim3(types), dim3(64), 0, s, game, seed0, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
