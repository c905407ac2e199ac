// pg_step.hip -- per-env step kernel: Game::step + BasicAbstractGame::game_step + the per-game
// game_step (reference game.cpp:136-171, basic-abstract-game.cpp:602-765, 1095-1159;
// games/coinrun.cpp:123-211, 451-498; bigfish.cpp:45-106; maze.cpp:107-131; heist.cpp:66-96,
// 205-209).  One wavefront per env; done envs are queued for pg_reset (level generation)
// and every env is then drawn by pg_render.  The kernel is a template over the game id:
// the physics core is shared, the reference's virtual hooks are `if constexpr` branches.
#include "pg_device.h"
#include <utility>

namespace {

struct Ctx {
    // the kernel argument itself (by reference: its fields are loaded from the kernarg segment where they
    // are used; a by-value copy here loaded every pointer at entry and spilled them for the whole step)
    const PGDev &d;
    // the env's scalars in HBM, for the agent's ghost only (ghost_*: read and written where the agent is
    // erased, a rare path -- kept out of the registers the whole step would otherwise hold them in)
    PGEnv *gp;
    int env;
    PGEnv s;        // uniform copy of this env's scalars
    char *Eb;       // this env's entity block (pg_ent_index): field f of slot i at byte (f * PG_CAP + i) * 4
    const int16_t *G; // this env's grid
    uint32_t *lds;  // 624-word twist staging
    int16_t *ilist; // LDS: ascending indices of entities that can interact in sub_step
    int nlist;
    int16_t *slist; // LDS: smart entity indices (fast step_entities path)
    float4 *ibox;   // LDS: static interactors' (x, y, rx, ry) for the lane-parallel smart steps
    int *iinfo;     // LDS: static interactors' index | will_erase << 31
    int8_t *grid8;  // LDS copy of the grid
    uint8_t *moved; // LDS has_moved map (miner)
    bool grid8_ok;
    bool ireg;      // interactors cached per lane (see build_interactor_list)
    int i_idx;
    float i_x, i_y, i_rx, i_ry;
    bool i_erase;
    int i_theme;
    float av_vy, av_ry; // the agent's vy / ry as other objects' steps see it (coinrun's crate rule)
    float *pstk;        // LDS: sub_step's suspended push frames (5 x {vx, vy, upper, acc} + the child's key)
    uint32_t *memo;     // LDS (aliases the twist staging, idle during step_entities): push-chain memo
    int nmemo;          // its entries (reset per basic_step_object)
    PTimer pt;      // diagnostic phase timer (PG_PROFILE builds only)
#ifdef PG_PROF_SMART
    uint64_t sm[6]; // diagnostic (PROFILE=1 EXTRA=-DPG_PROF_SMART): smart-entity census, prof[env][8..13]
#endif
    Census cs;      // diagnostic wave census (PG_CENSUS builds only)
};

// 32-bit byte offsets from the env's block: one base register pair for every entity access (the
// global_load saddr + voffset form) instead of 64-bit plane-address arithmetic per field
DEV uint32_t ent_off(int f, int slot) { return (uint32_t)(f * PG_CAP + slot) * 4u; }
DEV float &EF(Ctx &c, int f, int slot) { return *reinterpret_cast<float *>(c.Eb + ent_off(f, slot)); }
DEV int &EI(Ctx &c, int f, int slot) { return *reinterpret_cast<int *>(c.Eb + ent_off(f, slot)); }

// A whole entity held in registers (uniform).
struct Ent {
    float x, y, vx, vy, rx, ry, rotation, vrot, alpha, alpha_decay, grow_rate, friction;
    float collision_margin, health, theta, climber_spawn_x;
    int type, image_type, image_theme, render_z, life_time, expire_time, fire_time, spawn_time, flags;
};

DEV void load_ent(Ctx &c, int i, Ent &e) {
    e.x = EF(c, F_X, i); e.y = EF(c, F_Y, i); e.vx = EF(c, F_VX, i); e.vy = EF(c, F_VY, i);
    e.rx = EF(c, F_RX, i); e.ry = EF(c, F_RY, i); e.rotation = EF(c, F_ROTATION, i); e.vrot = EF(c, F_VROT, i);
    e.alpha = EF(c, F_ALPHA, i); e.alpha_decay = EF(c, F_ALPHA_DECAY, i); e.grow_rate = EF(c, F_GROW_RATE, i);
    e.friction = EF(c, F_FRICTION, i); e.collision_margin = EF(c, F_COLLISION_MARGIN, i);
    e.health = EF(c, F_HEALTH, i); e.theta = EF(c, F_THETA, i); e.climber_spawn_x = EF(c, F_CLIMBER_SPAWN_X, i);
    e.type = EI(c, F_TYPE, i); e.image_type = EI(c, F_IMAGE_TYPE, i); e.image_theme = EI(c, F_IMAGE_THEME, i);
    e.render_z = EI(c, F_RENDER_Z, i); e.life_time = EI(c, F_LIFE_TIME, i); e.expire_time = EI(c, F_EXPIRE_TIME, i);
    e.fire_time = EI(c, F_FIRE_TIME, i); e.spawn_time = EI(c, F_SPAWN_TIME, i); e.flags = EI(c, F_FLAGS, i);
}

DEV void store_ent(Ctx &c, int i, const Ent &e) {
    EF(c, F_X, i) = e.x; EF(c, F_Y, i) = e.y; EF(c, F_VX, i) = e.vx; EF(c, F_VY, i) = e.vy;
    EF(c, F_RX, i) = e.rx; EF(c, F_RY, i) = e.ry; EF(c, F_ROTATION, i) = e.rotation; EF(c, F_VROT, i) = e.vrot;
    EF(c, F_ALPHA, i) = e.alpha; EF(c, F_ALPHA_DECAY, i) = e.alpha_decay; EF(c, F_GROW_RATE, i) = e.grow_rate;
    EF(c, F_FRICTION, i) = e.friction; EF(c, F_COLLISION_MARGIN, i) = e.collision_margin;
    EF(c, F_HEALTH, i) = e.health; EF(c, F_THETA, i) = e.theta; EF(c, F_CLIMBER_SPAWN_X, i) = e.climber_spawn_x;
    EI(c, F_TYPE, i) = e.type; EI(c, F_IMAGE_TYPE, i) = e.image_type; EI(c, F_IMAGE_THEME, i) = e.image_theme;
    EI(c, F_RENDER_Z, i) = e.render_z; EI(c, F_LIFE_TIME, i) = e.life_time; EI(c, F_EXPIRE_TIME, i) = e.expire_time;
    EI(c, F_FIRE_TIME, i) = e.fire_time; EI(c, F_SPAWN_TIME, i) = e.spawn_time; EI(c, F_FLAGS, i) = e.flags;
}

// The fields a smart step (basic_step_object + Entity::step) reads, and the ones it can change: the
// other eight (collision_margin, health, theta, climber_spawn_x, image_theme, render_z, fire_time,
// spawn_time) are neither, and the read-only ones (vrot, friction, alpha_decay, grow_rate, type,
// expire_time) are not written back.
DEV void load_ent_step(Ctx &c, int i, Ent &e) {
    e.x = EF(c, F_X, i); e.y = EF(c, F_Y, i); e.vx = EF(c, F_VX, i); e.vy = EF(c, F_VY, i);
    e.rx = EF(c, F_RX, i); e.ry = EF(c, F_RY, i); e.rotation = EF(c, F_ROTATION, i); e.vrot = EF(c, F_VROT, i);
    e.alpha = EF(c, F_ALPHA, i); e.alpha_decay = EF(c, F_ALPHA_DECAY, i); e.grow_rate = EF(c, F_GROW_RATE, i);
    e.friction = EF(c, F_FRICTION, i);
    e.type = EI(c, F_TYPE, i); e.image_type = EI(c, F_IMAGE_TYPE, i);
    e.life_time = EI(c, F_LIFE_TIME, i); e.expire_time = EI(c, F_EXPIRE_TIME, i); e.flags = EI(c, F_FLAGS, i);
}
DEV void store_ent_step(Ctx &c, int i, const Ent &e) {
    EF(c, F_X, i) = e.x; EF(c, F_Y, i) = e.y; EF(c, F_VX, i) = e.vx; EF(c, F_VY, i) = e.vy;
    EF(c, F_RX, i) = e.rx; EF(c, F_RY, i) = e.ry; EF(c, F_ROTATION, i) = e.rotation; EF(c, F_ALPHA, i) = e.alpha;
    EI(c, F_IMAGE_TYPE, i) = e.image_type; EI(c, F_LIFE_TIME, i) = e.life_time; EI(c, F_FLAGS, i) = e.flags;
}

// Entity::step (entity.cpp:57-82)
DEV void entity_step(Ent &e) {
    if (!(e.flags & EF_SMART_STEP)) {
        e.x += e.vx;
        e.y += e.vy;
    }
    e.rotation += e.vrot;
    e.vx *= e.friction;
    e.vy *= e.friction;
    e.life_time += 1;
    if (e.expire_time > 0 && e.life_time > e.expire_time) e.flags |= EF_WILL_ERASE;
    if (e.type == EXPLOSION) {
        if (e.image_type < EXPLOSION5) e.image_type++;
    }
    e.rx *= e.grow_rate;
    e.ry *= e.grow_rate;
    e.alpha = e.alpha_decay * e.alpha;
}

// Entity::step of one slot in place (lane-parallel form): reads the fields the update
// depends on and writes back only the words whose bits changed.
DEV void entity_step_slot(Ctx &c, int i, bool skip_smart = false) {
    int flags = EI(c, F_FLAGS, i);
    if (skip_smart && (flags & EF_SMART_STEP)) return; // stepped from registers by the caller
    float x = EF(c, F_X, i), y = EF(c, F_Y, i), vx = EF(c, F_VX, i), vy = EF(c, F_VY, i);
    float rx = EF(c, F_RX, i), ry = EF(c, F_RY, i), rot = EF(c, F_ROTATION, i), vrot = EF(c, F_VROT, i);
    float fr = EF(c, F_FRICTION, i), alpha = EF(c, F_ALPHA, i), decay = EF(c, F_ALPHA_DECAY, i);
    float grow = EF(c, F_GROW_RATE, i);
    int life = EI(c, F_LIFE_TIME, i), expire = EI(c, F_EXPIRE_TIME, i), type = EI(c, F_TYPE, i);
    int img = EI(c, F_IMAGE_TYPE, i);
    float nx = x, ny = y;
    if (!(flags & EF_SMART_STEP)) {
        nx = x + vx;
        ny = y + vy;
    }
    float nrot = rot + vrot;
    float nvx = vx * fr, nvy = vy * fr;
    life += 1;
    int nflags = flags;
    if (expire > 0 && life > expire) nflags |= EF_WILL_ERASE;
    int nimg = img;
    if (type == EXPLOSION && img < EXPLOSION5) nimg = img + 1;
    float nrx = rx * grow, nry = ry * grow;
    float nalpha = decay * alpha;
#define PG_SET_IF_CHANGED(F, oldv, newv) \
    if (__float_as_uint(newv) != __float_as_uint(oldv)) EF(c, F, i) = newv;
    PG_SET_IF_CHANGED(F_X, x, nx)
    PG_SET_IF_CHANGED(F_Y, y, ny)
    PG_SET_IF_CHANGED(F_ROTATION, rot, nrot)
    PG_SET_IF_CHANGED(F_VX, vx, nvx)
    PG_SET_IF_CHANGED(F_VY, vy, nvy)
    PG_SET_IF_CHANGED(F_RX, rx, nrx)
    PG_SET_IF_CHANGED(F_RY, ry, nry)
    PG_SET_IF_CHANGED(F_ALPHA, alpha, nalpha)
#undef PG_SET_IF_CHANGED
    EI(c, F_LIFE_TIME, i) = life;
    if (nflags != flags) EI(c, F_FLAGS, i) = nflags;
    if (nimg != img) EI(c, F_IMAGE_TYPE, i) = nimg;
}

// ------------------------------------------------------------------ grid queries (basic-abstract-game.cpp:167-185)
// The step reads the grid (never writes it), so the env's grid is copied once into LDS as
// int8 (every coinrun cell value is a `char` from fill_elem or a small id from set_obj;
// any value outside int8 falls back to HBM reads) and all probes hit LDS.
#define PG_G8_HOLE (-128) // an LDS grid cell that was not staged (PG_GRID_ROWS): read from HBM instead
DEV int get_obj(Ctx &c, int x, int y) {
    if (!(0 <= y && y < c.s.main_height && 0 <= x && x < c.s.main_width)) return c.s.out_of_bounds_object;
    if (!c.grid8_ok) return (int)c.G[y * c.s.main_width + x];
    const int v = c.grid8[y * c.s.main_width + x];
#ifdef PG_GRID_ROWS
    if (v == PG_G8_HOLE) return (int)c.G[y * c.s.main_width + x];
#endif
    return v;
}

// PG_GRID_ROWS: only the rows within reach of the entities that move this step are staged -- every
// smart or moving entity's rows +- 8 (push chains of stacked objects included); the other 16-cell
// chunks hold PG_G8_HOLE, which get_obj resolves from HBM (the mirror never holds -128: reset).
template <int G>
DEV uint64_t grid_rows_needed(Ctx &c) {
    const int h = c.s.main_height;
    uint64_t m = 0;
    for (int base = 0; base < c.s.num_ents; base += 64) {
        const int i = base + LANE;
        if (i >= c.s.num_ents) continue;
        const int fl = EI(c, F_FLAGS, i);
        const bool moving = i == 0 || (fl & EF_SMART_STEP) || EF(c, F_VX, i) != 0 || EF(c, F_VY, i) != 0;
        if (!moving) continue;
        const float y = EF(c, F_Y, i), ry = EF(c, F_RY, i);
        int lo = (int)floorf(y - ry) - 8, hi = (int)floorf(y + ry) + 8;
        lo = max(lo, 0);
        hi = min(hi, h - 1);
        if (lo <= hi) m |= (hi >= 63 ? ~0ull : ((2ull << hi) - 1)) & ~((1ull << lo) - 1);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m |= __shfl_xor(m, o);
    return m;
}
// The int8 mirror's chunks of the game's largest world, loaded by the kernel before the env's scalars
// arrive (they do not depend on them), lane k <-> 16-byte chunk k + 64 q.
template <int G>
struct GridPre {
    static constexpr int NCH = (pg_game_max_w(G) * pg_game_max_h(G) + 15) / 16, NQ = (NCH + 63) / 64;
    uint4 v[NQ];
    DEV void load(const int8_t *g8) {
        const uint4 *src = reinterpret_cast<const uint4 *>(g8);
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int k = LANE + 64 * q;
            v[q] = k < NCH ? src[k] : make_uint4(0, 0, 0, 0);
        }
    }
};
template <int G>
DEV void load_grid_lds(Ctx &c, const GridPre<G> &pre) {
    int cells = c.s.main_width * c.s.main_height;
    bool bad = cells > PG_GRID_MAX;
#ifndef PG_GRID_ROWS
    if (!bad && c.s.grid8_ok && (cells + 15) / 16 <= GridPre<G>::NCH) { // the prefetched mirror
#pragma unroll
        for (int q = 0; q < GridPre<G>::NQ; q++) {
            const int k = LANE + 64 * q;
            if (k < (cells + 15) / 16) reinterpret_cast<uint4 *>(c.grid8)[k] = pre.v[q];
        }
        c.grid8_ok = true;
        wave_sync();
        return;
    }
#endif
    if (!bad && c.s.grid8_ok) { // int8 mirror written by the last reset: 4 KB per env
        const uint4 *src = reinterpret_cast<const uint4 *>(c.d.grid8 + (size_t)c.env * PG_GRID_MAX);
#ifdef PG_GRID_ROWS
        if constexpr (G != PG_GAME_MINER) { // miner's cell physics reads the whole grid
            if (c.s.main_height <= 64) {
                const uint64_t rows = grid_rows_needed<G>(c);
                const int w = c.s.main_width;
                const uint4 hole = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
                for (int k = LANE; k < (cells + 15) / 16; k += 64) {
                    const int r0 = (16 * k) / w, r1 = min((16 * k + 15) / w, 63);
                    const uint64_t span = ((r1 >= 63 ? ~0ull : ((2ull << r1) - 1)) & ~((1ull << r0) - 1));
                    reinterpret_cast<uint4 *>(c.grid8)[k] = (rows & span) ? src[k] : hole;
                }
                c.grid8_ok = true;
                wave_sync();
                return;
            }
        }
#endif
        for (int k = LANE; k < (cells + 15) / 16; k += 64) reinterpret_cast<uint4 *>(c.grid8)[k] = src[k];
        c.grid8_ok = true;
        wave_sync();
        return;
    }
    if (!bad) {
        const uint4 *src = reinterpret_cast<const uint4 *>(c.G); // 8 int16 cells per 16 B
        for (int k = LANE; k < (cells + 7) / 8; k += 64) {
            uint4 v = src[k];
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
            uint32_t packed[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                uint32_t p = 0;
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    uint32_t word = w[h * 2 + q];
                    int lo = (int16_t)(word & 0xffff), hi = (int16_t)(word >> 16);
                    if (lo < -127 || lo > 127 || hi < -127 || hi > 127) bad = true; // -128: PG_G8_HOLE
                    p |= ((uint32_t)(uint8_t)lo | ((uint32_t)(uint8_t)hi << 8)) << (16 * q);
                }
                packed[h] = p;
            }
            reinterpret_cast<uint2 *>(c.grid8)[k] = make_uint2(packed[0], packed[1]);
        }
    }
    c.grid8_ok = ballot(bad) == 0;
    wave_sync();
}
DEV int get_obj_from_floats(Ctx &c, float i, float j) {
    if (i < 0) return c.s.out_of_bounds_object;
    if (j < 0) return c.s.out_of_bounds_object;
    return get_obj(c, (int)floorf(i), (int)floorf(j));
}
// get_obj_from_floats of a per-lane point (every lane its own probe): branch-free, one LDS read for all
// lanes -- sub_step's four corner probes in one round trip instead of four dependent ones
DEV int get_obj_from_floats_lane(Ctx &c, float i, float j) {
    const int x = (int)floorf(i), y = (int)floorf(j);
    const bool out = i < 0 || j < 0 || !(0 <= y && y < c.s.main_height && 0 <= x && x < c.s.main_width);
    const int idx = out ? 0 : y * c.s.main_width + x;
    int v;
    if (c.grid8_ok) {
        v = c.grid8[idx];
#ifdef PG_GRID_ROWS
        if (v == PG_G8_HOLE) v = (int)c.G[idx];
#endif
    } else {
        v = (int)c.G[idx];
    }
    return out ? c.s.out_of_bounds_object : v;
}

// ------------------------------------------------------------------ per-game hooks
template <int G>
DEV bool is_blocked(Ctx &c, int src_type, int target) { // basic :494-501 + coinrun.cpp:204-211
    if (target == WALL_OBJ) return true;
    if (target == c.s.out_of_bounds_object) return true;
    if constexpr (G == PG_GAME_COINRUN)
        if (src_type == PLAYER && cr_is_wall(target)) return true;
    if constexpr (G == PG_GAME_CLIMBER) // climber.cpp:147-154
        if (src_type == PLAYER && cl_is_wall(target)) return true;
    if constexpr (G == PG_GAME_JUMPER) // jumper.cpp:117-124
        if (src_type == PLAYER && jp_is_wall(target)) return true;
    if constexpr (G == PG_GAME_CHASER) // chaser.cpp:94-99
        if (target == CH_MAZE_WALL) return true;
    if constexpr (G == PG_GAME_FRUITBOT) // fruitbot.cpp:83-85
        if (src_type == PLAYER && target == FB_OUT_OF_BOUNDS_WALL) return true;
    if constexpr (G == PG_GAME_MINER) // miner.cpp:68-75
        if (src_type == PLAYER && (target == MN_BOULDER || target == MN_MOVING_BOULDER || target == MN_OOB_WALL))
            return true;
    return false;
}
template <int G>
DEV bool will_reflect(int src, int target) { // coinrun.cpp:140-142; base :507-509 false
    if constexpr (G == PG_GAME_COINRUN) return src == CR_ENEMY && (cr_is_wall(target) || target == CR_ENEMY_BARRIER);
    if constexpr (G == PG_GAME_CLIMBER) // climber.cpp:113-115
        return src == CL_ENEMY && (cl_is_wall(target) || target == CL_ENEMY_BARRIER);
    if constexpr (G == PG_GAME_FRUITBOT) // fruitbot.cpp:79-81
        return src == FB_BAD_OBJ && (target == FB_BARRIER || target == WALL_OBJ);
    if constexpr (G == PG_GAME_CAVEFLYER) // caveflyer.cpp:120-122 (out_of_bounds_object = CAVEWALL)
        return src == CF_ENEMY && target == CF_CAVEWALL;
    if constexpr (G == PG_GAME_DODGEBALL) // dodgeball.cpp:98-100 (out_of_bounds_object = OOB_WALL)
        return src == DB_ENEMY && (target == DB_LAVA_WALL || target == DB_OOB_WALL);
    if constexpr (G == PG_GAME_MINER) // miner.cpp:77-79 (out_of_bounds_object = OOB_WALL)
        return src == MN_ENEMY && (target == MN_BOULDER || target == MN_DIAMOND || target == MN_MOVING_BOULDER ||
                                   target == MN_MOVING_DIAMOND || target == MN_OOB_WALL);
    return false;
}

// The scanned entity m of sub_step's loop: its index and the fields the loop body reads.  Interactors
// are static during step_entities (see build_interactor_list), so these come from the lane that
// caches m (ireg) or one set of loads -- never re-read per use inside the push chain.
struct IView {
    int m;
    float x, y, rx, ry;
    int theme;
};

// is_blocked_ents (basic :503-505; coinrun.cpp:187-202; heist.cpp:66-71).  The agent's vy / ry are
// the stepped object's own when it is the agent (slot 0), else the agent's pre-step state (c.av_*).
template <int G>
DEV bool is_blocked_ents(Ctx &c, int src_type, const IView &m, int t_type, bool is_h, int oi, const Ent &o) {
    if constexpr (G == PG_GAME_COINRUN) {
        if (t_type == CR_CRATE && !is_h) {
            const float avy = oi == 0 ? o.vy : c.av_vy, ary = oi == 0 ? o.ry : c.av_ry;
            if (avy >= 0) return false;
            if (c.s.action_vy < 0) return false;
            if (c.s.last_agent_y < (m.y + m.ry + ary)) return false;
            c.s.is_on_crate = 1;
            return true;
        }
    }
    if constexpr (G == PG_GAME_HEIST) {
        if (t_type == HS_LOCKED_DOOR) return !((c.s.has_keys >> m.theme) & 1);
    }
    return is_blocked<G>(c, src_type, t_type);
}

// ------------------------------------------------------------------ collision scan
// The body of sub_step's entity loop (basic-abstract-game.cpp:345-377) has an effect only
// when is_blocked_ents() or will_reflect() fires.  Per game that reduces to a few entity
// types ("interactors"): coinrun -- a CRATE on a vertical move (coinrun.cpp:187-211; base
// is_blocked needs WALL_OBJ / out_of_bounds_object / a wall type, will_reflect a wall or
// ENEMY_BARRIER type, and no coinrun entity has such a type); heist -- LOCKED_DOOR
// (heist.cpp:66-71); bigfish and maze -- none (no entity type is WALL_OBJ or the
// out-of-bounds object).  Every other (obj, m) pair is a no-op, so the scan visits only the
// interactors, collected once per step into LDS; entity indices do not change during
// step_entities (no insertion or erase there).
// dodgeball: LAVA_WALL reflects ENEMY (dodgeball.cpp:98-100); no entity type blocks.
template <int G>
DEV constexpr bool scan_needed(bool is_h) {
    if constexpr (G == PG_GAME_COINRUN) return !is_h;
    if constexpr (G == PG_GAME_HEIST) return true;
    if constexpr (G == PG_GAME_DODGEBALL) return true;
    return false;
}
// the one entity type that interacts in each scanning game (-1: none)
template <int G>
DEV constexpr int interactor_type() {
    if constexpr (G == PG_GAME_COINRUN) return CR_CRATE;
    if constexpr (G == PG_GAME_HEIST) return HS_LOCKED_DOOR;
    if constexpr (G == PG_GAME_DODGEBALL) return DB_LAVA_WALL;
    return -1;
}
template <int G>
DEV bool is_interactor(int type) { return interactor_type<G>() >= 0 && type == interactor_type<G>(); }
// games whose scan can only reflect the stepped object (no is_blocked_ents, hence no push chain)
template <int G>
DEV constexpr bool scan_reflects_only() { return G == PG_GAME_DODGEBALL; }

// Largest interactor index i < upper (i != oi, !will_erase) with has_collision(obj, e_i, POS_EPS),
// i.e. the next entity the reference's reverse loop would act on; lane-parallel over the list.
DEV float rlf(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
DEV int rli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

DEV void iview_load(Ctx &c, int m, IView &v) {
    v.m = m;
    v.x = EF(c, F_X, m); v.y = EF(c, F_Y, m); v.rx = EF(c, F_RX, m); v.ry = EF(c, F_RY, m);
    v.theme = EI(c, F_IMAGE_THEME, m);
}

// Fills `v` and returns true when there is a next collider.
DEV bool next_collider(Ctx &c, int oi, int upper, const Ent &o, IView &v) {
    if (c.ireg) { // <= 64 static interactors: lane k holds interactor k in registers
        int i = LANE < c.nlist ? c.i_idx : PG_CAP;
        bool hit = false;
        if (i < upper && i != oi && !c.i_erase) {
            float tx = (o.rx + c.i_rx) + POS_EPS;
            float ty = (o.ry + c.i_ry) + POS_EPS;
            hit = (fabsf(o.x - c.i_x) < tx) && (fabsf(o.y - c.i_y) < ty);
        }
        unsigned long long m = ballot(hit);
        if (!m) return false;
        const int l = top_bit(m);
        v.m = rli(i, l);
        v.x = rlf(c.i_x, l); v.y = rlf(c.i_y, l); v.rx = rlf(c.i_rx, l); v.ry = rlf(c.i_ry, l);
        v.theme = rli(c.i_theme, l);
        return true;
    }
    for (int base = (c.nlist - 1) & ~63; base >= 0; base -= 64) {
        int k = base + LANE;
        bool hit = false;
        int i = k < c.nlist ? c.ilist[k] : PG_CAP;
        if (i < upper && i != oi) {
            int fl = EI(c, F_FLAGS, i);
            if (!(fl & EF_WILL_ERASE)) {
                float tx = (o.rx + EF(c, F_RX, i)) + POS_EPS;
                float ty = (o.ry + EF(c, F_RY, i)) + POS_EPS;
                hit = (fabsf(o.x - EF(c, F_X, i)) < tx) && (fabsf(o.y - EF(c, F_Y, i)) < ty);
            }
        }
        unsigned long long m = ballot(hit);
        if (m) { // list is ascending by index
            iview_load(c, rli(i, top_bit(m)), v);
            return true;
        }
    }
    return false;
}

// Games whose smart entities step lane-parallel (step_entities_fast; measured per game,
// profiles/r02: a win where several smart entities take many sub-steps, a 2x loss for coinrun)
template <int G>
DEV constexpr bool pl_smart() {
#ifdef PG_PL_ALL
    return true;
#else
    return G == PG_GAME_CHASER || G == PG_GAME_CLIMBER || G == PG_GAME_NINJA || G == PG_GAME_CAVEFLYER ||
           G == PG_GAME_DODGEBALL;
#endif
}

// next_collider for a lane stepping its own entity (lane-parallel smart steps): the static
// interactors are read from LDS, the ascending list's last hit is the largest index.
DEV bool next_collider_pl(Ctx &c, int oi, int upper, const Ent &o, IView &v) {
    int best = -1;
    for (int k = 0; k < c.nlist; k++) {
        const int inf = c.iinfo[k];
        const int i = inf & 0x7fffffff;
        if (inf < 0 || i >= upper || i == oi) continue;
        const float4 b = c.ibox[k];
        float tx = (o.rx + b.z) + POS_EPS;
        float ty = (o.ry + b.w) + POS_EPS;
        if ((fabsf(o.x - b.x) < tx) && (fabsf(o.y - b.y) < ty)) best = i;
    }
    if (best < 0) return false;
    iview_load(c, best, v);
    return true;
}

template <int G>
DEV void build_interactor_list(Ctx &c) {
    int cnt = 0;
    c.nlist = 0;
    c.ireg = true;
    if (!scan_needed<G>(false) && !scan_needed<G>(true)) return;
    for (int base = 0; base < c.s.num_ents; base += 64) {
        int i = base + LANE;
        bool in = i < c.s.num_ents && is_interactor<G>(EI(c, F_TYPE, i));
        unsigned long long m = ballot(in);
        if (in) c.ilist[cnt + __popcll(m & ((1ull << LANE) - 1ull))] = (int16_t)i;
        cnt += __popcll(m);
    }
    c.nlist = cnt;
    wave_sync();
    // Interactors whose Entity::step cannot change x, y, rx, ry or will_erase during this
    // step (not smart, zero velocity, grow_rate 1, no expiry -- coinrun's crates) are held
    // in registers for the whole step: lane k <-> interactor k.
    c.ireg = false;
    if (cnt <= 64) {
        bool stat = true;
        if (LANE < cnt) {
            int i = c.ilist[LANE];
            c.i_idx = i;
            c.i_x = EF(c, F_X, i); c.i_y = EF(c, F_Y, i); c.i_rx = EF(c, F_RX, i); c.i_ry = EF(c, F_RY, i);
            int fl = EI(c, F_FLAGS, i);
            c.i_erase = (fl & EF_WILL_ERASE) != 0;
            c.i_theme = EI(c, F_IMAGE_THEME, i);
            stat = !(fl & EF_SMART_STEP) && EF(c, F_VX, i) == 0 && EF(c, F_VY, i) == 0 &&
                   EF(c, F_GROW_RATE, i) == 1 && EI(c, F_EXPIRE_TIME, i) <= 0;
        }
        c.ireg = ballot(!stat) == 0;
        if constexpr (pl_smart<G>()) {
            if (LANE < cnt) {
                c.ibox[LANE] = make_float4(c.i_x, c.i_y, c.i_rx, c.i_ry);
                c.iinfo[LANE] = c.i_idx | (c.i_erase ? (int)0x80000000u : 0);
            }
            wave_sync();
        }
    }
}

DEV double dsign(double x) { return x > 0 ? +1 : (x == 0 ? 0 : -1); }

// push_obj's target offset (basic-abstract-game.cpp:248-270; the target is always the stepped object)
DEV void push_offset(const IView &src, const Ent &o, bool is_h, float &t_vx, float &t_vy) {
    float sx = src.x, sy = src.y;
    float rsum = is_h ? (src.rx + o.rx) : (src.ry + o.ry);
    float delx = o.x - sx;
    float dely = o.y - sy;
    t_vx = 0;
    t_vy = 0;
    if (is_h) t_vx = (float)((double)sx + dsign(delx) * (double)rsum - (double)o.x);
    else t_vy = (float)((double)sy + dsign(dely) * (double)rsum - (double)o.y);
}

// Push-chain memo.  Within one basic_step_object call a nested sub_step (a push's child) is a pure
// function of (depth, the object's x, y, vx, vy, the move): the grid, the static interactors (the
// scan needs them register-cached: ireg), the agent state its crate rule reads, last_agent_y and
// action_vy do not change, and its only other effect, coinrun's is_on_crate = 1, is monotone over
// the call.  Overlapping interactors (coinrun's stacked duplicate crates: a push of 0 leaves the
// object where it was) make the reference's recursion revisit the same child up to 2^5 times;
// the memo replays a child's outcome instead of walking it again (coinrun's 280-sub_step crate
// piles fall to ~50).  Entry k (12 words): key {depth, x, y, vx, vy, move x, move y}, value
// {x, y, vx, vy, is_on_crate after}; lane k holds entry k's lookup.
constexpr int PG_MEMO_CAP = 48;
constexpr int PG_MEMO_W = 12;
static_assert(PG_MEMO_CAP * PG_MEMO_W <= PG_MT_N, "the memo lives in the twist staging words");

// the entry whose key matches, or -1
DEV int memo_find(Ctx &c, int depth, const Ent &o, float mvx, float mvy) {
    bool hit = false;
    if (LANE < c.nmemo) {
        const uint4 k0 = *reinterpret_cast<const uint4 *>(c.memo + LANE * PG_MEMO_W);
        const uint4 k1 = *reinterpret_cast<const uint4 *>(c.memo + LANE * PG_MEMO_W + 4);
        hit = k0.x == (uint32_t)depth && k0.y == __float_as_uint(o.x) && k0.z == __float_as_uint(o.y) &&
              k0.w == __float_as_uint(o.vx) && k1.x == __float_as_uint(o.vy) && k1.y == __float_as_uint(mvx) &&
              k1.z == __float_as_uint(mvy);
    }
    const unsigned long long m = ballot(hit);
    return m ? (int)__builtin_ctzll(m) : -1;
}

// basic-abstract-game.cpp:278-380 with push_obj (:247-276) folded in.  The reference recurses
// sub_step -> push_obj -> sub_step(depth + 1) while depth < 5; here the recursion is an explicit
// stack of at most 5 suspended frames (each: its move, the scan position, block || block2 so far),
// so the body exists once in the kernel instead of once per depth per call site (a 6-deep inlined
// chain per call site made the coinrun kernel 177 KB, far past the instruction cache).
// A child's return value is ignored by push_obj; after it returns the parent zeroes the pushed
// velocity component and resumes its reverse entity loop.
// PL: every lane steps its own entity (no cross-lane operation).
template <int G, bool PL>
DEV bool sub_step(Ctx &c, int oi, Ent &o, float _vx, float _vy) {
#ifdef PG_PROF_SMART
    c.sm[1] += 1;
#endif
    // the frame stack is wave-uniform LDS: the lane-parallel (PL) games never push -- they do not scan, or
    // (dodgeball) their scan only reflects: its one interactor type, LAVA_WALL, is neither WALL_OBJ nor the
    // out-of-bounds object, so is_blocked_ents never fires (dodgeball.cpp:98-100)
    static_assert(!PL || (!scan_needed<G>(true) && !scan_needed<G>(false)) || scan_reflects_only<G>(),
                  "PL games have no push chain");
    constexpr int MAXD = 5;
    int d = 0;
    bool fresh = true, acc = false;
    int upper = 0;
    for (;;) {
        bool is_h = _vx != 0;
        if (fresh) {
            if (o.flags & EF_WILL_ERASE) {
                acc = false;
                upper = -1; // return false without scanning
            } else {
                float ny = o.y + _vy;
                float nx = o.x + _vx;
                const float margin = 0.98f;
                bool block = false, reflect = false;
                if constexpr (!PL) {
                    // the four corner probes of the reference's (i, j) loop, lane q <-> corner (q >> 1, q & 1)
                    // (lanes >= 4 repeat them); the loop only ORs its predicates, and ninja's star stop zeroes
                    // a velocity the probes do not read, so the corners may be probed together
                    const int i = (LANE >> 1) & 1, j = LANE & 1;
                    const int type2 = get_obj_from_floats_lane(c, nx + o.rx * margin * (float)(2 * i - 1),
                                                               ny + o.ry * margin * (float)(2 * j - 1));
                    if constexpr (G == PG_GAME_NINJA) // ninja.cpp:132-138: a star that meets a wall stops
                        if (ballot(o.type == NJ_THROWING_STAR && type2 == NJ_WALL_MID)) { o.vx = 0; o.vy = 0; }
                    block = ballot(is_blocked<G>(c, o.type, type2)) != 0;
                    reflect = ballot(will_reflect<G>(o.type, type2)) != 0;
                } else {
#pragma unroll
                    for (int i = 0; i < 2; i++) {
#pragma unroll
                        for (int j = 0; j < 2; j++) {
                            int type2 = get_obj_from_floats(c, nx + o.rx * margin * (float)(2 * i - 1), ny + o.ry * margin * (float)(2 * j - 1));
                            if constexpr (G == PG_GAME_NINJA) // ninja.cpp:132-138: a star that meets a wall stops
                                if (o.type == NJ_THROWING_STAR && type2 == NJ_WALL_MID) { o.vx = 0; o.vy = 0; }
                            block = block || is_blocked<G>(c, o.type, type2);
                            reflect = reflect || will_reflect<G>(o.type, type2);
                        }
                    }
                }
                if (reflect) {
                    if (is_h) {
                        float delta;
                        if (_vx < 0) delta = ceilf(nx - o.rx) - (nx - o.rx);
                        else delta = floorf(nx + o.rx) - (nx + o.rx);
                        o.vx = -1 * o.vx;
                        nx = nx + 2 * delta;
                    } else {
                        float delta;
                        if (_vy < 0) delta = ceilf(ny - o.ry) - (ny - o.ry);
                        else delta = floorf(ny + o.ry) - (ny + o.ry);
                        o.vy = -1 * o.vy;
                        ny = ny + 2 * delta;
                    }
                } else if (block) {
                    if (is_h) {
                        if (c.s.grid_step) nx = o.x;
                        else nx = _vx > 0 ? (floorf(nx + o.rx) - o.rx) : (ceilf(nx - o.rx) + o.rx);
                    } else {
                        if (c.s.grid_step) ny = o.y;
                        else ny = _vy > 0 ? (floorf(ny + o.ry) - o.ry) : (ceilf(ny - o.ry) + o.ry);
                    }
                }
                o.x = nx;
                o.y = ny;
                acc = block;
                upper = c.s.num_ents;
            }
        } else {
            // a child frame returned: the rest of push_obj (:271-275)
            if (is_h) o.vx = 0;
            else o.vy = 0;
        }
        fresh = false;
        while (upper >= 0 && scan_needed<G>(is_h)) {
            IView m;
            if (!(PL ? next_collider_pl(c, oi, upper, o, m) : next_collider(c, oi, upper, o, m))) break;
            upper = m.m;
            constexpr int mtype = interactor_type<G>(); // the scan lists hold only this type
            if (!PL && is_blocked_ents<G>(c, o.type, m, mtype, is_h, oi, o)) {
                acc = true; // block2 = block2 || curr_block
                float t_vx, t_vy;
                push_offset(m, o, is_h, t_vx, t_vy);
                if (d < MAXD) { // run sub_step(t_vx, t_vy, depth + 1)
                    const int hitk = memo_find(c, d + 1, o, t_vx, t_vy);
#ifdef PG_PROF_SMART
                    c.sm[4] += hitk >= 0 ? 1 : 0;
#endif
                    if (hitk >= 0) { // replay the child's outcome; push_obj then zeroes the pushed velocity
                        const uint32_t *v = c.memo + hitk * PG_MEMO_W + 7;
                        o.x = __uint_as_float(v[0]); o.y = __uint_as_float(v[1]);
                        o.vx = __uint_as_float(v[2]); o.vy = __uint_as_float(v[3]);
                        if constexpr (G == PG_GAME_COINRUN) c.s.is_on_crate |= (int)v[4];
                        if (is_h) o.vx = 0;
                        else o.vy = 0;
                        continue;
                    }
                    // suspend this frame: its move, scan position and block so far, plus the child's key
                    float *f = c.pstk + 10 * d;
                    f[0] = _vx; f[1] = _vy; f[2] = __int_as_float(upper); f[3] = acc ? 1.f : 0.f;
                    f[4] = o.x; f[5] = o.y; f[6] = o.vx; f[7] = o.vy; f[8] = t_vx; f[9] = t_vy;
                    d++;
                    _vx = t_vx;
                    _vy = t_vy;
                    fresh = true;
                    break;
                }
                if (is_h) o.vx = 0;
                else o.vy = 0;
            } else if (will_reflect<G>(o.type, mtype)) {
                if (is_h) {
                    float delx = m.x - o.x;
                    float rsum = m.rx + o.rx;
                    o.x += _vx > 0 ? -2 * (rsum - delx) : 2 * (rsum + delx);
                    o.vx = -1 * o.vx;
                } else {
                    float dely = m.y - o.y;
                    float rsum = m.ry + o.ry;
                    o.y += _vy > 0 ? -2 * (rsum - dely) : 2 * (rsum + dely);
                    o.vy = -1 * o.vy;
                }
            }
        }
        if (fresh) continue;
        if (d == 0) return acc;
        d--;
        const float *f = c.pstk + 10 * d;
        if (c.nmemo < PG_MEMO_CAP) { // record the finished child (depth d + 1)
            uint32_t *e = c.memo + c.nmemo * PG_MEMO_W;
            if (LANE < PG_MEMO_W) {
                uint32_t w;
                switch (LANE) {
                case 0: w = (uint32_t)(d + 1); break;
                case 7: w = __float_as_uint(o.x); break;
                case 8: w = __float_as_uint(o.y); break;
                case 9: w = __float_as_uint(o.vx); break;
                case 10: w = __float_as_uint(o.vy); break;
                case 11: w = (uint32_t)c.s.is_on_crate; break;
                default: w = __float_as_uint(f[3 + LANE]); break; // the key saved at suspension
                }
                e[LANE] = w;
            }
            c.nmemo++;
            wave_sync();
        }
        _vx = f[0]; _vy = f[1]; upper = __float_as_int(f[2]); acc = f[3] != 0.f;
    }
}

// basic-abstract-game.cpp:602-665
template <int G, bool PL = false>
DEV void basic_step_object(Ctx &c, int oi, Ent &o) {
    if (o.flags & EF_WILL_ERASE) return;
    c.nmemo = 0; // the memo holds this call's push children only
    if constexpr (G == PG_GAME_COINRUN) {
        // the agent as this object's crate checks see it: slot 0 is written only by its own step
        if (oi != 0) { c.av_vy = EF(c, F_VY, 0); c.av_ry = EF(c, F_RY, 0); }
    }
    int num_sub_steps;
    if (c.s.grid_step) {
        num_sub_steps = 1;
    } else {
        num_sub_steps = (int)(4 * sqrt((double)(o.vx * o.vx + o.vy * o.vy)));
        if (num_sub_steps < 4) num_sub_steps = 4;
    }
    float pct = (float)(1.0 / num_sub_steps);
    float cmp = fabsf(o.vx) - fabsf(o.vy);
    bool step_x_first = cmp == 0 ? c.s.step_rand_int % 2 == 0 : (cmp > 0);
    if (o.type == PLAYER) {
        if (c.s.action_vx != 0) step_x_first = true;
        if (c.s.action_vy != 0) step_x_first = false;
    }
    float vx_pct = 0, vy_pct = 0;
    for (int s = 0; s < num_sub_steps; s++) {
        // one sub_step call site for both half steps (the second reads the velocity the first
        // may have changed)
        bool block_x = false, block_y = false;
#pragma unroll 1
        for (int h = 0; h < 2; h++) {
            const bool xmove = (h == 0) == step_x_first;
            const bool b = sub_step<G, PL>(c, oi, o, xmove ? o.vx * pct : 0, xmove ? 0 : o.vy * pct);
            if (xmove) block_x = b;
            else block_y = b;
        }
        if (!block_x) vx_pct += 1;
        if (!block_y) vy_pct += 1;
        if (block_x && block_y) break;
    }
    vx_pct = vx_pct / (float)num_sub_steps;
    vy_pct = vy_pct / (float)num_sub_steps;
    o.vx *= vx_pct;
    o.vy *= vy_pct;
}

// basic-abstract-game.cpp:1095-1107: reverse order; runs of non-smart entities are
// independent (Entity::step touches only its own entity) and are stepped lane-parallel
// with slot i always owned by lane i % 64.
DEV void ent_readlane(const Ent &m, int l, Ent &o) {
    o.x = rlf(m.x, l); o.y = rlf(m.y, l); o.vx = rlf(m.vx, l); o.vy = rlf(m.vy, l);
    o.rx = rlf(m.rx, l); o.ry = rlf(m.ry, l); o.rotation = rlf(m.rotation, l); o.vrot = rlf(m.vrot, l);
    o.alpha = rlf(m.alpha, l); o.alpha_decay = rlf(m.alpha_decay, l); o.grow_rate = rlf(m.grow_rate, l);
    o.friction = rlf(m.friction, l); o.collision_margin = rlf(m.collision_margin, l);
    o.health = rlf(m.health, l); o.theta = rlf(m.theta, l); o.climber_spawn_x = rlf(m.climber_spawn_x, l);
    o.type = rli(m.type, l); o.image_type = rli(m.image_type, l); o.image_theme = rli(m.image_theme, l);
    o.render_z = rli(m.render_z, l); o.life_time = rli(m.life_time, l); o.expire_time = rli(m.expire_time, l);
    o.fire_time = rli(m.fire_time, l); o.spawn_time = rli(m.spawn_time, l); o.flags = rli(m.flags, l);
}

// Fast path of step_entities.  Within step_entities an entity's fields are written only
// by its own basic_step_object / Entity::step (push_obj moves the stepped object itself,
// the scans read only the register-cached static interactors), so every smart entity can
// be loaded lane-parallel up front (lane k <-> k-th smart entity), stepped from registers
// in the reference's reverse order, and stored lane-parallel at the end.

// The smart entities' steps of step_entities_fast / step_entities_regs from registers (lane k <->
// smart entity k, index my_i), stored back lane-parallel.
template <int G>
DEV void smart_steps(Ctx &c, Ent &mine, int my_i, int nsm) {
    // The smart entities' steps are independent of each other as well: a smart step writes only
    // its own entity and reads the grid, the static interactors and the agent (slot 0, stepped
    // last by the reverse loop, so every other smart step sees its pre-step state, which is what
    // HBM holds until the store below).  All but the agent step at once, lane k <-> smart entity k;
    // the one shared write, coinrun's is_on_crate = 1 (is_blocked_ents), is OR-ed back.
    // Measured per game (profiles/r02): a win where several smart entities take many sub-steps
    // (chaser, climber, ninja, caveflyer); coinrun's step ran 2x slower this way, so the others
    // keep the in-order loop.
    if constexpr (pl_smart<G>()) {
        if (LANE < nsm && my_i != 0) {
            basic_step_object<G, true>(c, my_i, mine);
            entity_step(mine);
        }
        if constexpr (G == PG_GAME_COINRUN) c.s.is_on_crate = ballot(c.s.is_on_crate != 0) ? 1 : 0;
    } else {
        const int jlo = (nsm > 0 && rli(my_i, 0) == 0) ? 1 : 0; // the agent goes last, below
#ifdef PG_PROF_SMART
        uint64_t t_sm = __builtin_amdgcn_s_memtime();
#endif
        for (int j = nsm - 1; j >= jlo; j--) {
            Ent o;
            ent_readlane(mine, j, o);
            basic_step_object<G>(c, rli(my_i, j), o);
            entity_step(o);
            if (LANE == j) mine = o;
        }
#ifdef PG_PROF_SMART
        c.sm[3] += __builtin_amdgcn_s_memtime() - t_sm;
#endif
    }
#ifdef PG_PROF_SMART
    c.sm[0] += nsm;
    uint64_t t_ag = __builtin_amdgcn_s_memtime();
#endif
    if (nsm > 0 && rli(my_i, 0) == 0) { // slist is ascending: the agent is smart entity 0
        Ent o;
        ent_readlane(mine, 0, o);
        basic_step_object<G>(c, 0, o);
        entity_step(o);
        if (LANE == 0) mine = o;
    }
#ifdef PG_PROF_SMART
    c.sm[2] += __builtin_amdgcn_s_memtime() - t_ag;
#endif
    if (LANE < nsm) store_ent_step(c, my_i, mine);
    wave_sync();
}

template <int G>
DEV bool step_entities_fast(Ctx &c, int16_t *slist) {
    int n = c.s.num_ents;
    int nsm = 0;
    for (int base = 0; base < n; base += 64) {
        int i = base + LANE;
        bool smart = i < n && (EI(c, F_FLAGS, i) & EF_SMART_STEP);
        unsigned long long m = ballot(smart);
        int pos = nsm + __popcll(m & ((1ull << LANE) - 1ull));
        if (smart && pos < 64) slist[pos] = (int16_t)i;
        nsm += __popcll(m);
    }
    if (nsm > 64 || !c.ireg) return false;
    wave_sync();
    Ent mine;
    int my_i = LANE < nsm ? slist[LANE] : 0;
    if (LANE < nsm) load_ent_step(c, my_i, mine);
    // The non-smart entities' Entity::step touches only their own slots and no smart step reads
    // them (the only entities a smart step reads are the static interactors, whose Entity::step
    // leaves x, y, rx, ry and will_erase as they are, and the agent, itself smart), so they are
    // stepped in one lane-parallel pass -- one round of loads for the whole list instead of one
    // per run between two smart entities of the reverse loop.
    for (int base = 0; base < n; base += 64) {
        int i = base + LANE;
        if (i < n) entity_step_slot(c, i, true);
    }
    c.pt.mark(7); // diagnostic build: interactor list + smart loads + the non-smart pass
    c.cs.mark(3);
    smart_steps<G>(c, mine, my_i, nsm);
    return true;
}

// Lane permutation: lane i's value goes to lane dst (ds_permute_b32; every lane sends to a distinct lane).
DEV int perm_i(int dst, int v) { return __builtin_amdgcn_ds_permute(dst * 4, v); }
DEV float perm_f(int dst, float v) { return __int_as_float(__builtin_amdgcn_ds_permute(dst * 4, __float_as_int(v))); }

// build_interactor_list + step_entities for a list of at most 64 entities from ONE round of loads: lane i
// loads entity i's step fields, and the interactor registers and the smart entities' registers are
// compacted from them by lane permutes (ballot ranks) instead of an LDS list and a second and third
// round of loads; the non-smart entities are stepped from the same registers.  The order of effects is
// step_entities_fast's (see there).  Returns false (nothing done) for longer lists or when the
// interactors are not static (the LDS-list paths then run).
template <int G>
DEV bool step_entities_regs(Ctx &c) {
    const int n = c.s.num_ents;
    if (n > 64) return false;
    const bool have = LANE < n;
    Ent e;
    int theme = 0;
    if (have) {
        load_ent_step(c, LANE, e);
        if constexpr (scan_needed<G>(false) || scan_needed<G>(true)) theme = EI(c, F_IMAGE_THEME, LANE);
    } else {
        e.type = -1;
        e.flags = 0;
    }
    const unsigned long long below = (1ull << LANE) - 1ull;
    // ---- interactors (build_interactor_list): lane k <-> the k-th interactor, ascending index
    c.nlist = 0;
    c.ireg = true;
    if constexpr (scan_needed<G>(false) || scan_needed<G>(true)) {
        const bool in = have && is_interactor<G>(e.type);
        const unsigned long long mi = ballot(in);
        const int cnt = __popcll(mi);
        const int dst = in ? __popcll(mi & below) : cnt + __popcll(~mi & below);
        const bool stat = !(e.flags & EF_SMART_STEP) && e.vx == 0 && e.vy == 0 && e.grow_rate == 1 && e.expire_time <= 0;
        if (ballot(in && !stat)) return false;
        c.nlist = cnt;
        c.i_idx = perm_i(dst, LANE);
        c.i_x = perm_f(dst, e.x); c.i_y = perm_f(dst, e.y); c.i_rx = perm_f(dst, e.rx); c.i_ry = perm_f(dst, e.ry);
        c.i_erase = perm_i(dst, e.flags & EF_WILL_ERASE) != 0;
        c.i_theme = perm_i(dst, theme);
        if constexpr (pl_smart<G>()) {
            if (LANE < cnt) {
                c.ibox[LANE] = make_float4(c.i_x, c.i_y, c.i_rx, c.i_ry);
                c.iinfo[LANE] = c.i_idx | (c.i_erase ? (int)0x80000000u : 0);
            }
            wave_sync();
        }
    }
    // ---- smart entities: lane k <-> the k-th smart entity, ascending index
    const bool smart = have && (e.flags & EF_SMART_STEP);
    const unsigned long long ms = ballot(smart);
    const int nsm = __popcll(ms);
    const int sdst = smart ? __popcll(ms & below) : nsm + __popcll(~ms & below);
    Ent mine;
    const int my_i = perm_i(sdst, LANE);
    mine.x = perm_f(sdst, e.x); mine.y = perm_f(sdst, e.y); mine.vx = perm_f(sdst, e.vx); mine.vy = perm_f(sdst, e.vy);
    mine.rx = perm_f(sdst, e.rx); mine.ry = perm_f(sdst, e.ry); mine.rotation = perm_f(sdst, e.rotation);
    mine.vrot = perm_f(sdst, e.vrot); mine.alpha = perm_f(sdst, e.alpha); mine.alpha_decay = perm_f(sdst, e.alpha_decay);
    mine.grow_rate = perm_f(sdst, e.grow_rate); mine.friction = perm_f(sdst, e.friction);
    mine.type = perm_i(sdst, e.type); mine.image_type = perm_i(sdst, e.image_type);
    mine.life_time = perm_i(sdst, e.life_time); mine.expire_time = perm_i(sdst, e.expire_time);
    mine.flags = perm_i(sdst, e.flags);
    // ---- the non-smart entities' Entity::step from the registers (entity_step_slot: changed words only)
    if (have && !smart) {
        Ent o = e;
        entity_step(o);
#define PG_SET_IF_CHANGED(F, f) \
    if (__float_as_uint(o.f) != __float_as_uint(e.f)) EF(c, F, LANE) = o.f;
        PG_SET_IF_CHANGED(F_X, x)
        PG_SET_IF_CHANGED(F_Y, y)
        PG_SET_IF_CHANGED(F_ROTATION, rotation)
        PG_SET_IF_CHANGED(F_VX, vx)
        PG_SET_IF_CHANGED(F_VY, vy)
        PG_SET_IF_CHANGED(F_RX, rx)
        PG_SET_IF_CHANGED(F_RY, ry)
        PG_SET_IF_CHANGED(F_ALPHA, alpha)
#undef PG_SET_IF_CHANGED
        EI(c, F_LIFE_TIME, LANE) = o.life_time;
        if (o.flags != e.flags) EI(c, F_FLAGS, LANE) = o.flags;
        if (o.image_type != e.image_type) EI(c, F_IMAGE_TYPE, LANE) = o.image_type;
    }
    c.pt.mark(7); // diagnostic build: interactor list + smart loads + the non-smart pass
    c.cs.mark(3);
    smart_steps<G>(c, mine, my_i, nsm);
    return true;
}

template <int G>
DEV void step_entities(Ctx &c, int16_t *slist) {
    if (step_entities_fast<G>(c, slist)) return;
    int hi = c.s.num_ents - 1;
    while (hi >= 0) {
        int sm = -1;
        for (int base = hi & ~63; base >= 0; base -= 64) {
            int i = base + LANE;
            bool smart = i <= hi && (EI(c, F_FLAGS, i) & EF_SMART_STEP);
            unsigned long long m = ballot(smart);
            if (m) {
                sm = base + top_bit(m);
                break;
            }
        }
        for (int base = (sm + 1) & ~63; base <= hi; base += 64) {
            int i = base + LANE;
            if (i > sm && i <= hi) entity_step_slot(c, i);
        }
        wave_sync();
        if (sm < 0) break;
        Ent o;
        load_ent_step(c, sm, o);
        basic_step_object<G>(c, sm, o);
        entity_step(o);
        store_ent_step(c, sm, o);
        wave_sync();
        hi = sm - 1;
    }
}

DEV bool is_out_of_bounds(Ctx &c, float x, float y, float rx, float ry) { // :1077-1093
    if (x + rx < 0) return true;
    if (y + ry < 0) return true;
    if (x - rx > c.s.main_width) return true;
    if (y - ry > c.s.main_height) return true;
    return false;
}

// basic-abstract-game.cpp:757-765: order-preserving removal, lane-parallel compaction
DEV void erase_if_needed(Ctx &c) {
    int n = c.s.num_ents;
    if (n > 0 && !c.s.agent_erased) {
        // the reference's `agent` shared_ptr outlives its removal from `entities`
        Ent a;
        load_ent(c, 0, a);
        bool er = (a.flags & EF_WILL_ERASE) || ((a.flags & EF_AUTO_ERASE) && is_out_of_bounds(c, a.x, a.y, a.rx, a.ry));
        if (er) {
            c.s.agent_erased = 1;
            c.gp->ghost_x = a.x; c.gp->ghost_y = a.y; c.gp->ghost_vx = a.vx; c.gp->ghost_vy = a.vy;
            c.gp->ghost_rx = a.rx; c.gp->ghost_ry = a.ry;
        }
    }
    int kept = 0;
    for (int base = 0; base < n; base += 64) {
        int i = base + LANE;
        bool keep = false;
        if (i < n) {
            int fl = EI(c, F_FLAGS, i);
            bool er = (fl & EF_WILL_ERASE) ||
                      ((fl & EF_AUTO_ERASE) && is_out_of_bounds(c, EF(c, F_X, i), EF(c, F_Y, i), EF(c, F_RX, i), EF(c, F_RY, i)));
            keep = !er;
        }
        unsigned long long km = ballot(keep);
        int dst = kept + __popcll(km & ((1ull << LANE) - 1ull));
        bool move = keep && dst != i;
        Ent e;
        if (move) load_ent(c, i, e); // only entities that shift are read whole
        wave_sync();
        if (move) store_ent(c, dst, e);
        wave_sync();
        kept += __popcll(km);
    }
    c.s.num_ents = kept;
}

// ------------------------------------------------------------------ agent control
DEV int append_entity(Ctx &c, float x, float y, float vx, float vy, float rx, float ry, int type);
template <int G>
DEV void set_action_xy(Ctx &c, int move_action) {
    if constexpr (G == PG_GAME_CAVEFLYER) { // caveflyer.cpp:267-287: thrust along the heading
        float acceleration = (float)(move_action % 3 - 1);
        if (acceleration < 0) acceleration *= 0.33f;
        const float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
        const float theta = -1 * EF(c, F_ROTATION, 0) + PI_F / 2;
        double sn, cs; // cos / sin of a float: the double C library functions (correctly rounded)
        pg_sincos_cr((double)theta, &sn, &cs);
        if (acceleration > 0) {
            wave_sync();
            const int e = append_entity(c, (float)((double)ax - (double)arx * cs), (float)((double)ay - (double)ary * sn), 0,
                                        0, (float)(.5 * arx), (float)(.5 * arx), CF_EXHAUST);
            if (e >= 0) {
                EI(c, F_EXPIRE_TIME, e) = 4;
                EF(c, F_ROTATION, e) = -1 * theta - PI_F / 2;
                EF(c, F_GROW_RATE, e) = 1.25f;
                EF(c, F_ALPHA_DECAY, e) = 0.8f;
            }
            wave_sync();
        }
        c.s.action_vy = (float)(acceleration * sn);
        c.s.action_vx = (float)(acceleration * cs);
        c.s.action_vrot = (float)(move_action / 3 - 1);
        return;
    }
    c.s.action_vx = (float)(move_action / 3 - 1); // basic :667-671
    c.s.action_vy = (float)((move_action % 3) - 1);
    if constexpr (G == PG_GAME_COINRUN) { // coinrun.cpp:451-472
        if (c.s.action_vx > 0) c.s.facing_right = 1;
        if (c.s.action_vx < 0) c.s.facing_right = 0;
        float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0), avy = EF(c, F_VY, 0);
        int b1 = get_obj_from_floats(c, (float)((double)ax - ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        int b2 = get_obj_from_floats(c, (float)((double)ax + ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        bool s1 = cr_is_wall(b1) || b1 == c.s.out_of_bounds_object;
        bool s2 = cr_is_wall(b2) || b2 == c.s.out_of_bounds_object;
        c.s.has_support = (c.s.is_on_crate || s1 || s2) && avy == 0;
        c.s.is_on_crate = 0;
        if (c.s.action_vy == 1) {
            if (!c.s.has_support) c.s.action_vy = 0;
        }
    } else if constexpr (G == PG_GAME_NINJA) { // ninja.cpp:387-418
        auto &N = c.s.gs.nj;
        if (c.s.action_vy < 0) c.s.action_vy = 0;
        if (c.s.action_vx > 0) c.s.facing_right = 1;
        if (c.s.action_vx < 0) c.s.facing_right = 0;
        float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
        int b1 = get_obj_from_floats(c, (float)((double)ax - ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        int b2 = get_obj_from_floats(c, (float)((double)ax + ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        c.s.has_support = (b1 == NJ_WALL_MID || b1 == c.s.out_of_bounds_object) ||
                          (b2 == NJ_WALL_MID || b2 == c.s.out_of_bounds_object); // can_support (:383-385)
        if (c.s.has_support && c.s.action_vy == 1) {
            c.s.action_vy = 1;
            N.jump_charge += N.jump_charge_inc;
            if (N.jump_charge > 1) N.jump_charge = 1;
        } else {
            c.s.action_vy = 0;
        }
        if (!c.s.has_support) N.jump_charge = 0;
    } else if constexpr (G == PG_GAME_JUMPER) { // jumper.cpp:389-422 (double jump with a cooldown)
        auto &J = c.s.gs.jp;
        if (c.s.action_vy < 0) c.s.action_vy = 0;
        if (c.s.action_vx > 0) c.s.facing_right = 1;
        if (c.s.action_vx < 0) c.s.facing_right = 0;
        float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
        int b1 = get_obj_from_floats(c, (float)((double)ax - ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        int b2 = get_obj_from_floats(c, (float)((double)ax + ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        J.jump_delta = 0;
        c.s.has_support = (jp_is_wall(b1) || b1 == c.s.out_of_bounds_object) ||
                          (jp_is_wall(b2) || b2 == c.s.out_of_bounds_object); // can_support (:385-387)
        if (c.s.has_support) J.jump_count = 2;
        if (c.s.action_vy == 1 && J.jump_count > 0 && (c.s.cur_time - J.jump_time > 3)) { // JUMP_COOLDOWN
            J.jump_count -= 1;
            J.jump_delta = -1;
        } else {
            c.s.action_vy = 0;
        }
        if (c.s.action_vy > 0) J.jump_time = c.s.cur_time;
        c.s.action_vrot = 0;
    } else if constexpr (G == PG_GAME_FRUITBOT) { // fruitbot.cpp:154-158
        c.s.action_vy = 0.2f;
        c.s.action_vrot = 0;
    } else if constexpr (G == PG_GAME_PLUNDER) { // plunder.cpp:110-114
        c.s.action_vy = 0;
        c.s.action_vrot = 0;
    } else if constexpr (G == PG_GAME_CLIMBER) { // climber.cpp:299-318
        if (c.s.action_vy < 0) c.s.action_vy = 0;
        if (c.s.action_vx > 0) c.s.facing_right = 1;
        if (c.s.action_vx < 0) c.s.facing_right = 0;
        float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
        int b1 = get_obj_from_floats(c, (float)((double)ax - ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        int b2 = get_obj_from_floats(c, (float)((double)ax + ((double)arx - .01)), (float)((double)ay - ((double)ary + .01)));
        bool s1 = cl_is_wall(b1) || b1 == c.s.out_of_bounds_object; // can_support (:295-297)
        bool s2 = cl_is_wall(b2) || b2 == c.s.out_of_bounds_object;
        c.s.has_support = s1 || s2;
        c.s.action_vy = (c.s.has_support && c.s.action_vy == 1) ? 1.0f : 0.0f;
    } else {
        c.s.action_vrot = 0;
        if constexpr (G == PG_GAME_MAZE || G == PG_GAME_MINER) // maze.cpp:107-111, miner.cpp:105-109
            if (c.s.action_vx != 0) c.s.action_vy = 0;
    }
}

DEV float clip_abs(float x, float y) {
    if (x > y) return y;
    if (x < -y) return -y;
    return x;
}

// decay_vel (leaper.cpp:220-226); VEL_DECAY = MAX_SPEED / NSTEP in float
DEV float lp_decay_vel(float vel) {
    const float vel_decay = (float)(2 / (LP_NSTEP - 1.0)) / LP_NSTEP;
    float x = (float)(1.0 * vel);
    float vel_sign = x > 0 ? +1 : (x == 0 ? 0 : -1);
    vel = fabsf(vel) - vel_decay;
    if (vel < 0) vel = 0;
    return vel * vel_sign;
}

template <int G>
DEV void update_agent_velocity(Ctx &c) {
    float vx = EF(c, F_VX, 0), vy = EF(c, F_VY, 0);
    if constexpr (G == PG_GAME_COINRUN) { // coinrun.cpp:156-173
        float mixrate_x = c.s.has_support ? c.s.mixrate : (c.s.mixrate * c.s.air_control);
        vx = (1 - mixrate_x) * vx + mixrate_x * c.s.maxspeed * c.s.action_vx;
        if (fabsf(vx) < mixrate_x * c.s.maxspeed) vx = 0;
        if (c.s.action_vy > 0) {
            vy = c.s.max_jump;
        } else {
            if (c.s.has_support) vy = (float)((double)vy + .2 * (double)c.s.action_vy);
        }
        if (!(c.s.has_support && c.s.action_vy > 0)) {
            vy -= c.s.gravity;
            vy = clip_abs(vy, c.s.max_jump);
        }
    } else if constexpr (G == PG_GAME_NINJA) { // ninja.cpp:108-121
        float mixrate_x = c.s.has_support ? c.s.mixrate : (c.s.mixrate * c.s.air_control);
        vx = (1 - mixrate_x) * vx + mixrate_x * c.s.maxspeed * c.s.action_vx;
        if (c.s.action_vy < 1 && c.s.gs.nj.jump_charge > 0) {
            vy = c.s.gs.nj.jump_charge * c.s.max_jump;
            c.s.gs.nj.jump_charge = 0;
        }
        if (!c.s.has_support) {
            if (vy > -2) vy -= c.s.gravity;
        }
    } else if constexpr (G == PG_GAME_JUMPER) { // jumper.cpp:98-105
        const float v_scale = 1.0f;
        vx = (1 - c.s.mixrate) * vx + c.s.mixrate * c.s.maxspeed * c.s.action_vx * v_scale;
        if (c.s.action_vy != 0) vy = c.s.maxspeed * c.s.action_vy * 2;
    } else if constexpr (G == PG_GAME_CAVEFLYER) { // caveflyer.cpp:73-81: no (1 - mixrate) decay
        const float v_scale = 1.0f;
        vx = (float)((double)vx + (double)(c.s.mixrate * c.s.maxspeed * c.s.action_vx * v_scale) * .2);
        vy = (float)((double)vy + (double)(c.s.mixrate * c.s.maxspeed * c.s.action_vy * v_scale) * .2);
        vx = (float)(.9 * (double)vx);
        vy = (float)(.9 * (double)vy);
    } else if constexpr (G == PG_GAME_CLIMBER) { // climber.cpp:117-128
        float mixrate_x = c.s.has_support ? c.s.mixrate : (c.s.mixrate * c.s.air_control);
        vx = (1 - mixrate_x) * vx + mixrate_x * c.s.maxspeed * c.s.action_vx;
        if (c.s.action_vy > 0) vy = c.s.max_jump;
        if (!c.s.has_support) {
            if (vy > -2) vy -= c.s.gravity;
        }
    } else if constexpr (G == PG_GAME_CHASER) { // chaser.cpp:83-92 (cpp-utils double sign)
        if (c.s.action_vx != 0) vx = c.s.maxspeed * c.s.action_vx;
        if (c.s.action_vy != 0) vy = c.s.maxspeed * c.s.action_vy;
        vx = (float)(dsign(vx) * c.s.maxspeed);
        vy = (float)(dsign(vy) * c.s.maxspeed);
    } else if constexpr (G == PG_GAME_LEAPER) { // leaper.cpp:228-244
        if (vx == 0 && vy == 0) {
            if (c.s.action_vx != 0) {
                vx = c.s.maxspeed * c.s.action_vx;
                EI(c, F_IMAGE_THEME, 0) = 1;
                EF(c, F_ROTATION, 0) = (vx > 0 ? 1 : -1) * PI_F / 2;
            } else if (c.s.action_vy != 0) {
                vy = c.s.maxspeed * c.s.action_vy;
                EI(c, F_IMAGE_THEME, 0) = 1;
                EF(c, F_ROTATION, 0) = vy > 0 ? 0 : PI_F;
            }
        }
        vx = lp_decay_vel(vx);
        vy = lp_decay_vel(vy);
    } else { // basic-abstract-game.cpp:678-693 (get_agent_acceleration_scale() = 1)
        const float v_scale = 1.0f;
        vx = (1 - c.s.mixrate) * vx;
        vy = (1 - c.s.mixrate) * vy;
        vx += c.s.mixrate * c.s.maxspeed * c.s.action_vx * v_scale;
        vy += c.s.mixrate * c.s.maxspeed * c.s.action_vy * v_scale;
        vx = (float)(.9 * (double)vx); // decay_agent_velocity
        vy = (float)(.9 * (double)vy);
    }
    EF(c, F_VX, 0) = vx;
    EF(c, F_VY, 0) = vy;
}

// asset_aspect_ratios of an image slot (basic-abstract-game.cpp:79-123): the image loaded for
// the slot after mask_theme_if_necessary, width * 1.0 / height
template <int G>
DEV bool preserve_theme(int type) { // should_preserve_type_themes (heist.cpp:42-44)
    if constexpr (G == PG_GAME_HEIST) return type == HS_KEY || type == HS_LOCKED_DOOR;
    if constexpr (G == PG_GAME_PLUNDER) return type == PL_SHIP; // plunder.cpp:83-85
    return false;
}
template <int G>
DEV float aspect_ratio(Ctx &c, int type, int theme) {
    if (c.s.opt_restrict_themes && !preserve_theme<G>(type)) theme = 0;
    int4 sp = reinterpret_cast<const int4 *>(c.d.sprites + (size_t)G * PG_NUM_SLOTS * 4)[type + theme * MAX_ASSETS];
    if (sp.y <= 0 || sp.z <= 0) {
        c.s.error = PG_ERR_BAD_OPTION;
        return 1.0f;
    }
    return (float)(sp.y * 1.0 / sp.z);
}

// ------------------------------------------------------------------ agent / entity collisions
// handle_agent_collision (basic :387-389; coinrun.cpp:123-131; bigfish.cpp:45-59; heist.cpp:80-96)
template <int G>
DEV void handle_agent_collision(Ctx &c, int m) {
    const int t = EI(c, F_TYPE, m);
    if constexpr (G == PG_GAME_COINRUN) {
        if (t == CR_ENEMY || t == CR_SAW) c.s.sd_done = 1;
    } else if constexpr (G == PG_GAME_BIGFISH) {
        if (t == BF_FISH) {
            const float arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
            if (EF(c, F_RX, m) > arx) {
                c.s.sd_done = 1;
            } else {
                c.s.sd_reward += 1; // POSITIVE_REWARD
                EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
                EF(c, F_RX, 0) = arx + c.s.r_inc;
                EF(c, F_RY, 0) = ary + c.s.r_inc;
                c.s.fish_eaten += 1;
            }
        }
    } else if constexpr (G == PG_GAME_JUMPER) { // jumper.cpp:86-96
        if (t == JP_GOAL) {
            c.s.sd_reward += 10.0f; // GOAL_REWARD
            c.s.sd_level_complete = 1;
            c.s.sd_done = 1;
        } else if (t == JP_SPIKE) {
            c.s.sd_done = 1;
        }
    } else if constexpr (G == PG_GAME_CAVEFLYER) { // caveflyer.cpp:57-71
        if (t == CF_GOAL) {
            c.s.sd_reward += 10.0f; // GOAL_REWARD
            c.s.sd_level_complete = 1;
            c.s.sd_done = 1;
        } else if (t == CF_OBSTACLE || t == CF_ENEMY || t == CF_TARGET) {
            c.s.sd_done = 1;
        }
    } else if constexpr (G == PG_GAME_NINJA) { // ninja.cpp:77-87
        if (t == EXPLOSION) {
            c.s.sd_done = 1;
        } else if (t == NJ_GOAL) {
            c.s.sd_reward += 10.0f; // GOAL_REWARD
            c.s.sd_level_complete = 1;
            c.s.sd_done = 1;
        }
    } else if constexpr (G == PG_GAME_BOSSFIGHT) { // bossfight.cpp:120-131
        if (t == BF_BOSS || t == BF_BARRIER || t == BF_ENEMY_BULLET) c.s.sd_done = 1;
    } else if constexpr (G == PG_GAME_STARPILOT) { // starpilot.cpp:126-136
        if (t == SP_FINISH_LINE) {
            c.s.sd_done = 1;
            c.s.sd_reward += 10.0f; // COMPLETION_BONUS
            c.s.sd_level_complete = 1;
        } else if (t == SP_FLYER || t == SP_FAST_FLYER || t == SP_BULLET2 || t == SP_BULLET3 || t == SP_TURRET ||
                   t == SP_METEOR) { // is_lethal (:346-350)
            c.s.sd_done = 1;
        }
    } else if constexpr (G == PG_GAME_DODGEBALL) { // dodgeball.cpp:102-118
        if (t == DB_ENEMY || t == DB_ENEMY_BALL || t == DB_LAVA_WALL) {
            c.s.sd_done = 1;
        } else if (t == DB_DOOR && c.s.num_enemies == 0) {
            c.s.sd_done = 1;
            c.s.sd_reward += 10.0f; // COMPLETION_BONUS
            c.s.sd_level_complete = 1;
        }
    } else if constexpr (G == PG_GAME_FRUITBOT) { // fruitbot.cpp:95-115
        if (t == FB_BARRIER || t == FB_LOCKED_DOOR) {
            c.s.sd_done = 1;
        } else if (t == FB_BAD_OBJ) {
            c.s.sd_reward += -4; // PENALTY (const int)
            EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
        } else if (t == FB_GOOD_OBJ) {
            c.s.sd_reward += 1; // POSITIVE_REWARD (const int)
            EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
        } else if (t == FB_PRESENT) {
            c.s.sd_reward += 10.0f; // COMPLETION_BONUS
            c.s.sd_done = 1;
            c.s.sd_level_complete = 1;
        }
    } else if constexpr (G == PG_GAME_CHASER) { // chaser.cpp:119-133
        if (t == CH_LARGE_ORB) {
            c.s.eat_time = c.s.cur_time;
            c.s.sd_reward += 0.04f; // ORB_REWARD
            EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
        } else if (t == CH_ENEMY) {
            if (c.s.cur_time - c.s.eat_time < c.s.eat_timeout) EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
            else c.s.sd_done = 1;
        }
    } else if constexpr (G == PG_GAME_LEAPER) { // leaper.cpp:76-84
        if (t == LP_CAR) {
            c.s.sd_done = 1;
        } else if (t == LP_FINISH_LINE && EF(c, F_VX, 0) == 0 && EF(c, F_VY, 0) == 0) {
            c.s.sd_reward += 10; // GOAL_REWARD (const int)
            c.s.sd_done = 1;
            c.s.sd_level_complete = 1;
        }
    } else if constexpr (G == PG_GAME_CLIMBER) { // climber.cpp:93-103
        if (t == CL_ENEMY) {
            c.s.sd_done = 1;
        } else if (t == CL_COIN) {
            c.s.sd_reward += 1.0f; // COIN_REWARD
            c.s.coins_collected += 1;
            EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
        }
    } else if constexpr (G == PG_GAME_MINER) { // miner.cpp:81-93
        if (t == MN_ENEMY) {
            c.s.sd_done = 1;
        } else if (t == MN_EXIT) {
            if (c.s.diamonds_remaining == 0) {
                c.s.sd_reward += 10.0f; // COMPLETION_BONUS
                c.s.sd_level_complete = 1;
                c.s.sd_done = 1;
            }
        }
    } else if constexpr (G == PG_GAME_HEIST) {
        if (t == HS_EXIT) {
            c.s.sd_done = 1;
            c.s.sd_reward = 10.0f; // COMPLETION_BONUS (assignment)
            c.s.sd_level_complete = 1;
        } else if (t == HS_KEY) {
            EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
            c.s.has_keys |= 1 << EI(c, F_IMAGE_THEME, m);
        } else if (t == HS_LOCKED_DOOR) {
            if ((c.s.has_keys >> EI(c, F_IMAGE_THEME, m)) & 1) EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
        }
    }
}

// The loop of game_step over entities (basic-abstract-game.cpp:728-750), reverse order.
// coinrun: the effects are order-free flags, one lane-parallel pass.  Other games: the
// colliding entities are handled one at a time from the top, re-testing below the last one
// with the current agent (bigfish grows the agent; heist keys open later doors).
// Entities with collides_with_entities (fruitbot's bullets) run their inner loop (:735-744) at
// their place in the same descending walk.  check_grid_collisions has an effect only in coinrun
// (handle_grid_collision, coinrun.cpp:144-154).
//
// handle_collision(src, target) (basic :383-385 empty; fruitbot.cpp:117-134)
DEV int append_entity(Ctx &c, float x, float y, float vx, float vy, float rx, float ry, int type);
DEV int find_type(Ctx &c, int type) { // first entity of a type (bossfight's boss / shields pointers)
    for (int base = 0; base < c.s.num_ents; base += 64) {
        const int i = base + LANE;
        const unsigned long long b = ballot(i < c.s.num_ents && EI(c, F_TYPE, i) == type);
        if (b) return base + __ffsll((long long)b) - 1;
    }
    return -1;
}
DEV void bf_prepare_boss(Ctx &c, int boss) { // bossfight.cpp:192-199
    auto &B = c.s.gs.bf;
    B.shields_are_up = 1;
    B.curr_vel_timeout = BF_BOSS_VEL_TIMEOUT;
    B.time_to_swap = B.invulnerable_duration;
    B.attack_mode = (int)((B.attack_modes >> (2 * (B.round_num % B.num_rounds))) & 3u);
    if (boss >= 0) {
        EF(c, F_VX, boss) = 0;
        EF(c, F_VY, boss) = 0;
    }
}
DEV bool sp_destructible(int t) { return t == SP_FLYER || t == SP_FAST_FLYER || t == SP_TURRET || t == SP_METEOR; }
template <int G>
DEV void handle_collision(Ctx &c, int si, int ti) {
    if constexpr (G == PG_GAME_CAVEFLYER) { // caveflyer.cpp:92-118: only a PLAYER_BULLET target acts
        if (EI(c, F_TYPE, ti) == CF_PLAYER_BULLET) {
            const int st = EI(c, F_TYPE, si);
            bool erase_bullet = false;
            if (st == CF_TARGET) {
                const float h = EF(c, F_HEALTH, si) - 1;
                EF(c, F_HEALTH, si) = h;
                erase_bullet = true;
                const int sf = EI(c, F_FLAGS, si);
                if (h <= 0 && !(sf & EF_WILL_ERASE)) {
                    const float sx = EF(c, F_X, si), sy = EF(c, F_Y, si), r = (float)(.5 * EF(c, F_RX, si));
                    wave_sync();
                    append_entity(c, sx, sy, 0, 0, r, r, EXPLOSION); // spawn_child(src, EXPLOSION, .5 * rx)
                    EI(c, F_FLAGS, si) = sf | EF_WILL_ERASE;
                    c.s.sd_reward += 3.0f; // TARGET_REWARD
                }
            } else if (st == CF_OBSTACLE || st == CF_ENEMY || st == CF_GOAL) {
                erase_bullet = true;
            }
            const int tf = EI(c, F_FLAGS, ti);
            if (erase_bullet && !(tf & EF_WILL_ERASE)) {
                EI(c, F_FLAGS, ti) = tf | EF_WILL_ERASE;
                const float tx = EF(c, F_X, ti), ty = EF(c, F_Y, ti), r = (float)(.5 * EF(c, F_RX, ti));
                const float svx = EF(c, F_VX, si), svy = EF(c, F_VY, si);
                wave_sync();
                append_entity(c, tx, ty, svx, svy, r, r, EXPLOSION); // explosion takes src's velocity
            }
        }
    }
    if constexpr (G == PG_GAME_BOSSFIGHT) { // bossfight.cpp:140-190
        auto &B = c.s.gs.bf;
        const int st = EI(c, F_TYPE, si), tt = EI(c, F_TYPE, ti);
        if (st == BF_PLAYER_BULLET) {
            bool will_erase = false;
            if (tt == BF_SHIELDS) {
                if (B.shields_are_up) {
                    EI(c, F_TYPE, si) = BF_REFLECTED_BULLET;
                    const float theta = (float)(PI_F * (1.25 + .5 * B.rand_pct));
                    double sn, cs;
                    pg_sincos_cr((double)theta, &sn, &cs);
                    EF(c, F_VY, si) = (float)(1 * sn * .5); // PLAYER_BULLET_VEL (const int 1)
                    EF(c, F_VX, si) = (float)(1 * cs * .5);
                    EI(c, F_EXPIRE_TIME, si) = 4;
                    EI(c, F_LIFE_TIME, si) = 0;
                    EF(c, F_ALPHA_DECAY, si) = 0.8f;
                }
            } else if (tt == BF_BOSS) {
                if (!B.shields_are_up) {
                    const float h = EF(c, F_HEALTH, ti) - 1;
                    EF(c, F_HEALTH, ti) = h;
                    will_erase = true;
                    if ((int)h % B.round_health == 0) {
                        c.s.sd_reward += 1; // POSITIVE_REWARD (const int)
                        if (h == 0) {
                            c.s.sd_done = 1;
                            c.s.sd_reward += 10; // COMPLETION_BONUS (const int)
                            c.s.sd_level_complete = 1;
                        } else {
                            B.round_num++;
                            wave_sync();
                            bf_prepare_boss(c, ti);
                            B.curr_vel_timeout = BF_BOSS_DAMAGED_TIMEOUT;
                            B.damaged_until_time = c.s.cur_time + BF_BOSS_DAMAGED_TIMEOUT;
                        }
                    }
                }
            }
            const int sf = EI(c, F_FLAGS, si);
            if (will_erase && !(sf & EF_WILL_ERASE)) {
                EI(c, F_FLAGS, si) = sf | EF_WILL_ERASE;
                const float sx = EF(c, F_X, si), sy = EF(c, F_Y, si), r = (float)(.5 * EF(c, F_RX, si));
                const float tvx = EF(c, F_VX, ti), tvy = EF(c, F_VY, ti);
                wave_sync();
                append_entity(c, sx, sy, tvx, tvy, r, r, EXPLOSION); // spawn_child + target velocity
            }
        } else if (st == BF_BARRIER) {
            if (tt == BF_ENEMY_BULLET || tt == BF_PLAYER_BULLET) {
                EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
                const float tx = EF(c, F_X, ti), ty = EF(c, F_Y, ti), r = (float)(.5 * EF(c, F_RX, ti));
                wave_sync();
                append_entity(c, tx, ty, 0, 0, r, r, EXPLOSION); // spawn_child(target, EXPLOSION, .5 * rx)
            } else if (tt == BF_LASER_TRAIL) {
                EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
            }
            wave_sync();
            if (EF(c, F_HEALTH, si) <= 0) { // barriers keep health 3: never taken
                const int sf = EI(c, F_FLAGS, si);
                if (!(sf & EF_WILL_ERASE)) {
                    const float sx = EF(c, F_X, si), sy = EF(c, F_Y, si), r = (float)(.5 * EF(c, F_RX, si));
                    const float svx = EF(c, F_VX, si), svy = EF(c, F_VY, si);
                    wave_sync();
                    append_entity(c, sx, sy, svx, svy, r, r, EXPLOSION);
                }
                EI(c, F_FLAGS, si) = EI(c, F_FLAGS, si) | EF_WILL_ERASE;
            }
        }
    }
    if constexpr (G == PG_GAME_STARPILOT) { // starpilot.cpp:138-145
        const int tt = EI(c, F_TYPE, ti);
        if (EI(c, F_TYPE, si) == SP_BULLET_PLAYER && tt != SP_CLOUD && sp_destructible(tt)) {
            EI(c, F_FLAGS, si) = EI(c, F_FLAGS, si) | EF_WILL_ERASE;
            EF(c, F_HEALTH, ti) = EF(c, F_HEALTH, ti) - 1;
            const float sx = EF(c, F_X, si), sy = EF(c, F_Y, si), tvx = EF(c, F_VX, ti), tvy = EF(c, F_VY, ti);
            const float r = (float)(.5 * EF(c, F_RX, si));
            wave_sync();
            append_entity(c, sx, sy, tvx, tvy, r, r, EXPLOSION);
        }
    }
    if constexpr (G == PG_GAME_PLUNDER) { // plunder.cpp:87-108
        if (EI(c, F_TYPE, si) == PL_PLAYER_BULLET) {
            const int tt = EI(c, F_TYPE, ti);
            bool target_erased = false;
            if (tt == PL_SHIP) {
                EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
                EI(c, F_FLAGS, si) = EI(c, F_FLAGS, si) | EF_WILL_ERASE;
                target_erased = true;
                if ((c.s.gs.pl.target_bools >> EI(c, F_IMAGE_THEME, ti)) & 1u) {
                    c.s.gs.pl.targets_hit += 1;
                    c.s.sd_reward += 1.0f; // POSITIVE_REWARD
                    c.s.gs.pl.juice_left += 0.1f;
                } else {
                    c.s.gs.pl.juice_left -= 0.1f;
                }
            } else if (tt == PL_PANEL) {
                EI(c, F_FLAGS, si) = EI(c, F_FLAGS, si) | EF_WILL_ERASE;
            }
            if (target_erased) { // add_entity(x, y, vx / 2, vy / 2, .5 * rx, EXPLOSION)
                const float tx = EF(c, F_X, ti), ty = EF(c, F_Y, ti);
                const float tvx = EF(c, F_VX, ti) / 2, tvy = EF(c, F_VY, ti) / 2;
                const float tr = (float)(.5 * EF(c, F_RX, ti));
                wave_sync();
                append_entity(c, tx, ty, tvx, tvy, tr, tr, EXPLOSION);
            }
        }
    }
    if constexpr (G == PG_GAME_DODGEBALL) { // dodgeball.cpp:120-151
        const int tt = EI(c, F_TYPE, ti), st = EI(c, F_TYPE, si);
        if (tt == DB_PLAYER_BALL) {
            if (st == DB_LAVA_WALL) {
                EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
            } else if (st == DB_ENEMY) {
                const float h = EF(c, F_HEALTH, si) - 1;
                EF(c, F_HEALTH, si) = h;
                EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
                const int sf = EI(c, F_FLAGS, si);
                if (h <= 0 && !(sf & EF_WILL_ERASE)) {
                    EI(c, F_FLAGS, si) = sf | EF_WILL_ERASE;
                    c.s.sd_reward += 2; // ENEMY_REWARD (const int 2.0f)
                    // spawn_child(src, DUST_CLOUD, src->rx) (basic-abstract-game.cpp:233-239)
                    const float sx = EF(c, F_X, si), sy = EF(c, F_Y, si), sr = EF(c, F_RX, si);
                    wave_sync();
                    const int k = append_entity(c, sx, sy, 0, 0, sr, sr, DB_DUST_CLOUD);
                    if (k >= 0) {
                        EF(c, F_VROT, k) = PI_F / 0.3f;
                        EF(c, F_GROW_RATE, k) = 1.0f / 1.2f;
                        EI(c, F_EXPIRE_TIME, k) = 4;
                        EF(c, F_ALPHA_DECAY, k) = 0.9f;
                        EI(c, F_IMAGE_THEME, k) = c.s.step_rand_int % c.d.num_themes[G * 100 + DB_DUST_CLOUD]; // choose_step_random_theme
                    }
                }
            }
        } else if (tt == DB_ENEMY_BALL) {
            if (st == DB_LAVA_WALL) EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
        }
    }
    if constexpr (G == PG_GAME_FRUITBOT) {
        if (EI(c, F_TYPE, si) == FB_PLAYER_BULLET) {
            const int tt = EI(c, F_TYPE, ti);
            if (tt == FB_BARRIER) {
                EI(c, F_FLAGS, si) = EI(c, F_FLAGS, si) | EF_WILL_ERASE;
            } else if (tt == FB_LOCK) {
                const float ty = EF(c, F_Y, ti);
                EI(c, F_FLAGS, si) = EI(c, F_FLAGS, si) | EF_WILL_ERASE;
                EI(c, F_FLAGS, ti) = EI(c, F_FLAGS, ti) | EF_WILL_ERASE;
                // the first LOCKED_DOOR in list order within 1 of the lock's y
                for (int base = 0; base < c.s.num_ents; base += 64) {
                    int k = base + LANE;
                    bool hit = k < c.s.num_ents && EI(c, F_TYPE, k) == FB_LOCKED_DOOR && fabsf(EF(c, F_Y, k) - ty) < 1;
                    unsigned long long b = ballot(hit);
                    if (b) {
                        int d = base + __ffsll((long long)b) - 1;
                        wave_sync();
                        EI(c, F_FLAGS, d) = EI(c, F_FLAGS, d) | EF_WILL_ERASE;
                        break;
                    }
                }
            }
        }
    }
    wave_sync();
}

// The collision walk's view of the entity list (lane = entity, lists of at most 64): the fields the
// walks test, loaded in one round instead of one round per scan.  A handler may change any entity or
// append one, so the cache is reloaded after every handler call (handlers are rare; scans are not).
struct ColCache {
    float x, y, rx, ry, mrg;
    int type, flags;
    bool ok; // the list fits one lane each and the registers hold HBM's current values
};
DEV void col_load(Ctx &c, ColCache &k) {
    k.ok = c.s.num_ents <= 64;
    if (!k.ok) return;
    const int i = LANE;
    if (i < c.s.num_ents) {
        k.x = EF(c, F_X, i); k.y = EF(c, F_Y, i); k.rx = EF(c, F_RX, i); k.ry = EF(c, F_RY, i);
        k.mrg = EF(c, F_COLLISION_MARGIN, i); k.type = EI(c, F_TYPE, i); k.flags = EI(c, F_FLAGS, i);
    } else {
        k.x = k.y = k.rx = k.ry = k.mrg = 0;
        k.type = -1;
        k.flags = EF_WILL_ERASE;
    }
}

// the inner loop of an entity with collides_with_entities: j descending, j != i, while neither
// side is will_erase
template <int G>
DEV void entity_collisions(Ctx &c, int i, ColCache &k) {
    int upper = c.s.num_ents;
    while (upper > 0) {
        if (k.ok) { // from the registers: one scan of <= 64 lanes
            if (rli(k.flags, i) & EF_WILL_ERASE) return;
            const float x = rlf(k.x, i), y = rlf(k.y, i), rx = rlf(k.rx, i), ry = rlf(k.ry, i), mrg = rlf(k.mrg, i);
            const int j = LANE;
            bool relevant = true;
            if constexpr (G == PG_GAME_CAVEFLYER) relevant = k.type == CF_PLAYER_BULLET;
            bool hit = false;
            if (relevant && j < upper && j != i && !(k.flags & EF_WILL_ERASE)) {
                float tx = (rx + k.rx) + mrg, ty = (ry + k.ry) + mrg;
                hit = (fabsf(x - k.x) < tx) && (fabsf(y - k.y) < ty);
            }
            const unsigned long long b = ballot(hit);
            if (!b) return;
            const int m = top_bit(b);
            handle_collision<G>(c, i, m);
            wave_sync();
            col_load(c, k);
            upper = m;
            continue;
        }
        if (EI(c, F_FLAGS, i) & EF_WILL_ERASE) return;
        const float x = EF(c, F_X, i), y = EF(c, F_Y, i), rx = EF(c, F_RX, i), ry = EF(c, F_RY, i);
        const float mrg = EF(c, F_COLLISION_MARGIN, i);
        int m = -1;
        for (int base = (upper - 1) & ~63; base >= 0; base -= 64) {
            int j = base + LANE;
            bool hit = false;
            bool relevant = true;
            if constexpr (G == PG_GAME_CAVEFLYER) relevant = j < upper && EI(c, F_TYPE, j) == CF_PLAYER_BULLET;
            if (relevant && j < upper && j != i && !(EI(c, F_FLAGS, j) & EF_WILL_ERASE)) {
                float tx = (rx + EF(c, F_RX, j)) + mrg, ty = (ry + EF(c, F_RY, j)) + mrg;
                hit = (fabsf(x - EF(c, F_X, j)) < tx) && (fabsf(y - EF(c, F_Y, j)) < ty);
            }
            unsigned long long b = ballot(hit);
            if (b) {
                m = base + top_bit(b);
                break;
            }
        }
        if (m < 0) return;
        handle_collision<G>(c, i, m);
        upper = m;
    }
}

// ninja's check_grid_collisions (basic-abstract-game.cpp:145-165 -> ninja.cpp:89-106) of smart
// entity m: the agent dies on FIRE / BOMB; a star that touches a BOMB clears the cell (HBM grid,
// its int8 mirror, this step's LDS copy) and leaves an EXPLOSION, and a star on a wall goes away
DEV void ninja_grid_collisions(Ctx &c, int m) {
    const float ax = EF(c, F_X, m), ay = EF(c, F_Y, m), arx = EF(c, F_RX, m), ary = EF(c, F_RY, m);
    const int t = EI(c, F_TYPE, m);
    const int min_x = (int)(ax - (arx + POS_EPS)), max_x = (int)(ax + (arx + POS_EPS));
    const int min_y = (int)(ay - (ary + POS_EPS)), max_y = (int)(ay + (ary + POS_EPS));
    for (int x = min_x; x <= max_x; x++) {
        for (int y = min_y; y <= max_y; y++) {
            const int gt = get_obj_from_floats(c, (float)x, (float)y);
            if (gt == SPACE) continue;
            if (t == PLAYER) {
                if (gt == NJ_FIRE || gt == NJ_BOMB) c.s.sd_done = 1;
            } else if (t == NJ_THROWING_STAR) {
                if (gt == NJ_BOMB) {
                    EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
                    const int cell = y * c.s.main_width + x; // set_obj(x, y, SPACE): in the world (a BOMB was read)
                    if (LANE == 0) {
                        c.d.grid[(size_t)c.env * PG_GRID_MAX + cell] = SPACE;
                        c.d.grid8[(size_t)c.env * PG_GRID_MAX + cell] = (int8_t)SPACE;
                        c.grid8[cell] = (int8_t)SPACE;
                    }
                    wave_sync();
                    append_entity(c, (float)(x + .5), (float)(y + .5), 0, 0, .5f, .5f, EXPLOSION);
                    wave_sync();
                }
                if (gt == NJ_WALL_MID) EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
            }
        }
    }
    wave_sync();
}

template <int G>
DEV void agent_collisions(Ctx &c) {
    if constexpr (G == PG_GAME_NINJA) {
        // descending walk (:727-751): entity m matters if it touches the agent (EXPLOSION / GOAL
        // effects) or is smart (its grid check: the agent, throwing stars); the stars'
        // collides_with_entities loop calls the empty base handle_collision
        int upper = c.s.num_ents;
        const bool gh = c.s.agent_erased;
        const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
        const float arx = gh ? c.gp->ghost_rx : EF(c, F_RX, 0), ary = gh ? c.gp->ghost_ry : EF(c, F_RY, 0);
        while (upper > 0) {
            int m = -1;
            bool agent_hit = false;
            for (int base = (upper - 1) & ~63; base >= 0; base -= 64) {
                const int i = base + LANE;
                bool hit = false, smart = false;
                if (i < upper) {
                    const int t = EI(c, F_TYPE, i);
                    if ((t == EXPLOSION || t == NJ_GOAL) && (gh || i != 0)) {
                        const float mrg = EF(c, F_COLLISION_MARGIN, i);
                        const float tx = (EF(c, F_RX, i) + arx) + mrg, ty = (EF(c, F_RY, i) + ary) + mrg;
                        hit = (fabsf(EF(c, F_X, i) - ax) < tx) && (fabsf(EF(c, F_Y, i) - ay) < ty);
                    }
                    smart = (EI(c, F_FLAGS, i) & EF_SMART_STEP) != 0;
                }
                const unsigned long long b = ballot(hit || smart);
                if (b) {
                    m = base + top_bit(b);
                    agent_hit = ballot(hit && i == m) != 0;
                    break;
                }
            }
            if (m < 0) break;
            if (agent_hit) handle_agent_collision<G>(c, m);
            wave_sync();
            if (EI(c, F_FLAGS, m) & EF_SMART_STEP) ninja_grid_collisions(c, m);
            upper = m;
        }
        return;
    }
    if constexpr (G == PG_GAME_COINRUN) {
        bool unsupported = false; // no coinrun entity has collides_with_entities
        for (int base = 0; base < c.s.num_ents; base += 64) {
            int i = base + LANE;
            if (i < c.s.num_ents && (EI(c, F_FLAGS, i) & EF_COLLIDES)) unsupported = true;
        }
        if (ballot(unsupported)) c.s.error = PG_ERR_BAD_OPTION;
    }
    if constexpr (G == PG_GAME_COINRUN) {
        float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
        bool any = false;
        for (int base = 0; base < c.s.num_ents; base += 64) {
            int i = base + LANE;
            bool hit = false;
            if (i < c.s.num_ents) {
                int t = EI(c, F_TYPE, i);
                if (t != PLAYER) {
                    float mrg = EF(c, F_COLLISION_MARGIN, i);
                    float tx = (EF(c, F_RX, i) + arx) + mrg, ty = (EF(c, F_RY, i) + ary) + mrg;
                    bool col = (fabsf(EF(c, F_X, i) - ax) < tx) && (fabsf(EF(c, F_Y, i) - ay) < ty);
                    hit = col && (t == CR_ENEMY || t == CR_SAW);
                }
            }
            any = any || ballot(hit) != 0;
        }
        if (any) c.s.sd_done = 1;
        // check_grid_collisions(agent) (:145-165 -> coinrun.cpp:144-154); enemies have no
        // grid-collision effect in coinrun.
        int min_x = (int)(ax - (arx + POS_EPS));
        int max_x = (int)(ax + (arx + POS_EPS));
        int min_y = (int)(ay - (ary + POS_EPS));
        int max_y = (int)(ay + (ary + POS_EPS));
        for (int x = min_x; x <= max_x; x++) {
            for (int y = min_y; y <= max_y; y++) {
                int t = get_obj_from_floats(c, (float)x, (float)y);
                if (t == SPACE) continue;
                if (t == CR_GOAL) {
                    c.s.sd_reward += 10.0f;
                    c.s.sd_done = 1;
                    c.s.sd_level_complete = 1;
                } else if (cr_is_lava(t)) {
                    c.s.sd_done = 1;
                }
            }
        }
    } else {
        int upper = c.s.num_ents;
        ColCache k;
        col_load(c, k);
        while (upper > 0) {
            // the reference's `agent` (a ghost once erased from `entities`, miner.cpp:329)
            const bool gh = c.s.agent_erased;
            if (k.ok) { // the same walk from the registers (lists of <= 64), reloaded after every handler
                const float ax = gh ? c.gp->ghost_x : rlf(k.x, 0), ay = gh ? c.gp->ghost_y : rlf(k.y, 0);
                const float arx = gh ? c.gp->ghost_rx : rlf(k.rx, 0), ary = gh ? c.gp->ghost_ry : rlf(k.ry, 0);
                const int i = LANE;
                bool hit = false, coll = false;
                if (i < upper) {
                    if (k.type != PLAYER && (gh || i != 0)) { // has_agent_collision (:1135-1140)
                        float tx = (k.rx + arx) + k.mrg, ty = (k.ry + ary) + k.mrg;
                        hit = (fabsf(k.x - ax) < tx) && (fabsf(k.y - ay) < ty);
                    }
                    coll = (k.flags & EF_COLLIDES) != 0;
                }
                const unsigned long long b = ballot(hit || coll);
                if (!b) break;
                const int m = top_bit(b);
                if (ballot(hit && i == m)) {
                    handle_agent_collision<G>(c, m);
                    wave_sync();
                    col_load(c, k);
                } else {
                    wave_sync();
                }
                if (k.ok ? (rli(k.flags, m) & EF_COLLIDES) : (EI(c, F_FLAGS, m) & EF_COLLIDES)) entity_collisions<G>(c, m, k);
                upper = m;
                continue;
            }
            const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
            const float arx = gh ? c.gp->ghost_rx : EF(c, F_RX, 0), ary = gh ? c.gp->ghost_ry : EF(c, F_RY, 0);
            int m = -1;
            bool agent_hit = false;
            for (int base = (upper - 1) & ~63; base >= 0; base -= 64) {
                int i = base + LANE;
                bool hit = false, coll = false;
                if (i < upper) {
                    if (EI(c, F_TYPE, i) != PLAYER && (gh || i != 0)) { // has_agent_collision (:1135-1140)
                        float mrg = EF(c, F_COLLISION_MARGIN, i);
                        float tx = (EF(c, F_RX, i) + arx) + mrg, ty = (EF(c, F_RY, i) + ary) + mrg;
                        hit = (fabsf(EF(c, F_X, i) - ax) < tx) && (fabsf(EF(c, F_Y, i) - ay) < ty);
                    }
                    coll = (EI(c, F_FLAGS, i) & EF_COLLIDES) != 0;
                }
                unsigned long long b = ballot(hit || coll);
                if (b) {
                    m = base + top_bit(b);
                    agent_hit = ballot(hit && i == m) != 0;
                    break;
                }
            }
            if (m < 0) break;
            if (agent_hit) handle_agent_collision<G>(c, m);
            wave_sync();
            if (EI(c, F_FLAGS, m) & EF_COLLIDES) entity_collisions<G>(c, m, k);
            upper = m;
        }
    }
}

// ------------------------------------------------------------------ per-game step tails
DEV void flag_reflected(Ctx &c, int slot, bool set) {
    int fl = EI(c, F_FLAGS, slot);
    EI(c, F_FLAGS, slot) = set ? (fl | EF_REFLECTED) : (fl & ~EF_REFLECTED);
}

// Entity(x, y, vx, vy, rx, ry, type) appended to `entities` (entity.cpp:8-47)
DEV int append_entity(Ctx &c, float x, float y, float vx, float vy, float rx, float ry, int type) {
    int i = c.s.num_ents;
    if (i >= PG_CAP - c.s.num_tail) {
        c.s.error = PG_ERR_ENTITY_OVERFLOW;
        return -1;
    }
    c.s.num_ents = i + 1;
    EF(c, F_X, i) = x; EF(c, F_Y, i) = y; EF(c, F_VX, i) = vx; EF(c, F_VY, i) = vy;
    EF(c, F_RX, i) = rx; EF(c, F_RY, i) = ry; EF(c, F_ROTATION, i) = 0; EF(c, F_VROT, i) = 0;
    EF(c, F_ALPHA, i) = 1.0f; EF(c, F_ALPHA_DECAY, i) = 1.0f; EF(c, F_GROW_RATE, i) = 1.0f;
    EF(c, F_FRICTION, i) = 1; EF(c, F_COLLISION_MARGIN, i) = 0; EF(c, F_HEALTH, i) = 1;
    EF(c, F_THETA, i) = -100; EF(c, F_CLIMBER_SPAWN_X, i) = 0;
    EI(c, F_TYPE, i) = type; EI(c, F_IMAGE_TYPE, i) = type; EI(c, F_IMAGE_THEME, i) = 0;
    EI(c, F_RENDER_Z, i) = 0; EI(c, F_LIFE_TIME, i) = 0; EI(c, F_EXPIRE_TIME, i) = -1;
    EI(c, F_FIRE_TIME, i) = -1; EI(c, F_SPAWN_TIME, i) = -1; EI(c, F_FLAGS, i) = EF_AUTO_ERASE;
    if (type == EXPLOSION) { // entity.cpp:40-43
        EF(c, F_GROW_RATE, i) = 1.4f;
        EI(c, F_EXPIRE_TIME, i) = 4;
    } else if (type == TRAIL) { // entity.cpp:44-46
        EF(c, F_GROW_RATE, i) = 1.05f;
        EF(c, F_ALPHA_DECAY, i) = 0.8f;
    }
    return i;
}

DEV void coinrun_step_tail(Ctx &c) { // coinrun.cpp:474-498
    if (!c.s.agent_erased) {
        int fl = EI(c, F_FLAGS, 0);
        if (c.s.action_vx > 0) fl &= ~EF_REFLECTED;
        if (c.s.action_vx < 0) fl |= EF_REFLECTED;
        EI(c, F_FLAGS, 0) = fl;
    }
    wave_sync();
    int n = c.s.num_ents;
    // enemies (reverse order) each append a trail; trail k belongs to the k-th enemy from the top
    int total_enemies = 0;
    for (int base = 0; base < n; base += 64) {
        int i = base + LANE;
        total_enemies += __popcll(ballot(i < n && EI(c, F_TYPE, i) == CR_ENEMY));
    }
    if (n + total_enemies > PG_CAP) {
        c.s.error = PG_ERR_ENTITY_OVERFLOW;
        total_enemies = 0;
    }
    int above = 0; // enemies at indices greater than the current chunk
    for (int base = (n - 1) & ~63; base >= 0 && total_enemies > 0; base -= 64) {
        int i = base + LANE;
        int t = i < n ? EI(c, F_TYPE, i) : -1;
        unsigned long long em = ballot(t == CR_ENEMY);
        if (t == CR_ENEMY) {
            int rank = above + __popcll(em >> LANE) - 1; // enemies at >= i in this chunk, minus self
            int ti = n + rank;
            float ex = EF(c, F_X, i);
            float ey = (float)((double)EF(c, F_Y, i) - (double)EF(c, F_RY, i) * .5);
            // Entity(x, y, 0, 0.01f, 0.3f, 0.2f, TRAIL) (entity.cpp:8-47) + expire_time 8, alpha .5
            EF(c, F_X, ti) = ex; EF(c, F_Y, ti) = ey; EF(c, F_VX, ti) = 0; EF(c, F_VY, ti) = 0.01f;
            EF(c, F_RX, ti) = 0.3f; EF(c, F_RY, ti) = 0.2f; EF(c, F_ROTATION, ti) = 0; EF(c, F_VROT, ti) = 0;
            EF(c, F_ALPHA, ti) = .5f; EF(c, F_ALPHA_DECAY, ti) = 0.8f; EF(c, F_GROW_RATE, ti) = 1.05f;
            EF(c, F_FRICTION, ti) = 1; EF(c, F_COLLISION_MARGIN, ti) = 0; EF(c, F_HEALTH, ti) = 1;
            EF(c, F_THETA, ti) = -100; EF(c, F_CLIMBER_SPAWN_X, ti) = 0;
            EI(c, F_TYPE, ti) = TRAIL; EI(c, F_IMAGE_TYPE, ti) = TRAIL; EI(c, F_IMAGE_THEME, ti) = 0;
            EI(c, F_RENDER_Z, ti) = 0; EI(c, F_LIFE_TIME, ti) = 0; EI(c, F_EXPIRE_TIME, ti) = 8;
            EI(c, F_FIRE_TIME, ti) = -1; EI(c, F_SPAWN_TIME, ti) = -1; EI(c, F_FLAGS, ti) = EF_AUTO_ERASE;
            EI(c, F_IMAGE_TYPE, i) = c.s.cur_time / 5 % 2 == 0 ? CR_ENEMY1 : CR_ENEMY2;
            int fl = EI(c, F_FLAGS, i);
            if (EF(c, F_VX, i) > 0) fl |= EF_REFLECTED;
            else fl &= ~EF_REFLECTED;
            EI(c, F_FLAGS, i) = fl;
        } else if (t == CR_SAW) {
            EI(c, F_IMAGE_TYPE, i) = c.s.cur_time % 2 == 0 ? CR_SAW : CR_SAW2;
        }
        above += __popcll(em);
    }
    if (total_enemies == 0) { // saws still animate when there is no enemy
        for (int base = 0; base < n; base += 64) {
            int i = base + LANE;
            if (i < n && EI(c, F_TYPE, i) == CR_SAW) EI(c, F_IMAGE_TYPE, i) = c.s.cur_time % 2 == 0 ? CR_SAW : CR_SAW2;
        }
    }
    c.s.num_ents = n + total_enemies;
    wave_sync();
    c.s.last_agent_y = c.s.agent_erased ? c.gp->ghost_y : EF(c, F_Y, 0);
}

// bigfish.cpp:84: (FISH_MAX_R - FISH_MIN_R) * pow(rand01(), 1.4) + FISH_MIN_R -- pow(float, double)
// resolves to the double pow; checked against the C library's pow for
// every value rand01() can return (tests/test_gpu_libm.py).
DEV float bigfish_fish_radius(float u) {
    return (float)((double)(BF_FISH_MAX_R - BF_FISH_MIN_R) * pow((double)u, 1.4) + (double)BF_FISH_MIN_R);
}

DEV void bigfish_step_tail(Ctx &c, uint32_t *rg) { // bigfish.cpp:80-106
    if (rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), 10) == 1) {
        float ent_r = bigfish_fish_radius(rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)));
        float ent_y = rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)) * (c.s.main_height - 2 * ent_r);
        float moves_right = (double)rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)) < .5 ? 1.0f : 0.0f;
        float ent_vx = (float)((.15 + (double)rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)) * .25) *
                               (moves_right != 0 ? 1 : -1));
        float ent_x = moves_right != 0 ? -1 * ent_r : c.s.main_width + ent_r;
        int theme = rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), c.d.num_themes[PG_GAME_BIGFISH * 100 + BF_FISH]); // choose_random_theme
        float ry = ent_r / aspect_ratio<PG_GAME_BIGFISH>(c, BF_FISH, theme);           // match_aspect_ratio
        int i = append_entity(c, ent_x, ent_y, ent_vx, 0, ent_r, ry, BF_FISH);
        if (i >= 0) {
            EI(c, F_IMAGE_THEME, i) = theme;
            if (moves_right == 0) EI(c, F_FLAGS, i) = EF_AUTO_ERASE | EF_REFLECTED;
        }
    }
    if (c.s.fish_eaten >= BF_FISH_QUOTA) {
        c.s.sd_done = 1;
        c.s.sd_reward += 10; // COMPLETION_BONUS
        c.s.sd_level_complete = 1;
    }
    if (c.s.action_vx > 0) flag_reflected(c, 0, false);
    if (c.s.action_vx < 0) flag_reflected(c, 0, true);
}

DEV void maze_step_tail(Ctx &c) { // maze.cpp:113-131
    if (c.s.action_vx > 0) flag_reflected(c, 0, true);
    if (c.s.action_vx < 0) flag_reflected(c, 0, false);
    int ix = (int)EF(c, F_X, 0);
    int iy = (int)EF(c, F_Y, 0);
    if (get_obj(c, ix, iy) == MZ_GOAL) {
        // set_obj(ix, iy, SPACE): the HBM grid, its int8 mirror and this step's LDS copy
        int cell = iy * c.s.main_width + ix;
        if (LANE == 0) {
            c.d.grid[(size_t)c.env * PG_GRID_MAX + cell] = SPACE;
            c.d.grid8[(size_t)c.env * PG_GRID_MAX + cell] = (int8_t)SPACE;
            c.grid8[cell] = (int8_t)SPACE;
            if (cell < PG_LATENT_GRID) c.d.latent[(size_t)c.env * PG_LATENT_N + 2 + cell] = SPACE;
        }
        wave_sync();
        c.s.sd_reward += 10.0f; // REWARD
        c.s.sd_level_complete = 1;
    }
    c.s.sd_done = c.s.sd_reward > 0;
    if (LANE == 0) { // latent agent_pos = int(agent->x), int(agent->y) (maze.cpp:144-145)
        c.d.latent[(size_t)c.env * PG_LATENT_N + 2 + PG_LATENT_GRID] = ix;
        c.d.latent[(size_t)c.env * PG_LATENT_N + 3 + PG_LATENT_GRID] = iy;
    }
}

DEV void climber_step_tail(Ctx &c) { // climber.cpp:320-346
    if (c.s.action_vx > 0) flag_reflected(c, 0, false);
    if (c.s.action_vx < 0) flag_reflected(c, 0, true);
    const int n = c.s.num_ents;
    for (int base = 0; base < n; base += 64) { // per-entity, order-free
        int i = base + LANE;
        if (i < n && EI(c, F_TYPE, i) == CL_ENEMY) {
            float x = EF(c, F_X, i), vx = EF(c, F_VX, i), sx = EF(c, F_CLIMBER_SPAWN_X, i);
            if (x > sx + 4.0f) vx = -1 * fabsf(vx); // PATROL_RANGE
            else if (x < sx - 4.0f) vx = fabsf(vx);
            EF(c, F_VX, i) = vx;
            EI(c, F_IMAGE_TYPE, i) = c.s.cur_time / 5 % 2 == 0 ? CL_ENEMY1 : CL_ENEMY2;
            int fl = EI(c, F_FLAGS, i);
            EI(c, F_FLAGS, i) = vx < 0 ? (fl | EF_REFLECTED) : (fl & ~EF_REFLECTED);
        }
    }
    wave_sync();
    if (c.s.coin_quota == c.s.coins_collected) {
        c.s.sd_done = 1;
        c.s.sd_reward += 10.0f; // COMPLETION_BONUS
        c.s.sd_level_complete = 1;
    }
}

DEV void heist_step_tail(Ctx &c) { // heist.cpp:205-209: agent->face_direction(action_vx, action_vy)
    if (c.s.agent_erased) return;
    float dx = c.s.action_vx, dy = c.s.action_vy;
    if (dx != 0 || dy != 0) EF(c, F_ROTATION, 0) = c.d.rot_angles[((int)dx + 1) * 3 + ((int)dy + 1)];
}

// ------------------------------------------------------------------ miner (games/miner.cpp, fork-modified)
// The grid lives in LDS (int8, c.grid8) for the whole step and is written back once at the end;
// has_moved is an LDS byte map (c.moved).
DEV int mn_get(Ctx &c, int idx) { // get_obj(int idx) (basic-abstract-game.cpp:194-199)
    if (!(0 <= idx && idx < c.s.main_width * c.s.main_height)) return c.s.out_of_bounds_object;
    return c.grid8[idx];
}
// c.moved: bit 0 = has_moved (miner.cpp), bit 1 = the cell was written this step (grid write-back)
DEV void mn_set(Ctx &c, int idx, int v) {
    if (LANE == 0) {
        c.grid8[idx] = (int8_t)v;
        c.moved[idx] |= 2;
    }
    wave_sync();
}
DEV void mn_mark(Ctx &c, int idx) {
    if (LANE == 0) c.moved[idx] |= 1;
    wave_sync();
}
DEV float mn_ax(Ctx &c) { return c.s.agent_erased ? c.gp->ghost_x : EF(c, F_X, 0); }
DEV float mn_ay(Ctx &c) { return c.s.agent_erased ? c.gp->ghost_y : EF(c, F_Y, 0); }
DEV int mn_agent_index(Ctx &c) { return (int)mn_ay(c) * c.s.main_width + (int)mn_ax(c); } // miner.cpp:98-100
DEV int mn_moving(int t) { return t == MN_DIAMOND ? MN_MOVING_DIAMOND : (t == MN_BOULDER ? MN_MOVING_BOULDER : t); }
DEV bool mn_is_moving(int t) { return t == MN_MOVING_BOULDER || t == MN_MOVING_DIAMOND; }
DEV int mn_stationary(int t) { return t == MN_MOVING_DIAMOND ? MN_DIAMOND : (t == MN_MOVING_BOULDER ? MN_BOULDER : t); }
DEV bool mn_is_round(int t) {
    return t == MN_BOULDER || t == MN_MOVING_BOULDER || t == MN_DIAMOND || t == MN_MOVING_DIAMOND;
}
DEV bool mn_is_free(Ctx &c, int idx, int agent_idx) { return mn_get(c, idx) == SPACE && agent_idx != idx; }

// entities.erase(entities.begin()) -- entities[0] is the agent; its shared_ptr lives on (ghost)
DEV void mn_erase_agent(Ctx &c) {
    if (c.s.agent_erased || c.s.num_ents <= 0) {
        c.s.error = PG_ERR_BAD_OPTION;
        return;
    }
    c.s.agent_erased = 1;
    c.gp->ghost_x = EF(c, F_X, 0); c.gp->ghost_y = EF(c, F_Y, 0); c.gp->ghost_vx = EF(c, F_VX, 0);
    c.gp->ghost_vy = EF(c, F_VY, 0); c.gp->ghost_rx = EF(c, F_RX, 0); c.gp->ghost_ry = EF(c, F_RY, 0);
    const int n = c.s.num_ents;
    for (int base = 1; base < n; base += 64) { // order-preserving shift down by one
        int i = base + LANE;
        Ent e;
        if (i < n) load_ent(c, i, e);
        wave_sync();
        if (i < n) store_ent(c, i - 1, e);
        wave_sync();
    }
    c.s.num_ents = n - 1;
}

// move_cell (miner.cpp:310-346) of one cell, uniform.  agent_idx: the agent's cell, fixed for the
// pass (the agent does not move while the cells do; an erased agent's ghost keeps its position)
DEV void mn_move_cell(Ctx &c, int idx, int agent_idx) {
    const int w = c.s.main_width;
    const bool current_moved = (c.moved[idx] & 1) != 0;
    const int obj = mn_get(c, idx);
    const int obj_x = idx % w;
    const int stat_type = mn_stationary(obj);
    // `BOULDER || DIAMOND && !moved`: && binds tighter
    if (!(stat_type == MN_BOULDER || (stat_type == MN_DIAMOND && !current_moved))) return;
    const int below_idx = idx - w;
    const int below_object = mn_get(c, below_idx);
    const bool agent_is_below = agent_idx == below_idx;
    if (below_object == SPACE && !agent_is_below) {
        const int two_below_obj = mn_get(c, below_idx - w);
        mn_set(c, idx, SPACE);
        mn_set(c, below_idx, two_below_obj == SPACE ? mn_moving(obj) : stat_type);
        mn_mark(c, below_idx);
    } else if (agent_is_below && mn_is_moving(obj)) {
        c.s.died = 1;
        mn_erase_agent(c);
        mn_set(c, below_idx, MN_DEAD_PLAYER);
    } else if (mn_is_round(below_object) && obj_x > 0 && mn_is_free(c, idx - 1, agent_idx) &&
               mn_is_free(c, idx - w - 1, agent_idx)) {
        mn_set(c, idx, SPACE);
        mn_set(c, idx - 1, stat_type);
        mn_mark(c, idx - 1);
    } else if (mn_is_round(below_object) && obj_x < w - 1 && mn_is_free(c, idx + 1, agent_idx) &&
               mn_is_free(c, idx - w + 1, agent_idx)) {
        mn_set(c, idx, SPACE);
        mn_set(c, idx + 1, stat_type);
        mn_mark(c, idx + 1);
    } else {
        mn_set(c, idx, stat_type);
    }
}

// move_cell over rows [y0, y1), x ascending.  Only BOULDER / DIAMOND-like cells act, so a row is
// a ballot (w <= 35 < 64 lanes) for the next acting cell at or right of the cursor, re-taken
// after every move (a slide to x + 1 makes that cell act next, as in the reference's loop).  A
// resting object -- stationary, on something neither free nor round (or on the agent's free cell)
// -- takes move_cell's last branch, which rewrites the cell with its own value: it is skipped.
// The cell below a row is final once the row's pass starts (only that cell's own fall writes it).
DEV void mn_move_rows(Ctx &c, int y0, int y1) {
    const int w = c.s.main_width;
    const int agent_idx = mn_agent_index(c);
    for (int y = y0; y < y1; y++) {
        int xc = 0;
        while (xc < w) {
            const int x = xc + LANE;
            bool act = false;
            if (LANE < w - xc) {
                const int idx = x + w * y;
                const int obj = c.grid8[idx];
                const int st = mn_stationary(obj);
                act = st == MN_BOULDER || (st == MN_DIAMOND && !(c.moved[idx] & 1));
                if (act && obj == st) {
                    const int below = mn_get(c, idx - w);
                    if (below == SPACE ? agent_idx == idx - w : !mn_is_round(below)) act = false;
                }
            }
            const unsigned long long b = ballot(act);
            if (!b) break;
            const int xa = xc + __ffsll((long long)b) - 1;
            mn_move_cell(c, xa + w * y, agent_idx);
            xc = xa + 1;
        }
    }
}

DEV void miner_pre_step(Ctx &c) {
    const int cells = c.s.main_width * c.s.main_height;
    if (!c.grid8_ok || cells > PG_GRID_MAX) {
        c.s.error = PG_ERR_GRID;
        return;
    }
    for (int i = LANE; i < cells; i += 64) c.moved[i] = 0;
    wave_sync();
    // for (int y = 0; y <= agent->y; ++y): int y against the float y
    int y1 = 0;
    while (y1 < c.s.main_height && (float)y1 <= mn_ay(c)) y1++;
    mn_move_rows(c, 0, y1);
}

DEV void miner_step_tail(Ctx &c) { // miner.cpp:262-307
    const int w = c.s.main_width, h = c.s.main_height;
    if (c.s.died) {
        c.s.sd_done = 1;
    } else {
        if (c.s.action_vx > 0) flag_reflected(c, 0, false);
        if (c.s.action_vx < 0) flag_reflected(c, 0, true);
        // handle_push (miner.cpp:262-281)
        const int agent_idx = mn_agent_index(c);
        const int agentx = agent_idx % w;
        const float avx = EF(c, F_VX, 0);
        if (c.s.action_vx == 1 && (avx == 0) && (agentx < w - 2) && mn_get(c, agent_idx + 1) == MN_BOULDER &&
            mn_get(c, agent_idx + 2) == SPACE) {
            mn_set(c, agent_idx + 1, SPACE);
            mn_set(c, agent_idx + 2, MN_BOULDER);
            mn_mark(c, agent_idx + 2);
            EF(c, F_X, 0) = EF(c, F_X, 0) + 1;
        } else if (c.s.action_vx == -1 && (avx == 0) && (agentx > 1) && mn_get(c, agent_idx - 1) == MN_BOULDER &&
                   mn_get(c, agent_idx - 2) == SPACE) {
            mn_set(c, agent_idx - 1, SPACE);
            mn_set(c, agent_idx - 2, MN_BOULDER);
            mn_mark(c, agent_idx - 2);
            EF(c, F_X, 0) = EF(c, F_X, 0) - 1;
        }
        wave_sync();
        const int ax = (int)EF(c, F_X, 0), ay = (int)EF(c, F_Y, 0);
        const int agent_obj = mn_stationary(get_obj(c, ax, ay));
        if (agent_obj == MN_DIAMOND) c.s.sd_reward += 1.0f; // DIAMOND_REWARD
        if (agent_obj == MN_DIRT || agent_obj == MN_MUD || agent_obj == MN_DIAMOND) {
            if (0 <= ax && ax < w && 0 <= ay && ay < h) mn_set(c, ay * w + ax, SPACE);
            else c.s.error = PG_ERR_GRID;
        }
        // for (int y = agent->y + 1; y < main_height; ++y)
        mn_move_rows(c, (int)(mn_ay(c) + 1), h);
        int diamonds = 0; // count_diamonds (miner.cpp:348-356)
        for (int base = 0; base < c.s.main_area; base += 64) {
            int i = base + LANE;
            diamonds += __popcll(ballot(i < c.s.main_area && mn_stationary(mn_get(c, i)) == MN_DIAMOND));
        }
        c.s.diamonds_remaining = diamonds;
    }
    // write the grid back: HBM int16 + its int8 mirror + the fork's latent state (miner.cpp:363-396),
    // the cells written this step only (the three copies agree with the LDS grid everywhere else)
    const int cells = w * h;
    int16_t *g = c.d.grid + (size_t)c.env * PG_GRID_MAX;
    int8_t *g8 = c.d.grid8 + (size_t)c.env * PG_GRID_MAX;
    int32_t *lat = c.d.latent + (size_t)c.env * PG_LATENT_N;
    if (c.s.error == 0)
        for (int i = LANE; i < cells; i += 64) {
            if (!(c.moved[i] & 2)) continue;
            const int v = c.grid8[i];
            g[i] = (int16_t)v;
            g8[i] = (int8_t)v;
            if (i < PG_LATENT_GRID) lat[2 + i] = v;
        }
    int ex = 0, ey = 0;
    for (int base = 0; base < c.s.num_ents; base += 64) { // the first EXIT entity
        int i = base + LANE;
        unsigned long long b = ballot(i < c.s.num_ents && EI(c, F_TYPE, i) == MN_EXIT);
        if (b) {
            int e = base + __ffsll((long long)b) - 1;
            ex = (int)EF(c, F_X, e);
            ey = (int)EF(c, F_Y, e);
            break;
        }
    }
    if (LANE == 0) {
        lat[0] = w;
        lat[1] = h;
        lat[2 + PG_LATENT_GRID] = (int)mn_ax(c);
        lat[3 + PG_LATENT_GRID] = (int)mn_ay(c);
        lat[4 + PG_LATENT_GRID] = ex;
        lat[5 + PG_LATENT_GRID] = ey;
    }
}

// has_any_collision(e, 0) (basic-abstract-game.cpp:1123-1133) of a not-yet-added entity
DEV bool any_collision(Ctx &c, float x, float y, float rx, float ry) {
    bool hit = false;
    for (int base = 0; base < c.s.num_ents; base += 64) {
        int i = base + LANE;
        if (i < c.s.num_ents && !(EI(c, F_FLAGS, i) & EF_AVOIDS)) {
            float tx = (rx + EF(c, F_RX, i)) + 0.0f, ty = (ry + EF(c, F_RY, i)) + 0.0f;
            if ((fabsf(x - EF(c, F_X, i)) < tx) && (fabsf(y - EF(c, F_Y, i)) < ty)) hit = true;
        }
    }
    return ballot(hit) != 0;
}

// spawn_entities (leaper.cpp:184-218)
DEV void lp_spawn_entities(Ctx &c, uint32_t *rg) {
    for (int lane = 0; lane < c.s.num_road_lanes; lane++) {
        const float speed = c.d.envs[c.env].road_lane_speeds[lane]; // read-only here (HBM: no dynamic index into c.s)
        const float spawn_prob = (float)(fabs((double)speed) / 6.0);
        if (rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)) < spawn_prob) {
            const float x = speed > 0 ? (-1 * LP_MONSTER_RADIUS) : (c.s.main_width + LP_MONSTER_RADIUS);
            const float y = (float)(c.s.bottom_road_y + lane + 0.5);
            const int theme = rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), c.d.num_themes[PG_GAME_LEAPER * 100 + LP_CAR]);
            if (!any_collision(c, x, y, 2 * LP_MONSTER_RADIUS, LP_MONSTER_RADIUS)) {
                int i = append_entity(c, x, y, speed, 0, 2 * LP_MONSTER_RADIUS, LP_MONSTER_RADIUS, LP_CAR);
                if (i >= 0) {
                    EI(c, F_IMAGE_THEME, i) = theme;
                    if (speed < 0) EF(c, F_ROTATION, i) = PI_F;
                }
            }
            wave_sync();
        }
    }
    for (int lane = 0; lane < c.s.num_water_lanes; lane++) {
        const float speed = c.d.envs[c.env].water_lane_speeds[lane];
        const float spawn_prob = (float)(fabs((double)speed) / 2.0);
        if (rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)) < spawn_prob) {
            const float x = speed > 0 ? (-1 * LP_LOG_RADIUS) : (c.s.main_width + LP_LOG_RADIUS);
            const float y = (float)(c.s.bottom_water_y + lane + 0.5);
            if (!any_collision(c, x, y, LP_LOG_RADIUS, LP_LOG_RADIUS))
                append_entity(c, x, y, speed, 0, LP_LOG_RADIUS, LP_LOG_RADIUS, LP_LOG);
            wave_sync();
        }
    }
}

DEV void leaper_pre_step(Ctx &c) { // leaper.cpp:253-256 (frog animation)
    const int th = EI(c, F_IMAGE_THEME, 0);
    wave_sync();
    if (th >= 1) EI(c, F_IMAGE_THEME, 0) = (th + 1) % LP_NSTEP;
    wave_sync();
}

DEV void leaper_step_tail(Ctx &c, uint32_t *rg) { // leaper.cpp:258-287
    lp_spawn_entities(c, rg);
    const bool gh = c.s.agent_erased; // the reference's `agent` outlives its erase
    const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
    const float arx = gh ? c.gp->ghost_rx : EF(c, F_RX, 0), ary = gh ? c.gp->ghost_ry : EF(c, F_RY, 0);
    const float avx = gh ? c.gp->ghost_vx : EF(c, F_VX, 0), avy = gh ? c.gp->ghost_vy : EF(c, F_VY, 0);
    // the last LOG (list order) the agent stands on gives log_vx
    const float margin = -1 * arx;
    int last = -1;
    for (int base = 0; base < c.s.num_ents; base += 64) {
        int i = base + LANE;
        bool hit = false;
        if (i < c.s.num_ents && EI(c, F_TYPE, i) == LP_LOG) {
            float tx = (arx + EF(c, F_RX, i)) + margin, ty = (ary + EF(c, F_RY, i)) + margin;
            hit = (fabsf(ax - EF(c, F_X, i)) < tx) && (fabsf(ay - EF(c, F_Y, i)) < ty);
        }
        unsigned long long b = ballot(hit);
        if (b) last = base + top_bit(b);
    }
    const bool standing_on_log = last >= 0;
    const float log_vx = standing_on_log ? EF(c, F_VX, last) : 0.0f;
    if (get_obj(c, (int)ax, (int)ay) == LP_WATER) {
        if (!standing_on_log && avx == 0 && avy == 0) c.s.sd_done = 1;
    }
    float nx = ax;
    if (standing_on_log) nx = ax + log_vx;
    wave_sync();
    if (standing_on_log) {
        if (gh) c.gp->ghost_x = nx;
        else EF(c, F_X, 0) = nx;
    }
    if (is_out_of_bounds(c, nx, ay, arx, ary)) c.s.sd_done = 1;
    wave_sync();
}

// chaser (chaser.cpp:286-376).  The reference's free_cells / is_space_vec are the non-MAZE_WALL
// cells of the grid in index order (walls never change after the reset), read from the grid.
DEV int ch_grid(Ctx &c, int idx) { return c.G[idx]; } // int16 grid in HBM (ORB = 1002 exceeds the int8 mirror)
DEV int ch_to_grid_idx(Ctx &c, int x, int y) {
    if (!(0 <= x && x < c.s.main_width && 0 <= y && y < c.s.main_height)) return -2; // INVALID_IDX
    return y * c.s.main_width + x;
}
// n-th (0-based) non-wall cell in index order
DEV int ch_nth_free(Ctx &c, int n) {
    const int cells = c.s.main_width * c.s.main_height;
    int seen = 0;
    for (int base = 0; base < cells; base += 64) {
        int i = base + LANE;
        bool f = i < cells && ch_grid(c, i) != CH_MAZE_WALL;
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
DEV int ch_num_free(Ctx &c) {
    const int cells = c.s.main_width * c.s.main_height;
    int cnt = 0;
    for (int base = 0; base < cells; base += 64) {
        int i = base + LANE;
        cnt += __popcll(ballot(i < cells && ch_grid(c, i) != CH_MAZE_WALL));
    }
    return cnt;
}
DEV void ch_spawn_egg(Ctx &c, int cell) { // spawn_egg (:259-262)
    const int md = c.s.maze_dim;
    int i = append_entity(c, (float)((cell % md) + .5), (float)((cell / md) + .5), 0, 0, .5f, .5f, CH_ENEMY_EGG);
    if (i >= 0) EF(c, F_HEALTH, i) = (float)c.s.egg_timeout;
    wave_sync();
}

DEV void chaser_step_tail(Ctx &c) {
    const int n = c.s.num_ents, w = c.s.main_width;
    const bool can_eat = c.s.cur_time - c.s.eat_time < c.s.eat_timeout;
    const float default_enemy_speed = .5;
    const float vscale = can_eat ? (default_enemy_speed * .5f) : default_enemy_speed;
    const float ax = c.s.agent_erased ? c.gp->ghost_x : EF(c, F_X, 0);
    const float ay = c.s.agent_erased ? c.gp->ghost_y : EF(c, F_Y, 0);
    const int agent_idx = ch_to_grid_idx(c, (int)ax, (int)ay);
    const bool be_agressive = c.s.step_rand_int % 2 == 0;
    const int dist_scale = can_eat ? -1 : 1;
    // every entity of the reverse loop is independent: lane-parallel, hatchlings appended in
    // the loop's (descending) order
    int num_enemies = 0, hatch_total = 0;
    for (int base = 0; base < n; base += 64) {
        int i = base + LANE;
        int t = i < n ? EI(c, F_TYPE, i) : -1;
        num_enemies += __popcll(ballot(t == CH_ENEMY_EGG || t == CH_ENEMY));
        bool hatch = false;
        if (t == CH_ENEMY_EGG) {
            float h = EF(c, F_HEALTH, i) - 1;
            EF(c, F_HEALTH, i) = h;
            if (h == 0) {
                hatch = true;
                EI(c, F_FLAGS, i) = EI(c, F_FLAGS, i) | EF_WILL_ERASE;
            }
        } else if (t == CH_ENEMY) {
            const float evx = EF(c, F_VX, i), evy = EF(c, F_VY, i);
            const float x = (float)(EF(c, F_X, i) - .5);
            const float y = (float)(EF(c, F_Y, i) - .5);
            const int enemy_idx = ch_to_grid_idx(c, (int)x, (int)y);
            const bool is_at_junction = fabs((double)x - round((double)x)) + fabs((double)y - round((double)y)) < .01;
            if ((evx == 0 && evy == 0) || is_at_junction) {
                const int prev_idx = ch_to_grid_idx(c, (int)(x - dsign(evx)), (int)(y - dsign(evy)));
                const int ex = enemy_idx % w, ey = enemy_idx / w;
                const int ox[4] = {-1, 0, 0, 1}, oy[4] = {0, -1, 1, 0}; // get_adjacent order (:269-284)
                int cand[4];
                bool ok[4];
                int min_dist = 2 * w;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    cand[k] = ch_to_grid_idx(c, ex + ox[k], ey + oy[k]);
                    ok[k] = cand[k] != -2 && ch_grid(c, cand[k]) != CH_MAZE_WALL && cand[k] != prev_idx;
                }
                int md[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    md[k] = (abs((cand[k] % w) - (agent_idx % w)) + abs((cand[k] / w) - (agent_idx / w))) * dist_scale;
                    if (ok[k] && be_agressive && md[k] < min_dist) min_dist = md[k];
                }
                int cnt = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (ok[k] && be_agressive && md[k] != min_dist) ok[k] = false;
                    cnt += ok[k];
                }
                if (cnt == 0) {
                    c.s.error = PG_ERR_GRID; // the reference divides by zero here
                } else {
                    int pick = (int)((unsigned)c.s.step_rand_int % (unsigned)cnt), neighbor = -1;
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        if (ok[k] && pick-- == 0) neighbor = cand[k];
                    const int nx = neighbor % w, ny = neighbor / w;
                    EF(c, F_VX, i) = (nx - x) * vscale;
                    EF(c, F_VY, i) = (ny - y) * vscale;
                }
            }
        }
        hatch_total += __popcll(ballot(hatch));
    }
    if (ballot(c.s.error != 0)) c.s.error = PG_ERR_GRID;
    wave_sync();
    // spawn_child(egg, ENEMY, .5) for the hatched eggs, highest index first
    if (hatch_total > 0) {
        if (n + hatch_total > PG_CAP) {
            c.s.error = PG_ERR_ENTITY_OVERFLOW;
        } else {
            int done = 0;
            for (int base = ((n - 1) & ~63); base >= 0; base -= 64) {
                int i = base + LANE;
                bool hatch = i < n && EI(c, F_TYPE, i) == CH_ENEMY_EGG && (EI(c, F_FLAGS, i) & EF_WILL_ERASE) &&
                             EF(c, F_HEALTH, i) == 0;
                unsigned long long b = ballot(hatch);
                float hx = 0, hy = 0;
                if (hatch) { hx = EF(c, F_X, i); hy = EF(c, F_Y, i); }
                wave_sync();
                if (hatch) {
                    // rank among this chunk's hatchlings, counted from the top
                    int rank = done + __popcll(b >> LANE) - 1;
                    int slot = n + rank;
                    EF(c, F_X, slot) = hx; EF(c, F_Y, slot) = hy; EF(c, F_VX, slot) = 0; EF(c, F_VY, slot) = 0;
                    EF(c, F_RX, slot) = .5f; EF(c, F_RY, slot) = .5f; EF(c, F_ROTATION, slot) = 0; EF(c, F_VROT, slot) = 0;
                    EF(c, F_ALPHA, slot) = 1.0f; EF(c, F_ALPHA_DECAY, slot) = 1.0f; EF(c, F_GROW_RATE, slot) = 1.0f;
                    EF(c, F_FRICTION, slot) = 1; EF(c, F_COLLISION_MARGIN, slot) = 0; EF(c, F_HEALTH, slot) = 1;
                    EF(c, F_THETA, slot) = -100; EF(c, F_CLIMBER_SPAWN_X, slot) = 0;
                    EI(c, F_TYPE, slot) = CH_ENEMY; EI(c, F_IMAGE_TYPE, slot) = CH_ENEMY; EI(c, F_IMAGE_THEME, slot) = 0;
                    EI(c, F_RENDER_Z, slot) = 0; EI(c, F_LIFE_TIME, slot) = 0; EI(c, F_EXPIRE_TIME, slot) = -1;
                    EI(c, F_FIRE_TIME, slot) = -1; EI(c, F_SPAWN_TIME, slot) = -1;
                    EI(c, F_FLAGS, slot) = EF_AUTO_ERASE | EF_SMART_STEP;
                }
                done += __popcll(b);
            }
            c.s.num_ents = n + hatch_total;
        }
    }
    wave_sync();
    if (num_enemies < c.s.total_enemies) {
        const int nfree = ch_num_free(c);
        if (nfree <= 0) {
            c.s.error = PG_ERR_GRID;
        } else {
            const int sel = (int)((unsigned)c.s.step_rand_int % (unsigned)nfree);
            ch_spawn_egg(c, ch_nth_free(c, sel));
        }
    }
    // get_agent_index (:176-178) and the orb under the agent
    const int aidx = (int)ay * w + (int)ax;
    const int cells = w * c.s.main_height;
    if (0 <= aidx && aidx < cells && ch_grid(c, aidx) == CH_ORB) {
        wave_sync();
        if (LANE == 0) c.d.grid[(size_t)c.env * PG_GRID_MAX + aidx] = SPACE;
        wave_sync();
        c.s.sd_reward += 0.04f; // ORB_REWARD
        c.s.orbs_collected += 1;
    }
    if (c.s.orbs_collected == c.s.total_orbs) {
        c.s.sd_reward += 10.0f; // COMPLETION_BONUS
        c.s.sd_level_complete = 1;
        c.s.sd_done = 1;
    }
    wave_sync();
}

// ------------------------------------------------------------------ dodgeball (dodgeball.cpp:226-238, 371-444)
DEV void db_choose_vel(Ctx &c, uint32_t *rg, int i) { // :226-238
    const float vel = DB_ENEMY_VEL * (rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), 2) * 2 - 1);
    if (rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), 2) == 0) {
        EF(c, F_VX, i) = vel;
        EF(c, F_VY, i) = 0;
    } else {
        EF(c, F_VY, i) = vel;
        EF(c, F_VX, i) = 0;
    }
    EI(c, F_SPAWN_TIME, i) = rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), 50) + 25;
}

DEV void db_fire_ball(Ctx &c, uint32_t *rg, int i, float vx, float vy) { // :371-376
    const float ex = EF(c, F_X, i), ey = EF(c, F_Y, i);
    wave_sync();
    const int b = append_entity(c, ex, ey, vx * c.s.db_ball_vscale, vy * c.s.db_ball_vscale, c.s.db_ball_r, c.s.db_ball_r,
                                DB_ENEMY_BALL);
    const int ft = c.s.cur_time + rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), 4);
    EI(c, F_FIRE_TIME, i) = ft;
    if (b >= 0) {
        EF(c, F_VROT, b) = PI_F * 0.23f; // BALL_V_ROT
        EI(c, F_EXPIRE_TIME, b) = 50;
    }
    wave_sync();
}

DEV void dodgeball_step_tail(Ctx &c, uint32_t *rg) { // :378-444
    const float vx = (float)(c.s.last_move_action / 3 - 1);
    const float vy = (float)(c.s.last_move_action % 3 - 1);
    const bool gh = c.s.agent_erased;
    if (!gh) EF(c, F_ROTATION, 0) = face_rotation(vx, vy, EF(c, F_ROTATION, 0));
    if (c.s.special_action == 1 && (c.s.cur_time - c.s.last_fire_time) >= 7) {
        const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
        wave_sync();
        const int b = append_entity(c, ax, ay, vx * c.s.db_ball_vscale, vy * c.s.db_ball_vscale, c.s.db_ball_r,
                                    c.s.db_ball_r, DB_PLAYER_BALL);
        if (b >= 0) {
            EI(c, F_FLAGS, b) = EF_AUTO_ERASE | EF_COLLIDES;
            EI(c, F_EXPIRE_TIME, b) = 50;
            EF(c, F_VROT, b) = PI_F * 0.23f;
        }
        c.s.last_fire_time = c.s.cur_time;
    }
    wave_sync();
    const int n0 = c.s.num_ents;
    // balls: each flags only itself (lane-parallel)
    for (int base = 0; base < n0; base += 64) {
        const int i = base + LANE;
        if (i < n0) {
            const int t = EI(c, F_TYPE, i);
            if (t == DB_PLAYER_BALL || t == DB_ENEMY_BALL) {
                const float x = EF(c, F_X, i), y = EF(c, F_Y, i), rx = EF(c, F_RX, i), ry = EF(c, F_RY, i);
                if (x < rx || x > (c.s.main_width - rx) || y < ry || y > (c.s.main_height - ry))
                    EI(c, F_FLAGS, i) = EI(c, F_FLAGS, i) | EF_WILL_ERASE;
            }
        }
    }
    wave_sync();
    // enemies in the reference's descending order (random draws in order)
    int num_enemies = 0;
    int upper = n0;
    while (upper > 0) {
        int m = -1;
        for (int base = (upper - 1) & ~63; base >= 0; base -= 64) {
            const int i = base + LANE;
            const unsigned long long b = ballot(i < upper && EI(c, F_TYPE, i) == DB_ENEMY);
            if (b) {
                m = base + top_bit(b);
                break;
            }
        }
        if (m < 0) break;
        upper = m;
        num_enemies++;
        const int st = EI(c, F_SPAWN_TIME, m);
        wave_sync();
        if (st == 0) db_choose_vel(c, rg, m);
        else EI(c, F_SPAWN_TIME, m) = st - 1;
        wave_sync();
        if ((c.s.cur_time - EI(c, F_FIRE_TIME, m)) >= c.s.enemy_fire_delay) {
            const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
            const float ex = EF(c, F_X, m), ey = EF(c, F_Y, m);
            const float dx = ex - ax, dy = ey - ay;
            const float bvelx = (float)(ex < ax ? 1 : -1);
            const float bvely = (float)(ey < ay ? 1 : -1);
            if (fabsf(dx) < 1) {
                db_fire_ball(c, rg, m, 0, bvely);
                EF(c, F_VX, m) = 0;
                EF(c, F_VY, m) = bvely * DB_ENEMY_VEL;
            } else if (fabsf(dy) < 1) {
                db_fire_ball(c, rg, m, bvelx, 0);
                EF(c, F_VX, m) = bvelx * DB_ENEMY_VEL;
                EF(c, F_VY, m) = 0;
            }
        }
        wave_sync();
        EF(c, F_ROTATION, m) = face_rotation(EF(c, F_VX, m), EF(c, F_VY, m), EF(c, F_ROTATION, m));
        wave_sync();
    }
    c.s.num_enemies = num_enemies;
    erase_if_needed(c);
}

// ------------------------------------------------------------------ plunder (plunder.cpp:194-241)
template <int G>
DEV float aspect_ratio(Ctx &c, int type, int theme);

DEV void plunder_step_tail(Ctx &c, uint32_t *rg) {
    auto &P = c.s.gs.pl;
    P.juice_left -= 0.0015f;
    if (rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds)) < P.spawn_prob) {
        const float ent_r = P.r_scale;
        const int lane = rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), P.num_lanes);
        const float ent_y = (float)((lane * .11 + .4) * (c.s.main_height / 2 - ent_r) + c.s.main_height / 2);
        const bool moves_right = (P.lane_dirs >> lane) & 1u;
        const float lv = lane == 0 ? P.lane_vels[0] : lane == 1 ? P.lane_vels[1] : lane == 2 ? P.lane_vels[2]
                       : lane == 3 ? P.lane_vels[3] : P.lane_vels[4];
        const float ent_vx = lv * (moves_right ? 1 : -1);
        const int k = rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), P.num_current_ship_types);
        const int theme = (int)((P.perm >> (4 * k)) & 15u);
        const float ent_ry = ent_r / aspect_ratio<PG_GAME_PLUNDER>(c, PL_SHIP, theme); // match_aspect_ratio
        const float ent_x = moves_right ? -1 * ent_r : (c.s.main_width + ent_r);
        // has_any_collision(ent) (:1123-1133), margin 0
        bool hit = false;
        for (int base = 0; base < c.s.num_ents; base += 64) {
            const int i = base + LANE;
            if (i < c.s.num_ents && !(EI(c, F_FLAGS, i) & EF_AVOIDS)) {
                const float tx = (ent_r + EF(c, F_RX, i)) + 0.0f, ty = (ent_ry + EF(c, F_RY, i)) + 0.0f;
                if ((fabsf(ent_x - EF(c, F_X, i)) < tx) && (fabsf(ent_y - EF(c, F_Y, i)) < ty)) hit = true;
            }
        }
        if (ballot(hit) == 0) {
            wave_sync();
            const int i = append_entity(c, ent_x, ent_y, ent_vx, 0, ent_r, ent_ry, PL_SHIP);
            if (i >= 0) {
                EI(c, F_IMAGE_THEME, i) = theme;
                if (!moves_right) EI(c, F_FLAGS, i) = EF_AUTO_ERASE | EF_REFLECTED;
            }
        }
        wave_sync();
    }
    const bool gh = c.s.agent_erased;
    if (c.s.special_action == 1 && (c.s.cur_time - c.s.last_fire_time) >= 3) {
        const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
        wave_sync();
        const int b = append_entity(c, ax, ay, 0, 1, .25f, .25f, PL_PLAYER_BULLET);
        if (b >= 0) {
            EI(c, F_FLAGS, b) = EF_AUTO_ERASE | EF_COLLIDES;
            EI(c, F_EXPIRE_TIME, b) = 50;
        }
        c.s.last_fire_time = c.s.cur_time;
        P.juice_left -= 0.02f;
    }
    if (P.juice_left <= 0) c.s.sd_done = 1;
    else if (P.juice_left >= 1) P.juice_left = 1;
    if (P.targets_hit >= P.target_quota) {
        c.s.sd_done = 1;
        c.s.sd_reward += 10.0f; // COMPLETION_BONUS
        c.s.sd_level_complete = 1;
    }
    wave_sync();
    if (gh) {
        if (c.gp->ghost_x < P.min_agent_x) c.gp->ghost_x = P.min_agent_x;
    } else if (EF(c, F_X, 0) < P.min_agent_x) {
        EF(c, F_X, 0) = P.min_agent_x;
    }
    wave_sync();
}

// ------------------------------------------------------------------ jumper (jumper.cpp:424-441)
DEV void jumper_step_tail(Ctx &c) {
    int fl = EI(c, F_FLAGS, 0);
    if (c.s.action_vx > 0) fl &= ~EF_REFLECTED;
    if (c.s.action_vx < 0) fl |= EF_REFLECTED;
    EI(c, F_FLAGS, 0) = fl;
    const float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), ary = EF(c, F_RY, 0);
    float vy = EF(c, F_VY, 0);
    const float vx = EF(c, F_VX, 0);
    wave_sync();
    if (fabs((double)vx) + fabs((double)vy) > .05) { // fabs of a float: the double C function
        const int t = append_entity(c, ax, (float)((double)ay - (double)ary * .5), 0, 0.01f, 0.3f, 0.2f, TRAIL);
        if (t >= 0) {
            EI(c, F_EXPIRE_TIME, t) = 8;
            EF(c, F_ALPHA, t) = .5f;
        }
        wave_sync();
    }
    if (vy > -2) {
        vy -= 0.15f;
        EF(c, F_VY, 0) = vy;
    }
    wave_sync();
}

// ------------------------------------------------------------------ caveflyer (caveflyer.cpp:289-324)
DEV void caveflyer_step_tail(Ctx &c) {
    if (c.s.special_action == 1) {
        const float arot = EF(c, F_ROTATION, 0), ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0);
        const float theta = -1 * arot + PI_F / 2;
        double sn, cs;
        pg_sincos_cr((double)theta, &sn, &cs);
        wave_sync();
        const int b = append_entity(c, ax, ay, (float)cs, (float)sn, 0.1f, 0.25f, CF_PLAYER_BULLET);
        if (b >= 0) {
            EI(c, F_EXPIRE_TIME, b) = 10;
            EF(c, F_ROTATION, b) = arot;
        }
        wave_sync();
    }
    // descending walk: enemies face their velocity (face_direction(vx, vy, -PI / 2)); a bullet
    // with a corner in a CAVEWALL goes away and leaves an explosion (appended in walk order)
    const int n = c.s.num_ents;
    for (int base = (n - 1) & ~63; base >= 0; base -= 64) {
        const int i = base + LANE;
        bool hit = false;
        float bx = 0, by = 0, br = 0;
        if (i < n) {
            const int t = EI(c, F_TYPE, i);
            if (t == CF_ENEMY) {
                const float vx = EF(c, F_VX, i), vy = EF(c, F_VY, i);
                if (vx != 0 || vy != 0) EF(c, F_ROTATION, i) = face_rotation(vx, vy, 0, -1 * PI_F / 2);
            } else if (t == CF_PLAYER_BULLET) {
                const float x = EF(c, F_X, i), y = EF(c, F_Y, i), rx = EF(c, F_RX, i), ry = EF(c, F_RY, i);
                bool wall = false;
#pragma unroll
                for (int a = 0; a < 2; a++)
#pragma unroll
                    for (int b = 0; b < 2; b++)
                        wall = wall || get_obj_from_floats(c, x + rx * (float)(2 * a - 1), y + ry * (float)(2 * b - 1)) == CF_CAVEWALL;
                if (wall) {
                    EI(c, F_FLAGS, i) = EI(c, F_FLAGS, i) | EF_WILL_ERASE;
                    hit = true;
                    bx = x;
                    by = y;
                    br = (float)(.5 * rx);
                }
            }
        }
        unsigned long long m = ballot(hit);
        wave_sync();
        while (m) {
            const int l = top_bit(m);
            m &= ~(1ull << l);
            const float ex = rlf(bx, l), ey = rlf(by, l), er = rlf(br, l);
            append_entity(c, ex, ey, 0, 0, er, er, EXPLOSION);
            wave_sync();
        }
    }
    erase_if_needed(c);
}

// ------------------------------------------------------------------ ninja (ninja.cpp:420-450)
DEV void ninja_step_tail(Ctx &c) {
    const bool gh = c.s.agent_erased;
    int fl = EI(c, F_FLAGS, 0);
    bool refl = (fl & EF_REFLECTED) != 0;
    if (!gh) {
        if (c.s.action_vx > 0) refl = false;
        if (c.s.action_vx < 0) refl = true;
        EI(c, F_FLAGS, 0) = refl ? (fl | EF_REFLECTED) : (fl & ~EF_REFLECTED);
    }
    wave_sync();
    if (c.s.special_action > 0 && (c.s.cur_time - c.s.last_fire_time) >= 3) {
        float theta = 0;
        const float bullet_vel = 1;
        if (c.s.special_action == 1) theta = 0;
        else if (c.s.special_action == 2) theta = PI_F / 4;
        else if (c.s.special_action == 3) theta = PI_F / 2;
        else if (c.s.special_action == 4) theta = -1 * PI_F / 4;
        if (refl) theta = PI_F - theta;
        double sn, cs;
        pg_sincos_cr((double)theta, &sn, &cs);
        const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
        wave_sync();
        const int b = append_entity(c, ax, ay, (float)(bullet_vel * cs), (float)(bullet_vel * sn), .25f, .25f,
                                    NJ_THROWING_STAR);
        if (b >= 0) {
            EI(c, F_FLAGS, b) = EF_AUTO_ERASE | EF_COLLIDES | EF_SMART_STEP;
            EI(c, F_EXPIRE_TIME, b) = 15;
        }
        c.s.last_fire_time = c.s.cur_time;
        wave_sync();
    }
}

// ------------------------------------------------------------------ bossfight (bossfight.cpp:252-392)
DEV void bf_boss_fire(Ctx &c, int boss, float bullet_r, float vel, float theta) { // :252-257
    double sn, cs;
    pg_sincos_cr((double)theta, &sn, &cs);
    const float bx = EF(c, F_X, boss), by = EF(c, F_Y, boss);
    wave_sync();
    const int e = append_entity(c, bx, by, (float)(vel * cs), (float)(vel * sn), bullet_r, bullet_r, BF_ENEMY_BULLET);
    if (e >= 0) {
        EI(c, F_IMAGE_THEME, e) = c.s.gs.bf.boss_laser_theme;
        EI(c, F_EXPIRE_TIME, e) = 50;
        EF(c, F_VROT, e) = PI_F / 8;
    }
    wave_sync();
}

DEV void bossfight_step_tail(Ctx &c, uint32_t *rg) {
    auto &B = c.s.gs.bf;
    const int boss = find_type(c, BF_BOSS), shields = find_type(c, BF_SHIELDS);
    if (boss < 0 || shields < 0) {
        c.s.error = PG_ERR_BAD_OPTION;
        return;
    }
    const float bx0 = EF(c, F_X, boss), by0 = EF(c, F_Y, boss);
    wave_sync();
    EF(c, F_X, shields) = bx0;
    EF(c, F_Y, shields) = by0;
    B.rand_pct = rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds));
    B.rand_fire_pct = rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds));
    B.rand_pct_x = rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds));
    B.rand_pct_y = rg_rand01_of(mt_next_global(rg, c.s.rg_mti, c.lds));
    if (B.curr_vel_timeout <= 0) {
        const float dest_x = B.rand_pct_x * (c.s.main_width - 2 * BF_BOSS_R) + BF_BOSS_R;
        const float dest_y = B.rand_pct_y * (c.s.main_height - 2 * BF_BOSS_R - BF_BOTTOM_MARGIN) + BF_BOSS_R + BF_BOTTOM_MARGIN;
        EF(c, F_VX, boss) = (dest_x - bx0) / BF_BOSS_VEL_TIMEOUT;
        EF(c, F_VY, boss) = (dest_y - by0) / BF_BOSS_VEL_TIMEOUT;
        B.curr_vel_timeout = BF_BOSS_VEL_TIMEOUT;
        if (B.time_to_swap > 0) {
            B.time_to_swap -= 1;
        } else {
            B.time_to_swap = B.shields_are_up ? 500 : B.invulnerable_duration; // vulnerable_duration = 500
            B.shields_are_up = !B.shields_are_up;
        }
    } else {
        B.curr_vel_timeout -= 1;
    }
    wave_sync();
    const bool gh = c.s.agent_erased;
    if (c.s.special_action == 1 && (c.s.cur_time - c.s.last_fire_time) >= 3) {
        const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
        wave_sync();
        const int e = append_entity(c, ax, ay, 0, 1, .25f, .25f, BF_PLAYER_BULLET);
        if (e >= 0) {
            EI(c, F_IMAGE_THEME, e) = B.player_laser_theme;
            EI(c, F_FLAGS, e) = EF_AUTO_ERASE | EF_COLLIDES;
            EI(c, F_EXPIRE_TIME, e) = 25;
        }
        c.s.last_fire_time = c.s.cur_time;
        wave_sync();
    }
    const int ct = c.s.cur_time;
    const float bv = B.boss_bullet_vel, rp = B.rand_pct;
    if (B.damaged_until_time >= ct) { // damaged_mode (:299-305)
        if (ct % 3 == 0) {
            const float pos_x = EF(c, F_X, boss) + (2 * B.rand_pct_x - 1) * EF(c, F_RX, boss);
            const float pos_y = EF(c, F_Y, boss) + (2 * B.rand_pct_y - 1) * EF(c, F_RY, boss);
            wave_sync();
            append_entity(c, pos_x, pos_y, 0, 0, .75f, .75f, EXPLOSION);
            wave_sync();
        }
    } else if (B.shields_are_up) { // active_attack (:307-317)
        const int am = B.attack_mode;
        if (am == 0) {
            if (ct % 8 == 0)
                for (int i = 0; i < 5; i++) bf_boss_fire(c, boss, .5f, bv, (float)(PI_F * 1.5 + (i - 2) * PI_F / 8));
        } else if (am == 1) {
            if (ct % 5 == 0) {
                int k = ct / 5;
                k = abs(8 - (k % 16));
                for (int i = 0; i < 4; i++)
                    bf_boss_fire(c, boss, .5f, bv, (float)(PI_F * (1.25 + .5 * k / 8.0) + i * PI_F / 2));
            }
        } else if (am == 2) {
            if (ct % 10 == 0) {
                const int num_bullets = 8;
                const float offset = rp * 2 * PI_F;
                for (int i = 0; i < num_bullets; i++) bf_boss_fire(c, boss, .5f, bv, 2 * PI_F / num_bullets * i + offset);
            }
        } else if (am == 3) {
            if (ct % 4 == 0) bf_boss_fire(c, boss, .5f, bv, PI_F * (1 + rp));
        }
    } else { // passive_attack_mode (:259-263), base_fire_prob = 0.1f
        if (B.rand_fire_pct < 0.1f) bf_boss_fire(c, boss, .5f, bv, PI_F * (1 + rp));
    }
    // each ENEMY_BULLET (descending) leaves a LASER_TRAIL (:375-391)
    const int n0 = c.s.num_ents;
    int cnt = 0;
    for (int base = 0; base < n0; base += 64) {
        const int i = base + LANE;
        cnt += __popcll(ballot(i < n0 && EI(c, F_TYPE, i) == BF_ENEMY_BULLET));
    }
    if (n0 + cnt > PG_CAP - c.s.num_tail) {
        c.s.error = PG_ERR_ENTITY_OVERFLOW;
        return;
    }
    int done = 0;
    for (int base = (n0 - 1) & ~63; base >= 0; base -= 64) {
        const int i = base + LANE;
        const bool eb = i < n0 && EI(c, F_TYPE, i) == BF_ENEMY_BULLET;
        const unsigned long long b = ballot(eb);
        if (eb) {
            // rank from the top: bullets above i in this chunk
            const int rank = done + __popcll(b & ~((2ull << LANE) - 1ull));
            const int t = n0 + rank;
            EF(c, F_X, t) = EF(c, F_X, i); EF(c, F_Y, t) = EF(c, F_Y, i);
            EF(c, F_VX, t) = EF(c, F_VX, i) * .5f; EF(c, F_VY, t) = EF(c, F_VY, i) * .5f;
            EF(c, F_RX, t) = EF(c, F_RX, i); EF(c, F_RY, t) = EF(c, F_RY, i);
            EF(c, F_ROTATION, t) = EF(c, F_ROTATION, i); EF(c, F_VROT, t) = EF(c, F_VROT, i);
            EF(c, F_ALPHA, t) = 1.0f; EF(c, F_ALPHA_DECAY, t) = 0.7f; EF(c, F_GROW_RATE, t) = 1.0f;
            EF(c, F_FRICTION, t) = 1; EF(c, F_COLLISION_MARGIN, t) = 0; EF(c, F_HEALTH, t) = 1;
            EF(c, F_THETA, t) = -100; EF(c, F_CLIMBER_SPAWN_X, t) = 0;
            EI(c, F_TYPE, t) = BF_LASER_TRAIL; EI(c, F_IMAGE_TYPE, t) = BF_ENEMY_BULLET;
            EI(c, F_IMAGE_THEME, t) = B.boss_laser_theme; EI(c, F_RENDER_Z, t) = 0; EI(c, F_LIFE_TIME, t) = 0;
            EI(c, F_EXPIRE_TIME, t) = 8; EI(c, F_FIRE_TIME, t) = -1; EI(c, F_SPAWN_TIME, t) = -1;
            EI(c, F_FLAGS, t) = EF_AUTO_ERASE;
        }
        done += __popcll(b);
    }
    c.s.num_ents = n0 + cnt;
    wave_sync();
}

// ------------------------------------------------------------------ starpilot (starpilot.cpp:356-430)
DEV void sp_copy_slot(Ctx &c, int from, int to) {
    for (int f = LANE; f < PG_NF; f += 64) EI(c, f, to) = EI(c, f, from);
}

DEV void starpilot_step_tail(Ctx &c, uint32_t *rg) {
    const int mode = c.s.opt_distribution_mode;
    const bool gh = c.s.agent_erased;
    const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
    const bool is_firing = c.s.special_action != 0;
    // entities that fire (should_fire, :356-366) or blow up, descending; each appends in order
    const int n0 = c.s.num_ents;
    int upper = n0;
    while (upper > 0) {
        int m = -1;
        for (int base = (upper - 1) & ~63; base >= 0; base -= 64) {
            const int i = base + LANE;
            bool act = false;
            if (i < upper) {
                const int t = EI(c, F_TYPE, i);
                if (t != PLAYER) {
                    const int ft = EI(c, F_FIRE_TIME, i), st = EI(c, F_SPAWN_TIME, i);
                    bool fire = false;
                    if (ft > 0) fire = t == SP_TURRET ? (c.s.cur_time - st) % ft == 0 : c.s.cur_time - st == ft;
                    const bool boom = EF(c, F_HEALTH, i) <= 0 && sp_destructible(t) && !(EI(c, F_FLAGS, i) & EF_WILL_ERASE);
                    act = fire || boom;
                }
            }
            const unsigned long long b = ballot(act);
            if (b) {
                m = base + top_bit(b);
                break;
            }
        }
        if (m < 0) break;
        upper = m;
        const int t = EI(c, F_TYPE, m), ft = EI(c, F_FIRE_TIME, m), st = EI(c, F_SPAWN_TIME, m);
        const float mx = EF(c, F_X, m), my = EF(c, F_Y, m);
        bool fire = false;
        if (ft > 0) fire = t == SP_TURRET ? (c.s.cur_time - st) % ft == 0 : c.s.cur_time - st == ft;
        if (fire) {
            const int bullet_type = t == SP_TURRET ? SP_BULLET3 : SP_BULLET2;
            const float bullet_r = sp_hp_bullet_r(mode);
            float b_vx = ax - mx, b_vy = ay - my;
            const float bv_scale = (float)(sp_hp_vs(mode, bullet_type) * SP_V_SCALE / sqrt((double)(b_vx * b_vx + b_vy * b_vy)));
            b_vx = b_vx * bv_scale;
            b_vy = b_vy * bv_scale;
            wave_sync();
            const int b = append_entity(c, mx, my, b_vx, b_vy, bullet_r, bullet_r, bullet_type);
            if (b >= 0) EF(c, F_ROTATION, b) = face_rotation(b_vx, b_vy, 0.0f, -1 * PI_F / 2);
            wave_sync();
        }
        if (EF(c, F_HEALTH, m) <= 0 && sp_destructible(t) && !(EI(c, F_FLAGS, m) & EF_WILL_ERASE)) {
            // spawn_child(m, EXPLOSION, .5 * rx, match_vel = true) (basic-abstract-game.cpp:233-239)
            const float mvx = EF(c, F_VX, m), mvy = EF(c, F_VY, m), cr = (float)(.5 * EF(c, F_RX, m));
            wave_sync();
            append_entity(c, mx, my, mvx, mvy, cr, cr, EXPLOSION);
            c.s.sd_reward += 1.0f; // ENEMY_REWARD
            EI(c, F_FLAGS, m) = EI(c, F_FLAGS, m) | EF_WILL_ERASE;
            wave_sync();
        }
    }
    // spawners due now move to `entities` (the back of the sorted list = slot PG_CAP - num_tail)
    while (c.s.num_tail > 0 && c.s.cur_time == EI(c, F_SPAWN_TIME, PG_CAP - c.s.num_tail)) {
        const int from = PG_CAP - c.s.num_tail;
        if (c.s.num_ents >= from) {
            c.s.error = PG_ERR_ENTITY_OVERFLOW;
            break;
        }
        wave_sync();
        sp_copy_slot(c, from, c.s.num_ents);
        wave_sync();
        c.s.num_ents += 1;
        c.s.num_tail -= 1;
    }
    if (is_firing) {
        const float theta = c.s.special_action == 2 ? PI_F : 0;
        const float v_scale = sp_hp_vs(mode, SP_BULLET_PLAYER) * SP_V_SCALE;
        double st, ct;
        pg_sincos_cr((double)theta, &st, &ct);
        const float vx = (float)(ct * v_scale), vy = (float)(st * v_scale);
        const float arx = gh ? c.gp->ghost_rx : EF(c, F_RX, 0);
        const float x_off = (float)(arx * ct);
        wave_sync();
        const int b = append_entity(c, ax + x_off, ay, vx, vy, sp_hp_bullet_r(mode), sp_hp_bullet_r(mode), SP_BULLET_PLAYER);
        if (b >= 0) {
            EI(c, F_FLAGS, b) = EF_AUTO_ERASE | EF_COLLIDES;
            float rot = face_rotation(vx, vy, 0.0f);
            rot -= PI_F / 2;
            EF(c, F_ROTATION, b) = rot;
        }
        wave_sync();
    }
    if (c.s.cur_time == SP_SHOOTER_WIN_TIME) {
        // Entity(main_width, main_height / 2, -slow_v * V_SCALE, 0, 2, main_height / 2, FINISH_LINE)
        const int theme = rg_randn_of(mt_next_global(rg, c.s.rg_mti, c.lds), c.d.num_themes[PG_GAME_STARPILOT * 100 + SP_FINISH_LINE]);
        const float fry = (float)(c.s.main_height / 2);
        const float frx = fry * aspect_ratio<PG_GAME_STARPILOT>(c, SP_FINISH_LINE, theme); // match_aspect_ratio(, false)
        wave_sync();
        const int f = append_entity(c, c.s.main_width + frx, fry, -1 * SP_HP_SLOW_V * SP_V_SCALE, 0, frx, fry, SP_FINISH_LINE);
        if (f >= 0) EI(c, F_IMAGE_THEME, f) = theme;
        wave_sync();
    }
}

DEV void fruitbot_step_tail(Ctx &c) { // fruitbot.cpp:247-258
    if (c.s.special_action == 1 && (c.s.cur_time - c.s.last_fire_time) >= FB_KEY_DURATION) {
        const bool gh = c.s.agent_erased;
        const float ax = gh ? c.gp->ghost_x : EF(c, F_X, 0), ay = gh ? c.gp->ghost_y : EF(c, F_Y, 0);
        const float vx = 0, vy = 1, bullet_vscale = .5;
        wave_sync();
        int i = append_entity(c, ax, ay, vx * bullet_vscale, vy * bullet_vscale, .25f, .25f, FB_PLAYER_BULLET);
        if (i >= 0) {
            EI(c, F_EXPIRE_TIME, i) = FB_KEY_DURATION;
            EI(c, F_FLAGS, i) = EF_AUTO_ERASE | EF_COLLIDES;
        }
        c.s.last_fire_time = c.s.cur_time;
        wave_sync();
    }
}

// ------------------------------------------------------------------ game_step
template <int G>
DEV void game_step(Ctx &c) {
    if constexpr (G == PG_GAME_LEAPER) leaper_pre_step(c);
    // miner moves the objects at or below the agent's row before the agent (miner.cpp:250-260)
    if constexpr (G == PG_GAME_MINER) miner_pre_step(c);
    // ---- BasicAbstractGame::game_step (basic-abstract-game.cpp:695-755)
    uint32_t *rg = c.d.mt + (size_t)c.env * 2 * PG_MT_WORDS;
    c.s.step_rand_int = rg_randint_of(mt_next_global(rg, c.s.rg_mti, c.lds), 0, 1000000);
    c.pt.mark(0);
    c.s.move_action = c.s.action % 9;
    c.s.special_action = 0;
    if (c.s.action >= 9) {
        c.s.special_action = c.s.action - 8;
        c.s.move_action = 4;
    }
    if (c.s.move_action != 4) c.s.last_move_action = c.s.move_action;
    c.s.action_vrot = 0;
    c.s.action_vx = 0;
    c.s.action_vy = 0;
    set_action_xy<G>(c, c.s.move_action);
    if (c.s.grid_step) {
        if (c.s.agent_erased) { // the erased agent's shared_ptr still takes the velocity
            c.gp->ghost_vx = c.s.action_vx;
            c.gp->ghost_vy = c.s.action_vy;
        } else {
            EF(c, F_VX, 0) = c.s.action_vx;
            EF(c, F_VY, 0) = c.s.action_vy;
        }
    } else {
        update_agent_velocity<G>(c);
        float vrot = EF(c, F_VROT, 0);
        vrot = MIXRATEROT * vrot;
        vrot += MIXRATEROT * (15 * PI_F / 180) * c.s.action_vrot;
        EF(c, F_VROT, 0) = vrot;
    }
    wave_sync();
    c.pt.mark(1);
    c.cs.mark(1);
    c.cs.mark(2);
    if (!step_entities_regs<G>(c)) {
        build_interactor_list<G>(c);
        step_entities<G>(c, c.slist);
    }
    c.pt.mark(2);
    c.cs.mark(4);
    agent_collisions<G>(c);
    c.pt.mark(3);
    erase_if_needed(c);
    c.pt.mark(4);
    float gx, gy, grx, gry;
    if (c.s.agent_erased) {
        gx = c.gp->ghost_x; gy = c.gp->ghost_y; grx = c.gp->ghost_rx; gry = c.gp->ghost_ry;
    } else {
        gx = EF(c, F_X, 0); gy = EF(c, F_Y, 0); grx = EF(c, F_RX, 0); gry = EF(c, F_RY, 0);
    }
    c.s.sd_done = c.s.sd_done || is_out_of_bounds(c, gx, gy, grx, gry);
    // ---- per-game tail
    if constexpr (G == PG_GAME_COINRUN) coinrun_step_tail(c);
    if constexpr (G == PG_GAME_BIGFISH) bigfish_step_tail(c, rg);
    if constexpr (G == PG_GAME_MAZE) maze_step_tail(c);
    if constexpr (G == PG_GAME_HEIST) heist_step_tail(c);
    if constexpr (G == PG_GAME_MINER) miner_step_tail(c);
    if constexpr (G == PG_GAME_CLIMBER) climber_step_tail(c);
    if constexpr (G == PG_GAME_LEAPER) leaper_step_tail(c, rg);
    if constexpr (G == PG_GAME_CHASER) chaser_step_tail(c);
    if constexpr (G == PG_GAME_FRUITBOT) fruitbot_step_tail(c);
    if constexpr (G == PG_GAME_DODGEBALL) dodgeball_step_tail(c, rg);
    if constexpr (G == PG_GAME_PLUNDER) plunder_step_tail(c, rg);
    if constexpr (G == PG_GAME_STARPILOT) starpilot_step_tail(c, rg);
    if constexpr (G == PG_GAME_BOSSFIGHT) bossfight_step_tail(c, rg);
    if constexpr (G == PG_GAME_NINJA) ninja_step_tail(c);
    if constexpr (G == PG_GAME_CAVEFLYER) caveflyer_step_tail(c);
    if constexpr (G == PG_GAME_JUMPER) jumper_step_tail(c);
    wave_sync();
    c.pt.mark(5);
}

// splitmix64 counter hash used for synthetic random actions (bench / parity tests)
DEV uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

#ifndef STEP_WAVES
#define STEP_WAVES 5 // <= 96 VGPRs: 5 waves per SIMD (measured +4% on the coinrun step)
#endif
struct StepLds {
    uint32_t *mt;
    int16_t *list, *slist;
    float4 *ibox;
    float *pstk;
    int *iinfo;
    int8_t *grid;
    uint8_t *moved;
};

// The kernel argument (a PGDev, the first argument of every kernel that calls step_env) through an
// opaque constant-address pointer to the kernarg segment: the compiler cannot move the loads of its
// fields above the point where the view is taken (step_env's epilogue).
typedef __attribute__((address_space(4))) const PGDev PGDevK;
DEV PGDevK &late_view() {
    PGDevK *p = (PGDevK *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}
// One PGEnv member of n words at word offset `off` into the write-back halves (lane q <-> word q / 64 + q).
// The agent's ghost words are written in HBM where they change (Ctx::gp), not from the registers.
// One v_writelane per word (the word's lane an inline constant: one SGPR operand per instruction).
template <int L>
DEV void writelane_c(uint32_t &w, uint32_t x) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"(x), "n"(L));
}
template <int OFF, typename T, int... Q>
DEV void wb_put_words(uint32_t &w0, uint32_t &w1, uint64_t &m0, uint64_t &m1, const T &v, std::integer_sequence<int, Q...>) {
    constexpr int G0 = (int)(offsetof(PGEnv, ghost_x) / 4), G1 = (int)(offsetof(PGEnv, ghost_ry) / 4);
    const uint32_t *u = reinterpret_cast<const uint32_t *>(&v);
    auto one = [&](auto qc) {
        constexpr int o = OFF + decltype(qc)::value;
        if constexpr (!(o >= G0 && o <= G1)) {
            const uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)u[decltype(qc)::value]); // uniform
            if constexpr (o < 64) {
                writelane_c<o>(w0, x);
                m0 |= 1ull << o;
            } else {
                writelane_c<o - 64>(w1, x);
                m1 |= 1ull << (o - 64);
            }
        }
    };
    (one(std::integral_constant<int, Q>{}), ...);
}
template <int OFF, typename T>
DEV void wb_put(uint32_t &w0, uint32_t &w1, uint64_t &m0, uint64_t &m1, const T &v) {
    wb_put_words<OFF>(w0, w1, m0, m1, v, std::make_integer_sequence<int, (int)(sizeof(T) / 4)>{});
}

// Game::step (game.cpp:136-171) of one env by the calling wave, minus reset (queued) and observe
// (pg_render)
template <int G>
DEV bool step_env(const PGDev &d, int env, const StepLds &L, int use_hash, uint64_t hash_seed, int32_t hash_t,
                  int slot, bool *done_out = nullptr) {
    uint32_t *lds_mt = L.mt;
    int16_t *lds_list = L.list, *lds_slist = L.slist;
    float4 *lds_ibox = L.ibox;
    float *lds_pstk = L.pstk;
    int *lds_iinfo = L.iinfo;
    int8_t *lds_grid = L.grid;
    GridPre<G> gpre;
    gpre.load(d.grid8 + (size_t)env * PG_GRID_MAX); // in flight while the scalars load
    Ctx c{d};
    c.moved = L.moved;
    c.env = env;
    c.gp = d.envs + env;
#ifdef PG_SCALAR_ENV
    c.s = *(const __attribute__((address_space(4))) PGEnv *)(d.envs + c.env);
#else
    c.s = d.envs[c.env];
#endif
    c.Eb = reinterpret_cast<char *>(d.ents + pg_ent_index(c.env, 0, 0));
    c.G = d.grid + (size_t)c.env * PG_GRID_MAX;
    c.lds = lds_mt;
    c.ilist = lds_list;
    c.slist = lds_slist;
    c.ibox = lds_ibox;
    c.pstk = lds_pstk;
    c.memo = lds_mt;
    c.nmemo = 0;
    c.iinfo = lds_iinfo;
    c.nlist = 0;
    c.grid8 = lds_grid;
    c.grid8_ok = false;
    c.cs.start();
    c.pt.start();
#ifdef PG_PROF_SMART
    for (int k = 0; k < 6; k++) c.sm[k] = 0;
    c.sm[5] = (uint64_t)c.s.num_ents;
#endif
    load_grid_lds<G>(c, gpre);
    c.cs.mark(0);

    int action;
    if (use_hash) {
        uint64_t g = (uint64_t)(uint32_t)(d.env_offset + c.env);
        action = (int)(splitmix64(hash_seed ^ (g << 32) ^ (uint64_t)(uint32_t)hash_t) % (uint64_t)d.num_actions);
        if (LANE == 0) d.actions[c.env] = action;
    } else {
        action = d.actions[c.env];
    }
    c.s.action = action;

    c.s.cur_time += 1;
    bool will_force_reset = false;
    if (c.s.action == -1) {
        c.s.action = c.s.default_action;
        will_force_reset = true;
    }
    c.s.sd_reward = 0;
    c.s.sd_done = 0;
    c.s.sd_level_complete = 0;
    game_step<G>(c);
    // slow-step predictor (launch order only, see pg_step_kernel): the agent ends the step touching
    // two or more static interactors (coinrun's crate piles: sub_step's push recursion branches on
    // every crate it overlaps) -- the next step is likely a slow one
    bool predicted = false;
    if constexpr (G == PG_GAME_COINRUN) {
#ifndef PG_SLOW_PREDICT_MARGIN
#define PG_SLOW_PREDICT_MARGIN 0.5f
#endif
        if (c.ireg && c.nlist >= 2 && !c.s.agent_erased) {
            const float ax = EF(c, F_X, 0), ay = EF(c, F_Y, 0), arx = EF(c, F_RX, 0), ary = EF(c, F_RY, 0);
            const bool near = LANE < c.nlist && !c.i_erase &&
                              fabsf(ax - c.i_x) < arx + c.i_rx + PG_SLOW_PREDICT_MARGIN &&
                              fabsf(ay - c.i_y) < ary + c.i_ry + PG_SLOW_PREDICT_MARGIN;
            predicted = __popcll(ballot(near)) >= 2;
        }
    }
    c.s.sd_done = c.s.sd_done || will_force_reset || (c.s.cur_time >= c.s.timeout);
    c.s.total_reward += c.s.sd_reward;
    if (c.s.sd_reward != 0) {
        c.s.last_reward_timer = 10;
        c.s.last_reward = c.s.sd_reward;
    }
    c.s.prev_level_seed = c.s.current_level_seed;
    bool done = c.s.sd_done;
    bool first = done;
    if (c.s.opt_use_sequential_levels && c.s.sd_level_complete) { // step_data.done = false (game.cpp:164-166)
        first = false;
        c.s.sd_done = 0;
    }
    c.s.episode_done = first;

    // The epilogue reads its output pointers through an opaque view of the kernel argument, so their
    // loads stay here instead of being merged into the entry's loads and spilled across the whole step.
    PGDevK &k = late_view();
    if (LANE == 0) {
        if (done) {
            int q = atomicAdd(k.reset_count + slot, 1);
            k.reset_queue[(size_t)slot * k.num_envs + q] = c.env;
        }
        k.done8[c.env] = (uint8_t)done;
        k.rew[c.env] = c.s.sd_reward;
        k.first[c.env] = (uint8_t)first;
        k.prev_level_seed[c.env] = c.s.prev_level_seed;
        k.prev_level_complete[c.env] = (uint8_t)c.s.sd_level_complete;
        k.level_seed[c.env] = c.s.current_level_seed;
        if (c.s.error) atomicOr(k.error_any, 1 << c.s.error);
    }
    // Write back only the PGEnv members this kernel can change (the rest is read-only here), as one
    // vector store per 64-word half of the struct: lane q holds word q (and 64 + q), the store is
    // masked to the written words -- 2 store instructions instead of one lane-0 store per member.
    {
        uint32_t w0 = 0, w1 = 0;
        uint64_t m0 = 0, m1 = 0;
#define PG_W(f) wb_put<(int)(offsetof(PGEnv, f) / 4)>(w0, w1, m0, m1, c.s.f);
        PG_STEP_WB_COMMON(PG_W) PG_W(error)
        if constexpr (G == PG_GAME_COINRUN) { PG_STEP_WB_COINRUN(PG_W) }
        if constexpr (G == PG_GAME_BIGFISH) { PG_STEP_WB_BIGFISH(PG_W) }
        if constexpr (G == PG_GAME_HEIST) { PG_STEP_WB_HEIST(PG_W) }
        if constexpr (G == PG_GAME_MINER) { PG_STEP_WB_MINER(PG_W) }
        if constexpr (G == PG_GAME_CLIMBER) { PG_STEP_WB_CLIMBER(PG_W) }
        if constexpr (G == PG_GAME_CHASER) { PG_STEP_WB_CHASER(PG_W) }
        if constexpr (G == PG_GAME_FRUITBOT) { PG_STEP_WB_FRUITBOT(PG_W) }
        if constexpr (G == PG_GAME_DODGEBALL) { PG_STEP_WB_DODGEBALL(PG_W) }
        if constexpr (G == PG_GAME_PLUNDER) { PG_STEP_WB_PLUNDER(PG_W) }
        if constexpr (G == PG_GAME_STARPILOT) { PG_STEP_WB_STARPILOT(PG_W) }
        if constexpr (G == PG_GAME_BOSSFIGHT) { PG_STEP_WB_BOSSFIGHT(PG_W) }
        if constexpr (G == PG_GAME_NINJA) { PG_STEP_WB_NINJA(PG_W) }
        if constexpr (G == PG_GAME_JUMPER) { PG_STEP_WB_JUMPER(PG_W) }
#undef PG_W
        uint32_t *o = reinterpret_cast<uint32_t *>(k.envs + c.env);
        if ((m0 >> LANE) & 1) o[LANE] = w0;
        if ((m1 >> LANE) & 1) o[64 + LANE] = w1;
    }
    c.pt.mark(6);
#ifdef PG_PROF_SMART
    if (LANE == 0 && d.prof)
        for (int k = 0; k < 6; k++) d.prof[(size_t)c.env * 16 + 8 + k] += c.sm[k];
#endif
#ifndef PG_PROF_STAMP // that diagnostic build fills these slots with the render's stamping sub-phases
    c.pt.flush(d.prof ? d.prof + (size_t)c.env * 16 : nullptr);
#endif
    c.cs.flush(d.prof ? d.prof + (size_t)c.env * 16 : nullptr);
    if (done_out) *done_out = done;
    return predicted && !done;
}


// Launch order: the previous step's slow envs first, then the game's env list in order.  An env is
// slow when its step took > d.heavy_ticks of wall clock (e.g. coinrun's crate-pile push chains,
// ~10x the median step); such envs tend to stay slow for several steps, and dispatching them first
// lets them overlap the bulk instead of forming the launch's tail (longest first).  The grid is
// n + PG_HEAVY_CAP workgroups: b < nh steps the b-th slow env; b >= nh the (b - nh)-th env of the
// list unless it was slow (already taken) or past the end -- those workgroups exit at once.  Each
// stepped env writes its flag and, when slow, appends itself to this step's list (one atomic per
// slow env only).  The order only affects scheduling: every env is stepped exactly once and envs
// are independent.  `parity` alternates per act: the previous step's list / flags are read, this
// step's are written.  env_list: the envs of this game (mixed batches), or null = envs 0..n-1.
template <int G>
__global__ __launch_bounds__(64, STEP_WAVES) void pg_step_kernel(PGDev d, const int32_t *env_list, int n, int parity,
                                                                int use_hash, uint64_t hash_seed, int32_t hash_t,
                                                                int slot) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_mt[PG_MT_N]; // 16-B aligned: the push memo reads uint4
    __shared__ int16_t lds_list[PG_CAP];
    __shared__ int16_t lds_slist[64];
    // the lane-parallel smart steps' interactor copy (pl_smart games only: LDS is what bounds the
    // workgroups per CU here)
    __shared__ float4 lds_ibox[pl_smart<G>() ? 64 : 1];
    __shared__ float lds_pstk[(scan_needed<G>(true) || scan_needed<G>(false)) ? 10 * 5 : 1];
    __shared__ int lds_iinfo[pl_smart<G>() ? 64 : 1];
    __shared__ __attribute__((aligned(16))) int8_t lds_grid[PG_GRID_MAX];
    __shared__ uint8_t lds_moved[G == PG_GAME_MINER ? 35 * 35 : 1];
    const int prev = parity ^ 1, b = (int)blockIdx.x;
    const int nh = min(d.sched[PG_SCHED_HC(prev) + slot], PG_HEAVY_CAP);
    int env;
    if (b < nh) {
        env = d.heavy[((size_t)prev * PG_NUM_GAMES + slot) * PG_HEAVY_CAP + b];
    } else {
        const int p = b - nh;
        if (p >= n) return;
        env = env_list ? env_list[p] : p;
        if (d.heavy_flag[(size_t)prev * d.num_envs + env]) return; // stepped as a slow item
    }
    const StepLds L{lds_mt, lds_list, lds_slist, lds_ibox, lds_pstk, lds_iinfo, lds_grid, lds_moved};
    const uint64_t t0 = wall_clock64();
    const bool predicted = step_env<G>(d, env, L, use_hash, hash_seed, hash_t, slot);
    const bool heavy = (int64_t)(wall_clock64() - t0) > d.heavy_ticks || (d.slow_predict && predicted);
    if (LANE == 0) {
        bool listed = false;
        if (heavy) {
            const int q = atomicAdd(d.sched + PG_SCHED_HC(parity) + slot, 1);
            listed = q < PG_HEAVY_CAP;
            if (listed) d.heavy[((size_t)parity * PG_NUM_GAMES + slot) * PG_HEAVY_CAP + q] = env;
        }
        d.heavy_flag[(size_t)parity * d.num_envs + env] = listed ? 1 : 0;
    }
}

} // namespace

#ifndef PG_FUSED_TU // pg_fused.hip includes this file for step_env
#ifndef PG_ONLY_GAME
#define PG_ONLY_GAME (-1) // experiment builds: instantiate one game's kernel only (-DPG_ONLY_GAME=5)
#endif
template <int G>
static void launch_step_g(const PGDev *d, const int32_t *env_list, int count, hipStream_t s, int use_hash,
                          uint64_t seed, int32_t t, int parity, int slot) {
    if constexpr (PG_ONLY_GAME < 0 || G == PG_ONLY_GAME)
        hipLaunchKernelGGL(pg_step_kernel<G>, dim3(count + (count < PG_HEAVY_CAP ? count : PG_HEAVY_CAP)), dim3(64),
                           0, s, *d, env_list, count, parity, use_hash, seed, t, slot);
}
// parity: alternates per act (the host zeroes this parity's slow-list length and the reset counts)
extern "C" void pg_launch_step(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s,
                               int use_hash, uint64_t seed, int32_t t, int parity, int slot) {
    if (count <= 0) return;
#define PG_CASE(G)                                                                                   \
    case G:                                                                                          \
        launch_step_g<G>(d, env_list, count, s, use_hash, seed, t, parity, slot);                    \
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

// Self-test of the libm-dependent device arithmetic (tests/test_gpu_libm.py): which = 0 ->
// bigfish_fish_radius(in[i]) (float out); 1 -> qt_rotation_matrix(in[i]) before its fuzzy-null
// clean-up (4 doubles out); 2 -> face_rotation(in[2i], in[2i+1]) (float out).
__global__ void pg_selftest_kernel(int which, const float *in, void *out, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (which == 0) {
        reinterpret_cast<float *>(out)[i] = bigfish_fish_radius(in[i]);
    } else if (which == 1) {
        double m[4];
        qt_rotation_matrix(in[i], m);
        const double a = (double)(in[i] * 180 / PI_F);
        if (a != 0 && a != 90. && a != -270. && a != 270. && a != -90. && a != 180.) { // undo the clean-up
            const double b = 0.017453292519943295769 * a;
            double sb, cb;
            pg_sincos_cr(b, &sb, &cb);
            m[1] = sb;
            m[2] = -sb;
        }
        double *o = reinterpret_cast<double *>(out) + 4 * i;
        o[0] = m[0]; o[1] = m[1]; o[2] = m[2]; o[3] = m[3];
    } else if (which == 2) {
        reinterpret_cast<float *>(out)[i] = face_rotation(in[2 * i], in[2 * i + 1], 0.0f);
    }
}

extern "C" int procgen_selftest_libm(int which, const float *d_in, void *d_out, int64_t n, void *stream) {
    if (which < 0 || which > 2 || n <= 0) return -1;
    int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(pg_selftest_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, which, d_in, d_out, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif // PG_FUSED_TU
