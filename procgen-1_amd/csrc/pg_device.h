// pg_device.h -- device-side helpers shared by the step / reset / render kernels.
//
// Execution model: one 64-lane wavefront per env (64-thread workgroups, so
// __syncthreads() is a single-wave barrier).  Game logic runs wave-uniform (every
// lane computes the same value, uniform state updates are stored by all lanes with
// the same value, so every later read of that word is a same-lane read); entity
// scans, entity updates, compaction, grid fills and pixel work run lane-parallel
// (lane = entity slot / cell / pixel), followed by a barrier before any other lane
// reads what they wrote.
//
// Floating point follows the reference's C++ promotion rules operation by
// operation; the build uses -ffp-contract=off so no mul+add is fused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pg_engine.h"
#include "pg_libm.h"

#define DEV __device__ __forceinline__
#define LANE ((int)threadIdx.x)

// ------------------------------------------------------------------ reference constants
// object-ids.h:9-27
#define INVALID_OBJ (-1)
#define PLAYER 0
#define SPACE 100
#define WALL_OBJ 51
#define EXPLOSION 54
#define EXPLOSION5 58
#define TRAIL 59
// basic-abstract-game.cpp:6-20
#define POS_EPS (-0.001f)
#define RENDER_EPS 0.02f
#define MIXRATEROT 0.5f
#define USE_ASSET_THRESHOLD 100
#define MAX_ASSETS 100
// coinrun.cpp:13-30
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

// bigfish.cpp:7-17
#define BF_FISH 2
#define BF_FISH_MIN_R .25f
#define BF_FISH_MAX_R 2.0f
#define BF_FISH_QUOTA 30
// maze.cpp:6-12
#define MZ_GOAL 2
// heist.cpp:10-15
#define HS_LOCKED_DOOR 1
#define HS_KEY 2
#define HS_EXIT 9
#define HS_KEY_ON_RING 11
// miner.cpp:10-23 (fork-modified)
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
// climber.cpp:12-26
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
DEV bool cl_is_wall(int t) { return t == CL_WALL_MID || t == CL_WALL_TOP; }
// fruitbot.cpp:12-23
#define FB_BARRIER 1
#define FB_OUT_OF_BOUNDS_WALL 2
#define FB_PLAYER_BULLET 3
#define FB_BAD_OBJ 4
#define FB_GOOD_OBJ 7
#define FB_LOCKED_DOOR 10
#define FB_LOCK 11
#define FB_PRESENT 12
#define FB_KEY_DURATION 8
// dodgeball.cpp:10-24
#define DB_LAVA_WALL 1
#define DB_PLAYER_BALL 3
#define DB_ENEMY 4
#define DB_DOOR 5
#define DB_ENEMY_BALL 6
#define DB_DOOR_OPEN 7
#define DB_DUST_CLOUD 8
#define DB_OOB_WALL 10
#define DB_ENEMY_VEL 0.05f
// plunder.cpp:11-15
#define PL_PLAYER_BULLET 1
#define PL_TARGET_LEGEND 2
#define PL_TARGET_BACKGROUND 3
#define PL_PANEL 6
#define PL_SHIP 7
// starpilot.cpp:6-26
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
#define SP_V_SCALE (2.0f / 5.0f)
// init_hps (starpilot.cpp:147-224) as functions of the distribution mode (the tables are constant
// per mode; deserialize recomputes them the same way, :437-442)
DEV float sp_hp_vs(int mode, int type) {
    if (type == SP_FAST_FLYER) return 1.5f;
    if (type == SP_BULLET_PLAYER || type == SP_BULLET3) return 2;
    if (type == SP_BULLET2) return mode == PG_EASY ? 1.25f : 2.0f;
    if (type == SP_FLYER && mode == PG_EASY) return .75f;
    return 1;
}
DEV float sp_hp_health(int mode, int type) {
    if (type == SP_METEOR) return 500;
    const bool ex = mode == PG_EXTREME;
    if (type == SP_TURRET) return ex ? 10 : 5;
    if (type == SP_FLYER) return ex ? 5 : 2;
    if (type == SP_FAST_FLYER) return ex ? 2 : 1;
    return 0;
}
DEV float sp_hp_bullet_r(int mode) { return mode == PG_EXTREME ? (float)(1.0f / 5) : (float)(1.0f / 2.5); }
DEV float sp_hp_object_r(int type) {
    return (type == SP_TURRET || type == SP_METEOR || type == SP_CLOUD) ? 1.0f * 2 : 1.0f / 2;
}
DEV float sp_hp_prob(int mode, int type) {
    if (type <= SP_BULLET3) return 0;
    if (type == SP_FLYER) return 3;
    if (mode == PG_EASY && (type == SP_METEOR || type == SP_CLOUD || type == SP_TURRET || type == SP_FAST_FLYER)) return 0;
    return 1;
}
#define SP_HP_SLOW_V .5f
// bossfight.cpp:8-30
#define BF_PLAYER_BULLET 1
#define BF_BOSS 2
#define BF_SHIELDS 3
#define BF_ENEMY_BULLET 4
#define BF_LASER_TRAIL 5
#define BF_REFLECTED_BULLET 6
#define BF_BARRIER 7
#define BF_BOSS_R 3.0f
#define BF_BOTTOM_MARGIN 6
#define BF_BOSS_VEL_TIMEOUT 20
#define BF_BOSS_DAMAGED_TIMEOUT 40
// jumper.cpp:11-27
#define JP_GOAL 1
#define JP_SPIKE 2
#define JP_CAVEWALL 6
#define JP_CAVEWALL_TOP 7
#define JP_PLAYER_JUMP 9
#define JP_PLAYER_LEFT1 10
#define JP_PLAYER_LEFT2 11
#define JP_PLAYER_RIGHT1 12
#define JP_PLAYER_RIGHT2 13
DEV bool jp_is_wall(int t) { return t == JP_CAVEWALL || t == JP_CAVEWALL_TOP; }
// caveflyer.cpp:12-21
#define CF_GOAL 1
#define CF_OBSTACLE 2
#define CF_TARGET 3
#define CF_PLAYER_BULLET 4
#define CF_ENEMY 5
#define CF_CAVEWALL 8
#define CF_EXHAUST 9
#define CF_MARKER 1003
// ninja.cpp:11-21
#define NJ_GOAL 1
#define NJ_BOMB 6
#define NJ_THROWING_STAR 7
#define NJ_PLAYER_RIGHT1 12
#define NJ_PLAYER_RIGHT2 13
#define NJ_FIRE 14
#define NJ_WALL_MID 20
// chaser.cpp:10-23
#define CH_LARGE_ORB 2
#define CH_ENEMY_WEAK 3
#define CH_ENEMY_EGG 4
#define CH_MAZE_WALL 5
#define CH_ENEMY 6
#define CH_MARKER 1001
#define CH_ORB 1002
// leaper.cpp:6-21
#define LP_LOG 1
#define LP_ROAD 2
#define LP_WATER 3
#define LP_CAR 4
#define LP_FINISH_LINE 5
#define LP_MONSTER_RADIUS 0.25f
#define LP_LOG_RADIUS 0.45f
#define LP_NSTEP 5
// object-ids.h
#define EXIT_OBJ 52
#define AGENT_OBJ 53
#define DOOR_OBJ 200
#define KEY_OBJ 300
// rot_table slots: face_direction(dx, dy) -> (dx + 1) * 3 + (dy + 1); ring keys (PI / 2)
#define PG_ROT_RING_KEY 9
#define PI_F 3.14159265358979323846264338327950288f

// Entity::face_direction(dx, dy, rotation_offset) (entity.cpp:84-88; atan2 = glibc atan2f, pg_libm.h)
DEV float face_rotation(float dx, float dy, float rot, float offset = 0.0f) {
    if (dx != 0 || dy != 0) rot = -1 * pg_atan2f(dy, dx) + offset;
    return rot;
}

// QTransform::rotate(rotation * 180 / PI) of draw_image (basic-abstract-game.cpp:912-913; Qt5
// qtransform.cpp): exact special cases for +-90 / 180 / 270, otherwise sin / cos of deg2rad * a in
// double (correctly rounded here, pg_libm.h); QTransform::type() then treats a qFuzzyIsNull sine
// (|s| <= 1e-12) as no rotation.
// m = {m11, m12, m21, m22}.  The host builds the same matrices with the C library for the
// angles of the rotation table; this is the device path for every other angle.
DEV void qt_rotation_matrix(float rotation, double *m) {
    const double a = (double)(rotation * 180 / PI_F);
    double sina = 0, cosa = 0;
    if (a == 0) {
        cosa = 1;
    } else if (a == 90. || a == -270.) {
        sina = 1;
    } else if (a == 270. || a == -90.) {
        sina = -1;
    } else if (a == 180.) {
        cosa = -1;
    } else {
        const double b = 0.017453292519943295769 * a;
        pg_sincos_cr(b, &sina, &cosa);
    }
    m[0] = cosa; m[1] = sina; m[2] = -sina; m[3] = cosa;
    if (fabs(sina) <= 0.000000000001) {
        m[1] = 0;
        m[2] = 0;
    }
}

DEV bool cr_is_wall(int t) { return t == CR_WALL_MID || t == CR_WALL_TOP; }
DEV bool cr_is_lava(int t) { return t == CR_LAVA_MID || t == CR_LAVA_TOP; }

DEV void wave_sync() { __syncthreads(); }

// Per-phase cycle accounting for diagnostic builds (make PROFILE=1): never in the product .so.
struct PTimer {
#ifdef PG_PROFILE
    uint64_t last, acc[8];
    DEV void start() {
        last = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < 8; k++) acc[k] = 0;
    }
    DEV void mark(int k) {
        uint64_t t = __builtin_amdgcn_s_memtime();
        acc[k] += t - last;
        last = t;
    }
    DEV void flush(uint64_t *p) {
        if (LANE == 0 && p)
            for (int k = 0; k < 8; k++) p[k] += acc[k];
    }
#else
    DEV void start() {}
    DEV void mark(int) {}
    DEV void flush(uint64_t *) {}
#endif
};

// Occupancy census (diagnostic PG_CENSUS builds only): a wave's start / end on the 100 MHz
// constant clock and where it ran (HW_ID: wave, SIMD, CU, SE; XCC_ID), so the host can rebuild how
// many waves of a launch were resident at once (scripts/census.py).
struct Census {
#ifdef PG_CENSUS
    uint64_t t0, tm[5];
    DEV void start() {
        t0 = __builtin_amdgcn_s_memrealtime();
        for (int k = 0; k < 5; k++) tm[k] = 0;
    }
    DEV void mark(int k) { tm[k] = __builtin_amdgcn_s_memrealtime(); }
    DEV void flush(uint64_t *p) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, 32 bits
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // HW_REG_XCC_ID
        if (threadIdx.x == 0 && p) {
            p[0] = t0;
            p[1] = t1;
            p[2] = (uint64_t)hw | ((uint64_t)xcc << 32);
            for (int k = 0; k < 5; k++) p[3 + k] = tm[k];
        }
    }
#else
    DEV void mark(int) {}
    DEV void start() {}
    DEV void flush(uint64_t *) {}
#endif
};

DEV unsigned long long ballot(bool p) { return __ballot(p); }
DEV int top_bit(unsigned long long m) { return 63 - __clzll(m); }

// ------------------------------------------------------------------ MT19937 (std::mt19937)
DEV uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// In-place twist of 624 words in LDS.  Ascending 64-word chunks, each read-then-write:
// word i reads i+1 (not yet rewritten) and (i+397)%624, which for i >= 227 is a word
// rewritten >= 163 positions earlier, i.e. in an earlier chunk -- exactly the
// sequential generator's data flow.
DEV void mt_twist_lds(uint32_t *mt) {
    for (int base = 0; base < PG_MT_N; base += 64) {
        int i = base + LANE;
        uint32_t nv = 0;
        if (i < PG_MT_N) {
            uint32_t a = mt[i], b = mt[(i + 1) % PG_MT_N], c = mt[(i + 397) % PG_MT_N];
            uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            nv = c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        wave_sync();
        if (i < PG_MT_N) mt[i] = nv;
        wave_sync();
    }
}

// std::mersenne_twister_engine::seed(s) into LDS (serial recurrence, uniform)
// The recurrence runs on the scalar unit (the seed is made wave-uniform) and each word is selected into
// its lane's register: 64 words per vector store instead of a masked LDS store per word.
DEV void mt_seed_lds(uint32_t *mt, uint32_t s) {
    uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
    for (int base = 0; base < PG_MT_N; base += 64) {
        int v = 0;
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const int i = base + q;
            if (i > 0 && i < PG_MT_N) x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
            v = LANE == q ? (int)x : v;
        }
        if (base + LANE < PG_MT_N) mt[base + LANE] = (uint32_t)v;
    }
    wave_sync();
}

// Generator whose words live in HBM (`g`, 624 words) with its position in *mti:
// one uniform load per draw; the rare twist is staged through LDS.
DEV uint32_t mt_next_global(uint32_t *g, int32_t &mti, uint32_t *lds) {
    uint32_t y;
    if (mti >= PG_MT_N) {
        for (int i = LANE; i < PG_MT_N; i += 64) lds[i] = g[i];
        wave_sync();
        mt_twist_lds(lds);
        for (int i = LANE; i < PG_MT_N; i += 64) g[i] = lds[i];
        y = lds[0];
        mti = 1;
        wave_sync();
    } else {
        y = g[mti];
        mti += 1;
    }
    return mt_temper(y);
}

// Generator resident in LDS
DEV uint32_t mt_next_lds(uint32_t *lds, int32_t &mti) {
    if (mti >= PG_MT_N) {
        mt_twist_lds(lds);
        mti = 0;
    }
    uint32_t y = lds[mti];
    mti += 1;
    return mt_temper(y);
}

// RandGen helpers over a raw draw (randgen.cpp:6-23)
DEV int rg_randint_of(uint32_t x, int low, int high) {
    uint32_t range = (uint32_t)high - (uint32_t)low;
    return (int)((uint32_t)low + (x % range));
}
DEV int rg_randn_of(uint32_t x, int high) { return (int)(x % (uint32_t)high); }
DEV float rg_rand01_of(uint32_t x) { return (float)((double)x / ((double)0xffffffffu + 1)); }

// ------------------------------------------------------------------ Qt raster restatement
// qRound / qFloor / qCeil (qglobal.h) and the scale blit of qblendfunctions_p.h
// (qt_scale_image_32bit), as pinned by tests/golden/qt_raster_goldens.npz.
DEV int qRound(double d) {
    return d >= 0.0 ? (int)(d + 0.5) : (int)(d - (double)((int)(d - 1)) + 0.5) + (int)(d - 1);
}

DEV uint32_t BYTE_MUL(uint32_t x, uint32_t a) {
    uint32_t t = (x & 0xff00ffu) * a;
    t = (t + ((t >> 8) & 0xff00ffu) + 0x800080u) >> 8;
    t &= 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a;
    x = (x + ((x >> 8) & 0xff00ffu) + 0x800080u);
    x &= 0xff00ff00u;
    return x | t;
}

// SourceOver of a premultiplied ARGB32 texel with painter opacity `const_alpha` (0..256)
DEV uint32_t blend_argb_pm(uint32_t dst, uint32_t src, int const_alpha) {
    if (const_alpha == 256) return src + BYTE_MUL(dst, (~src) >> 24);
    uint32_t a = (uint32_t)(const_alpha * 255) >> 8;
    uint32_t s = BYTE_MUL(src, a);
    return s + BYTE_MUL(dst, (~s) >> 24);
}

// SourceOver shortcut for a texel whose alpha is 0 or 255 at full opacity: BYTE_MUL(dst, 255) ==
// dst and BYTE_MUL(dst, 0) == 0 exactly, so blend_argb_pm(dst, src, 256) == over_binary(dst, src).
// Callers take it only when no lane of the wave holds a partial-alpha texel (alpha_partial),
// a wave-uniform branch, so the result is bit-identical to the full blend.
DEV uint32_t alpha_partial(uint32_t t) { return (t - 0x01000000u) < 0xfe000000u ? 1u : 0u; }
DEV uint32_t over_binary(uint32_t dst, uint32_t src) { return src + (src < 0x01000000u ? dst : 0u); }

DEV int qt_int_opacity(double o) {
    if (o < 0) o = 0;
    if (o > 1) o = 1;
    return (int)(o * 256);
}

// Geometry of QPainter::drawImage(QRectF(rx,ry,rw,rh), image iw x ih) on the 64x64 device.
struct Blit {
    int tx1, ty1, w, h;
    uint32_t basex, srcy;
    int ix, iy;
};

DEV bool qt_blit_setup(double rx, double ry, double rw, double rh, int iw, int ih, Blit &b) {
    if (!(rw > 0) || !(rh > 0) || iw <= 0 || ih <= 0) return false; // QRectF::isEmpty
    // qt_mapRect_non_normalizing(r, identity) == QRectF(topLeft, bottomRight)
    double t_w = (rx + rw) - rx, t_h = (ry + rh) - ry;
    double t_right = rx + t_w, t_bottom = ry + t_h;
    double sx = t_w / (double)iw, sy = t_h / (double)ih;
    int ix = (int)(65536.0 / sx);
    int iy = (int)(65536.0 / sy);
    int tx1 = qRound(rx), tx2 = qRound(t_right), ty1 = qRound(ry), ty2 = qRound(t_bottom);
    if (tx2 < tx1) { int t = tx2; tx2 = tx1; tx1 = t; }
    if (ty2 < ty1) { int t = ty2; ty2 = ty1; ty1 = t; }
    if (tx1 < 0) tx1 = 0;
    if (tx2 >= PG_RES) tx2 = PG_RES;
    if (tx1 >= tx2) return false;
    if (ty1 < 0) ty1 = 0;
    if (ty2 >= PG_RES) ty2 = PG_RES;
    if (ty1 >= ty2) return false;
    int h = ty2 - ty1, w = tx2 - tx1;
    uint32_t basex = (uint32_t)((int)ceil((tx1 + 0.5 - rx) * ix) - 1);
    uint32_t srcy = (uint32_t)((int)ceil((ty1 + 0.5 - ry) * iy) - 1);
    if ((int)(srcy >> 16) >= ih && iy < 0) { srcy += iy; --h; }
    if ((int)(basex >> 16) >= iw && ix < 0) { basex += ix; --w; }
    int yend = (int)((srcy + (uint32_t)(iy * (h - 1))) >> 16);
    if (yend < 0 || yend >= ih) --h;
    int xend = (int)((basex + (uint32_t)(ix * (w - 1))) >> 16);
    if (xend < 0 || xend >= iw) --w;
    if (w <= 0 || h <= 0) return false;
    b.tx1 = tx1; b.ty1 = ty1; b.w = w; b.h = h; b.basex = basex; b.srcy = srcy; b.ix = ix; b.iy = iy;
    return true;
}
