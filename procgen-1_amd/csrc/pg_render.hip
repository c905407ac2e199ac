// pg_render.hip -- Game::observe: 64x64 render + bgr32_to_rgb888 (reference game.cpp:8-23,
// 97-107, 173-191; basic-abstract-game.cpp:808-1075; games/coinrun.cpp:64-70, 133-138, 213-225;
// heist.cpp:42-44, 73-78).  A template over the game id (per-game hooks are `if constexpr`).
//
// One wavefront per env, a 16 KB RGB32 framebuffer in LDS.  The painter's algorithm of
// the reference is kept exactly, but each layer is rasterised the way a wave64 likes:
//   * background + grid tiles: pixel-centric -- lane = screen column, loop over rows.  A
//     pixel blends every tile covering it (<= 2 columns x 2 rows because of the RENDER_EPS
//     overlap) in the reference's x-major / y-minor draw order.  The Qt blit geometry of
//     every tile column (per lane) and tile row (lane = screen row, broadcast with
//     readlane) is computed once per frame; grid type -> sprite is an LDS table.
//   * entities: sprite-centric -- blit geometry of 64 entities at a time is computed
//     lane-parallel, then the entities are stamped one by one in list order (lanes =
//     footprint pixels), which is the only order-dependent part.
// Every blit reproduces Qt's raster scale blit (qt_scale_image_32bit fixed-point
// stepping, SourceOver on premultiplied ARGB32, painter opacity) bit for bit.
#include "pg_device.h"
#include "pg_assetgen.h"

namespace {

struct View {
    float unit, x_off, y_off, view_dim, visibility, center_x, center_y;
};

DEV float EFr(const PGDev &d, int f, int env, int slot) {
    return d.ents[pg_ent_index(env, f, slot)];
}
DEV int EIr(const PGDev &d, int f, int env, int slot) {
    return reinterpret_cast<const int *>(d.ents)[pg_ent_index(env, f, slot)];
}

// get_screen_rect (basic-abstract-game.cpp:808-810): float arithmetic, widened to qreal
DEV void screen_rect(const View &v, float x, float y, float dx, float dy, float eps, double &rx, double &ry,
                     double &rw, double &rh) {
    rx = (double)((x - eps) * v.unit - v.x_off);
    ry = (double)((v.view_dim - y - eps) * v.unit + v.y_off);
    rw = (double)((dx + 2 * eps) * v.unit);
    rh = (double)((dy + 2 * eps) * v.unit);
}

// One axis of Qt's scale blit setup (qt_scale_image_32bit); the x and y halves are independent.
struct Axis {
    int t1, n;       // first device pixel, pixel count (after clip and bound checks)
    uint32_t base;   // 16.16 source coordinate of pixel t1
    int step;
};

DEV bool axis_setup(double r, double rw, int iw, Axis &a) {
    a.n = 0;
    if (!(rw > 0) || iw <= 0) return false;
    double t_w = (r + rw) - r;  // qt_mapRect_non_normalizing: QRectF(topLeft, bottomRight)
    double t_right = r + t_w;
    double sx = t_w / (double)iw;
    int ix = (int)(65536.0 / sx);
    int t1 = qRound(r), t2 = qRound(t_right);
    if (t2 < t1) { int t = t2; t2 = t1; t1 = t; }
    if (t1 < 0) t1 = 0;
    if (t2 >= PG_RES) t2 = PG_RES;
    if (t1 >= t2) return false;
    int n = t2 - t1;
    uint32_t base = (uint32_t)((int)ceil((t1 + 0.5 - r) * ix) - 1);
    if ((int)(base >> 16) >= iw && ix < 0) { base += ix; --n; }
    int end = (int)((base + (uint32_t)(ix * (n - 1))) >> 16);
    if (end < 0 || end >= iw) --n;
    if (n <= 0) return false;
    a.t1 = t1; a.n = n; a.base = base; a.step = ix;
    return true;
}

DEV bool is_player_image(int t) {
    return t == PLAYER || t == CR_PLAYER_JUMP || t == CR_PLAYER_RIGHT1 || t == CR_PLAYER_RIGHT2;
}

DEV int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// The frame may be drawn in passes of h rows: the LDS frame buffer holds rows [y0, y0 + h) of the
// current pass, and every write is clipped to them.  Two 32-row passes halve the 16 KB frame and
// raise the workgroups an MI355X CU holds (LDS-bound at 8 with a full frame) -- for the games
// whose register budget allows 3 waves per SIMD (frame_rows below).
struct FB {
    uint32_t *p; // LDS rows of the pass
    int y0, h;
    uint32_t *own; // LDS bitmap of the pass's pixels (h * 64 bits, zero between batches): stamp_images' overlap test
#ifdef PG_PROF_STAMP
    PTimer *sp; // diagnostic: stamp_images' sub-phases (VARIANT=stamp EXTRA="-DPG_PROFILE -DPG_PROF_STAMP")
#endif
    DEV bool row_in(int row) const { return (unsigned)(row - y0) < (unsigned)h; }
    DEV bool o_in(int o) const { return (unsigned)(o - y0 * PG_RES) < (unsigned)(h * PG_RES); }
    DEV uint32_t &operator[](int o) const { return p[o - y0 * PG_RES]; }
};

// Size of the per-type grid sprite table (grid values 0..127 take the fast path).
#define NTYPES 64 // grid values 0..63 (and SPACE) take the fast path; anything else falls back
// Most tile rows a frame may span on the fast path: centred views of visibility 13 (coinrun) span
// 14-15, of visibility 16 17-18.  The frame buffer (16 KB) + colb + tile_off of coinrun / heist fit
// 20 KB, i.e. 8 workgroups per CU's 160 KB LDS.
template <int G>
DEV constexpr int crows() { return (G == PG_GAME_COINRUN || G == PG_GAME_HEIST) ? 15 : 18; }
// Rows per batch of the pixel-centric pass, entities per stamping group.
#ifndef RB
#define RB 8
#endif
// Chunks of 64 pixels of one large transform blit whose texel loads are issued together before the blends.
#ifndef ROTB
#define ROTB 1
#endif
// Rows / chunks of one large image whose texel loads are issued together before the blends.
#ifndef BB
#define BB 1
#endif
// runs of consecutive tile_image entities are stamped as one tile list (stamp_tile_run); 0: per entity
#ifndef RUN_TILES
#define RUN_TILES 1
#endif


// ------------------------------------------------------------------ per-game render hooks
// image_for_type (basic :446-448; coinrun.cpp:213-225): coinrun animates the player for the
// whole frame and hides ENEMY_BARRIER
template <int G>
DEV int player_image(const PGEnv &s, float agent_vx) {
    if constexpr (G == PG_GAME_CLIMBER) { // climber.cpp:156-166
        if (!s.has_support) return CL_PLAYER_JUMP;
        if (fabsf(agent_vx) < .01 && s.action_vx == 0 && s.has_support) return PLAYER;
        return (s.cur_time / 5 % 2 == 0 || !s.has_support) ? CL_PLAYER_RIGHT1 : CL_PLAYER_RIGHT2;
    }
    if constexpr (G == PG_GAME_JUMPER) { // jumper.cpp:126-135
        if (fabs((double)agent_vx) < .01 && s.action_vx == 0 && s.has_support) return PLAYER;
        const bool first = s.cur_time / 5 % 2 == 0 || !s.has_support;
        if (s.facing_right) return first ? JP_PLAYER_RIGHT1 : JP_PLAYER_RIGHT2;
        return first ? JP_PLAYER_LEFT1 : JP_PLAYER_LEFT2;
    }
    if constexpr (G == PG_GAME_NINJA) // ninja.cpp:143-153
        return (fabs((double)agent_vx) < .01 && s.action_vx == 0 && s.has_support)
                   ? PLAYER
                   : ((s.cur_time / 5 % 2 == 0 || !s.has_support) ? NJ_PLAYER_RIGHT1 : NJ_PLAYER_RIGHT2);
    if constexpr (G == PG_GAME_COINRUN)
        return (fabs((double)agent_vx) < .01 && s.action_vx == 0 && s.has_support)
                   ? PLAYER
                   : ((s.cur_time / 5 % 2 == 0 || !s.has_support) ? CR_PLAYER_RIGHT1 : CR_PLAYER_RIGHT2);
    return PLAYER;
}
template <int G>
DEV int image_for_type(const PGEnv &s, int type, int player_img) {
    if constexpr (G == PG_GAME_CHASER) { // chaser.cpp:101-113
        if (type == CH_ENEMY) {
            if (s.cur_time - s.eat_time < s.eat_timeout) return CH_ENEMY_WEAK;
            int rem = (s.cur_time / 2) % 4;
            if (rem == 3) rem = 1;
            return CH_ENEMY + rem;
        }
    }
    if constexpr (G == PG_GAME_NINJA || G == PG_GAME_JUMPER)
        if (type == PLAYER) return player_img;
    if constexpr (G == PG_GAME_COINRUN || G == PG_GAME_CLIMBER) { // ENEMY_BARRIER is 19 in both
        if (type == PLAYER) return player_img;
        if (type == CR_ENEMY_BARRIER) return -1;
    }
    if constexpr (G == PG_GAME_DODGEBALL) // dodgeball.cpp:90-96
        if (type == DB_DOOR) return s.num_enemies == 0 ? DB_DOOR_OPEN : DB_DOOR;
    if constexpr (G == PG_GAME_MINER) { // miner.cpp:95-103
        if (type == MN_MOVING_BOULDER) return MN_BOULDER;
        if (type == MN_MOVING_DIAMOND) return MN_DIAMOND;
    }
    return type < 0 ? -type : type;
}
template <int G>
DEV int grid_theme(const PGEnv &s, int type) { // theme_for_grid_obj (coinrun.cpp:133-138)
    if constexpr (G == PG_GAME_COINRUN) return cr_is_wall(type) ? s.wall_theme : 0;
    if constexpr (G == PG_GAME_CLIMBER) return cl_is_wall(type) ? s.wall_theme : 0; // climber.cpp:106-111
    if constexpr (G == PG_GAME_NINJA) return type == NJ_WALL_MID ? s.wall_theme : 0; // ninja.cpp:119-124
    if constexpr (G == PG_GAME_JUMPER) return jp_is_wall(type) ? s.wall_theme : 0;    // jumper.cpp:107-112
    return 0;
}
template <int G>
DEV int mask_theme(const PGEnv &s, int theme, int img_type) { // mask_theme_if_necessary (:454-462, heist.cpp:42-44)
    bool preserve = (G == PG_GAME_HEIST && (img_type == HS_KEY || img_type == HS_LOCKED_DOOR)) ||
                    (G == PG_GAME_PLUNDER && img_type == PL_SHIP) || // plunder.cpp:83-85
                    (G == PG_GAME_LEAPER && img_type == PLAYER); // leaper.cpp:91-93
    return (s.opt_restrict_themes && !preserve) ? 0 : theme;
}
template <int G>
DEV bool should_draw(const PGEnv &s, int type, int theme) { // should_draw_entity (heist.cpp:73-78)
    if constexpr (G == PG_GAME_BOSSFIGHT) // bossfight.cpp:133-138
        if (type == BF_SHIELDS) return s.gs.bf.shields_are_up != 0;
    if constexpr (G == PG_GAME_HEIST)
        if (type == HS_KEY_ON_RING) return (s.has_keys >> theme) & 1;
    return true;
}
// get_tile_aspect_ratio (basic :417-419; leaper.cpp:68-74): 0 = one image, > 0 tile horizontally
template <int G>
DEV float tile_aspect_ratio(int type, float rx, float ry) {
    if constexpr (G == PG_GAME_LEAPER) return type == LP_FINISH_LINE ? 1.0f : 0.0f;
    if constexpr (G == PG_GAME_DODGEBALL) return type == DB_LAVA_WALL ? (rx > ry ? 1.0f : -1.0f) : 0.0f; // :240-246
    if constexpr (G == PG_GAME_FRUITBOT) return type == FB_BARRIER ? 1.0f : (type == FB_LOCKED_DOOR ? 3.25f : 0.0f);
    return 0.0f;
}
template <int G>
DEV constexpr bool has_grid_tiles() { return G != PG_GAME_BIGFISH; } // bigfish: every cell is SPACE (never drawn)
// games whose entities can rotate (face_direction / rotation / vrot in games/*.cpp; the agent's
// action_vrot is 0 in every other game): elsewhere a rotation sets the error flag instead of
// keeping the transform-blit state live in registers
template <int G>
DEV constexpr bool has_rotation() {
    return G == PG_GAME_BOSSFIGHT || G == PG_GAME_CAVEFLYER || G == PG_GAME_DODGEBALL || G == PG_GAME_FRUITBOT ||
           G == PG_GAME_HEIST || G == PG_GAME_JUMPER || G == PG_GAME_LEAPER || G == PG_GAME_PLUNDER ||
           G == PG_GAME_STARPILOT;
}
// games with tile_image entities (get_tile_aspect_ratio != 0)
template <int G>
DEV constexpr bool has_tiled_entities() {
    return G == PG_GAME_LEAPER || G == PG_GAME_DODGEBALL || G == PG_GAME_FRUITBOT;
}
// Side of the square grid-tile images of the pixel-centric fast path (0: the game always takes the
// generic tile pass).  Coinrun and heist draw only such tiles; for the others a frame takes the fast
// path when every tile in its window is one (a window scan decides, e.g. jumper's and climber's
// 64x53 fourth wall theme or a visible ninja bomb send the frame to the generic pass).
template <int G>
DEV constexpr int tile_px() {
    if constexpr (G == PG_GAME_COINRUN || G == PG_GAME_HEIST || G == PG_GAME_CAVEFLYER) return 128;
    if constexpr (G == PG_GAME_JUMPER || G == PG_GAME_CLIMBER || G == PG_GAME_NINJA || G == PG_GAME_LEAPER) return 64;
    if constexpr (G == PG_GAME_DODGEBALL) return 12;
    return 0;
}
template <int G>
DEV constexpr bool uniform_tiles() { return tile_px<G>() > 0; }
// every drawable grid type of the game has a tile_px() image: no window scan needed
template <int G>
DEV constexpr bool always_uniform() { return G == PG_GAME_COINRUN || G == PG_GAME_HEIST || G == PG_GAME_CAVEFLYER; }
// the game has render_z = -1 entities (drawn between background and grid, :933)
template <int G>
DEV constexpr bool has_z_minus1() { return G == PG_GAME_MINER; } // miner's exit (miner.cpp:217)
// Games whose small-image batches are blended in one read-modify-write per round when no two images of the
// batch share a pixel (stamp_images' overlap bitmap): fruitbot 18.9 -> 21.3, dodgeball 27.6 -> 29.4, leaper
// 26.4 -> 27.5, starpilot 43.6 -> 44.2 M env-steps/s; bossfight, coinrun, jumper and plunder lose 1-2 %
// (their batches overlap, or are few), profiles/r06/r06_n_overlap_ab.txt
template <int G>
DEV constexpr bool overlap_blend() {
    return G == PG_GAME_FRUITBOT || G == PG_GAME_DODGEBALL || G == PG_GAME_LEAPER || G == PG_GAME_STARPILOT;
}
// an image the reference lists but the asset tree lacks (miner's mud.png, resources.cpp:511):
// drawn as nothing (the reference cannot load it; parity unpinned for MUD tiles)
template <int G>
DEV bool missing_image_ok(int img) { return G == PG_GAME_MINER && img == MN_MUD; }

// ------------------------------------------------------------------ rotated drawImage
// save(); translate(center); rotate(rotation * 180 / PI); drawImage(QRectF(-w/2, -h/2, w, h))
// (basic-abstract-game.cpp:908-916) -> Qt's qt_transform_image (qblendfunctions_p.h): the quad
// is split into 3 trapezoids, each scan line covers [x_l >> 16, x_r >> 16) with 16.16
// fixed-point texture stepping.  Along a scan line the in-source texels form one interval and
// the reference clamps the ones outside it, so a pixel's texel is clamp(u >> 16), clamp(v >> 16)
// with u = x * dudx + y * dudy + u0 -- evaluated per pixel (lane = column, loop over rows).
// The rotation matrix comes from the host table (exact C-library sin/cos, as Qt's qSin/qCos).
struct Trap { int from_y, to_y, x_l, dx_l, x_r, dx_r; };
struct QV { double x, y, u, v; };

DEV void trap_setup(const QV &tl, const QV &bl, const QV &tr, const QV &br, double topY, double bottomY, Trap &t) {
    t.from_y = max(qRound(topY), 0);
    t.to_y = min(qRound(bottomY), PG_RES);
    t.x_l = t.x_r = t.dx_l = t.dx_r = 0;
    if (t.from_y >= t.to_y) return;
    double leftSlope = (bl.x - tl.x) / (bl.y - tl.y);
    double rightSlope = (br.x - tr.x) / (br.y - tr.y);
    t.dx_l = (int)(leftSlope * 0x10000);
    t.dx_r = (int)(rightSlope * 0x10000);
    t.x_l = (int)((tl.x + (0.5 + t.from_y - tl.y) * leftSlope + 0.5) * 0x10000);
    t.x_r = (int)((tr.x + (0.5 + t.from_y - tr.y) * rightSlope + 0.5) * 0x10000);
}

// One axis of qt_scale_image_32bit for a mapped target rect whose extent may be negative (a
// TxScale transform from rotate(180), qblendfunctions_p.h: the sx < 0 branch steps back from
// the source rect's right edge).
DEV bool axis_setup_signed(double r, double rw, int iw, Axis &a) {
    a.n = 0;
    if (iw <= 0) return false;
    const double right = r + rw;
    const double sx = rw / (double)iw;
    const int ix = (int)(65536.0 / sx);
    int t1 = qRound(r), t2 = qRound(right);
    if (t2 < t1) { int t = t2; t2 = t1; t1 = t; }
    if (t1 < 0) t1 = 0;
    if (t2 >= PG_RES) t2 = PG_RES;
    if (t1 >= t2) return false;
    int n = t2 - t1;
    uint32_t base;
    if (sx < 0) base = (uint32_t)((double)iw * 65536) + (uint32_t)((int)floor((t1 + 0.5 - right) * ix) + 1);
    else base = (uint32_t)((int)ceil((t1 + 0.5 - r) * ix) - 1);
    if ((int)(base >> 16) >= iw && ix < 0) { base += ix; --n; }
    int end = (int)((base + (uint32_t)(ix * (n - 1))) >> 16);
    if (end < 0 || end >= iw) --n;
    if (n <= 0) return false;
    a.t1 = t1; a.n = n; a.base = base; a.step = ix;
    return true;
}

// The integer state of qt_transform_image for one rotated image: 3 trapezoids + texture stepping.
struct RotGeo {
    Trap tr[3];
    int dudx, dvdx, dudy, dvdy, u0, v0;
};

// Setup of save(); translate; rotate; drawImage(QRectF(-w/2, -h/2, w, h)): 0 = nothing drawn,
// 1 = TxScale (qt_scale_image_32bit with the signed axes ex / ey), 2 = a transform blit (g).
DEV int rot_prepare(double x, double y, double w, double h, double m11, double m12, double m21, double m22, int iw,
                    int ih, Axis &ex, Axis &ey, RotGeo &g) {
    if (!(w > 0) || !(h > 0) || iw <= 0 || ih <= 0) return 0; // QRectF::isEmpty: nothing drawn
    const double dx = x + w / 2, dy = y + h / 2;
    const double rx = -w / 2, ry = -h / 2, right = rx + w, bottom = ry + h;
    if (m12 == 0 && m21 == 0) {
        // QTransform::type() says TxScale / TxTranslate (the host zeroed qFuzzyIsNull m12 / m21):
        // qt_scale_image_32bit on qt_mapRect_non_normalizing(r, matrix) -- the TxScale map
        const double ax = m11 * rx + dx, ay = m22 * ry + dy;
        const double bx = m11 * right + dx, by = m22 * bottom + dy;
        if (!axis_setup_signed(ax, bx - ax, iw, ex) || !axis_setup_signed(ay, by - ay, ih, ey)) return 0;
        return 1;
    }
    QV v[4]; // TopLeft, TopRight, BottomRight, BottomLeft
    auto map = [&](double px, double py, QV &o) {
        o.x = m11 * px + m21 * py + dx;
        o.y = m12 * px + m22 * py + dy;
    };
    map(rx, ry, v[0]); map(right, ry, v[1]); map(right, bottom, v[2]); map(rx, bottom, v[3]);
    v[0].u = 0; v[0].v = 0; v[1].u = iw; v[1].v = 0; v[2].u = iw; v[2].v = ih; v[3].u = 0; v[3].v = ih;
    int topmost = 0;
    double top_y = v[0].y;
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (v[i].y < top_y) {
            topmost = i;
            top_y = v[i].y;
        }
    QV t;
    if (topmost == 1) {
        t = v[0]; v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = t;
    } else if (topmost == 2) {
        t = v[0]; v[0] = v[2]; v[2] = t;
        t = v[1]; v[1] = v[3]; v[3] = t;
    } else if (topmost == 3) {
        t = v[3]; v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = t;
    }
    double dx1 = v[1].x - v[0].x, dy1 = v[1].y - v[0].y;
    double dx2 = v[3].x - v[0].x, dy2 = v[3].y - v[0].y;
    if (dx1 * dy2 - dx2 * dy1 > 0) {
        t = v[1]; v[1] = v[3]; v[3] = t;
    }
    QV u = {v[1].x - v[0].x, v[1].y - v[0].y, v[1].u - v[0].u, v[1].v - v[0].v};
    QV ww = {v[2].x - v[0].x, v[2].y - v[0].y, v[2].u - v[0].u, v[2].v - v[0].v};
    double det = u.x * ww.y - u.y * ww.x;
    if (det == 0) return 0;
    double invDet = 1.0 / det;
    double n11 = (u.u * ww.y - u.y * ww.u) * invDet;
    double n12 = (u.x * ww.u - u.u * ww.x) * invDet;
    double n21 = (u.v * ww.y - u.y * ww.v) * invDet;
    double n22 = (u.x * ww.v - u.v * ww.x) * invDet;
    double mdx = v[0].u - n11 * v[0].x - n12 * v[0].y;
    double mdy = v[0].v - n21 * v[0].x - n22 * v[0].y;
    g.dudx = (int)(n11 * 0x10000); g.dvdx = (int)(n21 * 0x10000);
    g.dudy = (int)(n12 * 0x10000); g.dvdy = (int)(n22 * 0x10000);
    g.u0 = (int)ceil((0.5 * n11 + 0.5 * n12 + mdx) * 0x10000) - 1;
    g.v0 = (int)ceil((0.5 * n21 + 0.5 * n22 + mdy) * 0x10000) - 1;
    if (v[1].y < v[3].y) {
        trap_setup(v[0], v[1], v[0], v[3], v[0].y, v[1].y, g.tr[0]);
        trap_setup(v[1], v[2], v[0], v[3], v[1].y, v[3].y, g.tr[1]);
        trap_setup(v[1], v[2], v[3], v[2], v[3].y, v[2].y, g.tr[2]);
    } else {
        trap_setup(v[0], v[1], v[0], v[3], v[0].y, v[3].y, g.tr[0]);
        trap_setup(v[0], v[1], v[3], v[2], v[3].y, v[1].y, g.tr[1]);
        trap_setup(v[1], v[2], v[3], v[2], v[1].y, v[2].y, g.tr[2]);
    }
    return 2;
}

// returns false when the transform is not a rotation this path reproduces
DEV bool rotated_blit(const FB &fb, const uint32_t *pixels, uint32_t npix, double x, double y, double w, double h,
                      double m11, double m12, double m21, double m22, uint32_t soff, int iw, int ih, bool mir, int ca) {
    Axis ex, ey;
    RotGeo g;
    const int kind = rot_prepare(x, y, w, h, m11, m12, m21, m22, iw, ih, ex, ey, g);
    if (kind == 0) return true;
    if (kind == 1) {
        const int lane = LANE;
        bool ok = true;
        if (lane >= ex.t1 && lane < ex.t1 + ex.n) {
            int scol = (int)((ex.base + (uint32_t)((lane - ex.t1) * ex.step)) >> 16);
            if (mir) scol = iw - 1 - scol;
            const int klo = max(0, fb.y0 - ey.t1), khi = min(ey.n, fb.y0 + fb.h - ey.t1); // the pass's rows
            for (int k0 = klo; k0 < khi; k0 += BB) { // BB rows: every texel load issued before the blends
                uint32_t tv[BB];
#pragma unroll
                for (int r = 0; r < BB; r++) {
                    const int k = k0 + r;
                    const uint32_t idx = soff + (uint32_t)(((int)((ey.base + (uint32_t)(k * ey.step)) >> 16)) * iw + scol);
                    const bool in = k < khi && idx < npix;
                    if (k < khi && !in) ok = false;
                    tv[r] = pixels[in ? idx : 0u];
                }
#pragma unroll
                for (int r = 0; r < BB; r++) {
                    const int k = k0 + r;
                    if (k >= khi) break;
                    const int o = (ey.t1 + k) * PG_RES + lane;
                    fb[o] = blend_argb_pm(fb[o], tv[r], ca);
                }
            }
        }
        return ok;
    }
    const int lane = LANE;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const Trap T = g.tr[k];
        const int ylo = max(T.from_y, fb.y0), yhi = min(T.to_y, fb.y0 + fb.h); // the pass's scan lines
        for (int yb = ylo; yb < yhi; yb += BB) { // BB scan lines: loads first, then blends
            uint32_t tv[BB];
            bool on[BB];
#pragma unroll
            for (int r = 0; r < BB; r++) {
                const int yy = yb + r;
                const int xl = T.x_l + (yy - T.from_y) * T.dx_l, xr = T.x_r + (yy - T.from_y) * T.dx_r;
                const int fromX = max(xl >> 16, 0), toX = min(xr >> 16, PG_RES);
                on[r] = yy < yhi && lane >= fromX && lane < toX;
                int uu = (lane * g.dudx + yy * g.dudy + g.u0) >> 16;
                int vv = (lane * g.dvdx + yy * g.dvdy + g.v0) >> 16;
                uu = min(max(uu, 0), iw - 1);
                vv = min(max(vv, 0), ih - 1);
                if (mir) uu = iw - 1 - uu;
                const uint32_t idx = soff + (uint32_t)(vv * iw + uu);
                if (on[r] && idx >= npix) {
                    ok = false;
                    on[r] = false;
                }
                tv[r] = pixels[on[r] ? idx : 0u];
            }
#pragma unroll
            for (int r = 0; r < BB; r++)
                if (on[r]) fb[(yb + r) * PG_RES + lane] = blend_argb_pm(fb[(yb + r) * PG_RES + lane], tv[r], ca);
        }
    }
    return ok;
}


// ------------------------------------------------------------------ in-order image stamping
// The Qt scale blit of up to 64 images whose geometry lanes computed (lane k <-> image k),
// applied in ascending lane order.  EG images per group: the texel of this lane's footprint
// pixel is loaded for every image of the group first (loads are order-free), then the group
// is blended strictly in order.  Footprints wider than one wave (> 64 px) fall back to an
// in-order loop with inline loads; rotated images run the transform blit in place.
struct Img {
    bool draw;
    int rot;               // 0 scale blit, 1 transform blit (set up when stamped), 2 transform blit, descriptor rdi in LDS
    int rdi;
    uint32_t fill;         // != 0: an opaque fillRect of this colour over the ex / ey footprint
    Axis ex, ey;
    int soff, sw, sh, ca, mir, rslot, ez;
    int ntile;             // > 0: tile_image with this many tiles (seq path)
    float tw, th;          // tile size (float, as tile_image computes it)
    double rx, ry, rw, rh; // target rect of a rotated / tiled image
    double m11, m12, m21;  // rotation matrix of a rotated image (m22 = m11), built lane-parallel
};

DEV void img_clear(Img &im) {
    im.draw = false;
    im.rot = 0;
    im.rdi = 0;
    im.ntile = 0;
    im.tw = im.th = 0;
    im.fill = 0;
    im.ex.t1 = im.ex.n = im.ey.t1 = im.ey.n = 0;
    im.ex.base = im.ey.base = 0;
    im.ex.step = im.ey.step = 0;
    im.soff = im.sw = im.sh = im.mir = im.rslot = 0;
    im.ca = 256;
    im.ez = 0x7fffffff;
    im.rx = im.ry = im.rw = im.rh = 0;
}

// fillRect(QRectF, opaque colour) (qpaintengine_raster toNormalizedFillRect: qRound of the edges,
// pinned vs Qt 5.9.7 by tests/golden/qt_raster_fill_goldens.npz), clipped to the frame
DEV bool fill_setup(double x, double y, double w, double h, uint32_t argb, Img &im) {
    int x1 = qRound(x), y1 = qRound(y), x2 = qRound(x + w), y2 = qRound(y + h);
    if (x2 < x1) { int t = x1; x1 = x2; x2 = t; }
    if (y2 < y1) { int t = y1; y1 = y2; y2 = t; }
    x1 = max(x1, 0); y1 = max(y1, 0); x2 = min(x2, PG_RES); y2 = min(y2, PG_RES);
    if (x1 >= x2 || y1 >= y2) return false;
    im.ex.t1 = x1; im.ex.n = x2 - x1; im.ex.base = 0; im.ex.step = 0;
    im.ey.t1 = y1; im.ey.n = y2 - y1; im.ey.base = 0; im.ey.step = 0;
    im.fill = argb | 0xff000000u;
    im.draw = true;
    return true;
}

// draw_grid_obj overrides (basic-abstract-game.cpp:924-928): true when the game fills this
// grid object itself (chaser's orbs, chaser.cpp:111-117)
template <int G>
DEV bool grid_obj_fill(int img, double rx, double ry, double rw, double rh, Img &im) {
    if constexpr (G == PG_GAME_CHASER) {
        if (img == CH_ORB) {
            const float dim = 0.3f, k = 1 - dim;
            fill_setup(rx + rw * k / 2, ry + rh * k / 2, rw * dim, rh * dim, 0xff00ff00u, im);
            return true;
        }
    }
    return false;
}

// color_for_type (basic-abstract-game.cpp:464-490): the monochrome colour of (img_type, theme);
// 0 when the reference would fassert (type >= k^3 = 64)
template <int G>
DEV uint32_t color_for_type(const PGEnv &s, int type, int theme) {
    if (type < 0 || type >= 64) return 0;
    theme = mask_theme<G>(s, theme, type);
    int nt = (29 * (type + 1)) % 64;
    nt = (nt + 19 * theme) % 64;
    const uint32_t r = 64 * (nt / 16 + 1) - 1, g = 64 * ((nt / 4) % 4 + 1) - 1, b = 64 * (nt % 4 + 1) - 1;
    return 0xff000000u | (r << 16) | (g << 8) | b;
}

// draw_grid_obj (basic-abstract-game.cpp:924-928) for monochrome assets, after the game's own
// override (grid_obj_fill): fillRect(rect, color_for_type).  False when the reference fasserts.
template <int G>
DEV bool mono_fill(const PGEnv &s, int img, int theme, double rx, double ry, double rw, double rh, Img &im) {
    if (grid_obj_fill<G>(img, rx, ry, rw, rh, im)) return true;
    const uint32_t col = color_for_type<G>(s, img, theme);
    if (col == 0) return false;
    fill_setup(rx, ry, rw, rh, col, im);
    return true;
}

// to_shade (qt-utils.h:21-28)
DEV int to_shade(float f) {
    int shade = (int)(f * 255);
    return shade < 0 ? 0 : (shade > 255 ? 255 : shade);
}

// fillRect(QRectF, opaque colour) straight into the frame, lane-parallel (same edges as fill_setup)
DEV void fb_fill_rectf(const FB &fb, double x, double y, double w, double h, uint32_t argb) {
    Img im;
    im.draw = false;
    if (!fill_setup(x, y, w, h, argb, im)) return;
    const int nx = im.ex.n, ny = im.ey.n;
    for (int p = LANE; p < nx * ny; p += 64)
        if (fb.row_in(im.ey.t1 + p / nx)) fb[(im.ey.t1 + p / nx) * PG_RES + im.ex.t1 + p % nx] = im.fill;
}

// jumper's compass (jumper.cpp:137-177).  The dial ellipse, the cosmetic needle and the translucent
// jump ellipse are Qt 5.9.7 raster output tabulated per configuration / endpoint / rect size by
// tools/qt_compass_tables.cpp (atlas image slot PG_TABLE_SLOT, layout in procgen_amd/assets.py
// compass_table_words); lane = canvas row, each lane stamps the set bits of its row mask.
DEV void jp_stamp(const FB &fb, const uint32_t *rows, int dx, int dy, uint32_t argb, bool blend) {
    const int y = LANE, sy = y - dy;
    if (sy < 0 || sy >= PG_RES || dx <= -64 || dx >= 64 || !fb.row_in(y)) return;
    uint64_t m = (uint64_t)rows[2 * sy] | ((uint64_t)rows[2 * sy + 1] << 32);
    m = dx >= 0 ? (m << dx) : (m >> -dx);
    while (m) {
        const int x = __ffsll((long long)m) - 1;
        m &= m - 1;
        uint32_t *p = &fb[y * PG_RES + x];
        *p = blend ? argb + BYTE_MUL(*p, (~argb) >> 24) : argb;
    }
}
DEV bool jp_draw_compass(const FB &fb, const PGEnv &s, const View &v, const PGDev &d, int env) {
    const int4 ti = reinterpret_cast<const int4 *>(d.sprites)[PG_TABLE_SLOT];
    if (ti.y <= 0) return false;
    const uint32_t *t = d.pixels + (uint32_t)ti.x;
    const int NY = (int)t[1], NX = (int)t[2], MAXW = (int)t[3], MAXH = (int)t[4];
    const int cfg = (s.opt_distribution_mode == PG_EASY ? 0 : 1) + (s.opt_center_agent ? 0 : 2);
    const uint32_t *cg = t + 5 + 9 * cfg;
    const int bx0 = (int)cg[2], by0 = (int)cg[3], bnx = (int)cg[4], bny = (int)cg[5];
    const float cx = __uint_as_float(cg[6]), cy = __uint_as_float(cg[7]), cr = __uint_as_float(cg[8]);
    const uint32_t *dial = t + 5 + 36;
    const uint32_t *needle = dial + 4 * 128;
    const uint32_t *jump = needle + (size_t)4 * NY * NX * 128;
    const float u = v.unit, vd = v.view_dim, cd = s.gs.jp.compass_dim;
    const double rx = (double)((float)(vd - cd - .25) * u), rw = (double)(cd * u);
    if ((float)(rx + rw / 2) != cx) return false; // the table was built for this frame geometry
    jp_stamp(fb, dial + 128 * cfg, 0, 0, 0xffa8a69eu, false); // QColor(168, 166, 158)
    wave_sync();
    const float ax = EFr(d, F_X, env, 0), ay = EFr(d, F_Y, env, 0), arx = EFr(d, F_RX, env, 0), ary = EFr(d, F_RY, env, 0);
    const float gx = EFr(d, F_X, env, 1), gy = EFr(d, F_Y, env, 1);
    const float theta = (float)atan2((double)(gy - ay), (double)(gx - ax)); // get_theta (:241-246), double atan2
    double sn, cs;
    pg_sincos_cr((double)theta, &sn, &cs);
    const int x2 = (int)((double)cx + (double)cr * cs), y2 = (int)((double)cy - (double)cr * sn);
    if (x2 < bx0 || x2 >= bx0 + bnx || y2 < by0 || y2 >= by0 + bny) return false;
    jp_stamp(fb, needle + ((size_t)(cfg * NY + (y2 - by0)) * NX + (x2 - bx0)) * 128, 0, 0, 0xfffcba03u, false);
    wave_sync();
    const float ddx = ax - gx, ddy = ay - gy; // get_distance (:133-143)
    const float dist = (float)sqrt((double)(ddx * ddx + ddy * ddy));
    const float dist_pct = (float)((double)dist / (s.main_width * 1.4142135623730951)); // main_width * sqrt(2)
    const float bar_thickness = cd / 8;
    fb_fill_rectf(fb, (double)((float)(vd - cd - .25) * u), (double)((float)(.25 + cd) * u), (double)(cd * dist_pct * u),
                  (double)(bar_thickness * u), 0xfffcba03u);
    wave_sync();
    if (s.gs.jp.jump_delta < 0 && !s.has_support) { // drawEllipse(QRect(...)) of get_object_rect(agent)
        double r1x, r1y, r1w, r1h;
        screen_rect(v, ax - arx, ay + ary, 2 * arx, 2 * ary, 0, r1x, r1y, r1w, r1h);
        const int qx = (int)r1x, qy = (int)(r1y + r1h * (5.0 / 6)), qw = (int)r1w, qh = (int)(r1h / 3);
        if (qw < 0 || qw > MAXW || qh < 0 || qh > MAXH) return false;
        jp_stamp(fb, jump + (size_t)(qw * (MAXH + 1) + qh) * 128, qx - 20, qy - 20, 0x78787878u, true);
        wave_sync();
    }
    return true;
}

// game_draw additions drawn over the foreground (plunder.cpp:66-77)
template <int G>
DEV void game_overlay(const FB &fb, const PGEnv &s, const View &v, const PGDev &d, int env, bool &err) {
    if constexpr (G == PG_GAME_JUMPER)
        if (s.opt_distribution_mode != PG_MEMORY && !jp_draw_compass(fb, s, v, d, env)) err = true;
    if constexpr (G == PG_GAME_NINJA) { // jump charge bar (ninja.cpp:155-164), get_abs_rect (:812-814)
        const float u = v.unit, bar_height = 3 * s.gs.nj.jump_charge;
        fb_fill_rectf(fb, (double)(.25f * u), (double)((float)(v.visibility - .5 - bar_height) * u), (double)(.5f * u),
                      (double)(bar_height * u), 0xff42f587u); // QColor(66, 245, 135)
    }
    if constexpr (G == PG_GAME_PLUNDER) { // juice and progress bars, get_abs_rect (:812-814)
        const float u = v.unit;
        fb_fill_rectf(fb, (double)(.25f * u), (double)(.25f * u), (double)(s.main_width * s.gs.pl.juice_left * u),
                      (double)(.5f * u), 0xff42f587u); // QColor(66, 245, 135)
        const float prog = (float)(s.main_width * (s.gs.pl.targets_hit * 1.0 / s.gs.pl.target_quota));
        fb_fill_rectf(fb, (double)(.25f * u), (double)(.75f * u), (double)(prog * u), (double)(.5f * u),
                      0xfff54290u); // QColor(245, 66, 144)
    }
}

DEV double readlane_d(double x, int j) {
    long long b = __builtin_bit_cast(long long, x);
    int lo = readlane((int)(b & 0xffffffff), j), hi = readlane((int)(b >> 32), j);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// One scale blit, all lanes cooperating over its footprint (uniform arguments).
DEV void blit_seq(const FB &fb, const PGDev &d, const Axis &ex, const Axis &ey, uint32_t soff, int sw, int mir, int ca,
                  bool &err) {
    const int nx = ex.n, ny = ey.n;
    const float inv = 1.0f / (float)nx;
    // the footprint's rows inside the pass; its pixels are distinct, so BB chunks of 64 load their
    // texels before any blend
    const int pstart = max(0, fb.y0 - ey.t1) * nx, total = min(ny, fb.y0 + fb.h - ey.t1) * nx;
    for (int p0 = pstart + LANE; p0 < total; p0 += 64 * BB) {
        uint32_t tv[BB];
        int oo[BB];
#pragma unroll
        for (int r = 0; r < BB; r++) {
            const int p = p0 + 64 * r;
            const int py = (int)(((float)p + 0.5f) * inv);
            const int pxx = p - py * nx;
            int scol = (int)((ex.base + (uint32_t)(pxx * ex.step)) >> 16);
            const int srow = (int)((ey.base + (uint32_t)(py * ey.step)) >> 16);
            if (mir) scol = sw - 1 - scol;
            const uint32_t idx = soff + (uint32_t)(srow * sw + scol);
            const int o = (ey.t1 + py) * PG_RES + ex.t1 + pxx;
            const bool in = p < total && idx < d.num_pixels && o >= 0 && o < PG_RES * PG_RES;
            if (p < total && !in) err = true;
            oo[r] = in ? o : -1;
            tv[r] = d.pixels[in ? idx : 0u];
        }
#pragma unroll
        for (int r = 0; r < BB; r++)
            if (oo[r] >= 0) fb[oo[r]] = blend_argb_pm(fb[oo[r]], tv[r], ca);
    }
}

// Transform blit of image descriptor `rd` (rot_stage): lanes = pixels of its bounding box, each
// finds its scan line's trapezoid -- the pixels qt_transform_image's row loop would touch, in any
// order, since one image's pixels are distinct.
// Descriptor (6 int4 = 96 B): a0..a2 = trapezoid k's (x_l, dx_l, x_r, dx_r), a3 = (dudx, dvdx, dudy,
// dvdy), a4 = (u0, v0, soff, iw | ih << 16), a5 = (from0 | to0 << 8 | from1 << 16 | to1 << 24,
// from2 | to2 << 8 | mir << 16, ca | xmin << 16, nx | ymin << 8 | ny << 16)
#define ROT_DESC_BYTES 96
struct RotD { int4 a0, a1, a2, a3, a4, a5; };
DEV RotD rot_desc(const uint8_t *aux, int rd) {
    const int4 *D = reinterpret_cast<const int4 *>(aux) + 6 * rd;
    RotD r;
    r.a0 = D[0]; r.a1 = D[1]; r.a2 = D[2]; r.a3 = D[3]; r.a4 = D[4]; r.a5 = D[5];
    return r;
}
DEV int rot_nx(const RotD &r) { return r.a5.w & 255; }
DEV int rot_total(const RotD &r) { return (r.a5.w & 255) * ((r.a5.w >> 16) & 255); }
// pixel p of the bounding box (inv = 1 / nx): frame offset `o`, texel index, drawn or not
DEV bool rot_pixel(const RotD &r, int p, float inv, int &o, uint32_t &idx) {
    const int xmin = r.a5.z >> 16, nx = r.a5.w & 255, ymin = (r.a5.w >> 8) & 255;
    const int py = (int)(((float)p + 0.5f) * inv);
    const int yy = ymin + py;
    const int x = xmin + (p - py * nx);
    const int f0 = r.a5.x & 255, t0 = (r.a5.x >> 8) & 255, f1 = (r.a5.x >> 16) & 255, t1 = (r.a5.x >> 24) & 255;
    const int f2 = r.a5.y & 255, t2 = (r.a5.y >> 8) & 255;
    int from;
    int4 e;
    bool in = true;
    if (yy >= f0 && yy < t0) { from = f0; e = r.a0; }
    else if (yy >= f1 && yy < t1) { from = f1; e = r.a1; }
    else if (yy >= f2 && yy < t2) { from = f2; e = r.a2; }
    else { from = 0; e = make_int4(0, 0, 0, 0); in = false; }
    const int xlv = e.x + (yy - from) * e.y, xrv = e.z + (yy - from) * e.w;
    const int fromX = max(xlv >> 16, 0), toX = min(xrv >> 16, PG_RES);
    const int iw = r.a4.w & 0xffff, ih = r.a4.w >> 16;
    int uu = (x * r.a3.x + yy * r.a3.z + r.a4.x) >> 16;
    int vv = (x * r.a3.y + yy * r.a3.w + r.a4.y) >> 16;
    uu = min(max(uu, 0), iw - 1);
    vv = min(max(vv, 0), ih - 1);
    if ((r.a5.y >> 16) & 1) uu = iw - 1 - uu;
    idx = (uint32_t)r.a4.z + (uint32_t)(vv * iw + uu);
    o = yy * PG_RES + x;
    return in && x >= fromX && x < toX;
}
DEV void rot_stamp_lds(const FB &fb, const PGDev &d, const uint8_t *aux, int rd, bool &err) {
    const RotD r = rot_desc(aux, rd);
    const int total = rot_total(r);
    if (total <= 0) return;
    const float inv = 1.0f / (float)rot_nx(r);
    // ROTB chunks of 64 pixels load their texels before any blend (one image's pixels are distinct)
    for (int p0 = LANE; p0 < total; p0 += 64 * ROTB) {
        uint32_t tv[ROTB];
        int oo[ROTB];
#pragma unroll
        for (int k = 0; k < ROTB; k++) {
            const int p = p0 + 64 * k;
            int o;
            uint32_t idx;
            bool on = p < total && rot_pixel(r, p, inv, o, idx) && fb.o_in(o);
            if (on && idx >= d.num_pixels) {
                err = true;
                on = false;
            }
            oo[k] = on ? o : -1;
            tv[k] = d.pixels[on ? idx : 0u];
        }
#pragma unroll
        for (int k = 0; k < ROTB; k++)
            if (oo[k] >= 0) fb[oo[k]] = blend_argb_pm(fb[oo[k]], tv[k], r.a5.z & 0xffff);
    }
}

#ifdef PG_PROF_STAMP
#define SPM(k) fb.sp->mark(k)
#else
#define SPM(k)
#endif
// OWN: the overlap bitmap fb.own is used (overlap_blend); false compiles it out
template <bool TILES, int EGN, bool OWN>
DEV void stamp_images(const FB &fb, const PGDev &d, const uint8_t *aux, const Img &im, unsigned long long m, bool &err);

// Rows an image can touch, for skipping it in a pass that holds none of them: plain blits, fills
// and descriptor transform blits keep their row range in ey (rot_stage sets it); the others
// (in-order transform setup, tile lists) count as the whole frame.
DEV bool img_in_pass(const Img &im, const FB &fb) {
    int lo = 0, hi = PG_RES;
    if (im.rot != 1 && im.ntile == 0) {
        lo = im.ey.t1;
        hi = im.ey.t1 + im.ey.n;
    }
    return hi > fb.y0 && lo < fb.y0 + fb.h;
}

// tile_image (basic-abstract-game.cpp:849-877) of image j: the tiles (left to right / top to
// bottom) become lanes of a plain-image list, set up lane-parallel and stamped in order.
template <int EGN, bool OWN>
DEV void stamp_tiles(const FB &fb, const PGDev &d, const uint8_t *aux, const Img &im, int j, int caj, bool &err) {
    const int ntile = readlane(im.ntile, j);
    const double rx = readlane_d(im.rx, j), ry = readlane_d(im.ry, j);
    const float tw = __builtin_bit_cast(float, readlane(__builtin_bit_cast(int, im.tw), j));
    const float th = __builtin_bit_cast(float, readlane(__builtin_bit_cast(int, im.th), j));
    const int vert = readlane(im.rslot, j); // 1: vertical tiling (negative ratio)
    const int offj = readlane(im.soff, j);
    const int swj = readlane(im.sw, j), shj = readlane(im.sh, j), mirj = readlane(im.mir, j);
    // tiles that can reach the frame (2 px margin; axis_setup culls exactly)
    const double tsz = vert ? (double)th : (double)tw, org = vert ? ry : rx;
    int tlo = 0, thi = ntile;
    if (tsz > 0) {
        tlo = max(0, (int)floor((-2.0 - org) / tsz) - 1);
        thi = min(ntile, (int)ceil((PG_RES + 2.0 - org) / tsz) + 1);
    }
    for (int t0 = tlo; t0 < thi; t0 += 64) {
        Img ti;
        img_clear(ti);
        const int t = t0 + LANE;
        if (t < thi) {
            const double x = vert ? rx : rx + (double)(tw * (float)t);
            const double y = vert ? ry + (double)(th * (float)t) : ry;
            if (axis_setup(x, (double)tw, swj, ti.ex) && axis_setup(y, (double)th, shj, ti.ey)) {
                ti.draw = true;
                ti.soff = offj; ti.sw = swj; ti.sh = shj; ti.mir = mirj; ti.ca = caj;
            }
        }
        stamp_images<false, EGN, OWN>(fb, d, aux, ti, ballot(ti.draw && img_in_pass(ti, fb)), err);
    }
}

// inclusive prefix sum over the wave's lanes
DEV int wave_incl_scan(int v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(v, off);
        if (LANE >= off) v += t;
    }
    return v;
}

DEV double shfl_d(double x, int j) {
    long long b = __builtin_bit_cast(long long, x);
    int lo = __shfl((int)(b & 0xffffffff), j), hi = __shfl((int)(b >> 32), j);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// A run of consecutive tile_image entities (`run`: their lanes in `im`, ascending; fruitbot's walls):
// their tiles, in entity order then tile order, become one plain-image list -- 64 tiles per
// stamp_images call whatever wall they belong to, so a frame's walls share gather rounds instead of
// taking at least one each.  Per wall the tiles that can reach the frame (stamp_tiles' culling); lane
// = tile, its wall found by a walk over the run's tile-count prefix, its parameters read across lanes.
template <int EGN, bool OWN>
DEV void stamp_tile_run(const FB &fb, const PGDev &d, const uint8_t *aux, const Img &im, unsigned long long run, bool &err) {
    const int lane = LANE;
    // per wall (lane = entity of the run): the first tile that can reach the frame and the tile count
    int tlo = 0, cnt = 0;
    if ((run >> lane) & 1) {
        const double tsz = im.rslot ? (double)im.th : (double)im.tw, org = im.rslot ? im.ry : im.rx;
        int thi = im.ntile;
        if (tsz > 0) {
            tlo = max(0, (int)floor((-2.0 - org) / tsz) - 1);
            thi = min(im.ntile, (int)ceil((PG_RES + 2.0 - org) / tsz) + 1);
        }
        cnt = max(thi - tlo, 0);
    }
    const int incl = wave_incl_scan(cnt), total = readlane(incl, 63);
    for (int t0 = 0; t0 < total; t0 += 64) {
        const int g = t0 + lane;
        // the wall holding tile g: the first lane of the run whose inclusive prefix exceeds g
        int lo = 0, hi = 63;
#pragma unroll
        for (int it = 0; it < 6; it++) {
            const int mid = (lo + hi) >> 1;
            if (__shfl(incl, mid) > g) hi = mid;
            else lo = mid + 1;
        }
        const int j = lo;
        const int k = g - (__shfl(incl, j) - __shfl(cnt, j)) + __shfl(tlo, j); // tile index in wall j
        const double rx = shfl_d(im.rx, j), ry = shfl_d(im.ry, j);
        const float tw = __builtin_bit_cast(float, __shfl(__builtin_bit_cast(int, im.tw), j));
        const float th = __builtin_bit_cast(float, __shfl(__builtin_bit_cast(int, im.th), j));
        const int vert = __shfl(im.rslot, j), offj = __shfl(im.soff, j), swj = __shfl(im.sw, j), shj = __shfl(im.sh, j);
        const int mirj = __shfl(im.mir, j), caj = __shfl(im.ca, j);
        Img ti;
        img_clear(ti);
        if (g < total) {
            const double x = vert ? rx : rx + (double)(tw * (float)k);
            const double y = vert ? ry + (double)(th * (float)k) : ry;
            if (axis_setup(x, (double)tw, swj, ti.ex) && axis_setup(y, (double)th, shj, ti.ey)) {
                ti.draw = true;
                ti.soff = offj; ti.sw = swj; ti.sh = shj; ti.mir = mirj; ti.ca = caj;
            }
        }
        stamp_images<false, EGN, OWN>(fb, d, aux, ti, ballot(ti.draw && img_in_pass(ti, fb)), err);
    }
}

// One image that is not batched (a transform blit set up in order, a descriptor blit or plain blit of
// more than 64 px, a tile list): all lanes over its footprint, at its turn.
template <bool TILES, int EGN, bool OWN>
DEV void stamp_big(const FB &fb, const PGDev &d, const uint8_t *aux, const Img &im, int j, bool &err) {
    const int lane = LANE;
    const uint32_t npix = d.num_pixels;
    const int caj = readlane(im.ca, j);
    const int rk = readlane(im.rot, j);
    if (rk == 2) {
        rot_stamp_lds(fb, d, aux, readlane(im.rdi, j), err);
        SPM(2);
        return;
    }
    if (rk) {
        const double m11 = readlane_d(im.m11, j);
        if (!rotated_blit(fb, d.pixels, npix, readlane_d(im.rx, j), readlane_d(im.ry, j), readlane_d(im.rw, j),
                          readlane_d(im.rh, j), m11, readlane_d(im.m12, j), readlane_d(im.m21, j), m11,
                          (uint32_t)readlane(im.soff, j), readlane(im.sw, j), readlane(im.sh, j),
                          readlane(im.mir, j) != 0, caj))
            err = true;
        SPM(3);
        return;
    }
    if (readlane(im.ntile, j) > 0) {
        if constexpr (TILES) stamp_tiles<EGN, OWN>(fb, d, aux, im, j, caj, err);
        else err = true; // unreachable: tile lists hold plain images only
        SPM(4);
        return;
    }
    const int nx = readlane(im.ex.n, j), ny = readlane(im.ey.n, j);
    if (readlane((int)im.fill, j) != 0) {
        const uint32_t col = (uint32_t)readlane((int)im.fill, j);
        const int tx = readlane(im.ex.t1, j), ty = readlane(im.ey.t1, j);
        for (int p = lane; p < nx * ny; p += 64)
            if (fb.row_in(ty + p / nx)) fb[(ty + p / nx) * PG_RES + tx + p % nx] = col;
        SPM(5);
    } else {
        Axis ex, ey;
        ex.t1 = readlane(im.ex.t1, j); ex.n = nx; ex.base = (uint32_t)readlane((int)im.ex.base, j);
        ex.step = readlane(im.ex.step, j);
        ey.t1 = readlane(im.ey.t1, j); ey.n = ny; ey.base = (uint32_t)readlane((int)im.ey.base, j);
        ey.step = readlane(im.ey.step, j);
        blit_seq(fb, d, ex, ey, (uint32_t)readlane(im.soff, j), readlane(im.sw, j), readlane(im.mir, j), caj, err);
        SPM(6);
    }
}


// Images of `m` in ascending lane order.  "Small" images (a plain blit or fill of <= 64 px, a
// descriptor transform blit whose box is <= 64 px) are drawn in batches: a run of consecutive small
// images becomes up to EGN * 64 (image, pixel) jobs, lane = job, each round's texel loads issued
// before any blend (one gather latency per batch instead of one per few images), then the batch's
// images are blended strictly in order, each from the rounds holding its jobs.  The others are drawn
// at their turn (stamp_big).  Per image the result is the reference's in-order SourceOver.
template <bool TILES, int EGN, bool OWN>
DEV void stamp_images(const FB &fb, const PGDev &d, const uint8_t *aux, const Img &im, unsigned long long m, bool &err) {
    uint32_t *const own = OWN ? fb.own : nullptr;
    constexpr int CAP = EGN * 64;
    const int lane = LANE;
    const uint32_t npix = d.num_pixels;
    SPM(7);
    // this lane's image: small or not, and its job count (its pixels, or its transform blit's box)
    int cnt = 0;
    bool small = false;
    if ((m >> lane) & 1) {
        if (im.rot == 2) {
            const int tot = rot_total(rot_desc(aux, im.rdi));
            small = tot <= 64;
            cnt = tot;
        } else if (im.rot == 0 && im.ntile == 0) {
            const int t = im.ex.n * im.ey.n;
            small = t <= 64;
            cnt = t;
        }
    }
    const unsigned long long smask = ballot(small);
    // tile_image entities (plain images tiled, no transform): batched per run (stamp_tile_run)
    const unsigned long long tmask = TILES ? ballot(((m >> lane) & 1) && im.rot == 0 && im.ntile > 0) : 0ull;
    while (m) {
        const int j0 = __ffsll((long long)m) - 1;
        if (!((smask >> j0) & 1)) {
            if constexpr (TILES) {
                if (((tmask >> j0) & 1) && RUN_TILES) { // a run of tile lists: their tiles batched together
                    const unsigned long long other = m & ~tmask;
                    const unsigned long long below = other ? ((1ull << (__ffsll((long long)other) - 1)) - 1) : ~0ull;
                    const unsigned long long run = m & tmask & below;
                    m &= ~run;
                    stamp_tile_run<EGN, OWN>(fb, d, aux, im, run, err);
                    asm volatile("" ::: "memory");
                    continue;
                }
            }
            m &= m - 1;
            stamp_big<TILES, EGN, OWN>(fb, d, aux, im, j0, err);
            asm volatile("" ::: "memory");
            continue;
        }
        // the run of small images up to the next big one, cut where its jobs exceed CAP
        const unsigned long long big = m & ~smask;
        const unsigned long long run = big ? (m & ((1ull << (__ffsll((long long)big) - 1)) - 1)) : m;
        const int v = ((run >> lane) & 1) ? cnt : 0;
        const int incl = wave_incl_scan(v), excl = incl - v;
        const unsigned long long bm = run & ballot(incl <= CAP);
        const int total = readlane(incl, 63 - __clzll(bm));
        m &= ~bm;
        // fetch: job q -> its image jj (the first lane whose inclusive prefix exceeds q), pixel q - excl.
        // The cross-lane reads (ds_bpermute) run with every lane active: a lane the branch would
        // disable does not supply its value.
        uint32_t tv[EGN];
        int fo[EGN], car[EGN];
        uint32_t part = 0;
#pragma unroll
        for (int r = 0; r < EGN; r++) {
            tv[r] = 0;
            fo[r] = -1;
            if (r * 64 >= total) continue; // uniform
            const int q = r * 64 + lane;
            const bool live = q < total;
            const int qq = live ? q : 0;
#ifdef PG_STAMP_LINEAR
            int jj = 0;
            for (unsigned long long bb = bm; bb; bb &= bb - 1) {
                const int j = __ffsll((long long)bb) - 1;
                if (qq >= readlane(excl, j) && qq < readlane(incl, j)) jj = j;
            }
#else
            int lo = 0, hi = 63;
#pragma unroll
            for (int it = 0; it < 6; it++) {
                const int mid = (lo + hi) >> 1;
                if (__shfl(incl, mid) > qq) hi = mid;
                else lo = mid + 1;
            }
            const int jj = lo;
#endif
            const int p = qq - __shfl(excl, jj);
            const int rk = __shfl(im.rot, jj), rdi = __shfl(im.rdi, jj);
            const int nx = __shfl(im.ex.n, jj), ext1 = __shfl(im.ex.t1, jj), eyt1 = __shfl(im.ey.t1, jj);
            const uint32_t fillj = (uint32_t)__shfl((int)im.fill, jj);
            const int swj = __shfl(im.sw, jj), mirj = __shfl((int)im.mir, jj), soffj = __shfl((int)im.soff, jj);
            const uint32_t exb = (uint32_t)__shfl((int)im.ex.base, jj), eyb = (uint32_t)__shfl((int)im.ey.base, jj);
            const int exs = __shfl(im.ex.step, jj), eys = __shfl(im.ey.step, jj);
            car[r] = own ? __shfl(im.ca, jj) : 0; // uniform
            int o = -1;
            uint32_t t = 0;
            bool ok = false;
            if (live) {
                if (rk == 2) {
                    const RotD rd = rot_desc(aux, rdi);
                    uint32_t idx;
                    if (rot_pixel(rd, p, 1.0f / (float)rot_nx(rd), o, idx) && fb.o_in(o)) {
                        if (idx < npix) {
                            t = d.pixels[idx];
                            ok = true;
                        } else {
                            err = true;
                        }
                    }
                } else {
                    const float inv = 1.0f / (float)nx;
                    const int py = (int)(((float)p + 0.5f) * inv);
                    const int pxx = p - py * nx;
                    o = (eyt1 + py) * PG_RES + ext1 + pxx;
                    if (!fb.o_in(o)) {
                        // another pass's row
                    } else if (fillj != 0) {
                        t = fillj;
                        ok = true;
                    } else {
                        int scol = (int)((exb + (uint32_t)(pxx * exs)) >> 16);
                        const int srow = (int)((eyb + (uint32_t)(py * eys)) >> 16);
                        if (mirj) scol = swj - 1 - scol;
                        const uint32_t idx = (uint32_t)soffj + (uint32_t)(srow * swj + scol);
                        if (idx < npix) {
                            t = d.pixels[idx];
                            ok = true;
                        } else {
                            err = true;
                        }
                    }
                }
            }
            // selects, not a conditional store: a conditional assignment into the tv / fo arrays was
            // miscompiled (gfx950, hipcc of ROCm 7.2: the texel path's offset lost in a 64-bit
            // register-pair copy of the array) -- parity caught it on coinrun
            tv[r] = ok ? t : 0u;
            fo[r] = ok ? o : -1;
        }
#ifdef PG_STAMP_DEBUG
        {
            const unsigned long long f0 = ballot(fo[0] >= 0), lv = ballot(lane < total);
            if ((bm & 1ull) && d.prof && lane == 0) {
                uint64_t *P = d.prof + (size_t)blockIdx.x * 16;
                P[0] = (uint64_t)total; P[1] = (uint64_t)incl; P[2] = (uint64_t)cnt; P[3] = (uint64_t)im.ex.n;
                P[4] = (uint64_t)im.ey.n; P[5] = bm; P[6] = run; P[7] = smask; P[8] = f0; P[9] = lv;
                P[10] = (uint64_t)fb.y0; P[11] = (uint64_t)im.ey.t1; P[12] = (uint64_t)im.ex.t1; P[13] += 1;
            }
        }
#endif
#pragma unroll
        for (int r = 0; r < EGN; r++) part |= fo[r] >= 0 ? alpha_partial(tv[r]) : 0u;
        const bool binary = ballot(part != 0) == 0; // every fetched texel has alpha 0 or 255
        SPM(0);
        // Overlap test: each job sets its pixel's bit in the pass bitmap; a bit already set means two images
        // of the batch share a pixel (an image's own jobs are distinct pixels).  Without overlap every pixel
        // of the batch is drawn by one image only, so the in-order result is each job's blend over the pixel
        // as it stands: one read-modify-write per round instead of one per image and round.
        bool clash = own == nullptr; // the games without the bitmap keep the per-image order
#pragma unroll
        for (int r = 0; r < EGN; r++) {
            if (r * 64 >= total || !own) continue; // uniform
            if (fo[r] >= 0) {
                const int o = fo[r] - fb.y0 * PG_RES;
                const uint32_t bit = 1u << (o & 31);
                clash |= (atomicOr(own + (o >> 5), bit) & bit) != 0;
            }
        }
        const bool overlap = !OWN || ballot(clash) != 0; // (ballot of a constant is not one: exec may be 0)
#pragma unroll
        for (int r = 0; r < EGN; r++) { // back to zero for the next batch
            if (r * 64 >= total || !own) continue;
            if (fo[r] >= 0) own[(fo[r] - fb.y0 * PG_RES) >> 5] = 0u;
        }
        if (!overlap) {
#pragma unroll
            for (int r = 0; r < EGN; r++) {
                if (r * 64 >= total) continue; // uniform
                if (fo[r] >= 0)
                    fb[fo[r]] = (binary && car[r] == 256) ? over_binary(fb[fo[r]], tv[r]) : blend_argb_pm(fb[fo[r]], tv[r], car[r]);
            }
            asm volatile("" ::: "memory");
            SPM(1);
            continue;
        }
        // blend, image by image in order, from the rounds that hold its jobs
        unsigned long long b = bm;
        while (b) {
            const int j = __ffsll((long long)b) - 1;
            b &= b - 1;
            const int jb = readlane(excl, j), je = readlane(incl, j), caj = readlane(im.ca, j);
            const bool ob = binary && caj == 256;
#pragma unroll
            for (int r = 0; r < EGN; r++) {
                if (jb >= (r + 1) * 64 || je <= r * 64) continue; // uniform
                const int q = r * 64 + lane;
                if (q >= jb && q < je && fo[r] >= 0)
                    fb[fo[r]] = ob ? over_binary(fb[fo[r]], tv[r]) : blend_argb_pm(fb[fo[r]], tv[r], caj);
            }
            // no hardware barrier between images (one wave issues its LDS operations in order), but a
            // compiler one: images of one round use the same per-lane address register (fo[r]) under
            // disjoint lane masks, and nothing else stops the compiler from keeping a lane's pixel in
            // a register across the loop -- the next image's lanes must read what this image's wrote
            asm volatile("" ::: "memory");
        }
        SPM(1);
    }
}

// Blit geometry of entity i (draw_entity -> get_object_rect -> draw_image, basic-abstract-game.cpp
// :808-826, 886-922, 1056-1059) into this lane's Img.
template <int G>
DEV void entity_setup(const PGDev &d, const PGEnv &s, const View &v, int env, int i, int n, int player_img, Img &im,
                      bool &err) {
    img_clear(im);
    if (i >= n) return;
    im.ez = EIr(d, F_RENDER_Z, env, i);
    float px_ = EFr(d, F_X, env, i), py_ = EFr(d, F_Y, env, i);
    float prx = EFr(d, F_RX, env, i), pry = EFr(d, F_RY, env, i);
    int flags = EIr(d, F_FLAGS, env, i);
    float alpha = EFr(d, F_ALPHA, env, i);
    float rotation = EFr(d, F_ROTATION, env, i);
    int etype = EIr(d, F_TYPE, env, i);
    int itype = EIr(d, F_IMAGE_TYPE, env, i);
    int theme = EIr(d, F_IMAGE_THEME, env, i);
    int img = image_for_type<G>(s, itype, player_img);
    if (img < 0 || !should_draw<G>(s, etype, theme)) return;
    // draw_grid_obj (monochrome / >= USE_ASSET_THRESHOLD) fills the unadjusted object rect;
    // rotation, reflection and alpha are unused there
    const bool grid_obj = s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD;
    if (grid_obj) {
        if (img == SPACE) return;
        if (!s.opt_use_monochrome_assets) { // color_for_type fasserts without monochrome (:467-487)
            err = true;
            return;
        }
    } else {
        theme = mask_theme<G>(s, theme, img);
        if (theme < 0 || theme >= 10) {
            err = true;
            return;
        }
    }
    double rx, ry, rw, rh;
    if (flags & EF_ABS_COORDS) { // get_abs_rect (:812-814) via get_object_rect (:820-826)
        float vd = v.view_dim;
        float ax = vd * (px_ - prx), ay = vd * (py_ + pry), aw = 2 * vd * prx, ah = 2 * vd * pry;
        rx = (double)(ax * v.unit); ry = (double)(ay * v.unit);
        rw = (double)(aw * v.unit); rh = (double)(ah * v.unit);
    } else {
        screen_rect(v, px_ - prx, py_ + pry, 2 * prx, 2 * pry, 0, rx, ry, rw, rh);
    }
    if (grid_obj) {
        if (!mono_fill<G>(s, img, theme, rx, ry, rw, rh, im)) err = true;
        return;
    }
    if constexpr (G == PG_GAME_COINRUN) {
        if (is_player_image(img)) { // coinrun get_adjusted_image_rect (coinrun.cpp:64-70)
            rx = rx + rw * 0.0;
            ry = ry + rh * -.7415;
            rw = rw * 1.0;
            rh = rh * 1.7415;
        }
    }
    if constexpr (G == PG_GAME_LEAPER) {
        if (img == PLAYER) { // leaper get_adjusted_image_rect (leaper.cpp:244-250)
            rx = rx + rw * 0.0;
            ry = ry + rh * -.275;
            rw = rw * 1.0;
            rh = rh * 1.55;
        }
    }
    int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
    im.ca = alpha != 1 ? qt_int_opacity((double)alpha) : 256;
    im.mir = (flags & EF_REFLECTED) != 0;
    im.soff = sp.x;
    im.sw = sp.y;
    im.sh = sp.z;
    if (sp.y <= 0) {
        err = true; // missing image
    } else if (!has_rotation<G>() && rotation != 0) {
        err = true; // not reachable in this game (has_rotation)
    } else if (has_rotation<G>() && rotation != 0) {
        // rotated: the Qt transform blit runs in order when this entity is stamped
        int rslot = -1;
        for (int k = 0; k < PG_ROT_N; k++)
            if (__float_as_uint(d.rot_angles[k]) == __float_as_uint(rotation)) rslot = k;
        // rslot < 0: an angle outside the host table, its matrix is built on the device
        // (qt_rotation_matrix), by this entity's lane, before the in-order stamping
        double mt[4];
        if (rslot >= 0) {
            const double *tm = d.rot_table + 4 * rslot;
            mt[0] = tm[0]; mt[1] = tm[1]; mt[2] = tm[2]; mt[3] = tm[3];
        } else {
            qt_rotation_matrix(rotation, mt);
        }
        if (mt[3] != mt[0]) err = true; // a rotation matrix has m22 == m11
        im.m11 = mt[0]; im.m12 = mt[1]; im.m21 = mt[2];
        im.rslot = rslot;
        im.tw = rotation;
        im.draw = true;
        im.rot = 1;
        im.rx = rx; im.ry = ry; im.rw = rw; im.rh = rh;
    } else if (has_tiled_entities<G>() && tile_aspect_ratio<G>(etype, prx, pry) != 0) {
        float tile_ratio = tile_aspect_ratio<G>(etype, prx, pry);
        int num_tiles;
        if (tile_ratio < 0) {
            tile_ratio = -1 * tile_ratio;
            num_tiles = (int)(rh / (rw * tile_ratio));
            if (num_tiles < 1) num_tiles = 1;
            im.th = (float)(rh / num_tiles);
            im.tw = (float)rw;
            im.rslot = 1;
        } else {
            num_tiles = (int)(rw / (rh * tile_ratio));
            if (num_tiles < 1) num_tiles = 1;
            im.tw = (float)(rw / num_tiles);
            im.th = (float)rh;
            im.rslot = 0;
        }
        im.ntile = num_tiles;
        im.rx = rx; im.ry = ry; im.rw = rw; im.rh = rh;
        // the tiles lie inside the rect (up to float rounding of the tile size): a rect 2 px clear
        // of the frame draws nothing (fruitbot's walls off screen)
        im.draw = rx + rw > -2 && rx < PG_RES + 2 && ry + rh > -2 && ry < PG_RES + 2;
    } else if (axis_setup(rx, rw, sp.y, im.ex) && axis_setup(ry, rh, sp.z, im.ey)) {
        im.draw = true;
    }
}

// Transform blits of a chunk's rotated images, set up lane-parallel: a TxScale map becomes a plain
// scale blit, a rotation's trapezoids and texture stepping go to descriptor slot `rank` in the aux
// LDS (dead once the tiles are drawn); past `cap` descriptors an image keeps the in-order setup.
// Descriptor slots start at `base` (the register-frame kernel continues the numbering over chunks);
// returns the number of images that wanted a descriptor.
DEV int rot_stage(Img &im, uint8_t *aux, int cap, int base = 0) {
    const int lane = LANE;
    Axis ex, ey;
    RotGeo g;
    int kind = 0;
    const bool cand = im.draw && im.rot == 1;
    if (cand) kind = rot_prepare(im.rx, im.ry, im.rw, im.rh, im.m11, im.m12, im.m21, im.m11, im.sw, im.sh, ex, ey, g);
    if (cand && kind == 0) im.draw = false;
    if (cand && kind == 1) { im.rot = 0; im.ex = ex; im.ey = ey; }
    const bool gen = cand && kind == 2;
    const unsigned long long gm = ballot(gen);
    const int rank = base + __popcll(gm & ((1ull << lane) - 1));
    if (gen && rank < cap) {
        int ymin = PG_RES, ymax = 0, xmin = PG_RES, xmax = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const Trap T = g.tr[k];
            if (T.from_y >= T.to_y) continue;
            ymin = min(ymin, T.from_y);
            ymax = max(ymax, T.to_y);
#pragma unroll
            for (int e = 0; e < 2; e++) { // fromX / toX are monotone in y: extremes at the end rows
                const int yy = e ? T.to_y - 1 : T.from_y;
                const int xl = T.x_l + (yy - T.from_y) * T.dx_l, xr = T.x_r + (yy - T.from_y) * T.dx_r;
                xmin = min(xmin, max(xl >> 16, 0));
                xmax = max(xmax, min(xr >> 16, PG_RES));
            }
        }
        const int nx = xmax > xmin ? xmax - xmin : 0, ny = ymax > ymin ? ymax - ymin : 0;
        // trap_setup clamps from / to to [0, 64]; an empty trapezoid is stored as 0..0
        int ft[3];
#pragma unroll
        for (int k = 0; k < 3; k++)
            ft[k] = g.tr[k].from_y < g.tr[k].to_y ? (g.tr[k].from_y | (g.tr[k].to_y << 8)) : 0;
        int4 *D = reinterpret_cast<int4 *>(aux) + 6 * rank;
        D[0] = make_int4(g.tr[0].x_l, g.tr[0].dx_l, g.tr[0].x_r, g.tr[0].dx_r);
        D[1] = make_int4(g.tr[1].x_l, g.tr[1].dx_l, g.tr[1].x_r, g.tr[1].dx_r);
        D[2] = make_int4(g.tr[2].x_l, g.tr[2].dx_l, g.tr[2].x_r, g.tr[2].dx_r);
        D[3] = make_int4(g.dudx, g.dvdx, g.dudy, g.dvdy);
        D[4] = make_int4(g.u0, g.v0, im.soff, (im.sw & 0xffff) | (im.sh << 16));
        D[5] = make_int4(ft[0] | (ft[1] << 16), ft[2] | ((im.mir ? 1 : 0) << 16), (im.ca & 0xffff) | (xmin << 16),
                         (nx & 255) | ((ymin & 255) << 8) | ((ny & 255) << 16));
        im.rot = 2;
        im.rdi = rank;
        im.ey.t1 = ymin; // the rows it covers, for the pass filter (ey is otherwise unused here)
        im.ey.n = ny;
    }
    return __popcll(gm);
}

// ------------------------------------------------------------------ general pixel-centric tile pass
// draw_foreground's grid loop (basic-abstract-game.cpp:930-964) for any mix of tile image sizes and
// draw_grid_obj fills, lane = screen column like the fast path.  Every drawable grid value of the game
// gets a typeinfo slot; tile images of one (w, h) -- or one fill geometry -- form a class, and the Qt
// blit setup (axis_setup / fillRect edges) of every window column and row is computed once per class.
// A pixel then blends the <= 2 x 2 tiles covering it in x-major / y-minor order: first tile column in
// the row pass (the background fused in when no z = -1 entity has to go between them), the second
// tile column of the few screen columns two tiles overlap in a lane = row pass.  Frames this cannot
// express (more classes than GEN_K, a window wider than 63 or larger than GEN_GW cells, a grid value
// outside the table, 3 tiles covering one pixel) take the stamped generic pass instead.
#define GEN_K 4       // tile classes per frame (their setup tables fill the 8 KB pass frame)
#define GEN_GW 1024   // window cells (u8 slot per cell)
#define GEN_NOTHING 64
#define GEN_BAD 15
template <int G>
DEV constexpr bool has_general() { return has_grid_tiles<G>() && !always_uniform<G>(); }
// aux LDS: typeinfo (65 int2) | window slots (GEN_GW u8) | xs0, xs1, ys0, ys1 (GEN_K x 64 int16 each)
#define GEN_TI_BYTES (65 * 8)
#define GEN_AUX_BYTES (GEN_TI_BYTES + GEN_GW + 4 * GEN_K * 64 * 2)
// typeinfo slot <-> grid value: values 0..62 map to themselves; chaser's ORB (1002) takes slot 63
template <int G>
DEV int gen_slot_type(int slot) {
    if constexpr (G == PG_GAME_CHASER) if (slot == 63) return CH_ORB;
    return slot;
}
template <int G>
DEV int gen_slot(int type) { // GEN_NOTHING: not drawn; -1: not on this path
    if (type == INVALID_OBJ || type == SPACE) return GEN_NOTHING;
    if constexpr (G == PG_GAME_CHASER) {
        if (type == CH_ORB) return 63;
        if (type == 63) return -1;
    }
    return (type >= 0 && type < 64) ? type : -1;
}

// fillRect(QRectF) edges of one axis (fill_setup), clipped to the frame
DEV bool fill_axis(double x, double w, Axis &a) {
    int x1 = qRound(x), x2 = qRound(x + w);
    if (x2 < x1) { int t = x1; x1 = x2; x2 = t; }
    x1 = max(x1, 0); x2 = min(x2, PG_RES);
    a.t1 = x1; a.n = x2 - x1; a.base = 0; a.step = 0;
    return x1 < x2;
}
// one axis of a class: kind 1 = Qt scale blit of an image of `isz` px, 2 = fillRect of the tile rect
// (monochrome draw_grid_obj), 3 = chaser's orb fillRect (chaser.cpp:111-117 via grid_obj_fill)
DEV bool class_axis(int kind, int isz, double r, double rw, Axis &a) {
    a.t1 = a.n = 0; a.base = 0; a.step = 0;
    if (kind == 1) return axis_setup(r, rw, isz, a);
    if (kind == 2) return fill_axis(r, rw, a);
    if (kind == 3) {
        const float dim = 0.3f, k = 1 - dim;
        return fill_axis(r + rw * k / 2, rw * dim, a);
    }
    return false;
}

struct GenLane {
    int cx0, cx1, ncx; // lane = screen column: covering window columns (relative to low_x)
    int ry0, ry1, ncy; // lane = screen row: covering window rows (relative to low_y)
};

// Builds the class tables (scratch in `tmp`, >= 2 * GEN_K * 64 int4, dead afterwards) and the
// per-lane coverage (wave-uniform result): 0 = the frame is not expressible, 1 = draw it with
// gen_draw, 2 = the window holds no drawn tile (nothing to draw).
template <int G>
DEV int gen_setup(const PGDev &d, const PGEnv &s, const View &v, const int16_t *Gd, int player_img, int low_x,
                   int low_y, int ww, int wh, int xg, int yg, uint8_t *aux, int4 *tmp, GenLane &gl) {
    const int lane = LANE;
    int2 *ti = reinterpret_cast<int2 *>(aux);
    uint8_t *gw = aux + GEN_TI_BYTES;
    int16_t *xs0 = reinterpret_cast<int16_t *>(aux + GEN_TI_BYTES + GEN_GW);
    int16_t *xs1 = xs0 + GEN_K * 64, *ys0 = xs1 + GEN_K * 64, *ys1 = ys0 + GEN_K * 64;
    int4 *xt = tmp, *yt = tmp + GEN_K * 64;
    if (ww > 63 || wh > 63 || ww * wh > GEN_GW) return 0;
    // ---- typeinfo (lane = slot): what draw_foreground does with this grid value
    int kind = 0, off = 0, iw = 0, ih = 0;
    {
        const int t = gen_slot_type<G>(lane);
        const int img = image_for_type<G>(s, t, player_img);
        if (img >= 0) {
            if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) { // draw_grid_obj (:924-928)
                if (img != SPACE) {
                    if (G == PG_GAME_CHASER && img == CH_ORB) {
                        kind = 3; off = (int)0xff00ff00u;
                    } else if (s.opt_use_monochrome_assets) {
                        const uint32_t col = color_for_type<G>(s, img, grid_theme<G>(s, t));
                        if (col == 0) kind = GEN_BAD;
                        else { kind = 2; off = (int)(col | 0xff000000u); }
                    } else {
                        kind = GEN_BAD;
                    }
                }
            } else {
                const int theme = mask_theme<G>(s, grid_theme<G>(s, t), img);
                const int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                if (sp.y > 0) { kind = 1; off = sp.x; iw = sp.y; ih = sp.z; }
                else if (!missing_image_ok<G>(img)) kind = GEN_BAD;
            }
        }
    }
    // ---- window grid -> slot (u8), and which slots the window holds; a cell this path cannot
    //      draw sends the frame to the generic pass
    bool bad = false;
    unsigned long long present = 0;
    for (int c = lane; c < ww * wh; c += 64) {
        const int x = low_x + c % ww, y = low_y + c / ww;
        const int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x]
                                                                                   : s.out_of_bounds_object;
        int sl = gen_slot<G>(type);
        if (sl < 0) { bad = true; sl = GEN_NOTHING; }
        if (sl < 64) present |= 1ull << sl;
        gw[c] = (uint8_t)sl;
    }
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const uint32_t lo = (uint32_t)present, hi = (uint32_t)(present >> 32);
        present |= (unsigned long long)(uint32_t)__shfl_xor((int)lo, sh) | ((unsigned long long)(uint32_t)__shfl_xor((int)hi, sh) << 32);
    }
    const bool here = (present >> lane) & 1;
    if (here && kind == GEN_BAD) bad = true;
    if (ballot(bad)) return 0;
    // ---- classes: one per distinct (kind, w, h) among the slots the window holds
    const bool drawn = here && kind >= 1 && kind <= 3;
    const int key = kind == 1 ? (iw | (ih << 12) | (1 << 24)) : (kind << 24);
    unsigned long long pend = ballot(drawn);
    int cls = 0, K = 0;
    int ck[GEN_K], cw[GEN_K], chh[GEN_K];
#pragma unroll
    for (int k = 0; k < GEN_K; k++) ck[k] = cw[k] = chh[k] = 0;
    while (pend) {
        const int f = __ffsll((long long)pend) - 1;
        const int kf = readlane(key, f);
        const unsigned long long mem = ballot(drawn && key == kf);
        if (K < GEN_K) {
            if (drawn && key == kf) cls = K;
#pragma unroll
            for (int k = 0; k < GEN_K; k++)
                if (k == K) { ck[k] = readlane(kind, f); cw[k] = readlane(iw, f); chh[k] = readlane(ih, f); }
        }
        K++;
        pend &= ~mem;
    }
    if (K > GEN_K) return 0;
    if (K == 0) return 2;
    ti[lane] = drawn ? make_int2(off, iw | (cls << 16) | (kind << 24)) : make_int2(0, 0);
    if (lane == 0) ti[GEN_NOTHING] = make_int2(0, 0);
    // ---- per class: the blit / fill setup of window column `lane` and window row `lane`
    {
        double rx = 0, rw = 0, ry = 0, rh = 0, t0, t1;
        if (lane < ww) screen_rect(v, (float)(low_x + lane), 0.0f, 1, 1, RENDER_EPS, rx, t0, rw, t1);
        if (lane < wh) screen_rect(v, 0.0f, (float)(low_y + lane + 1), 1, 1, RENDER_EPS, t0, ry, t1, rh);
#pragma unroll
        for (int k = 0; k < GEN_K; k++) {
            if (k >= K) break;
            Axis a, b;
            const bool okx = lane < ww && class_axis(ck[k], cw[k], rx, rw, a);
            const bool oky = lane < wh && class_axis(ck[k], chh[k], ry, rh, b);
            xt[k * 64 + lane] = make_int4(a.t1, okx ? a.n : 0, (int)a.base, a.step);
            yt[k * 64 + lane] = make_int4(b.t1, oky ? b.n : 0, (int)b.base, b.step);
        }
    }
    wave_sync();
    // ---- coverage: lane = screen column (columns), lane = screen row (rows); <= 2 each
    gl.cx0 = gl.cx1 = gl.ry0 = gl.ry1 = -1;
    gl.ncx = gl.ncy = 0;
    for (int x = xg - 2; x <= xg + 2; x++) {
        const int i = x - low_x;
        if (i < 0 || i >= ww) continue;
        bool cov = false;
        for (int k = 0; k < K; k++) {
            const int4 t = xt[k * 64 + i];
            cov |= t.y > 0 && lane >= t.x && lane < t.x + t.y;
        }
        if (cov) {
            if (gl.ncx == 0) gl.cx0 = i; else if (gl.ncx == 1) gl.cx1 = i; else bad = true;
            gl.ncx++;
        }
    }
    for (int y = yg - 2; y <= yg + 2; y++) {
        const int j = y - low_y;
        if (j < 0 || j >= wh) continue;
        bool cov = false;
        for (int k = 0; k < K; k++) {
            const int4 t = yt[k * 64 + j];
            cov |= t.y > 0 && lane >= t.x && lane < t.x + t.y;
        }
        if (cov) {
            if (gl.ncy == 0) gl.ry0 = j; else if (gl.ncy == 1) gl.ry1 = j; else bad = true;
            gl.ncy++;
        }
    }
    if (ballot(bad)) return 0;
    // ---- per class: source column of this lane's covering columns, source row of this row's
    for (int k = 0; k < K; k++) {
        int v0 = -1, v1 = -1, w0 = -1, w1 = -1;
        if (gl.ncx > 0) {
            const int4 t = xt[k * 64 + gl.cx0];
            if (t.y > 0 && lane >= t.x && lane < t.x + t.y) v0 = (int)(((uint32_t)t.z + (uint32_t)((lane - t.x) * t.w)) >> 16);
        }
        if (gl.ncx > 1) {
            const int4 t = xt[k * 64 + gl.cx1];
            if (t.y > 0 && lane >= t.x && lane < t.x + t.y) v1 = (int)(((uint32_t)t.z + (uint32_t)((lane - t.x) * t.w)) >> 16);
        }
        if (gl.ncy > 0) {
            const int4 t = yt[k * 64 + gl.ry0];
            if (t.y > 0 && lane >= t.x && lane < t.x + t.y) w0 = (int)(((uint32_t)t.z + (uint32_t)((lane - t.x) * t.w)) >> 16);
        }
        if (gl.ncy > 1) {
            const int4 t = yt[k * 64 + gl.ry1];
            if (t.y > 0 && lane >= t.x && lane < t.x + t.y) w1 = (int)(((uint32_t)t.z + (uint32_t)((lane - t.x) * t.w)) >> 16);
        }
        xs0[k * 64 + lane] = (int16_t)v0; xs1[k * 64 + lane] = (int16_t)v1;
        ys0[k * 64 + lane] = (int16_t)w0; ys1[k * 64 + lane] = (int16_t)w1;
    }
    wave_sync();
    return 1;
}

// texel of window cell `cell` at source column table `xs` (per class, this lane) / row `sr` table
DEV uint32_t gen_texel(const PGDev &d, const int2 t, int sc, int sr, bool &err) {
    const int kind = t.y >> 24;
    if (kind == 0 || sc < 0 || sr < 0) return 0u;
    if (kind != 1) return (uint32_t)t.x;
    const uint32_t idx = (uint32_t)t.x + (uint32_t)(sr * (t.y & 0xffff) + sc);
    if (idx >= d.num_pixels) { err = true; return 0u; }
    return d.pixels[idx];
}

// Row pass (first covering tile column) + second-column pass.  FUSE: the background texel of the
// pixel (bg_col / bg_base / bgrow as in the fast path) is the destination; else the frame buffer.
template <bool FUSE>
DEV void gen_draw(const FB &fb, const PGDev &d, const uint32_t *bgpix, const uint8_t *aux, const GenLane &gl, int ww, bool bg_col,
                  uint32_t bg_base, int bgrow, bool &err) {
    const int lane = LANE;
    const int2 *ti = reinterpret_cast<const int2 *>(aux);
    const uint8_t *gw = aux + GEN_TI_BYTES;
    const int16_t *xs0 = reinterpret_cast<const int16_t *>(aux + GEN_TI_BYTES + GEN_GW);
    const int16_t *xs1 = xs0 + GEN_K * 64, *ys0 = xs1 + GEN_K * 64, *ys1 = ys0 + GEN_K * 64;
    // per screen row (lane = row): its covering window rows, packed for one readlane per row
    const int rinfo = gl.ncy == 0 ? 0 : (gl.ry0 | ((gl.ncy > 1 ? gl.ry1 : 0) << 8) | (gl.ncy << 16));
    const int cxo = gl.ncx > 0 ? gl.cx0 : -1;
    for (int r0 = fb.y0; r0 < fb.y0 + fb.h; r0 += RB) {
        int info[RB], s0[RB], s1[RB];
        int2 t0[RB], t1[RB];
        uint32_t dst[RB], ta[RB], tb[RB];
#pragma unroll
        for (int k = 0; k < RB; k++) {
            info[k] = readlane(rinfo, r0 + k);
            const int ny = info[k] >> 16;
            s0[k] = (ny > 0 && cxo >= 0) ? gw[(info[k] & 255) * ww + cxo] : GEN_NOTHING;
            s1[k] = (ny > 1 && cxo >= 0) ? gw[((info[k] >> 8) & 255) * ww + cxo] : GEN_NOTHING;
        }
#pragma unroll
        for (int k = 0; k < RB; k++) {
            t0[k] = ti[s0[k]];
            t1[k] = ti[s1[k]];
        }
#pragma unroll
        for (int k = 0; k < RB; k++) {
            const int c0 = (t0[k].y >> 16) & 255, c1 = (t1[k].y >> 16) & 255;
            ta[k] = gen_texel(d, t0[k], xs0[c0 * 64 + lane], ys0[c0 * 64 + r0 + k], err);
            tb[k] = gen_texel(d, t1[k], xs0[c1 * 64 + lane], ys1[c1 * 64 + r0 + k], err);
        }
        if constexpr (FUSE) {
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int br = readlane(bgrow, r0 + k);
                const bool inb = bg_col && br >= 0;
                const uint32_t px = bgpix[inb ? bg_base + (uint32_t)br : 0u];
                dst[k] = inb ? px : 0xff000000u;
            }
        } else {
#pragma unroll
            for (int k = 0; k < RB; k++) dst[k] = fb[(r0 + k) * PG_RES + lane];
        }
        uint32_t part = 0;
#pragma unroll
        for (int k = 0; k < RB; k++) part |= alpha_partial(ta[k]) | alpha_partial(tb[k]);
        if (!ballot(part != 0)) {
#pragma unroll
            for (int k = 0; k < RB; k++) fb[(r0 + k) * PG_RES + lane] = over_binary(over_binary(dst[k], ta[k]), tb[k]);
        } else {
#pragma unroll
            for (int k = 0; k < RB; k++) {
                uint32_t px = dst[k];
                px = ta[k] + BYTE_MUL(px, (~ta[k]) >> 24);
                px = tb[k] + BYTE_MUL(px, (~tb[k]) >> 24);
                fb[(r0 + k) * PG_RES + lane] = px;
            }
        }
    }
    wave_sync();
    // second covering tile column of the screen columns two tiles overlap; lane = screen row
    unsigned long long m2 = ballot(gl.ncx > 1);
    while (m2) {
        const int c = __ffsll((long long)m2) - 1;
        m2 &= m2 - 1;
        const int x1 = readlane(gl.cx1, c);
        const int row = lane;
        if (gl.ncy > 0 && fb.row_in(row)) {
            uint32_t px = fb[row * PG_RES + c];
            for (int l = 0; l < gl.ncy; l++) {
                const int2 t = ti[gw[(l ? gl.ry1 : gl.ry0) * ww + x1]];
                const int cl = (t.y >> 16) & 255;
                const uint32_t tv = gen_texel(d, t, xs1[cl * 64 + c], (l ? ys1 : ys0)[cl * 64 + row], err);
                px = tv + BYTE_MUL(px, (~tv) >> 24);
            }
            fb[row * PG_RES + c] = px;
        }
    }
}

// The agent's image and prepare_for_drawing(rect_height = 64) (basic-abstract-game.cpp:828-847)
// with choose_center (:673-676; climber.cpp:291-295, fruitbot.cpp:138-142).
template <int G>
DEV View prepare_view(const PGDev &d, const PGEnv &s, int env, int &player_img) {
    float agent_x, agent_y, agent_vx;
    if (s.agent_erased) {
        agent_x = s.ghost_x; agent_y = s.ghost_y; agent_vx = s.ghost_vx;
    } else {
        agent_x = EFr(d, F_X, env, 0); agent_y = EFr(d, F_Y, env, 0); agent_vx = EFr(d, F_VX, env, 0);
    }
    player_img = player_image<G>(s, agent_vx);
    View v;
    v.center_x = (float)(s.main_width * .5);
    v.center_y = (float)(s.main_height * .5);
    v.visibility = s.visibility;
    if (s.opt_center_agent) {
        if constexpr (G == PG_GAME_CLIMBER) {
            const float agent_ry = s.agent_erased ? s.ghost_ry : EFr(d, F_RY, env, 0);
            v.center_x = (float)(s.main_width / 2.0);
            v.center_y = (float)((double)agent_y + s.main_width / 2.0 - (double)(5 * agent_ry));
            v.visibility = (float)s.main_width;
        } else if constexpr (G == PG_GAME_FRUITBOT) {
            const float agent_ry = s.agent_erased ? s.ghost_ry : EFr(d, F_RY, env, 0);
            v.center_x = (float)(s.main_width / 2.0);
            v.center_y = (float)((double)agent_y + s.main_width / 2.0 - (double)(2 * agent_ry));
            v.visibility = (float)s.main_width;
        } else {
            v.center_x = agent_x;
            v.center_y = agent_y;
        }
    } else {
        v.visibility = (float)(s.main_width > s.main_height ? s.main_width : s.main_height);
        if (v.visibility < s.min_visibility) v.visibility = s.min_visibility;
    }
    float raw_unit = 64 / v.visibility;
    v.unit = (float)((double)raw_unit * ((double)64.0f / 64.0));
    v.view_dim = (float)(64.0 / (double)raw_unit);
    v.x_off = v.unit * (v.center_x - v.view_dim / 2);
    v.y_off = v.unit * (v.center_y - v.view_dim / 2);
    return v;
}

} // namespace

// Frame rows per pass and waves per SIMD: the games without rotated / tiled entities fit 168 VGPRs
// (77-114 measured) and render in two 32-row passes at 3 waves per SIMD (12-15 KB of LDS), as do
// six rotating / tiling games; three keep one full-frame pass at 2 waves per SIMD.
#ifndef PG_RENDER_K
#define PG_RENDER_K 1
#endif
template <int G>
DEV constexpr int frame_rows() {
    // measured per game (profiles/r02/r02_k_variants.txt): two passes win for every game but
    // bossfight (48 rotated-image descriptors of LDS), jumper (compass overlay; 170 VGPRs spill) and
    // fruitbot (tile lists), which keep one full-frame pass at 2 waves per SIMD
#ifdef PG_CR_ROWS
    if (G == PG_GAME_COINRUN) return PG_CR_ROWS; // experiment: coinrun's LDS frame in passes of other sizes
#endif
    // coinrun and starpilot: four 16-row passes (a 4 KB frame: coinrun's workgroup needs 8 KB of LDS, 16
    // resident per CU at 4 waves per SIMD instead of 13): coinrun 44.1 -> 46.1, starpilot 35.5 -> 40.1 M
    // env-steps/s; heist, caveflyer, leaper and plunder lose 5-19 % with them, dodgeball ties
    // (profiles/r06/r06_f_render_ab.txt, r06_g_rows16.txt)
    if (G == PG_GAME_COINRUN || G == PG_GAME_STARPILOT) return 16;
#ifdef PG_ROWS32_ONEPASS
    if (G == PG_GAME_BOSSFIGHT || G == PG_GAME_JUMPER || G == PG_GAME_FRUITBOT) return PG_ROWS32_ONEPASS; // experiment
#endif
#ifdef PG_ROWS16_ALL
    if (G != PG_GAME_BOSSFIGHT && G != PG_GAME_JUMPER && G != PG_GAME_FRUITBOT) return 16; // experiment
#endif
    // fruitbot: two 32-row passes since round 6 (17.7 -> 18.8 M env-steps/s, profiles/r06/r06_j_onepass.txt;
    // bossfight and jumper still lose 6-16 % with them, and more with 16-row passes)
    return (G == PG_GAME_BOSSFIGHT || G == PG_GAME_JUMPER) ? 64 : 32;
}
template <int G>
DEV constexpr int render_waves() {
#ifdef PG_CR_WAVES
    if (G == PG_GAME_COINRUN) return PG_CR_WAVES; // experiment: coinrun's waves per SIMD (register budget)
#endif
    return frame_rows<G>() < 32 ? 4 : (frame_rows<G>() == 32 ? 3 : 2);
}
// rounds of 64 pixel jobs per batch of small images (stamp_images): 2, or 4 for leaper.  Round 6 sweep of 1-4
// rounds against the earlier 8 (one pass) / 4 (two passes): 2 rounds win 7 % for bossfight, 5.6 % for fruitbot,
// 1.5-4 % for coinrun, dodgeball, heist, jumper, plunder, starpilot (fewer registers live across a batch); leaper
// loses 1 % with them; the others tie (profiles/r06/r06_o_stamp_rounds.txt)
template <int G>
DEV constexpr int stamp_rounds() { return G == PG_GAME_LEAPER ? 4 : 2; }
// rotated-image descriptors per 64-entity chunk (beyond them an image takes the in-order setup)
template <int G>
DEV constexpr int rot_cap() {
    return G == PG_GAME_COINRUN ? 0 : ((G == PG_GAME_BOSSFIGHT || G == PG_GAME_STARPILOT) ? 48 : 16);
}

template <int G>
__global__ __launch_bounds__(64, render_waves<G>()) void pg_render_kernel(PGDev dg, const int32_t *env_list, int mode, int slot, int count) {
    const PGDev d = game_view(dg, G);
    constexpr int HR = frame_rows<G>();
#ifndef PG_LDS_PAD
#define PG_LDS_PAD 0 // experiment: extra LDS per workgroup (occupancy sensitivity)
#endif
    __shared__ __attribute__((aligned(16))) uint32_t fb_lds[HR * PG_RES + PG_LDS_PAD / 4]; // the rows of one pass
    // stamp_images' per-batch pixel bitmap (kept zero between batches), for the games whose batches it pays
    // for (overlap_blend); null in FB for the others
    // (declared only where used: coinrun's workgroup sits 4 bytes under the LDS of 16 per CU)
    uint32_t *own = nullptr;
    if constexpr (overlap_blend<G>()) {
        __shared__ uint32_t own_lds[HR * PG_RES / 32];
        for (int k = LANE; k < HR * PG_RES / 32; k += 64) own_lds[k] = 0;
        own = own_lds;
    }
    // grid type -> sprite pixel offset of a TILE_PX-square tile (fast path), -1 draws nothing,
    // <= -2 not drawable on the fast path
    constexpr int CR = crows<G>();
    // aux LDS, fast path: tile_off[NTYPES] | colb[CR * 64] -- colb: texel base of lane's first tile
    // column per tile row; before it is built, the same LDS holds the Qt blit setup (t1, n, base,
    // step) of every window tile column / row (class 0 at [0, 128), class 1 at [128, 256) in int4
    // units).  General tile pass (decided after the fast path): GEN_AUX_BYTES of tables.
    // games without uniform tiles never take the fast path: tile_off + the column / row axis tables
    // suffice.  On for fruitbot (one workgroup more per CU: render 4.22 -> 3.79 ms); bossfight's rotated
    // descriptors share aux and it lost 6 % (profiles/r04/r04_h_ab); PG_AUX_TIGHT applies it to all.
#ifdef PG_AUX_TIGHT
    constexpr bool TIGHT = !uniform_tiles<G>();
#else
    constexpr bool TIGHT = !uniform_tiles<G>() && G == PG_GAME_FRUITBOT;
#endif
    constexpr int FAST_BYTES = TIGHT ? (NTYPES + 2 * 64 * 4) * 4 : (NTYPES + CR * 64) * 4;
    constexpr int AUX_BYTES = has_general<G>() && GEN_AUX_BYTES > FAST_BYTES ? GEN_AUX_BYTES : FAST_BYTES;
    __shared__ __attribute__((aligned(16))) uint8_t aux[AUX_BYTES];
    int *const tile_off = reinterpret_cast<int *>(aux);
    int *const colb = tile_off + NTYPES;
    static_assert(CR * 64 >= 2 * 64 * 4, "colb doubles as the axis tables");
    // rotated-image descriptors: in one full-frame pass they reuse aux, whose tile tables are dead
    // once the tiles are drawn; with two passes the second pass still needs the tables
    constexpr bool ONE_PASS = HR == PG_RES;
    constexpr int ROT_CAP = ONE_PASS ? AUX_BYTES / ROT_DESC_BYTES : rot_cap<G>();
    __shared__ __attribute__((aligned(16))) uint8_t rdesc_own[ONE_PASS ? 16 : (ROT_CAP > 0 ? ROT_CAP : 1) * ROT_DESC_BYTES];
    uint8_t *const rdesc = ONE_PASS ? aux : rdesc_own;
    // rounds of 64 pixel jobs per batch of small images: 8 where the frame's LDS already bounds the
    // workgroups per CU (one pass: 16 more VGPRs cost no occupancy), else 4
#ifdef PG_STAMP_ROUNDS
    constexpr int EGK = PG_STAMP_ROUNDS;
#else
    constexpr int EGK = stamp_rounds<G>();
#endif
    int4 *const colax = reinterpret_cast<int4 *>(colb);
    int4 *const rowax = colax + 64;
    // mode 0: every env of the list; 1: the envs whose step did not end the episode (drawn while
    // the reset kernel regenerates the others); 2: this step's reset queue (after the reset)
    // PG_RENDER_K envs per workgroup, one after the other (experiment: fewer, longer workgroups)
    for (int kk = 0; kk < PG_RENDER_K; kk++) {
    const int bidx = (int)blockIdx.x * PG_RENDER_K + kk;
    int env;
    if (mode == 2) {
        if (bidx >= d.reset_count[slot]) break;
        env = d.reset_queue[(size_t)slot * d.num_envs + bidx];
    } else {
        if (bidx >= count) break;
        env = env_list ? env_list[bidx] : bidx;
        if (mode == 1 && d.done8[env]) continue;
    }
    const PGEnv s = d.envs[env];
    const int16_t *Gd = d.grid + (size_t)env * PG_GRID_MAX;
    bool err = false;

    int player_img;
    const View v = prepare_view<G>(d, s, env, player_img);

    const int lane = LANE;
    PTimer pt;
    Census census;
    census.start();
    pt.start();

    // ---- grid type -> sprite table for the fast path (theme_for_grid_obj, image_for_type,
    //      draw_image :886-922): TILE_PX-square tiles only; anything else is drawn by the
    //      generic tile pass (or flagged when met on the fast path)
    for (int t = lane; t < NTYPES; t += 64) {
        int off = -1;
        int img = image_for_type<G>(s, t, player_img);
        if (img >= 0) {
            if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) {
                off = (img == SPACE) ? -1 : -3; // draw_grid_obj fills: generic tile pass
            } else {
                int theme = mask_theme<G>(s, grid_theme<G>(s, t), img);
                int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                if (sp.y == tile_px<G>() && sp.z == tile_px<G>()) off = sp.x;
                else if (sp.y > 0) off = -2;
                else off = -3; // no image (missing_image_ok decides in the generic pass)
            }
        }
        tile_off[t] = off;
    }

    // ---- visible tile window (basic-abstract-game.cpp:937-948)
    int low_x, high_x, low_y, high_y;
    if (s.opt_center_agent) {
        double margin = (double)v.visibility / 2.0 + 1;
        low_x = (int)((double)v.center_x - margin);
        high_x = (int)((double)v.center_x + margin);
        low_y = (int)((double)v.center_y - margin);
        high_y = (int)((double)v.center_y + margin);
    } else {
        low_x = 0; high_x = s.main_width - 1; low_y = 0; high_y = s.main_height - 1;
    }
    const int ww = high_x - low_x + 1, wh = high_y - low_y + 1;
    // every tile column / row of the window gets its own lane for its Qt blit setup (lane 63:
    // the background), so the double-precision setup runs once per tile, not per pixel
    const bool tab = ww <= 63 && wh <= 63;

    // ---- draw_background (basic-abstract-game.cpp:988-1016): black fill + one scaled blit
    Axis bx, by;
    bool bg_ok = false;
    int4 bgi = make_int4(0, 0, 0, 0);
    // the background's pixels: the atlas, or (use_generated_assets) this env's AssetGen image, whose
    // table entry is (offset 0, 500, 500)
    const uint32_t *bgpix = d.gen_bg ? d.gen_bg + (size_t)env * (500 * 500) : d.pixels;
    double bg_rx = 0, bg_ry = 0, bg_rw = 0, bg_rh = 0;
    if (s.opt_use_backgrounds) {
        double mx, my, mw, mh;
        screen_rect(v, 0, (float)s.main_height, (float)s.main_width, (float)s.main_height, 0, mx, my, mw, mh);
        bgi = reinterpret_cast<const int4 *>(d.backgrounds)[s.background_index];
        float bgw = (float)bgi.y, bgh = (float)bgi.z;
        float bg_ar = bgw / bgh;
        float world_ar = (float)(s.main_width * 1.0 / s.main_height);
        float extra_w = bg_ar - world_ar;
        float offset_x = s.bg_pct_x * extra_w;
        // adjust_rect(main_rect, QRectF(-offset_x, 0, bg_ar / world_ar, 1)) (qt-utils.h:12-19)
        double ax = (double)(-offset_x), aw = (double)(bg_ar / world_ar);
        bg_rx = mx + mw * ax; bg_ry = my + mh * 0.0; bg_rw = mw * aw; bg_rh = mh * 1.0;
    }
    if (tab) {
        // one x-axis and one y-axis setup per lane: tile column low_x + lane, tile row
        // low_y + lane, or (lane 63) the background
        double xr = 0, xw = 0, yr = 0, yh = 0;
        int xiw = 0, yih = 0;
        if (lane == 63) {
            if (s.opt_use_backgrounds) { xr = bg_rx; xw = bg_rw; xiw = bgi.y; yr = bg_ry; yh = bg_rh; yih = bgi.z; }
        } else {
            double rx, ry, rw, rh;
            if (lane < ww) {
                screen_rect(v, (float)(low_x + lane), 0.0f, 1, 1, RENDER_EPS, rx, ry, rw, rh);
                xr = rx; xw = rw; xiw = tile_px<G>();
            }
            if (lane < wh) {
                screen_rect(v, 0.0f, (float)(low_y + lane + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
                yr = ry; yh = rh; yih = tile_px<G>();
            }
        }
        Axis a, b;
        const bool okx = axis_setup(xr, xw, xiw, a);
        const bool oky = axis_setup(yr, yh, yih, b);
        colax[lane] = make_int4(a.t1, okx ? a.n : 0, (int)a.base, a.step);
        rowax[lane] = make_int4(b.t1, oky ? b.n : 0, (int)b.base, b.step);
        bg_ok = readlane(okx && oky ? 1 : 0, 63) != 0;
        bx.t1 = readlane(a.t1, 63); bx.n = readlane(a.n, 63); bx.base = (uint32_t)readlane((int)a.base, 63); bx.step = readlane(a.step, 63);
        by.t1 = readlane(b.t1, 63); by.n = readlane(b.n, 63); by.base = (uint32_t)readlane((int)b.base, 63); by.step = readlane(b.step, 63);
        wave_sync();
    } else if (s.opt_use_backgrounds) {
        bg_ok = axis_setup(bg_rx, bg_rw, bgi.y, bx) && axis_setup(bg_ry, bg_rh, bgi.z, by);
    }
    // source row offset of screen row `lane` in the background (-1: outside the blit)
    int bg_lane_row = (bg_ok && lane >= by.t1 && lane < by.t1 + by.n)
                          ? (int)(((by.base + (uint32_t)((lane - by.t1) * by.step)) >> 16) * (uint32_t)bgi.y)
                          : -1;
    if (s.opt_use_backgrounds && s.bg_tile_ratio < 0) {
        // tile_image(main_rect, bg_tile_ratio < 0) (basic-abstract-game.cpp:849-862, 1003-1004): the
        // background repeated down the world; a screen row shows the last tile covering it
        double mx, my, mw, mh;
        screen_rect(v, 0, (float)s.main_height, (float)s.main_width, (float)s.main_height, 0, mx, my, mw, mh);
        const float tile_ratio = -1 * s.bg_tile_ratio;
        int num_tiles = (int)(mh / (mw * tile_ratio));
        if (num_tiles < 1) num_tiles = 1;
        const float th = (float)(mh / num_tiles), tw = (float)mw;
        bg_ok = axis_setup(mx, (double)tw, bgi.y, bx);
        bg_lane_row = -1;
        for (int t0 = 0; t0 < num_tiles; t0 += 64) {
            Axis ty;
            const int t = t0 + lane;
            const bool okt = t < num_tiles && axis_setup(my + (double)(th * (float)t), (double)th, bgi.z, ty);
            const int tt1 = okt ? ty.t1 : 0, tn = okt ? ty.n : 0, tstep = okt ? ty.step : 0;
            const uint32_t tbase = okt ? ty.base : 0u;
            for (int k = 0; k < 64 && t0 + k < num_tiles; k++) {
                const int a1 = readlane(tt1, k), an = readlane(tn, k);
                if (lane >= a1 && lane < a1 + an) {
                    const uint32_t b = (uint32_t)readlane((int)tbase, k);
                    const int st = readlane(tstep, k);
                    bg_lane_row = (int)(((b + (uint32_t)((lane - a1) * st)) >> 16) * (uint32_t)bgi.y);
                }
            }
        }
        if (!bg_ok) bg_lane_row = -1;
    }
    bool bg_col = bg_ok && lane >= bx.t1 && lane < bx.t1 + bx.n;
    uint32_t bg_col_base = (uint32_t)bgi.x + (bg_col ? (bx.base + (uint32_t)((lane - bx.t1) * bx.step)) >> 16 : 0);
    if constexpr (G == PG_GAME_STARPILOT) {
        // starpilot game_draw (starpilot.cpp:107-124): tile_image(r_bg, 1) of a background scrolled
        // left by cur_time -- 3456 x 192 px, 18 square tiles side by side; a screen column shows the
        // last tile covering it
        bg_ok = false;
        bg_col = false;
        bg_lane_row = -1;
        if (s.opt_use_backgrounds) {
            const float scale = (float)(PG_RES / s.main_height); // int / int
            const float bg_k = 3, t = (float)s.cur_time, BG_RATIO = 18;
            const float x_off = -t * scale * SP_HP_SLOW_V * 2 / s.char_dim;
            const double rx = (double)x_off, ry = (double)(-PG_RES * (bg_k - 1) / 2);
            const double rw = (double)(PG_RES * bg_k * BG_RATIO), rh = (double)(PG_RES * bg_k);
            int num_tiles = (int)(rw / (rh * 1.0f));
            if (num_tiles < 1) num_tiles = 1;
            const float tw = (float)(rw / num_tiles), th = (float)rh;
            bg_ok = axis_setup(ry, (double)th, bgi.z, by);
            bg_lane_row = (bg_ok && lane >= by.t1 && lane < by.t1 + by.n)
                              ? (int)(((by.base + (uint32_t)((lane - by.t1) * by.step)) >> 16) * (uint32_t)bgi.y)
                              : -1;
            for (int t0 = 0; t0 < num_tiles; t0 += 64) {
                Axis tx;
                const int k0 = t0 + lane;
                const bool okt = k0 < num_tiles && axis_setup(rx + (double)(tw * (float)k0), (double)tw, bgi.y, tx);
                const int tt1 = okt ? tx.t1 : 0, tn = okt ? tx.n : 0, tstep = okt ? tx.step : 0;
                const uint32_t tbase = okt ? tx.base : 0u;
                for (int k = 0; k < 64 && t0 + k < num_tiles; k++) {
                    const int a1 = readlane(tt1, k), an = readlane(tn, k);
                    if (lane >= a1 && lane < a1 + an) {
                        const uint32_t bb = (uint32_t)readlane((int)tbase, k);
                        const int st = readlane(tstep, k);
                        bg_col = true;
                        bg_col_base = (uint32_t)bgi.x + ((bb + (uint32_t)((lane - a1) * st)) >> 16);
                    }
                }
            }
            if (!bg_ok) bg_col = false;
        }
    }

    pt.mark(7); // diagnostic build: env / tile-table / window / background setup
    // fast path eligibility: square TILE_PX tiles only (uniform_tiles), no z = -1 entity
    // (drawn between background and grid), few tile rows per frame
    const int xg = (int)floorf(((float)lane + 0.5f + v.x_off) / v.unit);
    const int yg = (int)floorf((v.view_dim - ((float)lane + 0.5f - v.y_off) / v.unit));
    int cx0 = 0, cx1 = 0, ncx0 = 0, scol0 = 0, scol1 = 0;
    int ry0 = 0, ry1 = 0, ncy0 = 0, srow0 = 0, srow1 = 0;
    int nrows = 0, jy0 = 0;
    bool fast = false;
    if (uniform_tiles<G>() && !has_z_minus1<G>() && tab) {
        // tile columns covering screen column `lane` (<= 2, ascending x) for TILE_PX-wide images, and
        // tile rows covering screen row `lane` (<= 2, ascending y = the reference's draw order): the five
        // candidate table entries of each axis are read first (one LDS round trip), then scanned
        int4 tc[5], tr[5];
#pragma unroll
        for (int q = 0; q < 5; q++) {
            tc[q] = colax[min(max(xg - 2 + q - low_x, 0), 63)];
            tr[q] = rowax[min(max(yg - 2 + q - low_y, 0), 63)];
        }
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const int x = xg - 2 + q;
            if (x < low_x || x > high_x || ncx0 == 2) continue;
            const int4 t = tc[q];
            if (t.y > 0 && lane >= t.x && lane < t.x + t.y) {
                int scv = (int)(((uint32_t)t.z + (uint32_t)((lane - t.x) * t.w)) >> 16);
                if (ncx0 == 0) { cx0 = x; scol0 = scv; } else { cx1 = x; scol1 = scv; }
                ncx0++;
            }
        }
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const int y = yg - 2 + q;
            if (y < low_y || y > high_y || ncy0 == 2) continue;
            const int4 t = tr[q];
            if (t.y > 0 && lane >= t.x && lane < t.x + t.y) {
                int srv = (int)(((uint32_t)t.z + (uint32_t)((lane - t.x) * t.w)) >> 16);
                if (ncy0 == 0) { ry0 = y; srow0 = srv; } else { ry1 = y; srow1 = srv; }
                ncy0++;
            }
        }
        int jlo = ncy0 > 0 ? ry0 : 0x7fffffff, jhi = ncy0 > 1 ? ry1 : (ncy0 > 0 ? ry0 : -0x7fffffff);
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            jlo = min(jlo, __shfl_xor(jlo, sh));
            jhi = max(jhi, __shfl_xor(jhi, sh));
        }
        jy0 = jlo;
        nrows = jhi >= jlo ? jhi - jlo + 1 : 0;
        fast = nrows <= CR;
#ifdef PG_PROF_RSETUP // diagnostic: the fast path's setup split (slot 2: window column / row scan)
        pt.mark(2);
#endif
        if constexpr (!always_uniform<G>()) {
            if (fast) { // every tile of the window must be a tile_px() square (or nothing)
                bool other = false;
                for (int k = lane; k < ww * wh; k += 64) {
                    const int x = low_x + k % ww, y = low_y + k / ww;
                    const int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x]
                                                                                             : s.out_of_bounds_object;
                    if (type != INVALID_OBJ && type != SPACE && (type < 0 || type >= NTYPES || tile_off[type] <= -2))
                        other = true;
                }
                fast = ballot(other) == 0;
            }
        } else if (s.opt_use_monochrome_assets || d.gen_bg) {
            // monochrome: every drawable tile is a draw_grid_obj fill; use_generated_assets: the
            // tiles are 64 x 64 AssetGen images, not tile_px() squares -- generic tile pass
            fast = false;
        }
    }
    auto lookup_grid = [&](int x, int y) -> int {
        int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x]
                                                                               : s.out_of_bounds_object;
        return (type == INVALID_OBJ || type == SPACE) ? -1 : ((type >= 0 && type < NTYPES) ? tile_off[type] : -2);
    };
    wave_sync(); // tile table complete
    if (fast) {
        // ---- lookups for the fast path: every screen row's tile rows lie in [jy0, jy1]; for
        //      each of those rows the texel base of this lane's first tile column goes to LDS
        //      (colb), so a pixel costs one LDS read + one texel load + one blend.
        int code[CR];
#pragma unroll
        for (int j = 0; j < CR; j++) {
            code[j] = -1;
            if (j < nrows && ncx0 > 0) {
                const int y = jy0 + j, x = cx0;
                if (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) code[j] = Gd[y * s.main_width + x];
                else code[j] = s.out_of_bounds_object;
            }
        }
        wave_sync(); // colb's axis-table contents are dead from here
#ifdef PG_PROF_RSETUP // (slot 5: the tile codes' grid loads)
        pt.mark(5);
#endif
        // every row's table read first, then the writes (tile_off and colb share the aux array, so the
        // compiler would otherwise order each read after the previous row's write)
        int cj[CR];
#pragma unroll
        for (int j = 0; j < CR; j++) {
            const int t = code[j];
            cj[j] = (ncx0 == 0 || t == INVALID_OBJ || t == SPACE) ? -1 : ((t >= 0 && t < NTYPES) ? tile_off[t] : -2);
        }
#pragma unroll
        for (int j = 0; j < CR; j++) {
            if (j < nrows) {
                const int c = cj[j];
                if (c <= -2) err = true;
                colb[j * 64 + lane] = c >= 0 ? c + scol0 : -1;
            }
        }
    }
    wave_sync();
    // general tile pass for the frames the fast path does not take (class tables built in fb's LDS,
    // which is dead until the background pass)
    GenLane gl;
    gl.cx0 = gl.cx1 = gl.ry0 = gl.ry1 = -1;
    gl.ncx = gl.ncy = 0;
    bool gen = false, notiles = false;
    if constexpr (has_general<G>())
        if (!fast && tab) {
            static_assert(2 * GEN_K * 64 * 16 <= 32 * PG_RES * 4, "the class tables fit the pass frame");
            const int gs = gen_setup<G>(d, s, v, Gd, player_img, low_x, low_y, ww, wh, xg, yg, aux, reinterpret_cast<int4 *>(fb_lds), gl);
            gen = gs == 1;
            notiles = gs == 2;
        }

    pt.mark(0);
    Img im;
    img_clear(im);
    // ---- entities of one render_z, in list order (basic-abstract-game.cpp:1061-1075); one
    //      setup per 64-entity chunk, reused by every z pass and both frame passes when the list
    //      fits one chunk (and nothing else used `im` in between)
    const int n = s.num_ents;
    const bool one_chunk = n <= 64;
    bool ent_setup_valid = false;
#define PG_DRAW_ENTITIES(Z)                                                                   \
    for (int base = 0; base < n; base += 64) {                                                \
        pt.mark(4);                                                                           \
        if (!one_chunk || !ent_setup_valid) {                                                 \
            entity_setup<G>(d, s, v, env, base + lane, n, player_img, im, err);               \
            if (!has_z_minus1<G>()) rot_stage(im, rdesc, ROT_CAP);                            \
        }                                                                                     \
        ent_setup_valid = true;                                                               \
        pt.mark(3);                                                                           \
        stamp_images<true, EGK, overlap_blend<G>()>(fb, d, rdesc, im, ballot(im.draw && im.ez == (Z) && img_in_pass(im, fb)), err); \
    }

#ifdef PG_PROF_STAMP
    PTimer spt;
    spt.start();
#endif
    for (int pass = 0; pass < PG_RES / HR; pass++) {
#ifdef PG_PROF_STAMP
    const FB fb{fb_lds, pass * HR, HR, own, &spt};
#else
    const FB fb{fb_lds, pass * HR, HR, own};
#endif
    if (fast) {
        // ---- background + first tile column, pixel-centric, RB rows per batch (all loads of
        //      a batch are issued before the first blend).  A transparent texel (0) blends to
        //      the unchanged pixel exactly, so lanes without a tile carry 0.
        // per screen row (lane = row), packed for one readlane per row: source rows of its
        // tile rows (7 bits each), their colb rows (5 bits each), tile-row count (2 bits);
        // and the background source row offset (-1: outside the background blit)
        const int rinfo = ncy0 == 0 ? 0
                        : (srow0 | ((ncy0 > 1 ? srow1 : 0) << 7) | ((ry0 - jy0) << 14) |
                           ((ncy0 > 1 ? ry1 - jy0 : ry0 - jy0) << 19) | (ncy0 << 24));
        const int bgrow = bg_lane_row;
#ifndef PG_FAST_PIPE
#define PG_FAST_PIPE 0 // 1: software-pipelined batches (measured neutral at one workgroup fewer per CU, r06_e)
#endif
        // One batch = RB rows: its row infos, then the LDS reads of the batch's tile texel bases, then
        // every texel load of the batch (branch-free: an absent texel loads pixels[0] and is discarded).
        // With PG_FAST_PIPE the next batch's loads are issued before this batch blends, so a batch's
        // gather latency runs under the previous batch's blends and LDS stores.
        struct FastBatch {
            uint32_t bgv[RB], ta[RB], tb[RB];
            int info[RB];
        };
        auto issue = [&](int r0, FastBatch &B) {
            int bgr[RB], ca[RB], cbv[RB];
#pragma unroll
            for (int k = 0; k < RB; k++) {
                B.info[k] = readlane(rinfo, r0 + k);
                bgr[k] = readlane(bgrow, r0 + k);
            }
#pragma unroll
            for (int k = 0; k < RB; k++) { // LDS reads of the whole batch first
                ca[k] = colb[((B.info[k] >> 14) & 31) * 64 + lane];
                cbv[k] = colb[((B.info[k] >> 19) & 31) * 64 + lane];
            }
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const bool inb = bg_col && bgr[k] >= 0;
#ifdef PG_DIAG_NOBG // diagnostic knockout (wrong frames): no background texel loads
                const uint32_t px = 0xff000000u | (uint32_t)bgr[k];
#else
                const uint32_t px = bgpix[inb ? bg_col_base + (uint32_t)bgr[k] : 0u];
#endif
                B.bgv[k] = inb ? px : 0xff000000u;
            }
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int nr = B.info[k] >> 24;
                const bool ha = nr > 0 && ca[k] >= 0, hb = nr > 1 && cbv[k] >= 0;
#ifdef PG_DIAG_NOTILE // diagnostic knockout (wrong frames): no tile texel loads
                B.ta[k] = ha ? 0xff000000u | (uint32_t)ca[k] : 0u;
                B.tb[k] = hb ? 0xff000000u | (uint32_t)cbv[k] : 0u;
#elif defined(PG_FAST_BRANCHFREE) // experiment: every lane loads (measured slower, r06_e r8p0)
                const uint32_t pa = d.pixels[ha ? (uint32_t)ca[k] + (uint32_t)((B.info[k] & 127) * tile_px<G>()) : 0u];
                const uint32_t pb = d.pixels[hb ? (uint32_t)cbv[k] + (uint32_t)(((B.info[k] >> 7) & 127) * tile_px<G>()) : 0u];
                B.ta[k] = ha ? pa : 0u;
                B.tb[k] = hb ? pb : 0u;
#else // tile texels loaded only by the lanes that draw one (exec-masked loads: sky lanes issue none)
                B.ta[k] = 0u;
                B.tb[k] = 0u;
                if (ha) B.ta[k] = d.pixels[(uint32_t)ca[k] + (uint32_t)((B.info[k] & 127) * tile_px<G>())];
                if (hb) B.tb[k] = d.pixels[(uint32_t)cbv[k] + (uint32_t)(((B.info[k] >> 7) & 127) * tile_px<G>())];
#endif
            }
        };
        auto blend = [&](int r0, const FastBatch &B) {
            // a missing tile texel is 0, which blends to the unchanged pixel on either path
            uint32_t part = 0;
#pragma unroll
            for (int k = 0; k < RB; k++) part |= alpha_partial(B.ta[k]) | alpha_partial(B.tb[k]);
            if (!ballot(part != 0)) {
#pragma unroll
                for (int k = 0; k < RB; k++) fb[(r0 + k) * PG_RES + lane] = over_binary(over_binary(B.bgv[k], B.ta[k]), B.tb[k]);
            } else {
#pragma unroll
                for (int k = 0; k < RB; k++) {
                    const int nr = B.info[k] >> 24;
                    uint32_t px = B.bgv[k];
                    if (nr > 0) px = B.ta[k] + BYTE_MUL(px, (~B.ta[k]) >> 24);
                    if (nr > 1) px = B.tb[k] + BYTE_MUL(px, (~B.tb[k]) >> 24);
                    fb[(r0 + k) * PG_RES + lane] = px;
                }
            }
        };
        if (PG_FAST_PIPE) {
            FastBatch cur, nxt;
            issue(fb.y0, cur);
            for (int r0 = fb.y0; r0 < fb.y0 + fb.h; r0 += RB) {
                if (r0 + RB < fb.y0 + fb.h) issue(r0 + RB, nxt);
                blend(r0, cur);
                cur = nxt;
            }
        } else {
            for (int r0 = fb.y0; r0 < fb.y0 + fb.h; r0 += RB) {
                FastBatch cur;
                issue(r0, cur);
                blend(r0, cur);
            }
        }
        wave_sync();
        // ---- second tile column of the few screen columns two tiles overlap (RENDER_EPS):
        //      drawn after the first column's tiles, which is the reference's x-major order.
        //      Lane = screen row here, so the row tables are lane-local.
        unsigned long long m2 = ballot(ncx0 > 1);
        while (m2) {
            const int c = __ffsll((long long)m2) - 1;
            m2 &= m2 - 1;
            const int x1 = readlane(cx1, c), sc1 = readlane(scol1, c);
            const int row = lane;
            if (ncy0 > 0 && fb.row_in(row)) {
                uint32_t px = fb[row * PG_RES + c];
                for (int l = 0; l < ncy0; l++) {
                    const int code = lookup_grid(x1, l ? ry1 : ry0);
                    if (code <= -2) err = true;
                    if (code >= 0) {
                        const uint32_t t = d.pixels[(uint32_t)code + (uint32_t)((l ? srow1 : srow0) * tile_px<G>() + sc1)];
                        px = t + BYTE_MUL(px, (~t) >> 24);
                    }
                }
                fb[row * PG_RES + c] = px;
            }
        }
    } else if (gen && !has_z_minus1<G>()) {
        gen_draw<true>(fb, d, bgpix, aux, gl, ww, bg_col, bg_col_base, bg_lane_row, err);
    } else {
        // ---- background alone (lane = column), RB rows per batch
        const int bgrow = bg_lane_row;
        for (int r0 = fb.y0; r0 < fb.y0 + fb.h; r0 += RB) {
            uint32_t bgv[RB];
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int br = readlane(bgrow, r0 + k);
                const bool inb = bg_col && br >= 0;
                uint32_t px = bgpix[inb ? bg_col_base + (uint32_t)br : 0u];
                bgv[k] = inb ? px : 0xff000000u;
            }
#pragma unroll
            for (int k = 0; k < RB; k++) fb[(r0 + k) * PG_RES + lane] = bgv[k];
        }
    }
    wave_sync();

    pt.mark(1);
    if (!fast) {
        // ---- z = -1 entities, then the grid tiles in the reference's x-major / y-minor order
        //      (draw_foreground :930-964), stamped like entities: lane k <-> the k-th tile of
        //      a 64-tile chunk of the window
        if (has_z_minus1<G>()) {
            PG_DRAW_ENTITIES(-1)
        }
        if (notiles) {
        } else if (gen) {
            if constexpr (has_z_minus1<G>()) {
                wave_sync();
                gen_draw<false>(fb, d, bgpix, aux, gl, ww, false, 0u, -1, err);
            }
        } else if (has_grid_tiles<G>()) {
            ent_setup_valid = false; // the tile chunks reuse `im`
            const int ntiles = ww * wh;
            for (int base = 0; base < ntiles; base += 64) {
                const int k = base + lane;
                img_clear(im);
                if (k < ntiles) {
                    const int x = low_x + k / wh, y = low_y + k % wh;
                    int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x]
                                                                                           : s.out_of_bounds_object;
                    int img = type == INVALID_OBJ ? -1 : image_for_type<G>(s, type, player_img);
                    if (img >= 0) {
                        if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) {
                            double rx, ry, rw, rh;
                            screen_rect(v, (float)x, (float)(y + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
                            if (img != SPACE && !(s.opt_use_monochrome_assets
                                                      ? mono_fill<G>(s, img, grid_theme<G>(s, type), rx, ry, rw, rh, im)
                                                      : grid_obj_fill<G>(img, rx, ry, rw, rh, im)))
                                err = true; // color_for_type fasserts (:464-490)
                        } else {
                            int theme = mask_theme<G>(s, grid_theme<G>(s, type), img);
                            int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                            if (sp.y <= 0) {
                                if (!missing_image_ok<G>(img)) err = true;
                            } else {
                                double rx, ry, rw, rh;
                                screen_rect(v, (float)x, (float)(y + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
                                if (axis_setup(rx, rw, sp.y, im.ex) && axis_setup(ry, rh, sp.z, im.ey)) {
                                    im.draw = true;
                                    im.soff = sp.x;
                                    im.sw = sp.y;
                                    im.sh = sp.z;
                                }
                            }
                        }
                    }
                }
                stamp_images<true, EGK, overlap_blend<G>()>(fb, d, rdesc, im, ballot(im.draw && img_in_pass(im, fb)), err);
            }
        }
    } else if (has_z_minus1<G>()) {
        err = true; // unreachable: the fast path is never taken with z = -1 entities
    }
    pt.mark(2);
    // ---- entities, render_z 0 then 1 (basic-abstract-game.cpp:966-967)
    PG_DRAW_ENTITIES(0)
    PG_DRAW_ENTITIES(1)
    wave_sync();
    if (__builtin_expect(s.has_useful_vel_info && s.opt_paint_vel_info, 0)) { // paint_vel_info (basic-abstract-game.cpp:969-977)
        const float vx = s.agent_erased ? s.ghost_vx : EFr(d, F_VX, env, 0);
        const float vy = s.agent_erased ? s.ghost_vy : EFr(d, F_VY, env, 0);
        const float infodim = (float)(PG_RES * .2);
        const uint32_t s1 = (uint32_t)to_shade((float)(.5 * (double)vx / (double)s.maxspeed + .5));
        const uint32_t s2 = (uint32_t)to_shade((float)(.5 * (double)vy / (double)s.max_jump + .5));
        fb_fill_rectf(fb, 0, 0, infodim, infodim, 0xff000000u | (s1 * 0x010101u));
        fb_fill_rectf(fb, infodim, 0, infodim, infodim, 0xff000000u | (s2 * 0x010101u));
        wave_sync();
    }
    pt.mark(4);
    game_overlay<G>(fb, s, v, d, env, err);
    wave_sync();
    pt.mark(5);
    // ---- bgr32_to_rgb888 (game.cpp:8-23) of the pass's rows: lane writes 4 pixels = 12 bytes
    uint8_t *out = d.rgb + (size_t)env * PG_OBS_BYTES;
    for (int q = fb.y0 * (PG_RES / 4) + lane; q < (fb.y0 + fb.h) * (PG_RES / 4); q += 64) {
        uint4 p4 = reinterpret_cast<const uint4 *>(fb_lds)[q - fb.y0 * (PG_RES / 4)];
        // bytes r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
        uint32_t w0 = ((p4.x >> 16) & 0xff) | (p4.x & 0xff00) | ((p4.x & 0xff) << 16) | (((p4.y >> 16) & 0xff) << 24);
        uint32_t w1 = ((p4.y >> 8) & 0xff) | ((p4.y & 0xff) << 8) | (((p4.z >> 16) & 0xff) << 16) | (((p4.z >> 8) & 0xff) << 24);
        uint32_t w2 = (p4.z & 0xff) | (((p4.w >> 16) & 0xff) << 8) | (((p4.w >> 8) & 0xff) << 16) | ((p4.w & 0xff) << 24);
        uint32_t *o = reinterpret_cast<uint32_t *>(out + (size_t)q * 12);
        o[0] = w0;
        o[1] = w1;
        o[2] = w2;
    }
    wave_sync(); // the next pass overwrites the frame rows
    } // pass
#undef PG_DRAW_ENTITIES
    if (ballot(err) && lane == 0) atomicOr(d.error_any, 1 << PG_ERR_RENDER);
    pt.mark(6);
#ifndef PG_PROF_SMART // that diagnostic build fills these slots with the step's smart-entity census
    pt.flush(d.prof ? d.prof + (size_t)env * 16 + 8 : nullptr);
#endif
#ifdef PG_PROF_STAMP
    spt.mark(7);
    spt.flush(d.prof ? d.prof + (size_t)env * 16 : nullptr); // the step kernel's slots (it does not flush here)
#endif
    census.flush(d.prof ? d.prof + (size_t)env * 16 + 8 : nullptr);
    if (PG_RENDER_K > 1) wave_sync(); // the next env reuses the LDS
    } // kk
}


// ================================================================== register-frame render
// pg_render_rf_kernel<G>: the frame of pg_render_kernel, for the games and options it serves (rf_game,
// PGDev::render_rf, set by the host), drawn pixel-centrically with no LDS frame.  Lane = screen column;
// RF_RB screen rows at a time live in registers.  For every row batch, all texels the batch needs are
// loaded before the first blend -- the background, the <= 2 x 2 grid tiles covering the pixel (x-major,
// y-minor: basic-abstract-game.cpp:937-964) and the first RF_JOBS (image, row) jobs of the images that
// cross the batch (z = -1, then the tiles, then z = 0 / z = 1 entities in list order, the velocity
// squares and the game's overlays: :930-977, games/*.cpp game_draw) -- then blended in that order,
// packed to RGB888 across lanes (bgr32_to_rgb888, game.cpp:8-23) and stored.  Blending per pixel in
// draw order is the painter's algorithm of the reference pixel by pixel; every texel, edge and
// transform is the one the stamping kernel takes (the same Axis setup, Qt transform-blit descriptors,
// fillRect edges, Qt-tabulated compass rows).  The LDS holds only the tile tables and the visible
// images' descriptors (~6 KB for coinrun instead of the 12 KB frame kernel), so a CU keeps twice the
// waves resident to hide the gather latency (the render is latency-bound: +4 KB of LDS per workgroup
// cost +19 % render time, profiles/r05/).
#ifndef RF_RB
#define RF_RB 4 // 8 rows per batch spilled 21-50 registers (coinrun, maze) at the occupancy the kernel needs
#endif
#ifndef RF_JOBS
#define RF_JOBS 8
#endif
template <int G>
__host__ __device__ constexpr bool rf_game() {
    return G == PG_GAME_COINRUN || G == PG_GAME_BIGFISH || G == PG_GAME_MAZE || G == PG_GAME_HEIST || G == PG_GAME_MINER ||
           G == PG_GAME_CLIMBER || G == PG_GAME_CHASER || G == PG_GAME_NINJA || G == PG_GAME_CAVEFLYER ||
           G == PG_GAME_PLUNDER || G == PG_GAME_STARPILOT || G == PG_GAME_LEAPER || G == PG_GAME_DODGEBALL ||
           G == PG_GAME_JUMPER || G == PG_GAME_FRUITBOT;
    // bossfight: its frames hold more rotated trail images than the descriptor LDS takes (the
    // LDS-frame kernel stamps them)
}
// visible image descriptors per frame (tile_image entities become one per tile), Qt transform-blit
// descriptors (96 B each, rot_stage)
template <int G>
DEV constexpr int rf_dcap() { return has_tiled_entities<G>() ? 256 : 128; }
template <int G>
DEV constexpr int rf_rcap() { return has_rotation<G>() ? ((G == PG_GAME_BOSSFIGHT || G == PG_GAME_STARPILOT) ? 96 : 64) : 1; }
// descriptor kinds
#define RF_PLAIN 0  // scale blit or fill of an axis-aligned rect
#define RF_ROT 1    // Qt transform blit, descriptor in rdesc
#define RF_ROWS 2   // Qt-tabulated row bitmap of one colour (jumper's compass)

// General tile pass state, in registers (gen_setup without its LDS tables): lane = screen column: the
// covering window columns (relative to low_x); lane = screen row: the covering window rows; per class
// k the source column of this column's first | second covering window column (int16 each, -1: none)
// and the source row of this row's first | second covering window row.
struct RfGen {
    int cx0, cx1, ncx, ry0, ry1, ncy;
    int xs[GEN_K], ys[GEN_K];
};

// gen_setup for the register-frame kernel: ti (typeinfo, LDS) and gw (window slots, LDS) as there, the
// class axes held per lane (lane = window column / row) and read across lanes.  0: not expressible,
// 1: draw, 2: no drawn tile in the window.
template <int G>
DEV int rf_gen_setup(const PGDev &d, const PGEnv &s, const View &v, const int16_t *Gd, int player_img, int low_x,
                     int low_y, int ww, int wh, int xg, int yg, int2 *ti, uint8_t *gw, RfGen &g) {
    const int lane = LANE;
    g.cx0 = g.cx1 = g.ry0 = g.ry1 = -1;
    g.ncx = g.ncy = 0;
#pragma unroll
    for (int k = 0; k < GEN_K; k++) g.xs[k] = g.ys[k] = -1;
    if (ww > 63 || wh > 63 || ww * wh > GEN_GW) return 0;
    int kind = 0, off = 0, iw = 0, ih = 0;
    {
        const int t = gen_slot_type<G>(lane);
        const int img = image_for_type<G>(s, t, player_img);
        if (img >= 0) {
            if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) { // draw_grid_obj (:924-928)
                if (img != SPACE) {
                    if (G == PG_GAME_CHASER && img == CH_ORB) {
                        kind = 3; off = (int)0xff00ff00u;
                    } else if (s.opt_use_monochrome_assets) {
                        const uint32_t col = color_for_type<G>(s, img, grid_theme<G>(s, t));
                        if (col == 0) kind = GEN_BAD;
                        else { kind = 2; off = (int)(col | 0xff000000u); }
                    } else {
                        kind = GEN_BAD;
                    }
                }
            } else {
                const int theme = mask_theme<G>(s, grid_theme<G>(s, t), img);
                const int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                if (sp.y > 0) { kind = 1; off = sp.x; iw = sp.y; ih = sp.z; }
                else if (!missing_image_ok<G>(img)) kind = GEN_BAD;
            }
        }
    }
    bool bad = false;
    unsigned long long present = 0;
    for (int c = lane; c < ww * wh; c += 64) {
        const int x = low_x + c % ww, y = low_y + c / ww;
        const int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x]
                                                                                   : s.out_of_bounds_object;
        int sl = gen_slot<G>(type);
        if (sl < 0) { bad = true; sl = GEN_NOTHING; }
        if (sl < 64) present |= 1ull << sl;
        gw[c] = (uint8_t)sl;
    }
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const uint32_t lo = (uint32_t)present, hi = (uint32_t)(present >> 32);
        present |= (unsigned long long)(uint32_t)__shfl_xor((int)lo, sh) | ((unsigned long long)(uint32_t)__shfl_xor((int)hi, sh) << 32);
    }
    const bool here = (present >> lane) & 1;
    if (here && kind == GEN_BAD) bad = true;
    if (ballot(bad)) return 0;
    const bool drawn = here && kind >= 1 && kind <= 3;
    const int key = kind == 1 ? (iw | (ih << 12) | (1 << 24)) : (kind << 24);
    unsigned long long pend = ballot(drawn);
    int cls = 0, K = 0;
    int ck[GEN_K], cw[GEN_K], chh[GEN_K];
#pragma unroll
    for (int k = 0; k < GEN_K; k++) ck[k] = cw[k] = chh[k] = 0;
    while (pend) {
        const int f = __ffsll((long long)pend) - 1;
        const int kf = readlane(key, f);
        const unsigned long long mem = ballot(drawn && key == kf);
        if (K < GEN_K) {
            if (drawn && key == kf) cls = K;
#pragma unroll
            for (int k = 0; k < GEN_K; k++)
                if (k == K) { ck[k] = readlane(kind, f); cw[k] = readlane(iw, f); chh[k] = readlane(ih, f); }
        }
        K++;
        pend &= ~mem;
    }
    if (K > GEN_K) return 0;
    if (K == 0) return 2;
    ti[lane] = drawn ? make_int2(off, iw | (cls << 16) | (kind << 24)) : make_int2(0, 0);
    if (lane == 0) ti[GEN_NOTHING] = make_int2(0, 0);
    double rx = 0, rw = 0, ry = 0, rh = 0, t0, t1;
    if (lane < ww) screen_rect(v, (float)(low_x + lane), 0.0f, 1, 1, RENDER_EPS, rx, t0, rw, t1);
    if (lane < wh) screen_rect(v, 0.0f, (float)(low_y + lane + 1), 1, 1, RENDER_EPS, t0, ry, t1, rh);
    // coverage: does any class's blit of window column xg + dx cover this screen column (and rows)
    int covx = 0, covy = 0;
#pragma unroll
    for (int k = 0; k < GEN_K; k++) {
        if (k >= K) break;
        Axis a, b;
        const bool okx = lane < ww && class_axis(ck[k], cw[k], rx, rw, a);
        const bool oky = lane < wh && class_axis(ck[k], chh[k], ry, rh, b);
        const int ax = okx ? (a.t1 | (a.n << 8)) : 0, by = oky ? (b.t1 | (b.n << 8)) : 0;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const int x = xg - 2 + q, y = yg - 2 + q;
            const int tx = __shfl(ax, (x - low_x) & 63), ty = __shfl(by, (y - low_y) & 63);
            if (x >= low_x && x - low_x < ww && lane >= (tx & 255) && lane < (tx & 255) + (tx >> 8)) covx |= 1 << q;
            if (y >= low_y && y - low_y < wh && lane >= (ty & 255) && lane < (ty & 255) + (ty >> 8)) covy |= 1 << q;
        }
    }
#pragma unroll
    for (int q = 0; q < 5; q++) {
        if ((covx >> q) & 1) {
            const int i = xg - 2 + q - low_x;
            if (g.ncx == 0) g.cx0 = i; else if (g.ncx == 1) g.cx1 = i; else bad = true;
            g.ncx++;
        }
        if ((covy >> q) & 1) {
            const int j = yg - 2 + q - low_y;
            if (g.ncy == 0) g.ry0 = j; else if (g.ncy == 1) g.ry1 = j; else bad = true;
            g.ncy++;
        }
    }
    if (ballot(bad)) return 0;
    // per class: source column of this lane's covering columns, source row of this row's
#pragma unroll
    for (int k = 0; k < GEN_K; k++) {
        if (k >= K) break;
        Axis a, b;
        const bool okx = lane < ww && class_axis(ck[k], cw[k], rx, rw, a);
        const bool oky = lane < wh && class_axis(ck[k], chh[k], ry, rh, b);
        const int at1 = okx ? a.t1 : 0, an = okx ? a.n : 0, bt1 = oky ? b.t1 : 0, bn = oky ? b.n : 0;
        const int ab = okx ? (int)a.base : 0, as = okx ? a.step : 0, bb = oky ? (int)b.base : 0, bs = oky ? b.step : 0;
        int v0 = -1, v1 = -1, w0 = -1, w1 = -1;
        {
            const int i0 = g.cx0 & 63, i1 = g.cx1 & 63, j0 = g.ry0 & 63, j1 = g.ry1 & 63;
            const int t10 = __shfl(at1, i0), n0 = __shfl(an, i0), b0 = __shfl(ab, i0), s0 = __shfl(as, i0);
            const int t11 = __shfl(at1, i1), n1 = __shfl(an, i1), b1 = __shfl(ab, i1), s1 = __shfl(as, i1);
            const int u10 = __shfl(bt1, j0), m0 = __shfl(bn, j0), c0 = __shfl(bb, j0), r0 = __shfl(bs, j0);
            const int u11 = __shfl(bt1, j1), m1 = __shfl(bn, j1), c1 = __shfl(bb, j1), r1 = __shfl(bs, j1);
            if (g.ncx > 0 && n0 > 0 && lane >= t10 && lane < t10 + n0) v0 = (int)(((uint32_t)b0 + (uint32_t)((lane - t10) * s0)) >> 16);
            if (g.ncx > 1 && n1 > 0 && lane >= t11 && lane < t11 + n1) v1 = (int)(((uint32_t)b1 + (uint32_t)((lane - t11) * s1)) >> 16);
            if (g.ncy > 0 && m0 > 0 && lane >= u10 && lane < u10 + m0) w0 = (int)(((uint32_t)c0 + (uint32_t)((lane - u10) * r0)) >> 16);
            if (g.ncy > 1 && m1 > 0 && lane >= u11 && lane < u11 + m1) w1 = (int)(((uint32_t)c1 + (uint32_t)((lane - u11) * r1)) >> 16);
        }
        g.xs[k] = (v0 & 0xffff) | (v1 << 16);
        g.ys[k] = (w0 & 0xffff) | (w1 << 16);
    }
    return 1;
}

// the texel of general-pass cell t at the class's source column / row (gen_texel with packed tables)
// (the class selects are spelt out as a chain of conditional moves: written as a loop over the arrays,
// the compiler kept the arrays in scratch and indexed them)
static_assert(GEN_K == 4, "rf_gen_texel selects among 4 classes");
DEV int rf_sel4(int cl, int a0, int a1, int a2, int a3) {
    int v = cl == 1 ? a1 : a0;
    v = cl == 2 ? a2 : v;
    return cl == 3 ? a3 : v;
}
DEV uint32_t rf_gen_texel(const PGDev &d, const int2 t, const int (&xs)[GEN_K], const int (&ysr)[GEN_K], bool second_col,
                          bool second_row, bool &err) {
    const int kind = t.y >> 24;
    if (kind == 0) return 0u;
    const int cl = (t.y >> 16) & 255;
    const int xv = rf_sel4(cl, xs[0], xs[1], xs[2], xs[3]), yv = rf_sel4(cl, ysr[0], ysr[1], ysr[2], ysr[3]);
    const int sc = second_col ? (xv >> 16) : (int)(int16_t)(xv & 0xffff);
    const int sr = second_row ? (yv >> 16) : (int)(int16_t)(yv & 0xffff);
    return gen_texel(d, t, sc, sr, err);
}

// LDS of the register-frame render: FAST: tile_off[NTYPES] | codes[CR][64] (grid value of the first |
// second covering tile column per window tile row and lane, 255: nothing); GEN: typeinfo ti[65] |
// window slots gw[GEN_GW]; then the image descriptors (2 int4 each) and the transform-blit descriptors
template <int G>
DEV constexpr int rf_tab_bytes() {
    return always_uniform<G>() ? NTYPES * 4 + crows<G>() * 64 * 2 : (has_general<G>() ? GEN_TI_BYTES + GEN_GW : 16);
}
template <int G>
DEV constexpr int rf_lds_bytes() { return rf_tab_bytes<G>() + 32 * rf_dcap<G>() + 96 * rf_rcap<G>(); }

// One env's frame (d: the game's view, game_view).  tab / desc / rdesc: LDS of rf_tab_bytes,
// 2 * rf_dcap and 6 * rf_rcap int4, 16-B aligned; the caller's wave owns them for the call.
template <int G>
DEV void rf_render_env(const PGDev &d, int env, uint8_t *tab, int4 *desc, int4 *rdesc) {
    constexpr bool FAST = always_uniform<G>();             // square tile_px() tiles: grid value tables
    constexpr bool GEN = has_general<G>();                 // the general tile pass
    constexpr int CR = crows<G>();
    constexpr int TP = tile_px<G>();
    constexpr int DCAP = rf_dcap<G>(), RCAP = rf_rcap<G>();
    int *const tile_off = reinterpret_cast<int *>(tab);
    uint16_t *const codes = reinterpret_cast<uint16_t *>(tab + NTYPES * 4);
    int2 *const ti = reinterpret_cast<int2 *>(tab);
    uint8_t *const gw = tab + GEN_TI_BYTES;
    const int lane = LANE;
    const PGEnv s = d.envs[env];
    const int16_t *Gd = d.grid + (size_t)env * PG_GRID_MAX;
    bool err = false;
    int player_img;
    const View v = prepare_view<G>(d, s, env, player_img);

    if constexpr (FAST) { // grid type -> sprite pixel offset (theme_for_grid_obj, image_for_type, draw_image :886-922)
        int off = -1;
        const int img = image_for_type<G>(s, lane, player_img);
        if (img >= 0) {
            if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) {
                off = img == SPACE ? -1 : -3; // draw_grid_obj fills: not on this path
            } else {
                const int theme = mask_theme<G>(s, grid_theme<G>(s, lane), img);
                const int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                off = (sp.y == TP && sp.z == TP) ? sp.x : -2;
            }
        }
        tile_off[lane] = off;
    }
    // ---- visible tile window (basic-abstract-game.cpp:937-948): the host selects the frames whose
    //      window fits 63 x 63 tiles (centred views; uncentered ones of worlds below 64 tiles)
    int low_x, high_x, low_y, high_y;
    if (s.opt_center_agent) {
        const double margin = (double)v.visibility / 2.0 + 1;
        low_x = (int)((double)v.center_x - margin);
        high_x = (int)((double)v.center_x + margin);
        low_y = (int)((double)v.center_y - margin);
        high_y = (int)((double)v.center_y + margin);
    } else {
        low_x = 0; high_x = s.main_width - 1; low_y = 0; high_y = s.main_height - 1;
    }
    const int ww = high_x - low_x + 1, wh = high_y - low_y + 1;
    if (!pg_rf_serves(s) || d.gen_bg || ww > 63 || wh > 63) err = true; // the host routes such frames to kernel 3
    // ---- Qt blit setup of window tile column `lane`, window tile row `lane`, the background (lane 63)
    int4 bgi = make_int4(0, 0, 0, 0);
    double bg_rx = 0, bg_ry = 0, bg_rw = 0, bg_rh = 0;
    if (s.opt_use_backgrounds) {
        double mx, my, mw, mh;
        screen_rect(v, 0, (float)s.main_height, (float)s.main_width, (float)s.main_height, 0, mx, my, mw, mh);
        bgi = reinterpret_cast<const int4 *>(d.backgrounds)[s.background_index];
        const float bgw = (float)bgi.y, bgh = (float)bgi.z;
        const float bg_ar = bgw / bgh;
        const float world_ar = (float)(s.main_width * 1.0 / s.main_height);
        const float extra_w = bg_ar - world_ar;
        const float offset_x = s.bg_pct_x * extra_w;
        const double ax = (double)(-offset_x), aw = (double)(bg_ar / world_ar); // adjust_rect (qt-utils.h:12-19)
        bg_rx = mx + mw * ax; bg_ry = my + mh * 0.0; bg_rw = mw * aw; bg_rh = mh * 1.0;
    }
    Axis ca_ = {0, 0, 0u, 0}, ra_ = {0, 0, 0u, 0}; // this lane's column / row axis (FAST), lane 63: background
    bool okx, oky;
    {
        double xr = 0, xw = 0, yr = 0, yh = 0;
        int xiw = 0, yih = 0;
        if (lane == 63) {
            if (s.opt_use_backgrounds) { xr = bg_rx; xw = bg_rw; xiw = bgi.y; yr = bg_ry; yh = bg_rh; yih = bgi.z; }
        } else if (FAST) {
            double rx, ry, rw, rh;
            if (lane < ww) {
                screen_rect(v, (float)(low_x + lane), 0.0f, 1, 1, RENDER_EPS, rx, ry, rw, rh);
                xr = rx; xw = rw; xiw = TP;
            }
            if (lane < wh) {
                screen_rect(v, 0.0f, (float)(low_y + lane + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
                yr = ry; yh = rh; yih = TP;
            }
        }
        okx = axis_setup(xr, xw, xiw, ca_);
        oky = axis_setup(yr, yh, yih, ra_);
        if (!okx) ca_.n = 0;
        if (!oky) ra_.n = 0;
    }
    Axis bx, by;
    const bool bg_ok = readlane(okx && oky ? 1 : 0, 63) != 0;
    bx.t1 = readlane(ca_.t1, 63); bx.n = readlane(ca_.n, 63); bx.base = (uint32_t)readlane((int)ca_.base, 63); bx.step = readlane(ca_.step, 63);
    by.t1 = readlane(ra_.t1, 63); by.n = readlane(ra_.n, 63); by.base = (uint32_t)readlane((int)ra_.base, 63); by.step = readlane(ra_.step, 63);
    // source row offset of screen row `lane` in the background (-1: outside the blit)
    int bg_lane_row = (bg_ok && lane >= by.t1 && lane < by.t1 + by.n)
                          ? (int)(((by.base + (uint32_t)((lane - by.t1) * by.step)) >> 16) * (uint32_t)bgi.y)
                          : -1;
    bool bg_tiled_ok = bg_ok;
    if (s.opt_use_backgrounds && s.bg_tile_ratio < 0) { // tile_image(main_rect, bg_tile_ratio < 0) (:849-862, 1003-1004)
        double mx, my, mw, mh;
        screen_rect(v, 0, (float)s.main_height, (float)s.main_width, (float)s.main_height, 0, mx, my, mw, mh);
        const float tile_ratio = -1 * s.bg_tile_ratio;
        int num_tiles = (int)(mh / (mw * tile_ratio));
        if (num_tiles < 1) num_tiles = 1;
        const float th = (float)(mh / num_tiles), tw = (float)mw;
        bg_tiled_ok = axis_setup(mx, (double)tw, bgi.y, bx);
        bg_lane_row = -1;
        for (int t0 = 0; t0 < num_tiles; t0 += 64) {
            Axis ty;
            const int t = t0 + lane;
            const bool okt = t < num_tiles && axis_setup(my + (double)(th * (float)t), (double)th, bgi.z, ty);
            const int tt1 = okt ? ty.t1 : 0, tn = okt ? ty.n : 0, tstep = okt ? ty.step : 0;
            const uint32_t tbase = okt ? ty.base : 0u;
            for (int k = 0; k < 64 && t0 + k < num_tiles; k++) {
                const int a1 = readlane(tt1, k), an = readlane(tn, k);
                if (lane >= a1 && lane < a1 + an) {
                    const uint32_t b = (uint32_t)readlane((int)tbase, k);
                    const int st = readlane(tstep, k);
                    bg_lane_row = (int)(((b + (uint32_t)((lane - a1) * st)) >> 16) * (uint32_t)bgi.y);
                }
            }
        }
        if (!bg_tiled_ok) bg_lane_row = -1;
    }
    bool bg_col = bg_tiled_ok && lane >= bx.t1 && lane < bx.t1 + bx.n;
    uint32_t bg_col_base = (uint32_t)bgi.x + (bg_col ? (bx.base + (uint32_t)((lane - bx.t1) * bx.step)) >> 16 : 0);
    if constexpr (G == PG_GAME_STARPILOT) {
        // starpilot game_draw (starpilot.cpp:107-124): tile_image(r_bg, 1) of a background scrolled left
        // by cur_time -- 18 square tiles side by side; a screen column shows the last tile covering it
        bg_col = false;
        bg_lane_row = -1;
        if (s.opt_use_backgrounds) {
            const float scale = (float)(PG_RES / s.main_height); // int / int
            const float bg_k = 3, t = (float)s.cur_time, BG_RATIO = 18;
            const float x_off = -t * scale * SP_HP_SLOW_V * 2 / s.char_dim;
            const double rx = (double)x_off, ry = (double)(-PG_RES * (bg_k - 1) / 2);
            const double rw = (double)(PG_RES * bg_k * BG_RATIO), rh = (double)(PG_RES * bg_k);
            int num_tiles = (int)(rw / (rh * 1.0f));
            if (num_tiles < 1) num_tiles = 1;
            const float tw = (float)(rw / num_tiles), th = (float)rh;
            Axis sy;
            const bool sok = axis_setup(ry, (double)th, bgi.z, sy);
            bg_lane_row = (sok && lane >= sy.t1 && lane < sy.t1 + sy.n)
                              ? (int)(((sy.base + (uint32_t)((lane - sy.t1) * sy.step)) >> 16) * (uint32_t)bgi.y)
                              : -1;
            for (int t0 = 0; t0 < num_tiles; t0 += 64) {
                Axis tx;
                const int k0 = t0 + lane;
                const bool okt = k0 < num_tiles && axis_setup(rx + (double)(tw * (float)k0), (double)tw, bgi.y, tx);
                const int tt1 = okt ? tx.t1 : 0, tn = okt ? tx.n : 0, tstep = okt ? tx.step : 0;
                const uint32_t tbase = okt ? tx.base : 0u;
                for (int k = 0; k < 64 && t0 + k < num_tiles; k++) {
                    const int a1 = readlane(tt1, k), an = readlane(tn, k);
                    if (lane >= a1 && lane < a1 + an) {
                        const uint32_t bb = (uint32_t)readlane((int)tbase, k);
                        const int st = readlane(tstep, k);
                        bg_col = true;
                        bg_col_base = (uint32_t)bgi.x + ((bb + (uint32_t)((lane - a1) * st)) >> 16);
                    }
                }
            }
            if (!sok) bg_col = false;
        }
    }
    const uint32_t *bgpix = d.pixels;

    // ---- grid tiles: the tile columns covering screen column `lane` (<= 2, ascending x) and the tile
    //      rows covering screen row `lane` (<= 2, ascending y = the reference's draw order)
    const int xg = (int)floorf(((float)lane + 0.5f + v.x_off) / v.unit);
    const int yg = (int)floorf((v.view_dim - ((float)lane + 0.5f - v.y_off) / v.unit));
    int scol0 = 0, scol1 = 0, rinfo = 0; // FAST: source columns; per row (lane = row) the packed row info
    RfGen gn;
    bool tiles = false;
    if constexpr (FAST) {
        int cx0 = 0, cx1 = 0, ncx = 0, ry0 = 0, ry1 = 0, ncy = 0, srow0 = 0, srow1 = 0;
#pragma unroll
        for (int dx = -2; dx <= 2; dx++) {
            const int x = xg + dx, i = (x - low_x) & 63;
            const int t1 = __shfl(ca_.t1, i), n = __shfl(ca_.n, i), b = __shfl((int)ca_.base, i), st = __shfl(ca_.step, i);
            if (x >= low_x && x <= high_x && ncx < 2 && n > 0 && lane >= t1 && lane < t1 + n) {
                const int scv = (int)(((uint32_t)b + (uint32_t)((lane - t1) * st)) >> 16);
                if (ncx == 0) { cx0 = x; scol0 = scv; } else { cx1 = x; scol1 = scv; }
                ncx++;
            }
        }
#pragma unroll
        for (int dy = -2; dy <= 2; dy++) {
            const int y = yg + dy, i = (y - low_y) & 63;
            const int t1 = __shfl(ra_.t1, i), n = __shfl(ra_.n, i), b = __shfl((int)ra_.base, i), st = __shfl(ra_.step, i);
            if (y >= low_y && y <= high_y && ncy < 2 && n > 0 && lane >= t1 && lane < t1 + n) {
                const int srv = (int)(((uint32_t)b + (uint32_t)((lane - t1) * st)) >> 16);
                if (ncy == 0) { ry0 = y; srow0 = srv; } else { ry1 = y; srow1 = srv; }
                ncy++;
            }
        }
        int jlo = ncy > 0 ? ry0 : 0x7fffffff, jhi = ncy > 1 ? ry1 : (ncy > 0 ? ry0 : -0x7fffffff);
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            jlo = min(jlo, __shfl_xor(jlo, sh));
            jhi = max(jhi, __shfl_xor(jhi, sh));
        }
        const int jy0 = jlo, nrows = jhi >= jlo ? jhi - jlo + 1 : 0;
        if (nrows > CR) err = true; // more tile rows than the table holds (not met by centred views)
        auto grid_at = [&](int x, int y) -> int {
            return (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x] : s.out_of_bounds_object;
        };
        int g0[CR], g1[CR];
#pragma unroll
        for (int j = 0; j < CR; j++) {
            g0[j] = g1[j] = SPACE;
            if (j < nrows && ncx > 0) g0[j] = grid_at(cx0, jy0 + j);
            if (j < nrows && ncx > 1) g1[j] = grid_at(cx1, jy0 + j);
        }
        wave_sync(); // tile_off complete
        auto slot_of = [&](int t) -> int { // 255: nothing drawn; a tile the fast path cannot draw sets err
            if (t == INVALID_OBJ || t == SPACE) return 255;
            if (t < 0 || t >= NTYPES) { err = true; return 255; }
            if (tile_off[t] <= -2) err = true;
            return tile_off[t] == -1 ? 255 : t;
        };
#pragma unroll
        for (int j = 0; j < CR; j++)
            if (j < nrows) codes[j * 64 + lane] = (uint16_t)(slot_of(g0[j]) | (slot_of(g1[j]) << 8));
        // per screen row: source rows of its tile rows (7 bits each), their rows in `codes` (5 bits each),
        // tile-row count (2 bits)
        rinfo = ncy == 0 ? 0
              : (srow0 | ((ncy > 1 ? srow1 : 0) << 7) | ((ry0 - jy0) << 14) | ((ncy > 1 ? ry1 - jy0 : ry0 - jy0) << 19) |
                 (ncy << 24));
        tiles = true;
    } else if constexpr (GEN) {
        const int gs = rf_gen_setup<G>(d, s, v, Gd, player_img, low_x, low_y, ww, wh, xg, yg, ti, gw, gn);
        if (gs == 0) err = true; // not expressible (LDS-frame kernel: the stamped tile pass)
        tiles = gs == 1;
        rinfo = gn.ncy == 0 ? 0 : (gn.ry0 | ((gn.ncy > 1 ? gn.ry1 : 0) << 8) | (gn.ncy << 16));
    }

    // ---- visible images in draw order: z = -1, 0, 1 entities (the list order within each), the
    //      velocity squares (:969-977), the game's overlays.  D0 = (ex.t1 | ex.n << 8 | ey.t1 << 16 |
    //      ey.n << 24, A, B, C), D1 = (E, F, sw | mir << 13 | (z + 1) << 14 | kind << 17 | ca << 19, fill);
    //      plain: A..F = ex.base, ex.step, ey.base, ey.step, soff; RF_ROT: A = rdesc slot; RF_ROWS: A = row
    //      table offset, B, C = dx, dy, fill = colour
    int nd = 0, nrot = 0;
    auto put = [&](bool vis, const Img &im, int z, int kind, int a, int b, int c) {
        const unsigned long long vm = ballot(vis);
        const int rank = nd + __popcll(vm & ((1ull << lane) - 1));
        if (vis && rank < DCAP) {
            const bool pl = kind == RF_PLAIN;
            desc[2 * rank] = make_int4(im.ex.t1 | (im.ex.n << 8) | (im.ey.t1 << 16) | (im.ey.n << 24),
                                       pl ? (int)im.ex.base : a, pl ? im.ex.step : b, pl ? (int)im.ey.base : c);
            desc[2 * rank + 1] = make_int4(pl ? im.ey.step : 0, pl ? im.soff : 0,
                                           (im.sw & 0x1fff) | (im.mir ? 1 << 13 : 0) | ((z + 1) << 14) | (kind << 17) | (im.ca << 19),
                                           (int)im.fill);
        }
        nd += __popcll(vm);
    };
    auto put_plain = [&](bool vis, const Img &im, int z) { put(vis, im, z, RF_PLAIN, 0, 0, 0); };
    const int n = s.num_ents;
    for (int base = 0; base < n; base += 64) {
        Img im;
        entity_setup<G>(d, s, v, env, base + lane, n, player_img, im, err);
        if constexpr (has_rotation<G>()) {
            nrot += rot_stage(im, reinterpret_cast<uint8_t *>(rdesc), RCAP, nrot);
            if (im.draw && im.rot == 1) err = true; // past RCAP descriptors
        }
        const bool vis = im.draw && (im.ez == 0 || im.ez == 1 || (has_z_minus1<G>() && im.ez == -1));
        const int z = vis ? im.ez : 0;
        const unsigned long long tm = has_tiled_entities<G>() ? ballot(vis && im.ntile > 0) : 0ull;
        if (!tm) {
            put(vis, im, z, im.rot == 2 ? RF_ROT : RF_PLAIN, im.rdi, 0, 0);
        } else {
            // tile_image entities (:849-877) become one plain descriptor per tile, in the entity's place
            unsigned long long rem = ballot(vis);
            while (rem) {
                const unsigned long long tl = rem & tm;
                const int jt = tl ? __ffsll((long long)tl) - 1 : 64;
                const unsigned long long run = rem & (jt < 64 ? ((1ull << jt) - 1) : ~0ull);
                put(((run >> lane) & 1) != 0, im, z, im.rot == 2 ? RF_ROT : RF_PLAIN, im.rdi, 0, 0);
                rem &= ~run;
                if (jt == 64) break;
                rem &= ~(1ull << jt);
                const int ntile = readlane(im.ntile, jt), zj = readlane(z, jt);
                const double rx = readlane_d(im.rx, jt), ry = readlane_d(im.ry, jt);
                const float tw = __builtin_bit_cast(float, readlane(__builtin_bit_cast(int, im.tw), jt));
                const float th = __builtin_bit_cast(float, readlane(__builtin_bit_cast(int, im.th), jt));
                const int vert = readlane(im.rslot, jt);
                const int offj = readlane(im.soff, jt), swj = readlane(im.sw, jt), shj = readlane(im.sh, jt);
                const int mirj = readlane(im.mir, jt), caj = readlane(im.ca, jt);
                const double tsz = vert ? (double)th : (double)tw, org = vert ? ry : rx;
                int tlo = 0, thi = ntile;
                if (tsz > 0) {
                    tlo = max(0, (int)floor((-2.0 - org) / tsz) - 1);
                    thi = min(ntile, (int)ceil((PG_RES + 2.0 - org) / tsz) + 1);
                }
                for (int t0 = tlo; t0 < thi; t0 += 64) {
                    Img tim;
                    img_clear(tim);
                    const int t = t0 + lane;
                    bool ok = false;
                    if (t < thi) {
                        const double x = vert ? rx : rx + (double)(tw * (float)t);
                        const double y = vert ? ry + (double)(th * (float)t) : ry;
                        ok = axis_setup(x, (double)tw, swj, tim.ex) && axis_setup(y, (double)th, shj, tim.ey);
                        tim.soff = offj; tim.sw = swj; tim.sh = shj; tim.mir = mirj; tim.ca = caj;
                    }
                    put_plain(ok, tim, zj);
                }
            }
        }
    }
    if (__builtin_expect(s.has_useful_vel_info && s.opt_paint_vel_info, 0)) { // paint_vel_info (:969-977)
        const float vx = s.agent_erased ? s.ghost_vx : EFr(d, F_VX, env, 0);
        const float vy = s.agent_erased ? s.ghost_vy : EFr(d, F_VY, env, 0);
        const float infodim = (float)(PG_RES * .2);
        const uint32_t s1 = (uint32_t)to_shade((float)(.5 * (double)vx / (double)s.maxspeed + .5));
        const uint32_t s2 = (uint32_t)to_shade((float)(.5 * (double)vy / (double)s.max_jump + .5));
        Img im;
        img_clear(im);
        bool vis = false;
        if (lane == 0) vis = fill_setup(0, 0, infodim, infodim, 0xff000000u | (s1 * 0x010101u), im);
        if (lane == 1) vis = fill_setup(infodim, 0, infodim, infodim, 0xff000000u | (s2 * 0x010101u), im);
        put_plain(vis, im, 2);
    }
    // ---- game_draw overlays (game_overlay): fills, jumper's compass rows
    if constexpr (G == PG_GAME_NINJA || G == PG_GAME_PLUNDER) {
        Img im;
        img_clear(im);
        bool vis = false;
        const float u = v.unit;
        if constexpr (G == PG_GAME_NINJA) { // jump charge bar (ninja.cpp:155-164)
            const float bar_height = 3 * s.gs.nj.jump_charge;
            if (lane == 0)
                vis = fill_setup((double)(.25f * u), (double)((float)(v.visibility - .5 - bar_height) * u), (double)(.5f * u),
                                 (double)(bar_height * u), 0xff42f587u, im);
        } else { // juice and progress bars (plunder.cpp:66-77)
            const float prog = (float)(s.main_width * (s.gs.pl.targets_hit * 1.0 / s.gs.pl.target_quota));
            if (lane == 0)
                vis = fill_setup((double)(.25f * u), (double)(.25f * u), (double)(s.main_width * s.gs.pl.juice_left * u),
                                 (double)(.5f * u), 0xff42f587u, im);
            if (lane == 1)
                vis = fill_setup((double)(.25f * u), (double)(.75f * u), (double)(prog * u), (double)(.5f * u), 0xfff54290u, im);
        }
        put_plain(vis, im, 3);
    }
    if constexpr (G == PG_GAME_JUMPER) {
        if (s.opt_distribution_mode != PG_MEMORY) { // jp_draw_compass (jumper.cpp:137-177)
            bool ok = true;
            const int4 tix = reinterpret_cast<const int4 *>(d.sprites)[PG_TABLE_SLOT];
            const uint32_t toff = (uint32_t)tix.x;
            const uint32_t *t = d.pixels + toff;
            int NY = 0, NX = 0, MAXW = 0, MAXH = 0;
            if (tix.y <= 0) ok = false;
            else { NY = (int)t[1]; NX = (int)t[2]; MAXW = (int)t[3]; MAXH = (int)t[4]; }
            const int cfg = (s.opt_distribution_mode == PG_EASY ? 0 : 1) + (s.opt_center_agent ? 0 : 2);
            const float u = v.unit, vd = v.view_dim, cd = s.gs.jp.compass_dim;
            int rows[3] = {-1, -1, -1}, rdx[3] = {0, 0, 0}, rdy[3] = {0, 0, 0};
            uint32_t rcol[3] = {0xffa8a69eu, 0xfffcba03u, 0x78787878u};
            Img bar;
            img_clear(bar);
            bool bar_vis = false;
            if (ok) {
                const uint32_t *cg = t + 5 + 9 * cfg;
                const int bx0 = (int)cg[2], by0 = (int)cg[3], bnx = (int)cg[4], bny = (int)cg[5];
                const float cx = __uint_as_float(cg[6]), cy = __uint_as_float(cg[7]), cr = __uint_as_float(cg[8]);
                const uint32_t dial = 5 + 36, needle = dial + 4 * 128;
                const uint32_t jump = needle + (uint32_t)(4 * NY * NX * 128);
                const double rx = (double)((float)(vd - cd - .25) * u), rw = (double)(cd * u);
                if ((float)(rx + rw / 2) != cx) ok = false; // the table was built for this frame geometry
                rows[0] = (int)(toff + dial + 128 * cfg);
                const float ax = EFr(d, F_X, env, 0), ay = EFr(d, F_Y, env, 0), arx = EFr(d, F_RX, env, 0), ary = EFr(d, F_RY, env, 0);
                const float gx = EFr(d, F_X, env, 1), gy = EFr(d, F_Y, env, 1);
                const float theta = (float)atan2((double)(gy - ay), (double)(gx - ax)); // get_theta (:241-246)
                double sn, cs;
                pg_sincos_cr((double)theta, &sn, &cs);
                const int x2 = (int)((double)cx + (double)cr * cs), y2 = (int)((double)cy - (double)cr * sn);
                if (x2 < bx0 || x2 >= bx0 + bnx || y2 < by0 || y2 >= by0 + bny) ok = false;
                else rows[1] = (int)(toff + needle + (uint32_t)(((cfg * NY + (y2 - by0)) * NX + (x2 - bx0)) * 128));
                const float ddx = ax - gx, ddy = ay - gy; // get_distance (:133-143)
                const float dist = (float)sqrt((double)(ddx * ddx + ddy * ddy));
                const float dist_pct = (float)((double)dist / (s.main_width * 1.4142135623730951));
                const float bar_thickness = cd / 8;
                bar_vis = fill_setup((double)((float)(vd - cd - .25) * u), (double)((float)(.25 + cd) * u),
                                     (double)(cd * dist_pct * u), (double)(bar_thickness * u), 0xfffcba03u, bar);
                if (s.gs.jp.jump_delta < 0 && !s.has_support) { // drawEllipse(QRect(...)) of get_object_rect(agent)
                    double r1x, r1y, r1w, r1h;
                    screen_rect(v, ax - arx, ay + ary, 2 * arx, 2 * ary, 0, r1x, r1y, r1w, r1h);
                    const int qx = (int)r1x, qy = (int)(r1y + r1h * (5.0 / 6)), qw = (int)r1w, qh = (int)(r1h / 3);
                    if (qw < 0 || qw > MAXW || qh < 0 || qh > MAXH) ok = false;
                    else { rows[2] = (int)(toff + jump + (uint32_t)((qw * (MAXH + 1) + qh) * 128)); rdx[2] = qx - 20; rdy[2] = qy - 20; }
                }
            }
            if (!ok) err = true;
            // the row bitmaps in draw order (dial, needle; bar; jump ellipse), each with the rows it sets
            for (int k = 0; k < 3; k++) {
                if (k == 2) put_plain(lane == 0 && bar_vis, bar, 3);
                if (rows[k] < 0 || rdx[k] <= -64 || rdx[k] >= 64) continue;
                const int sy = lane; // bitmap row
                const uint32_t w0 = d.pixels[(uint32_t)rows[k] + 2 * sy], w1 = d.pixels[(uint32_t)rows[k] + 2 * sy + 1];
                uint64_t m = (uint64_t)w0 | ((uint64_t)w1 << 32);
                m = rdx[k] >= 0 ? (m << rdx[k]) : (m >> -rdx[k]);
                const int y = sy + rdy[k];
                const unsigned long long nz = ballot(m != 0 && y >= 0 && y < PG_RES);
                if (!nz) continue;
                const int y0 = __ffsll((long long)nz) - 1 + rdy[k], y1 = 63 - __clzll(nz) + rdy[k] + 1;
                Img im;
                img_clear(im);
                im.ex.t1 = 0; im.ex.n = PG_RES; im.ey.t1 = y0; im.ey.n = y1 - y0; im.fill = rcol[k];
                put(lane == 0, im, 3, RF_ROWS, rows[k], rdx[k], rdy[k]);
            }
        }
    }
    if (nd > DCAP) err = true;
    nd = min(nd, DCAP);
    wave_sync(); // tables and descriptors complete

    const int bgrow = bg_lane_row;
    const uint32_t npix = d.num_pixels;
    uint32_t *out = reinterpret_cast<uint32_t *>(d.rgb + (size_t)env * PG_OBS_BYTES);
    for (int r0 = 0; r0 < PG_RES; r0 += RF_RB) {
        // ---- image jobs: a cursor over the images crossing rows [r0, r0 + RF_RB) in draw order,
        //      segments (z, descriptor group of 64) from z = zlo
        int seg = 0, segend = 0, grp = 0;
        unsigned long long mask = 0;
        int C0 = 0, C1 = 0, C2 = 0, C3 = 0, C4 = 0, C5 = 0, C6 = 0, C7 = 0; // the current image's descriptor (uniform)
        int y = 0, yend = 0;
        constexpr int NG = DCAP / 64;
        auto next_image = [&]() -> bool {
            while (mask == 0) {
                if (seg >= segend) return false;
                const int z = seg / NG - 1;
                grp = (seg % NG) * 64;
                seg++;
                if (grp >= nd) continue;
                const int k = grp + lane;
                const bool live = k < nd;
                const int4 A = desc[2 * (live ? k : 0)];
                const int zz = ((desc[2 * (live ? k : 0) + 1].z >> 14) & 7) - 1;
                const int yt1 = (A.x >> 16) & 255, yn = (A.x >> 24) & 255;
                mask = ballot(live && zz == z && yt1 < r0 + RF_RB && yt1 + yn > r0);
            }
            const int cur = __ffsll((long long)mask) - 1;
            mask &= mask - 1;
            const int4 A = desc[2 * (grp + cur)], B = desc[2 * (grp + cur) + 1];
            C0 = __builtin_amdgcn_readfirstlane(A.x); C1 = __builtin_amdgcn_readfirstlane(A.y);
            C2 = __builtin_amdgcn_readfirstlane(A.z); C3 = __builtin_amdgcn_readfirstlane(A.w);
            C4 = __builtin_amdgcn_readfirstlane(B.x); C5 = __builtin_amdgcn_readfirstlane(B.y);
            C6 = __builtin_amdgcn_readfirstlane(B.z); C7 = __builtin_amdgcn_readfirstlane(B.w);
            const int yt1 = (C0 >> 16) & 255, yn = (C0 >> 24) & 255;
            y = max(r0, yt1);
            yend = min(r0 + RF_RB, yt1 + yn);
            return true;
        };
        auto start = [&](int zlo, int zhi) { // segments of z in [zlo, zhi]
            seg = (zlo + 1) * NG;
            segend = (zhi + 2) * NG;
            mask = 0;
            return next_image();
        };
        uint32_t jt[RF_JOBS];
        int jr[RF_JOBS], jca[RF_JOBS];
        bool more = false;
        auto issue_jobs = [&]() {
#pragma unroll
            for (int q = 0; q < RF_JOBS; q++) {
                jr[q] = -1;
                jt[q] = 0;
                jca[q] = 256;
                if (more) {
                    const int w2 = C6, kind = (w2 >> 17) & 3;
                    const int ca = (w2 >> 19) & 511;
                    uint32_t t = 0;
                    if (kind == RF_PLAIN) {
                        const uint32_t exb = (uint32_t)C1, eyb = (uint32_t)C3, soff = (uint32_t)C5, fill = (uint32_t)C7;
                        const int exs = C2, eys = C4;
                        const int xt1 = C0 & 255, xn = (C0 >> 8) & 255, yt1 = (C0 >> 16) & 255;
                        const int sw = w2 & 0x1fff;
                        const int dxl = lane - xt1;
                        if ((unsigned)dxl < (unsigned)xn) {
                            if (fill != 0) {
                                t = fill;
                            } else {
                                int scol = (int)((exb + (uint32_t)(dxl * exs)) >> 16);
                                if ((w2 >> 13) & 1) scol = sw - 1 - scol;
                                const int srow = (int)((eyb + (uint32_t)((y - yt1) * eys)) >> 16);
                                const uint32_t idx = soff + (uint32_t)(srow * sw + scol);
                                if (idx < npix) t = d.pixels[idx];
                                else err = true;
                            }
                        }
                        jca[q] = ca;
                    } else if (has_rotation<G>() && kind == RF_ROT) {
                        // rot_pixel at (lane, y): the trapezoid holding scan line y, its [fromX, toX)
                        const int4 *R = rdesc + 6 * C1;
                        const int4 a5 = R[5];
                        const int f0 = a5.x & 255, e0 = (a5.x >> 8) & 255, f1 = (a5.x >> 16) & 255, e1 = (a5.x >> 24) & 255;
                        const int f2 = a5.y & 255, e2 = (a5.y >> 8) & 255;
                        const int tk = (y >= f0 && y < e0) ? 0 : ((y >= f1 && y < e1) ? 1 : ((y >= f2 && y < e2) ? 2 : 3));
                        if (tk < 3) {
                            const int from = tk == 0 ? f0 : (tk == 1 ? f1 : f2);
                            const int4 e = R[tk], a3 = R[3], a4 = R[4];
                            const int xlv = e.x + (y - from) * e.y, xrv = e.z + (y - from) * e.w;
                            const int fromX = max(xlv >> 16, 0), toX = min(xrv >> 16, PG_RES);
                            if (lane >= fromX && lane < toX) {
                                const int iw = a4.w & 0xffff, ih = a4.w >> 16;
                                int uu = (lane * a3.x + y * a3.z + a4.x) >> 16;
                                int vv = (lane * a3.y + y * a3.w + a4.y) >> 16;
                                uu = min(max(uu, 0), iw - 1);
                                vv = min(max(vv, 0), ih - 1);
                                if ((a5.y >> 16) & 1) uu = iw - 1 - uu;
                                const uint32_t idx = (uint32_t)a4.z + (uint32_t)(vv * iw + uu);
                                if (idx < npix) t = d.pixels[idx];
                                else err = true;
                            }
                        }
                        jca[q] = a5.z & 0xffff;
                    } else if (G == PG_GAME_JUMPER && kind == RF_ROWS) {
                        const int sy = y - C3, bit = lane - C2;
                        if (sy >= 0 && sy < PG_RES && bit >= 0 && bit < 64) {
                            const uint32_t w = d.pixels[(uint32_t)C1 + 2 * sy + (bit >> 5)];
                            if ((w >> (bit & 31)) & 1) t = (uint32_t)C7;
                        }
                        jca[q] = 256;
                    }
                    jt[q] = t;
                    jr[q] = y - r0;
                    if (++y >= yend) more = next_image();
                }
            }
        };
        auto blend_jobs = [&](uint32_t (&px)[RF_RB]) {
#pragma unroll
            for (int q = 0; q < RF_JOBS; q++) {
                if (jr[q] < 0) break; // uniform
#pragma unroll
                for (int k = 0; k < RF_RB; k++)
                    if (k == jr[q]) px[k] = blend_argb_pm(px[k], jt[q], jca[q]);
            }
        };
        // ---- background + grid tile texels of the batch
        uint32_t px[RF_RB], t00[RF_RB], t01[RF_RB], t10[RF_RB], t11[RF_RB];
#pragma unroll
        for (int k = 0; k < RF_RB; k++) {
            const int br = readlane(bgrow, r0 + k);
            const bool inb = bg_col && br >= 0;
            const uint32_t bv = bgpix[inb ? bg_col_base + (uint32_t)br : 0u];
            px[k] = inb ? bv : 0xff000000u;
            t00[k] = t01[k] = t10[k] = t11[k] = 0;
            if constexpr (FAST) {
                const int info = readlane(rinfo, r0 + k);
                const int nr = info >> 24;
                const int c0 = codes[((info >> 14) & 31) * 64 + lane];
                const int c1 = nr > 1 ? codes[((info >> 19) & 31) * 64 + lane] : 0xffff;
                const int sr0 = (info & 127) * TP, sr1 = ((info >> 7) & 127) * TP;
#ifdef RF_DIAG_NOCOL // diagnostic only (wrong frames): every lane of a tile reads its first column
                scol0 = scol1 = 0;
#endif
                if (nr > 0 && (c0 & 255) != 255) t00[k] = d.pixels[(uint32_t)tile_off[c0 & 255] + (uint32_t)(sr0 + scol0)];
                if (nr > 1 && (c1 & 255) != 255) t01[k] = d.pixels[(uint32_t)tile_off[c1 & 255] + (uint32_t)(sr1 + scol0)];
                if (nr > 0 && (c0 >> 8) != 255) t10[k] = d.pixels[(uint32_t)tile_off[c0 >> 8] + (uint32_t)(sr0 + scol1)];
                if (nr > 1 && (c1 >> 8) != 255) t11[k] = d.pixels[(uint32_t)tile_off[c1 >> 8] + (uint32_t)(sr1 + scol1)];
            } else if constexpr (GEN) {
                if (tiles) {
                    const int info = readlane(rinfo, r0 + k);
                    const int ny = info >> 16, y0 = info & 255, y1 = (info >> 8) & 255;
                    int ysr[GEN_K];
#pragma unroll
                    for (int q = 0; q < GEN_K; q++) ysr[q] = readlane(gn.ys[q], r0 + k);
                    if (ny > 0 && gn.ncx > 0) t00[k] = rf_gen_texel(d, ti[gw[y0 * ww + gn.cx0]], gn.xs, ysr, false, false, err);
                    if (ny > 1 && gn.ncx > 0) t01[k] = rf_gen_texel(d, ti[gw[y1 * ww + gn.cx0]], gn.xs, ysr, false, true, err);
                    if (ny > 0 && gn.ncx > 1) t10[k] = rf_gen_texel(d, ti[gw[y0 * ww + gn.cx1]], gn.xs, ysr, true, false, err);
                    if (ny > 1 && gn.ncx > 1) t11[k] = rf_gen_texel(d, ti[gw[y1 * ww + gn.cx1]], gn.xs, ysr, true, true, err);
                }
            }
        }
        if constexpr (has_z_minus1<G>()) { // z = -1 entities go between the background and the tiles (:933)
            more = start(-1, -1);
            while (more) {
                issue_jobs();
                blend_jobs(px);
            }
        }
        more = start(0, 3);
        issue_jobs(); // the first round of image texels rides on the same memory round trip
        uint32_t part = 0;
#pragma unroll
        for (int k = 0; k < RF_RB; k++) part |= alpha_partial(t00[k]) | alpha_partial(t01[k]) | alpha_partial(t10[k]) | alpha_partial(t11[k]);
        if (!ballot(part != 0)) {
#pragma unroll
            for (int k = 0; k < RF_RB; k++)
                px[k] = over_binary(over_binary(over_binary(over_binary(px[k], t00[k]), t01[k]), t10[k]), t11[k]);
        } else {
#pragma unroll
            for (int k = 0; k < RF_RB; k++) {
                px[k] = blend_argb_pm(px[k], t00[k], 256);
                px[k] = blend_argb_pm(px[k], t01[k], 256);
                px[k] = blend_argb_pm(px[k], t10[k], 256);
                px[k] = blend_argb_pm(px[k], t11[k], 256);
            }
        }
        blend_jobs(px);
        while (more) {
            issue_jobs();
            blend_jobs(px);
        }
        // ---- bgr32_to_rgb888 (game.cpp:8-23): dword w of a row's 192 bytes takes bytes of pixels
        //      4w / 3 and 4w / 3 + 1 (phase w % 3); lanes 0..47 store one dword each
        // v_perm_b32 picks the four bytes of {b, a} (a = bytes 0-3: B G R A of pixel 4w / 3):
        // phase 0 -> R_a G_a B_a R_b, 1 -> G_a B_a R_b G_b, 2 -> B_a R_b G_b B_b
        const int p1 = (4 * lane) / 3, ph = lane % 3;
        const uint32_t sel = ph == 0 ? 0x06000102u : (ph == 1 ? 0x05060001u : 0x04050600u);
#pragma unroll
        for (int k = 0; k < RF_RB; k++) {
            const uint32_t a = (uint32_t)__shfl((int)px[k], p1 & 63), b = (uint32_t)__shfl((int)px[k], (p1 + 1) & 63);
            if (lane < 48) out[(r0 + k) * 48 + lane] = __builtin_amdgcn_perm(b, a, sel);
        }
    }
    if (ballot(err) && lane == 0) atomicOr(d.error_any, 1 << PG_ERR_RENDER);
}

// waves per SIMD the register budget is set for (launch bound): 80 VGPRs hold coinrun's and the general
// tile pass's batches without spills at 4 rows per batch; the transform-blit / tile-list games get 128
template <int G>
__host__ __device__ constexpr int rf_waves() {
    return G == PG_GAME_BIGFISH ? 8
         : ((G == PG_GAME_COINRUN || G == PG_GAME_MAZE || G == PG_GAME_MINER || G == PG_GAME_CHASER || G == PG_GAME_CLIMBER ||
             G == PG_GAME_NINJA) ? 6 : 4);
}

template <int G>
__global__ __launch_bounds__(64, rf_waves<G>()) void pg_render_rf_kernel(PGDev dg, const int32_t *env_list, int mode, int slot, int count) {
    if constexpr (rf_game<G>()) {
        const PGDev d = game_view(dg, G);
        __shared__ __attribute__((aligned(16))) uint8_t tab[rf_tab_bytes<G>()];
#ifndef RF_LDS_PAD
#define RF_LDS_PAD 0 // experiment: LDS bytes added per workgroup (caps the waves the render keeps resident)
#endif
        __shared__ __attribute__((aligned(16))) int4 desc[2 * rf_dcap<G>() + RF_LDS_PAD / 16];
        __shared__ __attribute__((aligned(16))) int4 rdesc[6 * rf_rcap<G>()];
        const int bidx = (int)blockIdx.x;
        int env;
        if (mode == 2) {
            if (bidx >= d.reset_count[slot]) return;
            env = d.reset_queue[(size_t)slot * d.num_envs + bidx];
        } else {
            if (bidx >= count) return;
            env = env_list ? env_list[bidx] : bidx;
            if (mode == 1 && d.done8[env]) return;
        }
        rf_render_env<G>(d, env, tab, desc, rdesc);
    }
}

// ================================================================== render_mode="rgb_array"
// The RENDER_RES x RENDER_RES frame of info["rgb"] (vecgame.cpp:318-330, 415-423: Game::render_to_buf
// with antialias = true, game.cpp:97-107): the same game_draw as the observation, painted with
// QPainter::Antialiasing + SmoothPixmapTransform.  The primitives are the oracle's pinned restatement
// (oracle/procgen_oracle.c qt_smooth_*, tests/test_smooth_pins.py against the real Qt 5.9.7):
//   * a rect -> QRasterizer::rasterizeLine spans (<= 3 per row, 8-bit coverage, 256-span buffer
//     flushes), computed per pixel in closed form;
//   * drawImage -> fetchTransformedBilinearARGB32PM of each span run (a pixel's weights -- 4-bit in
//     the downscale helper's groups of 4, else 8-bit -- follow from its offset in the run), then
//     SourceOver (premultiplied sprites) / Source (opaque RGB32 backgrounds) with the coverage;
//   * fillRect(opaque colour) -> Source with the coverage.
// One 256-thread workgroup per env; the frame lives in HBM (1 MB per env), every primitive is
// painted by all threads over its footprint and a barrier orders it before the next.  The games
// whose draws are all axis-aligned images and fills are built (bigfish, chaser, climber, coinrun,
// maze, miner, ninja); libenv_make rejects render_mode="rgb_array" for the others.
#define HR_RES 512
#define HR_THREADS 256

struct HRect { // QRasterizer::rasterizeLine of one axis-aligned rect (uniform)
    int n;                 // spans per row (0: nothing drawn)
    int xs[3], lens[3], cov[3];
    int r0, r1;            // first / last row
    int yPa, yPb;          // 16.16 top / bottom
    int k1;                // nonzero spans of the first row
    int kM;                // nonzero spans of a full row
};

DEV int hr_span_cov(const HRect &R, int r, int i) {
    const int yFP = r << 16;
    const int rh = min(yFP + 65536, R.yPb) - max(yFP, R.yPa);
    return (int)((((int64_t)rh * (int64_t)(255 * R.cov[i])) >> 16) >> 16) & 0xff;
}
DEV int hr_row_count(const HRect &R, int r) {
    int c = 0;
    for (int i = 0; i < R.n; i++) c += hr_span_cov(R, r, i) != 0;
    return c;
}
DEV void hr_rect(double x, double y, double w, double h, HRect &R) {
    R.n = 0;
    const double ax = (x + x) * 0.5, ay = (y + (y + h)) * 0.5;
    const double bx = ((x + w) + (x + w)) * 0.5, by = ay;
    double width = h / w;
    double pax = ax, pay = ay, pbx = bx, pby = by;
    if (ax == bx && ay == by) return;
    {
        const double offx = fabs(by - ay) * width * 0.5, offy = fabs(bx - ax) * width * 0.5;
        const double cl = 0 - offx, ct = 0 - offy;
        const double cr = cl + ((HR_RES - 1 + 1 + offx) - cl), cb = ct + ((HR_RES - 1 + 1 + offy) - ct);
        const bool in_a = cl <= pax && pax <= cr && ct <= pay && pay <= cb;
        const bool in_b = cl <= pbx && pbx <= cr && ct <= pby && pby <= cb;
        if (!in_a || !in_b) {
            double t1 = 0, t2 = 1;
            const double o[2] = {pax, pay}, dd[2] = {pbx - pax, pby - pay};
            const double low[2] = {cl, ct}, high[2] = {cr, cb};
            for (int i = 0; i < 2; i++) {
                if (dd[i] == 0) {
                    if (o[i] <= low[i] || o[i] >= high[i]) return;
                    continue;
                }
                const double dinv = 1 / dd[i];
                double tl = (low[i] - o[i]) * dinv, th = (high[i] - o[i]) * dinv;
                if (tl > th) { const double t = tl; tl = th; th = t; }
                if (t1 < tl) t1 = tl;
                if (t2 > th) t2 = th;
                if (t1 >= t2) return;
            }
            const double nax = pax + (pbx - pax) * t1, nay = pay + (pby - pay) * t1;
            const double nbx = pax + (pbx - pax) * t2, nby = pay + (pby - pay) * t2;
            pax = nax; pay = nay; pbx = nbx; pby = nby;
        }
    }
    {
        const double d0x = ax - bx, d0y = ay - by, w0 = d0x * d0x + d0y * d0y;
        const double dx = pax - pbx, dy = pay - pby, ww = dx * dx + dy * dy;
        if (ww == 0) return;
        width *= sqrt(w0 / ww);
    }
    {
        const double xm = (pax + pbx) * 0.5f, dx = fabs(pbx - pax) * 0.5f, yy = pay, dy = width * dx;
        pax = xm; pay = yy - dy;
        pbx = xm; pby = yy + dy;
        width = 1 / width;
    }
    if (pay > pby) { const double t = pay; pay = pby; pby = t; }
    const double dy = pby - pay, half = 0.5f * width * dy;
    double left = pax - half, right = pax + half;
    left = left < 0 ? 0 : (left > HR_RES ? HR_RES : left);
    right = right < 0 ? 0 : (right > HR_RES ? HR_RES : right);
    pay = pay < 0 ? 0 : (pay > HR_RES ? HR_RES : pay);
    pby = pby < 0 ? 0 : (pby > HR_RES ? HR_RES : pby);
    if ((int)(left * 64) == (int)(right * 64) || (int)(pay * 64) == (int)(pby * 64)) return;
    const int iL = (int)left, iR = (int)right;
    const int lw = ((iL + 1) << 16) - (int)(left * 65536.), rw = (int)(right * 65536.) - (iR << 16);
    int n = 1;
    if (iL == iR) {
        R.cov[0] = lw + rw; // (sic, Qt 5.9)
        R.xs[0] = iL;
        R.lens[0] = 1;
    } else {
        R.cov[0] = lw; R.xs[0] = iL; R.lens[0] = 1;
        if (lw == 65536) {
            R.lens[0] = iR - iL;
        } else if (iR - iL > 1) {
            R.cov[1] = 65536; R.xs[1] = iL + 1; R.lens[1] = iR - iL - 1;
            n++;
        }
        if (rw) {
            R.cov[n] = rw; R.xs[n] = iR; R.lens[n] = 1;
            n++;
        }
    }
    R.n = n;
    R.r0 = (int)pay;
    R.r1 = min((int)pby, HR_RES - 1);
    R.yPa = (int)(pay * 65536.);
    R.yPb = (int)(pby * 65536.);
    R.k1 = hr_row_count(R, R.r0);
    R.kM = R.r0 + 1 < R.r1 ? hr_row_count(R, R.r0 + 1) : 0;
}
// global index (in the rasterizer's emission order) of row r's first span
DEV int hr_row_base(const HRect &R, int r) {
    if (r == R.r0) return 0;
    return R.k1 + (r - R.r0 - 1) * R.kM;
}

DEV uint32_t hr_interp_256(uint32_t x, uint32_t a, uint32_t y, uint32_t b) {
    uint32_t t = (x & 0xff00ffu) * a + (y & 0xff00ffu) * b;
    t = (t >> 8) & 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a + ((y >> 8) & 0xff00ffu) * b;
    return (x & 0xff00ff00u) | t;
}
DEV uint32_t hr_interp4_8(uint32_t tl, uint32_t tr, uint32_t bl, uint32_t br, uint32_t dx, uint32_t dy) {
    const uint32_t l = hr_interp_256(tl, 256 - dy, bl, dy), r = hr_interp_256(tr, 256 - dy, br, dy);
    return hr_interp_256(l, 256 - dx, r, dx);
}
DEV uint32_t hr_interp4_4(uint32_t tl, uint32_t tr, uint32_t bl, uint32_t br, uint32_t dx, uint32_t dy) {
    const uint32_t dxy = dx * dy;
    const uint32_t wtl = 16 * 16 - 16 * dx - 16 * dy + dxy, wtr = dx * 16 - dxy, wbl = dy * 16 - dxy, wbr = dxy;
    const uint32_t rb = (tl & 0xff00ffu) * wtl + (tr & 0xff00ffu) * wtr + (bl & 0xff00ffu) * wbl + (br & 0xff00ffu) * wbr;
    const uint32_t ag = ((tl >> 8) & 0xff00ffu) * wtl + ((tr >> 8) & 0xff00ffu) * wtr + ((bl >> 8) & 0xff00ffu) * wbl +
                        ((br >> 8) & 0xff00ffu) * wbr;
    return ((rb >> 8) & 0xff00ffu) | (ag & 0xff00ff00u);
}
DEV uint32_t hr_interp_255(uint32_t x, uint32_t a, uint32_t y, uint32_t b) {
    uint32_t t = (x & 0xff00ffu) * a + (y & 0xff00ffu) * b;
    t = (t + ((t >> 8) & 0xff00ffu) + 0x800080u) >> 8;
    t &= 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a + ((y >> 8) & 0xff00ffu) * b;
    x = (x + ((x >> 8) & 0xff00ffu) + 0x800080u);
    x &= 0xff00ff00u;
    return x | t;
}

// n range [lo, hi] (clipped to [0, len)) with 0 <= f0 + n * d <= top
DEV void hr_nrange(int f0, int d, int64_t top, int len, int64_t &lo, int64_t &hi) {
    lo = 0;
    hi = (int64_t)len - 1;
    const int64_t L = -(int64_t)f0, H = top - f0; // n d in [L, H]
    if (d > 0) {
        lo = max(lo, L >= 0 ? (L + d - 1) / d : -((-L) / d));
        hi = min(hi, H >= 0 ? H / d : -((-H + d - 1) / d));
    } else if (d < 0) {
        const int64_t e = -(int64_t)d, a = -H, b = -L; // n e in [a, b]
        lo = max(lo, a >= 0 ? (a + e - 1) / e : -((-a) / e));
        hi = min(hi, b >= 0 ? b / e : -((-b + e - 1) / e));
    } else if (!(L <= 0 && 0 <= H)) {
        lo = hi + 1;
    }
}
// the scale helpers of fetchTransformedBilinearARGB32PM (fdy == 0): pixel n of a run of `len`
struct HTex { const uint32_t *px; int iw, ih, mir; };
DEV uint32_t hr_tex(const HTex &T, int r, int c) { return T.px[(size_t)r * T.iw + (T.mir ? T.iw - 1 - c : c)]; }
DEV uint32_t hr_fetch_scale(const HTex &T, int fx0, int fy, int fdx, double m22, int len, int n) {
    int y1 = fy >> 16, y2;
    if (y1 < 0) y1 = y2 = 0;
    else if (y1 >= T.ih - 1) y1 = y2 = T.ih - 1;
    else y2 = y1 + 1;
    const uint32_t dy8 = (uint32_t)(fy & 0xffff) >> 8, dy4 = (dy8 + 8) >> 4;
    const bool down = !(fdx > 0 && fdx <= 65536) && !(fdx < 0 && fdx > -8192) && !(fabs(m22) < 1. / 8.);
    // leading pixels on a clamped column (vertical interpolation only) end at the first n whose column
    // is inside [0, iw - 1)
    int n0 = len;
    {
        int64_t lo, hi;
        hr_nrange(fx0, fdx, (int64_t)(T.iw - 1) * 65536 - 1, len, lo, hi);
        if (lo <= hi) n0 = (int)lo;
    }
    int64_t bend = len;
    const int fxn0 = fx0 + n0 * fdx;
    if (n0 < len) {
        if (fdx > 0) bend = min(bend, (int64_t)n0 + ((int64_t)(T.iw - 1) * 65536 - fxn0) / fdx);
        else if (fdx < 0) bend = min(bend, (int64_t)n0 + (0 - (int64_t)fxn0) / fdx);
    }
    const int64_t groups = (down && bend - n0 >= 4) ? (bend - n0) / 4 : 0;
    const int fx = fx0 + n * fdx;
    if (n < n0) {
        const int c = (fx >> 16) < 0 ? 0 : T.iw - 1;
        return hr_interp_256(hr_tex(T, y1, c), 256 - dy8, hr_tex(T, y2, c), dy8);
    }
    if (n < n0 + 4 * groups) {
        const int c = fx >> 16;
        const uint32_t dx4 = (((uint32_t)(fx & 0xffff) >> 8) + 8) >> 4;
        return hr_interp4_4(hr_tex(T, y1, c), hr_tex(T, y1, c + 1), hr_tex(T, y2, c), hr_tex(T, y2, c + 1), dx4, dy4);
    }
    int c1 = fx >> 16, c2;
    if (c1 < 0) c1 = c2 = 0;
    else if (c1 >= T.iw - 1) c1 = c2 = T.iw - 1;
    else c2 = c1 + 1;
    return hr_interp4_8(hr_tex(T, y1, c1), hr_tex(T, y1, c2), hr_tex(T, y2, c1), hr_tex(T, y2, c2),
                        (uint32_t)(fx & 0xffff) >> 8, dy8);
}
// one primitive (uniform arguments); all threads of the workgroup
struct HOp {
    int kind;              // 0 image, 1 opaque fill
    double x, y, w, h;
    const uint32_t *px;    // image pixels (row-major iw x ih)
    int iw, ih, rgb32, mir, ca;
    uint32_t argb;
};

DEV void hr_blend(uint32_t *dp, uint32_t s, int cov, bool rgb32) {
    if (rgb32) { // SourceOver of an opaque image = Source (comp_func_Source)
        *dp = cov == 255 ? s : hr_interp_255(s, (uint32_t)cov, *dp, 255 - (uint32_t)cov);
    } else if (cov == 255) { // comp_func_SourceOver
        if (s >= 0xff000000u) *dp = s;
        else if (s != 0) *dp = s + BYTE_MUL(*dp, (~s) >> 24);
    } else {
        s = BYTE_MUL(s, (uint32_t)cov);
        *dp = s + BYTE_MUL(*dp, (~s) >> 24);
    }
}

DEV void hr_paint(uint32_t *frame, const HOp &op) {
    const int tid = threadIdx.x;
    if (op.kind == 0 && op.w == (double)op.iw && op.h == (double)op.ih) {
        // not stretched: untransformed texture fill of the qRound'ed rect (aliased)
        const int x1 = qRound(op.x), y1 = qRound(op.y), x2 = qRound(op.x + op.w), y2 = qRound(op.y + op.h);
        const int cx1 = max(x1, 0), cy1 = max(y1, 0), cx2 = min(x2, HR_RES), cy2 = min(y2, HR_RES);
        const int cov = (255 * op.ca) >> 8;
        if (cov == 0 || cx1 >= cx2 || cy1 >= cy2) return;
        const int cw = cx2 - cx1, tot = cw * (cy2 - cy1);
        for (int p = tid; p < tot; p += HR_THREADS) {
            const int yy = cy1 + p / cw, xx = cx1 + p % cw;
            const int sy = yy - y1, sx = xx - x1;
            if (sy < 0 || sy >= op.ih || sx < 0 || sx >= op.iw) continue;
            hr_blend(frame + (size_t)yy * HR_RES + xx, op.px[(size_t)sy * op.iw + (op.mir ? op.iw - 1 - sx : sx)], cov,
                     op.rgb32 != 0);
        }
        return;
    }
    double x = op.x, y = op.y, w = op.w, h = op.h;
    if (op.kind == 1) {
        if (w < 0) { x += w; w = -w; }
        if (h < 0) { y += h; h = -h; }
        if (w <= 0 || h <= 0) return;
    }
    HRect R;
    hr_rect(x, y, w, h, R);
    if (R.n == 0 || R.r1 < R.r0) return;
    const int x0 = R.xs[0], x1 = R.xs[R.n - 1] + R.lens[R.n - 1];
    const int cw = x1 - x0, tot = cw * (R.r1 - R.r0 + 1);
    // drawImage: inverse of (translate(1/65536) * QTransform(sx, 0, 0, sy, x, y)) (QSpanData::setupMatrix)
    double m11 = 0, m22 = 0, mdx = 0, mdy = 0;
    int fdx = 0;
    const HTex T = {op.px, op.iw, op.ih, op.mir};
    if (op.kind == 0) {
        const double sxs = w / op.iw, sys = h / op.ih;
        const double tdx = (1.0 / 65536) * sxs + x, tdy = (1.0 / 65536) * sys + y;
        m11 = 1. / sxs; m22 = 1. / sys; mdx = -tdx * m11; mdy = -tdy * m22;
        fdx = (int)(m11 * 65536);
    }
    for (int p = tid; p < tot; p += HR_THREADS) {
        const int r = R.r0 + p / cw, xx = x0 + p % cw;
        int j = 0; // the span of this pixel
        while (j + 1 < R.n && xx >= R.xs[j] + R.lens[j]) j++;
        const int cov0 = hr_span_cov(R, r, j);
        if (cov0 == 0) continue;
        uint32_t *dp = frame + (size_t)r * HR_RES + xx;
        if (op.kind == 1) {
            const uint32_t c = cov0 == 255 ? op.argb : BYTE_MUL(op.argb, (uint32_t)cov0);
            *dp = cov0 == 255 ? c : c + BYTE_MUL(*dp, 255 - (uint32_t)cov0);
            continue;
        }
        // the fetch run of this pixel: this row's emitted spans, restarting at every 256-span flush
        const int base = hr_row_base(R, r);
        int e = 0, seg_s = -1, seg_e = -1;
        for (int i = 0; i < R.n; i++) {
            if (hr_span_cov(R, r, i) == 0) continue;
            const bool restart = seg_s < 0 || ((base + e) % 256) == 0;
            if (restart) {
                if (i > j) break;
                seg_s = R.xs[i];
            }
            seg_e = R.xs[i] + R.lens[i];
            e++;
            if (i >= j) {
                // extend over the following emitted spans of the same run
                int k = e;
                for (int i2 = i + 1; i2 < R.n; i2++) {
                    if (hr_span_cov(R, r, i2) == 0) continue;
                    if (((base + k) % 256) == 0) break;
                    seg_e = R.xs[i2] + R.lens[i2];
                    k++;
                }
                break;
            }
        }
        const int n = xx - seg_s, len = seg_e - seg_s;
        const double cy = r + 0.5;
        const int fx0 = (int)((0.0 * cy + m11 * (seg_s + 0.5) + mdx) * 65536) - 32768;
        const int fy = (int)((m22 * cy + 0.0 * (seg_s + 0.5) + mdy) * 65536) - 32768;
        const uint32_t src = hr_fetch_scale(T, fx0, fy, fdx, m22, len, n);
        hr_blend(dp, src, (cov0 * op.ca) >> 8, op.rgb32 != 0);
    }
}

// ---------------------------------------------------------------- rotated drawImage (render_mode="rgb_array")
// QPainter::translate(centre); rotate(deg); drawImage(QRectF(-w/2, -h/2, w, h)) (basic-abstract-game.cpp:
// 908-916) under Antialiasing + SmoothPixmapTransform: QRasterPaintEngine::drawImage's transformed
// branch, restated in the oracle (qt_smooth_draw_image_rot) from Qt 5.9.7's own machine code and
// pinned there against the real library (tests/test_smooth_pins.py):
//   * QTransform arithmetic per (fuzzy) type -- the mid line mapped, the texture matrix
//     translate(1/65536) * (m * translate(rx, ry) * scale(w / iw, h / ih)) inverted;
//   * QRasterizer::rasterizeLine antialiased: near-horizontal lines turned vertical (q26Dot6Compare),
//     the vertical branch's <= 3 spans per row, else the general branch -- the rectangle's corners
//     snapped to the 26.6 grid, four edge slopes, per row single-pixel spans at the edges
//     (intersectPixelFP) and one full-coverage run between them;
//   * the fetch of each run (spans merged while adjacent within a 256-span flush): the scale helpers
//     when fdy == 0, else the rotate helpers (8-bit beyond an 8x zoom; otherwise 8-bit lead-in,
//     4-bit groups of 4, 8-bit rest), or the floating-point path outside fast_matrix.
// On the device the rows are independent (every accumulator of the rasterizer's row loop is an exact
// integer recurrence, so row r's state is closed-form): threads generate the rows' spans into LDS in
// emission order (counts, a block scan, then the spans), then every pixel of every span is fetched and
// blended independently (a pixel's run and its place in the helpers' phases are closed-form too).
enum { HQ_NONE = 0, HQ_TRANSLATE = 1, HQ_SCALE = 2, HQ_ROTATE = 4, HQ_SHEAR = 8 };
struct HXf { double m11, m12, m21, m22, dx, dy; int type; };
DEV bool hq_fz(double d) { return fabs(d) <= 0.000000000001; } // qFuzzyIsNull
DEV int hq_classify(const HXf &t) {
    if (!hq_fz(t.m12) || !hq_fz(t.m21)) return hq_fz(t.m11 * t.m12 + t.m21 * t.m22) ? HQ_ROTATE : HQ_SHEAR;
    if (!hq_fz(t.m11 - 1) || !hq_fz(t.m22 - 1)) return HQ_SCALE;
    if (!hq_fz(t.dx) || !hq_fz(t.dy)) return HQ_TRANSLATE;
    return HQ_NONE;
}
DEV void hq_translate(HXf &t, double dx, double dy) {
    if (dx == 0 && dy == 0) return;
    if (t.type == HQ_NONE) { t.dx = dx; t.dy = dy; }
    else if (t.type == HQ_TRANSLATE) { t.dx += dx; t.dy += dy; }
    else if (t.type == HQ_SCALE) { t.dx += dx * t.m11; t.dy += dy * t.m22; }
    else { t.dx += dx * t.m11 + dy * t.m21; t.dy += dy * t.m22 + dx * t.m12; }
    t.type = hq_classify(t);
}
DEV void hq_scale(HXf &t, double sx, double sy) {
    if (sx == 1 && sy == 1) return;
    if (t.type == HQ_NONE || t.type == HQ_TRANSLATE) { t.m11 = sx; t.m22 = sy; }
    else {
        if (t.type != HQ_SCALE) { t.m12 *= sx; t.m21 *= sy; }
        t.m11 *= sx; t.m22 *= sy;
    }
    t.type = hq_classify(t);
}
DEV HXf hq_delta_times(const HXf &o) { // translate(1/65536, 1/65536) * o
    const double dd = 1.0 / 65536;
    HXf r = {1, 0, 0, 1, 0, 0, HQ_NONE};
    const int type = o.type > HQ_TRANSLATE ? o.type : HQ_TRANSLATE;
    if (type == HQ_TRANSLATE) { r.dx = dd + o.dx; r.dy = dd + o.dy; }
    else if (type == HQ_SCALE) { r.m11 = 1 * o.m11; r.m22 = 1 * o.m22; r.dx = dd * o.m11 + o.dx; r.dy = dd * o.m22 + o.dy; }
    else {
        r.m11 = 1 * o.m11 + 0 * o.m21; r.m12 = 1 * o.m12 + 0 * o.m22;
        r.m21 = 0 * o.m11 + 1 * o.m21; r.m22 = 0 * o.m12 + 1 * o.m22;
        r.dx = dd * o.m11 + dd * o.m21 + o.dx; r.dy = dd * o.m12 + dd * o.m22 + o.dy;
    }
    r.type = hq_classify(r);
    return r;
}
DEV HXf hq_inverted(const HXf &t) {
    HXf r = {1, 0, 0, 1, 0, 0, HQ_NONE};
    if (t.type == HQ_TRANSLATE) { r.dx = -t.dx; r.dy = -t.dy; }
    else if (t.type == HQ_SCALE) {
        r.m11 = 1. / t.m11; r.m22 = 1. / t.m22; r.dx = -t.dx * r.m11; r.dy = -t.dy * r.m22;
    } else if (t.type != HQ_NONE) { // QMatrix::inverted
        const double dtr = t.m11 * t.m22 - t.m12 * t.m21, dinv = 1.0 / dtr;
        r.m11 = t.m22 * dinv; r.m12 = -t.m12 * dinv; r.m21 = -t.m21 * dinv; r.m22 = t.m11 * dinv;
        r.dx = (t.m21 * t.dy - t.m22 * t.dx) * dinv; r.dy = (t.m12 * t.dx - t.m11 * t.dy) * dinv;
    }
    r.type = hq_classify(r);
    return r;
}
DEV void hq_map(const HXf &t, double x, double y, double &nx, double &ny) {
    if (t.type == HQ_NONE) { nx = x; ny = y; }
    else if (t.type == HQ_TRANSLATE) { nx = x + t.dx; ny = y + t.dy; }
    else if (t.type == HQ_SCALE) { nx = t.m11 * x + t.dx; ny = t.m22 * y + t.dy; }
    else { nx = t.m11 * x + t.m21 * y + t.dx; ny = t.m12 * x + t.m22 * y + t.dy; }
}
// QTransform().translate(tx, ty).rotate(deg) (qtransform.cpp rotate: exact 90 / 180 / 270 cases)
DEV HXf hq_translate_rotate(double tx, double ty, double a) {
    HXf t = {1, 0, 0, 1, tx, ty, HQ_NONE};
    if (a != 0) {
        double sina = 0, cosa = 0;
        if (a == 90. || a == -270.) sina = 1;
        else if (a == 270. || a == -90.) sina = -1;
        else if (a == 180.) cosa = -1;
        else pg_sincos_cr(0.017453292519943295769 * a, &sina, &cosa);
        t.m11 = cosa; t.m12 = sina; t.m21 = -sina; t.m22 = cosa;
    }
    t.type = hq_classify(t);
    return t;
}

// qrasterizer.cpp helpers (qSafeFloatToQ16Dot16, qSafeDivide, Q16Dot16Multiply, snapTo26Dot6Grid)
DEV int hq_fp(double x) {
    const double v = x * 65536.;
    if (v > 2147483647.0) return 0x7fffffff;
    if (v < -2147483648.0) return -2147483647;
    return (int)v;
}
DEV double hq_sdiv(double x, double y) { return y == 0 ? (x > 0 ? 1e20 : -1e20) : x / y; }
DEV int hq_mul(int x, int y) { return (int)(((int64_t)x * (int64_t)y) >> 16); }
DEV int hq_wadd(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }           // the loop's wrapping +=
DEV int hq_wmul(int r, int s) { return (int)((uint32_t)r * (uint32_t)s); }
DEV void hq_snap(double &x, double &y) {
    const double ny = floor(y * 64) * 0.015625, nx = floor(x * 64) * 0.015625;
    x = nx;
    y = ny;
}
DEV int hq_intersect(int x, int top, int bottom, int lix, int rix, int slope, int inv) { // intersectPixelFP
    const int leftX = x << 16, rightX = leftX + 65536;
    const int liy = top + hq_mul(slope > 0 ? leftX - lix : leftX - rix, inv);
    const int riy = liy + inv;
    if (lix >= leftX && rix <= rightX) return hq_mul(bottom - top, lix - leftX + ((rix - lix) >> 1));
    if (lix >= rightX) return bottom - top;
    if (lix >= leftX) return (bottom - top) - ((((rightX - lix) >> 1) * (slope > 0 ? riy - top : bottom - riy)) >> 16);
    if (rix <= leftX) return 0;
    if (rix <= rightX) return (((rix - leftX) >> 1) * (slope > 0 ? bottom - liy : liy - top)) >> 16;
    if (slope > 0) return (bottom - riy) + ((riy - liy) >> 1);
    return (riy - top) + ((liy - riy) >> 1);
}

// rasterizeLine(a, b, width) set up (uniform): kind 0 nothing, 1 vertical (HRect), 2 general
struct HLine {
    int kind;
    HRect V;
    int nrows, iTopFP, iLeftFP, iRightFP, iBottomFP, yLeftFP, yRightFP, yBottomFP, rowTop0;
    int leftAf0, rightAf0, leftBf0, rightBf0, leftBfL, rightBfR, tlAf0, trAf0;
    int tlS, trS, blS, brS, itlS, itrS, iblS, ibrS;
};
DEV void hr_line(double ax, double ay, double bx, double by, double width, HLine &L, bool squareCap = false) {
    L.kind = 0;
    L.V.n = 0;
    double pax = ax, pay = ay, pbx = bx, pby = by;
    if ((hq_fz(ax - bx) && hq_fz(ay - by)) || width == 0) return;
    if (squareCap) { // a wide pen's square caps: the line grows by half its (relative) width at both ends
        const double c = 0.5f * width, dx = pbx - pax, dy = pby - pay;
        pax -= dx * c;
        pay -= dy * c;
        pbx += dx * c;
        pby += dy * c;
    }
    {
        const double offx = fabs(by - ay) * width * 0.5, offy = fabs(bx - ax) * width * 0.5;
        const double cl = 0 - offx, ct = 0 - offy;
        const double cr = cl + ((HR_RES - 1 + 1 + offx) - cl), cb = ct + ((HR_RES - 1 + 1 + offy) - ct);
        const bool in_a = cl <= pax && pax <= cr && ct <= pay && pay <= cb;
        const bool in_b = cl <= pbx && pbx <= cr && ct <= pby && pby <= cb;
        if (!in_a || !in_b) {
            double t1 = 0, t2 = 1;
            const double o[2] = {pax, pay}, dd[2] = {pbx - pax, pby - pay};
            const double low[2] = {cl, ct}, high[2] = {cr, cb};
            for (int i = 0; i < 2; i++) {
                if (dd[i] == 0) {
                    if (o[i] <= low[i] || o[i] >= high[i]) return;
                    continue;
                }
                const double dinv = 1 / dd[i];
                double tl = (low[i] - o[i]) * dinv, th = (high[i] - o[i]) * dinv;
                if (tl > th) { const double t = tl; tl = th; th = t; }
                if (t1 < tl) t1 = tl;
                if (t2 > th) t2 = th;
                if (t1 >= t2) return;
            }
            const double nax = pax + (pbx - pax) * t1, nay = pay + (pby - pay) * t1;
            const double nbx = pax + (pbx - pax) * t2, nby = pay + (pby - pay) * t2;
            pax = nax; pay = nay; pbx = nbx; pby = nby;
        }
    }
    {
        const double d0x = ax - bx, d0y = ay - by, w0 = d0x * d0x + d0y * d0y;
        const double dx = pax - pbx, dy = pay - pby, ww = dx * dx + dy * dy;
        if (ww == 0) return;
        width *= sqrt(w0 / ww);
    }
    if ((int)((pby - pay) * 64.) == 0) { // horizontal -> vertical
        const double xm = (pax + pbx) * 0.5f, dx = fabs(pbx - pax) * 0.5f, yy = pay, dy = width * dx;
        pax = xm; pay = yy - dy;
        pbx = xm; pby = yy + dy;
        width = 1 / width;
    }
    if ((int)((pbx - pax) * 64.) == 0) { // vertical: <= 3 spans per row (hr_rect's tail)
        if (pay > pby) {
            double t = pay; pay = pby; pby = t;
            t = pax; pax = pbx; pbx = t;
        }
        HRect &R = L.V;
        const double dy = pby - pay, half = 0.5f * width * dy;
        double left = pax - half, right = pax + half;
        left = left < 0 ? 0 : (left > HR_RES ? HR_RES : left);
        right = right < 0 ? 0 : (right > HR_RES ? HR_RES : right);
        pay = pay < 0 ? 0 : (pay > HR_RES ? HR_RES : pay);
        pby = pby < 0 ? 0 : (pby > HR_RES ? HR_RES : pby);
        if ((int)(left * 64) == (int)(right * 64) || (int)(pay * 64) == (int)(pby * 64)) return;
        const int iL = (int)left, iR = (int)right;
        const int lw = ((iL + 1) << 16) - (int)(left * 65536.), rw = (int)(right * 65536.) - (iR << 16);
        int n = 1;
        if (iL == iR) {
            R.cov[0] = lw + rw; R.xs[0] = iL; R.lens[0] = 1;
        } else {
            R.cov[0] = lw; R.xs[0] = iL; R.lens[0] = 1;
            if (lw == 65536) R.lens[0] = iR - iL;
            else if (iR - iL > 1) { R.cov[1] = 65536; R.xs[1] = iL + 1; R.lens[1] = iR - iL - 1; n++; }
            if (rw) { R.cov[n] = rw; R.xs[n] = iR; R.lens[n] = 1; n++; }
        }
        R.n = n;
        R.r0 = (int)pay;
        R.r1 = min((int)pby, HR_RES - 1);
        R.yPa = (int)(pay * 65536.);
        R.yPb = (int)(pby * 65536.);
        L.kind = R.r1 >= R.r0 ? 1 : 0;
        L.nrows = R.r1 - R.r0 + 1;
        return;
    }
    // general branch
    if (pay > pby) {
        double t = pax; pax = pbx; pbx = t;
        t = pay; pay = pby; pby = t;
    }
    const double hw = 0.5f * width;
    const double dlx = (pbx - pax) * hw, dly = (pby - pay) * hw;
    const double prx = dly, pry = -dlx;
    double tx, ty, lx, ly, rx, ry, qx, qy; // top, left, right, bottom corners
    if (pax < pbx) {
        tx = pax + prx; ty = pay + pry; lx = pax - prx; ly = pay - pry;
        rx = pbx + prx; ry = pby + pry; qx = pbx - prx; qy = pby - pry;
    } else {
        tx = pax - prx; ty = pay - pry; lx = pbx - prx; ly = pby - pry;
        rx = pax + prx; ry = pay + pry; qx = pbx + prx; qy = pby + pry;
    }
    hq_snap(tx, ty);
    hq_snap(qx, qy);
    hq_snap(lx, ly);
    hq_snap(rx, ry);
    const double topBound = ty < 0 ? 0 : (ty > HR_RES - 1 ? HR_RES - 1 : ty);
    const double bottomBound = qy < 0 ? 0 : (qy > HR_RES - 1 ? HR_RES - 1 : qy);
    const double tlI = hq_sdiv(lx - tx, ly - ty), blI = hq_sdiv(qx - lx, qy - ly);
    const double trI = hq_sdiv(rx - tx, ry - ty), brI = hq_sdiv(qx - rx, qy - ry);
    L.tlS = hq_fp(tlI); L.trS = hq_fp(trI); L.blS = hq_fp(blI); L.brS = hq_fp(brI);
    L.itlS = hq_fp(hq_sdiv(1, tlI)); L.itrS = hq_fp(hq_sdiv(1, trI));
    L.iblS = hq_fp(hq_sdiv(1, blI)); L.ibrS = hq_fp(hq_sdiv(1, brI));
    const int iTop = (int)topBound;
    L.iTopFP = iTop << 16;
    L.iLeftFP = ((int)ly) << 16;
    L.iRightFP = ((int)ry) << 16;
    L.iBottomFP = ((int)bottomBound) << 16;
    L.leftAf0 = hq_fp(tx + (iTop - ty) * tlI);
    L.rightAf0 = hq_fp(tx + (iTop - ty) * trI);
    L.leftBf0 = L.iLeftFP < L.iTopFP ? hq_fp(lx + (iTop - ly) * blI) : 0;
    L.rightBf0 = L.iRightFP < L.iTopFP ? hq_fp(rx + (iTop - ry) * brI) : 0;
    L.leftBfL = hq_fp(lx + ((L.iLeftFP >> 16) - ly) * blI);
    L.rightBfR = hq_fp(rx + ((L.iRightFP >> 16) - ry) * brI);
    const int yTopFP = hq_fp(ty);
    L.yLeftFP = hq_fp(ly);
    L.yRightFP = hq_fp(ry);
    L.yBottomFP = hq_fp(qy);
    L.rowTop0 = L.iTopFP > yTopFP ? L.iTopFP : yTopFP;
    L.tlAf0 = L.leftAf0 + hq_mul(L.tlS, L.rowTop0 - L.iTopFP);
    L.trAf0 = L.rightAf0 + hq_mul(L.trS, L.rowTop0 - L.iTopFP);
    if (L.iBottomFP < L.iTopFP) return;
    L.nrows = ((L.iBottomFP - L.iTopFP) >> 16) + 1;
    L.kind = 2;
}

// the spans of row r (emission order) of a general line: fills up to `cap` (x, len, cov) and returns
// how many are emitted (nonzero coverage and length); with out == nullptr it only counts
struct HRow {
    int yFP, yi, rowTop, rowBottom, rowBottomLeft, rowBottomRight, rowTopLeft, rowTopRight;
    int tlAf, trAf, tlBf, blAf, trBf, brAf, blBf, brBf;
    int leftMin, leftMax, rightMin, rightMax;
};
DEV void hr_row_setup(const HLine &L, int r, HRow &w) {
    const int yFP = hq_wadd(L.iTopFP, r << 16);
    w.yFP = yFP;
    w.yi = yFP >> 16;
    const int leftAf = hq_wadd(L.leftAf0, hq_wmul(r, L.tlS)), rightAf = hq_wadd(L.rightAf0, hq_wmul(r, L.trS));
    const int rowL = (L.iLeftFP - L.iTopFP) >> 16, rowR = (L.iRightFP - L.iTopFP) >> 16;
    int leftBf, rightBf;
    if (L.iLeftFP < L.iTopFP || r < rowL) leftBf = hq_wadd(L.leftBf0, hq_wmul(r, L.blS));
    else leftBf = hq_wadd(L.leftBfL, hq_wmul(r - rowL, L.blS));
    if (L.iRightFP < L.iTopFP || r < rowR) rightBf = hq_wadd(L.rightBf0, hq_wmul(r, L.brS));
    else rightBf = hq_wadd(L.rightBfR, hq_wmul(r - rowR, L.brS));
    w.rowTop = r == 0 ? L.rowTop0 : yFP;
    w.tlAf = r == 0 ? L.tlAf0 : leftAf;
    w.trAf = r == 0 ? L.trAf0 : rightAf;
    w.rowBottomLeft = min(yFP + 65536, L.yLeftFP);
    w.rowBottomRight = min(yFP + 65536, L.yRightFP);
    w.rowTopLeft = max(yFP, L.yLeftFP);
    w.rowTopRight = max(yFP, L.yRightFP);
    w.rowBottom = min(yFP + 65536, L.yBottomFP);
    if (yFP == L.iLeftFP) {
        w.tlBf = leftBf + hq_mul(L.blS, w.rowTopLeft - yFP);
        w.blAf = leftAf + hq_mul(L.tlS, w.rowBottomLeft - yFP);
    } else {
        w.tlBf = leftBf;
        w.blAf = leftAf + L.tlS;
    }
    if (yFP == L.iRightFP) {
        w.trBf = rightBf + hq_mul(L.brS, w.rowTopRight - yFP);
        w.brAf = rightAf + hq_mul(L.trS, w.rowBottomRight - yFP);
    } else {
        w.trBf = rightBf;
        w.brAf = rightAf + L.trS;
    }
    if (yFP == L.iBottomFP) {
        w.blBf = leftBf + hq_mul(L.blS, w.rowBottom - yFP);
        w.brBf = rightBf + hq_mul(L.brS, w.rowBottom - yFP);
    } else {
        w.blBf = leftBf + L.blS;
        w.brBf = rightBf + L.brS;
    }
    if (yFP < L.iLeftFP) { w.leftMin = w.blAf >> 16; w.leftMax = w.tlAf >> 16; }
    else if (yFP == L.iLeftFP) { w.leftMin = max(w.blAf, w.tlBf) >> 16; w.leftMax = max(w.tlAf, w.blBf) >> 16; }
    else { w.leftMin = w.tlBf >> 16; w.leftMax = w.blBf >> 16; }
    w.leftMin = min(max(w.leftMin, 0), HR_RES - 1);
    w.leftMax = min(max(w.leftMax, 0), HR_RES - 1);
    if (yFP < L.iRightFP) { w.rightMin = w.trAf >> 16; w.rightMax = w.brAf >> 16; }
    else if (yFP == L.iRightFP) { w.rightMin = min(w.trAf, w.brBf) >> 16; w.rightMax = min(w.brAf, w.trBf) >> 16; }
    else { w.rightMin = w.brBf >> 16; w.rightMax = w.trBf >> 16; }
    w.rightMin = min(max(w.rightMin, 0), HR_RES - 1);
    w.rightMax = min(max(w.rightMax, 0), HR_RES - 1);
    if (w.leftMax > w.rightMax) w.leftMax = w.rightMax;
    if (w.rightMin < w.leftMin) w.rightMin = w.leftMin;
}
DEV int hr_row_cov(const HLine &L, const HRow &w, int x, bool left_part) {
    int ex = 0;
    if (left_part) {
        if (w.yFP <= L.iLeftFP) ex += hq_intersect(x, w.rowTop, w.rowBottomLeft, w.blAf, w.tlAf, L.tlS, L.itlS);
        if (w.yFP >= L.iLeftFP) ex += hq_intersect(x, w.rowTopLeft, w.rowBottom, w.tlBf, w.blBf, L.blS, L.iblS);
    }
    if (!left_part || x >= w.rightMin) {
        if (w.yFP <= L.iRightFP)
            ex += (w.rowBottomRight - w.rowTop) - hq_intersect(x, w.rowTop, w.rowBottomRight, w.trAf, w.brAf, L.trS, L.itrS);
        if (w.yFP >= L.iRightFP)
            ex += (w.rowBottom - w.rowTopRight) - hq_intersect(x, w.rowTopRight, w.rowBottom, w.brBf, w.trBf, L.brS, L.ibrS);
    }
    return ((255 * (w.rowBottom - w.rowTop - ex)) >> 16) & 0xff;
}
// emits row r's spans (emission order) through emit(x, len, y, cov); returns the count
template <class F>
DEV int hr_row_spans(const HLine &L, int r, F emit) {
    int k = 0;
    if (L.kind == 1) {
        const HRect &R = L.V;
        const int rr = R.r0 + r;
        for (int i = 0; i < R.n; i++) {
            const int c = hr_span_cov(R, rr, i);
            if (c && R.lens[i]) { emit(R.xs[i], R.lens[i], rr, c); k++; }
        }
        return k;
    }
    HRow w;
    hr_row_setup(L, r, w);
    int x = w.leftMin;
    for (; x <= w.leftMax; x++) {
        const int c = hr_row_cov(L, w, x, true);
        if (c) { emit(x, 1, w.yi, c); k++; }
    }
    if (x < w.rightMin) {
        const int c = ((255 * (w.rowBottom - w.rowTop)) >> 16) & 0xff;
        if (c) { emit(x, w.rightMin - x, w.yi, c); k++; }
        x = w.rightMin;
    }
    for (; x <= w.rightMax; x++) {
        const int c = hr_row_cov(L, w, x, false);
        if (c) { emit(x, 1, w.yi, c); k++; }
    }
    return k;
}

#define HR_SPAN_CAP 4096
struct HSpanLds { // one chunk of rows' spans (runs never cross rows, so chunks end on row boundaries)
    int16_t x[HR_SPAN_CAP], y[HR_SPAN_CAP], len[HR_SPAN_CAP];
    uint8_t cov[HR_SPAN_CAP];
    int pre[HR_SPAN_CAP + 1]; // pixel prefix over the chunk's spans
};
// exclusive block scan of v over the 256 threads (returns the prefix, *sum = the total)
DEV int hr_scan(int v, int *tmp, int &sum) {
    const int tid = threadIdx.x;
    tmp[tid] = v;
    __syncthreads();
    for (int off = 1; off < HR_THREADS; off <<= 1) {
        const int a = tid >= off ? tmp[tid - off] : 0;
        __syncthreads();
        tmp[tid] += a;
        __syncthreads();
    }
    sum = tmp[HR_THREADS - 1];
    const int ex = tmp[tid] - v;
    __syncthreads();
    return ex;
}

// the rotate helpers (fdy != 0): pixel n of a run of `len`
DEV uint32_t hr_fetch_rot(const HTex &T, int fx0, int fy0, int fdx, int fdy, bool fast, int len, int n) {
    const int fx = fx0 + n * fdx, fy = fy0 + n * fdy;
    bool four = false;
    if (fast && T.iw >= 2 && T.ih >= 2) {
        int64_t xlo, xhi, ylo, yhi;
        hr_nrange(fx0, fdx, (int64_t)(T.iw - 1) * 65536 - 1, len, xlo, xhi);
        hr_nrange(fy0, fdy, (int64_t)(T.ih - 1) * 65536 - 1, len, ylo, yhi);
        const int64_t a = max(xlo, ylo), b = min(xhi, yhi);
        if (a <= b) { // the lead-in ends at n = a; the unclamped middle is bounded by the end
            const int64_t fxa = fx0 + a * fdx, fya = fy0 + a * fdy;
            int64_t bend = len;
            if (fdx > 0) bend = min(bend, a + ((int64_t)(T.iw - 1) * 65536 - fxa) / fdx);
            else if (fdx < 0) bend = min(bend, a + (0 - fxa) / fdx);
            if (fdy > 0) bend = min(bend, a + ((int64_t)(T.ih - 1) * 65536 - fya) / fdy);
            else if (fdy < 0) bend = min(bend, a + (0 - fya) / fdy);
            const int64_t groups = bend - a >= 4 ? (bend - a) / 4 : 0;
            four = n >= a && n < a + 4 * groups;
        }
    }
    if (four) {
        const int c = fx >> 16, r = fy >> 16;
        const uint32_t dx4 = (((uint32_t)(fx & 0xffff) >> 8) + 8) >> 4, dy4 = (((uint32_t)(fy & 0xffff) >> 8) + 8) >> 4;
        return hr_interp4_4(hr_tex(T, r, c), hr_tex(T, r, c + 1), hr_tex(T, r + 1, c), hr_tex(T, r + 1, c + 1), dx4, dy4);
    }
    int x1 = fx >> 16, x2, y1 = fy >> 16, y2;
    if (x1 < 0) x1 = x2 = 0;
    else if (x1 >= T.iw - 1) x1 = x2 = T.iw - 1;
    else x2 = x1 + 1;
    if (y1 < 0) y1 = y2 = 0;
    else if (y1 >= T.ih - 1) y1 = y2 = T.ih - 1;
    else y2 = y1 + 1;
    return hr_interp4_8(hr_tex(T, y1, x1), hr_tex(T, y1, x2), hr_tex(T, y2, x1), hr_tex(T, y2, x2),
                        (uint32_t)(fx & 0xffff) >> 8, (uint32_t)(fy & 0xffff) >> 8);
}
// the floating-point path (outside fast_matrix): the reference steps fx, fy by repeated addition
DEV uint32_t hr_fetch_float(const HTex &T, const HXf &m, int x0, int y, int n) {
    const double cx = x0 + 0.5, cy = y + 0.5;
    double fx = m.m21 * cy + m.m11 * cx + m.dx, fy = m.m22 * cy + m.m12 * cx + m.dy;
    for (int k = 0; k < n; k++) { fx += m.m11; fy += m.m12; }
    const double pxv = fx * 1.0 - 0.5, pyv = fy * 1.0 - 0.5;
    int x1 = (int)pxv - (pxv < 0), x2, y1 = (int)pyv - (pyv < 0), y2;
    const int distx = (int)((pxv - x1) * 256), disty = (int)((pyv - y1) * 256);
    if (x1 < 0) x1 = x2 = 0;
    else if (x1 >= T.iw - 1) x1 = x2 = T.iw - 1;
    else x2 = x1 + 1;
    if (y1 < 0) y1 = y2 = 0;
    else if (y1 >= T.ih - 1) y1 = y2 = T.ih - 1;
    else y2 = y1 + 1;
    return hr_interp4_8(hr_tex(T, y1, x1), hr_tex(T, y1, x2), hr_tex(T, y2, x1), hr_tex(T, y2, x2), (uint32_t)distx,
                        (uint32_t)disty);
}

// translate(x + w/2, y + h/2); rotate(deg); drawImage(QRectF(-w/2, -h/2, w, h), img) on the frame
// (tmp: HR_THREADS + 1 ints of LDS)
DEV void hr_draw_rotated(uint32_t *frame, HSpanLds &S, int *tmp, double x, double y, double w, double h, double deg,
                         const HTex &T, bool rgb32, int ca) {
    if (T.iw <= 0 || T.ih <= 0 || !(w > 0) || !(h > 0)) return;
    const int tid = threadIdx.x;
    const double rx = -w / 2, ry = -h / 2;
    const HXf m = hq_translate_rotate(x + w / 2, y + h / 2, deg);
    double ax, ay, bx, by;
    hq_map(m, (rx + rx) * 0.5f, (ry + (ry + h)) * 0.5f, ax, ay);
    hq_map(m, ((rx + w) + (rx + w)) * 0.5f, (ry + (ry + h)) * 0.5f, bx, by);
    HXf copy = m;
    hq_translate(copy, rx, ry);
    hq_scale(copy, w / T.iw, h / T.ih);
    const HXf inv = hq_inverted(hq_delta_times(copy));
    const bool fastm = inv.m11 * inv.m11 + inv.m21 * inv.m21 < 1e4 && inv.m12 * inv.m12 + inv.m22 * inv.m22 < 1e4 &&
                       fabs(inv.dx) < 1e4 && fabs(inv.dy) < 1e4;
    HLine L;
    hr_line(ax, ay, bx, by, h / w, L);
    if (L.kind == 0) return;
    const int fdx = (int)(inv.m11 * 65536), fdy = (int)(inv.m12 * 65536);
    const bool fastrot = !(fabs(inv.m11) < 1. / 8. || fabs(inv.m22) < 1. / 8.);
    // rows in chunks: as many of the next 256 rows as fit the LDS span list (at least one: a row has at
    // most HR_RES spans); `base` = the global index of the chunk's first span (the 256-span flushes)
    int base = 0;
    for (int rs = 0; rs < L.nrows;) {
        const int r = rs + tid;
        const int c = r < L.nrows ? hr_row_spans(L, r, [](int, int, int, int) {}) : 0;
        int sum;
        const int ex = hr_scan(c, tmp, sum);
        const bool fits = r < L.nrows && ex + c <= HR_SPAN_CAP;
        const int nfit = __syncthreads_count(fits);
        if (tid < nfit) {
            int k = ex;
            hr_row_spans(L, r, [&](int sx, int sl, int sy, int sc) {
                S.x[k] = (int16_t)sx; S.len[k] = (int16_t)sl; S.y[k] = (int16_t)sy; S.cov[k] = (uint8_t)sc;
                k++;
            });
            if (tid == nfit - 1) tmp[HR_THREADS] = ex + c;
        }
        __syncthreads();
        const int nsp = tmp[HR_THREADS];
        // pixel prefix over the chunk's spans
        {
            const int per = (nsp + HR_THREADS - 1) / HR_THREADS, lo = min(nsp, tid * per), hi = min(nsp, lo + per);
            int loc = 0;
            for (int k = lo; k < hi; k++) loc += S.len[k];
            int tot;
            int run = hr_scan(loc, tmp, tot);
            for (int k = lo; k < hi; k++) { S.pre[k] = run; run += S.len[k]; }
            if (tid == 0) S.pre[nsp] = tot;
            __syncthreads();
        }
        const int P = S.pre[nsp];
        // every pixel: its run (adjacent spans of one row within one 256-span flush), fetch, blend
        for (int p = tid; p < P; p += HR_THREADS) {
            int lo = 0, hi = nsp - 1; // the last span with pre <= p
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (S.pre[mid] <= p) lo = mid;
                else hi = mid - 1;
            }
            const int k = lo, yy = S.y[k], xx = S.x[k] + (p - S.pre[k]);
            int k0 = k, k1 = k;
            while (k0 > 0 && ((base + k0) % 256) != 0 && S.y[k0 - 1] == yy && S.x[k0 - 1] + S.len[k0 - 1] == S.x[k0]) k0--;
            while (k1 + 1 < nsp && ((base + k1 + 1) % 256) != 0 && S.y[k1 + 1] == yy && S.x[k1] + S.len[k1] == S.x[k1 + 1])
                k1++;
            const int x0 = S.x[k0], len = S.x[k1] + S.len[k1] - x0, n = xx - x0;
            uint32_t src;
            if (!fastm) {
                src = hr_fetch_float(T, inv, x0, yy, n);
            } else {
                const double cx = x0 + 0.5, cy = yy + 0.5;
                const int fx0 = (int)((inv.m21 * cy + inv.m11 * cx + inv.dx) * 65536) - 32768;
                const int fy0 = (int)((inv.m22 * cy + inv.m12 * cx + inv.dy) * 65536) - 32768;
                if (fdy == 0) src = hr_fetch_scale(T, fx0, fy0, fdx, inv.m22, len, n);
                else src = hr_fetch_rot(T, fx0, fy0, fdx, fdy, fastrot, len, n);
            }
            hr_blend(frame + (size_t)yy * HR_RES + xx, src, ((int)S.cov[k] * ca) >> 8, rgb32);
        }
        __syncthreads();
        base += nsp;
        rs += nfit;
    }
}

DEV void hr_run(uint32_t *frame, const HOp &op) {
    hr_paint(frame, op);
    __syncthreads();
}

// LDS of the rotated path (only the games with rotating entities reserve it)
struct HRotLds {
    HSpanLds S;
    int tmp[HR_THREADS + 1];
};

// tile_image (basic-abstract-game.cpp:849-877): num_tiles side by side (ratio > 0) or stacked (< 0)
DEV void hr_tiles(uint32_t *frame, HOp op, float tile_ratio) {
    const double x = op.x, y = op.y, w = op.w, h = op.h;
    if (tile_ratio == 0) {
        hr_run(frame, op);
        return;
    }
    const bool stacked = tile_ratio < 0;
    int num_tiles;
    float tw, th;
    if (stacked) {
        tile_ratio = -1 * tile_ratio;
        num_tiles = (int)(h / (w * tile_ratio));
        if (num_tiles < 1) num_tiles = 1;
        th = (float)(h / num_tiles);
        tw = (float)w;
    } else {
        num_tiles = (int)(w / (h * tile_ratio));
        if (num_tiles < 1) num_tiles = 1;
        tw = (float)(w / num_tiles);
        th = (float)h;
    }
    op.w = tw;
    op.h = th;
    for (int i = 0; i < num_tiles; i++) {
        op.x = stacked ? x : x + tw * i;
        op.y = stacked ? y + th * i : y;
        // a tile a pixel clear of the frame rasterises to nothing (the clip in rasterizeLine)
        if (op.x + op.w < -1 || op.x > HR_RES + 1 || op.y + op.h < -1 || op.y > HR_RES + 1) continue;
        hr_run(frame, op);
    }
}

// draw_image (basic-abstract-game.cpp:886-922) at RENDER_RES: tiles, rotation (:908-916)
template <int G>
DEV bool hr_draw_image(uint32_t *frame, const PGDev &d, const PGEnv &s, double bx, double by, double bw, double bh,
                       bool refl, int base_type, int theme, float alpha, int player_img, float rotation, float tile_ratio,
                       HRotLds *L) {
    const int img = image_for_type<G>(s, base_type, player_img);
    if (img < 0) return true;
    HOp op;
    op.kind = 1; op.px = nullptr; op.iw = op.ih = 0; op.rgb32 = 0; op.mir = 0; op.ca = 256; op.argb = 0;
    if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) { // draw_grid_obj (:924-928)
        if (img == SPACE) return true;
        if (G == PG_GAME_CHASER && img == CH_ORB) { // chaser.cpp:111-117
            const float dim = 0.3f, k = 1 - dim;
            op.x = bx + bw * k / 2; op.y = by + bh * k / 2; op.w = bw * dim; op.h = bh * dim; op.argb = 0xff00ff00u;
            hr_run(frame, op);
            return true;
        }
        const uint32_t col = color_for_type<G>(s, img, theme);
        if (col == 0) return false;
        op.x = bx; op.y = by; op.w = bw; op.h = bh; op.argb = col;
        hr_run(frame, op);
        return true;
    }
    theme = mask_theme<G>(s, theme, img);
    if (theme < 0 || theme >= 10) return false;
    if constexpr (G == PG_GAME_COINRUN) {
        if (is_player_image(img)) { // coinrun.cpp:64-70
            by = by + bh * -.7415;
            bh = bh * 1.7415;
            bx = bx + bw * 0.0;
            bw = bw * 1.0;
        }
    }
    if constexpr (G == PG_GAME_LEAPER) {
        if (img == PLAYER) { // leaper.cpp:244-250
            bx = bx + bw * 0.0;
            by = by + bh * -.275;
            bw = bw * 1.0;
            bh = bh * 1.55;
        }
    }
    const int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
    if (sp.y <= 0) return missing_image_ok<G>(img);
    if (!(bw > 0) || !(bh > 0)) return true; // QRectF::isEmpty
    if ((size_t)sp.x + (size_t)sp.y * sp.z > d.num_pixels) return false;
    op.kind = 0; op.x = bx; op.y = by; op.w = bw; op.h = bh;
    op.px = d.pixels + sp.x; op.iw = sp.y; op.ih = sp.z; op.mir = refl ? 1 : 0;
    op.ca = alpha != 1 ? qt_int_opacity((double)alpha) : 256;
    if (rotation != 0) {
        if constexpr (has_rotation<G>()) {
            const HTex T = {op.px, op.iw, op.ih, op.mir};
            hr_draw_rotated(frame, L->S, L->tmp, bx, by, bw, bh, (double)(rotation * 180 / PI_F), T, false, op.ca);
            return true;
        }
        return false;
    }
    hr_tiles(frame, op, tile_ratio);
    return true;
}

template <int G>
DEV bool hr_entities(uint32_t *frame, const PGDev &d, const PGEnv &s, const View &v, int env, int z, int player_img,
                     HRotLds *L) {
    bool ok = true;
    for (int i = 0; i < s.num_ents; i++) {
        if (EIr(d, F_RENDER_Z, env, i) != z) continue;
        const int etype = EIr(d, F_TYPE, env, i);
        const int itype = EIr(d, F_IMAGE_TYPE, env, i), theme = EIr(d, F_IMAGE_THEME, env, i);
        if (!should_draw<G>(s, etype, theme)) continue;
        const float px_ = EFr(d, F_X, env, i), py_ = EFr(d, F_Y, env, i);
        const float prx = EFr(d, F_RX, env, i), pry = EFr(d, F_RY, env, i);
        const int flags = EIr(d, F_FLAGS, env, i);
        double rx, ry, rw, rh;
        if (flags & EF_ABS_COORDS) { // get_abs_rect (:812-814)
            const float vd = v.view_dim;
            const float ax = vd * (px_ - prx), ay = vd * (py_ + pry), aw = 2 * vd * prx, ah = 2 * vd * pry;
            rx = (double)(ax * v.unit); ry = (double)(ay * v.unit); rw = (double)(aw * v.unit); rh = (double)(ah * v.unit);
        } else {
            screen_rect(v, px_ - prx, py_ + pry, 2 * prx, 2 * pry, 0, rx, ry, rw, rh);
        }
        ok = hr_draw_image<G>(frame, d, s, rx, ry, rw, rh, (flags & EF_REFLECTED) != 0, itype, theme,
                              EFr(d, F_ALPHA, env, i), player_img, EFr(d, F_ROTATION, env, i),
                              tile_aspect_ratio<G>(etype, prx, pry), L) && ok;
    }
    return ok;
}

// ---- jumper's compass at RENDER_RES (jumper.cpp:137-177 under Antialiasing; the oracle's
// jp_draw_compass_smooth, pinned primitive by primitive against Qt 5.9.7 in tests/test_smooth_pins.py):
//   drawEllipse(QRectF) with a brush and a 1-px pen -> the flattened 26.6 outline filled by the gray raster
//       (qgrayraster.c cells accumulated by one lane into LDS, then swept one row per thread), then the
//       antialiased QCosmeticStroker (one lane, on the dial's pixels staged in LDS);
//   drawLine(QLine) with a wide pen -> rasterizeLine with square caps (rows across threads);
//   fillRect(QRectF) -> hr_paint; drawEllipse(QRect) with a translucent brush -> the gray raster.
#define HC_CX 136 // gray-raster cells per row, column 0 = the cells left of the clip
#define HC_CY 134
struct HCompassLds {
    AgLds ag;
    int n_poly;
    int area[HC_CX * HC_CY]; // also the stroke's staged pixels
    int16_t cover[HC_CX * HC_CY];
};
struct HcPainter { AgLds *ls; int err; }; // what ag_flatten needs of a painter

// solid colour at coverage `cov` (blend_color_argb / comp_func_solid_SourceOver with const_alpha = cov)
DEV void hc_blend_solid(uint32_t *d, uint32_t pm, int cov) {
    if (cov <= 0) return;
    const uint32_t c = cov == 255 ? pm : BYTE_MUL(pm, (uint32_t)cov);
    const uint32_t a = c >> 24;
    *d = a == 255 ? c : c + BYTE_MUL(*d, 255u - a);
}

// qgrayraster.c with PIXEL_BITS 8: cells (area, cover) in 24.8 inside the clip box (cells left of it in
// column -1, right of it dropped)
#define HC_PB 8
#define HC_ONE (1 << HC_PB)
struct HcRas {
    int min_ex, max_ex, min_ey, max_ey, count_ex, count_ey;
    int ex, ey, invalid, area, cover, x, y, last_ey;
    int *ca;
    int16_t *cc;
};
DEV void hc_record(HcRas &r) {
    if (!r.invalid && (r.area | r.cover)) {
        const int k = r.ey * (r.count_ex + 1) + (r.ex + 1);
        r.ca[k] += r.area;
        r.cc[k] = (int16_t)(r.cc[k] + r.cover);
    }
}
DEV void hc_set_cell(HcRas &r, int ex, int ey) {
    ey -= r.min_ey;
    if (ex > r.max_ex) ex = r.max_ex;
    ex -= r.min_ex;
    if (ex < 0) ex = -1;
    if (ex != r.ex || ey != r.ey) {
        hc_record(r);
        r.area = 0;
        r.cover = 0;
    }
    r.ex = ex;
    r.ey = ey;
    r.invalid = ((unsigned)ey >= (unsigned)r.count_ey || ex >= r.count_ex);
}
DEV void hc_start_cell(HcRas &r, int ex, int ey) {
    if (ex > r.max_ex) ex = r.max_ex;
    if (ex < r.min_ex) ex = r.min_ex - 1;
    r.area = 0;
    r.cover = 0;
    r.ex = ex - r.min_ex;
    r.ey = ey - r.min_ey;
    r.last_ey = ey << HC_PB;
    r.invalid = 0;
    hc_set_cell(r, ex, ey);
}
DEV int hc_trunc(int64_t x) { return (int)(x >> HC_PB); }
DEV void hc_scanline(HcRas &r, int ey, int64_t x1, int y1, int64_t x2, int y2) {
    int64_t dx = x2 - x1;
    int ex1 = hc_trunc(x1), ex2 = hc_trunc(x2);
    const int fx1 = (int)(x1 - ((int64_t)ex1 << HC_PB)), fx2 = (int)(x2 - ((int64_t)ex2 << HC_PB));
    if (y1 == y2) {
        hc_set_cell(r, ex2, ey);
        return;
    }
    if (ex1 == ex2) {
        const int delta = y2 - y1;
        r.area += (fx1 + fx2) * delta;
        r.cover += delta;
        return;
    }
    int64_t p = (int64_t)(HC_ONE - fx1) * (y2 - y1);
    int first = HC_ONE, incr = 1;
    if (dx < 0) {
        p = (int64_t)fx1 * (y2 - y1);
        first = 0;
        incr = -1;
        dx = -dx;
    }
    int delta = (int)(p / dx), mod = (int)(p % dx);
    if (mod < 0) {
        delta--;
        mod += (int)dx;
    }
    r.area += (fx1 + first) * delta;
    r.cover += delta;
    ex1 += incr;
    hc_set_cell(r, ex1, ey);
    y1 += delta;
    if (ex1 != ex2) {
        p = (int64_t)HC_ONE * (y2 - y1 + delta);
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
            r.area += HC_ONE * delta;
            r.cover += delta;
            y1 += delta;
            ex1 += incr;
            hc_set_cell(r, ex1, ey);
        }
    }
    delta = y2 - y1;
    r.area += (fx2 + HC_ONE - first) * delta;
    r.cover += delta;
}
DEV void hc_line_to(HcRas &r, int64_t to_x, int64_t to_y) {
    int ey1 = hc_trunc(r.last_ey), ey2 = hc_trunc(to_y);
    const int fy1 = (int)(r.y - r.last_ey), fy2 = (int)(to_y - ((int64_t)ey2 << HC_PB));
    int64_t dx = to_x - r.x, dy = to_y - r.y;
    const int mn = min(ey1, ey2), mx = max(ey1, ey2);
    if (mn >= r.max_ey || mx < r.min_ey) {
        // outside the clip rows: the pen moves, no cell
    } else if (ey1 == ey2) {
        hc_scanline(r, ey1, r.x, fy1, to_x, fy2);
    } else if (dx == 0) {
        int incr = 1;
        const int ex = hc_trunc(r.x);
        const int two_fx = (int)(((int64_t)r.x - ((int64_t)ex << HC_PB)) << 1);
        int first = HC_ONE;
        if (dy < 0) {
            first = 0;
            incr = -1;
        }
        int delta = first - fy1;
        r.area += two_fx * delta;
        r.cover += delta;
        ey1 += incr;
        hc_set_cell(r, ex, ey1);
        delta = first + first - HC_ONE;
        const int area = two_fx * delta;
        while (ey1 != ey2) {
            r.area += area;
            r.cover += delta;
            ey1 += incr;
            hc_set_cell(r, ex, ey1);
        }
        delta = fy2 - HC_ONE + first;
        r.area += two_fx * delta;
        r.cover += delta;
    } else {
        int incr = 1;
        int64_t p = (int64_t)(HC_ONE - fy1) * dx;
        int first = HC_ONE;
        if (dy < 0) {
            p = (int64_t)fy1 * dx;
            first = 0;
            incr = -1;
            dy = -dy;
        }
        int delta = (int)(p / dy), mod = (int)(p % dy);
        if (mod < 0) {
            delta--;
            mod += (int)dy;
        }
        int64_t x = r.x + delta;
        hc_scanline(r, ey1, r.x, fy1, x, first);
        ey1 += incr;
        hc_set_cell(r, hc_trunc(x), ey1);
        if (ey1 != ey2) {
            p = (int64_t)HC_ONE * dx;
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
                const int64_t x2 = x + delta;
                hc_scanline(r, ey1, x, HC_ONE - first, x2, first);
                x = x2;
                ey1 += incr;
                hc_set_cell(r, hc_trunc(x), ey1);
            }
        }
        hc_scanline(r, ey1, x, HC_ONE - first, to_x, fy2);
    }
    r.x = (int)to_x;
    r.y = (int)to_y;
    r.last_ey = ey2 << HC_PB;
}
DEV int hc_coverage(int area) { // gray_hline, odd-even
    int c = area >> (HC_PB * 2 + 1 - 8);
    if (c < 0) c = -c;
    c &= 511;
    if (c > 256) c = 512 - c;
    else if (c == 256) c = 255;
    return c;
}
// fill the closed 26.6 contour C.ag.poly[0, n) odd-even in `pm` (every thread calls it);
// false = the cell box does not fit the LDS
DEV bool hc_gray_fill(HCompassLds &C, int n, uint32_t pm, uint32_t *frame) {
    const int tid = threadIdx.x;
    if (n <= 0) return true;
    int xmn = C.ag.poly[0].x, xmx = xmn, ymn = C.ag.poly[0].y, ymx = ymn;
    for (int i = 1; i < n; i++) {
        const int2 q = C.ag.poly[i];
        xmn = min(xmn, q.x); xmx = max(xmx, q.x);
        ymn = min(ymn, q.y); ymx = max(ymx, q.y);
    }
    HcRas r;
    r.min_ex = xmn >> 6; r.min_ey = ymn >> 6; r.max_ex = (xmx + 63) >> 6; r.max_ey = (ymx + 63) >> 6;
    if (r.max_ex <= 0 || r.min_ex >= HR_RES || r.max_ey <= 0 || r.min_ey >= HR_RES) return true;
    r.min_ex = max(r.min_ex, 0); r.min_ey = max(r.min_ey, 0);
    r.max_ex = min(r.max_ex, HR_RES); r.max_ey = min(r.max_ey, HR_RES);
    r.count_ex = r.max_ex - r.min_ex;
    r.count_ey = r.max_ey - r.min_ey;
    if (r.count_ex + 1 > HC_CX || r.count_ey > HC_CY) return false;
    const int stride = r.count_ex + 1, ncell = r.count_ey * stride;
    for (int k = tid; k < ncell; k += HR_THREADS) {
        C.area[k] = 0;
        C.cover[k] = 0;
    }
    __syncthreads();
    if (tid == 0) { // gray_move_to(first), gray_line_to each point and back to the first (the close)
        r.ca = C.area;
        r.cc = C.cover;
        r.invalid = 1;
        r.ex = r.ey = 0;
        r.area = r.cover = 0;
        const int64_t x0 = (int64_t)C.ag.poly[0].x << (HC_PB - 6), y0 = (int64_t)C.ag.poly[0].y << (HC_PB - 6);
        hc_start_cell(r, hc_trunc(x0), hc_trunc(y0));
        r.x = (int)x0;
        r.y = (int)y0;
        for (int i = 1; i <= n; i++) {
            const int2 q = C.ag.poly[i < n ? i : 0];
            hc_line_to(r, (int64_t)q.x << (HC_PB - 6), (int64_t)q.y << (HC_PB - 6));
        }
        hc_record(r);
    }
    __syncthreads();
    if (tid < r.count_ey) { // gray_sweep, one row per thread
        uint32_t *row = frame + (size_t)(tid + r.min_ey) * HR_RES + r.min_ex;
        const int *ca = C.area + tid * stride;
        const int16_t *cc = C.cover + tid * stride;
        int cover = 0, x = 0;
        for (int cx = -1; cx < r.count_ex; cx++) {
            if (ca[cx + 1] == 0 && cc[cx + 1] == 0) continue;
            if (cx > x && cover != 0) {
                const int c = hc_coverage(cover * (HC_ONE * 2));
                for (int k = x; k < cx; k++) hc_blend_solid(&row[k], pm, c);
            }
            cover += cc[cx + 1];
            const int area = cover * (HC_ONE * 2) - ca[cx + 1];
            if (area != 0 && cx >= 0) hc_blend_solid(&row[cx], pm, hc_coverage(area));
            x = cx + 1;
        }
        if (r.count_ex > x && cover != 0) {
            const int c = hc_coverage(cover * (HC_ONE * 2));
            for (int k = x; k < r.count_ex; k++) hc_blend_solid(&row[k], pm, c);
        }
    }
    __syncthreads();
    return true;
}
// QRasterPaintEngine::fill's early out: the control points' rect, toRect(), must meet the device
DEV bool hc_path_on_device(const AgPtD *p, int n) {
    double x0 = p[0].x, x1 = p[0].x, y0 = p[0].y, y1 = p[0].y;
    for (int i = 1; i < n; i++) {
        x0 = fmin(x0, p[i].x); x1 = fmax(x1, p[i].x);
        y0 = fmin(y0, p[i].y); y1 = fmax(y1, p[i].y);
    }
    const int rx = qRound(x0), ry = qRound(y0), rw = qRound(x1 - x0), rh = qRound(y1 - y0);
    if (rw == 0 && rh == 0) return false; // QRect::isNull
    const int ax2 = rx + rw - 1, ay2 = ry + rh - 1;
    int l1 = rx, r1 = rx, t1 = ry, b1 = ry;
    if (ax2 - rx + 1 < 0) l1 = ax2; else r1 = ax2;
    if (ay2 - ry + 1 < 0) t1 = ay2; else b1 = ay2;
    return !(l1 > HR_RES - 1 || 0 > r1 || t1 > HR_RES - 1 || 0 > b1);
}
// the ellipse path filled by the gray raster: QOutlineMapper flattens the four curves (0.25) and
// rounds to 26.6 (wave 0 flattens: the Bezier stack is shared LDS)
DEV bool hc_fill_ellipse(HCompassLds &C, const AgPtD pts[13], uint32_t pm, uint32_t *frame) {
    if (threadIdx.x < 64) {
        HcPainter p = {&C.ag, 0};
        C.ag.poly[0] = make_int2(ag_fixed(pts[0].x), ag_fixed(pts[0].y));
        int n = 1;
        AgPtD last = pts[0];
        for (int k = 0; k < 4; k++) {
            const AgBez b = {last.x, last.y, pts[3 * k + 1].x, pts[3 * k + 1].y, pts[3 * k + 2].x, pts[3 * k + 2].y,
                             pts[3 * k + 3].x, pts[3 * k + 3].y};
            n = ag_flatten(p, b, n);
            last = pts[3 * k + 3];
        }
        if (threadIdx.x == 0) C.n_poly = p.err ? -1 : n;
    }
    __syncthreads();
    const int n = C.n_poly;
    if (n < 0) return false;
    return hc_gray_fill(C, n, pm, frame);
}

// QCosmeticStroker::drawLineAntialiased<drawPixel, NoDasher> (lane 0): two pixels per major step
// weighted by the minor fraction, the end pixels by their 26.6 coverage; pixels inside the staged box
// [bx0, bx0 + bw) x [by0, by0 + bh) are blended in LDS (`box`), the others in the frame
struct HcStroke {
    uint32_t pm;
    uint32_t *frame, *box;
    int bx0, by0, bw, bh;
};
DEV void hc_cs_pixel(const HcStroke &k, int x, int y, int cov) {
    if (x < 0 || x > HR_RES - 1 || y < 0 || y > HR_RES - 1) return;
    const int lx = x - k.bx0, ly = y - k.by0;
    uint32_t *d = (k.box && lx >= 0 && lx < k.bw && ly >= 0 && ly < k.bh) ? k.box + ly * k.bw + lx
                                                                           : k.frame + (size_t)y * HR_RES + x;
    hc_blend_solid(d, k.pm, (cov * 256) >> 8);
}
DEV void hc_cs_line(const HcStroke &k, AgStroker &s, double rx1, double ry1, double rx2, double ry2, int caps) {
    if (ag_cs_clip(s, rx1, ry1, rx2, ry2)) return;
    int x1 = ag_f26(rx1), y1 = ag_f26(ry1), x2 = ag_f26(rx2), y2 = ag_f26(ry2);
    const int dx = x2 - x1, dy = y2 - y1;
    if (abs(dx) < abs(dy)) { // vertical
        const int xinc = ag_fdiv(dx, dy);
        if (y1 > y2) {
            int t = y1; y1 = y2; y2 = t;
            t = x1; x1 = x2; x2 = t;
            caps = ag_swap_caps(caps);
        }
        int x = (x1 - 32) * 1024;
        x -= (((y1 & 63) - 32) * xinc) >> 6;
        ag_cap_adjust(caps, y1, y2, x, xinc);
        int y = y1 >> 6;
        const int ys = y2 >> 6;
        int aS, aE;
        if (y == ys) { aS = y2 - y1; aE = 0; }
        else { aS = 64 - (y1 & 63); aE = y2 & 63; }
        {
            const unsigned al = (uint8_t)(x >> 8);
            hc_cs_pixel(k, x >> 16, y, (int)((255 - al) * aS) >> 6);
            hc_cs_pixel(k, (x >> 16) + 1, y, (int)(al * aS) >> 6);
        }
        x += xinc;
        ++y;
        if (y < ys) {
            do {
                const unsigned al = (uint8_t)(x >> 8);
                hc_cs_pixel(k, x >> 16, y, (int)(255 - al));
                hc_cs_pixel(k, (x >> 16) + 1, y, (int)al);
                x += xinc;
            } while (++y < ys);
        }
        if (aE) {
            const unsigned al = (uint8_t)(x >> 8);
            hc_cs_pixel(k, x >> 16, y, (int)((255 - al) * aE) >> 6);
            hc_cs_pixel(k, (x >> 16) + 1, y, (int)(al * aE) >> 6);
        }
    } else { // horizontal
        if (!dx) return;
        const int yinc = ag_fdiv(dy, dx);
        if (x1 > x2) {
            int t = x1; x1 = x2; x2 = t;
            t = y1; y1 = y2; y2 = t;
            caps = ag_swap_caps(caps);
        }
        int y = (y1 - 32) * 1024;
        y -= (((x1 & 63) - 32) * yinc) >> 6;
        ag_cap_adjust(caps, x1, x2, y, yinc);
        int x = x1 >> 6;
        const int xs = x2 >> 6;
        int aS, aE;
        if (x == xs) { aS = x2 - x1; aE = 0; }
        else { aS = 64 - (x1 & 63); aE = x2 & 63; }
        {
            const unsigned al = (uint8_t)(y >> 8);
            hc_cs_pixel(k, x, y >> 16, (int)((255 - al) * aS) >> 6);
            hc_cs_pixel(k, x, (y >> 16) + 1, (int)(al * aS) >> 6);
        }
        y += yinc;
        ++x;
        if (x < xs) {
            do {
                const unsigned al = (uint8_t)(y >> 8);
                hc_cs_pixel(k, x, y >> 16, (int)(255 - al));
                hc_cs_pixel(k, x, (y >> 16) + 1, (int)al);
                y += yinc;
            } while (++x < xs);
        }
        if (aE) {
            const unsigned al = (uint8_t)(y >> 8);
            hc_cs_pixel(k, x, y >> 16, (int)((255 - al) * aE) >> 6);
            hc_cs_pixel(k, x, (y >> 16) + 1, (int)(al * aE) >> 6);
        }
    }
}
// the 1-px pen along the four curves (renderCubicSubdivision on an explicit stack, no caps); the dial's
// pixels are staged in LDS around lane 0's sequential blends
DEV void hc_stroke_ellipse(HCompassLds &C, const AgPtD pts[13], uint32_t pm, uint32_t *frame) {
    const int tid = threadIdx.x;
    double x0 = pts[0].x, x1 = x0, y0 = pts[0].y, y1 = y0;
    for (int i = 1; i < 13; i++) {
        x0 = fmin(x0, pts[i].x); x1 = fmax(x1, pts[i].x);
        y0 = fmin(y0, pts[i].y); y1 = fmax(y1, pts[i].y);
    }
    HcStroke k;
    k.pm = pm;
    k.frame = frame;
    k.bx0 = max(0, (int)floor(x0) - 2);
    k.by0 = max(0, (int)floor(y0) - 2);
    k.bw = min(HR_RES, (int)ceil(x1) + 3) - k.bx0;
    k.bh = min(HR_RES, (int)ceil(y1) + 3) - k.by0;
    const bool staged = k.bw > 0 && k.bh > 0 && k.bw * k.bh <= HC_CX * HC_CY;
    k.box = staged ? reinterpret_cast<uint32_t *>(C.area) : nullptr;
    if (staged)
        for (int p = tid; p < k.bw * k.bh; p += HR_THREADS)
            k.box[p] = frame[(size_t)(k.by0 + p / k.bw) * HR_RES + k.bx0 + p % k.bw];
    __syncthreads();
    if (tid == 0) {
        AgStroker s;
        s.pm = pm;
        s.xmin = -1; s.xmax = HR_RES + 1; s.ymin = -1; s.ymax = HR_RES + 1;
        s.lastx = s.lasty = AG_INT_MIN;
        s.lastDir = AG_L2R;
        s.lastAxisAligned = false;
        AgPtD *q = C.ag.cs;
        int *st = C.ag.cstack;
        for (int c = 0; c < 4; c++) {
            q[3] = pts[3 * c];
            q[2] = pts[3 * c + 1];
            q[1] = pts[3 * c + 2];
            q[0] = pts[3 * c + 3];
            int sp = 0;
            st[0] = 0 | (AG_CS_MAXSUB << 8);
            while (sp >= 0) {
                const int off = st[sp] & 0xff, level = st[sp] >> 8;
                sp--;
                AgPtD *pp = q + off;
                if (level) {
                    const double dx = pp[3].x - pp[0].x, dy = pp[3].y - pp[0].y;
                    const double len = ((double).25) * (fabs(dx) + fabs(dy));
                    if (fabs(dx * (pp[0].y - pp[2].y) - dy * (pp[0].x - pp[2].x)) >= len ||
                        fabs(dx * (pp[0].y - pp[1].y) - dy * (pp[0].x - pp[1].x)) >= len) {
                        ag_cs_split(pp);
                        st[++sp] = off | ((level - 1) << 8);
                        st[++sp] = (off + 3) | ((level - 1) << 8);
                        continue;
                    }
                }
                hc_cs_line(k, s, pp[3].x, pp[3].y, pp[0].x, pp[0].y, 0);
            }
        }
    }
    __syncthreads();
    if (staged)
        for (int p = tid; p < k.bw * k.bh; p += HR_THREADS)
            frame[(size_t)(k.by0 + p / k.bw) * HR_RES + k.bx0 + p % k.bw] = k.box[p];
    __syncthreads();
}
// drawEllipse(QRectF(x, y, w, h)): brush (0 = none) then a 1-px pen (0 = none), non-premultiplied ARGB
DEV bool hc_draw_ellipse(HCompassLds &C, double x, double y, double w, double h, uint32_t brush, uint32_t pen,
                         uint32_t *frame) {
    if (w <= 0 || h <= 0) return true;
    AgPtD pts[13];
    ag_ellipse_points(x, y, w, h, pts);
    bool ok = true;
    if ((brush >> 24) && hc_path_on_device(pts, 13)) ok = hc_fill_ellipse(C, pts, ag_solid_premul(brush), frame);
    if (pen >> 24) hc_stroke_ellipse(C, pts, ag_solid_premul(pen), frame);
    return ok;
}
// drawLine(QLine(x1, y1, x2, y2)) with QPen(colour, width > 1), SquareCap: rasterizeLine(width / length)
DEV void hc_wide_line(int x1, int y1, int x2, int y2, int width, uint32_t argb, uint32_t *frame) {
    const double dx = (double)x2 - x1, dy = (double)y2 - y1, len = sqrt(dx * dx + dy * dy);
    HLine L;
    if (len == 0) // a point: the square cap alone, a horizontal line of the pen's width, relative width 1
        hr_line(x1 - width * 0.5, y1, x1 + width * 0.5, y1, 1, L, false);
    else
        hr_line(x1, y1, x2, y2, width / len, L, true);
    const uint32_t pm = ag_solid_premul(argb);
    if (L.kind != 0)
        for (int r = threadIdx.x; r < L.nrows; r += HR_THREADS)
            hr_row_spans(L, r, [&](int sx, int sl, int sy, int sc) {
                for (int xx = sx; xx < sx + sl; xx++) hc_blend_solid(frame + (size_t)sy * HR_RES + xx, pm, sc);
            });
    __syncthreads();
}
DEV bool hc_draw_compass(HCompassLds &C, uint32_t *frame, const PGDev &d, const PGEnv &s, const View &v, int env) {
    const float u = v.unit, vd = v.view_dim, cd = s.gs.jp.compass_dim;
    const float ax = (float)(vd - cd - .25), ay = .25f; // get_abs_rect (:812-814)
    const double rx = (double)(ax * u), ry = (double)(ay * u), rw = (double)(cd * u), rh = (double)(cd * u);
    bool ok = hc_draw_ellipse(C, rx, ry, rw, rh, 0xffa8a69eu, 0xffa8a69eu, frame); // QColor(168, 166, 158)
    const float pen_thickness = (float)(HR_RES / (256.0 / cd));
    const float cx = (float)(rx + rw / 2), cy = (float)(ry + rh / 2); // QRectF::center
    const float cr = (float)(rw / 2 * .95);
    const float agx = EFr(d, F_X, env, 0), agy = EFr(d, F_Y, env, 0), arx = EFr(d, F_RX, env, 0), ary = EFr(d, F_RY, env, 0);
    const float gx = EFr(d, F_X, env, 1), gy = EFr(d, F_Y, env, 1);
    const float theta = (float)atan2((double)(gy - agy), (double)(gx - agx)); // get_theta (:241-246)
    double sn, cs;
    pg_sincos_cr((double)theta, &sn, &cs);
    const int x1 = (int)cx, y1 = (int)cy; // QPainter::drawLine(int, int, int, int)
    const int x2 = (int)((double)cx + (double)cr * cs), y2 = (int)((double)cy - (double)cr * sn);
    hc_wide_line(x1, y1, x2, y2, (int)pen_thickness, 0xfffcba03u, frame); // QColor(252, 186, 3)
    const float ddx = agx - gx, ddy = agy - gy; // get_distance (:133-143)
    const float dist = (float)sqrt((double)(ddx * ddx + ddy * ddy));
    const float dist_pct = (float)((double)dist / (s.main_width * 1.4142135623730951));
    const float bar_thickness = cd / 8;
    HOp op;
    op.kind = 1; op.px = nullptr; op.iw = op.ih = 0; op.rgb32 = 0; op.mir = 0; op.ca = 256;
    op.x = (double)((float)(vd - cd - .25) * u); op.y = (double)((float)(.25 + cd) * u);
    op.w = (double)(cd * dist_pct * u); op.h = (double)(bar_thickness * u); op.argb = 0xfffcba03u;
    hr_run(frame, op);
    if (s.gs.jp.jump_delta < 0 && !s.has_support) { // drawEllipse(QRect(...)), QColor(255, 255, 255, 120)
        double r1x, r1y, r1w, r1h;
        screen_rect(v, agx - arx, agy + ary, 2 * arx, 2 * ary, 0, r1x, r1y, r1w, r1h);
        const int qx = (int)r1x, qy = (int)(r1y + r1h * (5.0 / 6)), qw = (int)r1w, qh = (int)(r1h / 3);
        ok = hc_draw_ellipse(C, qx, qy, qw, qh, 0x78ffffffu, 0, frame) && ok;
    }
    return ok;
}

// the kernel's LDS: the rotated path's span lists (games with rotating entities) and, for jumper, the
// compass's cells in the same bytes (the compass is painted after every entity)
template <bool ROT, bool J> struct HLds { int unused; DEV HRotLds *rot() { return nullptr; } DEV HCompassLds *compass() { return nullptr; } };
template <> struct HLds<true, false> { HRotLds r; DEV HRotLds *rot() { return &r; } DEV HCompassLds *compass() { return nullptr; } };
template <> struct HLds<true, true> {
    union { HRotLds r; HCompassLds c; };
    DEV HRotLds *rot() { return &r; }
    DEV HCompassLds *compass() { return &c; }
};

template <int G>
__global__ __launch_bounds__(HR_THREADS) void pg_render_hires_kernel(PGDev dg, const int32_t *env_list, uint32_t *frames,
                                                                     uint8_t *rgb) {
    const PGDev d = game_view(dg, G);
    __shared__ HLds<has_rotation<G>(), G == PG_GAME_JUMPER> lds;
    HRotLds *L = lds.rot();
    const int env = env_list ? env_list[blockIdx.x] : (int)blockIdx.x;
    const int slot = blockIdx.x; // frame / rgb rows of this launch
    uint32_t *frame = frames + (size_t)slot * HR_RES * HR_RES;
    const PGEnv s = d.envs[env];
    const int16_t *Gd = d.grid + (size_t)env * PG_GRID_MAX;
    bool ok = true;
    float agent_x, agent_y, agent_vx, agent_vy;
    if (s.agent_erased) {
        agent_x = s.ghost_x; agent_y = s.ghost_y; agent_vx = s.ghost_vx; agent_vy = s.ghost_vy;
    } else {
        agent_x = EFr(d, F_X, env, 0); agent_y = EFr(d, F_Y, env, 0);
        agent_vx = EFr(d, F_VX, env, 0); agent_vy = EFr(d, F_VY, env, 0);
    }
    const int player_img = player_image<G>(s, agent_vx);
    // prepare_for_drawing(rect_height = RENDER_RES) (basic-abstract-game.cpp:828-847)
    View v;
    v.center_x = (float)(s.main_width * .5);
    v.center_y = (float)(s.main_height * .5);
    v.visibility = s.visibility;
    if (s.opt_center_agent) {
        if constexpr (G == PG_GAME_CLIMBER) { // climber.cpp:291-295
            const float agent_ry = s.agent_erased ? s.ghost_ry : EFr(d, F_RY, env, 0);
            v.center_x = (float)(s.main_width / 2.0);
            v.center_y = (float)((double)agent_y + s.main_width / 2.0 - (double)(5 * agent_ry));
            v.visibility = (float)s.main_width;
        } else if constexpr (G == PG_GAME_FRUITBOT) { // fruitbot.cpp:138-142
            const float agent_ry = s.agent_erased ? s.ghost_ry : EFr(d, F_RY, env, 0);
            v.center_x = (float)(s.main_width / 2.0);
            v.center_y = (float)((double)agent_y + s.main_width / 2.0 - (double)(2 * agent_ry));
            v.visibility = (float)s.main_width;
        } else {
            v.center_x = agent_x;
            v.center_y = agent_y;
        }
    } else {
        v.visibility = (float)(s.main_width > s.main_height ? s.main_width : s.main_height);
        if (v.visibility < s.min_visibility) v.visibility = s.min_visibility;
    }
    const float raw_unit = 64 / v.visibility;
    v.unit = (float)((double)raw_unit * ((double)(float)HR_RES / 64.0));
    v.view_dim = (float)(64.0 / (double)raw_unit);
    v.x_off = v.unit * (v.center_x - v.view_dim / 2);
    v.y_off = v.unit * (v.center_y - v.view_dim / 2);

    // draw_background (:988-1016): fillRect(rect, black) + the background image
    HOp op;
    op.kind = 1; op.x = 0; op.y = 0; op.w = HR_RES; op.h = HR_RES; op.argb = 0xff000000u;
    op.px = nullptr; op.iw = op.ih = 0; op.rgb32 = 0; op.mir = 0; op.ca = 256;
    hr_run(frame, op);
    if constexpr (G == PG_GAME_STARPILOT) {
        // starpilot game_draw (starpilot.cpp:107-124): no draw_background; tile_image(r_bg, 1) of the
        // background scrolled left by cur_time, r_bg in RENDER_RES units
        if (s.opt_use_backgrounds) {
            const float scale = (float)(HR_RES / s.main_height); // int / int
            const float bg_k = 3, t = (float)s.cur_time, BG_RATIO = 18;
            const float x_off = -t * scale * SP_HP_SLOW_V * 2 / s.char_dim;
            const int4 bgi = reinterpret_cast<const int4 *>(d.backgrounds)[s.background_index];
            op.kind = 0; op.x = (double)x_off; op.y = (double)(-HR_RES * (bg_k - 1) / 2);
            op.w = (double)(HR_RES * bg_k * BG_RATIO); op.h = (double)(HR_RES * bg_k);
            op.px = (d.gen_bg ? d.gen_bg + (size_t)env * (500 * 500) : d.pixels + bgi.x);
            op.iw = bgi.y; op.ih = bgi.z; op.rgb32 = 1; op.mir = 0; op.ca = 256;
            if (op.iw > 0 && op.ih > 0) hr_tiles(frame, op, 1.0f);
        }
    } else if (s.opt_use_backgrounds) {
        double mx, my, mw, mh;
        screen_rect(v, 0, (float)s.main_height, (float)s.main_width, (float)s.main_height, 0, mx, my, mw, mh);
        const int4 bgi = reinterpret_cast<const int4 *>(d.backgrounds)[s.background_index];
        const float bgw = (float)bgi.y, bgh = (float)bgi.z;
        const float bg_ar = bgw / bgh;
        const float world_ar = (float)(s.main_width * 1.0 / s.main_height);
        const float offset_x = s.bg_pct_x * (bg_ar - world_ar);
        const double ax = (double)(-offset_x), aw = (double)(bg_ar / world_ar);
        op.kind = 0; op.x = mx + mw * ax; op.y = my + mh * 0.0; op.w = mw * aw; op.h = mh * 1.0;
        op.px = (d.gen_bg ? d.gen_bg + (size_t)env * (500 * 500) : d.pixels + bgi.x);
        op.iw = bgi.y; op.ih = bgi.z; op.rgb32 = 1; op.mir = 0; op.ca = 256;
        if (s.bg_tile_ratio < 0) { // fruitbot (fruitbot.cpp:30-40): the world rect tiled (:1003-1004)
            op.x = mx; op.y = my; op.w = mw; op.h = mh;
            if (op.w > 0 && op.h > 0 && op.iw > 0 && op.ih > 0) hr_tiles(frame, op, s.bg_tile_ratio);
        } else if (op.w > 0 && op.h > 0 && op.iw > 0 && op.ih > 0) {
            hr_run(frame, op);
        }
    }
    // draw_foreground (:930-979)
    if constexpr (has_z_minus1<G>()) ok = hr_entities<G>(frame, d, s, v, env, -1, player_img, L) && ok;
    int low_x, high_x, low_y, high_y;
    if (s.opt_center_agent) {
        const double margin = (double)v.visibility / 2.0 + 1;
        low_x = (int)((double)v.center_x - margin);
        high_x = (int)((double)v.center_x + margin);
        low_y = (int)((double)v.center_y - margin);
        high_y = (int)((double)v.center_y + margin);
    } else {
        low_x = 0; high_x = s.main_width - 1; low_y = 0; high_y = s.main_height - 1;
    }
    for (int x = low_x; x <= high_x; x++) {
        for (int y = low_y; y <= high_y; y++) {
            const int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? Gd[y * s.main_width + x]
                                                                                       : s.out_of_bounds_object;
            if (type == INVALID_OBJ) continue;
            double rx, ry, rw, rh;
            screen_rect(v, (float)x, (float)(y + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
            ok = hr_draw_image<G>(frame, d, s, rx, ry, rw, rh, false, type, grid_theme<G>(s, type), 1.0f, player_img, 0.0f,
                                  0.0f, L) && ok;
        }
    }
    ok = hr_entities<G>(frame, d, s, v, env, 0, player_img, L) && ok;
    ok = hr_entities<G>(frame, d, s, v, env, 1, player_img, L) && ok;
    if (s.has_useful_vel_info && s.opt_paint_vel_info) { // :969-977
        const float infodim = (float)(HR_RES * .2);
        const int s1 = to_shade((float)(.5 * (double)agent_vx / (double)s.maxspeed + .5));
        const int s2 = to_shade((float)(.5 * (double)agent_vy / (double)s.max_jump + .5));
        op.kind = 1; op.x = 0; op.y = 0; op.w = infodim; op.h = infodim; op.argb = 0xff000000u | (uint32_t)(s1 * 0x010101);
        hr_run(frame, op);
        op.x = infodim; op.argb = 0xff000000u | (uint32_t)(s2 * 0x010101);
        hr_run(frame, op);
    }
    if constexpr (G == PG_GAME_NINJA) { // ninja.cpp:155-164: jump charge bar, get_abs_rect (:812-814)
        const float u = v.unit, bar_height = 3 * s.gs.nj.jump_charge;
        op.kind = 1; op.x = (double)(.25f * u); op.y = (double)((float)(v.visibility - .5 - bar_height) * u);
        op.w = (double)(.5f * u); op.h = (double)(bar_height * u); op.argb = 0xff42f587u;
        hr_run(frame, op);
    }
    if constexpr (G == PG_GAME_JUMPER) // the compass (jumper.cpp:137-177), outside memory mode
        if (s.opt_distribution_mode != PG_MEMORY) ok = hc_draw_compass(*lds.compass(), frame, d, s, v, env) && ok;
    if constexpr (G == PG_GAME_PLUNDER) { // plunder.cpp:66-77: juice and progress bars, get_abs_rect (:812-814)
        const float u = v.unit;
        op.kind = 1; op.x = (double)(.25f * u); op.y = (double)(.25f * u);
        op.w = (double)(s.main_width * s.gs.pl.juice_left * u); op.h = (double)(.5f * u); op.argb = 0xff42f587u;
        hr_run(frame, op);
        const float prog = (float)(s.main_width * (s.gs.pl.targets_hit * 1.0 / s.gs.pl.target_quota));
        op.x = (double)(.25f * u); op.y = (double)(.75f * u); op.w = (double)(prog * u); op.h = (double)(.5f * u);
        op.argb = 0xfff54290u;
        hr_run(frame, op);
    }
    // bgr32_to_rgb888 (game.cpp:8-23) into info["rgb"]
    uint8_t *out = rgb + (size_t)slot * HR_RES * HR_RES * 3;
    for (int p = threadIdx.x; p < HR_RES * HR_RES; p += HR_THREADS) {
        const uint32_t c = frame[p];
        out[3 * p + 0] = (uint8_t)(c >> 16);
        out[3 * p + 1] = (uint8_t)(c >> 8);
        out[3 * p + 2] = (uint8_t)c;
    }
    if (!ok && threadIdx.x == 0) atomicOr(d.error_any, 1 << PG_ERR_RENDER);
}

#ifndef PG_FUSED_TU // pg_fused.hip includes this file for rf_render_env
// mode: see pg_render_kernel (0 all, 1 envs not done, 2 the reset queue: `count` bounds its length)
extern "C" void pg_launch_render(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s, int mode,
                                 int slot) {
    if (count <= 0) return;
#define PG_CASE(G)                                                                              \
    case G:                                                                                     \
        if (rf_game<G>() && ((d->render_rf >> G) & 1))                                          \
            hipLaunchKernelGGL(pg_render_rf_kernel<G>, dim3(count), dim3(64), 0, s, *d, env_list, mode, slot, count); \
        else                                                                                    \
            hipLaunchKernelGGL(pg_render_kernel<G>, dim3((count + PG_RENDER_K - 1) / PG_RENDER_K), dim3(64), 0, s, *d, env_list, mode, slot, count); \
        break;
    switch (game) {
#ifdef PG_ONLY_GAME // resource checks of one game's kernels (hipcc -DPG_ONLY_GAME=11 -Rpass-analysis=...)
        PG_CASE(PG_ONLY_GAME)
#else
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
#endif
    default: break;
    }
#undef PG_CASE
}

// Debug aid (PROCGEN_MI355X_POISON_LDS=1): fill the LDS of every CU with a pattern before each
// engine kernel, so a kernel that reads LDS before writing it shows up as a parity failure
// instead of silently inheriting the previous wave's data.
extern "C" __global__ __launch_bounds__(256) void pg_poison_lds_kernel(uint32_t pattern) {
    __shared__ volatile uint32_t buf[16384]; // 64 KB
    for (int k = threadIdx.x; k < 16384; k += 256) buf[k] = pattern ^ (uint32_t)(k * 0x9E3779B9u);
}

extern "C" void pg_launch_poison(hipStream_t s, uint32_t pattern) {
    hipLaunchKernelGGL(pg_poison_lds_kernel, dim3(2048), dim3(256), 0, s, pattern);
}

// render_mode="rgb_array": frames / rgb hold `count` RENDER_RES^2 slots (the game's envs in list order)
extern "C" int pg_launch_render_hires(const PGDev *d, int game, const int32_t *env_list, int count, uint32_t *frames,
                                      uint8_t *rgb, hipStream_t s) {
    if (count <= 0) return 0;
#ifdef PG_ONLY_GAME
    (void)d; (void)env_list; (void)frames; (void)rgb; (void)s;
    return -1;
#else
    switch (game) {
#define PG_CASE(G)                                                                                               \
    case G:                                                                                                      \
        hipLaunchKernelGGL(pg_render_hires_kernel<G>, dim3(count), dim3(HR_THREADS), 0, s, *d, env_list, frames, rgb); \
        return 0;
        PG_CASE(PG_GAME_BIGFISH)
        PG_CASE(PG_GAME_CHASER)
        PG_CASE(PG_GAME_CLIMBER)
        PG_CASE(PG_GAME_COINRUN)
        PG_CASE(PG_GAME_MAZE)
        PG_CASE(PG_GAME_MINER)
        PG_CASE(PG_GAME_NINJA)
        PG_CASE(PG_GAME_BOSSFIGHT)
        PG_CASE(PG_GAME_CAVEFLYER)
        PG_CASE(PG_GAME_DODGEBALL)
        PG_CASE(PG_GAME_FRUITBOT)
        PG_CASE(PG_GAME_HEIST)
        PG_CASE(PG_GAME_LEAPER)
        PG_CASE(PG_GAME_PLUNDER)
        PG_CASE(PG_GAME_STARPILOT)
        PG_CASE(PG_GAME_JUMPER)
#undef PG_CASE
    default: return -1;
    }
#endif
}
#endif // PG_FUSED_TU
