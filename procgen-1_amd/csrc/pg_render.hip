// pg_render.hip -- Game::observe: 64x64 render + bgr32_to_rgb888 (reference game.cpp:8-23,
// 97-107, 173-191; basic-abstract-game.cpp:808-1075; games/coinrun.cpp:64-70, 133-138, 213-225).
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

namespace {

struct View {
    float unit, x_off, y_off, view_dim, visibility, center_x, center_y;
};

DEV float EFr(const PGDev &d, int f, int env, int slot) {
    return d.ents[(size_t)f * d.num_envs * PG_CAP + (size_t)env * PG_CAP + slot];
}
DEV int EIr(const PGDev &d, int f, int env, int slot) {
    return reinterpret_cast<const int *>(d.ents)[(size_t)f * d.num_envs * PG_CAP + (size_t)env * PG_CAP + slot];
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

// Size of the per-type grid sprite table (grid values 0..127 take the fast path).
#define NTYPES 128
// Tile images all have this size in coinrun (other sizes are flagged, not drawn wrongly).
#define TILE_PX 128
// Most tile rows a frame may span on the fast path (centred coinrun views span 14-15).
#define CROWS 16
// Rows per batch of the pixel-centric pass, entities per stamping group.
#ifndef RB
#define RB 8
#endif
#ifndef EG
#define EG 8
#endif

} // namespace

extern "C" __global__ __launch_bounds__(64) void pg_render_kernel(PGDev d) {
    __shared__ __attribute__((aligned(16))) uint32_t fb[PG_RES * PG_RES];
    __shared__ int tile_off[NTYPES];  // sprite pixel offset of a grid type, -1: draws nothing, <= -2: unsupported
    // fast path: texel base of lane's first tile column per tile row.  Before it is built, the
    // same LDS holds the Qt blit setup (t1, n, base, step) of every window tile column / row.
    __shared__ __attribute__((aligned(16))) int colb[CROWS * 64];
    static_assert(CROWS * 64 >= 2 * 64 * 4, "colb doubles as the axis tables");
    int4 *const colax = reinterpret_cast<int4 *>(colb);
    int4 *const rowax = colax + 64;
    const int env = blockIdx.x;
    const PGEnv s = d.envs[env];
    const int16_t *G = d.grid + (size_t)env * PG_GRID_MAX;
    bool err = false;

    float agent_x, agent_y, agent_vx;
    if (s.agent_erased) {
        agent_x = s.ghost_x; agent_y = s.ghost_y; agent_vx = s.ghost_vx;
    } else {
        agent_x = EFr(d, F_X, env, 0); agent_y = EFr(d, F_Y, env, 0); agent_vx = EFr(d, F_VX, env, 0);
    }
    // image_for_type(PLAYER) (coinrun.cpp:213-219): one animation frame for the whole frame
    const int player_img = (fabs((double)agent_vx) < .01 && s.action_vx == 0 && s.has_support)
                               ? PLAYER
                               : ((s.cur_time / 5 % 2 == 0 || !s.has_support) ? CR_PLAYER_RIGHT1 : CR_PLAYER_RIGHT2);

    // ---- prepare_for_drawing(rect_height = 64) (basic-abstract-game.cpp:828-847)
    View v;
    v.center_x = (float)(s.main_width * .5);
    v.center_y = (float)(s.main_height * .5);
    v.visibility = s.visibility;
    if (s.opt_center_agent) {
        v.center_x = agent_x;
        v.center_y = agent_y;
    } else {
        v.visibility = (float)(s.main_width > s.main_height ? s.main_width : s.main_height);
        if (v.visibility < s.min_visibility) v.visibility = s.min_visibility;
    }
    float raw_unit = 64 / v.visibility;
    v.unit = (float)((double)raw_unit * ((double)64.0f / 64.0));
    v.view_dim = (float)(64.0 / (double)raw_unit);
    v.x_off = v.unit * (v.center_x - v.view_dim / 2);
    v.y_off = v.unit * (v.center_y - v.view_dim / 2);

    const int lane = LANE;
    PTimer pt;
    pt.start();

    // ---- grid type -> sprite table (theme_for_grid_obj coinrun.cpp:133-138, image_for_type :213-225,
    //      draw_image basic-abstract-game.cpp:886-922)
    for (int t = lane; t < NTYPES; t += 64) {
        int off = -1;
        int img = t == PLAYER ? player_img : (t == CR_ENEMY_BARRIER ? -1 : t);
        if (img >= 0) {
            if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) {
                off = (img == SPACE) ? -1 : -3; // draw_grid_obj fills: not in this build
            } else {
                int theme = cr_is_wall(t) ? s.wall_theme : 0;
                if (s.opt_restrict_themes) theme = 0;
                int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                if (sp.y == TILE_PX && sp.z == TILE_PX) off = sp.x;
                else if (sp.y > 0) off = -2;
                else off = -3; // generated assets: not in this build
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
                xr = rx; xw = rw; xiw = TILE_PX;
            }
            if (lane < wh) {
                screen_rect(v, 0.0f, (float)(low_y + lane + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
                yr = ry; yh = rh; yih = TILE_PX;
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
    const bool bg_col = bg_ok && lane >= bx.t1 && lane < bx.t1 + bx.n;
    const uint32_t bg_col_base = (uint32_t)bgi.x + (bg_col ? (bx.base + (uint32_t)((lane - bx.t1) * bx.step)) >> 16 : 0);

    // tile columns covering screen column `lane` (<= 2, ascending x) for TILE_PX-wide images
    int cx0 = 0, cx1 = 0, ncx = 0;
    Axis ax0, ax1;
    ax0.n = ax1.n = 0;
    {
        int xg = (int)floorf(((float)lane + 0.5f + v.x_off) / v.unit);
        for (int x = xg - 2; x <= xg + 2; x++) {
            if (x < low_x || x > high_x || ncx == 2) continue;
            Axis a;
            bool ok;
            if (tab) {
                const int4 t = colax[x - low_x];
                a.t1 = t.x; a.n = t.y; a.base = (uint32_t)t.z; a.step = t.w;
                ok = t.y > 0;
            } else {
                double rx, ry, rw, rh;
                screen_rect(v, (float)x, 0.0f, 1, 1, RENDER_EPS, rx, ry, rw, rh);
                ok = axis_setup(rx, rw, TILE_PX, a);
            }
            if (ok && lane >= a.t1 && lane < a.t1 + a.n) {
                if (ncx == 0) { cx0 = x; ax0 = a; } else { cx1 = x; ax1 = a; }
                ncx++;
            }
        }
    }
    const int scol0 = ncx > 0 ? (int)((ax0.base + (uint32_t)((lane - ax0.t1) * ax0.step)) >> 16) : 0;
    const int scol1 = ncx > 1 ? (int)((ax1.base + (uint32_t)((lane - ax1.t1) * ax1.step)) >> 16) : 0;
    // tile rows covering screen row `lane` (<= 2, ascending y = the reference's draw order)
    int ry0 = 0, ry1 = 0, ncy = 0, srow0 = 0, srow1 = 0;
    {
        int yg = (int)floorf((v.view_dim - ((float)lane + 0.5f - v.y_off) / v.unit));
        for (int y = yg - 2; y <= yg + 2; y++) {
            if (y < low_y || y > high_y || ncy == 2) continue;
            Axis a;
            bool ok;
            if (tab) {
                const int4 t = rowax[y - low_y];
                a.t1 = t.x; a.n = t.y; a.base = (uint32_t)t.z; a.step = t.w;
                ok = t.y > 0;
            } else {
                double rx, ry, rw, rh;
                screen_rect(v, 0.0f, (float)(y + 1), 1, 1, RENDER_EPS, rx, ry, rw, rh);
                ok = axis_setup(ry, rh, TILE_PX, a);
            }
            if (ok && lane >= a.t1 && lane < a.t1 + a.n) {
                int sr = (int)((a.base + (uint32_t)((lane - a.t1) * a.step)) >> 16);
                if (ncy == 0) { ry0 = y; srow0 = sr; } else { ry1 = y; srow1 = sr; }
                ncy++;
            }
        }
    }

    // ---- lookups for the fast path: every screen row's tile rows lie in [jy0, jy1]; for
    //      each of those rows the texel base of this lane's first tile column goes to LDS
    //      (colb), so a pixel costs one LDS read + one texel load + one blend.
    int jlo = ncy > 0 ? ry0 : 0x7fffffff, jhi = ncy > 1 ? ry1 : (ncy > 0 ? ry0 : -0x7fffffff);
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        jlo = min(jlo, __shfl_xor(jlo, sh));
        jhi = max(jhi, __shfl_xor(jhi, sh));
    }
    const int jy0 = jlo, nrows = jhi >= jlo ? jhi - jlo + 1 : 0;
    const bool fast = nrows <= CROWS;
    auto lookup_grid = [&](int x, int y) -> int {
        int type = (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) ? G[y * s.main_width + x]
                                                                               : s.out_of_bounds_object;
        return type == INVALID_OBJ ? -1 : ((type >= 0 && type < NTYPES) ? tile_off[type] : -2);
    };
    wave_sync(); // tile_off complete
    if (fast) {
        int code[CROWS];
#pragma unroll
        for (int j = 0; j < CROWS; j++) {
            code[j] = -1;
            if (j < nrows && ncx > 0) {
                const int y = jy0 + j, x = cx0;
                if (0 <= y && y < s.main_height && 0 <= x && x < s.main_width) code[j] = G[y * s.main_width + x];
                else code[j] = s.out_of_bounds_object;
            }
        }
#pragma unroll
        for (int j = 0; j < CROWS; j++) {
            if (j < nrows) {
                int t = code[j];
                int c = (ncx == 0 || t == INVALID_OBJ) ? -1 : ((t >= 0 && t < NTYPES) ? tile_off[t] : -2);
                if (c <= -2) err = true;
                colb[j * 64 + lane] = c >= 0 ? c + scol0 : -1;
            }
        }
    }
    wave_sync();

    pt.mark(0);
    if (fast) {
        // ---- background + first tile column, pixel-centric, RB rows per batch (all loads of
        //      a batch are issued before the first blend).  A transparent texel (0) blends to
        //      the unchanged pixel exactly, so lanes without a tile carry 0.
        // per screen row (lane = row), packed for one readlane per row: source rows of its
        // tile rows (7 bits each), their colb rows (5 bits each), tile-row count (2 bits);
        // and the background source row offset (-1: outside the background blit)
        const int prow = lane;
        const int rinfo = ncy == 0 ? 0
                        : (srow0 | ((ncy > 1 ? srow1 : 0) << 7) | ((ry0 - jy0) << 14) |
                           ((ncy > 1 ? ry1 - jy0 : ry0 - jy0) << 19) | (ncy << 24));
        const int bgrow = (bg_ok && prow >= by.t1 && prow < by.t1 + by.n)
                              ? (int)(((by.base + (uint32_t)((prow - by.t1) * by.step)) >> 16) * (uint32_t)bgi.y)
                              : -1;
        for (int r0 = 0; r0 < PG_RES; r0 += RB) {
            uint32_t bgv[RB], ta[RB], tb[RB];
            int info[RB], bgr[RB], ca[RB], cbv[RB];
#pragma unroll
            for (int k = 0; k < RB; k++) {
                info[k] = readlane(rinfo, r0 + k);
                bgr[k] = readlane(bgrow, r0 + k);
            }
#pragma unroll
            for (int k = 0; k < RB; k++) { // LDS reads of the whole batch first
                ca[k] = colb[((info[k] >> 14) & 31) * 64 + lane];
                cbv[k] = colb[((info[k] >> 19) & 31) * 64 + lane];
            }
#pragma unroll
            for (int k = 0; k < RB; k++) { // branch-free: an out-of-blit pixel loads pixels[0] and discards it
                const bool inb = bg_col && bgr[k] >= 0;
                uint32_t v = d.pixels[inb ? bg_col_base + (uint32_t)bgr[k] : 0u];
                bgv[k] = inb ? v : 0xff000000u;
            }
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int nr = info[k] >> 24;
                ta[k] = 0;
                tb[k] = 0;
                if (nr > 0 && ca[k] >= 0) ta[k] = d.pixels[(uint32_t)ca[k] + (uint32_t)((info[k] & 127) * TILE_PX)];
                if (nr > 1 && cbv[k] >= 0) tb[k] = d.pixels[(uint32_t)cbv[k] + (uint32_t)(((info[k] >> 7) & 127) * TILE_PX)];
            }
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int nr = info[k] >> 24;
                uint32_t px = bgv[k];
                if (nr > 0) px = ta[k] + BYTE_MUL(px, (~ta[k]) >> 24);
                if (nr > 1) px = tb[k] + BYTE_MUL(px, (~tb[k]) >> 24);
                fb[(r0 + k) * PG_RES + lane] = px;
            }
        }
        wave_sync();
        // ---- second tile column of the few screen columns two tiles overlap (RENDER_EPS):
        //      drawn after the first column's tiles, which is the reference's x-major order.
        //      Lane = screen row here, so the row tables are lane-local.
        unsigned long long m2 = ballot(ncx > 1);
        while (m2) {
            const int c = __ffsll((long long)m2) - 1;
            m2 &= m2 - 1;
            const int x1 = readlane(cx1, c), sc1 = readlane(scol1, c);
            const int row = lane;
            if (ncy > 0) {
                uint32_t px = fb[row * PG_RES + c];
                for (int l = 0; l < ncy; l++) {
                    const int code = lookup_grid(x1, l ? ry1 : ry0);
                    if (code <= -2) err = true;
                    if (code >= 0) {
                        const uint32_t t = d.pixels[(uint32_t)code + (uint32_t)((l ? srow1 : srow0) * TILE_PX + sc1)];
                        px = t + BYTE_MUL(px, (~t) >> 24);
                    }
                }
                fb[row * PG_RES + c] = px;
            }
        }
    } else {
        // ---- generic pixel-centric pass (uncentred / very large views): a pixel blends every
        //      tile covering it (<= 2 columns x 2 rows) in the reference's x-major order.
        for (int r0 = 0; r0 < PG_RES; r0 += RB) {
            uint32_t bgv[RB], tex[RB][4];
            uint32_t valid = 0;
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int row = r0 + k;
                const bool inb = bg_col && row >= by.t1 && row < by.t1 + by.n;
                {
                    uint32_t srow = (by.base + (uint32_t)((row - by.t1) * by.step)) >> 16;
                    uint32_t v = d.pixels[inb ? bg_col_base + srow * (uint32_t)bgi.y : 0u];
                    bgv[k] = inb ? v : 0xff000000u;
                }
                const int nr = readlane(ncy, row);
                const int y_a = readlane(ry0, row), y_b = readlane(ry1, row);
                const int sr_a = readlane(srow0, row), sr_b = readlane(srow1, row);
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const int kk = c >> 1, l = c & 1;
                    const bool cand = kk < ncx && l < nr;
                    const int x = kk ? cx1 : cx0, y = l ? y_b : y_a;
                    const int off = cand ? lookup_grid(x, y) : -1;
                    if (off <= -2) err = true;
                    const bool on = off >= 0;
                    const int scol = kk ? scol1 : scol0, srow = l ? sr_b : sr_a;
                    tex[k][c] = 0;
                    if (on) tex[k][c] = d.pixels[(uint32_t)off + (uint32_t)(srow * TILE_PX + scol)];
                    valid |= (on ? 1u : 0u) << (k * 4 + c);
                }
            }
#pragma unroll
            for (int k = 0; k < RB; k++) {
                uint32_t px = bgv[k];
#pragma unroll
                for (int c = 0; c < 4; c++) // draw order: (x0,y0) (x0,y1) (x1,y0) (x1,y1)
                    if (valid & (1u << (k * 4 + c))) px = tex[k][c] + BYTE_MUL(px, (~tex[k][c]) >> 24);
                fb[(r0 + k) * PG_RES + lane] = px;
            }
        }
    }
    wave_sync();

    pt.mark(1);
    // ---- entities, render_z 0 then 1, in list order (basic-abstract-game.cpp:966-967, 1061-1075)
    const int n = s.num_ents;
    const bool one_chunk = n <= 64; // blit setups computed once and reused by both z passes
    bool draw = false;
    int ez = 0;
    Axis ex, ey;
    int soff = 0, sw = 0, ca = 256, mir = 0;
    for (int z = 0; z <= 1; z++) {
        for (int base = 0; base < n; base += 64) {
            // lane-parallel blit setup of entity base + lane
            const int i = base + lane;
            if (!one_chunk || z == 0) {
                draw = false;
                ez = 0;
                soff = 0; sw = 0; ca = 256; mir = 0;
                if (i < n) {
                    ez = EIr(d, F_RENDER_Z, env, i);
                    float px_ = EFr(d, F_X, env, i), py_ = EFr(d, F_Y, env, i);
                    float prx = EFr(d, F_RX, env, i), pry = EFr(d, F_RY, env, i);
                    int flags = EIr(d, F_FLAGS, env, i);
                    float alpha = EFr(d, F_ALPHA, env, i);
                    float rotation = EFr(d, F_ROTATION, env, i);
                    int itype = EIr(d, F_IMAGE_TYPE, env, i);
                    int theme = EIr(d, F_IMAGE_THEME, env, i);
                    int img = itype == PLAYER ? player_img : (itype == CR_ENEMY_BARRIER ? -1 : (itype < 0 ? -itype : itype));
                    if (img >= 0 && (ez == 0 || ez == 1)) {
                        if ((flags & EF_ABS_COORDS) || rotation != 0 || s.opt_use_monochrome_assets ||
                            img >= USE_ASSET_THRESHOLD) {
                            if (img != SPACE) err = true; // not in this build
                        } else {
                            if (s.opt_restrict_themes) theme = 0;
                            double rx, ry, rw, rh;
                            screen_rect(v, px_ - prx, py_ + pry, 2 * prx, 2 * pry, 0, rx, ry, rw, rh);
                            if (is_player_image(img)) { // coinrun get_adjusted_image_rect (coinrun.cpp:64-70)
                                rx = rx + rw * 0.0;
                                ry = ry + rh * -.7415;
                                rw = rw * 1.0;
                                rh = rh * 1.7415;
                            }
                            int4 sp = reinterpret_cast<const int4 *>(d.sprites)[img + theme * MAX_ASSETS];
                            if (axis_setup(rx, rw, sp.y, ex) && axis_setup(ry, rh, sp.z, ey)) {
                                draw = true;
                                soff = sp.x;
                                sw = sp.y;
                                ca = alpha != 1 ? qt_int_opacity((double)alpha) : 256;
                                mir = (flags & EF_REFLECTED) != 0;
                            }
                        }
                    }
                }
            }
            // Stamp in list order, EG entities per group: the texel of this lane's footprint
            // pixel is loaded for every entity of the group first (loads are order-free), then
            // the group is blended into the framebuffer strictly in order.  Footprints wider
            // than one wave (> 64 px) fall back to an in-order loop with inline loads.
            const float inv_l = 1.0f / (float)(draw ? ex.n : 1);
            unsigned long long m = ballot(draw && ez == z);
            while (m) {
                int js[EG];
#pragma unroll
                for (int g = 0; g < EG; g++) {
                    js[g] = m ? __ffsll((long long)m) - 1 : -1;
                    if (m) m &= m - 1;
                }
                uint32_t tv[EG];
                int fo[EG];
                bool on[EG];
#pragma unroll
                for (int g = 0; g < EG; g++) {
                    on[g] = false;
                    tv[g] = 0;
                    fo[g] = 0;
                    const int j = js[g];
                    if (j < 0) continue;
                    const int nx = readlane(ex.n, j), ny = readlane(ey.n, j);
                    if (nx * ny > 64) continue;
                    const int p = lane;
                    if (p < nx * ny) {
                        const float inv = __builtin_bit_cast(float, readlane(__builtin_bit_cast(int, inv_l), j));
                        const int py = (int)(((float)p + 0.5f) * inv);
                        const int pxx = p - py * nx;
                        const uint32_t bxj = (uint32_t)readlane((int)ex.base, j), byj = (uint32_t)readlane((int)ey.base, j);
                        const int sxj = readlane(ex.step, j), syj = readlane(ey.step, j);
                        const int swj = readlane(sw, j);
                        int scol = (int)((bxj + (uint32_t)(pxx * sxj)) >> 16);
                        const int srow = (int)((byj + (uint32_t)(py * syj)) >> 16);
                        if (readlane(mir, j)) scol = swj - 1 - scol;
                        tv[g] = d.pixels[(uint32_t)readlane(soff, j) + (uint32_t)(srow * swj + scol)];
                        fo[g] = (readlane(ey.t1, j) + py) * PG_RES + readlane(ex.t1, j) + pxx;
                        on[g] = true;
                    }
                }
#pragma unroll
                for (int g = 0; g < EG; g++) {
                    const int j = js[g];
                    if (j < 0) continue;
                    const int nx = readlane(ex.n, j), ny = readlane(ey.n, j);
                    const int caj = readlane(ca, j);
                    if (nx * ny <= 64) {
                        if (on[g]) fb[fo[g]] = blend_argb_pm(fb[fo[g]], tv[g], caj);
                    } else {
                        const int tx = readlane(ex.t1, j), ty = readlane(ey.t1, j);
                        const uint32_t bxj = (uint32_t)readlane((int)ex.base, j), byj = (uint32_t)readlane((int)ey.base, j);
                        const int sxj = readlane(ex.step, j), syj = readlane(ey.step, j);
                        const uint32_t offj = (uint32_t)readlane(soff, j);
                        const int swj = readlane(sw, j), mirj = readlane(mir, j);
                        const float inv = 1.0f / (float)nx;
                        for (int p = lane; p < nx * ny; p += 64) {
                            int py = (int)(((float)p + 0.5f) * inv);
                            int pxx = p - py * nx;
                            int scol = (int)((bxj + (uint32_t)(pxx * sxj)) >> 16);
                            int srow = (int)((byj + (uint32_t)(py * syj)) >> 16);
                            if (mirj) scol = swj - 1 - scol;
                            uint32_t src = d.pixels[offj + (uint32_t)(srow * swj + scol)];
                            int o = (ty + py) * PG_RES + tx + pxx;
                            fb[o] = blend_argb_pm(fb[o], src, caj);
                        }
                    }
                    // no barrier between entities: one wave issues its LDS operations in order
                }
            }
        }
    }
    wave_sync();

    pt.mark(2);
    // ---- bgr32_to_rgb888 (game.cpp:8-23): lane writes 4 pixels = 12 bytes per iteration
    uint8_t *out = d.rgb + (size_t)env * PG_OBS_BYTES;
    for (int q = lane; q < PG_RES * PG_RES / 4; q += 64) {
        uint4 p4 = reinterpret_cast<const uint4 *>(fb)[q];
        // bytes r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
        uint32_t w0 = ((p4.x >> 16) & 0xff) | (p4.x & 0xff00) | ((p4.x & 0xff) << 16) | (((p4.y >> 16) & 0xff) << 24);
        uint32_t w1 = ((p4.y >> 8) & 0xff) | ((p4.y & 0xff) << 8) | (((p4.z >> 16) & 0xff) << 16) | (((p4.z >> 8) & 0xff) << 24);
        uint32_t w2 = (p4.z & 0xff) | (((p4.w >> 16) & 0xff) << 8) | (((p4.w >> 8) & 0xff) << 16) | ((p4.w & 0xff) << 24);
        uint32_t *o = reinterpret_cast<uint32_t *>(out + (size_t)q * 12);
        o[0] = w0;
        o[1] = w1;
        o[2] = w2;
    }
    if (ballot(err) && lane == 0) atomicOr(d.error_any, 1 << PG_ERR_BAD_OPTION);
    pt.mark(3);
    pt.flush(d.prof ? d.prof + (size_t)env * 16 + 8 : nullptr);
}

extern "C" void pg_launch_render(const PGDev *d, hipStream_t s) {
    hipLaunchKernelGGL(pg_render_kernel, dim3(d->num_envs), dim3(64), 0, s, *d);
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
