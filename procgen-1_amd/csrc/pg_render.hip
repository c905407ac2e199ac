// pg_render.hip -- Game::observe: 64x64 render + bgr32_to_rgb888 (reference game.cpp:8-23,
// 97-107, 173-191; basic-abstract-game.cpp:808-1075; games/coinrun.cpp:64-70, 133-138, 213-225).
//
// One wavefront per env, a 16 KB RGB32 framebuffer in LDS.  The painter's algorithm of
// the reference is kept exactly, but each layer is rasterised the way the GPU likes:
//   * background + grid tiles: pixel-centric -- lane = screen column, loop over rows; a
//     pixel blends every tile covering it (<= 2 columns x 2 rows because of RENDER_EPS
//     overlap) in the reference's x-major / y-minor draw order;
//   * entities: sprite-centric -- one entity at a time in list order, lanes = the
//     entity's footprint pixels.
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

// One axis of qt_blit_setup (the x and y halves are independent).
struct Axis {
    int t1, n;       // first device pixel, pixel count (after clip and bound checks)
    uint32_t base;   // fixed-point source coordinate of pixel t1
    int step;
};

DEV bool axis_setup(double r, double rw, int iw, Axis &a) {
    if (!(rw > 0) || iw <= 0) return false;
    double t_w = (r + rw) - r;
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

// image_for_type (coinrun.cpp:213-225, basic-abstract-game.cpp:446-448)
DEV int image_for_type(const PGEnv &s, float agent_vx, int type) {
    if (type == PLAYER) {
        if (fabs((double)agent_vx) < .01 && s.action_vx == 0 && s.has_support) return PLAYER;
        return (s.cur_time / 5 % 2 == 0 || !s.has_support) ? CR_PLAYER_RIGHT1 : CR_PLAYER_RIGHT2;
    } else if (type == CR_ENEMY_BARRIER) {
        return -1;
    }
    return type < 0 ? -type : type;
}
DEV bool is_player_image(int t) {
    return t == PLAYER || t == CR_PLAYER_JUMP || t == CR_PLAYER_RIGHT1 || t == CR_PLAYER_RIGHT2;
}

DEV int4 sprite_of(const PGDev &d, int slot) {
    return reinterpret_cast<const int4 *>(d.sprites)[slot];
}

} // namespace

extern "C" __global__ __launch_bounds__(64) void pg_render_kernel(PGDev d) {
    __shared__ __attribute__((aligned(16))) uint32_t fb[PG_RES * PG_RES];
    const int env = blockIdx.x;
    const PGEnv s = d.envs[env];
    const int16_t *G = d.grid + (size_t)env * PG_GRID_MAX;
    int err = 0;

    float agent_x, agent_y, agent_vx;
    if (s.agent_erased) {
        agent_x = s.ghost_x; agent_y = s.ghost_y; agent_vx = s.ghost_vx;
    } else {
        agent_x = EFr(d, F_X, env, 0); agent_y = EFr(d, F_Y, env, 0); agent_vx = EFr(d, F_VX, env, 0);
    }

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

    const int col = LANE;

    // ---- draw_background (basic-abstract-game.cpp:988-1016): black fill + one scaled blit
    Axis bx, by;
    bool bg_ok = false;
    int4 bgi = make_int4(0, 0, 0, 0);
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
        double rx = mx + mw * ax, ry = my + mh * 0.0, rw = mw * aw, rh = mh * 1.0;
        bg_ok = axis_setup(rx, rw, bgi.y, bx) && axis_setup(ry, rh, bgi.z, by);
    }
    bool bg_col = bg_ok && col >= bx.t1 && col < bx.t1 + bx.n;
    int bg_scol = bg_col ? (int)((bx.base + (uint32_t)((col - bx.t1) * bx.step)) >> 16) : 0;

    // ---- grid tile columns covering this lane's screen column
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
    const float tile_eps = RENDER_EPS;
    // candidate tile columns: the one under the pixel and its neighbours; keep those whose
    // Qt pixel span (for the 128-px tile images used by every coinrun grid type) covers col
    int cand_x[2];
    Axis cand_ax[2];
    int ncx = 0;
    int iw_cached = 128;
    {
        int xg = (int)floorf(((float)col + 0.5f + v.x_off) / v.unit);
        for (int x = xg - 2; x <= xg + 2; x++) {
            if (x < low_x || x > high_x || ncx == 2) continue;
            double rx, ry, rw, rh;
            screen_rect(v, (float)x, 0.0f, 1, 1, tile_eps, rx, ry, rw, rh);
            Axis a;
            if (axis_setup(rx, rw, iw_cached, a) && col >= a.t1 && col < a.t1 + a.n) {
                cand_x[ncx] = x;
                cand_ax[ncx] = a;
                ncx++;
            }
        }
    }

    // ---- pixel-centric background + tiles, row by row (row-uniform tile rows)
    for (int row = 0; row < PG_RES; row++) {
        uint32_t px = 0xff000000u;
        if (bg_col && row >= by.t1 && row < by.t1 + by.n) {
            int srow = (int)((by.base + (uint32_t)((row - by.t1) * by.step)) >> 16);
            px = d.pixels[(uint32_t)bgi.x + (uint32_t)(srow * bgi.y + bg_scol)];
        }
        // tile rows covering this row (uniform): draw order is y ascending
        int yg = (int)floorf((v.view_dim - ((float)row + 0.5f - v.y_off) / v.unit));
        int cand_y[2];
        Axis cand_ay[2];
        int ncy = 0;
        for (int y = yg - 2; y <= yg + 2; y++) {
            if (y < low_y || y > high_y || ncy == 2) continue;
            double rx, ry, rw, rh;
            screen_rect(v, 0.0f, (float)(y + 1), 1, 1, tile_eps, rx, ry, rw, rh);
            Axis a;
            if (axis_setup(ry, rh, 128, a) && row >= a.t1 && row < a.t1 + a.n) {
                cand_y[ncy] = y;
                cand_ay[ncy] = a;
                ncy++;
            }
        }
        for (int k = 0; k < ncx; k++) {
            for (int l = 0; l < ncy; l++) {
                int x = cand_x[k], y = cand_y[l];
                int type;
                if (!(0 <= y && y < s.main_height && 0 <= x && x < s.main_width)) type = s.out_of_bounds_object;
                else type = G[y * s.main_width + x];
                if (type == INVALID_OBJ) continue;
                int theme = cr_is_wall(type) ? s.wall_theme : 0; // theme_for_grid_obj (coinrun.cpp:133-138)
                int img = image_for_type(s, agent_vx, type);
                if (img < 0) continue;
                if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) {
                    if (img != SPACE) err = PG_ERR_BAD_OPTION; // draw_grid_obj fills: not in this build
                    continue;
                }
                if (s.opt_restrict_themes) theme = 0;
                int4 sp = sprite_of(d, img + theme * MAX_ASSETS);
                if (sp.y != iw_cached || sp.z != 128) { err = PG_ERR_NO_ATLAS; continue; }
                const Axis &ax = cand_ax[k];
                const Axis &ay = cand_ay[l];
                int scol = (int)((ax.base + (uint32_t)((col - ax.t1) * ax.step)) >> 16);
                int srow = (int)((ay.base + (uint32_t)((row - ay.t1) * ay.step)) >> 16);
                uint32_t src = d.pixels[(uint32_t)sp.x + (uint32_t)(srow * sp.y + scol)];
                px = src + BYTE_MUL(px, (~src) >> 24);
            }
        }
        fb[row * PG_RES + col] = px;
    }
    wave_sync();

    // ---- entities, render_z 0 then 1, in list order (basic-abstract-game.cpp:966-967, 1061-1075)
    const int n = s.num_ents;
    for (int z = 0; z <= 1; z++) {
        for (int base = 0; base < n; base += 64) {
            int i = base + LANE;
            unsigned long long m = ballot(i < n && EIr(d, F_RENDER_Z, env, i) == z);
            while (m) {
                int e = base + __ffsll((long long)m) - 1;
                m &= m - 1;
                float ex = EFr(d, F_X, env, e), ey = EFr(d, F_Y, env, e);
                float erx = EFr(d, F_RX, env, e), ery = EFr(d, F_RY, env, e);
                int flags = EIr(d, F_FLAGS, env, e);
                float alpha = EFr(d, F_ALPHA, env, e);
                float rotation = EFr(d, F_ROTATION, env, e);
                int itype = EIr(d, F_IMAGE_TYPE, env, e);
                int theme = EIr(d, F_IMAGE_THEME, env, e);
                if (flags & EF_ABS_COORDS) { err = PG_ERR_BAD_OPTION; continue; }
                double rx, ry, rw, rh;
                screen_rect(v, ex - erx, ey + ery, 2 * erx, 2 * ery, 0, rx, ry, rw, rh);
                int img = image_for_type(s, agent_vx, itype);
                if (img < 0) continue;
                if (s.opt_use_monochrome_assets || img >= USE_ASSET_THRESHOLD) {
                    if (img != SPACE) err = PG_ERR_BAD_OPTION;
                    continue;
                }
                if (rotation != 0) { err = PG_ERR_BAD_OPTION; continue; }
                if (s.opt_restrict_themes) theme = 0;
                if (is_player_image(img)) { // coinrun get_adjusted_image_rect: adjust_rect(r, (0, -.7415, 1, 1.7415))
                    rx = rx + rw * 0.0;
                    ry = ry + rh * -.7415;
                    rw = rw * 1.0;
                    rh = rh * 1.7415;
                }
                int4 sp = sprite_of(d, img + theme * MAX_ASSETS);
                Axis ax, ay;
                if (!(axis_setup(rx, rw, sp.y, ax) && axis_setup(ry, rh, sp.z, ay))) continue;
                int ca = alpha != 1 ? qt_int_opacity((double)alpha) : 256;
                bool mir = (flags & EF_REFLECTED) != 0;
                int npx = ax.n * ay.n;
                for (int p = LANE; p < npx; p += 64) {
                    int py = p / ax.n, pxx = p - py * ax.n;
                    int scol = (int)((ax.base + (uint32_t)(pxx * ax.step)) >> 16);
                    int srow = (int)((ay.base + (uint32_t)(py * ay.step)) >> 16);
                    if (mir) scol = sp.y - 1 - scol;
                    uint32_t src = d.pixels[(uint32_t)sp.x + (uint32_t)(srow * sp.y + scol)];
                    int o = (ay.t1 + py) * PG_RES + ax.t1 + pxx;
                    fb[o] = blend_argb_pm(fb[o], src, ca);
                }
                wave_sync();
            }
        }
    }
    wave_sync();

    // ---- bgr32_to_rgb888 (game.cpp:8-23): 768 x 16-byte chunks per env
    uint8_t *out = d.rgb + (size_t)env * PG_OBS_BYTES;
    for (int ch = LANE; ch < PG_OBS_BYTES / 16; ch += 64) {
        uint32_t w4[4];
        int b0 = ch * 16;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t word = 0;
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                int byte = b0 + q * 4 + bb;
                int p = byte / 3, c3 = byte - p * 3;
                uint32_t pxv = fb[p];
                uint32_t v8 = c3 == 0 ? (pxv >> 16) & 0xff : (c3 == 1 ? (pxv >> 8) & 0xff : pxv & 0xff);
                word |= v8 << (8 * bb);
            }
            w4[q] = word;
        }
        reinterpret_cast<uint4 *>(out)[ch] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    if (err) {
        if (LANE == 0) atomicOr(d.error_any, 1 << err);
    }
}

extern "C" void pg_launch_render(const PGDev *d, hipStream_t s) {
    hipLaunchKernelGGL(pg_render_kernel, dim3(d->num_envs), dim3(64), 0, s, *d);
}
