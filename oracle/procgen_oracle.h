/*
 * procgen_oracle.h -- CPU restatement of the reference step path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity CHECKER for the MI355X engine.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is
 * never linked into, called by, or used as a fallback for the product path
 * (procgen-1_amd/).
 *
 * Parity status (see DESIGN.md "Oracle"): the reference game sources cannot be
 * built here (they include <cheerp/client.h>, absent from the image), so this is
 * a restatement.  Pinned pieces:
 *   - MT19937 / RandGen draws: against reference randgen.cpp compiled from
 *     /root/reference (oracle/_ref) and the C++-standard known answer;
 *   - Entity::step: against reference entity.cpp compiled from /root/reference;
 *   - Qt raster compositing: against the real Qt 5.9.7 raster engine
 *     (tools/qt_raster_golden.cpp -> tests/golden/qt_raster_*.npz);
 *   - asset pixels: decoded by Qt itself (tools/make_asset_pack.py).
 * Game logic (coinrun.cpp, basic-abstract-game.cpp, game.cpp) is a line-by-line
 * restatement with no reference-side golden: "parity unpinned" for that layer.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* atlas image descriptor (same layout as pg_image in include/procgen_mi355x.h) */
typedef struct {
    uint32_t offset; /* first pixel in the pixel array */
    int32_t w, h;    /* 0x0 = no image */
    int32_t pad;
} or_image;

typedef struct {
    const uint32_t *pixels;     /* 0xAARRGGBB */
    const or_image *sprites;    /* [1000]: slot = type + 100 * theme (ARGB32 premultiplied) */
    const or_image *backgrounds;/* [num_backgrounds] (RGB32) */
    int32_t num_backgrounds;
    const int32_t *num_themes;  /* [100] asset_num_themes per type */
} or_atlas;

typedef struct {
    int32_t num_levels, start_level, rand_seed;
    int32_t distribution_mode;
    int32_t center_agent, use_backgrounds, restrict_themes, use_sequential_levels;
    int32_t use_monochrome_assets, paint_vel_info, debug_mode;
    int32_t use_generated_assets; /* AssetGen sprites + per-env procedural backgrounds */
} or_options;

/* Create `count` envs of game `env_name` whose GLOBAL indices are
 * env_offset .. env_offset+count-1 (level-seed generator seeded with the
 * global index's draw of rand_seed's MT, reference vecgame.cpp:349-362).
 * The atlas memory must outlive the handle. Returns NULL on bad options. */
void *oracle_make(const char *env_name, int count, int env_offset, const or_options *opt,
                  const or_atlas *atlas);
/* The same for global indices env_offset + n * stride (one game's envs of a mixed batch, which plays
 * name n % #names at env n, vecgame.cpp:357-358). */
void *oracle_make_strided(const char *env_name, int count, int env_offset, int stride, const or_options *opt,
                          const or_atlas *atlas);
void oracle_close(void *h);
/* initial reset + observe (reference vecgame.cpp:126-131) */
void oracle_start(void *h);
/* one libenv act: per-env action, step, auto-reset, observe */
void oracle_step(void *h, const int32_t *actions);
/* copy the last observation set out (any pointer may be NULL) */
void oracle_observe(void *h, uint8_t *rgb, float *rew, uint8_t *first,
                    int32_t *prev_level_seed, uint8_t *prev_level_complete, int32_t *level_seed);
/* fork latent-state info per env: grid_size[2], grid[35*35], agent_pos[2], exit_pos[2] */
void oracle_latent(void *h, int32_t *grid_size, int32_t *grid, int32_t *agent_pos, int32_t *exit_pos);
/* miner.cpp:423-449 game_set_state on env i, then re-render; 0 ok, -1 where the reference crashes */
int oracle_miner_set_state(void *h, int i, const int32_t *grid, int grid_width, int grid_height, int agent_x,
                           int agent_y, int exit_x, int exit_y);
/* debug: a few scalars of env i: [num_entities, cur_time, agent_x_bits, agent_y_bits,
 * background_index, wall_theme, episodes... ] (see .c) */
int oracle_debug(void *h, int i, int32_t *out, int n);
/* env i's entity list, 31 words per entity in Entity::serialize order; returns the count */
int oracle_entity_words(void *h, int i, int32_t *out, int cap);
/* AssetGen pins (assetgen.cpp + the Qt raster paths it uses) */
int oracle_qt_shape(int w, int h, int fmt, int kind, double x, double y, double rw, double rh, uint32_t c1, uint32_t c2,
                    int source, uint32_t *inout);
void oracle_qt_polyline(int w, int h, const double *pts, int n, uint32_t color, uint32_t *inout);
int oracle_generate_resource(int32_t seed, int pre_draws, int w, int h, int fmt, int num_recurse, int blotch_scale,
                             int is_rect, uint32_t init, uint32_t *out, int32_t *next);

/* ------------ pinning helpers (compared against oracle/_ref and Qt goldens) ------------ */
/* fill out[n] with successive 32-bit outputs of an MT19937 seeded with `seed` */
void oracle_mt_stream(uint32_t seed, uint32_t *out, int n);
/* run a scripted RandGen sequence: ops[i] = (kind, a, b) ; writes one i32 (or float bits) per op */
void oracle_randgen_script(uint32_t seed, const int32_t *ops, int nops, int32_t *out);
/* MazeGen (mazegen.cpp) restatement: mode 0 generate_maze, 1 no_dead_ends, 2 with_doors(num_doors),
 * then place_objects if num_objs > 0; writes the array_dim^2 grid, returns array_dim */
int oracle_mazegen(int32_t seed, int maze_dim, int mode, int num_doors, int start_obj, int num_objs, int32_t *out,
                   uint32_t *next_draw);
/* bigfish.cpp:84 fish radius 1.75 * pow(u, 1.4) + .25 with the C library's pow */
/* qt-utils.h adjust_rect / to_shade and grid.h Grid pins */
void oracle_adjust_rect(const double *base, const double *adj, double *out, int64_t n);
void oracle_to_shade(const float *f, int32_t *out, int64_t n);
int oracle_grid_ops(int w, int h, const int32_t *xy, int n, int32_t *out);
void oracle_diag_counters(long long *out, int reset);
int oracle_render_rgb_array(void *h, uint8_t *rgb, int res, double *log, int cap);
void oracle_qt_smooth(int cw, int ch, uint32_t *inout, int kind, const uint32_t *img, int iw, int ih, int fmt,
                      int mirrored, double x, double y, double w, double h, double opacity, uint32_t argb);
void oracle_qt_smooth_rot(int cw, int ch, uint32_t *inout, const uint32_t *img, int iw, int ih, int fmt, int mirrored,
                          double x, double y, double w, double h, double deg, double opacity);
void oracle_qt_prim(int cw, int ch, uint32_t *inout, int kind, double x, double y, double w, double h, uint32_t argb,
                    int penw);
void oracle_bigfish_radius(const float *u, float *out, int64_t n);
/* Qt raster replay of the tools/qt_raster_golden.cpp command format on a 64x64 RGB32 canvas */
int oracle_qt_replay(const uint8_t *cmds, int64_t nbytes, uint32_t *canvas_inout);

#ifdef __cplusplus
}
#endif
