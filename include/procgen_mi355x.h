/*
 * procgen_mi355x.h -- extensions of libprocgen_mi355x.so beyond the libenv ABI.
 *
 * Like the reference (vecgame.cpp:144-153 global_init -> images_load, resources.cpp:20-30),
 * libenv_make loads the sprite atlas itself: from the `resource_root` option when given, else
 * from the package's assets directory (Qt-decoded .npz packs + manifest.txt, see
 * csrc/pg_assets.cpp).  The library keeps every env's state resident in HBM and can hand out
 * device pointers so a consumer on the same GPU never copies observations to the host.
 *
 * Call order for a libenv host (gym3 CEnv, unchanged):  libenv_make ->
 *   libenv_get_tensortypes x3 -> libenv_set_buffers -> (libenv_act, libenv_observe)* -> libenv_close.
 * Device-resident order:  libenv_make -> procgen_start ->
 *   (procgen_act_device | procgen_act_hashed, procgen_wait)* -> libenv_close.
 * procgen_upload_atlas optionally replaces the loaded atlas before the first reset.
 */
#pragma once
#include <stdint.h>
#include "libenv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* atlas image descriptor: pixels[offset .. offset + w*h) row-major 0xAARRGGBB */
struct pg_image {
    uint32_t offset;
    int32_t w, h;
    int32_t pad;
};

/* Device pointers of the observation / reward / info tensors (row = env). */
struct pg_device_buffers {
    uint8_t *rgb;                /* [num_envs][64][64][3] */
    float *rew;                  /* [num_envs] */
    uint8_t *first;              /* [num_envs] */
    int32_t *prev_level_seed;    /* [num_envs] */
    uint8_t *prev_level_complete;/* [num_envs] */
    int32_t *level_seed;         /* [num_envs] */
    int32_t *actions;            /* [num_envs] action staging buffer read by the step kernel */
    void *stream;                /* hipStream_t every kernel of this env is enqueued on */
};

#define PG_NUM_GAMES 16   /* game id = index in procgen/env.py:15-32 (bigfish 0 ... starpilot 15) */
#define PG_NUM_SLOTS 1000 /* image slot = type + 100 * theme (basic-abstract-game.cpp:896) */
#define PG_MAX_BG 64

/* Replace the decoded sprite atlas (reference: images_load + each game's asset_for_type and
 * background group, resources.cpp:20-30, 837-979).  One pixel array for all games; per-game
 * tables indexed by game id: sprites [PG_NUM_GAMES][PG_NUM_SLOTS], backgrounds
 * [PG_NUM_GAMES][PG_MAX_BG], num_backgrounds [PG_NUM_GAMES], num_themes [PG_NUM_GAMES][100].
 * Only the games of the batch need to be filled.  Returns 0 on success. */
LIBENV_API int procgen_upload_atlas(libenv_env *env, const uint32_t *pixels, int64_t num_pixels,
                                    const struct pg_image *sprites, const struct pg_image *backgrounds,
                                    const int32_t *num_backgrounds, const int32_t *num_themes);
/* Initial reset + render of every env (what libenv_set_buffers triggers). */
LIBENV_API int procgen_start(libenv_env *env);
/* Step with actions already on the device (d_actions: int32[num_envs]); asynchronous. */
LIBENV_API int procgen_act_device(libenv_env *env, const int32_t *d_actions);
/* Step with actions generated on the device: a = splitmix64(seed ^ ((u64)global_env << 32) ^ t) % num_actions. */
LIBENV_API int procgen_act_hashed(libenv_env *env, uint64_t seed, int32_t t);
/* Block until every enqueued step finished (the device half of libenv_observe). */
LIBENV_API int procgen_wait(libenv_env *env);
LIBENV_API int procgen_device_buffers(libenv_env *env, struct pg_device_buffers *out);
/* Render the following steps into d_rgb (device memory of the env's GPU, uint8
 * [num_envs][64][64][3], owned by the caller) instead of the library's observation tensor; NULL
 * switches back.  Takes effect for steps enqueued after the call (the target is captured at
 * launch), so a consumer can alternate two buffers and read / all-gather step t's observations
 * while step t+1 renders (procgen_amd/gather.py).  Every step rewrites every env's frame.
 * The library keeps the raw pointer: the caller must switch back (NULL) before freeing d_rgb.
 * set_state / procgen_set_snapshot / procgen_set_latent_state re-render every env into the bound
 * buffer on the env's stream: a caller still reading it on another stream orders that first
 * (ObsGather.sync_engine). */
LIBENV_API int procgen_set_obs_buffer(libenv_env *env, void *d_rgb);
/* The shard plan libenv_make builds a vec env from (host only, no GPU; vecgame.cpp:349-362, 357-358):
 * for `num_envs` envs at global env index `env_offset` of the comma list `env_names`, local env e's
 * game id (game_of[e], procgen/env.py:15-32 order), the seed of its level-seed generator
 * (lsg_seed[e]: the (env_offset + e)-th draw of mt19937(rand_seed)) and, for a mixed batch, the
 * per-game local env lists (lists[k * num_envs / G + q]: game k owns the envs whose global index is
 * k mod G).  Any output may be NULL.  Returns G (the number of names) or -1.  A shard at
 * env_offset = r * E of N ranks reproduces rows [r * E, (r + 1) * E) of the unsharded plan. */
LIBENV_API int procgen_shard_plan(const char *env_names, int num_envs, int env_offset, int rand_seed, int32_t *game_of,
                                  uint32_t *lsg_seed, int32_t *lists);
/* Copy the outputs of `count` envs (ids env_ids[k]) to host arrays of `count` rows after the
 * enqueued steps finish; any pointer may be NULL.  For consumers (and tests) that sample a few
 * envs of a device-resident batch without copying the whole observation tensor. */
/* The outputs of EVERY env after the enqueued steps finish, for parity checks of whole populations
 * (tests/test_gpu_population.py): obs_digest[e] = sum over k < 1536 of w_k * x_k mod 2^64, x_k the
 * k-th little-endian 64-bit word of env e's 64x64x3 observation and w_k = splitmix64(k) | 1 (the
 * splitmix64 of procgen_act_hashed), computed on the device; the scalar outputs are copied whole.
 * Host arrays of num_envs entries; any may be NULL.  Returns 0 on success. */
LIBENV_API int procgen_read_outputs(libenv_env *env, uint64_t *obs_digest, float *rew, uint8_t *first,
                                    int32_t *prev_level_seed, uint8_t *prev_level_complete, int32_t *level_seed);
LIBENV_API int procgen_read_envs(libenv_env *env, const int32_t *env_ids, int count, uint8_t *rgb, float *rew,
                                 uint8_t *first, int32_t *prev_level_seed, uint8_t *prev_level_complete,
                                 int32_t *level_seed);
/* Build the atlas libenv_make would load for `env_name` (comma list) from `resource_root` (NULL or
 * "" = the package's assets directory) on the host only: returns the pixel count (copied into
 * `pixels` when capacity allows) and fills the tables (layouts as procgen_upload_atlas); < 0 on
 * error (message via procgen_error_string(NULL)).  Lets a CPU test check the loader. */
LIBENV_API int64_t procgen_atlas_host(const char *env_name, const char *resource_root, uint32_t *pixels,
                                      int64_t capacity, struct pg_image *sprites, struct pg_image *backgrounds,
                                      int32_t *num_backgrounds, int32_t *num_themes);
/* This build's own per-env snapshot (PGEnv + entity planes + grid + both generators): exact for
 * every state the engine can hold, including ones the upstream format cannot carry (an erased
 * agent).  libenv's get_state / set_state use the upstream byte format (pg_state.cpp). */
LIBENV_API int procgen_get_snapshot(libenv_env *env, int env_idx, char *data, int length);
LIBENV_API void procgen_set_snapshot(libenv_env *env, int env_idx, const char *data, int length);

/* Pinning helper: RandGen::serialize's text (randgen.cpp:100-106) of 624 MT words + position. */
LIBENV_API int procgen_mt_text(const uint32_t *words, int pos, char *out, int length);

/* MinerGame::game_set_state (reference games/miner.cpp:423-449, exposed by the fork's JS binding as
 * setState, cheerpgame.cpp:54-56): grid values (grid_width x grid_height, row-major, a DEAD_PLAYER
 * cell sets `died`), agent and exit cell positions (+ .5); the frame is re-rendered.  0 ok, < 0 error. */
LIBENV_API int procgen_set_latent_state(libenv_env *env, int env_idx, const int32_t *grid, int grid_width,
                                        int grid_height, int agent_x, int agent_y, int exit_x, int exit_y);

/* Sticky error: 0 ok; otherwise a code (see PG_ERR_*), message via procgen_error_string. */
LIBENV_API int procgen_last_error(libenv_env *env);
LIBENV_API const char *procgen_error_string(libenv_env *env);
/* Per-kernel timing of the last `n` steps measured with HIP events on the env's stream:
 * out[0] = step kernel ms, out[1] = reset kernel ms, out[2] = render kernel ms (averages; a
 * single game split into parts reports the mean launch over one part's envs), out[3] = the act's
 * wall span, then 3 per game. */
LIBENV_API int procgen_kernel_times(libenv_env *env, float *out, int n);
/* Chains one single-game act is split into (env option PROCGEN_MI355X_PARTS, contiguous env
 * ranges, each step -> reset -> render chain on its own stream); 1 for mixed batches. */
LIBENV_API int procgen_num_parts(libenv_env *env);
LIBENV_API int procgen_set_timing(libenv_env *env, int enabled);
/* Diagnostic builds only (libprocgen_mi355x_prof.so): per-phase cycle sums, out[16]. */
LIBENV_API int procgen_profile_read(libenv_env *env, uint64_t *out);
/* Diagnostic builds: the raw per-env buffer behind procgen_profile_read, uint64 [num_envs][16]
 * (PG_CENSUS builds: per launch, words 0-2 / 8-10 = the step / render wave's start and end on the
 * 100 MHz clock and its HW_ID | XCC_ID << 32). */
LIBENV_API int procgen_profile_raw(libenv_env *env, uint64_t *out);
/* Self-test of libm-dependent device arithmetic on device buffers (tests/test_gpu_libm.py):
 * which = 0: bigfish fish radius 1.75 * pow(u, 1.4) + .25 (bigfish.cpp:84) for n floats u (float out);
 * 1: QTransform::rotate matrix of an entity rotation (4 doubles out); 2: face_direction rotation of
 * n (dx, dy) pairs (float out). */
LIBENV_API int procgen_selftest_libm(int which, const float *d_in, void *d_out, int64_t n, void *stream);
/* Debug read-back of one env's scalar state, see pg_engine.h PGEnv (returns bytes copied). */
LIBENV_API int procgen_debug_env(libenv_env *env, int env_idx, void *out, int length);

#define PG_ERR_NONE 0
#define PG_ERR_ENTITY_OVERFLOW 1
#define PG_ERR_BAD_OPTION 2
#define PG_ERR_NO_ATLAS 3
#define PG_ERR_HIP 4
#define PG_ERR_GRID 5
#define PG_ERR_ASSETGEN 6 /* use_generated_assets: the device painter met a path it does not restate */
#define PG_ERR_RENDER 7   /* a draw referenced pixels outside the atlas or a case the renderer lacks */

#ifdef __cplusplus
}
#endif
