/*
 * libenv.h -- the libenv C ABI that the reference's vectorised env exports, as
 * implemented by libprocgen_mi355x.so.
 *
 * gym3's libenv.h is not part of the reference tree (gym3 is a pip dependency of
 * procgen/env.py:5-7, not installed here), so the layouts below are reconstructed
 * from the reference's own uses of it:
 *   - enum libenv_dtype / struct libenv_option / struct libenv_options:
 *       procgen/src/vecoptions.h:15-41 (LIBENV_MAX_NAME_LEN, dtype values)
 *   - struct libenv_tensortype (name, scalar_type, dtype, shape, ndim, low, high):
 *       procgen/src/vecgame.cpp:212-330
 *   - struct libenv_buffers (ob, ac, info pointer arrays indexed
 *       space_idx * num_envs + env_idx; rew; first): procgen/src/vecgame.cpp:30-40, 74-83
 * Every entry point below replaces the reference function cited next to it.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LIBENV_API __attribute__((visibility("default")))
#define LIBENV_VERSION 1
#define LIBENV_MAX_NAME_LEN 128
#define LIBENV_MAX_NDIM 16

enum libenv_dtype {
    LIBENV_DTYPE_UNUSED = 0,
    LIBENV_DTYPE_UINT8 = 1,
    LIBENV_DTYPE_INT32 = 2,
    LIBENV_DTYPE_FLOAT32 = 3,
};

enum libenv_scalar_type {
    LIBENV_SCALAR_TYPE_UNUSED = 0,
    LIBENV_SCALAR_TYPE_REAL = 1,
    LIBENV_SCALAR_TYPE_DISCRETE = 2,
};

enum libenv_space_name {
    LIBENV_SPACE_UNUSED = 0,
    LIBENV_SPACE_OBSERVATION = 1,
    LIBENV_SPACE_ACTION = 2,
    LIBENV_SPACE_INFO = 3,
};

union libenv_value {
    uint8_t uint8;
    int32_t int32;
    float float32;
};

struct libenv_tensortype {
    char name[LIBENV_MAX_NAME_LEN];
    enum libenv_scalar_type scalar_type;
    enum libenv_dtype dtype;
    int shape[LIBENV_MAX_NDIM];
    int ndim;
    union libenv_value low;
    union libenv_value high;
};

struct libenv_option {
    char name[LIBENV_MAX_NAME_LEN];
    enum libenv_dtype dtype;
    int count;
    void *data;
};

struct libenv_options {
    struct libenv_option *items;
    int count;
};

struct libenv_buffers {
    void **ob;    /* [num_ob_spaces * num_envs] */
    void **ac;    /* [num_ac_spaces * num_envs] */
    void **info;  /* [num_info_spaces * num_envs] */
    float *rew;   /* [num_envs] */
    uint8_t *first; /* [num_envs] */
};

typedef void libenv_env;

/* vecgame.cpp:43-45 */
LIBENV_API int libenv_version(void);
/* vecgame.cpp:47-50.  Options: vecgame.cpp:183-190 (env_name, num_levels, start_level,
 * num_actions, rand_seed, num_threads, resource_root, render_human) and game.cpp:62-95
 * (paint_vel_info, use_generated_assets, use_monochrome_assets, restrict_themes,
 * use_backgrounds, center_agent, use_sequential_levels, distribution_mode, debug_mode,
 * use_easy_jump, plain_assets, physics_mode, game_type).  Unknown option => NULL
 * (the reference exits; see procgen_last_error()). */
LIBENV_API libenv_env *libenv_make(int num_envs, const struct libenv_options options);
/* vecgame.cpp:52-72 */
LIBENV_API int libenv_get_tensortypes(libenv_env *env, enum libenv_space_name name, struct libenv_tensortype *out_types);
/* vecgame.cpp:74-83 + 381-409: keeps the pointers and runs the initial reset + observe */
LIBENV_API void libenv_set_buffers(libenv_env *env, struct libenv_buffers *bufs);
/* vecgame.cpp:85-88 + 411-424: blocks until the last act() finished, fills host buffers */
LIBENV_API void libenv_observe(libenv_env *env);
/* vecgame.cpp:90-93 + 426-449: reads actions, enqueues the step, returns immediately */
LIBENV_API void libenv_act(libenv_env *env);
/* vecgame.cpp:95-98 */
LIBENV_API void libenv_close(libenv_env *env);
/* vecgame.cpp:485-505: per-env state in upstream procgen's serialize format (game.cpp:196-255,
 * basic-abstract-game.cpp:1178-1225, games/*.cpp, END_OF_BUFFER; pg_state.cpp) -- the fork's own
 * buffer writes are stubs, so the byte layout is parity unpinned beyond the RandGen text.
 * get_state returns bytes written, -1 if length is too small; set_state of a malformed or
 * out-of-range state sets a sticky error (procgen_last_error) instead of the reference's fassert.
 * This build's exact own format is procgen_get/set_snapshot (procgen_mi355x.h). */
LIBENV_API int get_state(libenv_env *env, int env_idx, char *data, int length);
LIBENV_API void set_state(libenv_env *env, int env_idx, char *data, int length);

#ifdef __cplusplus
}
#endif
