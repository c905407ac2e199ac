// pg_capi.cpp -- the drop-in C ABI (include/libenv.h + include/procgen_mi355x.h).
//
// Host half of the reference's VecGame (procgen/src/vecgame.cpp): option parsing with the
// reference's consume-once semantics (vecoptions.cpp:47-94), tensor types
// (vecgame.cpp:212-330), level-seed derivation (vecgame.cpp:332-378), the act/observe
// hand-off (vecgame.cpp:411-449) -- with the per-env work replaced by HIP launches on one
// stream: pg_step (all envs) -> pg_reset (queued envs) -> pg_render, one launch of each per
// game of the batch (mixed batches: env n plays game n % #games, vecgame.cpp:357-358).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/libenv.h"
#include "../../include/procgen_mi355x.h"

#define PG_EV_G 7 // timing events per game and act: step start / end, reset start / end (side stream),
                  // render of the unfinished envs end, render of the finished envs start / end
#include "pg_assets.h"
#include "pg_state.h"
#include "pg_engine.h"

extern "C" {
void pg_launch_step(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s, int use_hash,
                    uint64_t seed, int32_t t, int parity, int slot);
void pg_launch_reset(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s, int mode, int grid,
                     int act, int slot);
void pg_launch_render(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s, int mode, int slot);
int pg_launch_fused(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s, int use_hash, uint64_t seed,
                    int32_t t, int parity, int slot);
int pg_launch_render_hires(const PGDev *d, int game, const int32_t *env_list, int count, uint32_t *frames, uint8_t *rgb,
                           hipStream_t s);
int pg_launch_assetgen_sprites(int game, uint32_t seed0, uint32_t *d_out, int types, hipStream_t s);
void pg_launch_poison(hipStream_t s, uint32_t pattern);

// PROCGEN_MI355X_POISON_LDS=1: scribble over LDS before every engine kernel (debug aid, see
// pg_poison_lds_kernel); off by default
static bool poison_lds() {
    static const bool on = getenv("PROCGEN_MI355X_POISON_LDS") && getenv("PROCGEN_MI355X_POISON_LDS")[0] == '1';
    return on;
}
#define PG_POISON(stream) \
    do {                  \
        if (poison_lds()) pg_launch_poison(stream, 0xFFFFFFFFu); \
    } while (0)
}

namespace {

std::string g_last_make_error;

// ------------------------------------------------------------------ host MT19937 (level seeds)
struct HostMT {
    uint32_t mt[624];
    int mti;
    void seed(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        mti = 624;
    }
    uint32_t next() {
        if (mti >= 624) {
            for (int i = 0; i < 624; i++) {
                uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            mti = 0;
        }
        uint32_t y = mt[mti++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
};

// ------------------------------------------------------------------ options (vecoptions.cpp:47-94)
struct Options {
    std::vector<libenv_option> items;
    std::string error;
    bool find(const char *name, libenv_dtype dt, libenv_option *out) {
        for (size_t i = 0; i < items.size(); i++) {
            if (strncmp(items[i].name, name, LIBENV_MAX_NAME_LEN) == 0) {
                if (items[i].dtype != dt) {
                    if (error.empty()) error = std::string("invalid dtype for option ") + name;
                    return false;
                }
                *out = items[i];
                items.erase(items.begin() + i);
                return true;
            }
        }
        return false;
    }
    void consume_string(const char *name, std::string *v) {
        libenv_option o;
        if (find(name, LIBENV_DTYPE_UINT8, &o) && o.data) *v = std::string((const char *)o.data, o.count);
    }
    void consume_int(const char *name, int32_t *v) {
        libenv_option o;
        if (find(name, LIBENV_DTYPE_INT32, &o) && o.data) *v = *(const int32_t *)o.data;
    }
    void consume_bool(const char *name, bool *v) {
        libenv_option o;
        if (find(name, LIBENV_DTYPE_UINT8, &o) && o.data) {
            uint8_t b = *(const uint8_t *)o.data;
            if (b != 0 && b != 1 && error.empty()) error = std::string("bool option not 0/1: ") + name;
            *v = b != 0;
        }
    }
};

int game_id(const std::string &name) {
    if (name == "coinrun") return PG_GAME_COINRUN;
    if (name == "bigfish") return PG_GAME_BIGFISH;
    if (name == "maze") return PG_GAME_MAZE;
    if (name == "heist") return PG_GAME_HEIST;
    if (name == "miner") return PG_GAME_MINER;
    if (name == "climber") return PG_GAME_CLIMBER;
    if (name == "leaper") return PG_GAME_LEAPER;
    if (name == "chaser") return PG_GAME_CHASER;
    if (name == "fruitbot") return PG_GAME_FRUITBOT;
    if (name == "dodgeball") return PG_GAME_DODGEBALL;
    if (name == "plunder") return PG_GAME_PLUNDER;
    if (name == "starpilot") return PG_GAME_STARPILOT;
    if (name == "bossfight") return PG_GAME_BOSSFIGHT;
    if (name == "ninja") return PG_GAME_NINJA;
    if (name == "caveflyer") return PG_GAME_CAVEFLYER;
    if (name == "jumper") return PG_GAME_JUMPER;
    return -1;
}
const char *SUPPORTED_GAMES = "bigfish, bossfight, caveflyer, chaser, climber, coinrun, dodgeball, fruitbot, heist, jumper, leaper, maze, miner, ninja, plunder, starpilot";

std::vector<std::string> split_names(const std::string &s) { // vecgame.cpp:20-28 split(",")
    std::vector<std::string> out;
    size_t p = 0;
    while (true) {
        size_t q = s.find(',', p);
        out.push_back(s.substr(p, q == std::string::npos ? std::string::npos : q - p));
        if (q == std::string::npos) break;
        p = q + 1;
    }
    return out;
}

// Game ctor (game.cpp:25-39) + BasicAbstractGame ctor (basic-abstract-game.cpp:22-46) + the
// game's own ctor
void construct_env(PGEnv &s, int gid) {
    memset(&s, 0, sizeof(s));
    s.game_id = gid;
    s.timeout = 1000;
    s.episodes_remaining = 0;
    s.last_reward = -1;
    s.reset_count = 0;
    s.current_level_seed = 0;
    s.sd_reward = 0;
    s.sd_done = 1;
    s.sd_level_complete = 0;
    s.char_dim = 5;
    s.visibility = 16;
    s.min_visibility = 0;
    s.mixrate = 0.5f;
    s.maxspeed = 0.5f;
    s.max_jump = s.maxspeed;
    s.default_action = 4;
    s.last_move_action = 7;
    s.bg_tile_ratio = 0;
    s.out_of_bounds_object = -1; // INVALID_OBJ
    s.has_useful_vel_info = 1;
    s.random_agent_start = 1;
    if (gid == PG_GAME_COINRUN) { // coinrun.cpp:49-58
        s.visibility = 13;
        s.mixrate = 0.2f;
        s.main_width = 64;
        s.main_height = 64;
        s.out_of_bounds_object = 15; // WALL_MID
    } else if (gid == PG_GAME_BIGFISH) { // bigfish.cpp:24-29
        s.timeout = 6000;
        s.main_width = 20;
        s.main_height = 20;
    } else if (gid == PG_GAME_MAZE) { // maze.cpp:20-28
        s.timeout = 500;
        s.random_agent_start = 0;
        s.has_useful_vel_info = 0;
        s.out_of_bounds_object = 51; // WALL_OBJ
        s.visibility = 8.0f;
    } else if (gid == PG_GAME_FRUITBOT) { // fruitbot.cpp:30-40
        s.mixrate = .5f;
        s.maxspeed = 0.85f;
        s.bg_tile_ratio = -1;
        s.out_of_bounds_object = 2; // OUT_OF_BOUNDS_WALL
    } else if (gid == PG_GAME_CAVEFLYER) { // caveflyer.cpp:25-29
        s.mixrate = 0.9f;
    } else if (gid == PG_GAME_NINJA) { // ninja.cpp:35-41
        s.main_width = 64;
        s.main_height = 64;
        s.out_of_bounds_object = 20; // WALL_MID
    } else if (gid == PG_GAME_BOSSFIGHT) { // bossfight.cpp:60-68
        s.timeout = 4000;
        s.main_width = 20;
        s.main_height = 20;
        s.mixrate = .5;
        s.maxspeed = 0.85f;
    } else if (gid == PG_GAME_STARPILOT) { // starpilot.cpp:50-54
        s.main_width = 16;
        s.main_height = 16;
    } else if (gid == PG_GAME_PLUNDER) { // plunder.cpp:33-43
        s.timeout = 4000;
        s.main_width = 20;
        s.main_height = 20;
        s.mixrate = .5;
        s.maxspeed = 0.85f;
        s.has_useful_vel_info = 0;
    } else if (gid == PG_GAME_DODGEBALL) { // dodgeball.cpp:37-44
        s.mixrate = .5;
        s.enemy_fire_delay = 50;
        s.out_of_bounds_object = 10; // OOB_WALL
    } else if (gid == PG_GAME_CHASER) { // chaser.cpp:37-47
        s.mixrate = 1;
        s.maxspeed = .5f;
        s.eat_timeout = 75;
        s.egg_timeout = 50;
        s.has_useful_vel_info = 0;
    } else if (gid == PG_GAME_LEAPER) { // leaper.cpp:34-38 (MAX_SPEED = 2 / (NSTEP - 1.0))
        s.maxspeed = (float)(2 / (5 - 1.0));
        s.timeout = 500;
    } else if (gid == PG_GAME_CLIMBER) { // climber.cpp:38-41
        s.out_of_bounds_object = 15; // WALL_MID
    } else if (gid == PG_GAME_MINER) { // miner.cpp:30-43
        s.main_width = 20;
        s.main_height = 20;
        s.main_area = 400;
        s.mixrate = .5f;
        s.maxspeed = .5f;
        s.has_useful_vel_info = 0;
        s.out_of_bounds_object = 10; // OOB_WALL
        s.visibility = 8.0f;
        s.diamonds_remaining = -1;
    } else if (gid == PG_GAME_HEIST) { // heist.cpp:23-35
        s.has_useful_vel_info = 0;
        s.main_width = 20;
        s.main_height = 20;
        s.out_of_bounds_object = 51; // WALL_OBJ
        s.visibility = 8.0f;
    }
}

// Rotations the games draw at (entity rotation values, radians) and the QTransform each one
// becomes: draw_image's p.rotate(rotation * 180 / PI) (basic-abstract-game.cpp:908-916) ->
// QTransform::rotate (exact special cases for +-90 / 180 / 270, otherwise qSin / qCos of
// deg2rad * a -- the C library's sin / cos, evaluated here on the host so the device matrix
// is bit-identical).  Slots (dx + 1) * 3 + (dy + 1): Entity::face_direction(dx, dy) =
// -atan2f(dy, dx) + 0 (entity.cpp:84-88, heist.cpp:208); slot 9: heist's ring keys (PI / 2,
// heist.cpp:195).
void build_rot_table(float *angles, double *table) {
    const float PI_F = 3.14159265358979323846264338327950288f;
    for (int k = 0; k < PG_ROT_N; k++) {
        uint32_t nan_bits = 0x7fc00000u + (uint32_t)k;
        memcpy(&angles[k], &nan_bits, 4); // unused slots match no entity rotation
        table[4 * k + 0] = 1; table[4 * k + 1] = 0; table[4 * k + 2] = 0; table[4 * k + 3] = 1;
    }
    for (int dx = -1; dx <= 1; dx++)
        for (int dy = -1; dy <= 1; dy++)
            if (dx != 0 || dy != 0) angles[(dx + 1) * 3 + (dy + 1)] = -1 * atan2f((float)dy, (float)dx) + 0.0f;
    angles[9] = PI_F / 2;   // heist ring keys; leaper frog (1 * PI / 2)
    angles[10] = -1 * PI_F / 2; // leaper frog facing left (-1 * PI / 2, leaper.cpp:241)
    angles[11] = PI_F;          // leaper frog facing down / cars moving left (leaper.cpp:245, 186)
    for (int k = 0; k < PG_ROT_N; k++) {
        float rot = angles[k];
        if (std::isnan(rot)) continue;
        double a = (double)(rot * 180 / PI_F);
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
            const double deg2rad = 0.017453292519943295769;
            double b = deg2rad * a;
            sina = std::sin(b);
            cosa = std::cos(b);
        }
        table[4 * k + 0] = cosa; table[4 * k + 1] = sina; table[4 * k + 2] = -sina; table[4 * k + 3] = cosa;
        // QTransform::type(): qFuzzyIsNull(m12) && qFuzzyIsNull(m21) makes it a TxScale, drawn by
        // the scale blit whose map ignores m12 / m21 (rotate(-180): sin = -1.2e-16)
        if (std::fabs(sina) <= 0.000000000001) {
            table[4 * k + 1] = 0;
            table[4 * k + 2] = 0;
        }
    }
}

struct VecEnv {
    uint64_t *d_digest = nullptr; // procgen_read_outputs' per-env observation digests (allocated on first use)
    int rf_make = 0;               // PGDev::render_rf chosen at make time
    std::vector<uint8_t> rf_bad;   // [num_envs] env holds a restored state the register-frame render cannot draw
    int rf_bad_n[PG_NUM_GAMES] = {}; // such envs per game (their game renders with the LDS-frame kernel)
    int num_envs = 0;
    int env_offset = 0;
    int num_actions = 15;
    bool render_human = false; // render_mode="rgb_array": info["rgb"] at RENDER_RES (vecgame.cpp:318-330, 415-423)
    uint32_t *hr_frames = nullptr; // [num_envs][512 * 512] RGB32 frames of the antialiased render
    uint8_t *hr_rgb = nullptr;     // [num_envs][512 * 512 * 3] their bgr32_to_rgb888
    size_t hr_info = 0;            // index of the "rgb" info tensor
    PGDev dev{};
    hipStream_t stream = nullptr;
    std::vector<libenv_tensortype> ob_types, ac_types, info_types;
    // host buffers from libenv_set_buffers (per env pointers, reference convert_bufs layout)
    std::vector<void *> ob_ptrs, ac_ptrs, info_ptrs;
    float *rew_host = nullptr;
    uint8_t *first_host = nullptr;
    bool buffers_set = false;
    bool atlas = false;
    bool gen_assets = false; // use_generated_assets: AssetGen sprites + per-env procedural backgrounds
    bool fused = false;      // step + render in one launch where the register-frame render serves the game (pg_fused.hip)
    int parity = 0;          // alternates per act: which slow-env list the step launches write
    bool started = false;
    // device allocations
    std::vector<void *> allocs;
    uint32_t *d_pixels = nullptr;
    int32_t *d_sprites = nullptr, *d_bgs = nullptr, *d_themes = nullptr;
    uint8_t *own_rgb = nullptr;   // the library's observation tensor (dev.rgb may point elsewhere,
                                  // procgen_set_obs_buffer)
    int32_t *h_actions = nullptr; // page-locked staging of libenv_act's actions
    hipEvent_t act_copied = nullptr; // the last action upload has read h_actions
    bool act_pending = false;
    std::vector<uint8_t> h_staging;
    uint8_t *pinned = nullptr;  // page-locked landing zone of copy_out (all output planes)
    size_t pinned_bytes = 0;
    // caller buffers that are one contiguous array per output plane (what gym3 allocates) are
    // page-locked in place with hipHostRegister and written by DMA directly (no staging copy)
    std::vector<void *> registered;
    bool direct = false;
    void *hr_host = nullptr; // the caller's info["rgb"] plane, page-locked when contiguous (render_mode="rgb_array")
    // libenv_act with direct buffers: each part's obs DMA is enqueued on its chain's stream right after
    // its render (vecgame.cpp:426-444: the reference's stepping threads also write the caller's obs
    // buffers before observe), so part 0's copy runs while part 1 still renders; copy_out then only
    // moves the small planes
    bool obs_early = false, obs_inflight = false;
    // host buffers with parts: part 0 starts once part 1 rendered, so part 1's copy (the first on the
    // copy stream) starts sooner and part 0 computes under it (PROCGEN_MI355X_HOST_SERIAL=0: off)
    bool host_serial = true;
    // the per-part obs DMAs (obs_early) run on their own normal-priority stream: issued on a part's
    // high-priority chain stream the runtime made them a blit kernel (copyBuffer) that held the CUs
    // for the whole 7 ms transfer and stalled the other part's render behind it
    hipStream_t cstream = nullptr;
    // render_mode="rgb_array" into page-locked caller arrays: the 512x512 frames render in chunks on
    // hstream while the engine stream DMAs the finished chunks (PROCGEN_MI355X_HR_CHUNKS, default 8)
    hipStream_t hstream = nullptr;
    std::vector<hipEvent_t> hr_ev;
    hipEvent_t ev_cdone = nullptr;
    std::vector<hipEvent_t> ev_rendered;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev; // per timed step: 4 per game (before step, after step, after reset,
                                // after render) + 2 on the main stream (before the fork, after the join)
    int t_used = 0;             // timed steps recorded since procgen_set_timing
    int device = 0;
    int error = 0;
    std::string error_msg;
    // games of the batch: env n plays games[n % games.size()]
    std::vector<int> games;
    int32_t *d_lists = nullptr;            // [games.size()][num_envs / games.size()] env ids (mixed only)
    std::vector<int32_t> h_lists;          // host copy of d_lists
    // mixed batches: each game's step -> reset -> render chain runs on its own stream (the games'
    // envs are disjoint), forked from and joined back into `stream` every act
    std::vector<hipStream_t> gstreams;
    std::vector<int> launch_order; // chains in enqueue order (mixed: costliest first)
    std::vector<hipEvent_t> gdone;
    // single game split into `parts` chains over contiguous env ranges (PROCGEN_MI355X_PARTS): each
    // part's step -> reset -> render chain on its own stream (gstreams), so one part renders while
    // another is still stepping -- a step launch ends on its slowest env (coinrun's crate-pile push
    // chains: one env can take 400-650 us), and a lone tail wave leaves the GPU idle.  The per-chain
    // bookkeeping (reset queue, slow-env list, spare requests) lives in PGDev slot k (a single-game
    // batch leaves the other games' slots free); d_ident = 0..num_envs-1 supplies the part lists.
    int parts = 1;
    int32_t *d_ident = nullptr;
    // chain k's stream: 0 = the engine stream, j > 0 = gstreams[j]; a mixed batch packs its chains onto
    // PROCGEN_MI355X_MIXED_STREAMS (default 4) streams, longest first onto the least loaded
    std::vector<int> chain_stream;
    size_t chains() const { return games.size() > 1 ? games.size() : (size_t)parts; }
    int chain_game(size_t k) const { return games.size() > 1 ? games[k] : games[0]; }
    int chain_slot(size_t k) const { return games.size() > 1 ? games[k] : (int)k; }
    int chain_lo(size_t k) const { return (int)((size_t)num_envs * k / (size_t)parts); }
    const int32_t *chain_list(size_t k) const {
        return games.size() > 1 ? list_of(k) : (parts > 1 ? d_ident + chain_lo(k) : nullptr);
    }
    int chain_count(size_t k) const {
        return games.size() > 1 ? count_of() : (int)((size_t)num_envs * (k + 1) / (size_t)parts) - chain_lo(k);
    }
    // per game: the stream the reset kernel runs on while the envs that did not finish render, and
    // the events ordering step -> reset -> render of the finished envs
    std::vector<hipStream_t> rstreams;
    std::vector<hipEvent_t> ev_stepped, ev_reset;
    // level prefetch (PGDev::sp_*): the spare generation of act t runs on pstreams[t % npstreams];
    // the reset of act t waits for the generation launched at act t - lag (ev_pre[t % lag])
    bool prefetch = false;
    uint32_t prefetch_games = 0; // bit g: game g's chains use the prefetch (mixed batches: only some)
    int act_no = 0, lag = 2, npstreams = 1;
    // mixed batches, PROCGEN_MI355X_PREFETCH_INBAND=1: the spare generation of the prefetched chains runs
    // as one more job of the 4-stream packing, on chain stream gen_si after that stream's chains
    bool inband = false;
    int gen_si = 0;
    hipStream_t pstreams[2] = {nullptr, nullptr};
    hipEvent_t ev_pre[PG_SP_LAG_MAX] = {};
    bool ev_pre_set[PG_SP_LAG_MAX] = {};
    hipEvent_t fork = nullptr;
    bool has_latent = false;               // maze fills the fork's latent-state info
    // game of env e: the global index decides (vecgame.cpp:357-358), so a shard at env_offset
    // plays exactly the games of the same envs of one unsharded vec env
    int game_of(int e) const { return games[(size_t)(env_offset + e) % games.size()]; }
    const int32_t *list_of(size_t k) const {
        return games.size() > 1 ? d_lists + k * (size_t)(num_envs / games.size()) : nullptr;
    }
    int count_of() const { return num_envs / (int)games.size(); }
};

#define HIPCHECK(x)                                                                      \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "procgen_mi355x: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return fail(v, PG_ERR_HIP, hipGetErrorString(e_));                           \
        }                                                                                \
    } while (0)

// Every other host<->device copy is ordered on the env's own (non-blocking) stream and complete
// on return: a null-stream hipMemcpy is not ordered with that stream, and from pageable
// memory it may return before its DMA has landed (kernels could read half-written data).
static hipError_t copy_sync(VecEnv *v, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, v->stream);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(v->stream);
}

int upload_atlas(VecEnv *v, const uint32_t *pixels, int64_t num_pixels, const pg_image *sprites,
                 const pg_image *backgrounds, const int32_t *num_backgrounds, const int32_t *num_themes);
int copy_latent(VecEnv *v);
int copy_latent_grid(VecEnv *v);
static hipError_t d2h_registered(void *dst, const void *src, size_t n, hipStream_t s);

int fail(VecEnv *v, int code, const char *msg) {
    if (v && !v->error) {
        v->error = code;
        v->error_msg = msg ? msg : "";
    }
    return -code;
}

template <typename T>
int dalloc(VecEnv *v, T **p, size_t count) {
    void *q = nullptr;
    HIPCHECK(hipMalloc(&q, count * sizeof(T) > 0 ? count * sizeof(T) : 16));
    HIPCHECK(hipMemsetAsync(q, 0, count * sizeof(T) > 0 ? count * sizeof(T) : 16, v->stream));
    v->allocs.push_back(q);
    *p = (T *)q;
    return 0;
}

libenv_tensortype make_type(const char *name, libenv_dtype dt, std::vector<int> shape, int lo, int hi) {
    libenv_tensortype s;
    memset(&s, 0, sizeof(s));
    snprintf(s.name, sizeof(s.name), "%s", name);
    s.scalar_type = LIBENV_SCALAR_TYPE_DISCRETE;
    s.dtype = dt;
    s.ndim = (int)shape.size();
    for (size_t i = 0; i < shape.size(); i++) s.shape[i] = shape[i];
    if (dt == LIBENV_DTYPE_UINT8) {
        s.low.uint8 = (uint8_t)lo;
        s.high.uint8 = (uint8_t)hi;
    } else {
        s.low.int32 = lo;
        s.high.int32 = hi;
    }
    return s;
}

// games that render with the register-frame kernel by default (pg_render.hip pg_render_rf_kernel):
// where it measured faster at 65,536 envs (profiles/r05/r05_h_rf_games.txt, 4 rows per batch, no spills:
// bigfish 58.7 -> 69.1 M, climber 27.7 -> 39.8, ninja 24.2 -> 34.7, miner 25.6 -> 30.7, maze 33.2 -> 33.8,
// chaser 29.0 -> 29.2); coinrun ties (36.8 vs 36.7 M)
#define RF_DEFAULT ((1 << PG_GAME_BIGFISH) | (1 << PG_GAME_CLIMBER) | (1 << PG_GAME_NINJA) | (1 << PG_GAME_MINER) | \
                    (1 << PG_GAME_MAZE) | (1 << PG_GAME_CHASER))

// The games whose frames the register-frame render draws (PGDev::render_rf): it serves centred,
// non-monochrome, atlas-asset frames (pg_render.hip rf_game).  PROCGEN_MI355X_RENDER_RF=0 keeps every
// game on the LDS-frame kernel; "all" or a comma list of game names picks the games (default:
// RF_DEFAULT, the games where it measured faster).
static int rf_mask(bool center_agent, bool monochrome, bool generated) {
    if (monochrome || generated) return 0;
    // without center_agent the window is the whole world: 64 tiles wide for the games that honour the
    // option, too wide for the register-frame tables (the others override it and have small worlds)
    const int centred_games = (1 << PG_GAME_COINRUN) | (1 << PG_GAME_CLIMBER) | (1 << PG_GAME_NINJA) |
                              (1 << PG_GAME_JUMPER) | (1 << PG_GAME_CAVEFLYER) | (1 << PG_GAME_FRUITBOT);
    const int keep = center_agent ? ~0 : ~centred_games;
    const char *rf = getenv("PROCGEN_MI355X_RENDER_RF");
    if (!rf) return RF_DEFAULT & keep;
    if (rf[0] == '0') return 0;
    if (!strcmp(rf, "all")) return ((1 << PG_NUM_GAMES) - 1) & keep;
    int mask = 0;
    std::string list(rf);
    size_t p0 = 0;
    while (p0 <= list.size()) {
        const size_t p1 = std::min(list.find(',', p0), list.size());
        const std::string name = list.substr(p0, p1 - p0);
        for (int g = 0; g < PG_NUM_GAMES; g++)
            if (name == pg_game_name(g)) mask |= 1 << g;
        p0 = p1 + 1;
    }
    return mask & keep;
}

int launch_step(VecEnv *v, int use_hash, uint64_t seed, int32_t t) {
    if (!v->atlas) return fail(v, PG_ERR_NO_ATLAS, "procgen_upload_atlas was not called");
    HIPCHECK(hipSetDevice(v->device));
    const size_t C = v->chains(); // a mixed batch's games, or a single game's parts
    const bool split = v->games.size() == 1;
    hipEvent_t *e = nullptr; // PG_EV_G per chain (see procgen_kernel_times); then 2 wall
    const size_t per = PG_EV_G * C + 2;
    if (v->timing) {
        size_t need = (size_t)(v->t_used + 1) * per;
        while (v->ev.size() < need) {
            hipEvent_t x;
            HIPCHECK(hipEventCreate(&x));
            v->ev.push_back(x);
        }
        e = &v->ev[(size_t)v->t_used * per];
        v->t_used++;
    }
    if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * C], v->stream));
    // reset counts and the slow-list length of this act's step order (PGDev::sched)
    v->parity ^= 1;
    HIPCHECK(hipMemsetAsync(v->dev.sched + PG_SCHED_CLEAR(v->parity), 0, sizeof(int32_t) * 32, v->stream));
    const int act = v->act_no;
    if (v->prefetch && C > 1) { // this act's spare-request ring slot, cleared once for every chain
        const int i = act % v->lag;
        if (v->ev_pre_set[i]) HIPCHECK(hipStreamWaitEvent(v->stream, v->ev_pre[i], 0));
        HIPCHECK(hipMemsetAsync(v->dev.sp_count + i * PG_NUM_GAMES, 0, PG_NUM_GAMES * 4, v->stream));
    }
    if (C > 1) HIPCHECK(hipEventRecord(v->fork, v->stream));
    std::vector<char> seen(v->gstreams.size() + 1, 0); // streams that already waited on the fork
    const bool host_serial = v->obs_early && split && C > 1 && v->host_serial;
    bool pre_waited = false; // this act's prefetch stream already waits for the previous act's generation
    std::vector<size_t> gen_chains; // inband prefetch: chains whose spare generation follows every chain
    for (size_t ki = 0; ki < C; ki++) {
        const size_t k = host_serial ? (ki + 1) % C : C > 1 ? (size_t)v->launch_order[ki] : ki;
        // single game: the finished envs' resets (level generation: long single-wave chains) run on
        // a side stream while the envs that did not finish render; a mixed batch keeps each game's
        // step -> reset -> render chain on its stream (its 16 chains already overlap, and twice as
        // many streams over the GPU_MAX_HW_QUEUES queues measured slower: 14.5 vs 17.4 M env-steps/s)
        const int game = v->chain_game(k), slot = v->chain_slot(k), cnt = v->chain_count(k);
        const int32_t *list = v->chain_list(k);
        // chain 0 runs on the engine stream itself: every extra stream shares one of the
        // GPU_MAX_HW_QUEUES (4) hardware queues, and a chain whose queue also carries the join's
        // waits is serialized behind them
        const int si = C > 1 ? v->chain_stream[k] : 0;
        hipStream_t s = si > 0 ? v->gstreams[si] : v->stream, r = split ? v->rstreams[k] : s;
        if (si > 0 && !seen[si]) HIPCHECK(hipStreamWaitEvent(s, v->fork, 0)); // first chain on the stream
        seen[si] = true;
        if (host_serial && k == 0) HIPCHECK(hipStreamWaitEvent(s, v->ev_rendered[1], 0)); // enqueued last
        if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 0], s));
        PG_POISON(s);
        // fused: step + render of the envs that did not finish in one launch (pg_fused.hip)
        const bool fz = v->fused && ((v->dev.render_rf >> game) & 1) &&
                        pg_launch_fused(&v->dev, game, list, cnt, s, use_hash, seed, t, v->parity, slot) == 0;
        if (!fz) pg_launch_step(&v->dev, game, list, cnt, s, use_hash, seed, t, v->parity, slot);
        if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 1], s));
        if (split) {
            HIPCHECK(hipEventRecord(v->ev_stepped[k], s));
            HIPCHECK(hipStreamWaitEvent(r, v->ev_stepped[k], 0));
        }
        if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 2], r));
        PG_POISON(r);
        if (v->prefetch && C == 1) { // the spares the swaps may use (requested at act - lag) are complete
            const int i = act % v->lag; // also the ring slot of this act's requests
            if (v->ev_pre_set[i]) HIPCHECK(hipStreamWaitEvent(r, v->ev_pre[i], 0));
            HIPCHECK(hipMemsetAsync(v->dev.sp_count + i * PG_NUM_GAMES, 0, PG_NUM_GAMES * 4, r));
        }
        const bool pfk = v->prefetch && ((v->prefetch_games >> game) & 1);
        PGDev dk = v->dev;
        if (!pfk) dk.sp_envs = nullptr; // this chain neither swaps in spares nor requests them
        pg_launch_reset(&dk, game, list, cnt, r, 0, 0, act, slot);
        if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 3], r));
        if (pfk && v->inband && C > 1) { // generated after every chain, on the packing's gen stream
            HIPCHECK(hipEventRecord(v->ev_stepped[k], r));
            gen_chains.push_back(k);
        } else if (pfk) { // the next levels of the envs just reset, off the critical path
            hipStream_t p = v->pstreams[act % v->npstreams];
            HIPCHECK(hipEventRecord(v->ev_stepped[k], r));
            HIPCHECK(hipStreamWaitEvent(p, v->ev_stepped[k], 0));
            // with 2 prefetch streams, acts a and a+1 generate on different streams: an env whose
            // episode ends at both would have both write its spare rows, so act a+1's generation
            // also waits for act a's (ring slot (act - 1) % lag, not yet reused: lag >= 2 here) -- once,
            // before the first generation this act enqueues on that stream, whichever chain it is
            // (host_serial, MIXED_ORDER and PREFETCH_GAMES change which chain comes first)
            const int prev = (act + v->lag - 1) % v->lag;
            if (v->npstreams > 1 && v->lag > 1 && !pre_waited && v->ev_pre_set[prev])
                HIPCHECK(hipStreamWaitEvent(p, v->ev_pre[prev], 0));
            pre_waited = true;
            pg_launch_reset(&v->dev, game, list, cnt, p, 2, 0, act, slot);
            HIPCHECK(hipEventRecord(v->ev_pre[act % v->lag], p));
            v->ev_pre_set[act % v->lag] = true;
        }
        PG_POISON(s);
        if (split) {
            HIPCHECK(hipEventRecord(v->ev_reset[k], r));
            if (!fz) pg_launch_render(&v->dev, game, list, cnt, s, 1, slot);
            if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 4], s));
            HIPCHECK(hipStreamWaitEvent(s, v->ev_reset[k], 0));
            if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 5], s));
            pg_launch_render(&v->dev, game, list, cnt, s, 2, slot);
        } else {
            if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 4], s)); // unused without the split
            if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 5], s));
            pg_launch_render(&v->dev, game, list, cnt, s, fz ? 2 : 0, slot); // fused: only the reset envs remain
        }
        if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * k + 6], s));
        if (v->obs_early && split) HIPCHECK(hipEventRecord(v->ev_rendered[k], s));
    }
    if (!gen_chains.empty()) { // inband prefetch: the spare generations, one job on stream gen_si
        hipStream_t p = v->gen_si > 0 ? v->gstreams[v->gen_si] : v->stream;
        for (size_t k : gen_chains) {
            HIPCHECK(hipStreamWaitEvent(p, v->ev_stepped[k], 0));
            pg_launch_reset(&v->dev, v->chain_game(k), v->chain_list(k), v->chain_count(k), p, 2, 0, act, v->chain_slot(k));
        }
        HIPCHECK(hipEventRecord(v->ev_pre[act % v->lag], p));
        v->ev_pre_set[act % v->lag] = true;
    }
    if (v->obs_early && split) {
        // host buffers: each part's observations leave as soon as it rendered, on one copy stream in the
        // order the parts finish: part 1 (highest priority) first, part 0 (the engine stream) last --
        // in chain order part 1's copy waited behind part 0's render (0.3 ms per act, r04_n trace)
        if (!v->cstream) HIPCHECK(hipStreamCreateWithFlags(&v->cstream, hipStreamNonBlocking));
        for (size_t i = 0; i < C; i++) {
            const size_t k = (i + 1) % C;
            const size_t lo = (size_t)v->chain_lo(k) * PG_OBS_BYTES;
            HIPCHECK(hipStreamWaitEvent(v->cstream, v->ev_rendered[k], 0));
            HIPCHECK(d2h_registered((uint8_t *)v->registered[0] + lo, v->dev.rgb + lo,
                                    (size_t)v->chain_count(k) * PG_OBS_BYTES, v->cstream));
        }
        v->obs_inflight = true;
    }
    if (v->obs_inflight) { // observe() synchronizes the engine stream: it waits for the obs DMAs too
        HIPCHECK(hipEventRecord(v->ev_cdone, v->cstream));
        HIPCHECK(hipStreamWaitEvent(v->stream, v->ev_cdone, 0));
    }
    for (size_t j = 1; j < v->gstreams.size() && C > 1; j++) { // join, after every chain is enqueued
        bool used = false;
        for (size_t k = 0; k < C && !used; k++) used = v->chain_stream[k] == (int)j;
        if (!used) continue;
        HIPCHECK(hipEventRecord(v->gdone[j], v->gstreams[j]));
        HIPCHECK(hipStreamWaitEvent(v->stream, v->gdone[j], 0));
    }
    if (e) HIPCHECK(hipEventRecord(e[PG_EV_G * C + 1], v->stream));
    v->act_no++;
    HIPCHECK(hipGetLastError());
    return 0;
}

// Device -> page-locked (hipHostRegister'd) host copy.  Inside the engine the runtime carries these as
// copyBuffer blit kernels that hold CUs for the whole transfer (the same copy in a probe
// process goes to SDMA, scripts/d2h_probe2.hip).  Round 5 tried them as hipMemcpyDeviceToDeviceNoCU
// (an opt-in knob, removed in round 6): the trace still showed blits and the rate did not move.
static hipError_t d2h_registered(void *dst, const void *src, size_t n, hipStream_t s) {
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
}

// Host memcpy, split over a few threads for large frames (805 MB at 65,536 envs).
static void host_copy(void *dst, const void *src, size_t bytes) {
    const size_t chunk = 32u << 20;
    if (bytes <= 2 * chunk) {
        memcpy(dst, src, bytes);
        return;
    }
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt < 2 ? 2 : (nt > 8 ? 8 : nt);
    std::vector<std::thread> th;
    size_t per = (bytes + nt - 1) / nt;
    for (unsigned t = 0; t < nt; t++) {
        size_t lo = per * t, hi = lo + per < bytes ? lo + per : bytes;
        if (lo >= hi) break;
        th.emplace_back([=] { memcpy((char *)dst + lo, (const char *)src + lo, hi - lo); });
    }
    for (auto &x : th) x.join();
}

// The caller's buffers of one output plane, if they form one contiguous array (stride = element
// size): its base, else nullptr.
static void *contiguous(void **ptrs, size_t n, size_t elem) {
    for (size_t e = 1; e < n; e++)
        if ((char *)ptrs[e] != (char *)ptrs[0] + e * elem) return nullptr;
    return ptrs[0];
}

static void unregister_buffers(VecEnv *v) {
    for (void *p : v->registered) (void)hipHostUnregister(p);
    v->registered.clear();
    v->direct = false;
    if (v->hr_host) (void)hipHostUnregister(v->hr_host);
    v->hr_host = nullptr;
}

// libenv_set_buffers: page-lock the caller's planes when every one is a contiguous array
static void register_buffers(VecEnv *v) {
    unregister_buffers(v);
    const size_t n = (size_t)v->num_envs;
    if (v->render_human) { // info["rgb"]: 786 KB per env, DMA'd straight into the caller's array
        void *p = contiguous(&v->info_ptrs[v->hr_info * n], n, (size_t)512 * 512 * 3);
        if (p && hipHostRegister(p, (size_t)512 * 512 * 3 * n, hipHostRegisterDefault) == hipSuccess) v->hr_host = p;
        else (void)hipGetLastError();
    }
    void *planes[6] = {contiguous(&v->ob_ptrs[0], n, PG_OBS_BYTES), v->rew_host, v->first_host,
                       contiguous(&v->info_ptrs[0], n, 4), contiguous(&v->info_ptrs[n], n, 1),
                       contiguous(&v->info_ptrs[2 * n], n, 4)};
    const size_t sizes[6] = {PG_OBS_BYTES, 4, 1, 4, 1, 4};
    for (int k = 0; k < 6; k++)
        if (!planes[k]) return;
    for (int k = 0; k < 6; k++) {
        if (hipHostRegister(planes[k], sizes[k] * n, hipHostRegisterDefault) != hipSuccess) {
            (void)hipGetLastError();
            unregister_buffers(v);
            return;
        }
        v->registered.push_back(planes[k]);
    }
    v->direct = true;
}

int copy_out(VecEnv *v) {
    // device planes -> the caller's buffers: straight DMA into page-locked contiguous planes
    // (register_buffers), otherwise one page-locked landing zone (DMA, ordered on the env's
    // stream) -> the caller's per-env host pointers (contiguous runs become one memcpy).
    const size_t n = (size_t)v->num_envs;
    if (v->direct) {
        if (!v->obs_inflight) // else the act's chains issued the obs DMA part by part (launch_step)
            HIPCHECK(d2h_registered(v->registered[0], v->dev.rgb, PG_OBS_BYTES * n, v->stream));
        v->obs_inflight = false;
        HIPCHECK(d2h_registered(v->registered[1], v->dev.rew, 4 * n, v->stream));
        HIPCHECK(d2h_registered(v->registered[2], v->dev.first, n, v->stream));
        HIPCHECK(d2h_registered(v->registered[3], v->dev.prev_level_seed, 4 * n, v->stream));
        HIPCHECK(d2h_registered(v->registered[4], v->dev.prev_level_complete, n, v->stream));
        HIPCHECK(d2h_registered(v->registered[5], v->dev.level_seed, 4 * n, v->stream));
        HIPCHECK(hipStreamSynchronize(v->stream));
        return copy_latent(v);
    }
    const size_t sizes[6] = {PG_OBS_BYTES, 4, 1, 4, 1, 4};
    const void *dsrc[6] = {v->dev.rgb, v->dev.rew, v->dev.first, v->dev.prev_level_seed,
                           v->dev.prev_level_complete, v->dev.level_seed};
    size_t off[7];
    off[0] = 0;
    for (int k = 0; k < 6; k++) off[k + 1] = off[k] + ((sizes[k] * n + 255) & ~(size_t)255);
    if (v->pinned_bytes < off[6]) {
        if (v->pinned) (void)hipHostFree(v->pinned);
        v->pinned = nullptr;
        v->pinned_bytes = 0;
        HIPCHECK(hipHostMalloc((void **)&v->pinned, off[6], hipHostMallocDefault));
        v->pinned_bytes = off[6];
    }
    for (int k = 0; k < 6; k++)
        HIPCHECK(hipMemcpyAsync(v->pinned + off[k], dsrc[k], sizes[k] * n, hipMemcpyDeviceToHost, v->stream));
    HIPCHECK(hipStreamSynchronize(v->stream));
    auto scatter = [&](const uint8_t *src, size_t elem, void **ptrs) {
        size_t e = 0;
        while (e < n) {
            size_t k = e + 1;
            while (k < n && (char *)ptrs[k] == (char *)ptrs[k - 1] + elem) k++;
            host_copy(ptrs[e], src + elem * e, elem * (k - e));
            e = k;
        }
    };
    scatter(v->pinned + off[0], PG_OBS_BYTES, &v->ob_ptrs[0]);
    memcpy(v->rew_host, v->pinned + off[1], 4 * n);
    memcpy(v->first_host, v->pinned + off[2], n);
    scatter(v->pinned + off[3], 4, &v->info_ptrs[0 * n]);
    scatter(v->pinned + off[4], 1, &v->info_ptrs[1 * n]);
    scatter(v->pinned + off[5], 4, &v->info_ptrs[2 * n]);
    return copy_latent(v);
}

int copy_latent(VecEnv *v) {
    const size_t n = (size_t)v->num_envs;
    if (v->render_human) { // VecGame::observe: every env's frame at RENDER_RES (vecgame.cpp:415-423)
        const size_t per = (size_t)512 * 512, cnt = (size_t)v->count_of();
        if (v->hr_host) {
            // DMA into the page-locked caller array, each env's frame to its own slot.  The frames render
            // in chunks on hstream and each chunk leaves on the engine stream as soon as it is done (the
            // engine stream's copies run on SDMA): the copy of chunk j overlaps the render of
            // chunk j + 1, so only the first chunk's render is not under the D2H copy
            const size_t nch = v->hr_ev.size();
            uint8_t *dst = (uint8_t *)v->hr_host;
            // created on first use: a stream made in libenv_make shifts the chains' hardware queues (§4.6)
            if (!v->hstream) HIPCHECK(hipStreamCreateWithFlags(&v->hstream, hipStreamNonBlocking));
            HIPCHECK(hipEventRecord(v->hr_ev[0], v->stream)); // the act's state is complete
            HIPCHECK(hipStreamWaitEvent(v->hstream, v->hr_ev[0], 0));
            for (size_t k = 0; k < v->games.size(); k++)
                for (size_t j = 0; j < nch; j++) {
                    const size_t lo = cnt * j / nch, hi = cnt * (j + 1) / nch, b = k * cnt + lo;
                    if (hi <= lo) continue;
                    const int32_t *list = v->games.size() > 1 ? v->list_of(k) + lo : v->d_ident + lo;
                    if (pg_launch_render_hires(&v->dev, v->games[k], list, (int)(hi - lo), v->hr_frames + b * per,
                                               v->hr_rgb + b * per * 3, v->hstream) != 0)
                        return fail(v, PG_ERR_BAD_OPTION, "render_mode=rgb_array: game not built");
                    HIPCHECK(hipGetLastError());
                    HIPCHECK(hipEventRecord(v->hr_ev[j], v->hstream));
                    HIPCHECK(hipStreamWaitEvent(v->stream, v->hr_ev[j], 0));
                    if (v->games.size() == 1) {
                        HIPCHECK(d2h_registered(dst + lo * per * 3, v->hr_rgb + lo * per * 3, (hi - lo) * per * 3,
                                                v->stream));
                    } else {
                        for (size_t q = lo; q < hi; q++)
                            HIPCHECK(d2h_registered(dst + (size_t)v->h_lists[k * cnt + q] * per * 3,
                                                    v->hr_rgb + (k * cnt + q) * per * 3, per * 3, v->stream));
                    }
                }
            HIPCHECK(hipStreamSynchronize(v->stream));
            return copy_latent_grid(v);
        }
        for (size_t k = 0; k < v->games.size(); k++)
            if (pg_launch_render_hires(&v->dev, v->games[k], v->list_of(k), (int)cnt, v->hr_frames + k * cnt * per,
                                       v->hr_rgb + k * cnt * per * 3, v->stream) != 0)
                return fail(v, PG_ERR_BAD_OPTION, "render_mode=rgb_array: game not built");
        HIPCHECK(hipGetLastError());
        {
            std::vector<uint8_t> host(cnt * per * 3);
            for (size_t k = 0; k < v->games.size(); k++) {
                HIPCHECK(copy_sync(v, host.data(), v->hr_rgb + k * cnt * per * 3, host.size(), hipMemcpyDeviceToHost));
                for (size_t q = 0; q < cnt; q++) {
                    const size_t e = v->games.size() > 1 ? (size_t)v->h_lists[k * cnt + q] : q; // list_of(k) order
                    memcpy(v->info_ptrs[v->hr_info * n + e], host.data() + q * per * 3, per * 3);
                }
            }
        }
    }
    return copy_latent_grid(v);
}

int copy_latent_grid(VecEnv *v) {
    const size_t n = (size_t)v->num_envs;
    if (v->has_latent) { // grid_size, grid, agent_pos, exit_pos (vecgame.cpp:270-316)
        const size_t row = (size_t)PG_LATENT_N * 4;
        std::vector<int32_t> lat((size_t)PG_LATENT_N * n);
        HIPCHECK(copy_sync(v, lat.data(), v->dev.latent, row * n, hipMemcpyDeviceToHost));
        const size_t parts[4][2] = {{0, 2}, {2, PG_LATENT_GRID}, {2 + PG_LATENT_GRID, 2}, {4 + PG_LATENT_GRID, 2}};
        for (int k = 0; k < 4; k++)
            for (size_t e = 0; e < n; e++)
                memcpy(v->info_ptrs[(3 + k) * n + e], &lat[e * PG_LATENT_N + parts[k][0]], parts[k][1] * 4);
    }
    return 0;
}

int check_device_errors(VecEnv *v) {
    int32_t flags = 0;
    HIPCHECK(copy_sync(v, &flags, v->dev.error_any, 4, hipMemcpyDeviceToHost));
    if (flags && !v->error) {
        int code = __builtin_ctz((unsigned)flags);
        std::string msg = code == PG_ERR_ENTITY_OVERFLOW ? "entity capacity exceeded"
                          : code == PG_ERR_GRID        ? "grid write out of range"
                          : code == PG_ERR_ASSETGEN    ? "AssetGen background painter met a path it does not restate (reason bits " +
                                                          std::to_string((unsigned)flags >> 16) + ")"
                          : code == PG_ERR_RENDER      ? "render met an atlas reference or a case it does not have"
                                                       : "unsupported feature reached on device";
        fail(v, code, msg.c_str());
    }
    return 0;
}

} // namespace

extern "C" {

// The shard plan of a vec env of num_envs envs at global env index env_offset (multi-GPU: rank r of N
// owns [r * E, (r + 1) * E)): local env e plays game gids[(env_offset + e) % G] (vecgame.cpp:357-358),
// seeds its level-seed generator with the (env_offset + e)-th draw of rand_seed's mt19937
// (vecgame.cpp:349-362), and in a mixed batch game k's chain lists the local envs whose global index
// is k mod G.  libenv_make builds every env from this; procgen_shard_plan exports it (no GPU needed)
// so the multi-rank CPU tests check that shards concatenate to the unsharded plan.
static void shard_plan(size_t n, int env_offset, uint32_t rand_seed, const std::vector<int> &gids, int32_t *game_of,
                       uint32_t *lsg_seed, int32_t *lists) {
    HostMT seed_gen;
    seed_gen.seed(rand_seed);
    for (int k = 0; k < env_offset; k++) (void)seed_gen.next();
    const size_t ng = gids.size();
    for (size_t e = 0; e < n; e++) {
        if (game_of) game_of[e] = gids[((size_t)env_offset + e) % ng];
        const uint32_t sd = seed_gen.next();
        if (lsg_seed) lsg_seed[e] = sd;
    }
    if (lists && ng > 1)
        for (size_t k = 0; k < ng; k++) {
            const size_t r = (size_t)((((int64_t)k - env_offset) % (int64_t)ng + (int64_t)ng) % (int64_t)ng);
            for (size_t q = 0; q < n / ng; q++) lists[k * (n / ng) + q] = (int32_t)(q * ng + r);
        }
}

LIBENV_API int libenv_version(void) { return LIBENV_VERSION; }

LIBENV_API int procgen_shard_plan(const char *env_names, int num_envs, int env_offset, int rand_seed, int32_t *game_of,
                                  uint32_t *lsg_seed, int32_t *lists) {
    if (!env_names || num_envs <= 0 || env_offset < 0) return -1;
    std::vector<int> gids;
    for (const std::string &nm : split_names(env_names)) {
        const int gid = game_id(nm);
        if (gid < 0) return -1;
        gids.push_back(gid);
    }
    if (gids.empty() || num_envs % (int)gids.size() != 0) return -1;
    shard_plan((size_t)num_envs, env_offset, (uint32_t)rand_seed, gids, game_of, lsg_seed, lists);
    return (int)gids.size();
}

// use_generated_assets (basic-abstract-game.cpp:54-123): every image type of every game present is
// AssetGen'd on the device (pg_assetgen_sprites_kernel) -- asset_rand_gen seeded fixed_asset_seed +
// type with fixed_asset_seed = int(FNV-1a(env name)) (vecgame.cpp:156-167, 370-375) -- one theme,
// aspect ratio 1 and the same image for every theme index (the seed ignores the theme); one
// background slot (offset 0, 500 x 500) whose pixels are each env's gen_bg.  Slot 99 keeps jumper's
// tabulated compass raster.
static const int GEN_TYPES = 99;
static int generated_atlas(VecEnv *v, const std::vector<int> &gids, PGAtlasHost &at, std::string &err) {
    uint32_t *d_img = nullptr;
    if (hipMalloc((void **)&d_img, (size_t)GEN_TYPES * 4096 * 4) != hipSuccess) {
        err = "device allocation failed";
        return -1;
    }
    std::vector<uint32_t> img((size_t)GEN_TYPES * 4096);
    int rc = 0;
    for (int g : gids) {
        const char *name = pg_game_name(g);
        uint32_t h = 0x811c9dc5u;
        for (const char *c = name; *c; c++) h = (h ^ (uint8_t)*c) * 0x1000193u;
        if (pg_launch_assetgen_sprites(g, h, d_img, GEN_TYPES, v->stream) != 0 ||
            hipMemcpyAsync(img.data(), d_img, img.size() * 4, hipMemcpyDeviceToHost, v->stream) != hipSuccess ||
            hipStreamSynchronize(v->stream) != hipSuccess) {
            err = "sprite generation failed";
            rc = -1;
            break;
        }
        const uint32_t base = (uint32_t)at.pixels.size();
        for (int t = 0; t < GEN_TYPES; t++)
            if (img[(size_t)t * 4096] == 0xdeadbeefu) {
                err = std::string("AssetGen met a path it does not restate (") + name + " type " + std::to_string(t) + ")";
                rc = -1;
            }
        if (rc) break;
        at.pixels.insert(at.pixels.end(), img.begin(), img.end());
        int32_t *spr = at.sprites.data() + (size_t)g * PG_NUM_SLOTS * 4;
        int32_t *thm = at.num_themes.data() + (size_t)g * 100;
        for (int t = 0; t < GEN_TYPES; t++) {
            for (int th = 0; th < PG_NUM_SLOTS / 100; th++) {
                int32_t *e = spr + (size_t)(t + 100 * th) * 4;
                e[0] = (int32_t)(base + (uint32_t)t * 4096);
                e[1] = 64;
                e[2] = 64;
                e[3] = 0;
            }
            thm[t] = 1;
        }
        int32_t *bg = at.backgrounds.data() + (size_t)g * PG_MAX_BG * 4;
        bg[0] = 0;
        bg[1] = 500;
        bg[2] = 500;
        bg[3] = 0;
        at.num_backgrounds[g] = 1;
    }
    (void)hipFree(d_img);
    return rc;
}

LIBENV_API libenv_env *libenv_make(int num_envs, const struct libenv_options options) {
    g_last_make_error.clear();
    Options opts;
    for (int i = 0; i < options.count; i++) opts.items.push_back(options.items[i]);
    std::string env_name, resource_root;
    int32_t num_levels = 0, start_level = -1, num_actions = -1, rand_seed = 0, num_threads = 4, env_offset = 0;
    bool render_human = false;
    // VecGame options (vecgame.cpp:183-190) + this build's shard offset
    opts.consume_string("env_name", &env_name);
    opts.consume_int("num_levels", &num_levels);
    opts.consume_int("start_level", &start_level);
    opts.consume_int("num_actions", &num_actions);
    opts.consume_int("rand_seed", &rand_seed);
    opts.consume_int("num_threads", &num_threads);
    opts.consume_string("resource_root", &resource_root);
    opts.consume_bool("render_human", &render_human);
    opts.consume_int("env_offset", &env_offset);
    // game options (game.cpp:62-95), consumed once for all envs
    bool paint_vel_info = false, use_generated_assets = false, use_monochrome_assets = false,
         restrict_themes = false, use_backgrounds = true, center_agent = false, use_sequential_levels = false,
         use_easy_jump = false;
    int32_t distribution_mode = PG_EASY, plain_assets = 0, physics_mode = 0, debug_mode = 0, game_type = 0;
    opts.consume_bool("use_easy_jump", &use_easy_jump);
    opts.consume_bool("paint_vel_info", &paint_vel_info);
    opts.consume_bool("use_generated_assets", &use_generated_assets);
    opts.consume_bool("use_monochrome_assets", &use_monochrome_assets);
    opts.consume_bool("restrict_themes", &restrict_themes);
    opts.consume_bool("use_backgrounds", &use_backgrounds);
    opts.consume_bool("center_agent", &center_agent);
    opts.consume_bool("use_sequential_levels", &use_sequential_levels);
    opts.consume_int("distribution_mode", &distribution_mode);
    opts.consume_int("plain_assets", &plain_assets);
    opts.consume_int("physics_mode", &physics_mode);
    opts.consume_int("debug_mode", &debug_mode);
    opts.consume_int("game_type", &game_type);

    auto bad = [&](const std::string &m) -> libenv_env * {
        g_last_make_error = m;
        fprintf(stderr, "procgen_mi355x: libenv_make: %s\n", m.c_str());
        return nullptr;
    };
    if (!opts.error.empty()) return bad(opts.error);
    if (!opts.items.empty()) return bad(std::string("unused options found, first unused option: ") + opts.items[0].name);
    if (env_name.empty()) return bad("env_name missing");
    if (num_actions <= 0) return bad("num_actions must be > 0");
    if (num_levels < 0) return bad("num_levels must be >= 0");
    if (start_level < 0) return bad("start_level must be >= 0");
    if (num_envs <= 0) return bad("num_envs must be > 0");
    std::vector<std::string> names = split_names(env_name);
    std::vector<int> gids;
    for (const std::string &nm : names) {
        int gid = game_id(nm);
        if (gid < 0) return bad("env '" + nm + "' is not in this build (supported: " + SUPPORTED_GAMES + ")");
        // game.cpp:76-86 distribution mode validity
        // (game ids = procgen/env.py:15-32 order: caveflyer 2, jumper 9, starpilot 15)
        bool dm_ok = distribution_mode == PG_EASY || distribution_mode == PG_HARD ||
                     (distribution_mode == PG_EXTREME && (gid == PG_GAME_CHASER || gid == PG_GAME_DODGEBALL ||
                                                          gid == PG_GAME_LEAPER || gid == 15)) ||
                     (distribution_mode == PG_MEMORY && (gid == 2 || gid == PG_GAME_DODGEBALL || gid == PG_GAME_HEIST ||
                                                         gid == 9 || gid == PG_GAME_MAZE || gid == PG_GAME_MINER));
        if (!dm_ok) return bad("invalid distribution_mode for " + nm);
        gids.push_back(gid);
    }
    if (num_envs % (int)gids.size() != 0) return bad("num_envs must be a multiple of the number of env names"); // vecgame.cpp:345
    if (env_offset < 0) return bad("env_offset must be >= 0");
    VecEnv *v = new VecEnv();
    v->num_envs = num_envs;
    v->games = gids;
    for (int g : gids) v->has_latent = v->has_latent || g == PG_GAME_MAZE || g == PG_GAME_MINER;
    v->env_offset = env_offset;
    v->num_actions = num_actions;
    v->render_human = render_human;
    v->gen_assets = use_generated_assets;
    if (hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess) {
        delete v;
        return bad("hipStreamCreate failed");
    }
    {
        // default: coinrun alone in two parts, part 1 at high priority (its step launches end on single
        // crate-pile envs of 400-650 us; the other part's render fills that tail: 29.7 -> 33.6 M
        // env-steps/s).  Measured neutral for bigfish, maze, heist, starpilot, fruitbot, miner and
        // dodgeball, and a loss where the level prefetch adds a fifth stream over the 4 hardware
        // queues (caveflyer -13 %, jumper -23 %): profiles/r03/o_parts_games.
        const char *pp = getenv("PROCGEN_MI355X_PARTS"), *pf = getenv("PROCGEN_MI355X_PREFETCH");
        // coinrun with the register-frame render (PROCGEN_MI355X_RENDER_RF=coinrun) runs in one chain:
        // two parts measured 36.65 / 34.18 M against 37.75 / 35.17 M in one (two boxes, profiles/r05/)
        const bool rf_cr = (rf_mask(center_agent, use_monochrome_assets, use_generated_assets) >> PG_GAME_COINRUN) & 1;
        const bool dflt = gids.size() == 1 && gids[0] == PG_GAME_COINRUN && !(pf && pf[0] == '1') && !rf_cr;
        const int want = pp ? std::min(std::max(atoi(pp), 1), 8) : (dflt ? 2 : 1);
        v->parts = gids.size() == 1 && num_envs >= want * 64 ? want : 1;
    }
    const size_t nchains = gids.size() > 1 ? gids.size() : (size_t)v->parts;
    { // the reset's side stream (single game only: mixed batches keep each game's chain on one stream)
        // PROCGEN_MI355X_RESET_PRIO=1: at the highest stream priority, so the dispatcher places the
        // level generators' workgroups before the concurrent render's (the render of the reset envs
        // waits for them)
        const char *rp = getenv("PROCGEN_MI355X_RESET_PRIO");
        int rlo = 0, rhi = 0;
        const bool rprio = rp && rp[0] == '1' && hipDeviceGetStreamPriorityRange(&rlo, &rhi) == hipSuccess;
        bool ok = true;
        for (size_t k = 0; k < nchains && ok; k++) {
            hipStream_t s = nullptr;
            hipEvent_t a = nullptr, b = nullptr;
            ok = (gids.size() > 1 || (rprio ? hipStreamCreateWithPriority(&s, hipStreamNonBlocking, rhi)
                                            : hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) == hipSuccess) &&
                 hipEventCreateWithFlags(&a, hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&b, hipEventDisableTiming) == hipSuccess;
            hipEvent_t c = nullptr;
            ok = ok && hipEventCreateWithFlags(&c, hipEventDisableTiming) == hipSuccess;
            v->rstreams.push_back(s);
            v->ev_stepped.push_back(a);
            v->ev_reset.push_back(b);
            v->ev_rendered.push_back(c);
        }
        // the obs-copy stream (host buffers only) is created on first use: one more stream at make time
        // shifts the chain streams' hardware-queue assignment and cost coinrun 37 -> 28 M env-steps/s
        ok = ok && hipEventCreateWithFlags(&v->ev_cdone, hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            libenv_close((libenv_env *)v);
            return bad("hipStreamCreate failed");
        }
    }
    // a mixed batch packs its chains onto `ns` streams (below); only those are created: every stream
    // takes or shares a hardware queue at creation, so unused ones still shift the assignment
    // (PROCGEN_MI355X_ALL_GSTREAMS=1 creates one per chain, the round-3 layout)
    const char *ms = getenv("PROCGEN_MI355X_MIXED_STREAMS"), *ag = getenv("PROCGEN_MI355X_ALL_GSTREAMS");
    const int ns = gids.size() > 1 ? std::min(std::max(ms ? atoi(ms) : 4, 1), (int)nchains) : (int)nchains;
    const size_t ncreate = ag && ag[0] == '1' ? nchains : (size_t)ns;
    if (nchains > 1) {
        bool ok = hipEventCreateWithFlags(&v->fork, hipEventDisableTiming) == hipSuccess;
        // parts: part 1's stream gets the highest priority and the later parts' the lowest (part 0 runs
        // on the engine stream); PROCGEN_MI355X_PART_PRIO=0 leaves them all at the default
        const char *pr = getenv("PROCGEN_MI355X_PART_PRIO");
        int lo_prio = 0, hi_prio = 0;
        const bool prio = v->parts > 1 && !(pr && pr[0] == '0') && hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) == hipSuccess;
        for (size_t k = 0; k < ncreate && ok; k++) {
            hipStream_t s = nullptr;
            hipEvent_t d = nullptr;
            ok = (k == 0 || // chain 0 runs on the engine stream (launch_step)
                  (prio ? hipStreamCreateWithPriority(&s, hipStreamNonBlocking, k == 1 ? hi_prio : lo_prio)
                        : hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) == hipSuccess) &&
                 hipEventCreateWithFlags(&d, hipEventDisableTiming) == hipSuccess;
            v->gstreams.push_back(s);
            v->gdone.push_back(d);
        }
        if (!ok) {
            libenv_close((libenv_env *)v);
            return bad("hipStreamCreate failed");
        }
    }
    {
        const char *hs = getenv("PROCGEN_MI355X_HOST_SERIAL");
        v->host_serial = !(hs && hs[0] == '0');
    }
    v->chain_stream.resize(nchains);
    v->launch_order.resize(nchains);
    for (size_t k = 0; k < nchains; k++) v->chain_stream[k] = v->launch_order[k] = (int)k;
    if (gids.size() > 1) {
        // default: as many streams as GPU_MAX_HW_QUEUES (4), chains packed longest-first (all-16 mixed
        // shard 16.5 -> 18.7 M env-steps/s, profiles/r03/r03_q_mixed16*.json); 16 = one per game
        if (ns < (int)nchains) {
            // per-game chain cost, ms at 4,096 envs (step + reset + render per game inside the all-16 mixed
            // shard, profiles/r04/r04_l_mixed/mixed16_default.json per_game).  The round-5 generators
            // changed the costs (r05_q_mixed16.json), but packing on the new table measured slower on one
            // box (24.1-24.3 vs 24.5-24.7 M; render weighted 1.5x / 2x, reset 0.5x: 23.8-24.7 M,
            // profiles/r05/r05_r_packing.txt): the chains contend for CUs, so isolated costs are not the
            // objective.  This table stays.
            static const float cost0[PG_NUM_GAMES] = {0.21f, 0.85f, 1.13f, 0.67f, 0.46f, 0.50f, 0.66f, 0.74f,
                                                      0.49f, 1.45f, 0.99f, 0.51f, 0.51f, 0.47f, 0.35f, 0.67f};
            // inband prefetch (PROCGEN_MI355X_PREFETCH_INBAND=1 with PROCGEN_MI355X_PREFETCH_GAMES): a
            // prefetched chain's reset becomes a swap and its level generation (reset_cost, r05 mixed16
            // per_game) one job packed after every chain of the least loaded stream
            static const float reset_cost[PG_NUM_GAMES] = {0.10f, 0.05f, 0.18f, 0.16f, 0.07f, 0.08f, 0.08f, 0.21f,
                                                           0.18f, 0.37f, 0.40f, 0.28f, 0.10f, 0.08f, 0.07f, 0.31f};
            float cost[PG_NUM_GAMES];
            for (int g = 0; g < PG_NUM_GAMES; g++) cost[g] = cost0[g];
            // PROCGEN_MI355X_MIXED_COSTS: 16 comma-separated chain costs in game-id order (experiments)
            if (const char *mc = getenv("PROCGEN_MI355X_MIXED_COSTS")) {
                const char *q = mc;
                for (int g = 0; g < PG_NUM_GAMES && *q; g++) {
                    char *e = nullptr;
                    const float x = strtof(q, &e);
                    if (e == q) break;
                    cost[g] = x;
                    q = *e == ',' ? e + 1 : e;
                }
            }
            const char *ib = getenv("PROCGEN_MI355X_PREFETCH_INBAND"), *ipg = getenv("PROCGEN_MI355X_PREFETCH_GAMES");
            v->inband = ib && ib[0] == '1' && ipg && ipg[0];
            float gen_cost = 0.f;
            if (v->inband) {
                const std::string sel(ipg);
                for (int g : gids) {
                    bool on = sel == "all";
                    size_t a = 0;
                    while (!on && a <= sel.size()) {
                        const size_t b = std::min(sel.find(',', a), sel.size());
                        on = game_id(sel.substr(a, b - a)) == g;
                        a = b + 1;
                    }
                    if (on) {
                        cost[g] = cost[g] - reset_cost[g] + 0.05f; // the swap
                        gen_cost += reset_cost[g];
                    }
                }
            }
            std::vector<size_t> order(nchains);
            for (size_t k = 0; k < nchains; k++) order[k] = k;
            std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return cost[gids[a]] > cost[gids[b]]; });
            std::vector<float> load(ns, 0.f);
            for (size_t k : order) {
                int best = 0;
                for (int j = 1; j < ns; j++)
                    if (load[j] < load[best]) best = j;
                load[best] += cost[gids[k]];
                v->chain_stream[k] = best;
            }
            // then the best single move or swap out of the most loaded stream while it lowers the maximum
            // (all-16 shard: LPT's largest stream 2.80 ms of chains -> 2.67, the mean)
            for (int it = 0; it < 64; it++) {
                int hi = 0;
                for (int j = 1; j < ns; j++)
                    if (load[j] > load[hi]) hi = j;
                float best_max = load[hi] - 1e-4f;
                int bj = -1;
                long bx = -1, by = -1; // chains moved hi -> bj and bj -> hi (-1: none)
                for (int j = 0; j < ns; j++) {
                    if (j == hi) continue;
                    for (long x = -1; x < (long)nchains; x++) {
                        if (x >= 0 && v->chain_stream[x] != hi) continue;
                        for (long y = -1; y < (long)nchains; y++) {
                            if ((x < 0 && y < 0) || (y >= 0 && v->chain_stream[y] != j)) continue;
                            const float d = (x >= 0 ? cost[gids[x]] : 0.f) - (y >= 0 ? cost[gids[y]] : 0.f);
                            const float m = std::max(load[hi] - d, load[j] + d);
                            if (m < best_max) best_max = m, bj = j, bx = x, by = y;
                        }
                    }
                }
                if (bj < 0) break;
                const float d = (bx >= 0 ? cost[gids[bx]] : 0.f) - (by >= 0 ? cost[gids[by]] : 0.f);
                load[hi] -= d;
                load[bj] += d;
                if (bx >= 0) v->chain_stream[bx] = bj;
                if (by >= 0) v->chain_stream[by] = hi;
            }
            if (v->inband) { // the generation job goes to the least loaded stream (which holds chains)
                int lo = 0;
                for (int j = 1; j < ns; j++)
                    if (load[j] < load[lo]) lo = j;
                v->gen_si = lo;
                load[lo] += gen_cost;
            }
            // enqueue order: game id (default); PROCGEN_MI355X_MIXED_ORDER=desc enqueues the costliest
            // chains first (all-16 shard 21.7 -> 20.8 M env-steps/s, profiles/r04/r04_m_mixed), asc the
            // cheapest first
            const char *mo = getenv("PROCGEN_MI355X_MIXED_ORDER");
            const std::string mode = mo ? mo : "id";
            for (size_t k = 0; k < nchains && mode != "id"; k++)
                v->launch_order[k] = (int)order[mode == "asc" ? nchains - 1 - k : k];
        }
    }
    (void)hipGetDevice(&v->device);

    // spaces (vecgame.cpp:212-316)
    v->ob_types.push_back(make_type("rgb", LIBENV_DTYPE_UINT8, {64, 64, 3}, 0, 255));
    v->ac_types.push_back(make_type("action", LIBENV_DTYPE_INT32, {}, 0, num_actions - 1));
    v->info_types.push_back(make_type("prev_level_seed", LIBENV_DTYPE_INT32, {}, 0, INT32_MAX));
    v->info_types.push_back(make_type("prev_level_complete", LIBENV_DTYPE_UINT8, {}, 0, 1));
    v->info_types.push_back(make_type("level_seed", LIBENV_DTYPE_INT32, {}, 0, INT32_MAX));
    v->info_types.push_back(make_type("grid_size", LIBENV_DTYPE_INT32, {2}, 0, 35));
    v->info_types.push_back(make_type("grid", LIBENV_DTYPE_INT32, {35 * 35}, 0, INT32_MAX));
    v->info_types.push_back(make_type("agent_pos", LIBENV_DTYPE_INT32, {2}, 0, 35));
    v->info_types.push_back(make_type("exit_pos", LIBENV_DTYPE_INT32, {2}, 0, 35));
    if (render_human) { // vecgame.cpp:318-330
        v->hr_info = v->info_types.size();
        v->info_types.push_back(make_type("rgb", LIBENV_DTYPE_UINT8, {512, 512, 3}, 0, 255));
    }

    // level seed bounds (vecgame.cpp:332-341)
    int level_seed_low = 0, level_seed_high = 0;
    if (num_levels == 0) {
        level_seed_low = 0;
        level_seed_high = INT32_MAX;
    } else {
        level_seed_low = start_level;
        level_seed_high = start_level + num_levels;
    }

    size_t n = (size_t)num_envs;
    PGDev &d = v->dev;
    d.num_envs = num_envs;
    d.env_offset = env_offset;
    d.num_actions = num_actions;
    int rc = 0;
    rc |= dalloc(v, &d.envs, n);
    rc |= dalloc(v, &d.ents, (size_t)PG_NF * n * PG_CAP);
    rc |= dalloc(v, &d.grid, n * PG_GRID_MAX);
    rc |= dalloc(v, &d.grid8, n * PG_GRID_MAX);
    rc |= dalloc(v, &d.mt, n * 2 * PG_MT_WORDS);
    rc |= dalloc(v, &d.actions, n);
    rc |= dalloc(v, &d.rgb, n * PG_OBS_BYTES);
    v->own_rgb = d.rgb;
    rc |= dalloc(v, &d.rew, n);
    rc |= dalloc(v, &d.first, n);
    rc |= dalloc(v, &d.prev_level_seed, n);
    rc |= dalloc(v, &d.prev_level_complete, n);
    rc |= dalloc(v, &d.level_seed, n);
    rc |= dalloc(v, &d.reset_queue, n * PG_NUM_GAMES);
    rc |= dalloc(v, &d.sched, 48);
    rc |= dalloc(v, &d.done8, n);
    // level prefetch: random level seeds (a sequential level's seed depends on
    // how the episode ends), no generated backgrounds (1 MB per env per spare).  On by default for the
    // games whose reset is on the critical path (long level generation that outlasts the render of
    // the other envs: caveflyer 24.5 -> 29.6, jumper 20.6 -> 21.7 M env-steps/s); the others lose
    // 1-5 % to the extra work (profiles/r03/prefetch_sweep.txt).  PROCGEN_MI355X_PREFETCH=0 / 1 forces
    // it off / on.
    // In a mixed batch it is off by default: forced on for every game it lost (16.3 -> 10.7 M
    // env-steps/s, profiles/r03/k_mixed16_prefetch), and so did serving only the chains whose level
    // generation bounds them (jumper, caveflyer: 20.5 -> 14.4 M, profiles/r04/r04_d_*).
    // PROCGEN_MI355X_PREFETCH_GAMES (a comma list of game names, or "all") picks the chains.
    {
        const char *pf = getenv("PROCGEN_MI355X_PREFETCH");
        const char *pg = getenv("PROCGEN_MI355X_PREFETCH_GAMES");
        const bool by_game = (gids.size() == 1 && (gids[0] == PG_GAME_CAVEFLYER || gids[0] == PG_GAME_JUMPER)) ||
                             (pg != nullptr && pg[0] != 0);
        v->prefetch = !use_generated_assets && !use_sequential_levels && (pf ? pf[0] != '0' : by_game);
        v->prefetch_games = 0;
        std::string sel = pg ? std::string(pg) : "all";
        uint32_t want = 0;
        if (sel == "all") {
            want = ~0u;
        } else {
            size_t a = 0;
            while (a <= sel.size()) {
                const size_t b = std::min(sel.find(',', a), sel.size());
                const int g = game_id(sel.substr(a, b - a));
                if (g >= 0) want |= 1u << g;
                a = b + 1;
            }
        }
        for (int g : gids) v->prefetch_games |= want & (1u << g);
        if (!v->prefetch_games) v->prefetch = false;
        const char *lg = getenv("PROCGEN_MI355X_PREFETCH_LAG"), *ps = getenv("PROCGEN_MI355X_PREFETCH_STREAMS");
        if (lg) v->lag = std::min(std::max(atoi(lg), 1), PG_SP_LAG_MAX);
        if (ps) v->npstreams = std::min(std::max(atoi(ps), 1), 2);
        d.sp_lag = v->lag;
    }
    if (v->prefetch) {
        rc |= dalloc(v, &d.sp_envs, n);
        rc |= dalloc(v, &d.sp_ents, (size_t)PG_NF * n * PG_CAP);
        rc |= dalloc(v, &d.sp_grid, n * PG_GRID_MAX);
        rc |= dalloc(v, &d.sp_grid8, n * PG_GRID_MAX);
        rc |= dalloc(v, &d.sp_mt, n * 2 * PG_MT_WORDS);
        if (v->has_latent) rc |= dalloc(v, &d.sp_latent, n * PG_LATENT_N);
        rc |= dalloc(v, &d.sp_level_seed, n);
        rc |= dalloc(v, &d.sp_in, (size_t)v->lag * n);
        rc |= dalloc(v, &d.sp_in_lsg, (size_t)v->lag * n * PG_MT_WORDS);
        rc |= dalloc(v, &d.sp_gen, n);
        rc |= dalloc(v, &d.sp_queue, (size_t)v->lag * PG_NUM_GAMES * n);
        rc |= dalloc(v, &d.sp_count, (size_t)v->lag * PG_NUM_GAMES);
        if (!rc && hipMemsetAsync(d.sp_gen, 0x80, n * 4, v->stream) != hipSuccess) rc = 1;
        // the PGEnv words the step kernel writes back (PG_STEP_WB_ALL, pg_engine.h) except `error`
        const size_t offs[][2] = {
#define PG_F(f) {offsetof(PGEnv, f), sizeof(((PGEnv *)0)->f)},
            PG_STEP_WB_ALL(PG_F)
#undef PG_F
        };
        for (auto &o : offs)
            for (size_t b = o[0]; b < o[0] + o[1]; b += 4) d.sp_mask[b / 128] |= 1u << ((b / 4) & 31);
        bool ok = true;
        for (int i = 0; i < v->npstreams && ok; i++)
            ok = hipStreamCreateWithFlags(&v->pstreams[i], hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; i < v->lag && ok; i++) ok = hipEventCreateWithFlags(&v->ev_pre[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) rc = 1;
    }
    d.reset_count = d.sched + PG_SCHED_RC;
    rc |= dalloc(v, &d.heavy, 2 * (size_t)PG_NUM_GAMES * PG_HEAVY_CAP);
    rc |= dalloc(v, &d.heavy_flag, 2 * n);
    d.heavy_ticks = 10000; // 100 us: ~3x the median coinrun step wave
    {
        // PROCGEN_MI355X_HEAVY_US: the slow-env threshold in microseconds (tests: 0 lists every env, which
        // also overflows the PG_HEAVY_CAP slow list, so both launch-order paths run on every act)
        const char *hu = getenv("PROCGEN_MI355X_HEAVY_US");
        if (hu && hu[0]) d.heavy_ticks = atoi(hu) > 0 ? (int64_t)atoi(hu) * 100 : -1;
    }
    {
        // the register-frame render (pg_render_rf_kernel) for the games and options it serves;
        // PROCGEN_MI355X_RENDER_RF=0 keeps every game on the LDS-frame kernel
        d.render_rf = rf_mask(center_agent, use_monochrome_assets, use_generated_assets);
        v->rf_make = d.render_rf;
        v->rf_bad.assign(n, 0);
        const char *fz = getenv("PROCGEN_MI355X_FUSED"); // 1: fuse step and render (pg_fused.hip)
        v->fused = fz && fz[0] == '1';
    }
    {
        const char *sp = getenv("PROCGEN_MI355X_SLOW_PREDICT");
        d.slow_predict = sp ? atoi(sp) : 0;
    }
    if (v->has_latent) rc |= dalloc(v, &d.latent, n * PG_LATENT_N);
    if (render_human) {
        rc |= dalloc(v, &v->hr_frames, n * 512 * 512);
        rc |= dalloc(v, &v->hr_rgb, n * 512 * 512 * 3);
        const char *hc = getenv("PROCGEN_MI355X_HR_CHUNKS");
        v->hr_ev.assign(std::min(std::max(hc ? atoi(hc) : 8, 1), 64), nullptr);
        for (auto &e : v->hr_ev) rc |= hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess;
    }
    if (gids.size() > 1) rc |= dalloc(v, &v->d_lists, n);
    if (v->parts > 1 || render_human) { // part lists; the rgb_array chunks of a single-game batch
        rc |= dalloc(v, &v->d_ident, n);
        if (!rc) {
            std::vector<int32_t> id(n);
            for (size_t e = 0; e < n; e++) id[e] = (int32_t)e;
            if (copy_sync(v, v->d_ident, id.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) rc = 1;
        }
    }
    float *d_rot_angles = nullptr;
    double *d_rot_table = nullptr;
    rc |= dalloc(v, &d_rot_angles, PG_ROT_N);
    rc |= dalloc(v, &d_rot_table, PG_ROT_N * 4);
    d.rot_angles = d_rot_angles;
    d.rot_table = d_rot_table;
    rc |= dalloc(v, &d.error_any, 1);
    rc |= dalloc(v, &d.prof, n * 16); // written only by PG_PROFILE (diagnostic) builds
    // use_generated_assets: each env owns a 500 x 500 RGB32 background (main_bg_images_ptr of one
    // QImage, basic-abstract-game.cpp:58-63), 1 MB per env
    if (use_generated_assets) rc |= dalloc(v, &d.gen_bg, n * PG_GEN_BG_PX);
    if (rc) {
        libenv_close(v);
        return bad("device allocation failed");
    }

    // per-env construction: Game + BasicAbstractGame + CoinRun ctors (game.cpp:25-39,
    // basic-abstract-game.cpp:22-46, coinrun.cpp:49-58) and level-seed generator seeding
    // from rand_seed's MT, global env index n taking the n-th draw (vecgame.cpp:349-362)
    std::vector<PGEnv> h(n);
    std::vector<uint32_t> hmt(n * 2 * PG_MT_WORDS, 0);
    std::vector<int32_t> plan_game(n), lists(gids.size() > 1 ? n : 0);
    std::vector<uint32_t> plan_seed(n);
    shard_plan(n, env_offset, (uint32_t)rand_seed, gids, plan_game.data(), plan_seed.data(), lists.data());
    for (size_t e = 0; e < n; e++) {
        PGEnv &s = h[e];
        construct_env(s, plan_game[e]);
        s.level_seed_low = level_seed_low;
        s.level_seed_high = level_seed_high;
        s.game_n = env_offset + (int)e;
        s.opt_distribution_mode = distribution_mode;
        s.opt_center_agent = center_agent;
        s.opt_use_backgrounds = use_backgrounds;
        s.opt_restrict_themes = restrict_themes;
        s.opt_use_sequential_levels = use_sequential_levels;
        s.opt_debug_mode = debug_mode;
        s.opt_paint_vel_info = paint_vel_info;
        s.opt_use_monochrome_assets = use_monochrome_assets;
        s.rg_mti = PG_MT_N;
        HostMT lsg;
        lsg.seed(plan_seed[e]);
        memcpy(&hmt[(e * 2 + 1) * PG_MT_WORDS], lsg.mt, sizeof(lsg.mt));
        s.lsg_mti = lsg.mti;
    }
    // env lists of a mixed batch (shard_plan): game k owns the envs whose global index is k mod G
    const size_t ng = gids.size();
    if (ng > 1) v->h_lists = lists;
    float rot_angles[PG_ROT_N];
    double rot_table[PG_ROT_N * 4];
    build_rot_table(rot_angles, rot_table);
    if (hipMemcpyAsync(d.envs, h.data(), sizeof(PGEnv) * n, hipMemcpyHostToDevice, v->stream) != hipSuccess ||
        hipMemcpyAsync(d.mt, hmt.data(), hmt.size() * 4, hipMemcpyHostToDevice, v->stream) != hipSuccess ||
        (ng > 1 && hipMemcpyAsync(v->d_lists, lists.data(), n * 4, hipMemcpyHostToDevice, v->stream) != hipSuccess) ||
        hipMemcpyAsync(d_rot_angles, rot_angles, sizeof(rot_angles), hipMemcpyHostToDevice, v->stream) != hipSuccess ||
        hipMemcpyAsync(d_rot_table, rot_table, sizeof(rot_table), hipMemcpyHostToDevice, v->stream) != hipSuccess ||
        hipStreamSynchronize(v->stream) != hipSuccess) {
        libenv_close(v);
        return bad("device upload failed");
    }
    if (hipHostMalloc((void **)&v->h_actions, (size_t)n * 4 + 4, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&v->act_copied, hipEventDisableTiming) != hipSuccess) {
        if (!v->h_actions) v->h_actions = nullptr;
        libenv_close(v);
        return bad("pinned host allocation failed");
    }
    // images: global_init -> images_load from resource_root (vecgame.cpp:144-153, 189-193), here
    // the committed Qt-decoded packs (pg_assets.cpp); procgen_upload_atlas may replace them later
    {
        PGAtlasHost at;
        std::string err, root = resource_root.empty() ? pg_default_asset_root() : resource_root;
        if (!pg_atlas_load(root, gids, &at, &err)) {
            libenv_close(v);
            return bad("asset load failed: " + err);
        }
        if (use_generated_assets && generated_atlas(v, gids, at, err) != 0) {
            libenv_close(v);
            return bad("generated assets: " + err);
        }
        if (upload_atlas(v, at.pixels.data(), (int64_t)at.pixels.size(), (const pg_image *)at.sprites.data(),
                         (const pg_image *)at.backgrounds.data(), at.num_backgrounds.data(), at.num_themes.data()) != 0) {
            std::string m = "atlas upload failed: " + v->error_msg;
            libenv_close(v);
            return bad(m);
        }
    }
    return (libenv_env *)v;
}

LIBENV_API int libenv_get_tensortypes(libenv_env *env, enum libenv_space_name name, struct libenv_tensortype *out) {
    VecEnv *v = (VecEnv *)env;
    const std::vector<libenv_tensortype> *t;
    if (name == LIBENV_SPACE_OBSERVATION) t = &v->ob_types;
    else if (name == LIBENV_SPACE_ACTION) t = &v->ac_types;
    else if (name == LIBENV_SPACE_INFO) t = &v->info_types;
    else return 0;
    if (out) memcpy(out, t->data(), t->size() * sizeof(libenv_tensortype));
    return (int)t->size();
}

LIBENV_API int procgen_upload_atlas(libenv_env *env, const uint32_t *pixels, int64_t num_pixels,
                                    const struct pg_image *sprites, const struct pg_image *backgrounds,
                                    const int32_t *num_backgrounds, const int32_t *num_themes) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION;
    if (v->started) return fail(v, PG_ERR_NO_ATLAS, "procgen_upload_atlas after the first reset");
    return upload_atlas(v, pixels, num_pixels, sprites, backgrounds, num_backgrounds, num_themes);
}

LIBENV_API int64_t procgen_atlas_host(const char *env_name, const char *resource_root, uint32_t *pixels,
                                      int64_t capacity, struct pg_image *sprites, struct pg_image *backgrounds,
                                      int32_t *num_backgrounds, int32_t *num_themes) {
    std::vector<int> gids;
    for (const std::string &nm : split_names(env_name ? env_name : "")) {
        int g = game_id(nm);
        if (g < 0) return -PG_ERR_BAD_OPTION;
        gids.push_back(g);
    }
    PGAtlasHost at;
    std::string err, root = resource_root && resource_root[0] ? resource_root : pg_default_asset_root();
    if (!pg_atlas_load(root, gids, &at, &err)) {
        g_last_make_error = err;
        return -PG_ERR_NO_ATLAS;
    }
    if (pixels && capacity >= (int64_t)at.pixels.size()) memcpy(pixels, at.pixels.data(), at.pixels.size() * 4);
    if (sprites) memcpy(sprites, at.sprites.data(), at.sprites.size() * 4);
    if (backgrounds) memcpy(backgrounds, at.backgrounds.data(), at.backgrounds.size() * 4);
    if (num_backgrounds) memcpy(num_backgrounds, at.num_backgrounds.data(), at.num_backgrounds.size() * 4);
    if (num_themes) memcpy(num_themes, at.num_themes.data(), at.num_themes.size() * 4);
    return (int64_t)at.pixels.size();
}

}  // extern "C"

namespace {
int upload_atlas(VecEnv *v, const uint32_t *pixels, int64_t num_pixels, const pg_image *sprites,
                 const pg_image *backgrounds, const int32_t *num_backgrounds, const int32_t *num_themes) {
    for (int g : v->games)
        if (num_backgrounds[g] <= 0 || num_backgrounds[g] > PG_MAX_BG)
            return fail(v, PG_ERR_NO_ATLAS, "bad background count for a game of the batch");
    if (num_pixels <= 0 || num_pixels >= 0xffffffffLL) return fail(v, PG_ERR_NO_ATLAS, "bad atlas pixel count");
    const size_t slots = (size_t)PG_NUM_GAMES * PG_NUM_SLOTS, bgs = (size_t)PG_NUM_GAMES * PG_MAX_BG;
    for (void *old : {(void *)v->d_pixels, (void *)v->d_sprites, (void *)v->d_bgs, (void *)v->d_themes}) {
        if (!old) continue;
        for (size_t i = 0; i < v->allocs.size(); i++)
            if (v->allocs[i] == old) {
                (void)hipFree(old);
                v->allocs.erase(v->allocs.begin() + i);
                break;
            }
    }
    v->d_pixels = nullptr;
    v->d_sprites = v->d_bgs = v->d_themes = nullptr;
    v->atlas = false;
    if (dalloc(v, &v->d_pixels, (size_t)num_pixels) || dalloc(v, &v->d_sprites, slots * 4) ||
        dalloc(v, &v->d_bgs, bgs * 4) || dalloc(v, &v->d_themes, (size_t)PG_NUM_GAMES * 100))
        return -PG_ERR_HIP;
    HIPCHECK(copy_sync(v, v->d_pixels, pixels, (size_t)num_pixels * 4, hipMemcpyHostToDevice));
    HIPCHECK(copy_sync(v, v->d_sprites, sprites, slots * sizeof(pg_image), hipMemcpyHostToDevice));
    HIPCHECK(copy_sync(v, v->d_bgs, backgrounds, bgs * sizeof(pg_image), hipMemcpyHostToDevice));
    HIPCHECK(copy_sync(v, v->d_themes, num_themes, (size_t)PG_NUM_GAMES * 100 * 4, hipMemcpyHostToDevice));
    v->dev.pixels = v->d_pixels;
    v->dev.num_pixels = (uint32_t)num_pixels;
    v->dev.sprites = v->d_sprites;
    v->dev.backgrounds = v->d_bgs;
    v->dev.num_themes = v->d_themes;
    for (int g = 0; g < PG_NUM_GAMES; g++) v->dev.num_bg[g] = num_backgrounds[g];
    v->atlas = true;
    return 0;
}
} // namespace

extern "C" {

LIBENV_API int procgen_start(libenv_env *env) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    if (!v->atlas) return fail(v, PG_ERR_NO_ATLAS, "procgen_upload_atlas was not called");
    if (v->started) return 0;
    if (v->prefetch) HIPCHECK(hipMemsetAsync(v->dev.sp_count, 0, PG_NUM_GAMES * 4, v->stream)); // ring slot 0, every game
    for (size_t k = 0; k < v->games.size(); k++) {
        PG_POISON(v->stream);
        const bool pfk = v->prefetch && ((v->prefetch_games >> v->games[k]) & 1);
        PGDev dk = v->dev;
        if (!pfk) dk.sp_envs = nullptr;
        pg_launch_reset(&dk, v->games[k], v->list_of(k), v->count_of(), v->stream, 1, 0, -v->lag, v->games[k]);
        if (pfk) { // the spares of the first episodes (requested at act -lag, ring slot 0, usable from act 0)
            HIPCHECK(hipEventRecord(v->ev_reset[k], v->stream));
            HIPCHECK(hipStreamWaitEvent(v->pstreams[0], v->ev_reset[k], 0));
            pg_launch_reset(&v->dev, v->games[k], v->list_of(k), v->count_of(), v->pstreams[0], 2, 0, -v->lag, v->games[k]);
            HIPCHECK(hipEventRecord(v->ev_pre[0], v->pstreams[0]));
            v->ev_pre_set[0] = true;
        }
    }
    for (size_t k = 0; k < v->games.size(); k++) {
        PG_POISON(v->stream);
        pg_launch_render(&v->dev, v->games[k], v->list_of(k), v->count_of(), v->stream, 0, v->games[k]);
    }
    HIPCHECK(hipGetLastError());
    v->started = true;
    return 0;
}

LIBENV_API void libenv_set_buffers(libenv_env *env, struct libenv_buffers *bufs) {
    VecEnv *v = (VecEnv *)env;
    size_t n = (size_t)v->num_envs;
    v->ob_ptrs.assign(bufs->ob, bufs->ob + v->ob_types.size() * n);
    v->ac_ptrs.assign(bufs->ac, bufs->ac + v->ac_types.size() * n);
    v->info_ptrs.assign(bufs->info, bufs->info + v->info_types.size() * n);
    v->rew_host = bufs->rew;
    v->first_host = bufs->first;
    v->buffers_set = true;
    (void)hipSetDevice(v->device);
    register_buffers(v);
    // latent-state info tensors (grid_size, grid, agent_pos, exit_pos) are only filled by
    // maze/miner (maze.cpp:152-165, miner.cpp:378-396); zero them for the other games (copy_out
    // overwrites them every observe when a game of the batch has a latent state)
    for (size_t k = 3; k < v->info_types.size(); k++) {
        size_t bytes = v->info_types[k].dtype == LIBENV_DTYPE_UINT8 ? 1 : 4;
        for (int dd = 0; dd < v->info_types[k].ndim; dd++) bytes *= (size_t)v->info_types[k].shape[dd];
        for (size_t e = 0; e < n; e++) memset(v->info_ptrs[k * n + e], 0, bytes);
    }
    if (procgen_start(env) == 0) copy_out(v);
}

LIBENV_API void libenv_act(libenv_env *env) {
    VecEnv *v = (VecEnv *)env;
    size_t n = (size_t)v->num_envs;
    // each act keeps its own actions (the reference waits for the stepping threads before
    // reading them, vecgame.cpp:426-444): the previous upload must have read the staging buffer
    if (v->act_pending && hipEventSynchronize(v->act_copied) != hipSuccess) {
        fail(v, PG_ERR_HIP, "action upload wait failed");
        return;
    }
    for (size_t e = 0; e < n; e++) v->h_actions[e] = *(const int32_t *)v->ac_ptrs[e];
    if (hipMemcpyAsync(v->dev.actions, v->h_actions, n * 4, hipMemcpyHostToDevice, v->stream) != hipSuccess ||
        hipEventRecord(v->act_copied, v->stream) != hipSuccess) {
        fail(v, PG_ERR_HIP, "action upload failed");
        return;
    }
    v->act_pending = true;
    v->obs_early = v->direct && v->buffers_set && v->games.size() == 1 && !v->render_human;
    launch_step(v, 0, 0, 0);
    v->obs_early = false;
}

LIBENV_API void libenv_observe(libenv_env *env) {
    VecEnv *v = (VecEnv *)env;
    (void)hipSetDevice(v->device);
    if (v->buffers_set) copy_out(v);
    else hipStreamSynchronize(v->stream);
    check_device_errors(v);
}

LIBENV_API void libenv_close(libenv_env *env) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return;
    // every stream that may still run a kernel on the allocations (the level prefetch's side stream
    // is joined to the engine stream only lag acts later) drains before anything is freed
    for (auto &p : v->pstreams)
        if (p) (void)hipStreamSynchronize(p);
    for (auto &s : v->rstreams)
        if (s) (void)hipStreamSynchronize(s);
    for (auto &s : v->gstreams)
        if (s) (void)hipStreamSynchronize(s);
    if (v->cstream) (void)hipStreamSynchronize(v->cstream);
    if (v->hstream) (void)hipStreamSynchronize(v->hstream);
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    unregister_buffers(v);
    for (void *p : v->allocs) hipFree(p);
    if (v->d_digest) (void)hipFree(v->d_digest);
    if (v->pinned) (void)hipHostFree(v->pinned);
    if (v->h_actions) (void)hipHostFree(v->h_actions);
    if (v->act_copied) hipEventDestroy(v->act_copied);
    for (auto &e : v->ev)
        if (e) hipEventDestroy(e);
    for (auto &e : v->gdone)
        if (e) hipEventDestroy(e);
    for (auto &e : v->ev_stepped)
        if (e) hipEventDestroy(e);
    for (auto &e : v->ev_reset)
        if (e) hipEventDestroy(e);
    for (auto &e : v->ev_rendered)
        if (e) hipEventDestroy(e);
    if (v->ev_cdone) hipEventDestroy(v->ev_cdone);
    if (v->cstream) hipStreamDestroy(v->cstream);
    if (v->hstream) hipStreamDestroy(v->hstream);
    for (auto &e : v->hr_ev)
        if (e) hipEventDestroy(e);
    for (auto &s : v->rstreams)
        if (s) hipStreamDestroy(s);
    for (auto &p : v->pstreams)
        if (p) {
            (void)hipStreamSynchronize(p);
            hipStreamDestroy(p);
        }
    for (auto &e : v->ev_pre)
        if (e) hipEventDestroy(e);
    if (v->fork) hipEventDestroy(v->fork);
    for (auto &s : v->gstreams)
        if (s) hipStreamDestroy(s);
    if (v->stream) hipStreamDestroy(v->stream);
    delete v;
}

LIBENV_API int procgen_act_device(libenv_env *env, const int32_t *d_actions) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    if (d_actions != v->dev.actions)
        HIPCHECK(hipMemcpyAsync(v->dev.actions, d_actions, (size_t)v->num_envs * 4, hipMemcpyDeviceToDevice, v->stream));
    return launch_step(v, 0, 0, 0);
}

LIBENV_API int procgen_act_hashed(libenv_env *env, uint64_t seed, int32_t t) {
    if (!env) return -PG_ERR_BAD_OPTION;
    return launch_step((VecEnv *)env, 1, seed, t);
}

LIBENV_API int procgen_wait(libenv_env *env) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    HIPCHECK(hipSetDevice(v->device));
    HIPCHECK(hipStreamSynchronize(v->stream));
    check_device_errors(v);
    return v->error ? -v->error : 0;
}

LIBENV_API int procgen_device_buffers(libenv_env *env, struct pg_device_buffers *out) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    out->rgb = v->dev.rgb;
    out->rew = v->dev.rew;
    out->first = v->dev.first;
    out->prev_level_seed = v->dev.prev_level_seed;
    out->prev_level_complete = v->dev.prev_level_complete;
    out->level_seed = v->dev.level_seed;
    out->actions = v->dev.actions;
    out->stream = (void *)v->stream;
    return 0;
}

LIBENV_API int procgen_set_obs_buffer(libenv_env *env, void *d_rgb) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    v->dev.rgb = d_rgb ? (uint8_t *)d_rgb : v->own_rgb;
    return 0;
}

LIBENV_API int procgen_read_envs(libenv_env *env, const int32_t *env_ids, int count, uint8_t *rgb, float *rew,
                                 uint8_t *first, int32_t *prev_level_seed, uint8_t *prev_level_complete,
                                 int32_t *level_seed) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    HIPCHECK(hipSetDevice(v->device));
    for (int k = 0; k < count; k++) {
        size_t e = (size_t)env_ids[k];
        if (env_ids[k] < 0 || e >= (size_t)v->num_envs) return fail(v, PG_ERR_BAD_OPTION, "procgen_read_envs: bad env id");
        if (rgb) HIPCHECK(hipMemcpyAsync(rgb + (size_t)k * PG_OBS_BYTES, v->dev.rgb + e * PG_OBS_BYTES, PG_OBS_BYTES,
                                         hipMemcpyDeviceToHost, v->stream));
        if (rew) HIPCHECK(hipMemcpyAsync(rew + k, v->dev.rew + e, 4, hipMemcpyDeviceToHost, v->stream));
        if (first) HIPCHECK(hipMemcpyAsync(first + k, v->dev.first + e, 1, hipMemcpyDeviceToHost, v->stream));
        if (prev_level_seed)
            HIPCHECK(hipMemcpyAsync(prev_level_seed + k, v->dev.prev_level_seed + e, 4, hipMemcpyDeviceToHost, v->stream));
        if (prev_level_complete)
            HIPCHECK(hipMemcpyAsync(prev_level_complete + k, v->dev.prev_level_complete + e, 1, hipMemcpyDeviceToHost,
                                    v->stream));
        if (level_seed) HIPCHECK(hipMemcpyAsync(level_seed + k, v->dev.level_seed + e, 4, hipMemcpyDeviceToHost, v->stream));
    }
    HIPCHECK(hipStreamSynchronize(v->stream));
    return 0;
}

// procgen_read_outputs: one wave per env sums its 1,536 observation words times splitmix64(k) | 1
__device__ __forceinline__ uint64_t pg_mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
__global__ __launch_bounds__(64) void pg_obs_digest_kernel(const uint8_t *rgb, uint64_t *out, int n) {
    const int e = (int)blockIdx.x;
    if (e >= n) return;
    const uint64_t *w = reinterpret_cast<const uint64_t *>(rgb + (size_t)e * PG_OBS_BYTES);
    uint64_t acc = 0;
    for (int k = (int)threadIdx.x; k < PG_OBS_BYTES / 8; k += 64) acc += w[k] * (pg_mix64((uint64_t)k) | 1ull);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (threadIdx.x == 0) out[e] = acc;
}

LIBENV_API int procgen_read_outputs(libenv_env *env, uint64_t *obs_digest, float *rew, uint8_t *first,
                                    int32_t *prev_level_seed, uint8_t *prev_level_complete, int32_t *level_seed) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    HIPCHECK(hipSetDevice(v->device));
    const size_t n = (size_t)v->num_envs;
    if (obs_digest) {
        if (!v->d_digest && hipMalloc(&v->d_digest, n * 8) != hipSuccess) {
            v->d_digest = nullptr;
            return fail(v, PG_ERR_HIP, "procgen_read_outputs: out of device memory");
        }
        hipLaunchKernelGGL(pg_obs_digest_kernel, dim3((unsigned)n), dim3(64), 0, v->stream, v->dev.rgb, v->d_digest,
                           (int)n);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(obs_digest, v->d_digest, n * 8, hipMemcpyDeviceToHost, v->stream));
    }
    if (rew) HIPCHECK(hipMemcpyAsync(rew, v->dev.rew, n * 4, hipMemcpyDeviceToHost, v->stream));
    if (first) HIPCHECK(hipMemcpyAsync(first, v->dev.first, n, hipMemcpyDeviceToHost, v->stream));
    if (prev_level_seed) HIPCHECK(hipMemcpyAsync(prev_level_seed, v->dev.prev_level_seed, n * 4, hipMemcpyDeviceToHost, v->stream));
    if (prev_level_complete)
        HIPCHECK(hipMemcpyAsync(prev_level_complete, v->dev.prev_level_complete, n, hipMemcpyDeviceToHost, v->stream));
    if (level_seed) HIPCHECK(hipMemcpyAsync(level_seed, v->dev.level_seed, n * 4, hipMemcpyDeviceToHost, v->stream));
    HIPCHECK(hipStreamSynchronize(v->stream));
    return 0;
}

LIBENV_API int procgen_last_error(libenv_env *env) {
    if (!env) return g_last_make_error.empty() ? 0 : PG_ERR_BAD_OPTION;
    return ((VecEnv *)env)->error;
}

LIBENV_API const char *procgen_error_string(libenv_env *env) {
    if (!env) return g_last_make_error.c_str();
    return ((VecEnv *)env)->error_msg.c_str();
}

LIBENV_API int procgen_set_timing(libenv_env *env, int enabled) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    v->timing = enabled != 0;
    v->t_used = 0;
    return 0;
}

// Averages over the steps timed since procgen_set_timing(env, 1), ms:
//   out[0] step kernel, out[1] reset kernel, out[2] render kernel -- each the SUM over the
//          batch's games (a mixed batch runs the games' chains concurrently on their own streams,
//          so these sums can exceed the step's wall time; a single game's reset runs on a side
//          stream concurrently with the render of the envs that did not finish, and its render
//          time is both passes);
//   out[3] wall span of the whole step on the env's stream (before the fork -> after the join);
//   out[4 + 3g .. 6 + 3g] step / reset / render of game slot g (v->games order).
LIBENV_API int procgen_kernel_times(libenv_env *env, float *out, int n) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    // per chain (a mixed batch's games, or a single game's parts: averaged over the parts, i.e. the
    // mean duration of one launch over one part's envs)
    const size_t G = v->games.size(), C = v->chains(), per = PG_EV_G * C + 2;
    const double wpart = G == 1 ? 1.0 / (double)C : 1.0;
    std::vector<double> sum(4 + 3 * G, 0.0);
    if (v->t_used > 0) {
        HIPCHECK(hipStreamSynchronize(v->stream));
        for (int k = 0; k < v->t_used; k++) {
            hipEvent_t *base = &v->ev[(size_t)k * per];
            for (size_t ch = 0; ch < C; ch++) {
                const size_t g = G > 1 ? ch : 0;
                hipEvent_t *e = base + PG_EV_G * ch;
                float a = 0, b = 0, c1 = 0, c2 = 0;
                HIPCHECK(hipEventElapsedTime(&a, e[0], e[1]));  // step
                HIPCHECK(hipEventElapsedTime(&b, e[2], e[3]));  // reset (side stream)
                if (G == 1) HIPCHECK(hipEventElapsedTime(&c1, e[1], e[4])); // render of the unfinished envs
                HIPCHECK(hipEventElapsedTime(&c2, e[5], e[6])); // render of the finished envs
                const double c = (double)(c1 + c2) * wpart;
                sum[0] += a * wpart; sum[1] += b * wpart; sum[2] += c;
                sum[4 + 3 * g] += a * wpart; sum[5 + 3 * g] += b * wpart; sum[6 + 3 * g] += c;
            }
            float w = 0;
            HIPCHECK(hipEventElapsedTime(&w, base[PG_EV_G * C], base[PG_EV_G * C + 1]));
            sum[3] += w;
        }
    }
    for (int i = 0; i < n && i < (int)sum.size(); i++) out[i] = v->t_used ? (float)(sum[i] / v->t_used) : 0.f;
    return v->t_used;
}

// Chains a single-game act is split into (PROCGEN_MI355X_PARTS; 1 for mixed batches).
LIBENV_API int procgen_num_parts(libenv_env *env) { return env ? ((VecEnv *)env)->parts : 0; }

// Diagnostic builds (make PROFILE=1): per-phase s_memtime cycle sums over all envs since
// creation; out[0..7] step-kernel phases, out[8..15] render-kernel phases.
LIBENV_API int procgen_profile_read(libenv_env *env, uint64_t *out) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    HIPCHECK(hipStreamSynchronize(v->stream));
    std::vector<uint64_t> h((size_t)v->num_envs * 16);
    HIPCHECK(copy_sync(v, h.data(), v->dev.prof, h.size() * 8, hipMemcpyDeviceToHost));
    for (int k = 0; k < 16; k++) out[k] = 0;
    for (size_t e = 0; e < (size_t)v->num_envs; e++)
        for (int k = 0; k < 16; k++) out[k] += h[e * 16 + k];
    return 0;
}

// the whole per-env diagnostic buffer, [num_envs][16] words (PG_PROFILE phase sums or PG_CENSUS
// wave records: words 0-2 step, 8-10 render)
LIBENV_API int procgen_profile_raw(libenv_env *env, uint64_t *out) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    HIPCHECK(hipStreamSynchronize(v->stream));
    HIPCHECK(copy_sync(v, out, v->dev.prof, (size_t)v->num_envs * 16 * 8, hipMemcpyDeviceToHost));
    return 0;
}

LIBENV_API int procgen_debug_env(libenv_env *env, int env_idx, void *out, int length) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    if (env_idx < 0 || env_idx >= v->num_envs || length < (int)sizeof(PGEnv)) return -1;
    HIPCHECK(hipStreamSynchronize(v->stream));
    HIPCHECK(copy_sync(v, out, v->dev.envs + env_idx, sizeof(PGEnv), hipMemcpyDeviceToHost));
    return (int)sizeof(PGEnv);
}

// ---- snapshots: this build's own per-env format (PGEnv + entity planes + grid + generators)
// [u32 magic][u32 version][PGEnv][num_ents x PG_NF words][num_tail x PG_NF words (the reserved top
// slots, starpilot's spawners)][grid cells int16][2 x 625 mt words][END]
static const uint32_t STATE_MAGIC = 0x50474d33u; // "PGM3"
// largest main_width x main_height of each game over its distribution modes (choose_world_dim of
// bigfish.cpp:27, bossfight.cpp:65, caveflyer.cpp:128-142, chaser.cpp:135-152, climber.cpp:230-232,
// coinrun.cpp:54, dodgeball.cpp:248-256, fruitbot.cpp:147-154, heist.cpp:98-112, jumper.cpp:204-218,
// leaper.cpp:103-115, maze.cpp:44-56, miner.cpp:127-138, ninja.cpp:36, plunder.cpp:37, starpilot.cpp:52)
static const int32_t END_OF_BUFFER = (int32_t)0xCAFECAFE;

// Bounds of every PGEnv member a kernel uses as an array / LDS / table index (shared by the own
// format and the upstream format, which reaches the device through procgen_set_snapshot too).
// Returns the reason a state is rejected, or null.
static const char *validate_env(const VecEnv *v, const PGEnv &s) {
    if (s.num_ents < 0 || s.num_tail < 0 || s.num_ents + s.num_tail > PG_CAP || s.main_width < 0 ||
        s.main_height < 0 || s.main_width > pg_game_max_w(s.game_id) || s.main_height > pg_game_max_h(s.game_id))
        return "set_state: entity count or world size out of range for the game";
    if (s.rg_mti < 0 || s.rg_mti > PG_MT_N || s.lsg_mti < 0 || s.lsg_mti > PG_MT_N)
        return "set_state: RandGen position out of range";
    const int nbg = v->dev.num_bg[s.game_id];
    if (s.background_index < 0 || s.background_index >= PG_MAX_BG || (nbg > 0 && s.background_index >= nbg))
        return "set_state: background_index out of range for the game's backgrounds";
    if (s.game_id == PG_GAME_LEAPER && (s.num_road_lanes < 0 || s.num_road_lanes > 5 || s.num_water_lanes < 0 ||
                                        s.num_water_lanes > 5))
        return "set_state: leaper lane count out of range";
    if (s.game_id == PG_GAME_BOSSFIGHT &&
        (s.gs.bf.num_rounds < 1 || s.gs.bf.num_rounds > 5 || s.gs.bf.round_num < 0 || s.gs.bf.attack_mode < 0 ||
         s.gs.bf.attack_mode > 3))
        return "set_state: bossfight round counts out of range";
    if (s.game_id == PG_GAME_HEIST && (s.num_keys < 0 || s.num_keys > 31))
        return "set_state: heist key count out of range";
    if (s.game_id == PG_GAME_PLUNDER) {
        const auto &p = s.gs.pl;
        if (p.num_lanes < 0 || p.num_lanes > 5 || p.num_current_ship_types < 1 || p.num_current_ship_types > 6)
            return "set_state: plunder lane / ship-type count out of range";
        for (int i = 0; i < 6; i++)
            if (((p.perm >> (4 * i)) & 15u) > 5) return "set_state: plunder image permutation out of range";
    }
    return nullptr;
}

LIBENV_API int procgen_get_snapshot(libenv_env *env, int env_idx, char *data, int length) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    if (env_idx < 0 || env_idx >= v->num_envs) return -1;
    if (hipStreamSynchronize(v->stream) != hipSuccess) return -1;
    PGEnv s;
    if (copy_sync(v, &s, v->dev.envs + env_idx, sizeof(s), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    size_t ents = (size_t)s.num_ents, tail = (size_t)s.num_tail;
    size_t cells = (size_t)s.main_width * s.main_height;
    const size_t bgb = v->dev.gen_bg ? (size_t)PG_GEN_BG_PX * 4 : 0; // the env's generated background
    size_t need = 8 + sizeof(PGEnv) + (ents + tail) * PG_NF * 4 + cells * 2 + 2 * PG_MT_WORDS * 4 + bgb + 4;
    if ((size_t)length < need) return -1;
    char *p = data;
    memcpy(p, &STATE_MAGIC, 4); p += 4;
    uint32_t ver = 2; memcpy(p, &ver, 4); p += 4;
    memcpy(p, &s, sizeof(s)); p += sizeof(s);
    for (int f = 0; f < PG_NF; f++) {
        if (ents && copy_sync(v, p, v->dev.ents + pg_ent_index(env_idx, f, 0), ents * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        p += ents * 4;
    }
    for (int f = 0; f < PG_NF; f++) {
        if (tail && copy_sync(v, p, v->dev.ents + pg_ent_index(env_idx, f, (int)(PG_CAP - tail)), tail * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        p += tail * 4;
    }
    if (cells && copy_sync(v, p, v->dev.grid + (size_t)env_idx * PG_GRID_MAX, cells * 2, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    p += cells * 2;
    if (copy_sync(v, p, v->dev.mt + (size_t)env_idx * 2 * PG_MT_WORDS, 2 * PG_MT_WORDS * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    p += 2 * PG_MT_WORDS * 4;
    if (bgb && copy_sync(v, p, v->dev.gen_bg + (size_t)env_idx * PG_GEN_BG_PX, bgb, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    p += bgb;
    memcpy(p, &END_OF_BUFFER, 4); p += 4;
    return (int)(p - data);
}

static void invalidate_spare(VecEnv *v, int env_idx);

LIBENV_API void procgen_set_snapshot(libenv_env *env, int env_idx, const char *data, int length) {
    VecEnv *v = (VecEnv *)env;
    if (env_idx < 0 || env_idx >= v->num_envs || length < (int)(8 + sizeof(PGEnv) + 4)) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: bad arguments");
        return;
    }
    invalidate_spare(v, env_idx);
    hipStreamSynchronize(v->stream);
    const char *p = data;
    uint32_t magic, ver;
    memcpy(&magic, p, 4); p += 4;
    memcpy(&ver, p, 4); p += 4;
    PGEnv s;
    memcpy(&s, p, sizeof(s)); p += sizeof(s);
    if (magic != STATE_MAGIC || ver != 2) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: not a state of this build");
        return;
    }
    // the slot's game must match (the reference: fassert(game_name == b->read_string()),
    // game.cpp:259), and every size must be one that game's kernels are built for
    if (s.game_id != v->game_of(env_idx)) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: the state belongs to another game than this env slot");
        return;
    }
    if (const char *why = validate_env(v, s)) {
        fail(v, PG_ERR_BAD_OPTION, why);
        return;
    }
    size_t ents = (size_t)s.num_ents, tail = (size_t)s.num_tail, cells = (size_t)s.main_width * s.main_height;
    const size_t bgb = v->dev.gen_bg ? (size_t)PG_GEN_BG_PX * 4 : 0;
    size_t need = 8 + sizeof(PGEnv) + (ents + tail) * PG_NF * 4 + cells * 2 + 2 * PG_MT_WORDS * 4 + bgb + 4;
    int32_t end = 0;
    if ((size_t)length < need || cells > PG_GRID_MAX) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: truncated state");
        return;
    }
    memcpy(&end, data + need - 4, 4);
    if (end != END_OF_BUFFER) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: missing END_OF_BUFFER");
        return;
    }
    // a restored env draws with the options its state carries: the register-frame render serves
    // centred, non-monochrome frames only (pg_render.hip rf_game), so its game falls back otherwise
    {
        // a game stays on the register-frame render while every live env of it is one the kernel serves
        // (pg_rf_serves): a restored state carries its own options (game.cpp:266), which then persist
        const uint8_t bad = pg_rf_serves(s) ? 0 : 1;
        if (bad != v->rf_bad[env_idx]) {
            v->rf_bad_n[s.game_id] += bad ? 1 : -1;
            v->rf_bad[env_idx] = bad;
        }
        int off = 0;
        for (int g = 0; g < PG_NUM_GAMES; g++)
            if (v->rf_bad_n[g] > 0) off |= 1 << g;
        v->dev.render_rf = v->rf_make & ~off;
    }
    s.grid8_ok = 0; // the int8 mirror is rebuilt at the next reset; until then the step reads int16
    copy_sync(v, v->dev.envs + env_idx, &s, sizeof(s), hipMemcpyHostToDevice);
    const char *ent_base = p; // the live entity planes
    for (int f = 0; f < PG_NF; f++) {
        if (ents) copy_sync(v, v->dev.ents + pg_ent_index(env_idx, f, 0), p, ents * 4, hipMemcpyHostToDevice);
        p += ents * 4;
    }
    for (int f = 0; f < PG_NF; f++) {
        if (tail) copy_sync(v, v->dev.ents + pg_ent_index(env_idx, f, (int)(PG_CAP - tail)), p, tail * 4, hipMemcpyHostToDevice);
        p += tail * 4;
    }
    if (cells) copy_sync(v, v->dev.grid + (size_t)env_idx * PG_GRID_MAX, p, cells * 2, hipMemcpyHostToDevice);
    if (v->has_latent && (s.game_id == PG_GAME_MAZE || s.game_id == PG_GAME_MINER)) { // latent mirrors the state
        std::vector<int32_t> lat(PG_LATENT_N, 0);
        lat[0] = s.main_width;
        lat[1] = s.main_height;
        for (size_t k = 0; k < cells && k < PG_LATENT_GRID; k++) {
            int16_t cv;
            memcpy(&cv, p + 2 * k, 2);
            lat[2 + k] = cv;
        }
        float ax, ay;
        memcpy(&ax, ent_base + (size_t)F_X * ents * 4, 4); // entity 0 = the agent
        memcpy(&ay, ent_base + (size_t)F_Y * ents * 4, 4);
        if (s.agent_erased) {
            ax = s.ghost_x;
            ay = s.ghost_y;
        }
        lat[2 + PG_LATENT_GRID] = (ents || s.agent_erased) ? (int)ax : 0;
        lat[3 + PG_LATENT_GRID] = (ents || s.agent_erased) ? (int)ay : 0;
        if (s.game_id == PG_GAME_MINER) { // the first EXIT entity (type 6)
            for (size_t e = 0; e < ents; e++) {
                int32_t ty;
                float ex, ey;
                memcpy(&ty, ent_base + (size_t)F_TYPE * ents * 4 + e * 4, 4);
                if (ty != 6) continue;
                memcpy(&ex, ent_base + (size_t)F_X * ents * 4 + e * 4, 4);
                memcpy(&ey, ent_base + (size_t)F_Y * ents * 4 + e * 4, 4);
                lat[4 + PG_LATENT_GRID] = (int)ex;
                lat[5 + PG_LATENT_GRID] = (int)ey;
                break;
            }
        }
        copy_sync(v, v->dev.latent + (size_t)env_idx * PG_LATENT_N, lat.data(), PG_LATENT_N * 4, hipMemcpyHostToDevice);
    }
    p += cells * 2;
    copy_sync(v, v->dev.mt + (size_t)env_idx * 2 * PG_MT_WORDS, p, 2 * PG_MT_WORDS * 4, hipMemcpyHostToDevice);
    p += 2 * PG_MT_WORDS * 4;
    if (bgb) copy_sync(v, v->dev.gen_bg + (size_t)env_idx * PG_GEN_BG_PX, p, bgb, hipMemcpyHostToDevice);
    // the reference re-observes after set_state (vecgame.cpp:503); rendering all envs is
    // harmless (render is a pure function of state)
    // ... and Game::observe (game.cpp:173-191) reports the restored step data: reward, done (first),
    // prev_level_seed, prev_level_complete, level_seed
    {
        const float rew = s.sd_reward;
        const uint8_t first = (uint8_t)(s.sd_done != 0), plc = (uint8_t)(s.sd_level_complete != 0);
        copy_sync(v, v->dev.rew + env_idx, &rew, 4, hipMemcpyHostToDevice);
        copy_sync(v, v->dev.first + env_idx, &first, 1, hipMemcpyHostToDevice);
        copy_sync(v, v->dev.prev_level_seed + env_idx, &s.prev_level_seed, 4, hipMemcpyHostToDevice);
        copy_sync(v, v->dev.prev_level_complete + env_idx, &plc, 1, hipMemcpyHostToDevice);
        copy_sync(v, v->dev.level_seed + env_idx, &s.current_level_seed, 4, hipMemcpyHostToDevice);
    }
    for (size_t k = 0; k < v->games.size(); k++)
        pg_launch_render(&v->dev, v->games[k], v->list_of(k), v->count_of(), v->stream, 0, v->games[k]);
    hipStreamSynchronize(v->stream);
    v->obs_inflight = false; // an act's early obs DMA predates this frame: observe copies again
}

// MinerGame::game_set_state (miner.cpp:423-449; the fork's JS binding's setState,
// cheerpgame.cpp:54-56) on one env, through this build's own snapshot: the grid values are
// written cell by cell (a DEAD_PLAYER cell sets `died`); if `died`, the PLAYER entity leaves the
// list (the agent's state stays addressable, as the reference's `agent` shared_ptr); else the agent
// goes to (agent_x + .5, agent_y + .5); the first EXIT entity to (exit_x + .5, exit_y + .5).  The
// frame is re-rendered, as after set_state.  Where the reference would crash (another game, a grid
// larger than the world, no EXIT entity) this fails with a sticky error instead.
LIBENV_API int procgen_set_latent_state(libenv_env *env, int env_idx, const int32_t *grid, int grid_width,
                                        int grid_height, int agent_x, int agent_y, int exit_x, int exit_y) {
    VecEnv *v = (VecEnv *)env;
    if (!v) return -PG_ERR_BAD_OPTION; // a closed / never-made env
    if (!v || env_idx < 0 || env_idx >= v->num_envs || (!grid && grid_width * grid_height > 0))
        return fail(v, PG_ERR_BAD_OPTION, "set_latent_state: bad arguments");
    if (v->game_of(env_idx) != PG_GAME_MINER)
        return fail(v, PG_ERR_BAD_OPTION, "set_latent_state: only miner has a game_set_state (miner.cpp:423-449)");
    const size_t bgb = v->dev.gen_bg ? (size_t)PG_GEN_BG_PX * 4 : 0;
    const size_t cap = 8 + sizeof(PGEnv) + (size_t)PG_CAP * PG_NF * 4 + (size_t)PG_GRID_MAX * 2 + 2 * PG_MT_WORDS * 4 +
                       bgb + 4;
    std::vector<char> buf(cap);
    if (procgen_get_snapshot(env, env_idx, buf.data(), (int)cap) < 0)
        return fail(v, PG_ERR_BAD_OPTION, "set_latent_state: could not read the env's state");
    PGEnv s;
    memcpy(&s, buf.data() + 8, sizeof(s));
    size_t ents = (size_t)s.num_ents;
    const size_t tail = (size_t)s.num_tail, cells = (size_t)s.main_width * s.main_height;
    if (grid_width < 0 || grid_height < 0 || (size_t)grid_width * grid_height > cells)
        return fail(v, PG_ERR_BAD_OPTION, "set_latent_state: grid larger than the world");
    const char *P = buf.data() + 8 + sizeof(PGEnv);
    std::vector<std::vector<int32_t>> planes(PG_NF, std::vector<int32_t>(ents));
    for (int f = 0; f < PG_NF; f++)
        if (ents) memcpy(planes[f].data(), P + (size_t)f * ents * 4, ents * 4);
    const char *T = P + (size_t)PG_NF * ents * 4; // tail planes, then grid, then generators
    std::vector<int16_t> cellv(cells);
    if (cells) memcpy(cellv.data(), T + (size_t)PG_NF * tail * 4, cells * 2);
    const char *MT = T + (size_t)PG_NF * tail * 4 + cells * 2;
    auto find_type = [&](int ty) {
        for (size_t e = 0; e < ents; e++)
            if (planes[F_TYPE][e] == ty) return (long)e;
        return -1L;
    };
    if (find_type(6) < 0) return fail(v, PG_ERR_BAD_OPTION, "set_latent_state: the env has no EXIT entity");
    for (int idx = 0; idx < grid_width * grid_height; idx++) {
        const int obj = grid[idx];
        if (obj < -32768 || obj > 32767) return fail(v, PG_ERR_BAD_OPTION, "set_latent_state: grid value out of range");
        cellv[idx] = (int16_t)obj;
        if (obj == 12) s.died = 1; // DEAD_PLAYER
    }
    auto fbits = [](float x) { int32_t b; memcpy(&b, &x, 4); return b; };
    auto bitsf = [](int32_t b) { float x; memcpy(&x, &b, 4); return x; };
    if (s.died) {
        const long a = find_type(0); // PLAYER: entity 0 while the agent is listed
        if (a == 0 && !s.agent_erased) {
            s.agent_erased = 1;
            s.ghost_x = bitsf(planes[F_X][0]); s.ghost_y = bitsf(planes[F_Y][0]);
            s.ghost_vx = bitsf(planes[F_VX][0]); s.ghost_vy = bitsf(planes[F_VY][0]);
            s.ghost_rx = bitsf(planes[F_RX][0]); s.ghost_ry = bitsf(planes[F_RY][0]);
            for (int f = 0; f < PG_NF; f++) planes[f].erase(planes[f].begin());
            ents--;
        }
    } else if (s.agent_erased) {
        s.ghost_x = agent_x + 0.5f;
        s.ghost_y = agent_y + 0.5f;
    } else if (ents > 0) {
        planes[F_X][0] = fbits(agent_x + 0.5f);
        planes[F_Y][0] = fbits(agent_y + 0.5f);
    }
    const long ex = find_type(6);
    planes[F_X][ex] = fbits(exit_x + 0.5f);
    planes[F_Y][ex] = fbits(exit_y + 0.5f);
    s.num_ents = (int32_t)ents;
    std::vector<char> out(cap);
    char *q = out.data();
    memcpy(q, buf.data(), 8); q += 8;
    memcpy(q, &s, sizeof(s)); q += sizeof(s);
    for (int f = 0; f < PG_NF; f++) {
        if (ents) memcpy(q, planes[f].data(), ents * 4);
        q += ents * 4;
    }
    memcpy(q, T, (size_t)PG_NF * tail * 4); q += (size_t)PG_NF * tail * 4;
    if (cells) memcpy(q, cellv.data(), cells * 2);
    q += cells * 2;
    memcpy(q, MT, 2 * PG_MT_WORDS * 4); q += 2 * PG_MT_WORDS * 4;
    if (bgb) memcpy(q, MT + 2 * PG_MT_WORDS * 4, bgb); // the generated background, unchanged
    q += bgb;
    memcpy(q, &END_OF_BUFFER, 4); q += 4;
    procgen_set_snapshot(env, env_idx, out.data(), (int)(q - out.data()));
    return v->error ? -v->error : 0;
}

// Pinning helper (tests/test_state_cpu.py): RandGen::serialize's text of 624 MT words + position,
// as get_state writes it.  Returns the length, or -1 when `out` is too small.
LIBENV_API int procgen_mt_text(const uint32_t *words, int pos, char *out, int length) {
    const std::string t = pg_mt_text(words, pos);
    if ((int)t.size() > length) return -1;
    memcpy(out, t.data(), t.size());
    return (int)t.size();
}

// ---- get_state / set_state (vecgame.cpp:485-505) in the upstream byte format (pg_state.cpp)
static const size_t SNAP_CAP = 8 + sizeof(PGEnv) + (size_t)PG_CAP * PG_NF * 4 + (size_t)PG_GRID_MAX * 2 +
                               2 * PG_MT_WORDS * 4 + (size_t)PG_GEN_BG_PX * 4 + 4;

static int read_host_env(VecEnv *v, int env_idx, HostEnv &h) {
    std::vector<char> buf(SNAP_CAP);
    if (procgen_get_snapshot(v, env_idx, buf.data(), (int)SNAP_CAP) < 0) return -1;
    const char *p = buf.data() + 8;
    memcpy(&h.s, p, sizeof(PGEnv)); p += sizeof(PGEnv);
    const size_t ents = (size_t)h.s.num_ents, tail = (size_t)h.s.num_tail;
    const size_t cells = (size_t)h.s.main_width * h.s.main_height;
    for (int f = 0; f < PG_NF; f++) {
        h.ent[f].resize(ents);
        if (ents) memcpy(h.ent[f].data(), p, ents * 4);
        p += ents * 4;
    }
    for (int f = 0; f < PG_NF; f++) {
        h.tail[f].resize(tail);
        if (tail) memcpy(h.tail[f].data(), p, tail * 4);
        p += tail * 4;
    }
    h.cells.resize(cells);
    if (cells) memcpy(h.cells.data(), p, cells * 2);
    p += cells * 2;
    memcpy(h.mt, p, sizeof(h.mt));
    return 0;
}

// An env whose state the host replaced has no valid spare (its level-seed generator may differ)
static void invalidate_spare(VecEnv *v, int env_idx) {
    if (v->prefetch) (void)hipMemsetAsync(v->dev.sp_gen + env_idx, 0x80, 4, v->stream);
}

static void write_host_env(VecEnv *v, int env_idx, const HostEnv &h) {
    invalidate_spare(v, env_idx);
    std::vector<char> buf;
    buf.reserve(SNAP_CAP);
    auto put = [&](const void *d, size_t n) { buf.insert(buf.end(), (const char *)d, (const char *)d + n); };
    const uint32_t ver = 2;
    put(&STATE_MAGIC, 4);
    put(&ver, 4);
    put(&h.s, sizeof(PGEnv));
    for (int f = 0; f < PG_NF; f++) put(h.ent[f].data(), (size_t)h.s.num_ents * 4);
    for (int f = 0; f < PG_NF; f++) put(h.tail[f].data(), (size_t)h.s.num_tail * 4);
    put(h.cells.data(), h.cells.size() * 2);
    put(h.mt, sizeof(h.mt));
    put(&END_OF_BUFFER, 4);
    procgen_set_snapshot(v, env_idx, buf.data(), (int)buf.size());
}

LIBENV_API int get_state(libenv_env *env, int env_idx, char *data, int length) {
    VecEnv *v = (VecEnv *)env;
    if (!v || env_idx < 0 || env_idx >= v->num_envs || !data) return -1;
    if (v->gen_assets) // BasicAbstractGame::serialize fasserts !use_generated_assets (basic-abstract-game.cpp:1185)
        return fail(v, PG_ERR_BAD_OPTION, "get_state: states of use_generated_assets envs are not serializable");
    HostEnv h;
    if (read_host_env(v, env_idx, h) < 0) return -1;
    std::vector<char> out;
    pg_state_write(h, out);
    if (out.size() > (size_t)length) return -1; // the reference fasserts (buffer.h:96)
    memcpy(data, out.data(), out.size());
    return (int)out.size();
}

LIBENV_API void set_state(libenv_env *env, int env_idx, char *data, int length) {
    VecEnv *v = (VecEnv *)env;
    if (!v || env_idx < 0 || env_idx >= v->num_envs || !data || length < 0) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: bad arguments");
        return;
    }
    if (v->gen_assets) { // BasicAbstractGame::deserialize fasserts !use_generated_assets (:1240)
        fail(v, PG_ERR_BAD_OPTION, "set_state: use_generated_assets envs have no serialized state");
        return;
    }
    HostEnv h;
    if (read_host_env(v, env_idx, h) < 0) {
        fail(v, PG_ERR_BAD_OPTION, "set_state: could not read the env's state");
        return;
    }
    std::string err;
    if (!pg_state_read(data, (size_t)length, h, err)) { // the reference fasserts
        fail(v, PG_ERR_BAD_OPTION, err.c_str()); // copied into the env's error message
        return;
    }
    write_host_env(v, env_idx, h);
}

} // extern "C"
