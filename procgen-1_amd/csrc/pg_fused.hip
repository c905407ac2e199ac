// pg_fused.hip -- Game::step + Game::observe of one env in one wave (game.cpp:136-191): the step
// kernel's step_env followed, for an env whose episode did not end, by the register-frame render
// (rf_render_env) of the state the wave has just written.  One launch replaces the step launch and the
// render launch of the envs that did not finish (pg_render_kernel mode 1): no kernel boundary between
// them, so a wave renders as soon as its own env has stepped (the step launch's tail of slow envs is
// filled by other envs' renders instead of idling the chip), and the render's PGEnv / entity-plane
// reads hit what the step just wrote.  The envs whose episode ended are reset afterwards (the reset
// kernel drains the queue the steps filled) and rendered then (pg_launch_render mode 2), as before.
// The step's and the render's LDS share one buffer: the render's tables are built after the step's
// last LDS access (a wave barrier between them).
#define PG_FUSED_TU
#include "pg_step.hip"
#include "pg_render.hip"

namespace {

// the step's LDS arrays (pg_step_kernel) carved from one buffer, 16-B aligned each
constexpr int fa16(int x) { return (x + 15) & ~15; }
template <int G>
struct FusedLds {
    static constexpr int MT = 0;
    static constexpr int GRID = MT + fa16(PG_MT_N * 4);
    static constexpr int IBOX = GRID + fa16(PG_GRID_MAX);
    static constexpr int LIST = IBOX + fa16((pl_smart<G>() ? 64 : 1) * 16);
    static constexpr int SLIST = LIST + fa16(PG_CAP * 2);
    static constexpr int PSTK = SLIST + fa16(64 * 2);
    static constexpr int IINFO = PSTK + fa16(((scan_needed<G>(true) || scan_needed<G>(false)) ? 10 * 5 : 1) * 4);
    static constexpr int MOVED = IINFO + fa16((pl_smart<G>() ? 64 : 1) * 4);
    static constexpr int STEP_BYTES = MOVED + fa16(G == PG_GAME_MINER ? 35 * 35 : 1);
    static constexpr int TAB = 0;
    static constexpr int DESC = fa16(rf_tab_bytes<G>());
    static constexpr int RDESC = DESC + 32 * rf_dcap<G>();
    static constexpr int RENDER_BYTES = RDESC + 96 * rf_rcap<G>();
    static constexpr int BYTES = STEP_BYTES > RENDER_BYTES ? STEP_BYTES : RENDER_BYTES;
};

// The step kernel's launch order and slow-env bookkeeping (pg_step_kernel) around step_env, then the
// render of the stepped env when its episode continues.
template <int G>
__global__ __launch_bounds__(64, STEP_WAVES) void pg_fused_kernel(PGDev d, const int32_t *env_list, int n, int parity,
                                                                  int use_hash, uint64_t hash_seed, int32_t hash_t,
                                                                  int slot) {
    if constexpr (rf_game<G>()) {
        using F = FusedLds<G>;
        __shared__ __attribute__((aligned(16))) uint8_t lds[F::BYTES];
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
        const StepLds L{reinterpret_cast<uint32_t *>(lds + F::MT), reinterpret_cast<int16_t *>(lds + F::LIST),
                        reinterpret_cast<int16_t *>(lds + F::SLIST), reinterpret_cast<float4 *>(lds + F::IBOX),
                        reinterpret_cast<float *>(lds + F::PSTK), reinterpret_cast<int *>(lds + F::IINFO),
                        reinterpret_cast<int8_t *>(lds + F::GRID), lds + F::MOVED};
        const uint64_t t0 = wall_clock64();
        bool done = false;
        const bool predicted = step_env<G>(d, env, L, use_hash, hash_seed, hash_t, slot, &done);
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
        if (done) return; // rendered after its reset (pg_launch_render mode 2)
        wave_sync(); // the step's LDS is dead: the render's tables take it
        rf_render_env<G>(game_view(d, G), env, lds + F::TAB, reinterpret_cast<int4 *>(lds + F::DESC),
                         reinterpret_cast<int4 *>(lds + F::RDESC));
    }
}

} // namespace

// Step + render of the envs that did not finish, for the games the register-frame render serves
// (returns -1 for the others: the caller launches step and render separately).
extern "C" int pg_launch_fused(const PGDev *d, int game, const int32_t *env_list, int count, hipStream_t s, int use_hash,
                               uint64_t seed, int32_t t, int parity, int slot) {
    if (count <= 0) return 0;
#define PG_CASE(G)                                                                                             \
    case G:                                                                                                    \
        if (!rf_game<G>()) return -1;                                                                          \
        hipLaunchKernelGGL(pg_fused_kernel<G>, dim3(count + (count < PG_HEAVY_CAP ? count : PG_HEAVY_CAP)), dim3(64), 0, s, \
                           *d, env_list, count, parity, use_hash, seed, t, slot);                              \
        return 0;
    switch (game) {
        PG_CASE(PG_GAME_COINRUN)
    default: return -1;
    }
#undef PG_CASE
}
