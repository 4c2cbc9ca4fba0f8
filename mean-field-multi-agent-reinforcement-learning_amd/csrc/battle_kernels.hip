// battle_kernels.hip -- HIP/CDNA4 (gfx950) kernels of the Battle gridworld.
//
// Every kernel owns whole environments: workgroup b works on env b (or on a chunk of
// agents of env b for the observation kernel), so no inter-workgroup communication is
// ever needed.  The order-dependent parts of GridWorld::step (LCG attack shuffle,
// attack resolution, first-come move resolution -- GridWorld.cc:507-672) run on one
// lane against an LDS copy of the env; everything order-free (starve, reward rules,
// set_action classification, clear_dead compaction, observation extraction) is spread
// over the workgroup.  Semantics follow the reference single-thread engine exactly;
// see DESIGN.md for the per-kernel roofline.
//
// Compiled with -ffp-contract=off: every float op is the reference's own single
// IEEE operation (no FMA contraction, correctly-rounded division).
#include <hip/hip_runtime.h>

#include "battle_layout.h"
#include "battle_kernels.h"

namespace mfx {

// Diagnostic build only (-DMFX_STAMPS, build/libmagent_stamps.so): per-phase s_memtime deltas of
// k_rollout go to a stamp buffer nobody else reads.  The real build compiles these to nothing.  The buffer pointer
// sits in constant memory: a scalar load, so a stamp does not wait (vmcnt) for the stores the phase before it left in
// flight, as a vector load of a __device__ pointer did (which read those stores' latency into the phase).
#ifdef MFX_STAMPS
__constant__ unsigned long long* g_stamps;
constexpr int kStampW = 32;                  // stamps per env row
#define MFX_STAMP(i)                                                                        \
    do {                                                                                    \
        __syncthreads();                                                                    \
        if (TID == 0 && g_stamps) {                                                         \
            g_stamps[stamp_row * kStampW + (i)] = __builtin_amdgcn_s_memtime();                  \
            /* wall clock (100 MHz) at stamps 0 / 10 and the workgroup: scripts/timeline_rollout.py */ \
            if ((i) == 0) g_stamps[stamp_row * kStampW + 11] = __builtin_amdgcn_s_memrealtime();  \
            if ((i) == 0) g_stamps[stamp_row * kStampW + 27] = blockIdx.x;                        \
            if ((i) == 10) g_stamps[stamp_row * kStampW + 12] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                   \
    } while (0)
#define MFX_TSTAMP(kW, i)                                                                   \
    do {                                                                                    \
        psync<kW>();                                                                        \
        if (TID == 0 && g_stamps) g_stamps[stamp_row * kStampW + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define MFX_RSTAMP(kW, row, i)                                                              \
    do {                                                                                    \
        psync<kW>();                                                                        \
        if (TID == 0 && g_stamps && (row) >= 0) g_stamps[(row) * kStampW + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define MFX_BSTAMP(row, i)                                                                  \
    do {                                                                                    \
        __syncthreads();                                                                    \
        if (TID == 0 && g_stamps && (row) >= 0) g_stamps[(row) * kStampW + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// drop-in server: lane 0's clock at the phase boundaries of request `seq` (no extra barrier)
#define MFX_DSTAMP(seq, i)                                                                  \
    do {                                                                                    \
        if (TID == 0 && g_stamps) {                                                         \
            g_stamps[((seq) & 1023u) * kStampW + (i)] = __builtin_amdgcn_s_memtime();       \
            g_stamps[((seq) & 1023u) * kStampW + 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                   \
    } while (0)
#else
#define MFX_DSTAMP(seq, i) do {} while (0)
#define MFX_STAMP(i) do {} while (0)
#define MFX_TSTAMP(kW, i) do {} while (0)
#define MFX_BSTAMP(row, i) do {} while (0)
#define MFX_RSTAMP(kW, row, i) do {} while (0)
#endif

// --------------------------------------------------------------------------- utils
// Lane id in the workgroup, opaque to loop-invariant code motion: k_rollout is one long loop over
// envs, and every address derived from the lane id would otherwise be hoisted out of it and kept
// live (in VGPRs) for the whole launch.
__device__ __forceinline__ int mfx_tid() {
    int t = (int)__builtin_amdgcn_workitem_id_x();
    asm volatile("" : "+v"(t));
    return t;
}
#define TID mfx_tid()

// Read-only HBM struct seen through the constant address space with an opaque pointer: field reads
// become scalar loads at their use instead of values hoisted out of a loop and pinned in SGPRs.
template <class T>
__device__ __forceinline__ const T& kconst(const T* p) {
    auto q = (const __attribute__((address_space(4))) T*)p;
    asm volatile("" : "+s"(q));
    return *(const T*)q;
}

__device__ __forceinline__ uint32_t minstd_next(uint32_t x) {   // minstd_rand0, GridWorld.h:106
    uint64_t p = (uint64_t)x * 16807u;
    p = (p & 0x7FFFFFFFull) + (p >> 31);
    if (p >= 0x7FFFFFFFull) p -= 0x7FFFFFFFull;
    return (uint32_t)p;
}

__device__ __forceinline__ void set_err(const State& s, int code) { atomicCAS(s.err, 0, code); }

// Exclusive scan of a 0/1 flag over the workgroup (blockDim multiple of 64, <= 1024).
__device__ __forceinline__ int block_scan_flag(int flag, int* wave_tot, int& total) {
    const int lane = TID & 63, wid = TID >> 6, nw = blockDim.x >> 6;
    const unsigned long long m = __ballot(flag);
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wid] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < nw; ++w) { const int c = wave_tot[w]; off += (w < wid) ? c : 0; tot += c; }
    __syncthreads();
    total = tot;
    return off + pre;
}

__device__ __forceinline__ int cell_group_ch(int og, int g, int G, int per) {   // make_channel_trans
    return 1 + per * ((og - g + G) % G);
}

// ------------------------------------------------------------------------- env view
// Pointers to ONE env's state, either into LDS copies or straight into HBM slabs.
struct EnvView {
    uint16_t* cells;
    uint32_t* xy;
    float* hp;
    float* next_r;
    float* last_r;
    uint8_t* last_act;
    int32_t* op_obj;
    uint8_t* meta;
    uint16_t* grp_ids;     // [G][cap]
    float* food;           // [H*W] food amounts (food_mode) or null; always in HBM
    int32_t* grp_n;        // [G]
    int32_t* grp_dead;     // [G]
    float* grp_reward;     // [G]
    uint16_t* rid;         // [cap] reference id of each slot (HBM); null in LDS images (slot == id there)
    int cap;
};

// The reference's id of slot `id` (features, get_agent_id, policy keys)
__device__ __forceinline__ int ref_id(const EnvView& v, int id) { return v.rid ? (int)v.rid[id] : id; }

__device__ __forceinline__ EnvView global_view(const State& s, int e, int G) {
    EnvView v;
    const size_t a = (size_t)e * s.cap;
    v.cells = s.cells + (size_t)e * s.cells_n;
    v.xy = s.xy + a; v.hp = s.hp + a; v.next_r = s.next_r + a; v.last_r = s.last_r + a;
    v.last_act = s.last_act + a; v.op_obj = s.op_obj + a; v.meta = s.meta + a;
    v.grp_ids = s.grp_ids + (size_t)e * G * s.cap;
    v.food = s.food ? s.food + (size_t)e * s.cells_n : nullptr;
    v.grp_n = s.grp_n + e * G; v.grp_dead = s.grp_dead + e * G; v.grp_reward = s.grp_reward + e * G;
    v.rid = s.rid + a;
    v.cap = s.cap;
    return v;
}

#include "battle/reset.inc"
#include "battle/observe.inc"
#include "battle/step_serial.inc"
#include "battle/step_parallel.inc"
#include "battle/step_big.inc"
#include "battle/step_core.inc"
#include "battle/getters.inc"
#include "battle/rollout.inc"
#include "battle/dropin.inc"
// ==================================================================================
//  host-side launchers
// ==================================================================================
size_t observe_smem_bytes(const GameParams& gp, int g, int cells_in_lds, int cells_n, int cap) {
    const bool kB = is_battle_shape(gp);
    size_t b = obs_smem_core(gp, g, cap, 64, obs_stage_floats(gp, g, kB, 256), kB);
    if (cells_in_lds) b += (size_t)cells_n * 2;
    return b;
}

size_t step_smem_bytes(const GameParams& gp, int cells_n, int n_ids, int acap, int cap) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return r16((size_t)cells_n * 2) + 4 * r16((size_t)n_ids * 4) + r16(n_ids) + 2 * r16((size_t)acap * 4) +
           (gp.large_map ? r16((size_t)acap * 4) : 0) + (gp.par_step ? r16(step_par_bytes(acap, cap)) : 0);
}

hipError_t launch_reset(const GameParams* d_gp, const State& s, hipStream_t st) {
    k_reset<<<s.E, 256, 0, st>>>(d_gp, s);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_rid_fill(State s, int from) {
    uint16_t* r = s.rid + (size_t)blockIdx.x * s.cap;
    for (int i = from + TID; i < s.cap; i += blockDim.x) r[i] = (uint16_t)i;
}

hipError_t launch_rid_fill(const State& s, int from, hipStream_t st) {
    if (from >= s.cap) return hipSuccess;
    k_rid_fill<<<s.E, 256, 0, st>>>(s, from);
    return hipGetLastError();
}

hipError_t launch_add_agents(const GameParams* d_gp, const State& s, int group, int n, int method,
                             const int* d_xs, const int* d_ys, const int* d_dirs, int per_env_stride, hipStream_t st) {
    k_add_agents<<<(s.E + 63) / 64, 64, 0, st>>>(d_gp, s, group, n, method, d_xs, d_ys, d_dirs, per_env_stride);
    return hipGetLastError();
}

#include "battle/rollout_big.inc"
// State::cells after fused rollout steps: the walls-only image plus every live listed agent.
__global__ void __launch_bounds__(256) k_rebuild_cells(const GameParams* __restrict__ gp, State s,
                                                       const uint16_t* __restrict__ walls) {
    const int e = blockIdx.x, G = gp->n_groups, W = gp->W;
    EnvView v = global_view(s, e, G);
    for (int i = TID; i < s.cells_n; i += blockDim.x) v.cells[i] = walls[i];
    __syncthreads();
    for (int g = 0; g < G; ++g)
        for (int i = TID; i < v.grp_n[g]; i += blockDim.x) {
            const int id = v.grp_ids[g * s.cap + i];
            const uint32_t p = v.xy[id];
            if (!meta_dead(v.meta[id])) v.cells[(p >> 16) * W + (p & 0xFFFF)] = (uint16_t)id;
        }
}

hipError_t launch_rebuild_cells(const GameParams* d_gp, const State& s, const void* walls, hipStream_t st) {
    k_rebuild_cells<<<s.E, 256, 0, st>>>(d_gp, s, reinterpret_cast<const uint16_t*>(walls));
    return hipGetLastError();
}

// GridWorld::set_goal "random" (GridWorld.cc:729-740, deprecated): the goals are never read again, but
// the two LCG draws per agent move the engine's random stream.
__global__ void k_set_goal_random(const GameParams* __restrict__ gp, State s, int g) {
    const int e = blockIdx.x * blockDim.x + TID;
    if (e >= s.E) return;
    const int n = s.grp_n[e * gp->n_groups + g];
    uint32_t rng = s.rng[e];
    for (int i = 0; i < 2 * n; ++i) rng = minstd_next(rng);
    s.rng[e] = rng;
}

hipError_t launch_set_goal_random(const GameParams* d_gp, const State& s, int g, hipStream_t st) {
    k_set_goal_random<<<(s.E + 63) / 64, 64, 0, st>>>(d_gp, s, g);
    return hipGetLastError();
}

bool battle_shape(const GameParams& gp) { return is_battle_shape(gp); }

hipError_t launch_obs_prep(const GameParams* d_gp, const State& s, const RolloutArgs& ra, int par, hipStream_t st) {
    k_obs_prep<<<s.E, 256, 0, st>>>(d_gp, s, ra, par);
    return hipGetLastError();
}

hipError_t launch_observe_items(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutArgs& ra,
                                int par, int grid, hipStream_t st) {
    const size_t smem = obs_smem_core(gp, 0, 0, ra.obs_item_rows, obs_stage_floats(gp, 0, true, 256), true);
    k_observe_items<<<grid, 256, smem, st>>>(d_gp, s, ra, par);
    return hipGetLastError();
}

hipError_t observe_items_grid(const GameParams& gp, int rows, int* grid) {
    const size_t smem = obs_smem_core(gp, 0, 0, rows, obs_stage_floats(gp, 0, true, 256), true);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err == hipSuccess) err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (err == hipSuccess) err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_observe_items, 256, smem);
    if (err != hipSuccess) return err;
    *grid = cus * (per_cu > 0 ? per_cu : 1);
    return hipSuccess;
}

hipError_t launch_observe(const GameParams& gp, const GameParams* d_gp, const State& s, int g, int max_n,
                          float* d_view, float* d_feat, int rowcap, hipStream_t st) {
    // few envs (the drop-in's one env): 16-agent chunks, so one group's rows spread over more CUs
    const int chunk = (long long)s.E * ((max_n + 63) / 64) < 256 ? 16 : 64;
    const int chunks = max(1, (max_n + chunk - 1) / chunk);
    const int cells_in_lds = (size_t)s.cells_n * 2 <= 32768;
    const size_t smem = observe_smem_bytes(gp, g, cells_in_lds, s.cells_n, s.cap);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid(chunks, s.E);
    if (is_battle_shape(gp))
        k_observe<true><<<grid, 256, smem, st>>>(d_gp, s, g, chunk, d_view, d_feat, rowcap, cells_in_lds);
    else
        k_observe<false><<<grid, 256, smem, st>>>(d_gp, s, g, chunk, d_view, d_feat, rowcap, cells_in_lds);
    return hipGetLastError();
}

hipError_t launch_set_action(const GameParams* d_gp, const State& s, int g, const int* d_actions, int rowcap,
                             hipStream_t st) {
    k_set_action<<<s.E, 256, 0, st>>>(d_gp, s, g, d_actions, rowcap);
    return hipGetLastError();
}

hipError_t launch_step(const GameParams& gp, const GameParams* d_gp, const State& s, int max_ids,
                       uint32_t* d_sort_scratch, hipStream_t st) {
    const size_t smem = step_smem_bytes(gp, s.cells_n, max_ids, s.acap, s.cap) + step_sm_bytes(gp.n_groups);
    const int lds = smem <= 96 * 1024;
    const size_t big = big_step_smem_bytes(gp, s.cap, s.acap, false);
    if (!lds && !gp.dsl && gp.par_step && !gp.record_events && big <= 160 * 1024) {
        k_step_big<<<s.E, kBigThreads, big, st>>>(d_gp, s);      // HBM-resident env, parallel exact step
        return hipGetLastError();
    }
    const size_t dyn = lds ? smem : step_sm_bytes(gp.n_groups);
    bool body = gp.turn_mode != 0 || gp.food_mode != 0;   // bodies > 1x1, turn / food mode: the kernel with those forms
    for (int g = 0; g < gp.n_groups; ++g) body = body || gp.type[g].body_w != 1 || gp.type[g].body_h != 1;
    if (gp.dsl) {
        if (body) k_step<true, true><<<s.E, 256, dyn, st>>>(d_gp, s, lds, d_sort_scratch);
        else k_step<true, false><<<s.E, 256, dyn, st>>>(d_gp, s, lds, d_sort_scratch);
    } else {
        if (body) k_step<false, true><<<s.E, 256, dyn, st>>>(d_gp, s, lds, d_sort_scratch);
        else k_step<false, false><<<s.E, 256, dyn, st>>>(d_gp, s, lds, d_sort_scratch);
    }
    return hipGetLastError();
}

hipError_t launch_rollout_big(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                              uint32_t step_index, bool lds_env, hipStream_t st) {
    const size_t smem = big_step_smem_bytes(gp, s.cap, s.acap, true, lds_env);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    k_rollout_big<<<s.E, kBigRolloutThreads, smem, st>>>(d_gp, d_ctx, step_index);
    return hipGetLastError();
}

// The step's layout and an item's observation scratch share the LDS (a workgroup does one or the other), except in
// the pipelined form, where a stepper observes the items it took back (few_stolen) with its env still in LDS: the
// scratch then follows the step's layout.
size_t bigq_smem_bytes(const GameParams& gp, int cap, int acap, int rows, bool lds_env, bool pipe) {
    const size_t a = big_step_smem_bytes(gp, cap, acap, true, lds_env);
    const size_t b = obs_smem_core(gp, 0, 0, rows, obs_stage_floats(gp, 0, true, kBigRolloutThreads), true);
    return pipe ? a + b : a > b ? a : b;
}

hipError_t bigq_grid(const GameParams& gp, int cap, int acap, int rows, bool lds_env, int* grid, bool pipe) {
    const size_t smem = bigq_smem_bytes(gp, cap, acap, rows, lds_env, pipe);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err == hipSuccess) err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (err == hipSuccess)
        err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pipe ? k_rollout_bigq<true> : k_rollout_bigq<false>,
                                                           kBigRolloutThreads, smem);
    if (err != hipSuccess) return err;
    // one device of all 8 XCDs (SPX, 32 CUs each): every XCD gets workgroups of the full-occupancy grid,
    // and the XCC ids are 0-7 (k_rollout_bigq keeps each env on XCD e % 8)
    *grid = (cus % kXcds == 0 && cus >= 32 * kXcds) ? cus * (per_cu > 0 ? per_cu : 1) : 0;
    return hipSuccess;
}

hipError_t launch_bigq_seed(const GameParams* d_gp, const State& s, const RolloutArgs& ra, int par, uint32_t tag,
                            uint32_t step_index, hipStream_t st) {
    k_bigq_seed<<<s.E, 256, 0, st>>>(d_gp, s, ra, par, tag, step_index);
    return hipGetLastError();
}

hipError_t launch_rollout_bigq(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                               int rows, uint32_t si0, int n_sub, int par, uint32_t tag_cur, uint32_t tag_next,
                               int grid, bool lds_env, hipStream_t st, bool pipe) {
    const size_t smem = bigq_smem_bytes(gp, s.cap, s.acap, rows, lds_env, pipe);
    if (smem > 160 * 1024 || grid < 1 || n_sub < 1 || (pipe && !lds_env)) return hipErrorInvalidValue;
    if (pipe)
        k_rollout_bigq<true><<<grid, kBigRolloutThreads, smem, st>>>(d_gp, d_ctx, si0, n_sub, par, tag_cur, tag_next);
    else
        k_rollout_bigq<false><<<grid, kBigRolloutThreads, smem, st>>>(d_gp, d_ctx, si0, n_sub, par, tag_cur, tag_next);
    return hipGetLastError();
}

size_t few_snap_bytes(int cells_n, int cap, int G) { return snap_layout(cells_n, cap, G).total; }

hipError_t launch_clear_dead(const GameParams* d_gp, const State& s, hipStream_t st) {
    k_clear_dead<<<s.E, 256, 0, st>>>(d_gp, s);
    return hipGetLastError();
}

hipError_t set_stamp_buffer(unsigned long long* d_buf) {
#ifdef MFX_STAMPS
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_buf, sizeof(d_buf));
#else
    (void)d_buf;
    return hipErrorNotSupported;
#endif
}

// The register-prefetch instance needs the env image to fit the prefetch lanes (see EnvPrefetch).
static bool rollout_prefetch_ok(const GameParams& gp, const State& s) {
#ifdef MFX_NO_PF
    return false;                                     // experiments: the synchronous install
#endif
    const int c4 = s.cap >> 2, nc16 = s.cells_n >> 3;
    return (s.cells_n & 7) == 0 && nc16 + image_small_rows(c4, gp.n_groups) <= kPfRows;
}

template <class F>
static hipError_t with_rollout_kernel(const GameParams& gp, const State& s, bool split, F&& f) {
    if (is_battle_shape(gp)) {
        if (rollout_prefetch_ok(gp, s)) return split ? f(k_rollout<true, true, true>) : f(k_rollout<true, true, false>);
        return split ? f(k_rollout<true, false, true>) : f(k_rollout<true, false, false>);
    }
    return split ? f(k_rollout<false, false, true>) : f(k_rollout<false, false, false>);
}

template <class F>
static hipError_t with_rollout_obs_kernel(const GameParams& gp, const State& s, F&& f) {
    if (is_battle_shape(gp)) {
        if (rollout_prefetch_ok(gp, s)) return f(k_rollout_obs<true, true>);
        return f(k_rollout_obs<true, false>);
    }
    return f(k_rollout_obs<false, false>);
}

hipError_t launch_rollout(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                          int rows, uint32_t step_index, int work_sel, int qphase, int grid, int split,
                          int n_sub, hipStream_t st) {
    const size_t smem = rollout_smem_bytes(gp, s.cells_n, s.cap, s.acap, rows);
    if (smem > 160 * 1024 || n_sub < 1 || (split && n_sub != 1)) return hipErrorInvalidValue;
    return with_rollout_kernel(gp, s, split != 0, [&](auto kern) {
        kern<<<grid, MFX_ROLLOUT_THREADS, smem, st>>>(d_gp, d_ctx, step_index, work_sel, qphase, n_sub);
        return hipGetLastError();
    });
}

// A learned policy's launches (k_rollout kMode 1: act with ra.actions, step, observe; 2: observe only),
// one step each; the fused path only (LDS-sized envs, no pipeline).
hipError_t launch_rollout_mode(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                               int rows, uint32_t step_index, int work_sel, int qphase, int grid, int mode,
                               hipStream_t st) {
    const size_t smem = rollout_smem_bytes(gp, s.cells_n, s.cap, s.acap, rows);
    if (smem > 160 * 1024 || (mode != 1 && mode != 2)) return hipErrorInvalidValue;
    auto go = [&](auto kern) {
        kern<<<grid, MFX_ROLLOUT_THREADS, smem, st>>>(d_gp, d_ctx, step_index, work_sel, qphase, 1);
        return hipGetLastError();
    };
    if (is_battle_shape(gp)) {
        if (rollout_prefetch_ok(gp, s))
            return mode == 1 ? go(k_rollout<true, true, false, 1>) : go(k_rollout<true, true, false, 2>);
        return mode == 1 ? go(k_rollout<true, false, false, 1>) : go(k_rollout<true, false, false, 2>);
    }
    return mode == 1 ? go(k_rollout<false, false, false, 1>) : go(k_rollout<false, false, false, 2>);
}

// k_rollout_obs: the env image and the observation scratch
size_t rollout_obs_smem_bytes(const GameParams& gp, int cells_n, int cap, int rows) {
    const bool kB = is_battle_shape(gp);
    return env_image_bytes(cells_n, cap, gp.n_groups) +
           obs_smem_core(gp, 0, cap, rows * (kB ? gp.n_groups : 1), obs_stage_floats(gp, 0, kB, MFX_ROLLOUT_THREADS), kB);
}

hipError_t launch_rollout_obs(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                              int rows, int work_sel, int qphase, int grid, hipStream_t st) {
    const size_t smem = rollout_obs_smem_bytes(gp, s.cells_n, s.cap, rows);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    return with_rollout_obs_kernel(gp, s, [&](auto kern) {
        kern<<<grid, MFX_ROLLOUT_THREADS, smem, st>>>(d_gp, d_ctx, work_sel, qphase);
        return hipGetLastError();
    });
}

// Persistent grid of k_rollout: every workgroup that can be resident at once (more is harmless --
// the extra ones find the queue empty -- fewer would idle CUs).  per_cu > 0: that many per CU
// instead (the pipeline shares the CUs between k_rollout and k_rollout_obs).
hipError_t rollout_grid(const GameParams& gp, const State& s, int rows, int split, int per_cu_want, int* grid) {
    const size_t smem = rollout_smem_bytes(gp, s.cells_n, s.cap, s.acap, rows);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err == hipSuccess) err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (err != hipSuccess) return err;
    err = with_rollout_kernel(gp, s, split != 0, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, MFX_ROLLOUT_THREADS, smem);
    });
    if (err != hipSuccess) return err;
    if (per_cu_want > 0 && per_cu_want < per_cu) per_cu = per_cu_want;
    const long long want = (long long)cus * (per_cu > 0 ? per_cu : 1);
    *grid = (int)(want < s.E ? want : s.E);
    return hipSuccess;
}

hipError_t rollout_obs_grid(const GameParams& gp, const State& s, int rows, int per_cu_want, int* grid) {
    const size_t smem = rollout_obs_smem_bytes(gp, s.cells_n, s.cap, rows);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err == hipSuccess) err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (err != hipSuccess) return err;
    err = with_rollout_obs_kernel(gp, s, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, MFX_ROLLOUT_THREADS, smem);
    });
    if (err != hipSuccess) return err;
    if (per_cu_want > 0 && per_cu_want < per_cu) per_cu = per_cu_want;
    const long long want = (long long)cus * (per_cu > 0 ? per_cu : 1);
    *grid = (int)(want < s.E ? want : s.E);
    return hipSuccess;
}

hipError_t launch_reset_image(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutArgs& ra,
                              uint4* d_image, hipStream_t st) {
    const size_t smem = env_image_bytes(s.cells_n, s.cap, gp.n_groups);
    const int in_lds = smem <= 64 * 1024;
    k_reset_image<<<1, 256, in_lds ? smem : 0, st>>>(d_gp, s.cells_n, s.cap, ra, d_image, in_lds);
    return hipGetLastError();
}

hipError_t launch_get(const GameParams* d_gp, const State& s, int g, int what, void* d_out, int rowcap,
                      hipStream_t st) {
    k_get<<<s.E, 256, 0, st>>>(d_gp, s, g, what, d_out, rowcap);
    return hipGetLastError();
}

}  // namespace mfx
