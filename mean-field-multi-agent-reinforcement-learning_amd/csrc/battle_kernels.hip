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
// k_rollout go to a stamp buffer nobody else reads.  The real build compiles these to nothing.
#ifdef MFX_STAMPS
__device__ unsigned long long* g_stamps;
constexpr int kStampW = 32;                  // stamps per env row
#define MFX_STAMP(i)                                                                        \
    do {                                                                                    \
        __syncthreads();                                                                    \
        if (TID == 0 && g_stamps) {                                                         \
            g_stamps[stamp_row * kStampW + (i)] = __builtin_amdgcn_s_memtime();                  \
            if ((i) == 0) g_stamps[stamp_row * kStampW + 11] = __builtin_amdgcn_s_memrealtime();  \
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
#else
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
    int cap;
};

__device__ __forceinline__ EnvView global_view(const State& s, int e, int G) {
    EnvView v;
    const size_t a = (size_t)e * s.cap;
    v.cells = s.cells + (size_t)e * s.cells_n;
    v.xy = s.xy + a; v.hp = s.hp + a; v.next_r = s.next_r + a; v.last_r = s.last_r + a;
    v.last_act = s.last_act + a; v.op_obj = s.op_obj + a; v.meta = s.meta + a;
    v.grp_ids = s.grp_ids + (size_t)e * G * s.cap;
    v.food = s.food ? s.food + (size_t)e * s.cells_n : nullptr;
    v.grp_n = s.grp_n + e * G; v.grp_dead = s.grp_dead + e * G; v.grp_reward = s.grp_reward + e * G;
    v.cap = s.cap;
    return v;
}

// ==================================================================================
//  reset / add_agents
// ==================================================================================
// GridWorld::reset (GridWorld.cc:76-124) + Map::reset (Map.cc:23-47): border walls, no agents.
__global__ void __launch_bounds__(256) k_reset(const GameParams* __restrict__ gp, State s) {
    const int e = blockIdx.x, W = gp->W, H = gp->H, G = gp->n_groups;
    uint16_t* cells = s.cells + (size_t)e * s.cells_n;
    for (int c = TID; c < W * H; c += blockDim.x) {
        const int x = c % W, y = c / W;
        cells[c] = (x == 0 || y == 0 || x == W - 1 || y == H - 1) ? kCellWall : kCellEmpty;
    }
    if (TID < G) {                 // Group::clear (GridWorld.h:281-284): the group reward survives
        s.grp_n[e * G + TID] = 0;
        s.grp_dead[e * G + TID] = 0;
    }
    if (TID == 0) { s.id_counter[e] = 0; s.n_atk[e] = 0; s.n_mov[e] = 0; s.done[e] = 0; s.idx_mark[e] = 0; }
}

__device__ __forceinline__ bool is_blank(const uint16_t* cells, int W, int H, int x, int y, int self) {
    // Map::is_blank_area for a 1x1 body (Map.cc:466-482)
    if (x < 0 || y < 0 || x + 1 >= W || y + 1 >= H) return false;
    const uint32_t c = cells[y * W + x];
    return c == kCellEmpty || (int)c == self;
}

// Bodies of bw x bh cells (width x length; every agent faces NORTH without turn_mode).
__device__ __forceinline__ bool is_blank_area(const uint16_t* cells, int W, int H, int x, int y, int bw, int bh,
                                              int self) {
    if (x < 0 || y < 0 || x + bw >= W || y + bh >= H) return false;
    for (int i = 0; i < bw; ++i)
        for (int j = 0; j < bh; ++j) {
            const uint32_t c = cells[(y + j) * W + x + i];
            if (!(c == kCellEmpty || (int)c == self)) return false;
        }
    return true;
}

__device__ __forceinline__ void fill_area(uint16_t* cells, int W, int x, int y, int bw, int bh, uint16_t val) {
    for (int i = 0; i < bw; ++i)
        for (int j = 0; j < bh; ++j) cells[(y + j) * W + x + i] = val;
}

// Map::get_collide (Map.cc:498-513): the first other agent of the rectangle, column by column.
__device__ __forceinline__ int get_collide(const uint16_t* cells, int W, int H, int x, int y, int bw, int bh,
                                           int self) {
    if (x < 0 || y < 0 || x + bw >= W || y + bh >= H) return -1;
    for (int i = 0; i < bw; ++i)
        for (int j = 0; j < bh; ++j) {
            const uint32_t c = cells[(y + j) * W + x + i];
            if (c < kCellFood && (int)c != self) return (int)c;
        }
    return -1;
}

// Direction geometry (Map.cc:530-612): rela_to_abs, save_to_real, real_to_save, get_size_for_dir.
__device__ __forceinline__ void rela_to_abs(int cx, int cy, int dir, int rx, int ry, int& ax, int& ay) {
    if (dir == kDirNorth) { ax = cx + rx; ay = cy + ry; }
    else if (dir == kDirSouth) { ax = cx - rx; ay = cy - ry; }
    else if (dir == kDirWest) { ax = cx + ry; ay = cy - rx; }
    else { ax = cx - ry; ay = cy + rx; }
}

__device__ __forceinline__ void save_to_real(int px, int py, int dir, int w, int l, int& rx, int& ry) {
    if (dir == kDirNorth) { rx = px; ry = py; }
    else if (dir == kDirSouth) { rx = px + w - 1; ry = py + l - 1; }
    else if (dir == kDirWest) { rx = px; ry = py + w - 1; }
    else { rx = px + l - 1; ry = py; }
}

__device__ __forceinline__ void real_to_save(int rx, int ry, int dir, int w, int l, int& px, int& py) {
    if (dir == kDirNorth) { px = rx; py = ry; }
    else if (dir == kDirSouth) { px = rx - w + 1; py = ry - l + 1; }
    else if (dir == kDirWest) { px = rx; py = ry - w + 1; }
    else { px = rx - l + 1; py = ry; }
}

__device__ __forceinline__ void size_for_dir(int dir, int w, int l, int& bw, int& bh) {
    const bool ns = dir == kDirNorth || dir == kDirSouth;
    bw = ns ? w : l; bh = ns ? l : w;
}

// One lane per env: placements are order-dependent (an occupied cell is skipped and the
// id is not consumed -- GridWorld.cc:180-187).  method: 0 custom, 1 random, 2 fill.
__global__ void k_add_agents(const GameParams* __restrict__ gp, State s, int group, int n, int method,
                             const int* __restrict__ xs, const int* __restrict__ ys, const int* __restrict__ dirs,
                             int per_env_stride) {
    const int e = blockIdx.x * blockDim.x + TID;
    if (e >= s.E) return;
    const int W = gp->W, H = gp->H, G = gp->n_groups;
    EnvView v = global_view(s, e, G);
    const int* px = xs + (size_t)e * per_env_stride;
    const int* py = ys + (size_t)e * per_env_stride;
    uint32_t rng = s.rng[e];
    int idc = s.id_counter[e];
    auto place = [&](int x, int y, int dir) {
        if (group < 0) {                                         // Map::add_wall (Map.cc:108-115)
            if (x < 0 || y < 0 || x >= W || y >= H) return;
            uint16_t& c = v.cells[y * W + x];
            if (c == kCellEmpty || c == kCellWall) c = kCellWall;
            return;
        }
        const TypeParams& T = gp->type[group];
        int bw, bh;
        size_for_dir(dir, T.body_w, T.body_h, bw, bh);               // Map::add_agent (Map.cc:75-97)
        if (!is_blank_area(v.cells, W, H, x, y, bw, bh, -1)) return;
        if (idc >= s.cap || idc >= kCellFood) { set_err(s, 2); return; }
        const int id = idc++;
        fill_area(v.cells, W, x, y, bw, bh, (uint16_t)id);
        v.xy[id] = (uint32_t)x | ((uint32_t)y << 16);
        v.hp[id] = T.hp;
        v.last_r[id] = 0.0f;                                     // Agent ctor + init_reward()
        v.next_r[id] = T.step_reward;
        v.last_act[id] = T.n_action;
        v.op_obj[id] = -1;
        v.meta[id] = (uint8_t)meta_set_dir(meta_make(0, kOpNull, group), dir);
        int& n = v.grp_n[group];
        v.grp_ids[group * s.cap + n] = (uint16_t)id;
        ++n;
    };
    const bool turn = group >= 0 && gp->turn_mode;
    if (method == 0) {
        for (int i = 0; i < n; ++i) place(px[i], py[i], turn ? dirs[(size_t)e * per_env_stride + i] : kDirNorth);
    } else if (method == 1) {                                    // Map::get_random_blank (Map.cc:49-63)
        for (int i = 0; i < n; ++i) {
            int dir = kDirNorth;
            if (turn) { rng = minstd_next(rng); dir = (int)(rng % 4u); }   // GridWorld.cc:241
            int bw = 1, bh = 1;
            if (group >= 0) size_for_dir(dir, gp->type[group].body_w, gp->type[group].body_h, bw, bh);
            int x = 0, y = 0, tries = 0;
            for (;;) {
                rng = minstd_next(rng); x = (int)(rng % (uint32_t)(W - bw));
                rng = minstd_next(rng); y = (int)(rng % (uint32_t)(H - bh));
                if (is_blank_area(v.cells, W, H, x, y, bw, bh, -1)) break;
                if (tries++ > W * H) { set_err(s, 3); break; }
            }
            place(x, y, dir);
        }
    } else {                                                     // fill: xs = {x, y, w, h, dir}, body strides
        const int dir = turn ? px[4] : kDirNorth;
        int bw = 1, bh = 1;
        if (group >= 0) size_for_dir(dir, gp->type[group].body_w, gp->type[group].body_h, bw, bh);
        for (int x = px[0]; x < px[0] + px[2]; x += bw)
            for (int y = px[1]; y < px[1] + px[3]; y += bh) place(x, y, dir);
    }
    s.rng[e] = rng;
    s.id_counter[e] = idc;
}

// ==================================================================================
//  observation  (GridWorld::get_observation, GridWorld.cc:303-426; Map::extract_view,
//  Map.cc:130-218).  Output rows are staged in LDS K agents at a time and streamed out
//  as 16-byte coalesced stores.
// ==================================================================================
#ifndef MFX_OBS_K
#define MFX_OBS_K 4
#endif
constexpr int kObsK = MFX_OBS_K;  // agents per staging round (K*1183*4 B per round for Battle)
constexpr int kMaxCh = 1 + 3 * kMaxGroups;

struct ObsSmem {                  // LDS carve-up of the observation kernels
    float* stage;                 // [kObsK][VH*VW*n_ch]
    float* mm;                    // [G][VH*VW] minimap density
    int* hist;                    // [G][VH*VW]
    uint16_t* bin;                // [cap] minimap cell of every agent id (generic path only)
    uint32_t* mask;               // [ceil(VH*VW/32)] view mask bits (Range::is_in)
    float* type_hp;               // [G]
    uint32_t* info;               // [cap] wave-streamed path: hp / max hp bits | group << 31, or null
    uint32_t* aq;                 // [rows] wave-streamed path: per agent of the group being observed,
                                  //       view origin + 8 (12 bits x, 12 bits y) | minimap bin << 24
};

// Battle fast path (builtin/config/battle.py): 13x13 view, 7 channels, 2 groups, minimap, 34
// features.  kB = true folds every view/channel/feature dimension into a constant (no runtime
// integer division in the inner loops); kB = false is the generic path for any other config.
struct BattleShape { static constexpr int VW = 13, VH = 13, NC = 7, G = 2, F = 34; };

// Minimap of the observing group g: its own view size sets the scale (GridWorld.cc:338-340).
template <bool kB>
__device__ __forceinline__ void obs_minimap(const GameParams& gp, const EnvView& v, const ObsSmem& sm, int g) {
    const TypeParams& T0 = gp.type[g];
    const int VW = kB ? BattleShape::VW : T0.view_w, VH = kB ? BattleShape::VH : T0.view_h;
    const int G = kB ? BattleShape::G : gp.n_groups, NV = VW * VH;
    const int sw = (gp.W + VW - 1) / VW, sh = (gp.H + VH - 1) / VH;
    for (int i = TID; i < G * NV; i += blockDim.x) sm.hist[i] = 0;
    __syncthreads();
    for (int j = 0; j < G; ++j) {
        const int n = v.grp_n[j];
        for (int i = TID; i < n; i += blockDim.x) {
            const int id = v.grp_ids[j * v.cap + i];
            const uint32_t p = v.xy[id];
            const int b = ((int)(p >> 16) / sh) * VW + (int)(p & 0xFFFF) / sw;
            if (!kB) sm.bin[id] = (uint16_t)b;
            atomicAdd(&sm.hist[j * NV + b], 1);
            // hp / max hp (Map.cc:208), once per agent instead of once per viewer; the group rides
            // in the sign bit (a visible agent's hp is >= +0)
            if (sm.info) sm.info[id] = __float_as_uint(v.hp[id] / gp.type[j].hp) | ((uint32_t)j << 31);
        }
    }
    __syncthreads();
    for (int i = TID; i < G * NV; i += blockDim.x) {   // in place: mm aliases hist
        const int j = i / NV;
        const int n = v.grp_n[j];
        // 0/0 gives the x86 default NaN (0xFFC00000) in the reference; reproduce its bits.
        sm.mm[i] = n ? (float)sm.hist[i] / (float)n : __uint_as_float(0xFFC00000u);
    }
    __syncthreads();
}

// obs_minimap split for k_rollout, whose install already walks every listed agent: the histogram
// and info words of agent id of group j (Battle shape) ...
#ifndef MFX_MM_IN_INSTALL
#define MFX_MM_IN_INSTALL 1
#endif
// (and its agent record, obs_agent_records, when i < rows: list position i of group j)
__device__ __forceinline__ void obs_minimap_add(const GameParams& gp, const EnvView& v, const ObsSmem& sm, int j,
                                                int id, uint32_t p, int i, int rows) {
    constexpr int VW = BattleShape::VW, VH = BattleShape::VH, NV = VW * VH;
    const int sw = (gp.W + VW - 1) / VW, sh = (gp.H + VH - 1) / VH;
    const int x = (int)(p & 0xFFFF), y = (int)(p >> 16);
    const int b = (y / sh) * VW + x / sw;
    atomicAdd(&sm.hist[j * NV + b], 1);
    sm.info[id] = __float_as_uint(v.hp[id] / gp.type[j].hp) | ((uint32_t)j << 31);
    if (i < rows) {
        const TypeParams& T = gp.type[j];
        sm.aq[j * rows + i] = (uint32_t)(x + T.view_x1 + 8) | ((uint32_t)(y + T.view_y1 + 8) << 12) | ((uint32_t)b << 24);
    }
}
// ... and the conversion to densities once the histogram is complete (after a barrier)
template <bool kB>
__device__ __forceinline__ void obs_minimap_finish(const GameParams& gp, const EnvView& v, const ObsSmem& sm) {
    constexpr int NV = BattleShape::VW * BattleShape::VH;
    for (int i = TID; i < BattleShape::G * NV; i += blockDim.x) {   // in place: mm aliases hist
        const int n = v.grp_n[i / NV];
        sm.mm[i] = n ? (float)sm.hist[i] / (float)n : __uint_as_float(0xFFC00000u);
    }
    __syncthreads();
}

typedef float f32x4 __attribute__((ext_vector_type(4)));   // nontemporal-storable float4

// Fill the staging rows of agents [a0, a0+k) of group g, then stream them to out_view.
template <bool kB>
__device__ __forceinline__ void obs_rows(const GameParams& gp, const EnvView& v, const ObsSmem& sm,
                                         int g, int a0, int k, float* __restrict__ out_view,
                                         float* __restrict__ out_feat) {
    const TypeParams& T = gp.type[g];
    const int W = gp.W, H = gp.H;
    const int G = kB ? BattleShape::G : gp.n_groups, NC = kB ? BattleShape::NC : gp.n_ch;
    const int VW = kB ? BattleShape::VW : T.view_w, VH = kB ? BattleShape::VH : T.view_h;
    const int NV = VW * VH, VF = NV * NC;
    const bool MM = kB ? true : gp.minimap != 0;
    const int per = MM ? 3 : 2;
    const int cbase = (!kB && gp.food_mode) ? 2 : 1;     // group2channel(0) (GridWorld.cc:999-1008)
    const uint16_t* ids = v.grp_ids + g * v.cap;
    // ---- phase 1: one lane per (agent, view cell) computes that cell's NC channels
    for (int p = TID; p < k * NV; p += blockDim.x) {
        const int al = p / NV, c = p - al * NV;
        const int vy = c / VW, vx = c - vy * VW;
        const int id = ids[a0 + al];
        const uint32_t pos = v.xy[id];
        float o[kMaxCh];
#pragma unroll
        for (int q = 0; q < kMaxCh; ++q) o[q] = 0.0f;
        int mx = (int)(pos & 0xFFFF) + T.view_x1 + vx, my = (int)(pos >> 16) + T.view_y1 + vy;
        if (!kB && gp.turn_mode) {                      // Map::extract_view (Map.cc:130-218) as a gather
            const int dir = meta_dir(v.meta[id]);
            int rx, ry, ex, ey;
            save_to_real((int)(pos & 0xFFFF), (int)(pos >> 16), dir, T.body_w, T.body_h, rx, ry);
            rela_to_abs(rx, ry, dir, T.view_off_x, T.view_off_y, ex, ey);
            rela_to_abs(ex, ey, dir, T.view_lt_x + vx, T.view_lt_y + vy, mx, my);
        }
        if (((sm.mask[c >> 5] >> (c & 31)) & 1u) && mx >= 0 && my >= 0 && mx < W && my < H) {
            const uint32_t cv = v.cells[my * W + mx];
            if (cv == kCellWall) {
                o[0] = 1.0f;
            } else if (cv == kCellFood) {
                o[1] = 1.0f;                               // food_channel_id (Map.h:35), no hp
            } else if (cv != kCellEmpty) {
                const int og = meta_group(v.meta[cv]);
                const int ch = cbase + per * ((og - g + G) % G);
                const float hn = v.hp[cv] / sm.type_hp[og];
#pragma unroll
                for (int q = 0; q < kMaxCh; ++q) {
                    if (q == ch) o[q] = 1.0f;
                    if (q == ch + 1) o[q] = hn;
                }
            }
        }
        if (MM) {
            const bool self = c == (int)sm.bin[id];
            for (int j = 0; j < G; ++j) {
                const float m = sm.mm[j * NV + c];
                const int ch = cbase + 2 + per * ((j - g + G) % G);
#pragma unroll
                for (int q = 0; q < kMaxCh; ++q)
                    if (q == ch) o[q] = self ? m + 1.0f : m;
            }
        }
        float* dst = sm.stage + (size_t)al * VF + c * NC;
#pragma unroll
        for (int q = 0; q < kMaxCh; ++q)
            if (q < NC) dst[q] = o[q];
    }
    // ---- features (GridWorld.cc:411-421): written straight out, consecutive lanes = consecutive floats
    const int F = kB ? BattleShape::F : gp.feat_size[g];
    const int emb = gp.emb, na = T.n_action;
    for (int p = TID; p < k * F; p += blockDim.x) {
        const int al = p / F, f = p - al * F;
        const int id = ids[a0 + al];
        float val = 0.0f;
        if (f < emb) val = (float)((id >> f) & 1);
        if (f == emb + v.last_act[id]) val = 1.0f;
        if (f == emb + na) val = v.last_r[id];
        if (MM) {
            const uint32_t pos = v.xy[id];
            if (f == emb + na + 1) val = (float)(int)(pos & 0xFFFF) / (float)W;
            if (f == emb + na + 2) val = (float)(int)(pos >> 16) / (float)H;
        }
        out_feat[(size_t)(a0 + al) * F + f] = val;
    }
    __syncthreads();
    // ---- phase 2: stream k*VF floats; row a0 starts 16-B aligned when a0 % 4 == 0 (VF*4*4 % 16 == 0)
    float* dst = out_view + (size_t)a0 * VF;
    const int nf = k * VF;
    if ((((uintptr_t)dst) & 15) == 0) {
        const int n4 = nf >> 2;
        const f32x4* src4 = reinterpret_cast<const f32x4*>(sm.stage);
        f32x4* dst4 = reinterpret_cast<f32x4*>(dst);
        for (int i = TID; i < n4; i += blockDim.x) __builtin_nontemporal_store(src4[i], dst4 + i);
        for (int i = (n4 << 2) + TID; i < nf; i += blockDim.x) __builtin_nontemporal_store(sm.stage[i], dst + i);
    } else {
        for (int i = TID; i < nf; i += blockDim.x) __builtin_nontemporal_store(sm.stage[i], dst + i);
    }
    __syncthreads();
}

// ---- Battle fast path, wave-streamed: every wave takes 128 consecutive view cells of the group's
// output stream (row a, cell c -> stream cell a*169+c), two per lane, computes each cell's 7
// channels, transposes them through its own 1792-B LDS slice and stores them as float4s (1 KiB
// contiguous per store instruction).  No workgroup barrier inside the stream.  Needs the group's
// agent records (obs_agent_records) and sm.info (obs_minimap).
constexpr int kWaveCells = 64;
constexpr int kWaveStageFloats = kWaveCells * BattleShape::NC;   // 448 floats = 1792 B per wave

__device__ __forceinline__ void obs_agent_records(const GameParams& gp, const EnvView& v, const ObsSmem& sm, int g,
                                                  int n) {
    const TypeParams& T = gp.type[g];
    const uint16_t* ids = v.grp_ids + g * v.cap;
    constexpr int VW = BattleShape::VW, VH = BattleShape::VH;
    const int sw = (gp.W + VW - 1) / VW, sh = (gp.H + VH - 1) / VH;   // obs_minimap's scale
    for (int a = TID; a < n; a += blockDim.x) {
        const int id = ids[a];
        const uint32_t p = v.xy[id];
        const int x = (int)(p & 0xFFFF), y = (int)(p >> 16);
        const int ox = x + T.view_x1 + 8, oy = y + T.view_y1 + 8;        // >= 2, < 4096 (is_battle_shape)
        const int b = (y / sh) * VW + x / sw;
        sm.aq[a] = (uint32_t)ox | ((uint32_t)oy << 12) | ((uint32_t)b << 24);
    }
}

struct CellObs {              // one view cell: kind 0 nothing, 1 wall, 2 own agent, 3 enemy agent
    float hn, mo, me;
    int kind;
};

// Branch-free: every LDS read is issued from a safe index and the results are selected, so a wave
// never splits its exec mask (the branchy form spent ~40 % of its instructions on mask bookkeeping).
__device__ __forceinline__ CellObs obs_cell(const EnvView& v, const ObsSmem& sm, const float* mm_own,
                                            const float* mm_en, int W, int H, int g, int gc, int ncell) {
    constexpr int NV = BattleShape::VW * BattleShape::VH;
    const bool valid = gc < ncell;
    const int gs = valid ? gc : 0;
    const int a = gs / NV, c = gs - a * NV;
    const int vy = c / BattleShape::VW, vx = c - vy * BattleShape::VW;
    const uint32_t q = sm.aq[a];
    const uint32_t mk = (sm.mask[c >> 5] >> (c & 31)) & 1u;
    const float mo = mm_own[c], me = mm_en[c];
    const bool self = c == (int)(q >> 24);
    const int mx = (int)(q & 0xFFFu) - 8 + vx, my = (int)((q >> 12) & 0xFFFu) - 8 + vy;
    const bool ok = valid && mk != 0 && (unsigned)mx < (unsigned)W && (unsigned)my < (unsigned)H;
    const uint32_t cv = v.cells[ok ? my * W + mx : 0];
    const bool agent = ok && cv < kCellFood;
    const uint32_t inf = sm.info[agent ? cv : 0];
    CellObs o;
    o.mo = valid ? (self ? mo + 1.0f : mo) : 0.0f;
    o.me = valid ? (self ? me + 1.0f : me) : 0.0f;
    o.hn = agent ? __uint_as_float(inf & 0x7FFFFFFFu) : 0.0f;
    o.kind = (ok && cv == kCellWall) ? 1 : (agent ? ((int)(inf >> 31) == g ? 2 : 3) : 0);
    return o;
}

__device__ __forceinline__ void obs_stage_cell(float* st, int lane, const CellObs& o) {
    float* d = st + lane * BattleShape::NC;
    d[0] = o.kind == 1 ? 1.0f : 0.0f;
    d[1] = o.kind == 2 ? 1.0f : 0.0f;
    d[2] = o.kind == 2 ? o.hn : 0.0f;
    d[3] = o.mo;
    d[4] = o.kind == 3 ? 1.0f : 0.0f;
    d[5] = o.kind == 3 ? o.hn : 0.0f;
    d[6] = o.me;
}

// LDS hand-off between the lanes of ONE wave.  An asm memory clobber, not wavefront fences: from a
// single lane's view a write to x[lane] and a read of x[lane + k] never alias, so without a real
// compiler barrier the read may be hoisted above the other lanes' writes.
__device__ __forceinline__ void wave_sync_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// A "team" runs the per-agent phases of an env: the whole workgroup, or wave 0 alone (kWave) when
// every per-agent count fits in 64 lanes -- then each barrier is a wave-level LDS sync and scans
// and sums are ballots and lane shuffles.
template <bool kWave>
__device__ __forceinline__ void psync() {
    if (kWave) wave_sync_lds();
    else __syncthreads();
}

template <bool kWave>
__device__ __forceinline__ int team_lanes() { return kWave ? 64 : (int)blockDim.x; }

template <bool kWave>
__device__ __forceinline__ int team_scan(int flag, int* wave_tot, int& total) {
    if (!kWave) return block_scan_flag(flag, wave_tot, total);
    const unsigned long long m = __ballot(flag);
    total = __popcll(m);
    return __popcll(m & ((1ull << (TID & 63)) - 1ull));
}

__device__ __forceinline__ float wave_sum(float x) {         // fixed butterfly order
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

// Observation rows are written once and read only by the caller (next kernel / host), never by
// this launch: nontemporal (`nt`) stores keep them from displacing the env images in L2/MALL
// (+7.5 % k_rollout throughput measured, profiles/r01_nt_store_ab.txt).
// copy one staged 64-cell block (cells valid cells) to dst, 16-B aligned when cells == 64
__device__ __forceinline__ void obs_flush(float* __restrict__ dst, const float* st, int lane, int cells) {
    constexpr int NC = BattleShape::NC;
    if (cells == kWaveCells) {
        const f32x4* s4 = reinterpret_cast<const f32x4*>(st);
        f32x4* d4 = reinterpret_cast<f32x4*>(dst);
        __builtin_nontemporal_store(s4[lane], d4 + lane);
        if (lane < kWaveStageFloats / 4 - 64) __builtin_nontemporal_store(s4[64 + lane], d4 + 64 + lane);
    } else {
        for (int i = lane; i < cells * NC; i += 64) __builtin_nontemporal_store(st[i], dst + i);
    }
}

// Global-cells form of obs_cell, split so that a wave can have kObsPf cell loads in flight: the
// LDS-side part (record, mask, minimap, address) ...
struct CellPre {
    int idx;              // cell index to load (0 when the view cell is masked / off the map)
    float mo, me;         // minimap channels (own / enemy, +1 at the agent's own bin)
    bool ok;              // an in-map view cell
};

__device__ __forceinline__ CellPre obs_cell_pre(const ObsSmem& sm, const float* mm_own, const float* mm_en, int W,
                                                int H, int gc, int ncell) {
    constexpr int NV = BattleShape::VW * BattleShape::VH;
    const bool valid = gc < ncell;
    const int gs = valid ? gc : 0;
    const int a = gs / NV, c = gs - a * NV;
    const int vy = c / BattleShape::VW, vx = c - vy * BattleShape::VW;
    const uint32_t q = sm.aq[a];
    const uint32_t mk = (sm.mask[c >> 5] >> (c & 31)) & 1u;
    const float mo = mm_own[c], me = mm_en[c];
    const bool self = c == (int)(q >> 24);
    const int mx = (int)(q & 0xFFFu) - 8 + vx, my = (int)((q >> 12) & 0xFFFu) - 8 + vy;
    CellPre p;
    p.ok = valid && mk != 0 && (unsigned)mx < (unsigned)W && (unsigned)my < (unsigned)H;
    p.idx = p.ok ? my * W + mx : 0;
    p.mo = valid ? (self ? mo + 1.0f : mo) : 0.0f;
    p.me = valid ? (self ? me + 1.0f : me) : 0.0f;
    return p;
}

// ... and the part after the cell's occupant arrived
__device__ __forceinline__ CellObs obs_cell_post(const CellPre& p, uint32_t cv, const ObsSmem& sm, int g) {
    const bool agent = p.ok && cv < kCellFood;
    const uint32_t inf = sm.info[agent ? cv : 0];
    CellObs o;
    o.mo = p.mo;
    o.me = p.me;
    o.hn = agent ? __uint_as_float(inf & 0x7FFFFFFFu) : 0.0f;
    o.kind = (p.ok && cv == kCellWall) ? 1 : (agent ? ((int)(inf >> 31) == g ? 2 : 3) : 0);
    return o;
}

typedef __attribute__((address_space(1))) const uint16_t g_u16;

// obs_stream_battle with the cells in HBM (large envs): each wave issues the cell loads of kObsPf
// 64-cell blocks back to back, then stages and flushes them one by one, so one HBM round trip is
// paid per kObsPf blocks instead of per block (6: +1.5-2.7 % at 256x256 over 4; 8 loses;
// profiles/r01_big_sweeps.txt).  The explicit global address space keeps the
// loads off lgkmcnt (a flat load would be waited for by every LDS sync of the stream).
#ifndef MFX_OBS_PF
#define MFX_OBS_PF 6
#endif
constexpr int kObsPf = MFX_OBS_PF;
__device__ __forceinline__ void obs_stream_battle_global(const GameParams& gp, const EnvView& v, const ObsSmem& sm,
                                                         int g, int n, float* __restrict__ out_view,
                                                         float* __restrict__ out_feat, float* wave_stage) {
    constexpr int NV = BattleShape::VW * BattleShape::VH, NC = BattleShape::NC, F = BattleShape::F;
    const int lane = TID & 63, wid = TID >> 6, nw = blockDim.x >> 6;
    const int W = gp.W, H = gp.H;
    const TypeParams& T = gp.type[g];
    const uint16_t* ids = v.grp_ids + g * v.cap;
    const float* mm_own = sm.mm + g * NV;
    const float* mm_en = sm.mm + (g ^ 1) * NV;
    const int ncell = n * NV;
    g_u16* cells = (g_u16*)v.cells;
    float* st = wave_stage + wid * kWaveStageFloats;
    for (int base = wid * kObsPf * kWaveCells; base < ncell; base += nw * kObsPf * kWaveCells) {
        CellPre p[kObsPf];
        uint32_t cv[kObsPf];
#pragma unroll
        for (int d = 0; d < kObsPf; ++d) p[d] = obs_cell_pre(sm, mm_own, mm_en, W, H, base + d * kWaveCells + lane, ncell);
#pragma unroll
        for (int d = 0; d < kObsPf; ++d) cv[d] = cells[p[d].idx];
#pragma unroll
        for (int d = 0; d < kObsPf; ++d) {
            const int b = base + d * kWaveCells;
            if (b >= ncell) break;
            obs_stage_cell(st, lane, obs_cell_post(p[d], cv[d], sm, g));
            wave_sync_lds();
            obs_flush(out_view + (size_t)b * NC, st, lane, min(kWaveCells, ncell - b));
            wave_sync_lds();
        }
    }
    // features (GridWorld.cc:411-421): consecutive lanes write consecutive floats
    const int emb = gp.emb, na = T.n_action;
    for (int q = TID; q < n * F; q += blockDim.x) {
        const int a = q / F, f = q - a * F;
        const int id = ids[a];
        float val = 0.0f;
        if (f < emb) val = (float)((id >> f) & 1);
        if (f == emb + v.last_act[id]) val = 1.0f;
        if (f == emb + na) val = v.last_r[id];
        const uint32_t pos = v.xy[id];
        if (f == emb + na + 1) val = (float)(int)(pos & 0xFFFF) / (float)W;
        if (f == emb + na + 2) val = (float)(int)(pos >> 16) / (float)H;
        __builtin_nontemporal_store(val, out_feat + q);
    }
}

typedef __attribute__((address_space(1))) const uint32_t g_cu32;

// obs_cell_post with the occupant's info word loaded from HBM too (pipelined like the cells)
__device__ __forceinline__ CellObs obs_cell_post_g(const CellPre& p, uint32_t cv, uint32_t inf, int g) {
    const bool agent = p.ok && cv < kCellFood;
    CellObs o;
    o.mo = p.mo;
    o.me = p.me;
    o.hn = agent ? __uint_as_float(inf & 0x7FFFFFFFu) : 0.0f;
    o.kind = (p.ok && cv == kCellWall) ? 1 : (agent ? ((int)(inf >> 31) == g ? 2 : 3) : 0);
    return o;
}

__device__ __forceinline__ void obs_stream_battle(const GameParams& gp, const EnvView& v, const ObsSmem& sm, int g,
                                                  int n, float* __restrict__ out_view, float* __restrict__ out_feat,
                                                  float* wave_stage) {
    constexpr int NV = BattleShape::VW * BattleShape::VH, NC = BattleShape::NC, F = BattleShape::F;
    const int lane = TID & 63, wid = TID >> 6, nw = blockDim.x >> 6;
    const int W = gp.W, H = gp.H;
    const TypeParams& T = gp.type[g];
    const uint16_t* ids = v.grp_ids + g * v.cap;
    const float* mm_own = sm.mm + g * NV;
    const float* mm_en = sm.mm + (g ^ 1) * NV;
    const int ncell = n * NV;
    for (int base = wid * 2 * kWaveCells; base < ncell; base += nw * 2 * kWaveCells) {
        float* st = wave_stage + wid * kWaveStageFloats;
        const CellObs o0 = obs_cell(v, sm, mm_own, mm_en, W, H, g, base + lane, ncell);
        obs_stage_cell(st, lane, o0);
        wave_sync_lds();
        obs_flush(out_view + (size_t)base * NC, st, lane, min(kWaveCells, ncell - base));
        wave_sync_lds();
        if (base + kWaveCells < ncell) {
            const CellObs o1 = obs_cell(v, sm, mm_own, mm_en, W, H, g, base + kWaveCells + lane, ncell);
            obs_stage_cell(st, lane, o1);
            wave_sync_lds();
            obs_flush(out_view + (size_t)(base + kWaveCells) * NC, st, lane, min(kWaveCells, ncell - base - kWaveCells));
            wave_sync_lds();
        }
    }
    // features (GridWorld.cc:411-421): consecutive lanes write consecutive floats
    const int emb = gp.emb, na = T.n_action;
    for (int p = TID; p < n * F; p += blockDim.x) {
        const int a = p / F, f = p - a * F;
        const int id = ids[a];
        float val = 0.0f;
        if (f < emb) val = (float)((id >> f) & 1);
        if (f == emb + v.last_act[id]) val = 1.0f;
        if (f == emb + na) val = v.last_r[id];
        const uint32_t pos = v.xy[id];
        if (f == emb + na + 1) val = (float)(int)(pos & 0xFFFF) / (float)W;
        if (f == emb + na + 2) val = (float)(int)(pos >> 16) / (float)H;
        __builtin_nontemporal_store(val, out_feat + p);
    }
}

__host__ __device__ inline bool is_battle_shape(const GameParams& gp) {
    if (gp.n_groups != BattleShape::G || !gp.minimap || gp.n_ch != BattleShape::NC || gp.turn_mode || gp.food_mode)
        return false;
    if (gp.W > 4000 || gp.H > 4000) return false;                // packed view origins (obs_agent_records)
    for (int g = 0; g < gp.n_groups; ++g) {
        if (gp.type[g].body_w != 1 || gp.type[g].body_h != 1) return false;
        if (gp.type[g].view_w != BattleShape::VW || gp.type[g].view_h != BattleShape::VH ||
            gp.feat_size[g] != BattleShape::F || gp.type[g].view_x1 != gp.type[0].view_x1 ||
            gp.type[g].view_y1 != gp.type[0].view_y1)
            return false;
        for (int c = 0; c < BattleShape::VW * BattleShape::VH; ++c)
            if (gp.type[g].view_mask[c] != gp.type[0].view_mask[c]) return false;
    }
    return true;
}

// LDS of the observation phase.  stage_floats: the staging area (K rows for the staged path,
// one 448-float slice per wave for the wave-streamed path).
// rows: agents of one group observed per call (records of the wave-streamed path); kB: Battle path
// (no per-id minimap bins).
__host__ __device__ inline size_t obs_smem_core(const GameParams& gp, int g, int cap, int rows, size_t stage_floats,
                                                bool kB) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t NV = (size_t)gp.type[g].view_w * gp.type[g].view_h;
    return r16(stage_floats * 4) + r16((size_t)gp.n_groups * NV * 4) + (kB ? 0 : r16((size_t)cap * 2)) + 16 +
           r16((NV + 31) / 32 * 4) + r16((size_t)cap * 4) + r16((size_t)rows * 4);
}

__device__ __forceinline__ ObsSmem carve_obs(char* smem, const GameParams& gp, int g, int cap, int rows,
                                             size_t stage_floats, bool kB, size_t& off) {
    const TypeParams& T = gp.type[g];
    const size_t NV = (size_t)T.view_w * T.view_h, G = gp.n_groups;
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    ObsSmem sm;
    sm.stage = reinterpret_cast<float*>(smem + off); off += r16(stage_floats * 4);
    sm.mm = reinterpret_cast<float*>(smem + off);    // the histogram is converted in place
    sm.hist = reinterpret_cast<int*>(smem + off);    off += r16(G * NV * 4);
    sm.bin = kB ? nullptr : reinterpret_cast<uint16_t*>(smem + off); off += kB ? 0 : r16((size_t)cap * 2);
    sm.type_hp = reinterpret_cast<float*>(smem + off); off += 16;
    sm.mask = reinterpret_cast<uint32_t*>(smem + off); off += r16((NV + 31) / 32 * 4);
    sm.info = reinterpret_cast<uint32_t*>(smem + off); off += r16((size_t)cap * 4);
    sm.aq = reinterpret_cast<uint32_t*>(smem + off);  off += r16((size_t)rows * 4);
    return sm;
}

__host__ __device__ inline size_t obs_stage_floats(const GameParams& gp, int g, bool wave_streamed, int threads) {
    return wave_streamed ? (size_t)(threads / 64) * kWaveStageFloats
                         : (size_t)kObsK * gp.type[g].view_w * gp.type[g].view_h * gp.n_ch;
}

__device__ __forceinline__ void obs_prologue(const GameParams& gp, const ObsSmem& sm, int g) {
    const TypeParams& T = gp.type[g];
    const int NV = T.view_w * T.view_h;
    for (int w = TID; w < (NV + 31) / 32; w += blockDim.x) sm.mask[w] = T.view_bits[w];
    if (TID < gp.n_groups) sm.type_hp[TID] = gp.type[TID].hp;
}

// grid: (chunks, E).  Chunk c covers agents [c*chunk, (c+1)*chunk) of group g.
// out_view: [E][rowcap][VH][VW][NC], out_feat: [E][rowcap][F]
// grid: (chunks, E).  Chunk c covers agents [c*chunk, (c+1)*chunk) of group g.
// out_view: [E][rowcap][VH][VW][NC], out_feat: [E][rowcap][F]
template <bool kB>
__global__ void __launch_bounds__(256) k_observe(const GameParams* __restrict__ gpp, State s, int g, int chunk,
                                                 float* __restrict__ out_view, float* __restrict__ out_feat,
                                                 int rowcap, int cells_in_lds) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const GameParams& gp = *gpp;
    const int e = blockIdx.y, G = gp.n_groups;
    EnvView v = global_view(s, e, G);
    const int n = v.grp_n[g];
    const int a_begin = blockIdx.x * chunk;
    if (a_begin >= n) return;
    const int a_end = min(n, a_begin + chunk);
    if (a_end > rowcap) { if (TID == 0) set_err(s, 4); return; }
    size_t off = 0;
    ObsSmem sm = carve_obs(smem, gp, g, s.cap, chunk, obs_stage_floats(gp, g, kB, blockDim.x), kB, off);
    if (!kB) sm.info = nullptr;
    if (cells_in_lds) {
        uint16_t* lc = reinterpret_cast<uint16_t*>(smem + off);
        const int n2 = s.cells_n;
        for (int i = TID; i < n2; i += blockDim.x) lc[i] = v.cells[i];
        v.cells = lc;
    }
    obs_prologue(gp, sm, g);
    obs_minimap<kB>(gp, v, sm, g);
    const TypeParams& T = gp.type[g];
    const size_t VF = (size_t)T.view_w * T.view_h * gp.n_ch;
    const int F = gp.feat_size[g];
    float* ov = out_view + (size_t)e * rowcap * VF;
    float* of = out_feat + (size_t)e * rowcap * F;
    if (kB) {
        EnvView vc = v;                      // rows [a_begin, a_end): shift the group list and outputs
        vc.grp_ids = v.grp_ids + a_begin;
        const int na = a_end - a_begin;
        obs_agent_records(gp, vc, sm, g, na);
        __syncthreads();
        float* ovc = ov + (size_t)a_begin * VF;
        float* ofc = of + (size_t)a_begin * F;
        if (cells_in_lds) obs_stream_battle(gp, vc, sm, g, na, ovc, ofc, sm.stage);
        else obs_stream_battle_global(gp, vc, sm, g, na, ovc, ofc, sm.stage);
    } else {
        for (int a0 = a_begin; a0 < a_end; a0 += kObsK) obs_rows<kB>(gp, v, sm, g, a0, min(kObsK, a_end - a0), ov, of);
    }
}

// ==================================================================================
//  set_action (GridWorld.cc:430-496): classify in call order and append to the buffers.
// ==================================================================================
template <bool kW>
__device__ __forceinline__ void set_action_group(const GameParams& gp, const State& s, EnvView& v, int g,
                                                 const int* __restrict__ acts, uint32_t* atk, int& n_atk,
                                                 uint32_t* mov, int& n_mov, int* wave_tot, int acap) {
    const TypeParams& T = gp.type[g];
    const int n = v.grp_n[g];
    int base_a = n_atk, base_m = n_mov;
    psync<kW>();
    for (int i0 = 0; i0 < n; i0 += team_lanes<kW>()) {
        const int i = i0 + TID;
        int a = 0, id = 0, is_move = 0, is_atk = 0;
        uint32_t bucket = kBucketBoundary;
        if (i < n) {
            id = v.grp_ids[g * v.cap + i];
            a = acts[i];
            if (a < 0 || a >= T.n_action) { set_err(s, 5); a = T.turn_base > 6 ? 6 : 0; }
            v.last_act[id] = a;
            is_move = a < T.attack_base;                  // moves and turns (same buckets, GridWorld.cc:443-470)
            is_atk = !is_move;
            if (is_move && gp.large_map) {
                const int x = v.xy[id] & 0xFFFF, xr = x % gp.band_w;
                if (!(xr < 4 || xr > gp.band_w - 4)) bucket = (uint32_t)(x / gp.band_w);
            }
        }
        int tot_m, tot_a;
        const int rm = team_scan<kW>(is_move, wave_tot, tot_m);
        const int ra = team_scan<kW>(is_atk, wave_tot, tot_a);
        if (is_move && base_m + rm < acap) mov[base_m + rm] = ((uint32_t)id << 16) | ((uint32_t)a << 8) | bucket;
        if (is_atk && base_a + ra < acap) atk[base_a + ra] = ((uint32_t)id << 8) | (uint32_t)(a - T.attack_base);
        base_m += tot_m;
        base_a += tot_a;
    }
    if (base_m > acap || base_a > acap) { if (TID == 0) set_err(s, 6); }
    psync<kW>();
    if (TID == 0) { n_atk = min(base_a, acap); n_mov = min(base_m, acap); }
    psync<kW>();
}

__global__ void __launch_bounds__(256) k_set_action(const GameParams* __restrict__ gp, State s, int g,
                                                    const int* __restrict__ actions, int rowcap) {
    __shared__ int wave_tot[16];
    const int e = blockIdx.x;
    EnvView v = global_view(s, e, gp->n_groups);
    if (v.grp_n[g] > rowcap) { if (TID == 0) set_err(s, 4); return; }
    set_action_group<false>(*gp, s, v, g, actions + (size_t)e * rowcap, s.atk + (size_t)e * s.acap, s.n_atk[e],
                     s.mov + (size_t)e * s.acap, s.n_mov[e], wave_tot, s.acap);
}

// ==================================================================================
//  step (GridWorld.cc:498-694)
// ==================================================================================
struct SerialType {          // what the one-lane loops read per group, kept in LDS (the group
    float hp, damage, kill_supply, kill_reward, dead_penalty, attack_penalty;   // index is
    int attack_in_group, att_x_off, att_y_off, pad;                              // lane-varying:
    int n_attack, turn_base, attack_base, n_action;
    int body_w, body_h;
    float eat_ability, food_supply;
    int8_t att_dx[kMaxRangeCount], att_dy[kMaxRangeCount];                       // from global it
    int8_t move_dx[kMaxRangeCount], move_dy[kMaxRangeCount];                     // would be a vector
};                                                                               // load per use)

struct StepSmem {
    int wave_tot[16];
    int flags[8];       // [0..kMaxRules) rule triggers
    SerialType tt[kMaxGroups];
};

// StepSmem lives in dynamic LDS with room for the env's G type entries only.
__host__ __device__ inline size_t step_sm_bytes(int G) {
    return ((offsetof(StepSmem, tt) + (size_t)G * sizeof(SerialType)) + 15) & ~(size_t)15;
}

__device__ __forceinline__ void load_serial_types(const GameParams& gp, StepSmem& sm) {
    for (int g = 0; g < gp.n_groups; ++g) {
        const TypeParams& T = gp.type[g];
        SerialType& S = sm.tt[g];
        const int t = TID;
        if (t < kMaxRangeCount) {
            S.att_dx[t] = T.att_dx[t]; S.att_dy[t] = T.att_dy[t];
            S.move_dx[t] = T.move_dx[t]; S.move_dy[t] = T.move_dy[t];
        }
        if (t == 0) {
            S.hp = T.hp; S.damage = T.damage; S.kill_supply = T.kill_supply; S.kill_reward = T.kill_reward;
            S.dead_penalty = T.dead_penalty; S.attack_penalty = T.attack_penalty;
            S.attack_in_group = T.attack_in_group; S.att_x_off = T.att_x_off; S.att_y_off = T.att_y_off;
            S.n_attack = T.n_attack; S.turn_base = T.turn_base; S.attack_base = T.attack_base;
            S.n_action = T.n_action;
            S.body_w = T.body_w; S.body_h = T.body_h;
            S.eat_ability = T.eat_ability; S.food_supply = T.food_supply;
        }
    }
}

// ev (render, GridWorld.cc:531-535): every live attacker's (id, target x, target y), blank or not.
__device__ __forceinline__ void do_attack_serial(const GameParams& gp, const StepSmem& sm, EnvView& v, uint32_t* atk,
                                                 int n_atk, int32_t* ev) {
    // shuffled order, strictly sequential (the reference loop is racy with OMP>1; OMP=1 semantics)
    const int W = gp.W, H = gp.H;
    for (int i = 0; i < n_atk; ++i) {
        const uint32_t ent = atk[i];
        const int id = (int)(ent >> 8), ai = (int)(ent & 0xFF);
        uint32_t m = v.meta[id];
        if (meta_dead(m)) continue;
        const int g = meta_group(m);
        const SerialType& T = sm.tt[g];
        const uint32_t p = v.xy[id];
        int ox = (int)(p & 0xFFFF) + T.att_x_off + T.att_dx[ai];
        int oy = (int)(p >> 16) + T.att_y_off + T.att_dy[ai];
        if (gp.turn_mode) {                            // Map::get_attack_obj (Map.cc:220-263)
            const int dir = meta_dir(m);
            int rx, ry;
            save_to_real((int)(p & 0xFFFF), (int)(p >> 16), dir, T.body_w, T.body_h, rx, ry);
            rela_to_abs(rx, ry, dir, T.att_x_off + T.att_dx[ai], T.att_y_off + T.att_dy[ai], ox, oy);
        }
        if (ev) {
            const int k = ev[0];
            ev[1 + 3 * k] = id; ev[2 + 3 * k] = ox; ev[3 + 3 * k] = oy;
            ev[0] = k + 1;
        }
        uint32_t cv = kCellEmpty;
        if (ox >= 0 && ox < W && oy >= 0 && oy < H) cv = v.cells[oy * W + ox];
        if (cv >= kCellWall) { v.next_r[id] += T.attack_penalty; continue; }       // blank
        if (cv == kCellFood) {                       // Map::do_attack, OCC_FOOD (Map.cc:296-307)
            float& f = v.food[oy * W + ox];
            const float add = T.eat_ability < f ? T.eat_ability : f;
            const float h2 = v.hp[id] + add;
            v.hp[id] = T.hp < h2 ? T.hp : h2;
            f -= add;
            if ((double)f < 0.1) v.cells[oy * W + ox] = kCellEmpty;
            v.next_r[id] += 0.0f + T.attack_penalty;
            continue;
        }
        const uint32_t om = v.meta[cv];
        const int og = meta_group(om);
        if (!T.attack_in_group && og == g) { v.next_r[id] += T.attack_penalty; continue; }
        const SerialType& OT = sm.tt[og];
        float reward = 0.0f;
        const float ohp = v.hp[cv] - T.damage;                                    // Agent::be_attack
        v.hp[cv] = ohp;
        if (ohp < 0.0f) {
            v.meta[cv] = (uint8_t)meta_keep_dir(meta_make(1, meta_op(om), og), om);
            v.next_r[cv] = OT.dead_penalty;
            m = meta_keep_dir(meta_make(0, kOpKill, g), m);
            v.op_obj[id] = (int)cv;
            const uint32_t vp = v.xy[cv];                                           // remove_agent
            int vbw, vbh;
            size_for_dir(meta_dir(om), OT.body_w, OT.body_h, vbw, vbh);
            fill_area(v.cells, W, (int)(vp & 0xFFFF), (int)(vp >> 16), vbw, vbh, kCellEmpty);
            if (gp.food_mode) {                                                     // Map.cc:287-294
                v.cells[oy * W + ox] = kCellFood;
                v.food[oy * W + ox] = OT.food_supply;
            }
            v.grp_dead[og] += 1;
            const float h2 = v.hp[id] + OT.kill_supply;                             // add_hp
            v.hp[id] = T.hp < h2 ? T.hp : h2;
            reward = OT.kill_reward;
        } else {
            m = meta_keep_dir(meta_make(0, kOpAttack, g), m);
            v.op_obj[id] = (int)cv;
        }
        v.meta[id] = (uint8_t)m;
        v.next_r[id] += reward + T.attack_penalty;
    }
}

__device__ __forceinline__ void do_move_one(const GameParams& gp, const StepSmem& sm, EnvView& v, uint32_t ent) {
    // GridWorld.cc:631-660 + Map::do_move (Map.cc:324-369), NORTH, 1x1
    const int id = (int)(ent >> 16), mi = (int)((ent >> 8) & 0xFF);
    const uint32_t m = v.meta[id];
    if (meta_dead(m)) return;
    const int W = gp.W, H = gp.H;
    const SerialType& T = sm.tt[meta_group(m)];
    const uint32_t p = v.xy[id];
    const int x = p & 0xFFFF, y = p >> 16;
    if (mi >= T.turn_base) return;                 // a turn (turn_mode): done before the moves
    int dx = T.move_dx[mi], dy = T.move_dy[mi];
    const int dir = meta_dir(m);                   // GridWorld.cc:640-652
    if (dir == kDirSouth) { dx = -dx; dy = -dy; }
    else if (dir == kDirWest) { const int t = dx; dx = dy; dy = -t; }
    else if (dir == kDirEast) { const int t = dx; dx = -dy; dy = t; }
    const int nx = x + dx, ny = y + dy;
    if (T.body_w == 1 && T.body_h == 1) {
        if (nx < 0 || ny < 0 || nx + 1 >= W || ny + 1 >= H) return;     // out of board: no collide
        const uint32_t cv = v.cells[ny * W + nx];
        if (cv == kCellEmpty || (int)cv == id) {
            v.cells[y * W + x] = kCellEmpty;
            v.cells[ny * W + nx] = (uint16_t)id;
            v.xy[id] = (uint32_t)nx | ((uint32_t)ny << 16);
        } else if (cv < kCellFood) {
            v.meta[id] = (uint8_t)meta_keep_dir(meta_make(0, kOpCollide, meta_group(m)), m);
            v.op_obj[id] = (int)cv;
        }
        return;
    }
    int bw, bh;
    size_for_dir(dir, T.body_w, T.body_h, bw, bh);
    if (is_blank_area(v.cells, W, H, nx, ny, bw, bh, id)) {
        fill_area(v.cells, W, x, y, bw, bh, kCellEmpty);
        fill_area(v.cells, W, nx, ny, bw, bh, (uint16_t)id);
        v.xy[id] = (uint32_t)nx | ((uint32_t)ny << 16);
    } else {
        const int c = get_collide(v.cells, W, H, nx, ny, bw, bh, id);
        if (c >= 0) {
            v.meta[id] = (uint8_t)meta_keep_dir(meta_make(0, kOpCollide, meta_group(m)), m);
            v.op_obj[id] = c;
        }
    }
}

// Map::do_turn (Map.cc:372-410) as the step calls it: the action a in [turn_base, attack_base) turns by
// wise = 2a - 1 (GridWorld.cc:605), so the new direction is (dir + 2a - 1) mod 4 and, wise never
// being -1, the body pivots with the clockwise formula about its real corner (turn offsets are 0).
__device__ __forceinline__ void do_turn_one(const GameParams& gp, const StepSmem& sm, EnvView& v, uint32_t ent) {
    const int id = (int)(ent >> 16), a = (int)((ent >> 8) & 0xFF);
    const uint32_t m = v.meta[id];
    if (meta_dead(m)) return;
    const SerialType& T = sm.tt[meta_group(m)];
    if (a < T.turn_base) return;                   // a move
    const int W = gp.W, H = gp.H;
    const int wise = 2 * a - 1;
    const int dir = meta_dir(m), ndir = (dir + wise + 4) % 4;
    int bw, bh;
    size_for_dir(dir, T.body_w, T.body_h, bw, bh);
    const uint32_t p = v.xy[id];
    const int x = (int)(p & 0xFFFF), y = (int)(p >> 16);
    int rx, ry, ax, ay;
    save_to_real(x, y, dir, T.body_w, T.body_h, rx, ry);
    rela_to_abs(rx, ry, dir, 0, 0, ax, ay);        // anchor: turn_x_offset = turn_y_offset = 0
    const int ddx = rx - ax, ddy = ry - ay;
    const int nrx = ax + ddy, nry = ay - ddx;
    int sx, sy;
    real_to_save(nrx, nry, ndir, T.body_w, T.body_h, sx, sy);
    if (is_blank_area(v.cells, W, H, sx, sy, bh, bw, id)) {
        fill_area(v.cells, W, x, y, bw, bh, kCellEmpty);
        v.meta[id] = (uint8_t)meta_set_dir(m, ndir);
        fill_area(v.cells, W, sx, sy, bh, bw, (uint16_t)id);
        v.xy[id] = (uint32_t)sx | ((uint32_t)sy << 16);
    }
}

// ==================================================================================
//  parallel exact resolution of the order-dependent part of the step (gp.par_step)
// ==================================================================================
// The reference resolves the shuffled attacks and then the moves one by one
// (GridWorld.cc:507-558, 631-672).  The same results come out of a few data-parallel passes:
//  * shuffle: x_k = 16807^(k+1) x0 mod (2^31-1) (minstd jump-ahead), so every j_k = x_k % (k+1)
//    is independent; the forward Fisher-Yates then moves element i to j_i and on to k whenever a
//    later j_k hits its current position.
//  * attacks: with kill_supply == 0 a kill changes nothing but the victim, so the outcome is fixed
//    by the position at which each agent dies.  Iterate: assume the current death positions, let
//    every attack replay the sequential hp updates of its target up to itself (hits of attackers
//    still alive at their turn), and record where each target now dies.  Iteration t fixes the
//    t-th kill in shuffle order, so the loop ends after (#kills + 1) passes.
//  * moves: a mover may be resolved once it is the earliest unresolved mover that touches its
//    source or its target cell -- every earlier event on both cells is then applied, and no later
//    one is.  Rounds of "claim both cells (atomicMin), resolve the owners" reach the fixed
//    sequential order; a hashed claim table only adds false conflicts (extra rounds).
constexpr int kOwnerSlots = 512;
constexpr int16_t kNoDeath = 0x7FFF;

struct ParScratch {
    uint32_t* ord;       // [acap] attack entries in shuffled order
    uint16_t* jv;        // [acap] Fisher-Yates j_k
    uint16_t* att;       // [acap] attacker id by position
    int16_t* tgt;        // [acap] target id at phase start; -1 blank; -2 attacker already dead
    int16_t* eff;        // [acap] target if this position is a hit under the current deaths, else -1
    float* dmg;          // [acap] attacker damage by position
    int16_t* death;      // [cap] position of the attack that kills id, or kNoDeath
    int16_t* death_new;  // [cap]
    uint32_t* owner;     // [kOwnerSlots] move rounds (aliases the attack arrays)
    int* flag;           // [1]
};

__host__ __device__ inline size_t par_scratch_bytes(int acap, int cap) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t atk = r16((size_t)acap * 4) + 3 * r16((size_t)acap * 2) + r16((size_t)acap * 2) +
                       r16((size_t)acap * 4) + 2 * r16((size_t)cap * 2);
    const size_t mov = r16((size_t)kOwnerSlots * 4);
    return (atk > mov ? atk : mov) + 16;
}

__device__ __forceinline__ ParScratch carve_par(char* base, int acap, int cap) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    ParScratch p;
    size_t o = 0;
    p.ord = reinterpret_cast<uint32_t*>(base + o);  o += r16((size_t)acap * 4);
    p.jv = reinterpret_cast<uint16_t*>(base + o);   o += r16((size_t)acap * 2);
    p.att = reinterpret_cast<uint16_t*>(base + o);  o += r16((size_t)acap * 2);
    p.tgt = reinterpret_cast<int16_t*>(base + o);   o += r16((size_t)acap * 2);
    p.eff = reinterpret_cast<int16_t*>(base + o);   o += r16((size_t)acap * 2);
    p.dmg = reinterpret_cast<float*>(base + o);     o += r16((size_t)acap * 4);
    p.death = reinterpret_cast<int16_t*>(base + o); o += r16((size_t)cap * 2);
    p.death_new = reinterpret_cast<int16_t*>(base + o); o += r16((size_t)cap * 2);
    p.owner = reinterpret_cast<uint32_t*>(base);    // move rounds run after the attacks
    const size_t mov = r16((size_t)kOwnerSlots * 4);
    p.flag = reinterpret_cast<int*>(base + (o > mov ? o : mov));
    return p;
}

__device__ __forceinline__ uint32_t mulmod_m31(uint32_t a, uint32_t b) {
    uint64_t p = (uint64_t)a * b;
    p = (p & 0x7FFFFFFFull) + (p >> 31);
    p = (p & 0x7FFFFFFFull) + (p >> 31);
    if (p >= 0x7FFFFFFFull) p -= 0x7FFFFFFFull;
    return (uint32_t)p;
}

__device__ __forceinline__ uint32_t minstd_jump(uint32_t x0, uint32_t k) {   // k draws ahead of x0
    uint32_t r = x0, b = 16807u;
    while (k) {
        if (k & 1u) r = mulmod_m31(r, b);
        b = mulmod_m31(b, b);
        k >>= 1;
    }
    return r;
}


// Value of lane q of a wave-uniform loop (v_readlane: q must be uniform; ignores EXEC).
__device__ __forceinline__ int lane_i(int x, int q) { return __builtin_amdgcn_readlane(x, q); }
__device__ __forceinline__ float lane_f(float x, int q) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), q));
}

// attack_parallel for one wave (n <= 64): the same passes, with every per-position array that a lane
// scans (j_k, the hits, their damage) held one entry per lane and read with v_readlane in
// wave-uniform loops instead of a dependent chain of LDS loads; the fixed point keeps one "kills its
// target here" bit per position, so a pass that changes nothing is a ballot.
__device__ void attack_wave(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* atk, int n,
                            uint32_t& rng, const ParScratch& ps, int nid) {
    const int t = TID, W = gp.W, H = gp.H;
    // ---- shuffle: element t sits at j_t, then moves to every later k with j_k == its position
    uint32_t ent = 0;
    int jv = -1;
    if (t < n) {
        ent = atk[t];
        const uint32_t x = minstd_jump(rng, (uint32_t)t + 1u);
        jv = (int)(x % (uint32_t)(t + 1));
        if (t == n - 1) ps.flag[0] = (int)x;
    }
    for (int id = t; id < nid; id += 64) ps.death[id] = kNoDeath;
    int p = jv;
    for (int k = 1; k < n; ++k) {
        const int jk = lane_i(jv, k);
        if (k > t && jk == p) p = k;
    }
    if (t < n) ps.ord[p] = ent;
    wave_sync_lds();
    if (n > 0) rng = (uint32_t)ps.flag[0];
    // ---- per position: attacker, damage, target at phase start
    int A = -1, T = -2;
    float dmg = 0.0f;
    if (t < n) {
        const uint32_t e2 = ps.ord[t];
        A = (int)(e2 >> 8);
        const int ai = (int)(e2 & 0xFF);
        const uint32_t m = v.meta[A];
        if (!meta_dead(m)) {
            const int g = meta_group(m);
            const SerialType& S = sm.tt[g];
            const uint32_t pos = v.xy[A];
            const int ox = (int)(pos & 0xFFFF) + S.att_x_off + S.att_dx[ai];
            const int oy = (int)(pos >> 16) + S.att_y_off + S.att_dy[ai];
            uint32_t cv = kCellEmpty;
            if (ox >= 0 && ox < W && oy >= 0 && oy < H) cv = v.cells[oy * W + ox];
            T = -1;
            if (cv < kCellFood && (S.attack_in_group || (int)meta_group(v.meta[cv]) != g)) T = (int)cv;
            dmg = S.damage;
        }
    }
    const float hT = T >= 0 ? v.hp[T] : 0.0f;
    wave_sync_lds();
    // ---- fixed point on the death positions: kill = "this position's hit kills its target"
    bool kill = false;
    int eff = -1;
    for (int it = 0; it <= n + 1; ++it) {
        eff = (T >= 0 && ps.death[A] > t) ? T : -1;
        bool nk = false;
        if (eff >= 0) {
            float h = hT;
            bool stop = false;
            for (int q = 0; q < n; ++q) {
                const int eq = lane_i(eff, q);
                const float dq = lane_f(dmg, q);
                if (!stop && q <= t && eq == T) {
                    h = h - dq;                                  // Agent::be_attack
                    if (h < 0.0f) { stop = true; nk = q == t; }
                }
            }
        }
        if (__ballot(nk != kill) == 0ull) break;
        wave_sync_lds();                                         // every death[A] read is done
        if (kill && !nk) ps.death[T] = kNoDeath;
        wave_sync_lds();
        if (nk) ps.death[T] = (int16_t)t;
        kill = nk;
        wave_sync_lds();
    }
    // ---- apply: attackers (each agent attacks at most once per step), then hp, then deaths
    eff = (T >= 0 && ps.death[A] > t && ps.death[T] >= t) ? T : -1;
    bool last = false;
    float hl = 0.0f;
    if (eff >= 0) {                          // the last hit on T sets its hp: replay the hits up to it
        last = true;
        float h = hT;
        for (int q = 0; q < n; ++q) {
            const int eq = lane_i(eff, q);
            const float dq = lane_f(dmg, q);
            if (eq == T) {
                if (q <= t) h = h - dq;
                else last = false;
            }
        }
        hl = h;
    }
    if (t < n && T != -2 && ps.death[A] > t) {
        const uint32_t m = v.meta[A];
        const int g = meta_group(m);
        const SerialType& S = sm.tt[g];
        if (eff < 0) {
            v.next_r[A] += S.attack_penalty;                     // blank area (or a dead target)
        } else {
            const bool k = ps.death[T] == t;
            v.meta[A] = (uint8_t)meta_make(0, k ? kOpKill : kOpAttack, g);
            v.op_obj[A] = T;
            const float reward = k ? sm.tt[meta_group(v.meta[T])].kill_reward : 0.0f;
            v.next_r[A] += reward + S.attack_penalty;
        }
    }
    wave_sync_lds();
    if (last) v.hp[T] = hl;
    for (int id = t; id < nid; id += 64) {
        if (ps.death[id] == kNoDeath) continue;
        const uint32_t om = v.meta[id];
        const int og = meta_group(om);
        v.meta[id] = (uint8_t)meta_make(1, meta_op(om), og);
        v.next_r[id] = sm.tt[og].dead_penalty;
        const uint32_t pos = v.xy[id];
        v.cells[(pos >> 16) * W + (pos & 0xFFFF)] = kCellEmpty;   // remove_agent
        atomicAdd(&v.grp_dead[og], 1);
    }
    wave_sync_lds();
}

// Shuffle + attack resolution for n_atk <= lanes.  Leaves the attack effects applied to v.
template <bool kWave>
__device__ void attack_parallel(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* atk,
                                int n, uint32_t& rng, const ParScratch& ps, int nid) {
#ifndef MFX_ATTACK_LDS_SCAN
    if (kWave) { attack_wave(gp, sm, v, atk, n, rng, ps, nid); return; }
#endif
    const int t = TID, W = gp.W, H = gp.H;
    // ---- shuffle
    uint32_t ent = 0;
    if (t < n) {
        ent = atk[t];
        const uint32_t x = minstd_jump(rng, (uint32_t)t + 1u);
        ps.jv[t] = (uint16_t)(x % (uint32_t)(t + 1));
        if (t == n - 1) ps.flag[0] = (int)x;
    }
    for (int id = t; id < nid; id += (kWave ? 64 : (int)blockDim.x)) ps.death[id] = kNoDeath;
    psync<kWave>();
    if (n > 0) rng = (uint32_t)ps.flag[0];
    if (t < n) {
        int p = ps.jv[t];
        for (int k = t + 1; k < n; ++k) if (ps.jv[k] == p) p = k;
        ps.ord[p] = ent;
    }
    psync<kWave>();
    // ---- per position: attacker, damage, target at phase start
    int A = -1, T = -2;
    if (t < n) {
        const uint32_t e2 = ps.ord[t];
        A = (int)(e2 >> 8);
        const int ai = (int)(e2 & 0xFF);
        const uint32_t m = v.meta[A];
        if (!meta_dead(m)) {
            const int g = meta_group(m);
            const SerialType& S = sm.tt[g];
            const uint32_t pos = v.xy[A];
            const int ox = (int)(pos & 0xFFFF) + S.att_x_off + S.att_dx[ai];
            const int oy = (int)(pos >> 16) + S.att_y_off + S.att_dy[ai];
            uint32_t cv = kCellEmpty;
            if (ox >= 0 && ox < W && oy >= 0 && oy < H) cv = v.cells[oy * W + ox];
            T = -1;
            if (cv < kCellFood && (S.attack_in_group || (int)meta_group(v.meta[cv]) != g)) T = (int)cv;
            ps.dmg[t] = S.damage;
        }
        ps.att[t] = (uint16_t)A;
        ps.tgt[t] = (int16_t)T;
    }
    psync<kWave>();
    // ---- fixed point on the death positions
    for (int it = 0; it <= n + 1; ++it) {
        if (t < n) ps.eff[t] = (T >= 0 && ps.death[A] > t) ? (int16_t)T : (int16_t)-1;
        for (int id = t; id < nid; id += (kWave ? 64 : (int)blockDim.x)) ps.death_new[id] = kNoDeath;
        if (t == 0) ps.flag[0] = 0;
        psync<kWave>();
        if (t < n && ps.eff[t] >= 0) {
            float h = v.hp[T];
            for (int q = 0; q <= t; ++q) {
                if (ps.eff[q] != T) continue;
                h = h - ps.dmg[q];                               // Agent::be_attack
                if (h < 0.0f) {
                    if (q == t) ps.death_new[T] = (int16_t)t;
                    break;
                }
            }
        }
        psync<kWave>();
        for (int id = t; id < nid; id += (kWave ? 64 : (int)blockDim.x))
            if (ps.death_new[id] != ps.death[id]) { ps.death[id] = ps.death_new[id]; ps.flag[0] = 1; }
        psync<kWave>();
        if (!ps.flag[0]) break;
        psync<kWave>();
    }
    // ---- apply: attackers (each agent attacks at most once per step), then hp, then deaths.
    // eff = the hits; jv / ord (free after the shuffle) carry "last hit on its target" / its hp.
    if (t < n) ps.eff[t] = (T >= 0 && ps.death[A] > t && ps.death[T] >= t) ? (int16_t)T : (int16_t)-1;
    psync<kWave>();
    bool last = false;
    if (t < n && T != -2 && ps.death[A] > t) {
        const uint32_t m = v.meta[A];
        const int g = meta_group(m);
        const SerialType& S = sm.tt[g];
        if (ps.eff[t] < 0) {
            v.next_r[A] += S.attack_penalty;                     // blank area (or a dead target)
        } else {
            const bool kill = ps.death[T] == t;
            v.meta[A] = (uint8_t)meta_make(0, kill ? kOpKill : kOpAttack, g);
            v.op_obj[A] = T;
            const float reward = kill ? sm.tt[meta_group(v.meta[T])].kill_reward : 0.0f;
            v.next_r[A] += reward + S.attack_penalty;
            // the last hit on T sets its hp: replay the hits on T up to this one
            last = true;
            for (int q = t + 1; q < n; ++q) if (ps.eff[q] == T) { last = false; break; }
            if (last) {
                float h = v.hp[T];
                for (int q = 0; q <= t; ++q) if (ps.eff[q] == T) h = h - ps.dmg[q];
                ps.ord[t] = __float_as_uint(h);
            }
        }
    }
    psync<kWave>();
    if (last) v.hp[T] = __uint_as_float(ps.ord[t]);
    for (int id = t; id < nid; id += (kWave ? 64 : (int)blockDim.x)) {
        if (ps.death[id] == kNoDeath) continue;
        const uint32_t om = v.meta[id];
        const int og = meta_group(om);
        v.meta[id] = (uint8_t)meta_make(1, meta_op(om), og);
        v.next_r[id] = sm.tt[og].dead_penalty;
        const uint32_t pos = v.xy[id];
        v.cells[(pos >> 16) * W + (pos & 0xFFFF)] = kCellEmpty;   // remove_agent
        atomicAdd(&v.grp_dead[og], 1);
    }
    psync<kWave>();
}

// move_parallel for one wave (n <= 64).  A mover resolves once no earlier pending mover touches
// its source or target cell; the cells never change, so each lane's set of earlier movers sharing a
// cell is one 64-bit mask built once (v_readlane over the movers), and every round is a ballot.
__device__ void move_wave(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* order, int n) {
    const int t = TID, W = gp.W, H = gp.H;
    int id = -1, src = -1, dst = -2, nx = 0, ny = 0;
    bool pending = false;
    if (t < n) {
        const uint32_t ent = order[t];
        id = (int)(ent >> 16);
        const int mi = (int)((ent >> 8) & 0xFF);
        const uint32_t m = v.meta[id];
        if (!meta_dead(m)) {
            const SerialType& S = sm.tt[meta_group(m)];
            const uint32_t p = v.xy[id];
            const int x = p & 0xFFFF, y = p >> 16;
            nx = x + S.move_dx[mi]; ny = y + S.move_dy[mi];
            // out of board: no-op; a move onto itself succeeds without changing anything
            pending = !(nx < 0 || ny < 0 || nx + 1 >= W || ny + 1 >= H) && !(nx == x && ny == y);
            src = y * W + x; dst = ny * W + nx;
        }
    }
    if (!pending) { src = -1; dst = -2; }   // claims nothing
    unsigned long long conf = 0;
    for (int q = 0; q < n; ++q) {
        const int sq = lane_i(src, q), dq = lane_i(dst, q);
        if (q < t && (sq == src || sq == dst || dq == src || dq == dst)) conf |= 1ull << q;
    }
    unsigned long long pend = __ballot(pending);
    while (pend) {
        if (pending && (conf & pend) == 0) {
            const uint32_t cv = v.cells[dst];
            if (cv == kCellEmpty) {
                v.cells[src] = kCellEmpty;
                v.cells[dst] = (uint16_t)id;
                v.xy[id] = (uint32_t)nx | ((uint32_t)ny << 16);
            } else if (cv < kCellFood) {
                v.meta[id] = (uint8_t)meta_make(0, kOpCollide, meta_group(v.meta[id]));
                v.op_obj[id] = (int)cv;
            }
            pending = false;
        }
        wave_sync_lds();
        pend = __ballot(pending);
    }
}

// Move resolution for n_mov <= lanes in `order` (buffer order, or band order on large maps).
template <bool kWave>
__device__ void move_parallel(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* order, int n,
                              const ParScratch& ps) {
#ifndef MFX_MOVE_OWNER_ROUNDS
    if (kWave) { move_wave(gp, sm, v, order, n); return; }
#endif
    const int t = TID, W = gp.W, H = gp.H;
    int id = -1, src = 0, dst = 0, nx = 0, ny = 0;
    bool pending = false;
    if (t < n) {
        const uint32_t ent = order[t];
        id = (int)(ent >> 16);
        const int mi = (int)((ent >> 8) & 0xFF);
        const uint32_t m = v.meta[id];
        if (!meta_dead(m)) {
            const SerialType& S = sm.tt[meta_group(m)];
            const uint32_t p = v.xy[id];
            const int x = p & 0xFFFF, y = p >> 16;
            nx = x + S.move_dx[mi]; ny = y + S.move_dy[mi];
            // out of board: no-op; a move onto itself succeeds without changing anything
            pending = !(nx < 0 || ny < 0 || nx + 1 >= W || ny + 1 >= H) && !(nx == x && ny == y);
            src = y * W + x; dst = ny * W + nx;
        }
    }
    const uint32_t hs = (uint32_t)src % kOwnerSlots, hd = (uint32_t)dst % kOwnerSlots;
    for (int round = 0; round <= n; ++round) {
        for (int k = t; k < kOwnerSlots; k += (kWave ? 64 : (int)blockDim.x)) ps.owner[k] = 0xFFFFFFFFu;
        if (t == 0) ps.flag[0] = 0;
        psync<kWave>();
        if (pending) { atomicMin(&ps.owner[hs], (uint32_t)t); atomicMin(&ps.owner[hd], (uint32_t)t); }
        psync<kWave>();
        if (pending) {
            if (ps.owner[hs] == (uint32_t)t && ps.owner[hd] == (uint32_t)t) {
                const uint32_t cv = v.cells[dst];
                if (cv == kCellEmpty) {
                    v.cells[src] = kCellEmpty;
                    v.cells[dst] = (uint16_t)id;
                    v.xy[id] = (uint32_t)nx | ((uint32_t)ny << 16);
                } else if (cv < kCellFood) {
                    v.meta[id] = (uint8_t)meta_make(0, kOpCollide, meta_group(v.meta[id]));
                    v.op_obj[id] = (int)cv;
                }
                pending = false;
            } else {
                ps.flag[0] = 1;
            }
        }
        psync<kWave>();
        if (!ps.flag[0]) break;
        psync<kWave>();
    }
}

// ==================================================================================
//  parallel step for envs too large for one workgroup's lanes (256x256 / 4096 agents)
// ==================================================================================
// Same exact semantics as attack_parallel / move_parallel, with the state in HBM, the whole
// (1024-lane) workgroup as the team and every per-entry loop strided, so the cost grows
// O(n log n) instead of O(n^2):
//  * shuffle: element t sits at jv[t] after Fisher-Yates step t and moves again only at a later
//    step k with jv[k] == its position.  Buckets L(v) = {k > v : jv[k] == v} (CSR, sorted) give
//    the first later hit (successor of t in L(jv[t])) and then min L(p) per hop.
//  * attacks: the hits on every target in shuffle order (CSR by target, <= 8 per target for
//    1x1 bodies); a sweep re-walks each target's hits under the current death positions.  A
//    death at position q depends only on deaths at positions < q, so the fixed point is unique
//    and is the sequential result; a sweep that changes nothing ends the loop.
//  * moves: ownership rounds as in move_parallel, up to kBigMovPer movers per lane, claims on a
//    large hashed LDS table.
constexpr int kBigMovPer = 8;
constexpr int kBigOwnerSlots = 16384;
constexpr uint16_t kBigNone = 0xFFFF;       // no death / blank target
constexpr uint16_t kBigSkip = 0xFFFE;       // attacker already dead at the start of the step

struct BigScratch {
    uint32_t* ord;     // [A] attack entries in shuffled order
    uint16_t* jv;      // [A] Fisher-Yates j_k
    uint32_t* hd;      // [max(A, C) + 1] CSR bucket ends (shuffle buckets, then targets)
    uint16_t* lst;     // [A] CSR contents
    uint16_t* att;     // [A] attacker id by position
    uint16_t* tgt;     // [A] target id at phase start, kBigNone (blank), kBigSkip
    uint8_t* pg;       // [A] attacker group by position
    uint16_t* death;   // [C] position of the killing hit, or kBigNone
    uint32_t* owner;   // [kBigOwnerSlots] move claims (aliases the attack arrays)
    int* flag;         // [2]
    int acap;
    int srow;          // diagnostic stamp row (MFX_STAMPS build), -1 none
    int sbase;         //   and the first stamp slot of attack_big's internal stamps (minus 3)
    char* base;        // the whole scratch region (the moves reuse it), bytes long
    size_t bytes;
};

// Moves by pointer jumping (move_jump) reuse the region: a hashed bucket table of jump_slots(n)
// heads plus five per-mover arrays and an id -> mover map.
__host__ __device__ inline int jump_slots(int n) {
    int s = 64;
    while (s < 2 * n && s < 4096) s <<= 1;
    return s;
}
__host__ __device__ inline size_t move_jump_bytes(int n, int nid) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return r16((size_t)jump_slots(n) * 4) + r16((size_t)n * 4) + 4 * r16((size_t)n * 2) + r16((size_t)nid * 2);
}

// full: the HBM-state path (ownership-round claims and the band sort's counts share the region too);
// compact: the attack arrays and move_jump only (k_rollout's LDS union).
__host__ __device__ inline size_t big_attack_bytes(int acap, int cap) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t m = (size_t)(acap > cap ? acap : cap) + 1;
    return r16((size_t)acap * 4) + r16((size_t)acap * 2) + r16(m * 4) + 3 * r16((size_t)acap * 2) +
           r16((size_t)acap) + r16((size_t)cap * 2);
}
__host__ __device__ inline size_t big_region_bytes(int acap, int cap, bool full) {
    size_t r = big_attack_bytes(acap, cap);
    const size_t j = move_jump_bytes(acap, cap);
    if (j > r) r = j;
    if (full) {
        // k_rollout_big's staged xy + meta + group lists
        if ((size_t)cap * (5 + 2 * kMaxGroups) > r) r = (size_t)cap * (5 + 2 * kMaxGroups);
        if ((size_t)kBigOwnerSlots * 4 > r) r = (size_t)kBigOwnerSlots * 4;
        if ((size_t)17 * 1024 * 4 > r) r = (size_t)17 * 1024 * 4;     // band_sort_big: 16 bands x 1024 lanes
    }
    return (r + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t big_scratch_bytes(int acap, int cap, bool full = true) {
    return big_region_bytes(acap, cap, full) + 16;
}

// k_step's LDS-mode step scratch: the wave-team forms (ParScratch) or the workgroup forms
// (BigScratch, compact), at the same base
__host__ __device__ inline size_t step_par_bytes(int acap, int cap) {
    const size_t a = par_scratch_bytes(acap, cap), b = big_scratch_bytes(acap, cap, false);
    return a > b ? a : b;
}

__device__ __forceinline__ BigScratch carve_big(char* base, int acap, int cap, bool full = true) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t m = (size_t)(acap > cap ? acap : cap) + 1;
    BigScratch b;
    size_t o = 0;
    b.ord = reinterpret_cast<uint32_t*>(base + o);  o += r16((size_t)acap * 4);
    b.jv = reinterpret_cast<uint16_t*>(base + o);   o += r16((size_t)acap * 2);
    b.hd = reinterpret_cast<uint32_t*>(base + o);   o += r16(m * 4);
    b.lst = reinterpret_cast<uint16_t*>(base + o);  o += r16((size_t)acap * 2);
    b.att = reinterpret_cast<uint16_t*>(base + o);  o += r16((size_t)acap * 2);
    b.tgt = reinterpret_cast<uint16_t*>(base + o);  o += r16((size_t)acap * 2);
    b.pg = reinterpret_cast<uint8_t*>(base + o);    o += r16((size_t)acap);
    b.death = reinterpret_cast<uint16_t*>(base + o); o += r16((size_t)cap * 2);
    b.owner = reinterpret_cast<uint32_t*>(base);
    b.bytes = big_region_bytes(acap, cap, full);
    b.flag = reinterpret_cast<int*>(base + b.bytes);
    b.acap = acap;
    b.srow = -1;
    b.sbase = 0;
    b.base = base;
    return b;
}

// In-place exclusive scan of a[0..m) over the workgroup (each lane scans a contiguous chunk).
__device__ __forceinline__ void block_excl_scan(uint32_t* a, int m, int* wave_tot) {
    const int t = TID, T = blockDim.x, lane = t & 63, wid = t >> 6, nw = T >> 6;
    const int per = (m + T - 1) / T, b0 = min(m, t * per), b1 = min(m, b0 + per);
    uint32_t sum = 0;
    for (int i = b0; i < b1; ++i) sum += a[i];
    uint32_t inc = sum;                                   // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wave_tot[wid] = (int)inc;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wid; ++w) off += (uint32_t)wave_tot[w];
    (void)nw;
    off += inc - sum;
    for (int i = b0; i < b1; ++i) { const uint32_t c = a[i]; a[i] = off; off += c; }
    __syncthreads();
}

// CSR buckets of keys key(i) in [0, K) for i in [0, n) (key < 0: not bucketed).  Afterwards
// bucket v is lst[(v ? hd[v-1] : 0) .. hd[v]), ascending in i.
template <class KeyF>
__device__ __forceinline__ void big_buckets(const BigScratch& b, int n, int K, KeyF key, int* wave_tot) {
    const int t = TID, T = blockDim.x;
    for (int v = t; v <= K; v += T) b.hd[v] = 0;
    __syncthreads();
    for (int i = t; i < n; i += T) { const int k = key(i); if (k >= 0) atomicAdd(&b.hd[k], 1u); }
    __syncthreads();
    block_excl_scan(b.hd, K, wave_tot);
    for (int i = t; i < n; i += T) {
        const int k = key(i);
        if (k >= 0) b.lst[atomicAdd(&b.hd[k], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    for (int v = t; v < K; v += T) {                      // insertion sort (buckets are short)
        const int s0 = v ? (int)b.hd[v - 1] : 0, s1 = (int)b.hd[v];
        for (int i = s0 + 1; i < s1; ++i) {
            const uint16_t x = b.lst[i];
            int j = i - 1;
            while (j >= s0 && b.lst[j] > x) { b.lst[j + 1] = b.lst[j]; --j; }
            b.lst[j + 1] = x;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ int big_start(const BigScratch& b, int v) { return v ? (int)b.hd[v - 1] : 0; }

// Shuffle + attack resolution for any n (<= acap), whole workgroup.
__device__ void attack_big(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* atk, int n,
                           uint32_t& rng, const BigScratch& b, int nid, int* wave_tot) {
    const int t0 = TID, T = blockDim.x, W = gp.W, H = gp.H;
    // ---- Fisher-Yates draws (minstd jump-ahead per step)
    for (int k = t0; k < n; k += T) {
        const uint32_t x = minstd_jump(rng, (uint32_t)k + 1u);
        b.jv[k] = (uint16_t)(x % (uint32_t)(k + 1));
        if (k == n - 1) b.flag[1] = (int)x;
    }
    __syncthreads();
    if (n > 0) rng = (uint32_t)b.flag[1];
    MFX_BSTAMP(b.srow, b.sbase + 3);
    big_buckets(b, n, n, [&](int k) { const int j = b.jv[k]; return j < k ? j : -1; }, wave_tot);
    MFX_BSTAMP(b.srow, b.sbase + 4);
    for (int t = t0; t < n; t += T) {
        int p = b.jv[t];
        bool hop = false;
        {   // first later swap that hits position p: the successor of t in L(p)
            const int s1 = (int)b.hd[p];
            for (int i = big_start(b, p); i < s1; ++i) {
                const int k = b.lst[i];
                if (k > t) { p = k; hop = true; break; }
            }
        }
        while (hop) {       // at position p since step p: the next hit is min L(p) (all > p)
            const int s0 = big_start(b, p);
            hop = s0 < (int)b.hd[p];
            if (hop) p = b.lst[s0];
        }
        b.ord[p] = atk[t];
    }
    __syncthreads();
    // ---- per position: attacker, group, target at phase start
    for (int t = t0; t < n; t += T) {
        const uint32_t e2 = b.ord[t];
        const int A = (int)(e2 >> 8), ai = (int)(e2 & 0xFF);
        const uint32_t m = v.meta[A];
        uint16_t tg = kBigSkip;
        const int g = meta_group(m);
        if (!meta_dead(m)) {
            const SerialType& S = sm.tt[g];
            const uint32_t pos = v.xy[A];
            const int ox = (int)(pos & 0xFFFF) + S.att_x_off + S.att_dx[ai];
            const int oy = (int)(pos >> 16) + S.att_y_off + S.att_dy[ai];
            uint32_t cv = kCellEmpty;
            if (ox >= 0 && ox < W && oy >= 0 && oy < H) cv = v.cells[oy * W + ox];
            tg = kBigNone;
            if (cv < kCellFood && (S.attack_in_group || (int)meta_group(v.meta[cv]) != g)) tg = (uint16_t)cv;
        }
        b.att[t] = (uint16_t)A;
        b.tgt[t] = tg;
        b.pg[t] = (uint8_t)g;
    }
    for (int id = t0; id < nid; id += T) b.death[id] = kBigNone;
    __syncthreads();
    MFX_BSTAMP(b.srow, b.sbase + 5);
    // ---- hits per target, in shuffle order
    big_buckets(b, n, nid, [&](int q) { const int x = b.tgt[q]; return x < (int)kBigSkip ? x : -1; }, wave_tot);
    // ---- fixed point on the death positions (in place; a quiet sweep is the fixed point)
    for (int it = 0; it <= n + 1; ++it) {
        if (t0 == 0) b.flag[0] = 0;
        __syncthreads();
        for (int X = t0; X < nid; X += T) {
            const int s0 = big_start(b, X), s1 = (int)b.hd[X];
            if (s0 == s1) continue;
            float h = v.hp[X];
            int d = kBigNone;
            for (int i = s0; i < s1; ++i) {
                const int q = b.lst[i];
                if ((int)b.death[b.att[q]] <= q) continue;        // attacker dead at its turn
                h = h - sm.tt[b.pg[q]].damage;                    // Agent::be_attack
                if (h < 0.0f) { d = q; break; }
            }
            if (d != (int)b.death[X]) { b.death[X] = (uint16_t)d; b.flag[0] = 1; }
        }
        __syncthreads();
        if (!b.flag[0]) break;
        __syncthreads();
    }
    MFX_BSTAMP(b.srow, b.sbase + 6);
    // ---- apply: attackers (one attack per agent per step) ...
    for (int t = t0; t < n; t += T) {
        const int A = b.att[t], tg = b.tgt[t];
        if (tg == kBigSkip || (int)b.death[A] <= t) continue;
        const int g = b.pg[t];
        const SerialType& S = sm.tt[g];
        if (tg == kBigNone || (int)b.death[tg] < t) {
            v.next_r[A] += S.attack_penalty;                      // blank area (or a dead target)
        } else {
            const bool kill = (int)b.death[tg] == t;
            v.meta[A] = (uint8_t)meta_make(0, kill ? kOpKill : kOpAttack, g);
            v.op_obj[A] = tg;
            const float reward = kill ? sm.tt[meta_group(v.meta[tg])].kill_reward : 0.0f;
            v.next_r[A] += reward + S.attack_penalty;
        }
    }
    // ... and every target's hp after its effective hits
    for (int X = t0; X < nid; X += T) {
        const int s0 = big_start(b, X), s1 = (int)b.hd[X];
        if (s0 == s1) continue;
        float h = v.hp[X];
        for (int i = s0; i < s1; ++i) {
            const int q = b.lst[i];
            if ((int)b.death[b.att[q]] <= q) continue;
            h = h - sm.tt[b.pg[q]].damage;
            if (h < 0.0f) break;
        }
        v.hp[X] = h;
    }
    __syncthreads();
    // ---- deaths
    for (int id = t0; id < nid; id += T) {
        if (b.death[id] == kBigNone) continue;
        const uint32_t om = v.meta[id];
        const int og = meta_group(om);
        v.meta[id] = (uint8_t)meta_make(1, meta_op(om), og);
        v.next_r[id] = sm.tt[og].dead_penalty;
        const uint32_t pos = v.xy[id];
        v.cells[(pos >> 16) * W + (pos & 0xFFFF)] = kCellEmpty;     // remove_agent
        atomicAdd(&v.grp_dead[og], 1);
    }
    __syncthreads();
}

// Move resolution for n <= kBigMovPer * lanes movers in `order`, whole workgroup.
__device__ void move_big(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* order, int n,
                         const BigScratch& b) {
    const int t0 = TID, T = blockDim.x, W = gp.W, H = gp.H;
    int id[kBigMovPer], src[kBigMovPer], dst[kBigMovPer];
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < kBigMovPer; ++j) {
        const int i = t0 + j * T;
        id[j] = -1; src[j] = 0; dst[j] = 0;
        if (i < n) {
            const uint32_t ent = order[i];
            const int a = (int)(ent >> 16), mi = (int)((ent >> 8) & 0xFF);
            const uint32_t m = v.meta[a];
            id[j] = a;
            if (!meta_dead(m)) {
                const SerialType& S = sm.tt[meta_group(m)];
                const uint32_t p = v.xy[a];
                const int x = p & 0xFFFF, y = p >> 16;
                const int nx = x + S.move_dx[mi], ny = y + S.move_dy[mi];
                const bool go = !(nx < 0 || ny < 0 || nx + 1 >= W || ny + 1 >= H) && !(nx == x && ny == y);
                src[j] = y * W + x; dst[j] = ny * W + nx;
                if (go) pend |= 1u << j;
            }
        }
    }
    for (int round = 0; round <= n; ++round) {
        for (int k = t0; k < kBigOwnerSlots; k += T) b.owner[k] = 0xFFFFFFFFu;
        if (t0 == 0) b.flag[0] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kBigMovPer; ++j) {
            if (!(pend >> j & 1u)) continue;
            const uint32_t i = (uint32_t)(t0 + j * T);
            atomicMin(&b.owner[(uint32_t)src[j] % kBigOwnerSlots], i);
            atomicMin(&b.owner[(uint32_t)dst[j] % kBigOwnerSlots], i);
        }
        __syncthreads();
        bool more = false;
#pragma unroll
        for (int j = 0; j < kBigMovPer; ++j) {
            if (!(pend >> j & 1u)) continue;
            const uint32_t i = (uint32_t)(t0 + j * T);
            if (b.owner[(uint32_t)src[j] % kBigOwnerSlots] == i && b.owner[(uint32_t)dst[j] % kBigOwnerSlots] == i) {
                const uint32_t cv = v.cells[dst[j]];
                if (cv == kCellEmpty) {
                    v.cells[src[j]] = kCellEmpty;
                    v.cells[dst[j]] = (uint16_t)id[j];
                    v.xy[id[j]] = (uint32_t)(dst[j] % W) | ((uint32_t)(dst[j] / W) << 16);
                } else if (cv < kCellFood) {
                    v.meta[id[j]] = (uint8_t)meta_make(0, kOpCollide, meta_group(v.meta[id[j]]));
                    v.op_obj[id[j]] = (int)cv;
                }
                pend &= ~(1u << j);
            } else {
                more = true;
            }
        }
        if (more) b.flag[0] = 1;
        __syncthreads();
        if (!b.flag[0]) break;
        __syncthreads();
    }
}

// ==================================================================================
//  reward DSL (GridWorld::calc_reward + calc_rule + calc_event_node, RewardEngine.cc:216-443)
// ==================================================================================
// One lane walks the reference's DFS over agent bindings exactly: same level order
// (RewardRule::input_symbols), same agent order, the same `involved` marks (meta bit 3) and the
// same reward accumulation order.  Symbol bindings are agent ids (-1 = none).
constexpr uint8_t kMetaInvolved = 8;

__device__ __forceinline__ int dsl_agent_index(const EnvView& v, int mark, int id) {
    // Agent::index: 0 from the constructor (GridWorld.h:139) until a clear_dead sets the list
    // position (GridWorld.cc:718); positions do not move between two clear_dead calls.
    if (id >= mark) return 0;
    const int g = meta_group(v.meta[id]);
    const uint16_t* ids = v.grp_ids + g * v.cap;
    for (int i = 0; i < v.grp_n[g]; ++i)
        if (ids[i] == id) return i;
    return 0;
}

__device__ __forceinline__ bool dsl_bind(const DslSym& S, const EnvView& v, int mark, int ob) {
    // AgentSymbol::bind_with_check (RewardEngine.cc:14-23)
    if ((int)meta_group(v.meta[ob]) != S.group) return false;
    return S.index == -1 || S.index == dsl_agent_index(v, mark, ob);
}

__device__ __forceinline__ bool dsl_leaf(const GameParams& gp, const DslNode& N, const EnvView& v, const int* ent) {
    const DslProgram& P = gp.prog;
    const DslSym& S = P.sym[N.a];
    const bool all = S.index == -2;
    const uint16_t* ids = v.grp_ids + S.group * v.cap;
    const int n = all ? v.grp_n[S.group] : 1;
    const int sub = ent[N.a];
    switch (N.op) {
        case kEvAttack: case kEvKill: case kEvCollide: {
            const uint32_t want = N.op == kEvAttack ? kOpAttack : (N.op == kEvKill ? kOpKill : kOpCollide);
            const int obj = ent[N.b];
            for (int i = 0; i < n; ++i) {
                const int id = all ? ids[i] : sub;
                if (id < 0) return false;
                if (!(meta_op(v.meta[id]) == want && v.op_obj[id] == obj)) return false;
            }
            return true;
        }
        case kEvAt: case kEvIn: {
            for (int i = 0; i < n; ++i) {
                const int id = all ? ids[i] : sub;
                if (id < 0) return false;
                const int x = (int)(v.xy[id] & 0xFFFF), y = (int)(v.xy[id] >> 16);
                const bool in = N.op == kEvAt ? (x == N.i0 && y == N.i1)
                                              : (x > N.i0 && x < N.i2 && y > N.i1 && y < N.i3);
                if (!in) return false;
            }
            return true;
        }
        case kEvDie: {
            for (int i = 0; i < n; ++i) {
                const int id = all ? ids[i] : sub;
                if (id < 0) return false;
                if (!meta_dead(v.meta[id])) return false;
            }
            return true;
        }
        case kEvInALine: {                         // subject is 'all' (checked on the host)
            const int m = v.grp_n[S.group];
            if (m < 2) return true;
            const int x0 = (int)(v.xy[ids[0]] & 0xFFFF), y0 = (int)(v.xy[ids[0]] >> 16);
            const int dx = x0 - (int)(v.xy[ids[1]] & 0xFFFF), dy = y0 - (int)(v.xy[ids[1]] >> 16);
            if ((dx == 0) == (dy == 0)) return false;
            const bool vert = dx == 0;
            int lo = vert ? y0 : x0, hi = lo;
            bool line = true;
            for (int i = 1; i < m && line; ++i) {
                const int x = (int)(v.xy[ids[i]] & 0xFFFF), y = (int)(v.xy[ids[i]] >> 16);
                const int c = vert ? y : x;
                lo = c < lo ? c : lo; hi = c > hi ? c : hi;
                line = vert ? x == x0 : y == y0;
            }
            return line && hi - lo + 1 == m;
        }
        default:
            return false;
    }
}

__device__ __forceinline__ bool dsl_eval(const GameParams& gp, const DslRule& R, const EnvView& v, const int* ent) {
    const DslProgram& P = gp.prog;
    uint32_t bits = 0;                          // AND / OR / NOT have no side effects: no short cut needed
    for (int k = 0; k < R.n_post; ++k) {
        const int ni = R.post[k];
        const DslNode& N = P.node[ni];
        bool r;
        if (N.op == kEvAnd) r = ((bits >> N.a) & 1u) && ((bits >> N.b) & 1u);
        else if (N.op == kEvOr) r = ((bits >> N.a) & 1u) || ((bits >> N.b) & 1u);
        else if (N.op == kEvNot) r = !((bits >> N.a) & 1u);
        else r = dsl_leaf(gp, N, v, ent);
        bits |= (uint32_t)r << ni;
    }
    return (bits >> R.post[R.n_post - 1]) & 1u;
}

__device__ void dsl_rewards(const GameParams& gp, EnvView& v, int mark, int* flags) {
    const DslProgram& P = gp.prog;
    for (int r = 0; r < P.n_rules; ++r) {
        const DslRule& R = P.rule[r];
        int ent[kMaxSyms], it[kMaxSyms + 1], cur[kMaxSyms + 1];
        for (int k = 0; k < kMaxSyms; ++k) ent[k] = -1;
        int trig = 0, now = 0;
        it[0] = 0; cur[0] = -1;
        while (now >= 0) {
            if (now == R.n_in) {                   // DFS last layer (RewardEngine.cc:376-390)
                if (dsl_eval(gp, R, v, ent)) {
                    trig = 1;
                    for (int k = 0; k < R.n_recv; ++k) {
                        const DslSym& S = P.sym[R.recv[k]];
                        if (S.index == -2) v.grp_reward[S.group] += R.val[k];
                        else v.next_r[ent[R.recv[k]]] += R.val[k];
                    }
                }
                --now;
                continue;
            }
            const int si = R.in_sym[now], inf = R.infer[now];
            const DslSym& S = P.sym[si];
            const uint16_t* ids = v.grp_ids + S.group * v.cap;
            const int n = v.grp_n[S.group];
            bool down = false;
            if (S.index == -1) {                   // 'any': every agent not bound at a shallower level
                if (cur[now] >= 0) { v.meta[cur[now]] &= (uint8_t)~kMetaInvolved; cur[now] = -1; }
                while (!down && it[now] < n) {
                    const int id = ids[it[now]++];
                    ent[si] = id;
                    if (v.meta[id] & kMetaInvolved) continue;
                    v.meta[id] |= kMetaInvolved;
                    cur[now] = id;
                    if (inf < 0) { down = true; break; }
                    const int ob = v.op_obj[id];
                    if (ob >= 0 && dsl_bind(P.sym[inf], v, mark, ob)) { ent[inf] = ob; down = true; }
                    else { v.meta[id] &= (uint8_t)~kMetaInvolved; cur[now] = -1; }
                }
            } else if (it[now] == 0) {             // 'all' / a fixed index: a single pass
                it[now] = 1;
                if (S.index == -2) {
                    if (inf < 0) down = true;
                    else if (n > 0) {
                        const int ob = v.op_obj[ids[0]];
                        if (ob >= 0 && dsl_bind(P.sym[inf], v, mark, ob)) { ent[inf] = ob; down = true; }
                    }
                } else if (S.index < n) {          // without an inference the reference stops here
                    const int id = ids[S.index];
                    ent[si] = id;
                    const int ob = inf >= 0 ? v.op_obj[id] : -1;
                    if (ob >= 0 && dsl_bind(P.sym[inf], v, mark, ob)) { ent[inf] = ob; down = true; }
                }
            }
            if (down) { ++now; it[now] = 0; cur[now] = -1; }
            else --now;
        }
        flags[r] = trig;
    }
}

// Everything of GridWorld::step for one env, executed by the whole workgroup.
// atk/mov/sorted: pending buffers (any address space); sorted has room for n_mov entries.
// sm.tt must hold the serial type table (load_serial_types + barrier).
// ps: LDS scratch for the parallel resolution (nullptr: one-lane loops only); nid = id_counter.
// kDsl: reward rules through the DSL interpreter (gp.dsl), dsl_mark = State::idx_mark of the env.
// Move resolution without rounds (large envs).  A cell's history in the move phase is short: its
// occupant at the phase start may leave (at its own move, if that succeeds) and afterwards the FIRST
// later mover into it takes it for good (nobody moves twice).  So mover m (order index) succeeds iff
//   * its target was empty at the phase start and no earlier mover targets it, or
//   * its target's occupant moves at an earlier index m_o, that move succeeds, and no mover between
//     m_o and m targets the cell;
// i.e. success(m) = cond(m) AND success(m_o): a forest of AND-chains along "whose cell do I take",
// evaluated by pointer jumping in O(log chain) rounds instead of one round per link (a 32-column
// formation advancing into its own rear is a 32-link chain).  Movers are bucketed by target in a
// hashed LDS list; the latest earlier mover into the same cell (pred) decides cond(m).  A failing
// mover collides with the cell's occupant at its time: the phase-start occupant, or the first later
// mover into it (the filler).  Up to 4096 movers (12-bit links).
constexpr uint16_t kJumpNone = 0x7FFF;
__device__ __forceinline__ uint32_t jump_hash(uint32_t d, int bits) { return (d * 2654435761u) >> (32 - bits); }

template <bool kWave>
__device__ bool move_jump(const GameParams& gp, const StepSmem& sm, EnvView& v, const uint32_t* order, int n,
                          const BigScratch& b, int nid) {
    if (n > 4096 || move_jump_bytes(n, nid) > b.bytes) return false;
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const int T = team_lanes<kWave>(), t0 = TID, W = gp.W, H = gp.H;
    const int slots = jump_slots(n), hb = __ffs(slots) - 1;
    char* p = b.base;
    uint32_t* head = reinterpret_cast<uint32_t*>(p); p += r16((size_t)slots * 4);
    uint32_t* dstv = reinterpret_cast<uint32_t*>(p); p += r16((size_t)n * 4);     // target cell, ~0u if no move
    uint16_t* nxt = reinterpret_cast<uint16_t*>(p); p += r16((size_t)n * 2);      // hashed bucket links
    uint16_t* st0 = reinterpret_cast<uint16_t*>(p); p += r16((size_t)n * 2);      // cond << 15 | link
    uint16_t* st1 = reinterpret_cast<uint16_t*>(p); p += r16((size_t)n * 2);
    uint16_t* occ = reinterpret_cast<uint16_t*>(p); p += r16((size_t)n * 2);      // target's phase-start content
    uint16_t* mv_of = reinterpret_cast<uint16_t*>(p);                             // [nid] mover index of an id
    for (int k = t0; k < slots; k += T) head[k] = 0xFFFFFFFFu;
    for (int id = t0; id < nid; id += T) mv_of[id] = kJumpNone;
    psync<kWave>();
    // ---- movers: target cells, bucket lists, id -> mover
    for (int m = t0; m < n; m += T) {
        const uint32_t ent = order[m];
        const int id = (int)(ent >> 16), mi = (int)((ent >> 8) & 0xFF);
        const uint32_t meta = v.meta[id];
        uint32_t d = 0xFFFFFFFFu;
        if (!meta_dead(meta)) {
            const SerialType& S = sm.tt[meta_group(meta)];
            const uint32_t q = v.xy[id];
            const int x = q & 0xFFFF, y = q >> 16, nx = x + S.move_dx[mi], ny = y + S.move_dy[mi];
            // out of board: no-op; a move onto itself changes nothing (not a mover here)
            if (!(nx < 0 || ny < 0 || nx + 1 >= W || ny + 1 >= H) && !(nx == x && ny == y)) d = (uint32_t)(ny * W + nx);
        }
        dstv[m] = d;
        if (d != 0xFFFFFFFFu) {
            mv_of[id] = (uint16_t)m;
            nxt[m] = (uint16_t)atomicExch(&head[jump_hash(d, hb)], (uint32_t)m);
        }
    }
    psync<kWave>();
    // ---- cond(m) and link m_o from the phase-start cells
    for (int m = t0; m < n; m += T) {
        const uint32_t d = dstv[m];
        uint16_t st = kJumpNone;                           // cond 0, no link: fails
        uint16_t cv = kCellEmpty;
        if (d != 0xFFFFFFFFu) {
            cv = v.cells[d];
            int pred = -1;                                 // latest earlier mover into d
            for (uint32_t k = head[jump_hash(d, hb)]; k != 0xFFFFFFFFu && k != 0xFFFFu; k = nxt[k])
                if (dstv[k] == d && (int)k < m && (int)k > pred) pred = (int)k;
            if (cv == kCellEmpty) {
                st = (uint16_t)((pred < 0 ? 0x8000u : 0u) | kJumpNone);
            } else if (cv < kCellFood) {
                const int mo = mv_of[cv];
                if (mo != kJumpNone && mo < m) st = (uint16_t)((pred < mo ? 0x8000u : 0u) | (uint32_t)mo);
                else st = kJumpNone;
            } else {
                st = kJumpNone;                            // wall
            }
        }
        st0[m] = st;
        occ[m] = cv;
    }
    psync<kWave>();
    // ---- pointer jumping: cond(m) &= cond(link(m)), link(m) = link(link(m))
    uint16_t* a = st0;
    uint16_t* c = st1;
    for (int r = 0; r < 16; ++r) {
        if (t0 == 0) b.flag[0] = 0;
        psync<kWave>();
        bool more = false;
        for (int m = t0; m < n; m += T) {
            const uint16_t x = a[m];
            const int l = x & 0x7FFF;
            uint16_t y = x;
            if (l != kJumpNone) {
                const uint16_t z = a[l];
                y = (uint16_t)((x & z & 0x8000u) | (z & 0x7FFFu));
                more |= (z & 0x7FFFu) != kJumpNone;
            }
            c[m] = y;
        }
        if (more) b.flag[0] = 1;
        psync<kWave>();
        uint16_t* tmp = a; a = c; c = tmp;
        if (!b.flag[0]) break;
        psync<kWave>();                               // every lane has read the flag before it is reset
    }
    // a[m] >> 15: m succeeds.  ---- collisions (before any cell changes)
    for (int m = t0; m < n; m += T) {
        const uint32_t d = dstv[m];
        if (d == 0xFFFFFFFFu || (a[m] >> 15)) continue;
        const uint16_t cv = occ[m];
        int who = -1;                                      // occupant at time m
        if (cv < kCellFood) {
            const int mo = mv_of[cv];
            if (mo == kJumpNone || mo > m || !(a[mo] >> 15)) who = cv;
            else {
                int f = 0x7FFFFFFF;                        // the filler: first mover into d after m_o
                for (uint32_t k = head[jump_hash(d, hb)]; k != 0xFFFFFFFFu && k != 0xFFFFu; k = nxt[k])
                    if (dstv[k] == d && (int)k > mo && (int)k < f) f = (int)k;
                if (f < m) who = (int)(order[f] >> 16);
            }
        } else if (cv == kCellEmpty) {
            int f = 0x7FFFFFFF;                            // the first mover into d took it
            for (uint32_t k = head[jump_hash(d, hb)]; k != 0xFFFFFFFFu && k != 0xFFFFu; k = nxt[k])
                if (dstv[k] == d && (int)k < f) f = (int)k;
            if (f < m) who = (int)(order[f] >> 16);
        }
        if (who >= 0) {
            const int id = (int)(order[m] >> 16);
            v.meta[id] = (uint8_t)meta_make(0, kOpCollide, meta_group(v.meta[id]));
            v.op_obj[id] = who;
        }
    }
    // ---- apply: vacate, then fill (a vacated cell may be filled by a later mover)
    for (int m = t0; m < n; m += T) {
        if (dstv[m] == 0xFFFFFFFFu || !(a[m] >> 15)) continue;
        const uint32_t q = v.xy[order[m] >> 16];
        v.cells[(q >> 16) * W + (q & 0xFFFF)] = kCellEmpty;
    }
    psync<kWave>();
    for (int m = t0; m < n; m += T) {
        const uint32_t d = dstv[m];
        if (d == 0xFFFFFFFFu || !(a[m] >> 15)) continue;
        const int id = (int)(order[m] >> 16);
        v.cells[d] = (uint16_t)id;
        v.xy[id] = (d % (uint32_t)W) | ((d / (uint32_t)W) << 16);
    }
    psync<kWave>();
    return true;
}

// Large-map move order (GridWorld.cc:662-672: band buffers 0..n_sep-1, then the boundary buffer),
// as ONE stable counting sort over the workgroup: every lane counts the buckets of its contiguous
// segment of the buffer, one exclusive scan of the bucket-major [bucket][lane] counts gives every
// (bucket, lane) its output offset, and each lane re-walks its segment.  The counts live in the step
// scratch (dead between the attacks and the moves).
constexpr int kMaxBands = 16;
__device__ __forceinline__ void band_sort_big(const GameParams& gp, const uint32_t* mov, int n, uint32_t* sorted,
                                              const BigScratch& b, int* wave_tot) {
    const int T = blockDim.x, t = TID, nb = gp.n_sep + 1;
    const int per = (n + T - 1) / T, i0 = min(n, t * per), i1 = min(n, i0 + per);
    uint32_t* cnt = b.ord;                          // [nb][T]
    int c[kMaxBands + 1];
#pragma unroll
    for (int k = 0; k <= kMaxBands; ++k) c[k] = 0;
    for (int i = i0; i < i1; ++i) {
        const uint32_t w = mov[i] & 0xFF;
        const int k = w == kBucketBoundary ? nb - 1 : (int)w;
#pragma unroll
        for (int q = 0; q <= kMaxBands; ++q) c[q] += (q == k);
    }
#pragma unroll
    for (int k = 0; k <= kMaxBands; ++k) if (k < nb) cnt[k * T + t] = (uint32_t)c[k];
    __syncthreads();
    block_excl_scan(cnt, nb * T, wave_tot);
#pragma unroll
    for (int k = 0; k <= kMaxBands; ++k) c[k] = k < nb ? (int)cnt[k * T + t] : 0;
    for (int i = i0; i < i1; ++i) {
        const uint32_t ent = mov[i], w = ent & 0xFF;
        const int k = w == kBucketBoundary ? nb - 1 : (int)w;
        int o = 0;
#pragma unroll
        for (int q = 0; q <= kMaxBands; ++q) if (q == k) o = c[q]++;
        sorted[o] = ent;
    }
    __syncthreads();
}

template <bool kW, bool kDsl = false, bool kBig = false>
__device__ void step_env_core(const GameParams& gp, const State& s, EnvView& v, uint32_t* atk, int n_atk,
                              uint32_t* mov, int n_mov, uint32_t* sorted, uint32_t& rng, StepSmem& sm,
                              int& done_out, const bool have_ps, const ParScratch ps, int nid,
                              int32_t* ev = nullptr, int dsl_mark = 0, const BigScratch* bs = nullptr,
                              int stamp_row = -1) {
    (void)stamp_row;
    const int G = gp.n_groups;
#ifndef MFX_PAR_MASK
#define MFX_PAR_MASK 3
#endif
    const bool par0 = kBig ? (!ev && gp.par_step && n_atk <= bs->acap && n_mov <= kBigMovPer * (int)blockDim.x)
                           : (!ev && have_ps && gp.par_step && n_atk <= (int)blockDim.x && n_mov <= (int)blockDim.x);
    bool par = par0 && (MFX_PAR_MASK & 1);
    psync<kW>();
    // ---- shuffle + attack (GridWorld.cc:507-558)
#ifndef MFX_WAVE_STEP_MAX
#define MFX_WAVE_STEP_MAX 64
#endif
    MFX_RSTAMP(kW, stamp_row, 17);                 // diagnostic: the attacks start here
    if (kBig && par) {
        attack_big(gp, sm, v, atk, n_atk, rng, *bs, nid, sm.wave_tot);
        MFX_BSTAMP(bs->srow, 7);
    } else if (kW && par) {
        attack_parallel<true>(gp, sm, v, atk, n_atk, rng, ps, nid);
    } else if (par && n_atk <= MFX_WAVE_STEP_MAX) {
        if (TID < 64) attack_parallel<true>(gp, sm, v, atk, n_atk, rng, ps, nid);
        __syncthreads();
    } else if (par && bs) {                        // whole-workgroup team: O(n log n) form
        attack_big(gp, sm, v, atk, n_atk, rng, *bs, nid, sm.wave_tot);
    } else if (par) {
        attack_parallel<false>(gp, sm, v, atk, n_atk, rng, ps, nid);
    } else if (TID == 0) {
        uint32_t x = rng;
        for (int i = 0; i < n_atk; ++i) {
            x = minstd_next(x);
            const int j = (int)(x % (uint32_t)(i + 1));
            const uint32_t t = atk[i]; atk[i] = atk[j]; atk[j] = t;
        }
        rng = x;
        if (ev) ev[0] = 0;
        do_attack_serial(gp, sm, v, atk, n_atk, ev);
    }
    psync<kW>();
    MFX_RSTAMP(kW, stamp_row, 18);                 // attacks done
    // ---- starve (GridWorld.cc:570-595): independent per agent
    for (int g = 0; g < G; ++g) {
        const TypeParams& T = gp.type[g];
        const int n = v.grp_n[g];
        for (int i = TID; i < n; i += team_lanes<kW>()) {
            const int id = v.grp_ids[g * v.cap + i];
            const uint32_t m = v.meta[id];
            if (meta_dead(m)) continue;
            if (T.step_recover > 0.0f) {
                const float h2 = v.hp[id] + T.step_recover;
                v.hp[id] = T.hp < h2 ? T.hp : h2;
            } else {
                const float h2 = v.hp[id] - (-T.step_recover);
                v.hp[id] = h2;
                if (h2 < 0.0f) {
                    v.meta[id] = (uint8_t)(m | 1u);
                    v.next_r[id] = T.dead_penalty;
                    const uint32_t p = v.xy[id];
                    int bw, bh;
                    size_for_dir(meta_dir(m), T.body_w, T.body_h, bw, bh);
                    fill_area(v.cells, gp.W, (int)(p & 0xFFFF), (int)(p >> 16), bw, bh, kCellEmpty);
                    atomicAdd(&v.grp_dead[g], 1);
                }
            }
        }
    }
    psync<kW>();
    // ---- move order: large map = band buffers 0..n_sep-1 then boundary (GridWorld.cc:662-672)
    const uint32_t* order = mov;
    if (kBig && gp.large_map) {
        band_sort_big(gp, mov, n_mov, sorted, *bs, sm.wave_tot);
        order = sorted;
    } else if (gp.large_map) {
        int base = 0;
        for (int b = 0; b <= gp.n_sep; ++b) {
            const uint32_t want = b < gp.n_sep ? (uint32_t)b : kBucketBoundary;
            for (int i0 = 0; i0 < n_mov; i0 += team_lanes<kW>()) {
                const int i = i0 + TID;
                const uint32_t ent = i < n_mov ? mov[i] : 0u;
                const int f = i < n_mov && (ent & 0xFF) == want;
                int tot;
                const int r = team_scan<kW>(f, sm.wave_tot, tot);
                if (f) sorted[base + r] = ent;
                base += tot;
            }
        }
        psync<kW>();
        order = sorted;
    }
    MFX_RSTAMP(kW, stamp_row, 15);                 // diagnostic: the moves start here
    if (gp.turn_mode) {                            // turns first, same bucket order (GridWorld.cc:597-624)
        if (TID == 0)
            for (int i = 0; i < n_mov; ++i) do_turn_one(gp, sm, v, order[i]);
        psync<kW>();
    }
    par = par0 && (MFX_PAR_MASK & 2);
    if (kBig && par) {
        MFX_BSTAMP(bs->srow, 8);
#ifndef MFX_MOVE_JUMP
#define MFX_MOVE_JUMP 1
#endif
        if (!MFX_MOVE_JUMP || !move_jump<false>(gp, sm, v, order, n_mov, *bs, nid)) move_big(gp, sm, v, order, n_mov, *bs);
        MFX_BSTAMP(bs->srow, 9);
    } else if (kW && par) {                        // (move_jump<true> measured slower for <= 64 movers)
        move_parallel<true>(gp, sm, v, order, n_mov, ps);
    } else if (par && n_mov <= MFX_WAVE_STEP_MAX) {
        if (TID < 64) move_parallel<true>(gp, sm, v, order, n_mov, ps);
        __syncthreads();
    } else if (par && bs && move_jump<false>(gp, sm, v, order, n_mov, *bs, nid)) {
    } else if (par) {
        move_parallel<false>(gp, sm, v, order, n_mov, ps);
    } else {
        if (TID == 0)
            for (int i = 0; i < n_mov; ++i) do_move_one(gp, sm, v, order[i]);
        psync<kW>();
    }
    MFX_RSTAMP(kW, stamp_row, 19);                 // moves done
    // ---- reward rules (GridWorld::calc_reward, RewardEngine.cc:373-443), rule order
    if (kDsl) {
        if (TID == 0) dsl_rewards(gp, v, dsl_mark, sm.flags);
        psync<kW>();
    }
    for (int r = 0; r < (kDsl ? 0 : gp.n_rules); ++r) {
        const RuleParams& R = gp.rules[r];
        const int n = v.grp_n[R.subj_group];
        int obj_recv = 0;
        for (int k = 0; k < R.n_recv; ++k) obj_recv |= R.recv_is_obj[k];
        if (TID == 0) sm.flags[r] = 0;
        psync<kW>();
        for (int i = TID; i < n; i += team_lanes<kW>()) {
            const int id = v.grp_ids[R.subj_group * v.cap + i];
            const uint32_t m = v.meta[id];
            const int ob = v.op_obj[id];
            if ((int)meta_op(m) != R.op || ob < 0 || (int)meta_group(v.meta[ob]) != R.obj_group) continue;
            sm.flags[r] = 1;
            for (int k = 0; k < R.n_recv; ++k)
                if (!R.recv_is_obj[k]) v.next_r[id] += R.val[k];
        }
        psync<kW>();
        if (obj_recv && TID == 0) {       // object receivers: DFS order, one lane
            for (int i = 0; i < n; ++i) {
                const int id = v.grp_ids[R.subj_group * v.cap + i];
                const uint32_t m = v.meta[id];
                const int ob = v.op_obj[id];
                if ((int)meta_op(m) != R.op || ob < 0 || (int)meta_group(v.meta[ob]) != R.obj_group) continue;
                for (int k = 0; k < R.n_recv; ++k)
                    if (R.recv_is_obj[k]) v.next_r[ob] += R.val[k];
            }
        }
        psync<kW>();
    }
    // ---- done (GridWorld.cc:678-693)
    if (TID == 0) {
        int live = 0;
        for (int g = 0; g < G; ++g) live += (v.grp_n[g] - v.grp_dead[g]) > 0;
        int d = live < G;
        if (kDsl) for (int r = 0; r < gp.prog.n_rules; ++r) d |= sm.flags[r] && gp.prog.rule[r].terminal;
        else for (int r = 0; r < gp.n_rules; ++r) d |= sm.flags[r] && gp.rules[r].terminal;
        done_out = d;
    }
    psync<kW>();
}

// Copy an env into LDS, run the step, copy back.  When `lds` is 0 the env is worked on
// in place in HBM (maps / agent counts too large for LDS).
template <bool kDsl>
__global__ void __launch_bounds__(256) k_step(const GameParams* __restrict__ gpp, State s, int lds,
                                              uint32_t* __restrict__ sort_scratch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const GameParams& gp = *gpp;
    const int e = blockIdx.x, G = gp.n_groups;
    StepSmem& sm = *reinterpret_cast<StepSmem*>(smem);
    EnvView gv = global_view(s, e, G);
    EnvView v = gv;
    const int nid = s.id_counter[e];
    const int n_atk = s.n_atk[e], n_mov = s.n_mov[e];
    uint32_t* atk = s.atk + (size_t)e * s.acap;
    uint32_t* mov = s.mov + (size_t)e * s.acap;
    uint32_t* sorted = sort_scratch + (size_t)e * s.acap;
    char* par_base = nullptr;              // LDS mode: the parallel step's scratch (ParScratch / BigScratch)
    if (lds) {
        size_t off = step_sm_bytes(G);
        auto carve = [&](size_t bytes) { char* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
        v.cells = reinterpret_cast<uint16_t*>(carve((size_t)s.cells_n * 2));
        v.xy = reinterpret_cast<uint32_t*>(carve((size_t)nid * 4));
        v.hp = reinterpret_cast<float*>(carve((size_t)nid * 4));
        v.next_r = reinterpret_cast<float*>(carve((size_t)nid * 4));
        v.op_obj = reinterpret_cast<int32_t*>(carve((size_t)nid * 4));
        v.meta = reinterpret_cast<uint8_t*>(carve((size_t)nid));
        uint32_t* latk = reinterpret_cast<uint32_t*>(carve((size_t)n_atk * 4));
        uint32_t* lmov = reinterpret_cast<uint32_t*>(carve((size_t)n_mov * 4));
        uint32_t* lsort = reinterpret_cast<uint32_t*>(carve((size_t)(gp.large_map ? n_mov : 0) * 4));
        par_base = gp.par_step ? carve(step_par_bytes(s.acap, s.cap)) : nullptr;
        for (int i = TID; i < s.cells_n; i += blockDim.x) v.cells[i] = gv.cells[i];
        for (int i = TID; i < nid; i += blockDim.x) {
            v.xy[i] = gv.xy[i]; v.hp[i] = gv.hp[i]; v.next_r[i] = gv.next_r[i];
            v.op_obj[i] = gv.op_obj[i]; v.meta[i] = gv.meta[i];
        }
        for (int i = TID; i < n_atk; i += blockDim.x) latk[i] = atk[i];
        for (int i = TID; i < n_mov; i += blockDim.x) lmov[i] = mov[i];
        atk = latk; mov = lmov; sorted = lsort;
        __syncthreads();
    }
    uint32_t rng = s.rng[e];
    int done = 0;
    load_serial_types(gp, sm);
    int32_t* ev = (gp.record_events && e == 0) ? s.ev : nullptr;
    const ParScratch ps = par_base ? carve_par(par_base, s.acap, s.cap) : ParScratch{};
    const BigScratch bs = par_base ? carve_big(par_base, s.acap, s.cap, false) : BigScratch{};
    step_env_core<false, kDsl>(gp, s, v, atk, n_atk, mov, n_mov, sorted, rng, sm, done, par_base != nullptr, ps, nid,
                               ev, kDsl ? s.idx_mark[e] : 0, par_base ? &bs : nullptr);
    if (lds) {
        for (int i = TID; i < s.cells_n; i += blockDim.x) gv.cells[i] = v.cells[i];
        for (int i = TID; i < nid; i += blockDim.x) {
            gv.xy[i] = v.xy[i]; gv.hp[i] = v.hp[i]; gv.next_r[i] = v.next_r[i];
            gv.op_obj[i] = v.op_obj[i]; gv.meta[i] = v.meta[i];
        }
    }
    if (TID == 0) {
        s.rng[e] = rng;
        s.n_atk[e] = 0;
        s.n_mov[e] = 0;
        s.done[e] = done;
    }
}

// ==================================================================================
//  clear_dead (GridWorld.cc:696-728): ordered compaction + Agent::init_reward
// ==================================================================================
template <bool kW>
__device__ __forceinline__ void clear_dead_env(const GameParams& gp, EnvView& v, int* wave_tot) {
    for (int g = 0; g < gp.n_groups; ++g) {
        const float step_reward = gp.type[g].step_reward;
        const int n = v.grp_n[g];
        uint16_t* ids = v.grp_ids + g * v.cap;
        int base = 0;
        for (int i0 = 0; i0 < n; i0 += team_lanes<kW>()) {
            const int i = i0 + TID;
            int id = -1, alive = 0;
            if (i < n) { id = ids[i]; alive = !meta_dead(v.meta[id]); }
            int tot;
            const int r = team_scan<kW>(alive, wave_tot, tot);
            // in-place compaction is safe: destination index <= source index, and all reads of
            // this round happened before the barrier inside block_scan_flag
            if (alive) {
                ids[base + r] = (uint16_t)id;
                v.last_r[id] = v.next_r[id];
                v.next_r[id] = step_reward;
                v.op_obj[id] = -1;
                v.meta[id] = (uint8_t)meta_keep_dir(meta_make(0, kOpNull, g), v.meta[id]);
            }
            base += tot;
            psync<kW>();
        }
        if (TID == 0) { v.grp_n[g] = base; v.grp_dead[g] = 0; v.grp_reward[g] = 0.0f; }
        psync<kW>();
    }
}

__global__ void __launch_bounds__(256) k_clear_dead(const GameParams* __restrict__ gp, State s) {
    __shared__ int wave_tot[16];
    EnvView v = global_view(s, blockIdx.x, gp->n_groups);
    clear_dead_env<false>(*gp, v, wave_tot);
    if (TID == 0) s.idx_mark[blockIdx.x] = s.id_counter[blockIdx.x];
}

// The drop-in host cache's record of env 0 (one workgroup): header [group sizes (kMaxGroups),
// device error word, done flag, ...] (64 B), then per group ids i32 | reward f32 | pos 2 x i32 |
// alive u8, `rows` rows each (region rounded to 16 B) -- everything the reference's getters read
// after a step, copied to the host in ONE transfer.
__global__ void __launch_bounds__(256) k_get_env0(const GameParams* __restrict__ gp, State s, uint8_t* __restrict__ out,
                                                  int rows) {
    const int G = gp->n_groups;
    EnvView v = global_view(s, 0, G);
    int32_t* hdr = reinterpret_cast<int32_t*>(out);
    if (TID < kMaxGroups) hdr[TID] = TID < G ? v.grp_n[TID] : 0;
    if (TID == kMaxGroups) hdr[kMaxGroups] = *s.err;
    if (TID == kMaxGroups + 1) hdr[kMaxGroups + 1] = s.done[0];
    const size_t region = ((size_t)rows * 17 + 15) & ~(size_t)15;
    for (int g = 0; g < G; ++g) {
        const int n = min(v.grp_n[g], rows);
        uint8_t* b = out + 64 + (size_t)g * region;
        int32_t* ids = reinterpret_cast<int32_t*>(b);
        float* rew = reinterpret_cast<float*>(b + (size_t)rows * 4);
        int32_t* pos = reinterpret_cast<int32_t*>(b + (size_t)rows * 8);
        uint8_t* alive = b + (size_t)rows * 16;
        const uint16_t* gi = v.grp_ids + g * v.cap;
        for (int i = TID; i < n; i += blockDim.x) {
            const int id = gi[i];
            const uint32_t p = v.xy[id];
            ids[i] = id;
            rew[i] = v.next_r[id] + v.grp_reward[g];
            pos[2 * i] = (int)(p & 0xFFFF);
            pos[2 * i + 1] = (int)(p >> 16);
            alive[i] = !meta_dead(v.meta[id]);
        }
    }
}

hipError_t launch_get_env0(const GameParams* d_gp, const State& s, uint8_t* d_out, int rows, hipStream_t st) {
    k_get_env0<<<1, 256, 0, st>>>(d_gp, s, d_out, rows);
    return hipGetLastError();
}

// ==================================================================================
//  getters: reward (GridWorld.cc:760-770) and info num/id/pos/alive (GridWorld.cc:786-807)
// ==================================================================================
__global__ void __launch_bounds__(256) k_get(const GameParams* __restrict__ gp, State s, int g, int what,
                                             void* __restrict__ out, int rowcap) {
    const int e = blockIdx.x;
    EnvView v = global_view(s, e, gp->n_groups);
    const int n = v.grp_n[g];
    if (what == kGetNum) { if (TID == 0) reinterpret_cast<int*>(out)[e] = n; return; }
    if (n > rowcap) { if (TID == 0) set_err(s, 4); return; }
    const uint16_t* ids = v.grp_ids + g * v.cap;
    const size_t o = (size_t)e * rowcap;
    for (int i = TID; i < n; i += blockDim.x) {
        const int id = ids[i];
        switch (what) {
            case kGetReward: reinterpret_cast<float*>(out)[o + i] = v.next_r[id] + v.grp_reward[g]; break;
            case kGetId: reinterpret_cast<int*>(out)[o + i] = id; break;
            case kGetAlive: reinterpret_cast<uint8_t*>(out)[o + i] = !meta_dead(v.meta[id]); break;
            case kGetPos: {
                const uint32_t p = v.xy[id];
                reinterpret_cast<int*>(out)[2 * (o + i)] = (int)(p & 0xFFFF);
                reinterpret_cast<int*>(out)[2 * (o + i) + 1] = (int)(p >> 16);
            } break;
            case kGetHp: reinterpret_cast<float*>(out)[o + i] = v.hp[id]; break;
            case kGetLastAct: reinterpret_cast<int*>(out)[o + i] = v.last_act[id]; break;
            case kGetDir: reinterpret_cast<int*>(out)[o + i] = meta_dir(v.meta[id]); break;
            default: break;
        }
    }
}

// ==================================================================================
//  fused rollout step: the whole reference training-loop step for one env per workgroup,
//  env state resident in LDS for the duration of the launch (senario_battle.play :96-171:
//  get_observation x G -> policy -> set_action x G -> step -> get_reward -> mean action ->
//  clear_dead, plus episode restart at done / max_steps).
// ==================================================================================
__device__ __forceinline__ uint32_t mix32(uint32_t h) {      // murmur3 finalizer
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}

// Synthetic rush policy of SURVEY.md 8(d) (tests/battle_driver.rush_policy): attack the
// first attack cell (index order = view2attack row-major order) holding an enemy, else move
// 2 cells toward the map centre; with probability eps a uniform random action instead.
// The synthetic rush policy: attack the first enemy among the attack cells in
// view2attack order, else advance +-2 in x toward the centre; with probability eps a uniform
// action.  The group index is lane-varying, so the type fields come from the LDS table, and the
// attack cells are read 8 at a time (independent LDS reads instead of a dependent chain).
__device__ __forceinline__ int rush_action(const GameParams& gp, const SerialType& S, const EnvView& v, int g,
                                           int id, uint32_t key, float eps) {
    const uint32_t p = v.xy[id];
    const int x = p & 0xFFFF, y = p >> 16, W = gp.W, H = gp.H;
    int a = ((float)x / (float)W < 0.5f) ? 8 : 4;
    if (a >= S.turn_base) a = S.turn_base - 1;
    const int bx = x + S.att_x_off, by = y + S.att_y_off, na = S.n_attack;
    for (int k0 = 0; k0 < na; k0 += 8) {
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + j;
            const int ox = bx + S.att_dx[k], oy = by + S.att_dy[k];
            const bool in = k < na && ox >= 0 && oy >= 0 && ox < W && oy < H;
            const uint32_t cv = v.cells[in ? oy * W + ox : 0];
            c[j] = in ? cv : kCellEmpty;
        }
        int hit = -1;
#pragma unroll
        for (int j = 7; j >= 0; --j) {
            const uint32_t m = v.meta[c[j] < kCellFood ? c[j] : 0u];
            if (c[j] < kCellFood && (int)meta_group(m) != g) hit = k0 + j;
        }
        if (hit >= 0) { a = S.attack_base + hit; break; }
    }
    const uint32_t h = mix32(key);
    if ((float)(h >> 8) * (1.0f / 16777216.0f) < eps) a = (int)(mix32(h ^ 0x68E31DA4u) % (uint32_t)S.n_action);
    return a;
}

// Fixed-order workgroup sum in two barriers: butterfly within each wave, then the wave partials in
// wave order (red: one float per wave).
__device__ __forceinline__ float block_sum_waves(float x, float* red) {
    const int nw = blockDim.x >> 6;
    x = wave_sum(x);
    if ((TID & 63) == 0) red[TID >> 6] = x;
    __syncthreads();
    float r = 0.0f;
    for (int w = 0; w < nw; ++w) r += red[w];
    __syncthreads();
    return r;
}

#ifndef MFX_ROLLOUT_THREADS
#define MFX_ROLLOUT_THREADS 256
#endif
#ifndef MFX_ROLLOUT_OCC
#define MFX_ROLLOUT_OCC 5          // workgroups per CU the register budget is sized for
#endif
// LDS plan of k_rollout: the env (cells, per-id arrays, group lists) stays resident for the whole
// launch; one scratch region is shared by the observation phase (minimap, bins, hp/max, staging) and
// the policy/step phase (actions, histogram, attack/move buffers; the reduction reuses the actions).
struct RolloutUnion { size_t act, ahist, atk, mov, sorted, red, par, total; };

__host__ __device__ inline RolloutUnion rollout_union(const GameParams& gp, int cap, int acap, int threads) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    RolloutUnion u;
    size_t o = 0;
    u.act = o;    o += r16((size_t)(gp.n_groups * cap > threads ? gp.n_groups * cap : threads) * 4);
    u.red = u.act;                                 // block_sum after the step: the actions are dead
    u.ahist = o;  o += r16((size_t)gp.n_groups * 64 * 4);
    u.atk = o;    o += r16((size_t)acap * 4);
    u.mov = o;    o += r16((size_t)acap * 4);
    u.sorted = o; o += gp.large_map ? r16((size_t)acap * 4) : 0;
    // the step scratch: ParScratch (wave-team / small-n forms) or BigScratch in its compact form
    // (attack_big / move_jump for the whole-workgroup team), never both in one step
    const size_t pb = par_scratch_bytes(acap, cap), bb = big_scratch_bytes(acap, cap, false);
    u.par = o;    o += gp.par_step ? r16(pb > bb ? pb : bb) : 0;
    u.total = o;
    return u;
}

__host__ __device__ inline size_t rollout_scratch_bytes(const GameParams& gp, int cap, int acap, int rows, int threads,
                                                        bool kB) {
    // (Battle shape: the agent records of every group at once, rollout_observe_groups)
    const size_t obs = obs_smem_core(gp, 0, cap, rows * (kB ? gp.n_groups : 1), obs_stage_floats(gp, 0, kB, threads), kB);
    const size_t stp = rollout_union(gp, cap, acap, threads).total;
    return obs > stp ? obs : stp;
}

// Bytes of the resident env image in LDS: cells, the seven per-id arrays, the group lists.  The
// same layout is used for the reset image in HBM (RolloutArgs::reset_image).
__host__ __device__ inline size_t env_image_bytes(int cells_n, int cap, int G) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return r16((size_t)cells_n * 2) + 5 * r16((size_t)cap * 4) + 2 * r16(cap) + r16((size_t)G * cap * 2);
}

#ifndef MFX_LDS_PAD
#define MFX_LDS_PAD 0              // experiments only: extra dynamic LDS per workgroup (lowers occupancy)
#endif
// env image | scratch union | StepSmem (G type entries)
__host__ __device__ inline size_t rollout_main_bytes(const GameParams& gp, int cells_n, int cap, int acap, int rows,
                                                     bool kB) {
    return env_image_bytes(cells_n, cap, gp.n_groups) +
           rollout_scratch_bytes(gp, cap, acap, rows, MFX_ROLLOUT_THREADS, kB);
}

size_t rollout_smem_bytes(const GameParams& gp, int cells_n, int cap, int acap, int rows) {
    return rollout_main_bytes(gp, cells_n, cap, acap, rows, is_battle_shape(gp)) + step_sm_bytes(gp.n_groups) +
           MFX_LDS_PAD;
}

size_t rollout_reset_image_bytes(const GameParams& gp, int cells_n, int cap) {
    return env_image_bytes(cells_n, cap, gp.n_groups) + 64;
}

// Carve the env image out of LDS (or any base) in the layout above.
__device__ __forceinline__ EnvView carve_env(char* base, int cells_n, int cap, int G) {
    size_t off = 0;
    auto carve = [&](size_t bytes) { char* p = base + off; off += (bytes + 15) & ~(size_t)15; return p; };
    EnvView v;
    v.cap = cap;
    v.cells = reinterpret_cast<uint16_t*>(carve((size_t)cells_n * 2));
    v.xy = reinterpret_cast<uint32_t*>(carve((size_t)cap * 4));
    v.hp = reinterpret_cast<float*>(carve((size_t)cap * 4));
    v.next_r = reinterpret_cast<float*>(carve((size_t)cap * 4));
    v.last_r = reinterpret_cast<float*>(carve((size_t)cap * 4));
    v.op_obj = reinterpret_cast<int32_t*>(carve((size_t)cap * 4));
    v.last_act = reinterpret_cast<uint8_t*>(carve((size_t)cap));
    v.meta = reinterpret_cast<uint8_t*>(carve((size_t)cap));
    v.grp_ids = reinterpret_cast<uint16_t*>(carve((size_t)G * cap * 2));
    return v;
}

__device__ __forceinline__ void copy16(void* dst, const void* src, size_t bytes) {   // 16-B aligned, bytes % 16 == 0
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* q = reinterpret_cast<const uint4*>(src);
    for (size_t i = TID; i < (bytes >> 4); i += blockDim.x) d[i] = q[i];
}

// env.reset() + add_agents(custom) of the template (GridWorld.cc:76-124, Map.cc:23-47, 200-247),
// computed once per rollout_init by one workgroup; k_rollout copies it in at every episode start.
// in_lds 0: built in place in HBM (images larger than LDS, the k_rollout_big path).
__global__ void __launch_bounds__(256) k_reset_image(const GameParams* __restrict__ gpp, int cells_n, int cap,
                                                     RolloutArgs ra, uint4* __restrict__ image, int in_lds) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int scal[8];
    const GameParams& gp = *gpp;
    const int G = gp.n_groups, W = gp.W, H = gp.H;
    char* base = in_lds ? smem : reinterpret_cast<char*>(image);
    EnvView v = carve_env(base, cells_n, cap, G);
    const size_t bytes = env_image_bytes(cells_n, cap, G);
    for (size_t i = TID; i < bytes / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(base)[i] = 0;
    __syncthreads();
    for (int c = TID; c < W * H; c += blockDim.x) {
        const int x = c % W, y = c / W;
        v.cells[c] = (x == 0 || y == 0 || x == W - 1 || y == H - 1) ? kCellWall : kCellEmpty;
    }
    __syncthreads();
    if (TID == 0) {
        int idc = 0;
        for (int g = 0; g < kMaxGroups; ++g) scal[g] = 0;
        for (int g = 0; g < G; ++g) {
            const TypeParams& T = gp.type[g];
            for (int i = 0; i < ra.tmpl_n[g]; ++i) {
                const int x = ra.tmpl_x[g * ra.tmpl_cap + i], y = ra.tmpl_y[g * ra.tmpl_cap + i];
                if (!is_blank(v.cells, W, H, x, y, -1) || idc >= cap) continue;
                const int id = idc++;
                v.cells[y * W + x] = (uint16_t)id;
                v.xy[id] = (uint32_t)x | ((uint32_t)y << 16);
                v.hp[id] = T.hp; v.last_r[id] = 0.0f; v.next_r[id] = T.step_reward;
                v.last_act[id] = T.n_action; v.op_obj[id] = -1;
                v.meta[id] = (uint8_t)meta_make(0, kOpNull, g);
                v.grp_ids[g * cap + scal[g]++] = (uint16_t)id;
            }
        }
        scal[4] = idc;
        for (int k = 5; k < 8; ++k) scal[k] = 0;
    }
    __syncthreads();
    if (in_lds) copy16(image, smem, bytes);
    if (TID < 8) reinterpret_cast<int32_t*>(reinterpret_cast<char*>(image) + bytes)[TID] = scal[TID];
}

// Per-env scalars of k_rollout, held in LDS while the env is resident.  Word w of this struct is
// loaded / stored by lane w (addresses from PfTable).
struct EnvScalars {
    int32_t grp_n[kMaxGroups];          // words 0-3
    int32_t grp_dead[kMaxGroups];       // 4-7
    float grp_reward[kMaxGroups];       // 8-11
    float ep_return[kMaxGroups];        // 12-15
    int32_t id_counter;                 // 16
    uint32_t rng;                       // 17
    int32_t ep_len;                     // 18
    int32_t pad;                        // 19
    double stats[4];                    // 20-27
    unsigned long long agent_steps;     // 28-29
};
constexpr int kScalarWords = 30;

// Register prefetch of one env (k_rollout fast path): while env e is processed, every lane of
// waves 0-2 holds its share of env e+1's image (up to 5 rows of 16 B; wave 0 also one scalar word),
// so the next install is LDS stores only.  Wave 3 alone writes env e back: a wave's vmcnt is in
// order, so the prefetch waves must not have the write-back stores queued ahead of their loads.
// The image's 16-B rows are numbered in LDS order: the cells (nc16 rows), then
// [xy hp next_r last_r op_obj] (c4 = cap/4 rows each), [last_act] [meta] (c4/4 each), [grp_ids] (G*c4/2).
constexpr int kPfLanes = MFX_ROLLOUT_THREADS - 64; // every wave but the last
constexpr int kPfSlots = 5;
constexpr int kPfRows = kPfSlots * kPfLanes;
constexpr int kWbWave = MFX_ROLLOUT_THREADS / 64 - 1;   // the write-back wave

__host__ __device__ inline int image_small_rows(int c4, int G) { return 5 * c4 + 2 * (c4 >> 2) + G * (c4 >> 1); }

struct EnvPrefetch {
    uint4 r[kPfSlots];
    uint32_t w;
};

// Address plan of the env image, built once per workgroup in LDS: for each source array (the six
// 4-byte per-id arrays, meta, grp_ids) and each EnvScalars word, the env-0 address and the bytes
// per env.  A prefetch row is then ONE load from base + e * stride + offset; choosing among
// separate pointers per lane instead would serialise the loads (each predicated load into the same
// registers waits for the previous one).
struct PfTable {
    unsigned long long walls;           // RolloutArgs::wall_image (cells rows, shared by every env)
    unsigned long long base[8];         // xy hp next_r last_r op_obj, last_act, meta, grp_ids
    unsigned int stride[8];
    unsigned long long sbase[32];       // 0: word absent (group >= G, padding)
    unsigned int sstride[32];
};

__device__ __forceinline__ void pf_table_init(PfTable& pt, const State& s, const RolloutArgs& ra, int G) {
    const int t = TID;
    const unsigned cap4 = (unsigned)s.cap * 4u;
    if (t == 0) pt.walls = (unsigned long long)ra.wall_image;
    if (t < 8) {
        const void* p = nullptr;
        unsigned st = cap4;
        if (t == 0) p = s.xy;
        if (t == 1) p = s.hp;
        if (t == 2) p = s.next_r;
        if (t == 3) p = s.last_r;
        if (t == 4) p = s.op_obj;
        if (t == 5) { p = s.last_act; st = (unsigned)s.cap; }
        if (t == 6) { p = s.meta; st = (unsigned)s.cap; }
        if (t == 7) { p = s.grp_ids; st = (unsigned)s.cap * 2u * (unsigned)G; }
        pt.base[t] = (unsigned long long)p;
        pt.stride[t] = st;
    }
    if (t < 32) {
        const int g = t & 3;
        const char* p = nullptr;
        unsigned st = 4;
        if (t < 16 && g < G) {
            st = 4u * (unsigned)G;
            if ((t >> 2) == 0) p = reinterpret_cast<const char*>(s.grp_n + g);
            if ((t >> 2) == 1) p = reinterpret_cast<const char*>(s.grp_dead + g);
            if ((t >> 2) == 2) p = reinterpret_cast<const char*>(s.grp_reward + g);
            if ((t >> 2) == 3) p = reinterpret_cast<const char*>(ra.ep_return + g);
        }
        if (t == 16) p = reinterpret_cast<const char*>(s.id_counter);
        if (t == 17) p = reinterpret_cast<const char*>(s.rng);
        if (t == 18) p = reinterpret_cast<const char*>(ra.ep_len);
        if (t >= 20 && t < 28) { p = reinterpret_cast<const char*>(ra.stats) + 4 * (t - 20); st = 32; }
        if (t >= 28 && t < 30) { p = reinterpret_cast<const char*>(ra.agent_steps) + 4 * (t - 28); st = 8; }
        pt.sbase[t] = (unsigned long long)p;
        pt.sstride[t] = st;
    }
}

// Table addresses are integers: cast them to the GLOBAL address space.  A generic pointer would
// make these flat_load / flat_store, which also count in lgkmcnt, so every later LDS wait would
// wait for the HBM round trip too.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint32_t g_u32;

__device__ __forceinline__ uint4 ld_g16(const g_u32x4* p) {
#ifdef MFX_NT_LD
    const u32x4 x = __builtin_nontemporal_load(p);
#else
    const u32x4 x = *p;
#endif
    return make_uint4(x.x, x.y, x.z, x.w);
}

// Address of 16-B row k of the per-id / group-list part of env e's image (LDS order, see EnvPrefetch).
__device__ __forceinline__ const g_u32x4* small_row_addr(const PfTable& pt, int e, int k, int sh, int c4) {
    const int j = k >> sh, k2 = k - 5 * c4, q = c4 >> 2;
    const int a = j < 5 ? j : (k2 < q ? 5 : (k2 < 2 * q ? 6 : 7));
    const int r = j < 5 ? (k & (c4 - 1)) : (k2 < q ? k2 : (k2 < 2 * q ? k2 - q : k2 - 2 * q));
    return (const g_u32x4*)(pt.base[a] + (unsigned long long)e * pt.stride[a] + (unsigned)r * 16u);
}

// Address of row r of env e's whole image: the cells first, then the small part.
__device__ __forceinline__ const g_u32x4* image_row_addr(const PfTable& pt, const State& s, int e, int r, int nc16,
                                                         int sh, int c4) {
    const unsigned long long cells = pt.walls + (unsigned)r * 16u;            // walls only (L2-resident)
    return r < nc16 ? (const g_u32x4*)cells : small_row_addr(pt, e, r - nc16, sh, c4);
}

__device__ __forceinline__ g_u32* scalar_addr(const PfTable& pt, int e, int w) {
    const unsigned long long b = pt.sbase[w];
    return b ? (g_u32*)(b + (unsigned long long)e * pt.sstride[w]) : nullptr;
}

__device__ __forceinline__ uint32_t load_scalar_word(const PfTable& pt, int e, int w) {
    const g_u32* p = scalar_addr(pt, e, w);
    return p ? *p : 0u;
}

__device__ __forceinline__ void pf_issue(EnvPrefetch& pf, const PfTable& pt, const State& s, int e, int nrows,
                                         int nc16, int sh, int c4) {
    const int t = TID;
    if (t >= kPfLanes) return;
#pragma unroll
    for (int j = 0; j < kPfSlots; ++j) {
        const int r = t + j * kPfLanes;
        if (r < nrows) pf.r[j] = ld_g16(image_row_addr(pt, s, e, r, nc16, sh, c4));
    }
    if (t < kScalarWords) pf.w = load_scalar_word(pt, e, t);
}

__device__ __forceinline__ void pf_install(const EnvPrefetch& pf, char* image, EnvScalars& sc, int nrows) {
    // One unconditional vmcnt(0) (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15).  Left to the
    // compiler, the waits sit inside the exec-masked stores below, so along the skipped paths the
    // registers still look in flight and the next pf_issue waits again before every load.
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int t = TID;
    if (t >= kPfLanes) return;
    uint4* d = reinterpret_cast<uint4*>(image);
#pragma unroll
    for (int j = 0; j < kPfSlots; ++j) {
        const int r = t + j * kPfLanes;
        if (r < nrows) d[r] = pf.r[j];
    }
    if (t < kScalarWords) reinterpret_cast<uint32_t*>(&sc)[t] = pf.w;
}

// 16-B copy by one wave (lane stride 64).
__device__ __forceinline__ void wcopy16(void* dst, const void* src, size_t bytes, int lane) {
#ifdef MFX_NT_WB
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    u32x4_t* d = reinterpret_cast<u32x4_t*>(dst);
    const u32x4_t* q = reinterpret_cast<const u32x4_t*>(src);
    for (size_t i = lane; i < (bytes >> 4); i += 64) __builtin_nontemporal_store(q[i], d + i);
#else
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* q = reinterpret_cast<const uint4*>(src);
    for (size_t i = lane; i < (bytes >> 4); i += 64) d[i] = q[i];
#endif
}

// Generic install (maps / capacities beyond the prefetch budget): straight copies.
__device__ __forceinline__ void install_sync(const State& s, const PfTable& pt, int e, int G, const EnvView& v,
                                             EnvScalars& sc) {
    const EnvView gv = global_view(s, e, G);
    const int cap = s.cap;
    const uint16_t* walls = reinterpret_cast<const uint16_t*>(pt.walls);
    if ((s.cells_n & 7) == 0) {
        copy16(v.cells, walls, (size_t)s.cells_n * 2);
    } else {
        for (int i = TID; i < s.cells_n; i += blockDim.x) v.cells[i] = walls[i];
    }
    copy16(v.xy, gv.xy, (size_t)cap * 4);
    copy16(v.hp, gv.hp, (size_t)cap * 4);
    copy16(v.next_r, gv.next_r, (size_t)cap * 4);
    copy16(v.last_r, gv.last_r, (size_t)cap * 4);
    copy16(v.op_obj, gv.op_obj, (size_t)cap * 4);
    copy16(v.last_act, gv.last_act, (size_t)cap);
    copy16(v.meta, gv.meta, (size_t)cap);
    copy16(v.grp_ids, gv.grp_ids, (size_t)G * cap * 2);
    if (TID < kScalarWords)
        reinterpret_cast<uint32_t*>(&sc)[TID] = load_scalar_word(pt, e, TID);
}

// Work queue of k_rollout: envs heaviest first (an env's step time grows with its agent count), so
// a launch does not end on a tail of a few late episode starts.  Every workgroup files the envs it
// finishes under their new weight class in the next launch's class lists (buffered in LDS, one
// atomic per class per flush); the next launch walks the lists class by class.
constexpr int kOrderClasses = 8;

__device__ __forceinline__ int env_weight_class(int w) {
    return w >= 192 ? 0 : w >= 128 ? 1 : w >= 96 ? 2 : w >= 64 ? 3 : w >= 48 ? 4 : w >= 32 ? 5 : w >= 16 ? 6 : 7;
}



constexpr int kQueueBuf = 32;                      // envs buffered per workgroup before a flush

// Env at queue position i of this launch (qpre: prefix of the class counts, qpre[8] = E).
__device__ __forceinline__ int queue_env(const RolloutArgs& ra, const int* qpre, int i, int E, int qphase) {
    if (i >= E) return E;
    int c = 0;
    while (c < kOrderClasses - 1 && i >= qpre[c + 1]) ++c;
    return ra.cls_list[((size_t)(qphase & 1) * kOrderClasses + c) * ra.cls_stride + (i - qpre[c])];
}

// Thread 0: append the buffered envs to the next launch's class lists.
__device__ __forceinline__ void queue_flush(const RolloutArgs& ra, const int* wg_env, const uint8_t* wg_cls, int n,
                                            int qphase, int* tmp) {
    const int cn = (qphase + 1) % 3, ln = (qphase + 1) & 1;
    for (int c = 0; c < kOrderClasses; ++c) tmp[c] = 0;
    for (int k = 0; k < n; ++k) ++tmp[wg_cls[k]];
    for (int c = 0; c < kOrderClasses; ++c)
        tmp[c] = tmp[c] ? atomicAdd(ra.cls_cnt + cn * kOrderClasses + c, tmp[c]) : 0;
    for (int k = 0; k < n; ++k) {
        const int c = wg_cls[k];
        ra.cls_list[((size_t)ln * kOrderClasses + c) * ra.cls_stride + tmp[c]++] = wg_env[k];
    }
}

// Policy, mean action, set_action, step, get_reward and clear_dead of one env, run by a team (see
// psync): the whole workgroup, or wave 0 alone when the env has at most 64 agents.
#ifndef MFX_FUSED_BIG
#define MFX_FUSED_BIG 1            // k_rollout's workgroup teams use attack_big / move_jump
#endif
template <bool kB, bool kW>
__device__ __forceinline__ void agent_phase(const GameParams& gp, const State& s, const RolloutArgs& ra, EnvView& v,
                                            EnvScalars& sc, int* misc, StepSmem& sm, int32_t* act, int* ahist,
                                            uint32_t* atk, uint32_t* mov, uint32_t* sorted, float* red,
                                            const ParScratch ps, const BigScratch* bs, int e, uint32_t step_index,
                                            int stamp_row, uint32_t& rng, int& done, float& kills) {
    (void)stamp_row;
    const int G = gp.n_groups, cap = s.cap, acap = s.acap;
#ifdef MFX_STAMPS
    if (TID == 0 && g_stamps) g_stamps[stamp_row * kStampW + 16] = (unsigned long long)(v.grp_n[0] + (G > 1 ? v.grp_n[1] : 0));
#endif
    // ---------------- policy + mean action (former_act_prob), all groups in one pass
    {
        int ntot = 0;
        for (int g = 0; g < G; ++g) ntot += v.grp_n[g];
        for (int i = TID; i < G * 64; i += team_lanes<kW>()) ahist[i] = 0;
        psync<kW>();
        const uint32_t ekey = ra.policy_seed ^ mix32(step_index * 0x9E3779B9u + (uint32_t)e * 0x632BE5ABu);
        for (int t = TID; t < ntot; t += team_lanes<kW>()) {
            int g = 0, i = t;
            while (i >= v.grp_n[g]) { i -= v.grp_n[g]; ++g; }
            const int id = v.grp_ids[g * cap + i];
            const uint32_t key = ekey ^ mix32((uint32_t)id * 0x85EBCA77u + (uint32_t)g);
            const int a = rush_action(gp, sm.tt[g], v, g, id, key, ra.eps);
            act[g * cap + i] = a;
            if (i < ra.rowcap) ra.actions[((size_t)e * G + g) * ra.rowcap + i] = a;
            atomicAdd(&ahist[g * 64 + a], 1);
        }
        psync<kW>();
        for (int t = TID; t < G * 64; t += team_lanes<kW>()) {
            const int g = t >> 6, k = t & 63, na = sm.tt[g].n_action, n = v.grp_n[g];
            if (k < na)   // empty group: np.mean of nothing is NaN
                ra.mean_act[((size_t)e * G + g) * na + k] = n ? (double)ahist[t] / (double)n : __longlong_as_double(0x7FF8000000000000ll);
        }
    }
    MFX_TSTAMP(kW, 4);
    // ---------------- set_action (group order) and step
    for (int g = 0; g < G; ++g) set_action_group<kW>(gp, s, v, g, act + g * cap, atk, misc[0], mov, misc[1], sm.wave_tot, acap);
    MFX_TSTAMP(kW, 5);
    step_env_core<kW>(gp, s, v, atk, misc[0], mov, misc[1], sorted, rng, sm, done, true, ps, sc.id_counter, nullptr,
                      0, MFX_FUSED_BIG ? bs : nullptr, stamp_row);
    MFX_TSTAMP(kW, 6);
    // ---------------- get_reward, episode return, kills
    for (int g = 0; g < G; ++g) {
        const int n = v.grp_n[g];
        float part = 0.0f;
        for (int i = TID; i < n; i += team_lanes<kW>()) {
            const float r = v.next_r[v.grp_ids[g * cap + i]] + v.grp_reward[g];
            if (i < ra.rowcap) ra.rewards[((size_t)e * G + g) * ra.rowcap + i] = r;
            part += r;
        }
        const float tot = kW ? wave_sum(part) : block_sum_waves(part, red);
        if (TID == 0) { sc.ep_return[g] += tot; kills += (float)v.grp_dead[g]; }
    }
    MFX_TSTAMP(kW, 7);
    // ---------------- clear_dead
    clear_dead_env<kW>(gp, v, sm.wave_tot);
    MFX_TSTAMP(kW, 8);
}

// get_observation of every group of the env in LDS (after obs_prologue + obs_minimap): rows of
// env e in ra.view / ra.feat.
// records_ready: the agent records were written with the minimap (obs_minimap_add) and a barrier
// has passed since.
template <bool kB>
__device__ __forceinline__ void rollout_observe_groups(const GameParams& gp, const RolloutArgs& ra, const EnvView& v,
                                                       const ObsSmem& osm, int e, bool records_ready) {
    if (kB) {                                  // every group's records, one barrier, every group's stream
        if (!records_ready) {
            for (int g = 0; g < BattleShape::G; ++g) {
                ObsSmem og = osm;
                og.aq = osm.aq + g * ra.rowcap;
                obs_agent_records(gp, v, og, g, min(v.grp_n[g], ra.rowcap));
            }
            __syncthreads();
        }
#ifndef MFX_DIAG_NO_OBS                              // diagnostic builds only: everything but the stream
        for (int g = 0; g < BattleShape::G; ++g) {
            constexpr size_t VF = (size_t)BattleShape::VW * BattleShape::VH * BattleShape::NC;
            ObsSmem og = osm;
            og.aq = osm.aq + g * ra.rowcap;
            obs_stream_battle(gp, v, og, g, min(v.grp_n[g], ra.rowcap), ra.view[g] + (size_t)e * ra.rowcap * VF,
                              ra.feat[g] + (size_t)e * ra.rowcap * BattleShape::F, osm.stage);
        }
#endif
        __syncthreads();
        return;
    }
    for (int g = 0; g < gp.n_groups; ++g) {
        const TypeParams& T = gp.type[g];
        const size_t VF = (size_t)T.view_w * T.view_h * gp.n_ch;
        float* ov = ra.view[g] + (size_t)e * ra.rowcap * VF;
        float* of = ra.feat[g] + (size_t)e * ra.rowcap * gp.feat_size[g];
        const int n = min(v.grp_n[g], ra.rowcap);
        obs_prologue(gp, osm, g);
        __syncthreads();
        for (int a0 = 0; a0 < n; a0 += kObsK) obs_rows<kB>(gp, v, osm, g, a0, min(kObsK, n - a0), ov, of);
    }
}

// One launch = one training-loop step for every env.  Persistent workgroups: the grid is what
// fits on the chip at once, and each workgroup takes envs from a work queue, keeping env e in LDS
// while the next env's image is already in flight into registers.
// kSplit: the step half of the observation/step pipeline -- no observation, and env e is written
// back to ctx->w instead of ctx->s.
template <bool kB, bool kPf, bool kSplit>
__global__ void __launch_bounds__(MFX_ROLLOUT_THREADS, MFX_ROLLOUT_OCC) k_rollout(const GameParams* __restrict__ gpp,
                                                                 const RolloutCtx* __restrict__ ctx,
                                                                 uint32_t step_index, int work_sel, int qphase) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ EnvScalars sc;
    __shared__ int misc[8];                  // 0 n_atk, 1 n_mov, 3 episode end, 4 done, 5-7 queue hand-off
    __shared__ int32_t n_before[kMaxGroups];
    __shared__ PfTable pt;
    __shared__ PfTable ptw;                  // kSplit: the write-back copy's addresses
    __shared__ int qpre[kOrderClasses + 1], qtmp[kOrderClasses];
    __shared__ int wg_env[kQueueBuf];
    __shared__ uint8_t wg_cls[kQueueBuf];
    __shared__ int wg_n;                     // envs buffered in wg_env / wg_cls
    // StepSmem (serial type table, scan / flag words) follows the env image and the scratch union
    StepSmem& sm = *reinterpret_cast<StepSmem*>(
        smem + rollout_main_bytes(kconst(gpp), kconst(ctx).s.cells_n, kconst(ctx).s.cap, kconst(ctx).s.acap,
                                  kconst(ctx).ra.rowcap, kB));
    // Work queue: position i of this launch is env queue_env(i) (class lists, heaviest first).
    // The hand-off is pipelined so that no queue access is waited on: while env e_k is processed,
    // e_{k+1} is being prefetched, thread 0 holds e_{k+2} (o) and the queue slot of e_{k+3} (g),
    // and both loads land before the next install's vmcnt(0).
    int e, en;
    int o = 0, g = 0;
    EnvPrefetch pf;
#pragma unroll
    for (int j = 0; j < kPfSlots; ++j) pf.r[j] = make_uint4(0, 0, 0, 0);
    pf.w = 0;
    {
        const GameParams& gp = kconst(gpp);
        const State& s = kconst(ctx).s;
        const RolloutArgs& ra = kconst(ctx).ra;
        const int G = gp.n_groups, c4 = s.cap >> 2, sh = __ffs(c4) - 1;
        const int nc16 = s.cells_n >> 3, nrows = nc16 + image_small_rows(c4, G);
        if (TID == 0) {
            if (blockIdx.x == 0) {
                ra.work[work_sel ^ 1] = 0;
                for (int c = 0; c < kOrderClasses; ++c) ra.cls_cnt[((qphase + 2) % 3) * kOrderClasses + c] = 0;
            }
            int acc = 0;
            for (int c = 0; c < kOrderClasses; ++c) { qpre[c] = acc; acc += ra.cls_cnt[(qphase % 3) * kOrderClasses + c]; }
            qpre[kOrderClasses] = acc;
            for (int k = 5; k < 8; ++k) misc[k] = queue_env(ra, qpre, atomicAdd(ra.work + work_sel, 1), s.E, qphase);
            g = atomicAdd(ra.work + work_sel, 1);
            wg_n = 0;
        }
        load_serial_types(gp, sm);
        pf_table_init(pt, s, ra, G);
        if (kSplit) pf_table_init(ptw, kconst(ctx).w, ra, G);
        __syncthreads();
        e = misc[5]; en = misc[6];
        if (TID == 0) o = misc[7];
        if (kPf && e < s.E) pf_issue(pf, pt, s, e, nrows, nc16, sh, c4);
    }
    while (true) {
#ifdef MFX_STAMPS
    if (TID == 0 && g_stamps && e < kconst(ctx).s.E) g_stamps[e * kStampW + 14] = __builtin_amdgcn_s_memrealtime();
#endif
    // every iteration re-reads its parameters through scalar loads (see RolloutCtx)
    const GameParams& gp = kconst(gpp);
    const State& s = kconst(ctx).s;
    const RolloutArgs& ra = kconst(ctx).ra;
    if (e >= s.E) break;
    const int G = gp.n_groups, cap = s.cap, acap = s.acap;
    // ---------------- carve LDS
    EnvView v = carve_env(smem, s.cells_n, cap, G);
    v.grp_n = sc.grp_n; v.grp_dead = sc.grp_dead; v.grp_reward = sc.grp_reward;
    const size_t soff = env_image_bytes(s.cells_n, cap, G);
    char* uni = smem + soff;                 // scratch shared by the observation and the step phases
    size_t soff2 = soff;
    ObsSmem osm = carve_obs(smem, gp, 0, cap, ra.rowcap * (kB ? G : 1), obs_stage_floats(gp, 0, kB, blockDim.x), kB,
                            soff2);
    if (!kB) osm.info = nullptr;
    const RolloutUnion u = rollout_union(gp, cap, acap, blockDim.x);
    int32_t* act = reinterpret_cast<int32_t*>(uni + u.act);
    int* ahist = reinterpret_cast<int*>(uni + u.ahist);
    uint32_t* atk = reinterpret_cast<uint32_t*>(uni + u.atk);
    uint32_t* mov = reinterpret_cast<uint32_t*>(uni + u.mov);
    uint32_t* sorted = reinterpret_cast<uint32_t*>(uni + u.sorted);
    float* red = reinterpret_cast<float*>(uni + u.red);
    const size_t img_bytes = env_image_bytes(s.cells_n, cap, G);
    const int32_t* img_scal = reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(ra.reset_image) + img_bytes);
    const int c4 = cap >> 2, sh = __ffs(c4) - 1;
    const int nc16 = s.cells_n >> 3, nrows = nc16 + image_small_rows(c4, G);
    {
        const int stamp_row = e;
        (void)stamp_row;
        MFX_STAMP(0);
        // ---------------- install env e
        if (kPf) pf_install(pf, smem, sc, nrows);
        else install_sync(s, pt, e, G, v, sc);
        if (TID == 0) { misc[0] = 0; misc[1] = 0; misc[5] = o; }
        constexpr bool kMmFused = kB && !kSplit && MFX_MM_IN_INSTALL;
        if (kMmFused) {                          // the minimap histogram rides on the placement pass
            obs_prologue(gp, osm, 0);
            for (int i = TID; i < G * BattleShape::VW * BattleShape::VH; i += blockDim.x) osm.hist[i] = 0;
        }
        __syncthreads();
        // the agents onto the walls-only cells: every listed agent is alive at an install (the lists
        // were compacted at the end of the env's previous step)
        for (int q = 0; q < G; ++q) {
            const int nq = sc.grp_n[q];
            for (int i = TID; i < nq; i += blockDim.x) {
                const int id = v.grp_ids[q * cap + i];
                const uint32_t p = v.xy[id];
                if (!meta_dead(v.meta[id])) v.cells[(p >> 16) * gp.W + (p & 0xFFFF)] = (uint16_t)id;
                if (kMmFused) obs_minimap_add(gp, v, osm, q, id, p, i, ra.rowcap);
            }
        }
        __syncthreads();
        MFX_STAMP(13);
        if (TID < G) n_before[TID] = sc.grp_n[TID];
        if (kPf && en < s.E) pf_issue(pf, pt, s, en, nrows, nc16, sh, c4);
        if (TID == 0) {                        // lands long before the next install
            o = queue_env(ra, qpre, g, s.E, qphase);
            g = atomicAdd(ra.work + work_sel, 1);
        }
        MFX_STAMP(1);
        // ---------------- get_observation for every group (k_rollout_obs in the pipeline)
        if (!kSplit) {
            if (kB && MFX_MM_IN_INSTALL) {
                obs_minimap_finish<kB>(gp, v, osm);
            } else {
                obs_prologue(gp, osm, 0);
                obs_minimap<kB>(gp, v, osm, 0);      // one view size for every group (rollout_plan)
            }
            MFX_STAMP(2);
            rollout_observe_groups<kB>(gp, ra, v, osm, e, kB && MFX_MM_IN_INSTALL);
        }
        if (kSplit) __syncthreads();           // (rollout_observe_groups ends with one: the scratch changes hands)
        MFX_STAMP(3);
        // ---------------- policy, set_action, step, get_reward, clear_dead (agent_phase)
        uint32_t rng = sc.rng;
        int done = 0;
        float kills = 0.0f;
        {
            const ParScratch ps = carve_par(uni + u.par, acap, cap);
            BigScratch bs = carve_big(uni + u.par, acap, cap, false);
#ifdef MFX_STAMPS
            bs.srow = stamp_row; bs.sbase = 20;        // attack_big's stamps in slots 23-26
#endif
            int ntot = 0;
            for (int g = 0; g < G; ++g) ntot += v.grp_n[g];
#ifdef MFX_DIAG_OBS_ONLY                             // diagnostic builds only: the observation alone
            if (false) {
#else
            if (ntot <= 64) {
#endif
                if (TID < 64)                  // wave 0 (and its lane 0 below) alone; the others wait at
                    agent_phase<kB, true>(gp, s, ra, v, sc, misc, sm, act, ahist, atk, mov, sorted, red, ps, &bs, e,
                                          step_index, stamp_row, rng, done, kills);   // the episode-end barrier
            } else {
#ifndef MFX_DIAG_OBS_ONLY
                agent_phase<kB, false>(gp, s, ra, v, sc, misc, sm, act, ahist, atk, mov, sorted, red, ps, &bs, e,
                                       step_index, stamp_row, rng, done, kills);
#endif
            }
        }
        // ---------------- episode end -> reset + re-place the template (env.reset + add_agents)
        if (TID == 0) {
            sc.stats[3] += kills;
            int len = sc.ep_len + 1;
            misc[3] = 0;
            if (done || len >= ra.max_steps) {
                sc.stats[0] += 1.0;
                sc.stats[1] += sc.ep_return[0];
                sc.stats[2] += G > 1 ? sc.ep_return[1] : 0.0f;
                for (int g = 0; g < G; ++g) sc.ep_return[g] = 0.0f;
                len = 0;
                misc[3] = 1;
            }
            sc.ep_len = len;
            sc.rng = rng;
            misc[4] = done;
            unsigned long long tot = 0;
            for (int g = 0; g < G; ++g) tot += (unsigned)n_before[g];
            sc.agent_steps += tot;
        }
        __syncthreads();
        if (misc[3]) {
            copy16(v.cells, ra.reset_image, img_bytes);
            if (TID < G) {
                sc.grp_n[TID] = img_scal[TID];
                sc.grp_dead[TID] = 0;
                sc.grp_reward[TID] = 0.0f;
            }
            if (TID == 0) sc.id_counter = img_scal[4];
            __syncthreads();
        }
        MFX_STAMP(9);
        if (TID == 0) {                        // file the env for the next launch's queue
            int w = 0;
            for (int q = 0; q < G; ++q) w += sc.grp_n[q];
            wg_env[wg_n] = e;
            wg_cls[wg_n] = (uint8_t)env_weight_class(w);
            if (++wg_n == kQueueBuf) { queue_flush(ra, wg_env, wg_cls, wg_n, qphase, qtmp); wg_n = 0; }
        }
        // ---------------- write the env back (wave kWbWave only, see EnvPrefetch)
        if ((TID >> 6) == kWbWave) {
            const int lane = TID & 63;
            const EnvView gv = global_view(kSplit ? kconst(ctx).w : s, e, G);   // cells: rebuilt at the next install
            const int idc = sc.id_counter;
            const size_t n4 = ((size_t)idc + 3) & ~(size_t)3, n16 = ((size_t)idc + 15) & ~(size_t)15;
            wcopy16(gv.xy, v.xy, n4 * 4, lane);
            wcopy16(gv.hp, v.hp, n4 * 4, lane);
            wcopy16(gv.next_r, v.next_r, n4 * 4, lane);
            wcopy16(gv.last_r, v.last_r, n4 * 4, lane);
            wcopy16(gv.op_obj, v.op_obj, n4 * 4, lane);
            wcopy16(gv.last_act, v.last_act, n16, lane);
            wcopy16(gv.meta, v.meta, n16, lane);
            for (int g = 0; g < G; ++g)
                wcopy16(gv.grp_ids + g * cap, v.grp_ids + g * cap, (((size_t)v.grp_n[g] + 7) & ~(size_t)7) * 2, lane);
            if (lane < kScalarWords) {
                g_u32* p = scalar_addr(kSplit ? ptw : pt, e, lane);
                if (p) *p = reinterpret_cast<const uint32_t*>(&sc)[lane];
            }
            if (lane == 0) { s.n_atk[e] = 0; s.n_mov[e] = 0; s.done[e] = misc[4]; }
        }
        MFX_STAMP(10);
        __syncthreads();                       // LDS reads of the write-back are done; hand-off visible
        e = en;
        en = misc[5];
    }
    }
    if (TID == 0 && wg_n) queue_flush(kconst(ctx).ra, wg_env, wg_cls, wg_n, qphase, qtmp);
}

#ifndef MFX_OBS_OCC
#define MFX_OBS_OCC 8              // k_rollout_obs: <= 64 VGPRs, so it fits beside k_rollout's waves
#endif
// The observation half of the pipeline: get_observation of every env of the launch from the
// state before the step (ctx->s), beside k_rollout<.., kSplit> which steps the same envs from the
// same copy and writes the other.  Persistent workgroups on their own counter (RolloutArgs::work
// [2 + sel]) over the same heaviest-first queue; env e+1's image is in flight into registers
// while env e is observed.  LDS: the env image, then the observation scratch.
template <bool kB, bool kPf>
__global__ void __launch_bounds__(MFX_ROLLOUT_THREADS, MFX_OBS_OCC) k_rollout_obs(const GameParams* __restrict__ gpp,
                                                                                 const RolloutCtx* __restrict__ ctx,
                                                                                 int work_sel, int qphase) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ EnvScalars sc;
    __shared__ int misc[4];                  // 0-1 queue hand-off
    __shared__ PfTable pt;
    __shared__ int qpre[kOrderClasses + 1];
    int e, en;
    EnvPrefetch pf;
#pragma unroll
    for (int j = 0; j < kPfSlots; ++j) pf.r[j] = make_uint4(0, 0, 0, 0);
    pf.w = 0;
    {
        const GameParams& gp = kconst(gpp);
        const State& s = kconst(ctx).s;
        const RolloutArgs& ra = kconst(ctx).ra;
        const int G = gp.n_groups, c4 = s.cap >> 2, sh = __ffs(c4) - 1;
        const int nc16 = s.cells_n >> 3, nrows = nc16 + image_small_rows(c4, G);
        if (TID == 0) {
            if (blockIdx.x == 0) ra.work[2 + (work_sel ^ 1)] = 0;
            int acc = 0;
            for (int c = 0; c < kOrderClasses; ++c) { qpre[c] = acc; acc += ra.cls_cnt[(qphase % 3) * kOrderClasses + c]; }
            qpre[kOrderClasses] = acc;
            for (int k = 0; k < 2; ++k) misc[k] = queue_env(ra, qpre, atomicAdd(ra.work + 2 + work_sel, 1), s.E, qphase);
        }
        pf_table_init(pt, s, ra, G);
        __syncthreads();
        e = misc[0]; en = misc[1];
        if (kPf && e < s.E) pf_issue(pf, pt, s, e, nrows, nc16, sh, c4);
    }
    while (true) {
        const GameParams& gp = kconst(gpp);
        const State& s = kconst(ctx).s;
        const RolloutArgs& ra = kconst(ctx).ra;
        if (e >= s.E) break;
        const int G = gp.n_groups, cap = s.cap;
        EnvView v = carve_env(smem, s.cells_n, cap, G);
        v.grp_n = sc.grp_n; v.grp_dead = sc.grp_dead; v.grp_reward = sc.grp_reward;
        size_t soff = env_image_bytes(s.cells_n, cap, G);
        ObsSmem osm = carve_obs(smem, gp, 0, cap, ra.rowcap * (kB ? G : 1), obs_stage_floats(gp, 0, kB, blockDim.x),
                                kB, soff);
        if (!kB) osm.info = nullptr;
        const int c4 = cap >> 2, sh = __ffs(c4) - 1;
        const int nc16 = s.cells_n >> 3, nrows = nc16 + image_small_rows(c4, G);
        if (kPf) pf_install(pf, smem, sc, nrows);
        else install_sync(s, pt, e, G, v, sc);
        __syncthreads();
        for (int q = 0; q < G; ++q) {           // the listed agents onto the walls-only cells
            const int nq = sc.grp_n[q];
            for (int i = TID; i < nq; i += blockDim.x) {
                const int id = v.grp_ids[q * cap + i];
                const uint32_t p = v.xy[id];
                if (!meta_dead(v.meta[id])) v.cells[(p >> 16) * gp.W + (p & 0xFFFF)] = (uint16_t)id;
            }
        }
        if (TID == 0) misc[0] = queue_env(ra, qpre, atomicAdd(ra.work + 2 + work_sel, 1), s.E, qphase);
        __syncthreads();
        if (kPf && en < s.E) pf_issue(pf, pt, s, en, nrows, nc16, sh, c4);
        obs_prologue(gp, osm, 0);
        obs_minimap<kB>(gp, v, osm, 0);
        rollout_observe_groups<kB>(gp, ra, v, osm, e, false);
        __syncthreads();                        // the image and the hand-off change hands
        e = en;
        en = misc[0];
    }
}

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

hipError_t launch_add_agents(const GameParams* d_gp, const State& s, int group, int n, int method,
                             const int* d_xs, const int* d_ys, const int* d_dirs, int per_env_stride, hipStream_t st) {
    k_add_agents<<<(s.E + 63) / 64, 64, 0, st>>>(d_gp, s, group, n, method, d_xs, d_ys, d_dirs, per_env_stride);
    return hipGetLastError();
}

// ==================================================================================
//  envs too large for one workgroup's LDS (256x256 / 4096 agents): state stays in HBM
// ==================================================================================
// One 1024-lane workgroup per env.  LDS holds the step scratch (BigScratch), the move order and,
// for the rollout, the action buffers; the cells and per-id arrays are read and written in place.
constexpr int kBigThreads = 1024;
#ifndef MFX_BIG_ROLLOUT_THREADS
#define MFX_BIG_ROLLOUT_THREADS 512
#endif
// k_rollout_big shares its CUs with the other sub-batch's k_observe: 8 waves of <= 128 VGPRs and
// ~80 KB of LDS leave room for observation workgroups beside it
constexpr int kBigRolloutThreads = MFX_BIG_ROLLOUT_THREADS;

struct BigLayout { size_t sm, atk, mov, sorted, ahist, red, big, total; };

__host__ __device__ inline BigLayout big_layout(const GameParams& gp, int cap, int acap, bool rollout) {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    BigLayout L;
    size_t o = 0;
    L.sm = o;     o += step_sm_bytes(gp.n_groups);
    L.atk = o;                   // the rollout's attack / move buffers are State::atk / mov (HBM)
    L.mov = o;
    L.sorted = o; o += (gp.large_map && !rollout) ? r16((size_t)acap * 4) : 0;   // rollout: RolloutArgs::big_sort
    L.ahist = o;  o += rollout ? r16((size_t)gp.n_groups * 64 * 4) : 0;
    L.big = o;    o += r16(big_scratch_bytes(acap, cap));
    L.red = L.big;                   // block_sum runs after the step: the step scratch is dead
    L.total = o;
    return L;
}

size_t big_step_smem_bytes(const GameParams& gp, int cap, int acap, bool rollout) {
    return big_layout(gp, cap, acap, rollout).total;
}

// The inputs every observing chunk of env e shares (Battle shape): the per-group minimap density
// (obs_minimap) and the packed hp/max | group word of every listed agent, written to HBM once.
// hist: G * 169 ints of LDS.
__device__ void obs_prep_env(const GameParams& gp, const EnvView& v, float* __restrict__ mm_out,
                             uint32_t* __restrict__ info_out, int* hist) {
    constexpr int VW = BattleShape::VW, VH = BattleShape::VH, NV = VW * VH, G = BattleShape::G;
    const int sw = (gp.W + VW - 1) / VW, sh = (gp.H + VH - 1) / VH;
    for (int i = TID; i < G * NV; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int j = 0; j < G; ++j) {
        const int n = v.grp_n[j];
        const float mx = gp.type[j].hp;
        for (int i = TID; i < n; i += blockDim.x) {
            const int id = v.grp_ids[j * v.cap + i];
            const uint32_t p = v.xy[id];
            atomicAdd(&hist[j * NV + ((int)(p >> 16) / sh) * VW + (int)(p & 0xFFFF) / sw], 1);
            info_out[id] = __float_as_uint(v.hp[id] / mx) | ((uint32_t)j << 31);
        }
    }
    __syncthreads();
    for (int i = TID; i < G * NV; i += blockDim.x) {
        const int n = v.grp_n[i / NV];
        mm_out[i] = n ? (float)hist[i] / (float)n : __uint_as_float(0xFFC00000u);
    }
}

// File env e's observation work items for the step of parity par: one item per obs_item_rows
// agents of each group (lane 0; one atomic per env).
__device__ __forceinline__ void obs_file_items(const RolloutArgs& ra, const EnvView& v, int G, int e, int par) {
    if (TID != 0 || !ra.obs_items) return;
    const int R = ra.obs_item_rows;
    int k = 0;
    for (int g = 0; g < G; ++g) k += (v.grp_n[g] + R - 1) / R;
    if (!k) return;
    const int base = atomicAdd(ra.obs_cnt + 2 * par, k);
    uint32_t* out = ra.obs_items + par * ra.obs_par_stride + base;
    for (int g = 0, j = 0; g < G; ++g)
        for (int c = 0; c * R < v.grp_n[g]; ++c) out[j++] = ((uint32_t)e << 12) | ((uint32_t)g << 10) | (uint32_t)c;
}

__global__ void __launch_bounds__(256) k_obs_prep(const GameParams* __restrict__ gp, State s, RolloutArgs ra, int par) {
    __shared__ int hist[BattleShape::G * BattleShape::VW * BattleShape::VH];
    constexpr int NV = BattleShape::VW * BattleShape::VH;
    const int e = blockIdx.x;
    const EnvView v = global_view(s, e, gp->n_groups);
    obs_prep_env(*gp, v, ra.obs_mm + (size_t)e * BattleShape::G * NV, ra.obs_info + (size_t)e * s.cap, hist);
    obs_file_items(ra, v, gp->n_groups, e, par);
}

// get_observation of every group of the large envs as a stream of work items (obs_item_rows agents
// of one group of one env each), taken by persistent workgroups from the list the previous step
// filed, so the launch stays balanced whatever the spread of group sizes.  The shared inputs
// (minimap, per-id info) come from obs_prep_env; the cells and the info words are read from HBM
// kObsPf 64-cell blocks at a time.  Workgroup 0 clears the other parity's counters for the next
// step's filing (the previous k_rollout_big has finished with them).
__global__ void __launch_bounds__(256) k_observe_items(const GameParams* __restrict__ gpp, State s, RolloutArgs ra,
                                                       int par) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int item;
    constexpr int NV = BattleShape::VW * BattleShape::VH, NC = BattleShape::NC, F = BattleShape::F;
    const GameParams& gp = *gpp;
    const int G = BattleShape::G, R = ra.obs_item_rows, W = gp.W, H = gp.H;
    const int lane = TID & 63, wid = TID >> 6, nw = blockDim.x >> 6;
    size_t off = 0;
    ObsSmem sm = carve_obs(smem, gp, 0, 0, R, obs_stage_floats(gp, 0, true, blockDim.x), true, off);
    obs_prologue(gp, sm, 0);
    if (blockIdx.x == 0 && TID < 2) ra.obs_cnt[2 * (par ^ 1) + TID] = 0;
    const int n_items = ra.obs_cnt[2 * par];
    float* st = sm.stage + wid * kWaveStageFloats;
    while (true) {
        if (TID == 0) {
            const int i = atomicAdd(ra.obs_cnt + 2 * par + 1, 1);
            item = i < n_items ? (int)ra.obs_items[par * ra.obs_par_stride + i] : -1;
        }
        __syncthreads();
        const int it = item;
        if (it < 0) break;
        const int e = it >> 12, g = (it >> 10) & 3, a0 = (it & 1023) * R;
        const EnvView v = global_view(s, e, G);
        const int na = min(R, v.grp_n[g] - a0);
        const float* mmg = ra.obs_mm + (size_t)e * G * NV;
        for (int i = TID; i < G * NV; i += blockDim.x) sm.mm[i] = mmg[i];
        EnvView vc = v;
        vc.grp_ids = v.grp_ids + a0;
        obs_agent_records(gp, vc, sm, g, na);
        __syncthreads();
        const TypeParams& T = gp.type[g];
        float* ov = ra.view[g] + ((size_t)e * ra.rowcap + a0) * (NV * NC);
        float* of = ra.feat[g] + ((size_t)e * ra.rowcap + a0) * F;
        const float* mm_own = sm.mm + g * NV;
        const float* mm_en = sm.mm + (g ^ 1) * NV;
        g_u16* cells = (g_u16*)v.cells;
        g_cu32* info = (g_cu32*)(ra.obs_info + (size_t)e * s.cap);
        const int ncell = na * NV;
        for (int base = wid * kObsPf * kWaveCells; base < ncell; base += nw * kObsPf * kWaveCells) {
            CellPre p[kObsPf];
            uint32_t cv[kObsPf], inf[kObsPf];
#pragma unroll
            for (int d = 0; d < kObsPf; ++d)
                p[d] = obs_cell_pre(sm, mm_own, mm_en, W, H, base + d * kWaveCells + lane, ncell);
#pragma unroll
            for (int d = 0; d < kObsPf; ++d) cv[d] = cells[p[d].idx];
#pragma unroll
            for (int d = 0; d < kObsPf; ++d) inf[d] = info[(p[d].ok && cv[d] < kCellFood) ? cv[d] : 0u];
#pragma unroll
            for (int d = 0; d < kObsPf; ++d) {
                const int b = base + d * kWaveCells;
                if (b >= ncell) break;
                obs_stage_cell(st, lane, obs_cell_post_g(p[d], cv[d], inf[d], g));
                wave_sync_lds();
                obs_flush(ov + (size_t)b * NC, st, lane, min(kWaveCells, ncell - b));
                wave_sync_lds();
            }
        }
        // features (GridWorld.cc:411-421)
        const int emb = gp.emb, nact = T.n_action;
        for (int q = TID; q < na * F; q += blockDim.x) {
            const int a = q / F, f = q - a * F;
            const int id = vc.grp_ids[g * v.cap + a];
            float val = 0.0f;
            if (f < emb) val = (float)((id >> f) & 1);
            if (f == emb + v.last_act[id]) val = 1.0f;
            if (f == emb + nact) val = v.last_r[id];
            const uint32_t pos = v.xy[id];
            if (f == emb + nact + 1) val = (float)(int)(pos & 0xFFFF) / (float)W;
            if (f == emb + nact + 2) val = (float)(int)(pos >> 16) / (float)H;
            __builtin_nontemporal_store(val, of + q);
        }
        __syncthreads();                               // LDS (records, minimap, item) is reused
    }
}

// GridWorld::step for one env per workgroup, in place in HBM (the per-call path's large envs).
__global__ void __launch_bounds__(kBigThreads) k_step_big(const GameParams* __restrict__ gpp, State s) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const GameParams& gp = *gpp;
    const int e = blockIdx.x;
    const BigLayout L = big_layout(gp, s.cap, s.acap, false);
    StepSmem& sm = *reinterpret_cast<StepSmem*>(smem + L.sm);
    const BigScratch bs = carve_big(smem + L.big, s.acap, s.cap);
    EnvView v = global_view(s, e, gp.n_groups);
    uint32_t rng = s.rng[e];
    int done = 0;
    load_serial_types(gp, sm);
    step_env_core<false, false, true>(gp, s, v, s.atk + (size_t)e * s.acap, s.n_atk[e], s.mov + (size_t)e * s.acap,
                                      s.n_mov[e], reinterpret_cast<uint32_t*>(smem + L.sorted), rng, sm, done, false,
                                      ParScratch{}, s.id_counter[e], nullptr, 0, &bs);
    if (TID == 0) {
        s.rng[e] = rng;
        s.n_atk[e] = 0;
        s.n_mov[e] = 0;
        s.done[e] = done;
    }
}

// One training-loop step after get_observation (k_observe, per group) for one env per
// workgroup: the rush policy + mean action, set_action, step, get_reward, clear_dead, and the
// episode restart from the reset image -- what agent_phase and the tail of k_rollout do, in HBM.
__global__ void __launch_bounds__(kBigRolloutThreads) k_rollout_big(const GameParams* __restrict__ gpp,
                                                             const RolloutCtx* __restrict__ ctx, uint32_t step_index) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int misc[4];                       // 0 n_atk, 1 n_mov, 2 episode end
    const GameParams& gp = *gpp;
    const State& s = ctx->s;
    const RolloutArgs& ra = ctx->ra;
    const int e = blockIdx.x, G = gp.n_groups, cap = s.cap, acap = s.acap;
    const BigLayout L = big_layout(gp, cap, acap, true);
    StepSmem& sm = *reinterpret_cast<StepSmem*>(smem + L.sm);
    uint32_t* atk = s.atk + (size_t)e * acap;
    uint32_t* mov = s.mov + (size_t)e * acap;
    uint32_t* sorted = ra.big_sort + (size_t)e * acap;
    int* ahist = reinterpret_cast<int*>(smem + L.ahist);
    float* red = reinterpret_cast<float*>(smem + L.red);
    BigScratch bs = carve_big(smem + L.big, acap, cap);
#ifdef MFX_STAMPS
    bs.srow = ra.env_base + e;
#endif
    MFX_BSTAMP(bs.srow, 0);
    EnvView v = global_view(s, e, G);
    load_serial_types(gp, sm);
    if (TID == 0) { misc[0] = 0; misc[1] = 0; }
    int ntot = 0;
    for (int g = 0; g < G; ++g) ntot += v.grp_n[g];
    // ---------------- policy + mean action (former_act_prob)
    // meta and positions of every id staged in LDS (the step scratch is free until the attacks): the
    // policy's and set_action's dependent lookups become LDS reads; the cells stay in HBM
    EnvView vp = v;                        // (big_region_bytes holds cap * (5 + 2 * kMaxGroups) bytes)
    {
        const int idc = s.id_counter[e];
        uint32_t* xy_l = reinterpret_cast<uint32_t*>(bs.base);
        uint8_t* meta_l = reinterpret_cast<uint8_t*>(bs.base + (size_t)cap * 4);
        for (int i = TID; i < idc; i += blockDim.x) { xy_l[i] = v.xy[i]; meta_l[i] = v.meta[i]; }
        vp.xy = xy_l; vp.meta = meta_l;
#ifndef MFX_BIG_NO_IDS_STAGE
        uint16_t* ids_l = reinterpret_cast<uint16_t*>(bs.base + (size_t)cap * 5);
        for (int g = 0; g < G; ++g)
            for (int i = TID; i < v.grp_n[g]; i += blockDim.x) ids_l[g * cap + i] = v.grp_ids[g * cap + i];
        vp.grp_ids = ids_l;
#endif
    }
    for (int i = TID; i < G * 64; i += blockDim.x) ahist[i] = 0;
    __syncthreads();
    const uint32_t ekey = ra.policy_seed ^ mix32(step_index * 0x9E3779B9u + (uint32_t)(ra.env_base + e) * 0x632BE5ABu);
    // two agents per lane per pass: both policies' HBM loads (position, 8 attack cells, their
    // occupants) are in flight together, the stores come after
    for (int t = TID; t < ntot; t += 2 * blockDim.x) {
        int a[2], gg[2], ii[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            int g = 0, i = t + j * (int)blockDim.x;
            a[j] = -1; gg[j] = 0; ii[j] = i;
            if (i >= ntot) continue;
            while (i >= v.grp_n[g]) { i -= v.grp_n[g]; ++g; }
            const int id = vp.grp_ids[g * cap + i];
            const uint32_t key = ekey ^ mix32((uint32_t)id * 0x85EBCA77u + (uint32_t)g);
            a[j] = rush_action(gp, sm.tt[g], vp, g, id, key, ra.eps);
            gg[j] = g; ii[j] = i;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (a[j] < 0) continue;
            ra.actions[((size_t)e * G + gg[j]) * ra.rowcap + ii[j]] = a[j];
            atomicAdd(&ahist[gg[j] * 64 + a[j]], 1);
        }
    }
    __syncthreads();
    for (int t = TID; t < G * 64; t += blockDim.x) {
        const int g = t >> 6, k = t & 63, na = sm.tt[g].n_action, n = v.grp_n[g];
        if (k < na)   // empty group: np.mean of nothing is NaN
            ra.mean_act[((size_t)e * G + g) * na + k] =
                n ? (double)ahist[t] / (double)n : __longlong_as_double(0x7FF8000000000000ll);
    }
    MFX_BSTAMP(bs.srow, 1);
    // ---------------- set_action (group order) and step
    for (int g = 0; g < G; ++g)            // vp: positions from LDS, last_act written to HBM
        set_action_group<false>(gp, s, vp, g, ra.actions + ((size_t)e * G + g) * ra.rowcap, atk, misc[0], mov, misc[1],
                                sm.wave_tot, acap);
    MFX_BSTAMP(bs.srow, 2);
    uint32_t rng = s.rng[e];
    int done = 0;
    step_env_core<false, false, true>(gp, s, v, atk, misc[0], mov, misc[1], sorted, rng, sm, done, false, ParScratch{},
                                      s.id_counter[e], nullptr, 0, &bs);
    MFX_BSTAMP(bs.srow, 10);
    // ---------------- get_reward, episode return, kills
    float kills = 0.0f, ret[kMaxGroups];
    for (int g = 0; g < G; ++g) {
        const int n = v.grp_n[g];
        float part = 0.0f;
        for (int i = TID; i < n; i += blockDim.x) {
            const float r = v.next_r[v.grp_ids[g * cap + i]] + v.grp_reward[g];
            ra.rewards[((size_t)e * G + g) * ra.rowcap + i] = r;
            part += r;
        }
        ret[g] = block_sum_waves(part, red);
        kills += (float)v.grp_dead[g];
    }
    MFX_BSTAMP(bs.srow, 11);
    // ---------------- clear_dead
    clear_dead_env<false>(gp, v, sm.wave_tot);
    MFX_BSTAMP(bs.srow, 12);
    // ---------------- episode end -> reset image (env.reset + add_agents of the template)
    if (TID == 0) {
        double* st = ra.stats + (size_t)e * 4;
        st[3] += kills;
        float* er = ra.ep_return + (size_t)e * G;
        for (int g = 0; g < G; ++g) er[g] += ret[g];
        int len = ra.ep_len[e] + 1;
        misc[2] = 0;
        if (done || len >= ra.max_steps) {
            st[0] += 1.0;
            st[1] += er[0];
            st[2] += G > 1 ? er[1] : 0.0f;
            for (int g = 0; g < G; ++g) er[g] = 0.0f;
            len = 0;
            misc[2] = 1;
        }
        ra.ep_len[e] = len;
        ra.agent_steps[e] += (unsigned long long)ntot;
        s.rng[e] = rng;
        s.n_atk[e] = 0;
        s.n_mov[e] = 0;
        s.done[e] = done;
    }
    __syncthreads();
    if (misc[2]) {
        const EnvView im = carve_env(reinterpret_cast<char*>(const_cast<uint4*>(ra.reset_image)), s.cells_n, cap, G);
        const int32_t* img_scal = reinterpret_cast<const int32_t*>(
            reinterpret_cast<const char*>(ra.reset_image) + env_image_bytes(s.cells_n, cap, G));
        const int idc = img_scal[4];
        for (int i = TID; i < s.cells_n; i += blockDim.x) v.cells[i] = im.cells[i];
        for (int i = TID; i < idc; i += blockDim.x) {
            v.xy[i] = im.xy[i]; v.hp[i] = im.hp[i]; v.next_r[i] = im.next_r[i]; v.last_r[i] = im.last_r[i];
            v.op_obj[i] = im.op_obj[i]; v.last_act[i] = im.last_act[i]; v.meta[i] = im.meta[i];
        }
        for (int g = 0; g < G; ++g)
            for (int i = TID; i < img_scal[g]; i += blockDim.x) v.grp_ids[g * cap + i] = im.grp_ids[g * cap + i];
        if (TID < G) { v.grp_n[TID] = img_scal[TID]; v.grp_dead[TID] = 0; v.grp_reward[TID] = 0.0f; }
        if (TID == 0) s.id_counter[e] = idc;
        __syncthreads();
    }
    MFX_BSTAMP(bs.srow, 13);
    // ---------------- the next observation's shared inputs
    if (ra.obs_mm) {
        constexpr int NV = BattleShape::VW * BattleShape::VH;
        obs_prep_env(gp, v, ra.obs_mm + (size_t)e * G * NV, ra.obs_info + (size_t)e * cap,
                     reinterpret_cast<int*>(smem + L.big));
        if (ra.obs_items) {
            __syncthreads();
            obs_file_items(ra, v, G, e, (int)((step_index + 1) & 1));
        }
    }
    MFX_BSTAMP(bs.srow, 14);
}

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
    const int chunk = 64;
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
    if (gp.dsl) k_step<true><<<s.E, 256, dyn, st>>>(d_gp, s, lds, d_sort_scratch);
    else k_step<false><<<s.E, 256, dyn, st>>>(d_gp, s, lds, d_sort_scratch);
    return hipGetLastError();
}

hipError_t launch_rollout_big(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                              uint32_t step_index, hipStream_t st) {
    const size_t smem = big_step_smem_bytes(gp, s.cap, s.acap, true);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    k_rollout_big<<<s.E, kBigRolloutThreads, smem, st>>>(d_gp, d_ctx, step_index);
    return hipGetLastError();
}

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
                          hipStream_t st) {
    const size_t smem = rollout_smem_bytes(gp, s.cells_n, s.cap, s.acap, rows);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    return with_rollout_kernel(gp, s, split != 0, [&](auto kern) {
        kern<<<grid, MFX_ROLLOUT_THREADS, smem, st>>>(d_gp, d_ctx, step_index, work_sel, qphase);
        return hipGetLastError();
    });
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
