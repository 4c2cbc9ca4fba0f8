// policy_gemm.h -- the MFMA building blocks shared by the policy forwards (policy_kernels.hip: the Q network of
// ValueNet, algo/base.py:123-183; acnet_kernels.hip: the actor-critic network of ActorCritic / MFAC,
// algo/ac.py:53-98, :219-276): f32-input MFMA v_mfma_f32_16x16x4_f32, and the transposed workgroup GEMM whose
// accumulator tiles feed the next layer's B operand in registers.
// A and B operands of v_mfma_f32_16x16x4_f32: lane l holds A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15];
// D: lane l holds D[(l >> 4) * 4 + r][l & 15], r = 0..3 (cdna_hip_programming.md, fragment layout).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfx {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void qwave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// One workgroup = 4 waves x 16 agents.  Every layer is computed TRANSPOSED, out^T [N_out x 16 agents] =
// W^T [N_out x K] . in^T [K x 16]: the weights are the A operand (rows = output units on the lane's column
// index), the layer input the B operand (agents on the lane's column index).  The accumulator tile then has
// the agents on its lanes and the output units in its registers, which is exactly the B operand the next
// layer needs -- "an accumulator tile as the next MFMA's operand" (cdna_hip_programming.md): the
// activations never leave the registers, with the k order inside each 16-row chunk permuted to match
// (k-step s of chunk t takes units 16 t + 4 h + s, lane group h supplying its register s).  The weights
// are staged per 16-row chunk in LDS (double buffered, the next chunk in flight in registers) and shared
// by the four waves; LDS holds nothing else.
constexpr int kQHeadWaves = 4, kQKC = 16;                // agents per wave = 16; weight rows per chunk
// A staged row holds lane c's MT weights (units 16 t + c, t < MT) at c * P + t: 16-B reads of consecutive t.
// P = MT rounded up to 4, + 4 from 8 on (a 16-lane read then spans every bank group twice at most).
__host__ __device__ constexpr int qhead_p(int mt) { return ((mt + 3) & ~3) + (mt >= 8 ? 4 : 0); }
constexpr int kQMaxMT = 16;                              // the widest layer: 256 output units
constexpr int kQBLd = 16 * qhead_p(kQMaxMT);             // the widest staged row (256 units: 320 floats)
constexpr size_t kQHeadSmem = (size_t)2 * kQKC * kQBLd * 4;

// threadIdx.x, opaque to loop-invariant code motion: in a persistent kernel's tile loop the compiler would otherwise
// hoist every chunk's lane-derived addresses out of the loop and spill them (k_acnet: 3.8 KB of scratch).
__device__ __forceinline__ int tid_x() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// acc[MT] = W^T . V over K (K a multiple of 4, rows of W past K read as zero).  W: [K][MT * 16] row-major.
// v_at(ch, s): this lane's B operand for k = 16 ch + 4 h + s (agent = lane & 15).  NCH > 0: the chunk loop
// is unrolled (K <= 16 NCH), so a v_at that indexes the previous layer's accumulators by ch stays in
// registers.  kZero false: accumulate onto acc (a layer whose K arrives in parts).  Uniform call sites
// (barriers inside).
template <int MT, int NCH = 0, bool kZero = true, class VF>
__device__ __forceinline__ void wg_gemm_t(const float* __restrict__ W, int K, VF v_at, float* bsm, f32x4* acc) {
    static_assert(MT >= 1 && MT <= kQMaxMT, "layer wider than the staged row");
    constexpr int N = MT * 16;                           // staged row width; 16 rows = MT floats per thread
    const int lane = threadIdx.x & 63, h = lane >> 4, c = lane & 15;
    const int nchunk = (K + kQKC - 1) / kQKC;
    float pre[MT];
    auto load = [&](int ch) {
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int q = threadIdx.x + j * 256, r = q / N, col = q - r * N, k = ch * kQKC + r;
            pre[j] = k < K ? W[(size_t)k * N + col] : 0.f;
        }
    };
    constexpr int P = qhead_p(MT);
    auto store = [&](float* dst) {
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int q = threadIdx.x + j * 256, r = q / N, col = q - r * N;
            dst[r * kQBLd + (col & 15) * P + (col >> 4)] = pre[j];
        }
    };
    // this lane's MT weights of k-row kr of the staged chunk cur
    auto read_row = [&](const float* cur, int kr, float* dst) {
        const float* src = cur + kr * kQBLd + c * P;
        if constexpr (MT % 4 == 0) {
#pragma unroll
            for (int t4 = 0; t4 < MT / 4; ++t4) {
                const float4 x = reinterpret_cast<const float4*>(src)[t4];
                dst[4 * t4] = x.x; dst[4 * t4 + 1] = x.y; dst[4 * t4 + 2] = x.z; dst[4 * t4 + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int t = 0; t < MT; ++t) dst[t] = src[t];
        }
    };
    if (kZero) {
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
    }
    load(0);
    store(bsm);
    __syncthreads();
    auto chunk = [&](int ch) {
        const float* cur = bsm + (ch & 1) * kQKC * kQBLd;
        if (ch + 1 < nchunk) load(ch + 1);               // in flight during this chunk's MFMAs
        // k-step s + 1's MT weights are read from LDS while k-step s's MT MFMAs issue (the compiler alone
        // waits on each read right before its MFMA)
        float av[MT], an[MT];
        read_row(cur, 4 * h, av);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float v = v_at(ch, s);
            if (s + 1 < 4) read_row(cur, 4 * h + s + 1, an);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[t] = mfma4(av[t], v, acc[t]);
#pragma unroll
            for (int t = 0; t < MT; ++t) av[t] = an[t];
        }
        if (ch + 1 < nchunk) store(bsm + ((ch + 1) & 1) * kQKC * kQBLd);
        __syncthreads();
    };
    if constexpr (NCH > 0) {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
            if (ch < nchunk) chunk(ch);
    } else {
        for (int ch = 0; ch < nchunk; ++ch) chunk(ch);
    }
}

// ---- the same transposed GEMM over a weight IMAGE, staged by direct-to-LDS loads (k_acnet, round 5)
// wg_gemm_t stages each 16-row chunk through registers (a global load per weight, then LDS stores of the permuted
// row): 16 + MT registers per lane, and at 256 VGPRs the compiler reused a load's destination register and waited for
// the whole prefetch before the chunk's MFMAs.  Here the weights are stored once, at set_weights time, in the exact
// LDS order (the image), and each chunk is copied global -> LDS by global_load_lds_dwordx4 (16 B per lane, no
// register, no LDS store instruction), issued a chunk ahead and waited for only at the chunk's end barrier.
// Image of a [K][16 MT] matrix: per 16-row chunk (rows past K zero), 16 rows of img_row(MT) floats; in a row, lane
// c's MT weights (units 16 t + c) are contiguous, float4 t4 = t / 4 at the swizzled slot (t4 + c G / 16) mod G
// (G = MT / 4): the 16 lanes of a ds_read_b128 lane group then touch 16 distinct bank groups without the padding of
// wg_gemm_t's rows.  MT < 4: weight t of lane c at c * 4 + t.
__host__ __device__ constexpr int img_row(int mt) { return mt % 4 == 0 ? 16 * mt : 64; }
__host__ __device__ constexpr size_t img_floats(int K, int mt) { return (size_t)((K + 15) / 16) * 16 * img_row(mt); }
__host__ __device__ inline int img_pos(int mt, int c, int t) {
    if (mt % 4) return c * 4 + t;
    const int G = mt / 4;
    return c * mt + (((t >> 2) + c * G / 16) % G) * 4 + (t & 3);
}
constexpr int kImgBuf = 16 * 256;                        // floats of one staged chunk of the widest layer (16 KB)
constexpr size_t kImgSmem = (size_t)2 * kImgBuf * 4;     // the two chunk buffers

// A staged chunk holds SUB = 16 KB / (16 row floats) consecutive 16-row image chunks (the narrow layers take 64 rows
// per barrier).  pre(ch): called once per staged chunk right after the next chunk's weights were issued (k_acnet:
// the view rows two chunks ahead, direct to LDS); kVmTail: the vector-memory instructions it issues, which stay in
// flight across the chunk-end wait (exactly that many per chunk).
struct NoPre { __device__ void operator()(int) const {} };
template <int MT, int NCH = 0, bool kZero = true, int kVmTail = 0, class VF, class PF = NoPre>
__device__ __forceinline__ void wg_gemm_i(const float* __restrict__ img, int K, VF v_at, float* bsm, f32x4* acc,
                                          PF pre = PF()) {
    static_assert(MT >= 1 && MT <= kQMaxMT, "layer wider than the staged row");
    static_assert(kVmTail == 0 || kVmTail == 4, "chunk-end wait");
    constexpr int RW = img_row(MT), SUB = kImgBuf / (16 * RW), CF4 = 16 * RW * SUB / 4;   // float4 per staged chunk
    static_assert(CF4 % 256 == 0 && CF4 * 4 <= kImgBuf, "chunk image");
    static_assert(kVmTail == 0 || SUB == 1, "a view prefetch per staged chunk");
    const int tid = tid_x(), lane = tid & 63, h = lane >> 4, c = lane & 15, wid = tid >> 6;
    const int n16 = (K + kQKC - 1) / kQKC, nchunk = (n16 + SUB - 1) / SUB;
    auto issue = [&](int ch) {                           // staged chunk ch -> buffer ch & 1 (async)
        float* dst = bsm + (ch & 1) * kImgBuf;
        const float* src = img + (size_t)ch * CF4 * 4;
        const int lim = (n16 - ch * SUB) * 16 * RW / 4;  // (the last chunk: only the 16-row chunks the image has)
#pragma unroll
        for (int q = 0; q < CF4; q += 256) {
            const int i = q + tid;
            __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)(i < lim ? i : 0) * 4),
                                             (__attribute__((address_space(3))) void*)(dst + (q + wid * 64) * 4), 16,
                                             0, 0);
        }
    };
    constexpr int G = MT / 4;
    const int cb = c * (MT % 4 ? 4 : MT), sw = c * G / 16;
    auto read_row = [&](const float* cur, int kr, float* dst) {
        const float* src = cur + kr * RW + cb;
        if constexpr (MT % 4 == 0) {
#pragma unroll
            for (int t4 = 0; t4 < G; ++t4) {
                const float4 x = reinterpret_cast<const float4*>(src)[(t4 + sw) % G];
                dst[4 * t4] = x.x; dst[4 * t4 + 1] = x.y; dst[4 * t4 + 2] = x.z; dst[4 * t4 + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int t = 0; t < MT; ++t) dst[t] = src[t];
        }
    };
    if (kZero) {
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
    }
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    auto chunk = [&](int ch) {
        const float* buf = bsm + (ch & 1) * kImgBuf;
        if (ch + 1 < nchunk) issue(ch + 1);              // lands during this chunk's MFMAs
        pre(ch);
#pragma unroll
        for (int sub = 0; sub < SUB; ++sub) {
            const int c16 = ch * SUB + sub;
            if (SUB > 1 && c16 >= n16) break;
            const float* cur = buf + sub * 16 * RW;
            float av[MT], an[MT];
            read_row(cur, 4 * h, av);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float v = v_at(c16, s);
                if (s + 1 < 4) read_row(cur, 4 * h + s + 1, an);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < MT; ++t) acc[t] = mfma4(av[t], v, acc[t]);
#pragma unroll
                for (int t = 0; t < MT; ++t) av[t] = an[t];
            }
        }
        __builtin_amdgcn_sched_barrier(0);               // (the MFMAs stay ahead of the wait)
        // the next chunk has landed in LDS (every wave's part); v_at's own loads may stay in flight
        // then a bare barrier: __syncthreads()' release fence would make the compiler drain every load first, the
        // view rows pre() keeps two chunks ahead included.  (The barrier inside the asm: the compiler may not move
        // an LDS access across it.)
        if constexpr (kVmTail == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    if constexpr (NCH > 0) {
#pragma unroll
        for (int ch = 0; ch < (NCH + SUB - 1) / SUB; ++ch)
            if (ch < nchunk) chunk(ch);
    } else {
        for (int ch = 0; ch < nchunk; ++ch) chunk(ch);
    }
}

// acc[t] = bias[16 t + 4 h .. + 3] (a layer's accumulators start at its bias: one 16-B load per tile, issued
// together, instead of one dependent load per unit after the GEMM)
__device__ __forceinline__ void bias_init(f32x4* acc, const float* bias, int h) {
    const float4* b = reinterpret_cast<const float4*>(bias) + h;
    float4 v[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) v[t] = b[4 * t];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = {v[t].x, v[t].y, v[t].z, v[t].w};
}

// The image (img_row / img_pos layout above) of a [K][N] row-major weight matrix into dst (img_floats(K, N / 16)
// floats): one thread per image float, zero past K and in the MT < 4 padding (policy_kernels.hip k_weight_image).
hipError_t launch_weight_image(const float* src, int K, int N, float* dst, hipStream_t st);

// relu(acc + bias) of unit 16 t + 4 h + s: the B operand of the next layer's chunk t, k-step s.
__device__ __forceinline__ float relu_unit(const f32x4* acc, const float* __restrict__ bias, int t, int s) {
    const int h = (tid_x() & 63) >> 4;
    return fmaxf(acc[t][s] + bias[16 * t + 4 * h + s], 0.f);
}

// Compact agent i -> (view row, action slot, prob row): rows == null: (i, i, i); else row = rows[i]
// = e * rowcap + j of a rollout buffer, action slot e * act_env + act_off + j, prob row e.
struct QRowMap {
    const int32_t* rows;
    int rowcap, act_env, act_off;
};

// The compact row list of one group of a rollout batch (policy_kernels.hip k_qnet_rows): rows e * rowcap + j for
// j < min(n_e, rowcap) in env order, and their count in total[0] -- on the device, nothing read back.  total: 1 +
// ceil(E / 64) ints (the chunks' totals follow the count).
hipError_t launch_rollout_rows(const int32_t* counts, int E, int G, int g, int rowcap, int32_t* rows, int32_t* total,
                               hipStream_t st);

}  // namespace mfx
