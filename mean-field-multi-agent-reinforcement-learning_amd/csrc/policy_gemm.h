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

// relu(acc + bias) of unit 16 t + 4 h + s: the B operand of the next layer's chunk t, k-step s.
__device__ __forceinline__ float relu_unit(const f32x4* acc, const float* __restrict__ bias, int t, int s) {
    const int h = (threadIdx.x & 63) >> 4;
    return fmaxf(acc[t][s] + bias[16 * t + 4 * h + s], 0.f);
}

// Compact agent i -> (view row, action slot, prob row): rows == null: (i, i, i); else row = rows[i]
// = e * rowcap + j of a rollout buffer, action slot e * act_env + act_off + j, prob row e.
struct QRowMap {
    const int32_t* rows;
    int rowcap, act_env, act_off;
};

// The compact row list of one group of a rollout batch (policy_kernels.hip k_qnet_rows): rows e * rowcap + j for
// j < min(n_e, rowcap) in env order, and their count in *total -- on the device, nothing read back.
hipError_t launch_rollout_rows(const int32_t* counts, int E, int G, int g, int rowcap, int32_t* rows, int32_t* total,
                               hipStream_t st);

}  // namespace mfx
