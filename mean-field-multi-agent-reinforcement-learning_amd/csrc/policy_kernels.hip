// policy_kernels.hip -- the reference's Q network (ValueNet._construct_net, algo/base.py:123-183) and its
// greedy act (ValueNet.act, :228-254), forward only, hand-written for gfx950 on the f32-input MFMA
// v_mfma_f32_16x16x4_f32 (exact f32: each product rounded once into an f32 accumulator, the rate of the
// f32 VALU -- MI355X_MICROARCH.md; there is no xf32 / TF32 on gfx950).  The network, per agent:
//
//   view [13][13][7] --Conv1 3x3x32 valid, relu--> [11][11][32] --Conv2 3x3x32 valid, relu--> [9][9][32]
//   flatten (TF's NHWC order, 2,592) --Dense-Obs 256, relu--> h_obs
//   feature [F] --Dense-Emb 32, relu--> h_emb
//   (mean field) prob [A] --Prob-Emb 64, relu--> --Dense-Act-Prob 32, relu--> h_prob
//   concat(h_obs, h_emb[, h_prob]) --Dense2 128, relu--> --Dense-Out 64, relu--> --Q-Value A--> q
//   act = argmax q   (the reference takes argmax of softmax(q / T), the same index up to float ties)
//
// 3.4 MFLOP per agent (conv2 44 %, Dense-Obs 39 %, conv1 14 %): compute-bound at the f32 matrix rate
// (157 TF/s -> ~4.6e7 agents/s for the whole chip).  Two kernels:
//   k_qnet_conv  one wave per agent: the view staged in LDS, Conv1 as an implicit GEMM over 121
//                positions x 32 channels x K 63 (padded to 64), its output kept in LDS, Conv2 as an
//                implicit GEMM over 80 positions x 32 x K 288 (16-B operand reads, k permuted inside each
//                (ky, kx) block) and its 81st position on the VALU; the 2,592 activations to HBM (10 KB/agent)
//   k_qnet_head  four waves x 16 agents per workgroup: every layer transposed (weights as the A operand),
//                so each layer's accumulators are the next layer's B operand in registers; the weight
//                chunks staged in LDS and shared by the four waves; the Q values and the argmax
// A and B operands of v_mfma_f32_16x16x4_f32: lane l holds A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15];
// D: lane l holds D[(l >> 4) * 4 + r][l & 15], r = 0..3 (cdna_hip_programming.md, fragment layout).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>

#include <algorithm>

#include "mfx_common.h"
#include "policy_gemm.h"
#include "../../include/magent_amd.h"

namespace mfx {


constexpr int kQVH = 13, kQVW = 13, kQNC = 7;           // Battle view (13 x 13 x 7)
constexpr int kQViewF = kQVH * kQVW * kQNC;             // 1,183
constexpr int kQC1 = 11, kQC2 = 9, kQCh = 32;            // conv output sides, channels
constexpr int kQK1 = 64;                                 // conv1 K: 3 * 3 * 7 = 63, padded
constexpr int kQK2 = 3 * 3 * kQCh;                       // conv2 K: 288
constexpr int kQFlat = kQC2 * kQC2 * kQCh;               // 2,592
constexpr int kQHObs = 256, kQHEmb = 32, kQHP1 = 64, kQHP2 = 32, kQH2 = 128, kQHOut = 64, kQMaxA = 32;

// Device view of one packed weight blob (layout: QNetLayout; every matrix [K][N] row-major, K padded to a
// multiple of 4 with zero rows, N of the Q layer padded to 32 with zero columns).
struct QNetDev {
    const float *w1, *b1, *w2, *b2, *wd, *bd, *we, *be, *wp1, *bp1, *wp2, *bp2, *w2d, *b2d, *wo, *bo, *wq, *bq;
    int F, Fp, A, Ap, use_mf, Kc;   // Kc: Dense2 input width (288, or 320 with mean field)
    const float* wd_img;            // Dense-Obs's weight image (policy_gemm.h wg_gemm_i), made by set_weights
};

// One weight image: thread per image float -> the source weight (zero past K and in the MT < 4 padding).
__global__ void __launch_bounds__(256) k_weight_image(const float* __restrict__ src, int K, int N, float* __restrict__ dst,
                                                      size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int mt = N / 16, rw = img_row(mt);
    const int pos = (int)(i % rw), r = (int)((i / rw) % 16);
    const size_t ch = i / ((size_t)16 * rw);
    int c, t;
    if (mt % 4) {
        c = pos / 4;
        t = pos % 4;
    } else {
        const int G = mt / 4;
        c = pos / mt;
        const int rem = pos % mt, slot = rem / 4;
        t = 4 * ((slot - c * G / 16 + G) % G) + rem % 4;
    }
    const size_t k = ch * 16 + r;
    dst[i] = (t < mt && k < (size_t)K) ? src[k * N + 16 * t + c] : 0.f;
}

hipError_t launch_weight_image(const float* src, int K, int N, float* dst, hipStream_t st) {
    if (K < 1 || N < 16 || N % 16 || N / 16 > kQMaxMT) return hipErrorInvalidValue;
    const size_t n = img_floats(K, N / 16);
    k_weight_image<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(src, K, N, dst, n);
    return hipGetLastError();
}


// ------------------------------------------------------------------------------------------ conv
// LDS: w1 [64][32] and Conv2's weights transposed, w2t [32][292] (shared), per wave the view [1,184] and
// conv1's output [121][36] (134 KB per 4-wave workgroup).
constexpr int kQConvWaves = 4;
// Conv2's weights transposed, w2t [32 channels][288 + 4] (k contiguous per channel), and conv1's output rows
// at a 36-float stride: both 16-B aligned, so a lane reads its 8 consecutive k of one (ky, kx) block with two
// ds_read_b128 (the k order inside a block is permuted to make them consecutive: see Conv2 below).
constexpr int kQW2tLd = kQK2 + 4, kQC1Ld = 36;
constexpr int kQViewLds = 1184, kQC1Lds = kQC1 * kQC1 * kQC1Ld;
constexpr size_t kQConvSmem = (size_t)(kQK1 * kQCh + kQCh * kQW2tLd + kQConvWaves * (kQViewLds + kQC1Lds)) * 4;

// Offset of im2col column k (ky, kx, ci) in the staged 13 x 13 x 7 view; the pad column 63 reads
// element 0 against a zero weight row.
__device__ __forceinline__ int conv1_koff(int k) {
    if (k >= 63) return 0;
    const int ky = k / 21, kx = (k % 21) / 7, ci = k % 7;
    return (ky * kQVW + kx) * kQNC + ci;
}

// Conv1 + Conv2 (implicit GEMMs from LDS) with TWO waves per agent (8-wave workgroups, 4 agents per pass, one
// workgroup per CU): the pair shares its agent's staged view and conv1 output in LDS -- so the 134 KB above hold 4
// agents for 8 waves, two per SIMD (round 5; the round-3/4 one-wave-per-agent k_qnet_conv ran one) -- and splits the
// work: conv1's position tiles 0-3 / 4-7, conv2's output channels
// 0-15 / 16-31 (5 position tiles each, its position 80 on the VALU), the view's 64-float chunks even / odd.  Two
// workgroup barriers per pass: after the view is staged, after conv1.  <= 256 VGPRs (launch bounds 512, 1).
constexpr int kQConv2Agents = 4;
__global__ void __launch_bounds__(512, 1) k_qnet_conv2(QNetDev p, const float* __restrict__ view, size_t view_ld,
                                                       const int32_t* __restrict__ rows, int n, float* __restrict__ out,
                                                       const int32_t* __restrict__ d_n, int n_off) {
    extern __shared__ __attribute__((aligned(16))) float qsm[];
    if (d_n) n = min(max(*d_n - n_off, 0), n);
    if (n <= 0) return;
    float* w1 = qsm;
    float* w2 = w1 + kQK1 * kQCh;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 4, c = lane & 15;
    const int slot = wid >> 1, half = wid & 1;          // the agent slot of the pass, this wave's half of its work
    float* vs = w2 + kQCh * kQW2tLd + slot * (kQViewLds + kQC1Lds);
    float* c1 = vs + kQViewLds;
    for (int i = threadIdx.x; i < kQK1 * kQCh; i += blockDim.x) w1[i] = p.w1[i];
    for (int i = threadIdx.x; i < kQK2 * kQCh; i += blockDim.x) w2[(i % kQCh) * kQW2tLd + i / kQCh] = p.w2[i];
    __syncthreads();
    float b1r[16][2];
    int koff[16];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
        b1r[kk][0] = w1[(kk * 4 + h) * kQCh + c];
        b1r[kk][1] = w1[(kk * 4 + h) * kQCh + 16 + c];
        koff[kk] = conv1_koff(kk * 4 + h);
    }
    const float bias1a = p.b1[c], bias1b = p.b1[16 + c], bias2 = p.b2[16 * half + c];
    // this wave's 64-float chunks of the next pass's view (chunks half, half + 2, ...: 10 or 9 of 19), in flight
    constexpr int kVR2 = ((kQViewF + 63) / 64 + 1) / 2;
    float vr[kVR2];
    auto fetch = [&](int i) {
        if (i >= n) return;
        const float* src = view + (size_t)(rows ? rows[i] : i) * view_ld;
#pragma unroll
        for (int j = 0; j < kVR2; ++j) {
            const int q = lane + 64 * (2 * j + half);
            vr[j] = q < kQViewF ? src[q] : 0.f;
        }
    };
    const int step = gridDim.x * kQConv2Agents;
    int i = blockIdx.x * kQConv2Agents + slot;
    fetch(i);
    // every wave runs every pass (the barriers), computing only for an agent below n
    for (int i0 = blockIdx.x * kQConv2Agents; i0 < n; i0 += step, i += step) {
        const bool live = i < n;
#pragma unroll
        for (int j = 0; j < kVR2; ++j) {
            const int q = lane + 64 * (2 * j + half);
            if (q < kQViewF) vs[q] = vr[j];
        }
        __syncthreads();                                 // the pair's view is whole
        fetch(i + step);
        // ---- Conv1: this wave's 4 position tiles (tiles 4 half .. 4 half + 3; 121 of 128 rows) x 2 channel tiles
        if (live) {
            for (int m = 0; m < 4; ++m) {
                const int mt = 4 * half + m;
                const int pa = min(mt * 16 + c, kQC1 * kQC1 - 1);
                const int vb = ((pa / kQC1) * kQVW + pa % kQC1) * kQNC;
                f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {
                    const float a = vs[vb + koff[kk]];
                    d0 = mfma4(a, b1r[kk][0], d0);
                    d1 = mfma4(a, b1r[kk][1], d1);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int pos = mt * 16 + h * 4 + r;
                    if (pos < kQC1 * kQC1) {
                        c1[pos * kQC1Ld + c] = fmaxf(d0[r] + bias1a, 0.f);
                        c1[pos * kQC1Ld + 16 + c] = fmaxf(d1[r] + bias1b, 0.f);
                    }
                }
            }
        }
        __syncthreads();                                 // the pair's conv1 output is whole
        if (!live) continue;
        // ---- Conv2: output channels 16 half .. + 15 over positions 0-79 (5 tiles), K 288 = 9 (ky, kx) blocks x 32 ci
        // (lane group h takes ci = 8 h + j of each block: 8 consecutive floats of both operands, as k_qnet_conv)
        constexpr int kMT2 = 5;
        f32x4 acc[kMT2];
        int cb[kMT2];
#pragma unroll
        for (int mt = 0; mt < kMT2; ++mt) {
            const int pa = mt * 16 + c;
            cb[mt] = ((pa / kQC2) * kQC1 + pa % kQC2) * kQC1Ld + 8 * h;
            acc[mt] = {0.f, 0.f, 0.f, 0.f};
        }
        typedef float f32x8 __attribute__((ext_vector_type(8)));
        f32x8 p0[kMT2], q0, p1[kMT2], q1;
        const float* w2row = w2 + (16 * half + c) * kQW2tLd + 8 * h;
        auto conv2_part = [&](int b, f32x8* a, f32x8& w, int part) {
            const int ky = b / 3, kx = b % 3;
            const int so = (ky * kQC1 + kx) * kQC1Ld;
            if (part == 0) {
                w = *reinterpret_cast<const f32x8*>(w2row + b * 32);
#pragma unroll
                for (int mt = 0; mt < 3; ++mt) a[mt] = *reinterpret_cast<const f32x8*>(c1 + cb[mt] + so);
            } else {
#pragma unroll
                for (int mt = 3; mt < kMT2; ++mt) a[mt] = *reinterpret_cast<const f32x8*>(c1 + cb[mt] + so);
            }
        };
        auto conv2_half = [&](const f32x8* a, const f32x8& w, int j0) {
#pragma unroll
            for (int j = j0; j < j0 + 4; ++j)
#pragma unroll
                for (int mt = 0; mt < kMT2; ++mt) acc[mt] = mfma4(a[mt][j], w[j], acc[mt]);
        };
        auto conv2_step = [&](const f32x8* a, const f32x8& w, f32x8* na, f32x8& nw, int nb) {
            if (nb >= 0) conv2_part(nb, na, nw, 0);
            __builtin_amdgcn_sched_barrier(0);
            conv2_half(a, w, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (nb >= 0) conv2_part(nb, na, nw, 1);
            __builtin_amdgcn_sched_barrier(0);
            conv2_half(a, w, 4);
            __builtin_amdgcn_sched_barrier(0);
        };
        conv2_part(0, p0, q0, 0);
        conv2_part(0, p0, q0, 1);
#pragma unroll 1
        for (int b = 0; b < 8; b += 2) {                 // ping-pong: block b in (p0, q0), b + 1 in (p1, q1)
            conv2_step(p0, q0, p1, q1, b + 1);
            conv2_step(p1, q1, p0, q0, b + 2);
        }
        conv2_step(p0, q0, p1, q1, -1);                  // block 8
        float* o = out + (size_t)i * kQFlat + 16 * half;
#pragma unroll
        for (int mt = 0; mt < kMT2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[(mt * 16 + h * 4 + r) * kQCh + c] = fmaxf(acc[mt][r] + bias2, 0.f);
        {
            // position 80 (row 8, column 8) on the VALU: lane l sums channel 16 half + l % 16 over quarter l / 16 of
            // the 288 k (72 each), 16-B reads of the patch (broadcast within the quarter) and of w2t
            const int k0 = h * 72;
            const float4* wr = reinterpret_cast<const float4*>(w2 + (16 * half + c) * kQW2tLd + k0);
            float sum = 0.f;
#pragma unroll 6
            for (int q = 0; q < 18; ++q) {
                const int k = k0 + 4 * q, b = k >> 5, ci = k & 31;
                const float4 x = *reinterpret_cast<const float4*>(c1 + ((8 + b / 3) * kQC1 + 8 + b % 3) * kQC1Ld + ci);
                const float4 w = wr[q];
                sum = __builtin_fmaf(x.x, w.x, sum);
                sum = __builtin_fmaf(x.y, w.y, sum);
                sum = __builtin_fmaf(x.z, w.z, sum);
                sum = __builtin_fmaf(x.w, w.w, sum);
            }
            sum += __shfl_xor(sum, 16);
            sum += __shfl_xor(sum, 32);
            if (lane < 16) o[80 * kQCh + c] = fmaxf(sum + bias2, 0.f);
        }
    }
}

// ------------------------------------------------------------------------------------------ head

// kImg (the default): Dense-Obs over its weight image (wg_gemm_i, direct-to-LDS chunks) with the conv activations
// through an LDS ring filled two chunks ahead, its accumulators starting at the bias; else (no weights set yet) the
// register-staged wg_gemm_t.  LDS: the image path's 32 KB of chunks + the 12 KB ring, then the small layers'
// wg_gemm_t staging from offset 0.
constexpr size_t kQHeadImgSmem = kImgSmem + 3 * 1024 * 4 > kQHeadSmem ? kImgSmem + 3 * 1024 * 4 : kQHeadSmem;
template <typename PT, bool kImg>
__global__ void __launch_bounds__(256, 2) k_qnet_head(QNetDev p, const float* __restrict__ conv, int n,
                                                      const float* __restrict__ feat, size_t feat_ld,
                                                      const PT* __restrict__ prob, size_t prob_ld, QRowMap rm,
                                                      float* __restrict__ q_out, int32_t* __restrict__ act_out,
                                                      const int32_t* __restrict__ d_n, int n_off) {
    extern __shared__ __attribute__((aligned(16))) float qsm[];
    if (d_n) n = min(max(*d_n - n_off, 0), n);
    if ((int)blockIdx.x * kQHeadWaves * 16 >= n) return;          // (uniform: a launch sized for the upper bound)
    float* bsm = qsm;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 4, c = lane & 15;
    const int base = (blockIdx.x * kQHeadWaves + wid) * 16;
    const int ia = min(base + c, n - 1);                 // this lane's agent (clamped: junk rows, never written)
    const int row = rm.rows ? rm.rows[ia] : ia;
    const int env = rm.rows ? row / rm.rowcap : ia;
    // ---- Dense-Obs^T [256 x 16]: the conv activations of this lane's agent, 4 consecutive per chunk step
    f32x4 hobs[16];
    if constexpr (kImg) {
        // the activation rows through LDS: a ring of 3 chunks (64 agents x 16 floats each), filled two chunks ahead
        // by direct-to-LDS loads -- instruction q of wave w: agent 4 (4 w + q) + lane / 16, float lane % 16
        float* ring = bsm + 2 * kImgBuf;
        const float* src[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            src[q] = conv + (size_t)min((int)blockIdx.x * kQHeadWaves * 16 + 4 * (4 * wid + q) + (lane >> 4), n - 1) * kQFlat;
        auto ring_issue = [&](int ch) {
            float* dst = ring + (ch % 3) * 1024 + wid * 256;
            const int k = min(16 * ch + c, kQFlat - 1);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds((const void*)(src[q] + k),
                                                 (__attribute__((address_space(3))) void*)(dst + q * 64), 4, 0, 0);
        };
        ring_issue(0);
        ring_issue(1);
        float4 xv;
        auto vat = [&](int ch, int s) {
            if (s == 0) xv = reinterpret_cast<const float4*>(ring + (ch % 3) * 1024)[(16 * wid + c) * 4 + h];
            return s == 0 ? xv.x : s == 1 ? xv.y : s == 2 ? xv.z : xv.w;
        };
        bias_init(hobs, p.bd, h);
        wg_gemm_i<16, 0, false, 4>(p.wd_img, kQFlat, vat, bsm, hobs, [&](int ch) { ring_issue(ch + 2); });
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) hobs[t][r] = fmaxf(hobs[t][r], 0.f);
    } else {
        const float4* ar = reinterpret_cast<const float4*>(conv + (size_t)ia * kQFlat) + h;   // k = 16 ch + 4 h + s
        float4 cur4 = ar[0], nxt4 = cur4;
        int have = 0;
        wg_gemm_t<16>(p.wd, kQFlat, [&](int ch, int s) {
            if (s == 0) {                                // chunk ch's four values; chunk ch + 1's in flight
                if (have != ch) cur4 = nxt4;
                have = ch;
                if ((ch + 1) * kQKC < kQFlat) nxt4 = ar[(ch + 1) * 4];
            }
            return s == 0 ? cur4.x : s == 1 ? cur4.y : s == 2 ? cur4.z : cur4.w;
        }, bsm, hobs);
    }
    // ---- Dense-Emb^T [32 x 16]
    f32x4 hemb[2];
    {
        const float* fr = feat + (size_t)row * feat_ld;
        const int F = p.F;
        wg_gemm_t<2>(p.we, p.Fp, [&](int ch, int s) { const int k = 16 * ch + 4 * h + s; return k < F ? fr[k] : 0.f; },
                     bsm, hemb);
    }
    // ---- mean field: Prob-Emb^T [64 x 16], Dense-Act-Prob^T [32 x 16] (prob cast to float32 as the placeholder does)
    f32x4 hp[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (p.use_mf) {
        const PT* pr = prob + (size_t)env * prob_ld;
        const int A = p.A;
        f32x4 p1[4];
        wg_gemm_t<4>(p.wp1, p.Ap, [&](int ch, int s) { const int k = 16 * ch + 4 * h + s; return k < A ? (float)pr[k] : 0.f; },
                     bsm, p1);
        wg_gemm_t<2, kQHP1 / 16>(p.wp2, kQHP1, [&](int ch, int s) { return relu_unit(p1, p.bp1, ch, s); }, bsm, hp);
    }
    // ---- Dense2^T [128 x 16] over concat(h_obs 256, h_emb 32, h_prob 32): chunk ch < 16 is h_obs tile ch,
    // 16-17 h_emb, 18-19 h_prob
    f32x4 d2[8];
    wg_gemm_t<8, (kQHObs + kQHEmb + kQHP2) / 16>(p.w2d, p.Kc, [&](int ch, int s) {
        if (ch < 16) return kImg ? hobs[ch][s] : relu_unit(hobs, p.bd, ch, s);   // (kImg: activated in place)
        if (ch < 18) return relu_unit(hemb, p.be, ch - 16, s);
        return relu_unit(hp, p.bp2, ch - 18, s);
    }, bsm, d2);
    f32x4 d3[4];
    wg_gemm_t<4, kQH2 / 16>(p.wo, kQH2, [&](int ch, int s) { return relu_unit(d2, p.b2d, ch, s); }, bsm, d3);
    f32x4 qv[2];
    wg_gemm_t<2, kQHOut / 16>(p.wq, kQHOut, [&](int ch, int s) { return relu_unit(d3, p.bo, ch, s); }, bsm, qv);
    // ---- Q values: lane (h, c) holds actions 16 t + 4 h + r of agent c; argmax (first maximum) over the
    // four lanes of the agent
    const int A = p.A;
    float best = -__builtin_huge_valf();
    int bi = 1 << 30;
    const int i = base + c;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = 16 * t + 4 * h + r;
            if (a < A) {
                const float x = qv[t][r] + p.bq[a];
                if (q_out && i < n) q_out[(size_t)i * A + a] = x;
                if (x > best || (x == best && a < bi)) { best = x; bi = a; }
            }
        }
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {                  // lanes c, c + 16, c + 32, c + 48
        const float ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (h == 0 && i < n && act_out) {
        const int r = rm.rows ? rm.rows[i] : i;
        const size_t slot = rm.rows ? (size_t)(r / rm.rowcap) * rm.act_env + rm.act_off + r % rm.rowcap : (size_t)i;
        act_out[slot] = bi;
    }
}

// ------------------------------------------------------------------------------------------ rollout rows
// The compact row list of one group of a rollout batch: rows e * rowcap + j for j < n_e (n_e = the group's
// size in the [E][G] counts, capped at rowcap), in env order.  Two launches over chunks of 64 envs: k_rows_chunk
// scans each chunk's counts (one wave) into its total (total[1 + b]); k_qnet_rows gives workgroup b the sum of the
// totals before its chunk (at most E / 64 loads) and writes the chunk's rows with consecutive lanes on consecutive
// rows; the last chunk's workgroup writes the row count (total[0]).  (Round 5 summed the counts before the chunk in
// every workgroup: O(E^2 / 64) loads, ~1 GB per call at 131072 envs -- ADVICE r5; round 4 ran one workgroup for the
// whole batch: 0.29 ms per call at 8192 envs.)
constexpr int kRowsEnvs = 64;
__global__ void __launch_bounds__(64) k_rows_chunk(const int32_t* __restrict__ counts, int E, int G, int g, int rowcap,
                                                   int32_t* __restrict__ total) {
    const int e = blockIdx.x * kRowsEnvs + (int)threadIdx.x;
    int c = e < E ? min(counts[e * G + g], rowcap) : 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (threadIdx.x == 0) total[1 + blockIdx.x] = c;
}

__global__ void __launch_bounds__(256) k_qnet_rows(const int32_t* __restrict__ counts, int E, int G, int g, int rowcap,
                                                   int32_t* __restrict__ rows, int32_t* __restrict__ total) {
    __shared__ int red[4];
    __shared__ int cnt[kRowsEnvs], off[kRowsEnvs];
    __shared__ int chunk_total;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int e0 = blockIdx.x * kRowsEnvs, e1 = min(E, e0 + kRowsEnvs);
    int s = 0;
    for (int b = t; b < (int)blockIdx.x; b += blockDim.x) s += total[1 + b];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[wid] = s;
    if (t < kRowsEnvs) {
        const int c = e0 + t < e1 ? min(counts[(e0 + t) * G + g], rowcap) : 0;
        int inc = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        cnt[t] = c;
        off[t] = inc - c;
        if (t == kRowsEnvs - 1) chunk_total = inc;
    }
    __syncthreads();
    const int base = red[0] + red[1] + red[2] + red[3];
    for (int k = 0; k < e1 - e0; ++k) {
        const int m = cnt[k], o = base + off[k], e = e0 + k;
        for (int j = t; j < m; j += blockDim.x) rows[o + j] = e * rowcap + j;
    }
    if (e1 >= E && t == 0) *total = base + chunk_total;
}

hipError_t launch_rollout_rows(const int32_t* counts, int E, int G, int g, int rowcap, int32_t* rows, int32_t* total,
                               hipStream_t st) {
    const int grid = E > 0 ? (E + kRowsEnvs - 1) / kRowsEnvs : 1;   // (E = 0: one workgroup writes the total 0)
    if (E > 0) k_rows_chunk<<<grid, kRowsEnvs, 0, st>>>(counts, E, G, g, rowcap, total);
    k_qnet_rows<<<grid, 256, 0, st>>>(counts, E, G, g, rowcap, rows, total);
    return hipGetLastError();
}

}  // namespace mfx

// ------------------------------------------------------------------------------------------ C ABI
using namespace mfx;

namespace {
struct QNetHandle {
    QNetDev dev{};
    float* blob = nullptr;
    size_t blob_n = 0;
    DevBuf<float> conv;           // [n][2592] activations between the kernels
    float* img = nullptr;         // Dense-Obs's weight image (made by set_weights)
    bool imaged = false;
};

// Offsets (floats) of every matrix / bias in the packed blob, in the order of QNetDev.
void qnet_layout(int F, int A, int use_mf, size_t* off, size_t* total, int* Fp, int* Ap, int* Kc) {
    *Fp = (F + 3) & ~3;
    *Ap = (A + 3) & ~3;
    *Kc = kQHObs + kQHEmb + (use_mf ? kQHP2 : 0);
    const size_t sizes[18] = {(size_t)kQK1 * kQCh, kQCh, (size_t)kQK2 * kQCh, kQCh, (size_t)kQFlat * kQHObs, kQHObs,
                              (size_t)*Fp * kQHEmb, kQHEmb, (size_t)*Ap * kQHP1, kQHP1, (size_t)kQHP1 * kQHP2, kQHP2,
                              (size_t)*Kc * kQH2, kQH2, (size_t)kQH2 * kQHOut, kQHOut, (size_t)kQHOut * kQMaxA, kQMaxA};
    size_t o = 0;
    for (int k = 0; k < 18; ++k) { off[k] = o; o += (sizes[k] + 3) & ~(size_t)3; }
    *total = o;
}
}  // namespace

extern "C" {

MFX_API int mfx_qnet_blob_size(int feature, int n_action, int use_mf, size_t* n_floats, size_t* offsets) {
    if (feature < 1 || feature > 256 || n_action < 1 || n_action > kQMaxA) return fail("qnet: feature 1..256, n_action 1..32");
    size_t off[18];
    int Fp, Ap, Kc;
    qnet_layout(feature, n_action, use_mf, off, n_floats, &Fp, &Ap, &Kc);
    if (offsets) for (int k = 0; k < 18; ++k) offsets[k] = off[k];
    return 0;
}

MFX_API int mfx_qnet_create(int view_h, int view_w, int n_ch, int feature, int n_action, int use_mf, void** handle) {
    if (view_h != kQVH || view_w != kQVW || n_ch != kQNC)
        return fail("qnet: the HIP forward takes the Battle view (13 x 13 x 7); got %d x %d x %d", view_h, view_w, n_ch);
    size_t n = 0;
    MFX_CHECK(mfx_qnet_blob_size(feature, n_action, use_mf, &n, nullptr));
    auto* q = new QNetHandle();
    if (hipMalloc(&q->blob, n * sizeof(float)) != hipSuccess) { delete q; return fail("qnet: hipMalloc of %zu floats", n); }
    q->blob_n = n;
    size_t off[18];
    size_t tot;
    int Fp, Ap, Kc;
    qnet_layout(feature, n_action, use_mf, off, &tot, &Fp, &Ap, &Kc);
    const float** f[18] = {&q->dev.w1, &q->dev.b1, &q->dev.w2, &q->dev.b2, &q->dev.wd, &q->dev.bd, &q->dev.we, &q->dev.be,
                           &q->dev.wp1, &q->dev.bp1, &q->dev.wp2, &q->dev.bp2, &q->dev.w2d, &q->dev.b2d, &q->dev.wo,
                           &q->dev.bo, &q->dev.wq, &q->dev.bq};
    for (int k = 0; k < 18; ++k) *f[k] = q->blob + off[k];
    q->dev.F = feature; q->dev.Fp = Fp; q->dev.A = n_action; q->dev.Ap = Ap; q->dev.use_mf = use_mf; q->dev.Kc = Kc;
    if (hipMalloc(&q->img, img_floats(kQFlat, kQHObs / 16) * sizeof(float)) != hipSuccess) {
        (void)hipFree(q->blob);
        delete q;
        return fail("qnet: hipMalloc of the Dense-Obs image");
    }
    q->dev.wd_img = q->img;
    *handle = q;
    return 0;
}

MFX_API int mfx_qnet_destroy(void* handle) {
    auto* q = static_cast<QNetHandle*>(handle);
    if (!q) return 0;
    if (q->blob) (void)hipFree(q->blob);
    if (q->img) (void)hipFree(q->img);
    delete q;
    return 0;
}

// d_blob: n_floats packed by the caller (mfx_qnet_blob_size offsets), copied on `stream`.
MFX_API int mfx_qnet_set_weights(void* handle, const float* d_blob, size_t n_floats, void* stream) {
    auto* q = static_cast<QNetHandle*>(handle);
    if (n_floats != q->blob_n) return fail("qnet_set_weights: %zu floats, the layout has %zu", n_floats, q->blob_n);
    MFX_HIP(hipMemcpyAsync(q->blob, d_blob, n_floats * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    MFX_HIP(launch_weight_image(q->dev.wd, kQFlat, kQHObs, q->img, (hipStream_t)stream));
    q->imaged = true;
    return 0;
}

// Agents per conv -> head pass: the Conv2 activations of a pass sit in HBM between the two kernels
// (10 KB per agent: 2.7 GB at this size).
constexpr int kQPass = 1 << 18;

// n rows (d_n: the count on the device, n its upper bound -- nothing is read back; launches sized for n).
static int qnet_run(QNetHandle* q, const float* view, size_t view_ld, const float* feat, size_t feat_ld,
                    const void* prob, int prob_f64, size_t prob_ld, QRowMap rm, int n, float* q_out, int32_t* act,
                    hipStream_t st, const int32_t* d_n = nullptr) {
    if (n <= 0) return 0;
    if (q->dev.use_mf && !prob) return fail("qnet: the mean-field net needs prob");
    try { q->conv.ensure((size_t)std::min(n, kQPass) * kQFlat); } catch (const HipFailure& f) { return fail("%s", f.what()); }
    int dev = 0, cus = 0;
    MFX_HIP(hipGetDevice(&dev));
    MFX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (int off = 0; off < n; off += kQPass) {
        const int m = std::min(kQPass, n - off);
        QRowMap r = rm;
        if (r.rows) r.rows += off;
        // dense rows: pass `off` shifts every row-indexed input / output
        const float* v = r.rows ? view : view + (size_t)off * view_ld;
        const float* f = r.rows ? feat : feat + (size_t)off * feat_ld;
        const void* pb = prob;
        if (prob && !r.rows) pb = prob_f64 ? (const void*)(static_cast<const double*>(prob) + (size_t)off * prob_ld)
                                           : (const void*)(static_cast<const float*>(prob) + (size_t)off * prob_ld);
        float* qo = q_out ? q_out + (size_t)off * q->dev.A : nullptr;
        int32_t* ao = act ? (r.rows ? act : act + off) : nullptr;
        const int cgrid = std::min((m + kQConv2Agents - 1) / kQConv2Agents, cus);
        k_qnet_conv2<<<cgrid, 512, kQConvSmem, st>>>(q->dev, v, view_ld, r.rows, m, q->conv.p, d_n, off);
        MFX_HIP(hipGetLastError());
        const int hgrid = (m + 16 * kQHeadWaves - 1) / (16 * kQHeadWaves);
        const bool img = q->imaged;
#define MFX_QHEAD(PT, IMG)                                                                                         \
        k_qnet_head<PT, IMG><<<hgrid, 256, IMG ? kQHeadImgSmem : kQHeadSmem, st>>>(                                  \
            q->dev, q->conv.p, m, f, feat_ld, static_cast<const PT*>(pb), prob_ld, r, qo, ao, d_n, off)
        if (prob_f64) { if (img) MFX_QHEAD(double, true); else MFX_QHEAD(double, false); }
        else { if (img) MFX_QHEAD(float, true); else MFX_QHEAD(float, false); }
#undef MFX_QHEAD
        MFX_HIP(hipGetLastError());
    }
    return 0;
}

// The compact row list act_rollout builds (k_rows_chunk + k_qnet_rows), on its own: rows of group g of [E][G] counts.
MFX_API int mfx_rollout_rows(const int32_t* d_counts, int E, int G, int g, int rowcap, int32_t* d_rows, int32_t* d_total,
                             void* stream) {
    if (E < 0 || G < 1 || g < 0 || g >= G || rowcap < 1) return fail("rollout_rows: bad shape");
    MFX_HIP(launch_rollout_rows(d_counts, E, G, g, rowcap, d_rows, d_total, (hipStream_t)stream));
    return 0;
}

// n agents, dense rows: view [n][1183], feature [n][F], prob [n][A] float32 (mean field; else null).
// q_out [n][A] and act [n] (either may be null).
MFX_API int mfx_qnet_forward(void* handle, const float* d_view, const float* d_feat, const float* d_prob, int n,
                             float* d_q, int32_t* d_act, void* stream) {
    auto* q = static_cast<QNetHandle*>(handle);
    QRowMap rm{nullptr, 1, 0, 0};
    return qnet_run(q, d_view, kQViewF, d_feat, q->dev.F, d_prob, 0, q->dev.A, rm, n, d_q, d_act, (hipStream_t)stream);
}

// Group g of a rollout batch ([E][rowcap] view / feature rows, counts [E][G], former mean actions
// [E][G][mean_stride] float64): actions into d_act [E][G][rowcap] for the group's live rows.  d_rows:
// scratch of E * rowcap ints, d_total: one int.  The row list and its count stay on the device: the kernels
// are launched for the upper bound E * rowcap and read the count themselves (no host round trip, so the
// whole act step can be captured in a graph or queued behind the previous launch).
MFX_API int mfx_qnet_act_rollout(void* handle, const float* d_view, const float* d_feat, const int32_t* d_counts,
                                 const double* d_mean, int mean_stride, int E, int G, int g, int rowcap,
                                 int32_t* d_rows, int32_t* d_total, int32_t* d_act, void* stream) {
    auto* q = static_cast<QNetHandle*>(handle);
    hipStream_t st = (hipStream_t)stream;
    MFX_HIP(launch_rollout_rows(d_counts, E, G, g, rowcap, d_rows, d_total, st));
    QRowMap rm{d_rows, rowcap, G * rowcap, g * rowcap};
    return qnet_run(q, d_view, kQViewF, d_feat, q->dev.F, d_mean + (size_t)g * mean_stride, 1, (size_t)G * mean_stride,
                    rm, E * rowcap, nullptr, d_act, st, d_total);
}

}  // extern "C"
