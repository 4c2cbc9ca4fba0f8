// acnet_kernels.hip -- the reference's actor-critic network (ActorCritic._create_network, algo/ac.py:48-98, and
// MFAC._create_network, :219-276) and its act (tf.multinomial over log(policy), :43-46 / :213-217), forward only,
// hand-written for gfx950 on the f32-input MFMA v_mfma_f32_16x16x4_f32.  Per agent:
//
//   view [V] (flattened NHWC, V = 1,183 at 13 x 13 x 7) --dense 256, relu--> h_view
//   feature [F]                                        --dense 256, relu--> h_emb
//   concat(h_view, h_emb) [512] --dense 512, relu--> d
//   policy = clip(softmax(dense(d / 0.1) -> A), 1e-10, 1 - 1e-10);  act ~ multinomial(log policy)
//   value (AC):   dense(d -> 1)
//   value (MFAC): prob [A] --dense 64, relu--> --dense 32, relu--> p;  dense(relu(dense(concat(h_view, h_emb, p)
//                 [544] -> 256)) -> 1)
//
// The policy path is 1.17 MFLOP per agent (dense-view 52 %, dense-512 45 %): MFMA-bound at the f32 matrix rate
// (157 TF/s).  One kernel, k_acnet: four waves x 16 agents per workgroup, every layer transposed (weights as the
// A operand, staged in 16-row chunks in LDS and shared by the four waves; the layer's accumulators are the next
// layer's B operand in registers, policy_gemm.h).  The 512-wide layer is computed as two 256-unit halves, each
// folded into the policy logits (and the AC value) as soon as it is ready, so at most 3 x 256 activations per
// agent are live: h_view and h_emb (the concat) and one half of d.
//
// The draw: the reference samples tf.multinomial(log(policy)), i.e. action a with probability policy[a] /
// sum(policy).  Here u = a counter hash of (seed, step, group, row) -> [0, 1) (24 bits), and the action is the
// first a whose running f32 sum of policy[0..a] exceeds u * sum(policy) (the sums in action order) -- a pure
// function of the policy row and the counters, restated on the host by tests/acnet_ref.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "mfx_common.h"
#include "policy_gemm.h"
#include "../../include/magent_amd.h"

namespace mfx {

constexpr int kAH = 256;                 // hidden width (hidden_size[0])
constexpr int kAMaxA = 32;               // policy columns (n_action padded)
constexpr int kAMaxV = 4096;             // flattened view floats the kernel takes
constexpr int kABlocks = 19;

// Packed weights (every matrix [K][N] row-major, K padded to a multiple of 4 with zero rows):
//  0 wv  [Vp][256]  h_view          1 bv [256]
//  2 we  [Fp][256]  h_emb           3 be [256]
//  4 wd0 [512][256] dense, units 0..255     5 wd1 [512][256] units 256..511     6 bd [512]
//  7 wp  [512][32]  policy (A columns, zero-padded)                              8 bp [32]
//  9 wval [512][16] AC value (column 0)                                          10 bval [16]
// 11 wep [Ap][64]  MF emb_prob      12 bep [64]
// 13 wdp [64][32]  MF dense_prob    14 bdp [32]
// 15 wvd [544][256] MF value dense  16 bvd [256]
// 17 wvo [256][16] MF value (column 0)                                           18 bvo [16]
// (blocks 9-10 are empty with mean field, 11-18 without.)
// The weight images of the GEMM layers (policy_gemm.h wg_gemm_i; made at set_weights by launch_weight_image):
//  0 wv  1 wd0  2 wd1  3 wp (units 0..255 of d)  4 wp (units 256..511)  5 wval (0..255)  6 wval (256..511)
//  7 wep  8 wdp  9 wvd  10 wvo
constexpr int kAImg = 11;
struct ACNetDev {
    const float* w[kABlocks];
    const float* img[kAImg];
    int V, Vp, F, Fp, A, Ap, use_mf;
    // The view's input support (mfx_acnet_set_input_support; null: the dense order).  The view layer then runs over
    // the vK inputs that can be non-zero only -- e.g. the Battle view's cells outside the view circle carry nothing
    // but the two minimap channels (Map.cc:130-218), 280 of 1,183 inputs always zero -- in a packed order: packed
    // input 16 ch + j is view float vdesc[8 ch + 4] + byte j of vdesc[8 ch .. 8 ch + 3], and vimg is the image of
    // wv's rows in that order (mfx_acnet_set_input_support keeps the dense chain's order of the supported inputs).  A
    // skipped input is an exact zero, so each fma it leaves out of a chain would only have added 0 * w: the same
    // result bit for bit (the MFMA accumulates as an fmaf chain, MI355X_MICROARCH.md).
    const uint32_t* vdesc;
    const float* vimg;
    int vK;
};

// x / 0.1f, correctly rounded (the reference's dense / 0.1): q = x * 10, one fma residual and one fma correction --
// equal to the IEEE quotient for every f32 |x| >= 2^-100 (checked exhaustively, scripts/micro/div_tenth.c); tinier
// nonzero x take the division.
__device__ __forceinline__ float div_tenth(float x) {
    const float q = x * 10.0f, r = __builtin_fmaf(-q, 0.1f, x);
    float y = __builtin_fmaf(r, 10.0f, q);
    if (__builtin_expect(x != 0.f && __builtin_fabsf(x) < 0x1p-100f, 0)) y = x / 0.1f;
    return y;
}

__device__ __forceinline__ uint32_t ac_mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}

// The uniform of row `row` of group g at step `step` (tests/acnet_ref.py restates it).
__device__ __forceinline__ float ac_uniform(uint32_t seed, uint32_t step, int g, int row) {
    const uint32_t k = seed ^ ac_mix32(step * 0x9E3779B9u + (uint32_t)g * 0x632BE5ABu) ^
                       ac_mix32((uint32_t)row * 0x85EBCA77u + 0x165667B1u);
    return (float)(ac_mix32(k) >> 8) * (1.0f / 16777216.0f);
}

// rows (rm.rows): compact agent i -> view / feature row; the action slot as in QRowMap; the prob row of
// the env (mean field).  d_n: the row count on the device (launch sized for n).  policy_out [n][A],
// value_out [n], act_out: any may be null.
// kHeLds (features of at most kHeF floats, the Battle shape's 34): h_emb is never held.  Its weights sit in LDS for
// the whole kernel and each 16-unit tile of it is recomputed from the features (9 MFMAs, 9 feature registers) right
// where the concat needs it -- 3 % more MFMA work for 64 fewer registers per lane, which is what lets two
// workgroups share a CU (one wave per SIMD otherwise: 256 VGPRs + ~100 AGPRs).
constexpr int kHeF = 36;
#ifndef MFX_ACNET_SKIP
#define MFX_ACNET_SKIP 0      // A/B builds only (make variant): 1 view layer, 2 dense layers, 4 policy layer, 8 h_emb skipped
#endif
constexpr size_t kAcnetLdsSmem = kQHeadSmem + (size_t)kHeF * kAH * 4;
constexpr size_t kAcnetImgLdsSmem = kImgSmem + (size_t)kHeF * kAH * 4 + 3 * 1024 * 4;   // + the view ring: 80 KB

// kImg: the layers run wg_gemm_i over the weight images (direct-to-LDS staging; made by set_weights), else
// wg_gemm_t.  GEMM<MT, NCH, kZero>(block, image, K, v_at, acc) picks the form.
template <typename PT, bool kMF, bool kHeLds, bool kImg, bool kPack = false>
__global__ void __launch_bounds__(256, kHeLds ? 2 : 1) k_acnet(ACNetDev p, const float* __restrict__ view, size_t view_ld,
                                                  const float* __restrict__ feat, size_t feat_ld,
                                                  const PT* __restrict__ prob, size_t prob_ld, QRowMap rm, int n,
                                                  const int32_t* __restrict__ d_n, float* __restrict__ policy_out,
                                                  float* __restrict__ value_out, int32_t* __restrict__ act_out,
                                                  uint32_t seed, uint32_t step, int group) {
    extern __shared__ __attribute__((aligned(16))) float qsm[];
    if (d_n) n = min(*d_n, n);
    const int tiles = (n + kQHeadWaves * 16 - 1) / (kQHeadWaves * 16);
    if ((int)blockIdx.x >= tiles) return;                          // (uniform: a launch sized for the upper bound)
    float* bsm = qsm;
    const bool he_fold = kImg && p.F < kHeF;                       // (kImg: the folded form; A/B keeps the old one)
    const float* weS = bsm + (kImg ? 2 * kImgBuf : 2 * kQKC * kQBLd);   // kHeLds: We [kHeF][256] after the staging
    if (kHeLds) {
        // We in LDS for the workgroup's life; the bias as one more input row when the features leave one free
        // (k = F: weight be, input 1), so the recomputed tile needs no bias load
        float* wd = bsm + (kImg ? 2 * kImgBuf : 2 * kQKC * kQBLd);
        const int F = p.F;
        for (int i = threadIdx.x; i < kHeF * kAH; i += blockDim.x)
            wd[i] = i < F * kAH ? p.w[2][i] : (he_fold && i < (F + 1) * kAH) ? p.w[3][i - F * kAH] : 0.f;
        __syncthreads();
    }
    // persistent: tile after tile of 64 agents (the grid: the workgroups the CUs hold at once, or fewer)
    for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int tid = tid_x(), lane = tid & 63, wid = tid >> 6, h = lane >> 4, c = lane & 15;
    const int base = (tile * kQHeadWaves + wid) * 16;
    const int ia = min(base + c, n - 1);                            // this lane's agent (clamped: junk, never written)
    const int row = rm.rows ? rm.rows[ia] : ia;
    const int env = rm.rows ? row / rm.rowcap : ia;
    // the weight and image pointers, opaque per tile: else the compiler hoists every chunk's addresses out of the
    // tile loop and spills them
    const float* W[kABlocks];
    const float* I[kAImg];
#pragma unroll
    for (int k = 0; k < kABlocks; ++k) { W[k] = p.w[k]; asm volatile("" : "+s"(W[k])); }
#pragma unroll
    for (int k = 0; k < kAImg; ++k) { I[k] = p.img[k]; asm volatile("" : "+s"(I[k])); }
#define MFX_ACNET_GEMM(MT, NCH, ZERO, WB, IB, K, VAT, ACC)                                                              \
    do {                                                                                                              \
        if constexpr (kImg) wg_gemm_i<MT, NCH, ZERO>(IB, K, VAT, bsm, ACC);                                          \
        else wg_gemm_t<MT, NCH, ZERO>(WB, K, VAT, bsm, ACC);                                                         \
    } while (0)
    // ---- h_view^T [256 x 16]: view floats k = 16 ch + 4 h + s of this lane's agent, two chunks ahead in flight
    f32x4 hv[16];
    if constexpr (kImg) {
        // the view rows through LDS: a ring of 3 chunks (64 agents x 16 floats each, after We), filled two chunks
        // ahead by direct-to-LDS loads -- instruction q of wave w: agent 4 (4 w + q) + lane / 16, float lane % 16
        // (columns past V read float V - 1: its weights are zero)
        float* vring = bsm + 2 * kImgBuf + kHeF * kAH;
        const float* vsrc[4];
        // the packed order's chunk descriptors through the constant address space: scalar loads, each issued one
        // chunk before its use (a vector load here would wait, vmcnt being in order, for the chunk's image loads)
        // kPack: the packed order's chunk descriptors through the constant address space -- scalar loads, each issued
        // one chunk before its use (volatile: not sunk to the use), waited for by the chunk-end barrier's lgkmcnt(0)
        typedef const volatile __attribute__((address_space(4))) uint32_t* cdesc_t;
        cdesc_t dq = (cdesc_t)p.vdesc;
        asm volatile("" : "+s"(dq));
        uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0;
        auto dload = [&](int ch) {
            d0 = dq[8 * ch]; d1 = dq[8 * ch + 1]; d2 = dq[8 * ch + 2]; d3 = dq[8 * ch + 3]; d4 = dq[8 * ch + 4];
        };
        if (kPack) dload(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int a = min(tile * kQHeadWaves * 16 + 4 * (4 * wid + q) + (lane >> 4), n - 1);
            vsrc[q] = view + (size_t)(rm.rows ? rm.rows[a] : a) * view_ld;
        }
        const int V = p.V;
        auto view_issue = [&](int ch) {
            float* dst = vring + (ch % 3) * 1024 + wid * 256;
            int k;
            if constexpr (kPack) {                                 // the packed order
                const uint32_t lo = (c & 4) ? d1 : d0, hi = (c & 4) ? d3 : d2, w = (c & 8) ? hi : lo;
                k = (int)(d4 + ((w >> (8 * (c & 3))) & 255u));
                dload(ch + 1);
            } else {
                k = min(16 * ch + c, V - 1);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds((const void*)(vsrc[q] + k),
                                                 (__attribute__((address_space(3))) void*)(dst + q * 64), 4, 0, 0);
        };
        view_issue(0);
        view_issue(1);
        float4 xv;
        auto vat = [&](int ch, int s) {
            if (s == 0) xv = reinterpret_cast<const float4*>(vring + (ch % 3) * 1024)[(16 * wid + c) * 4 + h];
            return s == 0 ? xv.x : s == 1 ? xv.y : s == 2 ? xv.z : xv.w;
        };
        bias_init(hv, W[1], h);
        if (!(MFX_ACNET_SKIP & 1))
            wg_gemm_i<16, 0, false, 4>(kPack ? p.vimg : I[0], kPack ? p.vK : p.Vp, vat, bsm, hv,
                                       [&](int ch) { view_issue(ch + 2); });
    } else {
        const float* vr = view + (size_t)row * view_ld + 4 * h;
        const int V = p.V;
        float b0[4], b1[4], b2[4];
        auto fetch = [&](int ch, float* b) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = 16 * ch + 4 * h + s;
                b[s] = k < V ? vr[16 * ch + s] : 0.f;
            }
        };
        fetch(0, b0);
        fetch(1, b1);
        int have = -1;
        auto vat = [&](int ch, int s) {
            if (s == 0 && have != ch) {                             // rotate: chunk ch in b0, ch + 1 in b1
                if (have >= 0) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) { b0[j] = b1[j]; b1[j] = b2[j]; }
                }
                have = ch;
                fetch(ch + 2, b2);
            }
            return b0[s];
        };
        bias_init(hv, W[1], h);
        wg_gemm_t<16, 0, false>(W[0], p.Vp, vat, bsm, hv);
    }
    // the concat's h_view half, activated in place once (relu; the bias was the accumulators' start): read as is by
    // every later layer
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[t][r] = fmaxf(hv[t][r], 0.f);
    // ---- h_emb^T [256 x 16]: held (kHeLds false), or recomputed per tile from the LDS-resident weights
    f32x4 he[kHeLds ? 1 : 16];
    float fr4[kHeLds ? kHeF / 4 : 1];
    {
        const float* fr = feat + (size_t)row * feat_ld;
        const int F = p.F;
        if (kHeLds) {
#pragma unroll
            for (int ks = 0; ks < kHeF / 4; ++ks) {                 // k = 4 ks + h: this lane's B operands
                const int k = 4 * ks + h;
                fr4[ks] = k < F ? fr[k] : (he_fold && k == F) ? 1.f : 0.f;
            }
        } else {
            wg_gemm_t<16>(W[2], p.Fp, [&](int ch, int s) { const int k = 16 * ch + 4 * h + s; return k < F ? fr[k] : 0.f; },
                          bsm, he);                                 // (small K: registers staging either way)
        }
    }
    // h_emb tile t (units 16 t + 4 h + r in register r, agent c): A = We^T rows 16 t + c from LDS, B = the features.
    // Software-pipelined: tile t's 9 dependent MFMAs run spread over the four k-steps of the chunk before the one
    // that reads it (3 + 2 + 2 + 2, each behind the chunk's 16 independent MFMAs), not as a chain at its head.
    static_assert(kHeF == 36, "the k-step split of the h_emb tile");
    f32x4 he_cur = {0.f, 0.f, 0.f, 0.f}, he_nxt = {0.f, 0.f, 0.f, 0.f};
    auto he_part = [&](int t, int s) {
        const int lo = s == 0 ? 0 : 1 + 2 * s, hi = 3 + 2 * s;
#pragma unroll
        for (int ks = lo; ks < hi; ++ks) he_nxt = mfma4(weS[(4 * ks + h) * kAH + 16 * t + c], fr4[ks], he_nxt);
    };
    // concat unit k = 16 ch + 4 h + s: ch < 16 h_view tile ch, else h_emb tile ch - 16 (calls in (ch, s) order)
    auto concat_at = [&](int ch, int s) {
        if (MFX_ACNET_SKIP & 8) return hv[ch & 15][s];
        if (kHeLds) {
            if (ch >= 16 && s == 0) he_cur = he_nxt;
            if (ch >= 15 && ch < 31) {
                if (s == 0) he_nxt = {0.f, 0.f, 0.f, 0.f};
                he_part(ch - 15, s);
            }
        }
        if (ch < 16) return hv[ch][s];
        if (kHeLds) return he_fold ? fmaxf(he_cur[s], 0.f) : relu_unit(&he_cur, W[3] + 16 * (ch - 16), 0, s);
        return relu_unit(he, W[3], ch - 16, s);
    };
    // ---- dense [512] in two halves, each folded into the policy logits (and the AC value) at once
    f32x4 pl[2];
    f32x4 vv[1] = {{0.f, 0.f, 0.f, 0.f}};
    {
        f32x4 dh[16];
        auto act_half = [&](int half) {                             // relu in place (the bias: the GEMM's start)
#pragma unroll
            for (int t = 0; t < 16; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) dh[t][r] = fmaxf(dh[t][r], 0.f);
        };
        auto dsc = [&](int ch, int s) { return div_tenth(dh[ch][s]); };
        auto dval = [&](int ch, int s) { return dh[ch][s]; };
        bias_init(dh, W[6], h);
        if (!(MFX_ACNET_SKIP & 2)) MFX_ACNET_GEMM(16, 32, false, W[4], I[1], 2 * kAH, concat_at, dh);
        act_half(0);
        if (!(MFX_ACNET_SKIP & 4)) MFX_ACNET_GEMM(2, 16, true, W[7], I[3], kAH, dsc, pl);
        else pl[0] = pl[1] = dh[0];
        if (!kMF && value_out) MFX_ACNET_GEMM(1, 16, true, W[9], I[5], kAH, dval, vv);
        bias_init(dh, W[6] + kAH, h);
        if (!(MFX_ACNET_SKIP & 2)) MFX_ACNET_GEMM(16, 32, false, W[5], I[2], 2 * kAH, concat_at, dh);
        act_half(1);
        if (!(MFX_ACNET_SKIP & 4)) MFX_ACNET_GEMM(2, 16, false, W[7] + kAH * kAMaxA, I[4], kAH, dsc, pl);
        else pl[0] += dh[1];
        if (!kMF && value_out) MFX_ACNET_GEMM(1, 16, false, W[9] + kAH * 16, I[6], kAH, dval, vv);
    }
    // ---- MF value: emb_prob 64, dense_prob 32, dense 256 over concat(h_view, h_emb, p), value 1
    if (kMF && value_out) {
        const PT* pr = prob + (size_t)env * prob_ld;
        const int A = p.A;
        f32x4 e1[4], e2[2];
        auto pat = [&](int ch, int s) { const int k = 16 * ch + 4 * h + s; return k < A ? (float)pr[k] : 0.f; };
        MFX_ACNET_GEMM(4, 0, true, W[11], I[7], p.Ap, pat, e1);
        auto e1at = [&](int ch, int s) { return relu_unit(e1, W[12], ch, s); };
        MFX_ACNET_GEMM(2, 4, true, W[13], I[8], 64, e1at, e2);
        f32x4 vd[16];
        auto vdat = [&](int ch, int s) { return ch < 32 ? concat_at(ch, s) : relu_unit(e2, W[14], ch - 32, s); };
        MFX_ACNET_GEMM(16, 34, true, W[15], I[9], 2 * kAH + 32, vdat, vd);
        auto voat = [&](int ch, int s) { return relu_unit(vd, W[16], ch, s); };
        MFX_ACNET_GEMM(1, 16, true, W[17], I[10], kAH, voat, vv);
    }
    const int i = base + c;
    if (value_out && h == 0 && i < n) value_out[i] = vv[0][0] + W[kMF ? 18 : 10][0];   // unit 0: lanes h == 0, r 0
    // ---- policy: logits of agent c, actions 16 t + 4 h + r, through LDS to lane c of the wave (h == 0): softmax,
    // clip, the draw
    float* lg = bsm + wid * 16 * kAMaxA;                             // (the staging buffer is free: wg_gemm_t ended
#pragma unroll                                                       //  with a barrier)
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) lg[c * kAMaxA + 16 * t + 4 * h + r] = pl[t][r];
    qwave_sync();
    if (h == 0 && i < n) {
        const int A = p.A;
        const float* bp = W[8];
        float x[kAMaxA];
        float m = -__builtin_huge_valf();
#pragma unroll
        for (int a = 0; a < kAMaxA; ++a) {
            x[a] = a < A ? lg[c * kAMaxA + a] + bp[a] : 0.f;
            if (a < A) m = fmaxf(m, x[a]);
        }
        float sum = 0.f;
#pragma unroll
        for (int a = 0; a < kAMaxA; ++a)
            if (a < A) { x[a] = expf(x[a] - m); sum += x[a]; }
        float tot = 0.f;
#pragma unroll
        for (int a = 0; a < kAMaxA; ++a)
            if (a < A) { x[a] = fminf(fmaxf(x[a] / sum, 1e-10f), 1.0f - 1e-10f); tot += x[a]; }
        if (policy_out) {
            float* po = policy_out + (size_t)i * A;
            for (int a = 0; a < A; ++a) po[a] = x[a];
        }
        if (act_out) {
            const float thr = ac_uniform(seed, step, group, row) * tot;
            float run = 0.f;
            int pick = -1;
#pragma unroll
            for (int a = 0; a < kAMaxA; ++a)
                if (a < A) {
                    run += x[a];
                    if (pick < 0 && run > thr) pick = a;
                }
            if (pick < 0) pick = A - 1;                             // (rounding: u * tot at the very top)
            const size_t slot = rm.rows ? (size_t)(row / rm.rowcap) * rm.act_env + rm.act_off + row % rm.rowcap : (size_t)i;
            act_out[slot] = pick;
        }
    }
    __syncthreads();                                                 // (lg and the staging buffers: the next tile's)
    }
#undef MFX_ACNET_GEMM
}

}  // namespace mfx

// ------------------------------------------------------------------------------------------ C ABI
using namespace mfx;

namespace {
struct ACNetHandle {
    ACNetDev dev{};
    float* blob = nullptr;
    size_t blob_n = 0;
    float* img = nullptr;                 // the weight images (launch_weight_image), made by set_weights
    size_t img_n = 0;
    bool imaged = false;
    // the view's input support (mfx_acnet_set_input_support): packed order, its chunk descriptors, wv's rows in that
    // order (gathered, then imaged)
    int vK = 0;                           // packed rows (a multiple of 16: pads are zero rows)
    int vKn = 0;                          // supported inputs
    int* vperm = nullptr;                 // [vK] view row of packed input p (-1: a zero pad row)
    uint32_t* vdesc = nullptr;            // [(chunks + 2) * 8]
    float* vrows = nullptr;               // [vK][256]
    float* vimg = nullptr;
};

__global__ void k_gather_rows(const float* __restrict__ src, const int* __restrict__ idx, int rows, int cols,
                              float* __restrict__ dst) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (size_t)rows * cols) {
        const int r = idx[i / cols];
        dst[i] = r >= 0 ? src[(size_t)r * cols + i % cols] : 0.f;
    }
}

// wv's rows in the packed order -> the image the kernel reads (after set_weights and after a support change)
int acnet_support_image(ACNetHandle* q, hipStream_t st) {
    if (!q->vK || !q->imaged) return 0;
    const size_t n = (size_t)q->vK * kAH;
    k_gather_rows<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(q->dev.w[0], q->vperm, q->vK, kAH, q->vrows);
    MFX_HIP(hipGetLastError());
    MFX_HIP(launch_weight_image(q->vrows, q->vK, kAH, q->vimg, st));
    q->dev.vdesc = q->vdesc;
    q->dev.vimg = q->vimg;
    q->dev.vK = q->vK;
    return 0;
}

void acnet_support_free(ACNetHandle* q) {
    for (void* x : {(void*)q->vperm, (void*)q->vdesc, (void*)q->vrows, (void*)q->vimg})
        if (x) (void)hipFree(x);
    q->vperm = nullptr; q->vdesc = nullptr; q->vrows = nullptr; q->vimg = nullptr;
    q->vK = 0;
    q->vKn = 0;
    q->dev.vdesc = nullptr; q->dev.vimg = nullptr; q->dev.vK = 0;
}

// The imaged blocks: (blob block, row offset, K, N) of images 0..10 (ACNetDev::img).
struct ImgDesc { int block, row0, K, N; };
void acnet_images(const ACNetDev& d, ImgDesc* o) {
    const int mf = d.use_mf;
    const ImgDesc t[kAImg] = {{0, 0, d.Vp, kAH}, {4, 0, 2 * kAH, kAH}, {5, 0, 2 * kAH, kAH},
                              {7, 0, kAH, kAMaxA}, {7, kAH, kAH, kAMaxA},
                              {9, 0, mf ? 0 : kAH, 16}, {9, kAH, mf ? 0 : kAH, 16},
                              {11, 0, mf ? d.Ap : 0, 64}, {13, 0, mf ? 64 : 0, 32},
                              {15, 0, mf ? 2 * kAH + 32 : 0, kAH}, {17, 0, mf ? kAH : 0, 16}};
    for (int k = 0; k < kAImg; ++k) o[k] = t[k];
}

void acnet_sizes(int V, int F, int A, int use_mf, size_t* sz) {
    const size_t Vp = (V + 3) & ~3, Fp = (F + 3) & ~3, Ap = (A + 3) & ~3;
    const size_t mf = use_mf ? 1 : 0, ac = 1 - mf;
    const size_t s[kABlocks] = {Vp * kAH, kAH, Fp * kAH, kAH, 2 * kAH * kAH, 2 * kAH * kAH, 2 * kAH,
                                2 * kAH * kAMaxA, kAMaxA, ac * 2 * kAH * 16, ac * 16,
                                mf * Ap * 64, mf * 64, mf * 64 * 32, mf * 32, mf * (2 * kAH + 32) * kAH, mf * kAH,
                                mf * kAH * 16, mf * 16};
    for (int k = 0; k < kABlocks; ++k) sz[k] = s[k];
}
}  // namespace

extern "C" {

MFX_API int mfx_acnet_blob_size(int view_floats, int feature, int n_action, int use_mf, size_t* n_floats,
                                size_t* offsets) {
    if (view_floats < 1 || view_floats > kAMaxV || feature < 1 || feature > 256 || n_action < 2 || n_action > kAMaxA)
        return fail("acnet: view 1..%d floats, feature 1..256, n_action 2..%d", kAMaxV, kAMaxA);
    size_t sz[kABlocks], o = 0;
    acnet_sizes(view_floats, feature, n_action, use_mf, sz);
    for (int k = 0; k < kABlocks; ++k) {
        if (offsets) offsets[k] = o;
        o += (sz[k] + 3) & ~(size_t)3;
    }
    *n_floats = o;
    return 0;
}

MFX_API int mfx_acnet_create(int view_floats, int feature, int n_action, int use_mf, void** handle) {
    size_t n = 0, off[kABlocks];
    MFX_CHECK(mfx_acnet_blob_size(view_floats, feature, n_action, use_mf, &n, off));
    auto* q = new ACNetHandle();
    if (hipMalloc(&q->blob, n * sizeof(float)) != hipSuccess) { delete q; return fail("acnet: hipMalloc of %zu floats", n); }
    q->blob_n = n;
    for (int k = 0; k < kABlocks; ++k) q->dev.w[k] = q->blob + off[k];
    q->dev.V = view_floats; q->dev.Vp = (view_floats + 3) & ~3;
    q->dev.F = feature; q->dev.Fp = (feature + 3) & ~3;
    q->dev.A = n_action; q->dev.Ap = (n_action + 3) & ~3;
    q->dev.use_mf = use_mf ? 1 : 0;
    ImgDesc im[kAImg];
    acnet_images(q->dev, im);
    size_t io[kAImg], tot = 0;
    for (int k = 0; k < kAImg; ++k) { io[k] = tot; tot += im[k].K ? img_floats(im[k].K, im[k].N / 16) : 0; }
    if (hipMalloc(&q->img, tot * sizeof(float)) != hipSuccess) {
        (void)hipFree(q->blob);
        delete q;
        return fail("acnet: hipMalloc of %zu image floats", tot);
    }
    q->img_n = tot;
    for (int k = 0; k < kAImg; ++k) q->dev.img[k] = q->img + io[k];
    *handle = q;
    return 0;
}

MFX_API int mfx_acnet_destroy(void* handle) {
    auto* q = static_cast<ACNetHandle*>(handle);
    if (!q) return 0;
    if (q->blob) (void)hipFree(q->blob);
    if (q->img) (void)hipFree(q->img);
    acnet_support_free(q);
    delete q;
    return 0;
}

MFX_API int mfx_acnet_set_weights(void* handle, const float* d_blob, size_t n_floats, void* stream) {
    auto* q = static_cast<ACNetHandle*>(handle);
    if (n_floats != q->blob_n) return fail("acnet_set_weights: %zu floats, the layout has %zu", n_floats, q->blob_n);
    MFX_HIP(hipMemcpyAsync(q->blob, d_blob, n_floats * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    ImgDesc im[kAImg];
    acnet_images(q->dev, im);
    for (int k = 0; k < kAImg; ++k) {
        if (!im[k].K) continue;
        const size_t n = img_floats(im[k].K, im[k].N / 16);
        (void)n;
        MFX_HIP(launch_weight_image(q->dev.w[im[k].block] + (size_t)im[k].row0 * im[k].N, im[k].K, im[k].N,
                                    const_cast<float*>(q->dev.img[k]), (hipStream_t)stream));
    }
    q->imaged = true;
    return acnet_support_image(q, (hipStream_t)stream);
}

// The view inputs that can be non-zero: mask[n] (n = view floats; 1 = may be non-zero), e.g. from
// mfx_battle_view_support; null clears it (the dense order).  Every later forward / act_rollout skips the inputs
// outside the support -- the caller's contract: they are exactly zero there (the engine's observation buffers are);
// the results are then bit-identical to the dense order.
MFX_API int mfx_acnet_set_input_support(void* handle, const uint8_t* mask, int n, void* stream) {
    auto* q = static_cast<ACNetHandle*>(handle);
    acnet_support_free(q);
    if (!mask) return 0;
    if (n != q->dev.V) return fail("acnet_set_input_support: %d entries, the view has %d floats", n, q->dev.V);
    // The MFMA chain of one accumulator runs chunk by chunk, k-step s by k-step, lane group h by lane group (input
    // 16 ch + 4 h + s; an fmaf chain, MI355X_MICROARCH.md).  The supported inputs keep that order: the i-th one in
    // the dense chain takes the i-th place of the packed chain (chunk i / 16, k-step (i % 16) / 4, lane group i % 4,
    // i.e. packed input 16 (i / 16) + 4 (i % 4) + (i % 16) / 4), so the packed chain is the dense one without its
    // zero terms -- each fma(w, 0, acc) = acc -- and equal bit for bit.
    std::vector<int> chain;
    for (int ch = 0; 16 * ch < n; ++ch)
        for (int st = 0; st < 4; ++st)
            for (int hh = 0; hh < 4; ++hh) {
                const int k = 16 * ch + 4 * hh + st;
                if (k < n && mask[k]) chain.push_back(k);
            }
    if (chain.empty()) chain.push_back(0);                       // (an all-zero view: one zero-weight row)
    const int K = (int)chain.size(), nch = (K + 15) / 16;
    std::vector<int> orig((size_t)nch * 16, -1);                 // packed input -> view float (-1: a zero pad row)
    for (int i = 0; i < K; ++i) orig[16 * (i / 16) + 4 * (i % 4) + (i % 16) / 4] = chain[i];
    std::vector<uint32_t> desc((size_t)(nch + 2) * 8, 0u);
    for (int ch = 0; ch < nch + 2; ++ch) {
        int base = chain[K - 1];
        for (int j = 0; j < 16 && ch < nch; ++j)
            if (orig[16 * ch + j] >= 0) base = std::min(base, orig[16 * ch + j]);
        desc[8 * ch + 4] = (uint32_t)base;
        for (int j = 0; j < 16; ++j) {
            const int o = ch < nch && orig[16 * ch + j] >= 0 ? orig[16 * ch + j] : base;   // (pad rows: zero weights)
            if (o - base > 255) return fail("acnet_set_input_support: packed chunk %d spans %d floats", ch, o - base + 1);
            desc[8 * ch + j / 4] |= (uint32_t)(o - base) << (8 * (j % 4));
        }
    }
    std::vector<int> rows((size_t)nch * 16);                     // wv row of packed input p (pads: a zero row)
    for (int p = 0; p < nch * 16; ++p) rows[p] = orig[p] >= 0 ? orig[p] : -1;
    const int KR = nch * 16;                                     // packed rows, pads included
    const size_t nimg = img_floats(KR, kAH / 16);
    if (hipMalloc(&q->vperm, sizeof(int) * KR) != hipSuccess || hipMalloc(&q->vdesc, sizeof(uint32_t) * desc.size()) != hipSuccess ||
        hipMalloc(&q->vrows, sizeof(float) * KR * kAH) != hipSuccess || hipMalloc(&q->vimg, sizeof(float) * nimg) != hipSuccess) {
        acnet_support_free(q);
        return fail("acnet_set_input_support: hipMalloc");
    }
    MFX_HIP(hipMemcpy(q->vperm, rows.data(), sizeof(int) * KR, hipMemcpyHostToDevice));
    MFX_HIP(hipMemcpy(q->vdesc, desc.data(), sizeof(uint32_t) * desc.size(), hipMemcpyHostToDevice));
    q->vK = KR;
    q->vKn = K;
    return acnet_support_image(q, (hipStream_t)stream);
}

// Inputs the view layer runs over (0: the dense order).
MFX_API int mfx_acnet_input_support_size(void* handle, int* k) {
    *k = static_cast<ACNetHandle*>(handle)->vKn;
    return 0;
}

static int acnet_run(ACNetHandle* q, const float* view, size_t view_ld, const float* feat, size_t feat_ld,
                     const void* prob, int prob_f64, size_t prob_ld, QRowMap rm, int n, const int32_t* d_n,
                     float* policy, float* value, int32_t* act, uint32_t seed, uint32_t step, int group, hipStream_t st) {
    if (n <= 0) return 0;
    if (q->dev.use_mf && value && !prob) return fail("acnet: the mean-field value head needs prob");
    // persistent workgroups: as many as the CUs hold at once (two per CU with h_emb in LDS), at most one per tile
    int grid = (n + 16 * kQHeadWaves - 1) / (16 * kQHeadWaves);
    const bool lds = q->dev.Fp <= kHeF;                             // (wider features: h_emb held in registers)
    const bool img = q->imaged;
    grid = std::min(grid, (lds ? 2 : 1) * device_cus());
#define MFX_ACNET_LAUNCH1(PT, MF, LDS, IMG, PK, PB)                                                                     \
    k_acnet<PT, MF, LDS, IMG, PK><<<grid, 256, IMG && LDS ? kAcnetImgLdsSmem : (LDS ? kAcnetLdsSmem : kQHeadSmem),     \
                                    st>>>(q->dev, view, view_ld, feat, feat_ld, PB, prob_ld, rm, n, d_n, policy, value,   \
                                          act, seed, step, group)
    // (the packed view order: the image path with h_emb in LDS -- the view-ring form -- and a support set)
#define MFX_ACNET_LAUNCH(PT, MF, LDS, PB)                                                                              \
    do {                                                                                                              \
        if (img && LDS && q->dev.vdesc) MFX_ACNET_LAUNCH1(PT, MF, LDS, true, LDS, PB);                               \
        else if (img) MFX_ACNET_LAUNCH1(PT, MF, LDS, true, false, PB);                                                \
        else MFX_ACNET_LAUNCH1(PT, MF, LDS, false, false, PB);                                                        \
    } while (0)
    const double* pd = static_cast<const double*>(prob);
    const float* pf = static_cast<const float*>(prob);
    // (kMF selects only the value head: without value_out both forms compute the same policy, and the plain one
    // holds fewer registers)
    if (!value) {
        if (lds) MFX_ACNET_LAUNCH(float, false, true, pf); else MFX_ACNET_LAUNCH(float, false, false, pf);
    } else if (q->dev.use_mf && prob_f64) {
        if (lds) MFX_ACNET_LAUNCH(double, true, true, pd); else MFX_ACNET_LAUNCH(double, true, false, pd);
    } else if (q->dev.use_mf) {
        if (lds) MFX_ACNET_LAUNCH(float, true, true, pf); else MFX_ACNET_LAUNCH(float, true, false, pf);
    } else {
        if (lds) MFX_ACNET_LAUNCH(float, false, true, pf); else MFX_ACNET_LAUNCH(float, false, false, pf);
    }
#undef MFX_ACNET_LAUNCH
#undef MFX_ACNET_LAUNCH1
    MFX_HIP(hipGetLastError());
    return 0;
}

// n agents, dense rows: view [n][V], feature [n][F], prob [n][A] float32 (the MF value head; else null).
// policy [n][A], value [n], act [n]: any may be null.  The draw of row i uses (seed, step, group 0, row i).
MFX_API int mfx_acnet_forward(void* handle, const float* d_view, const float* d_feat, const float* d_prob, int n,
                              float* d_policy, float* d_value, int32_t* d_act, uint32_t seed, uint32_t step,
                              void* stream) {
    auto* q = static_cast<ACNetHandle*>(handle);
    QRowMap rm{nullptr, 1, 0, 0};
    return acnet_run(q, d_view, q->dev.V, d_feat, q->dev.F, d_prob, 0, q->dev.A, rm, n, nullptr, d_policy, d_value,
                     d_act, seed, step, 0, (hipStream_t)stream);
}

// Group g of a rollout batch (as mfx_qnet_act_rollout): sampled actions into d_act [E][G][rowcap] for the group's
// live rows, row j of env e drawn with (seed, step, g, e * rowcap + j).  Nothing is read back.
MFX_API int mfx_acnet_act_rollout(void* handle, const float* d_view, const float* d_feat, const int32_t* d_counts,
                                  int E, int G, int g, int rowcap, int32_t* d_rows, int32_t* d_total, int32_t* d_act,
                                  uint32_t seed, uint32_t step, void* stream) {
    auto* q = static_cast<ACNetHandle*>(handle);
    hipStream_t st = (hipStream_t)stream;
    MFX_HIP(launch_rollout_rows(d_counts, E, G, g, rowcap, d_rows, d_total, st));
    QRowMap rm{d_rows, rowcap, G * rowcap, g * rowcap};
    return acnet_run(q, d_view, q->dev.V, d_feat, q->dev.F, nullptr, 0, 0, rm, E * rowcap, d_total, nullptr, nullptr,
                     d_act, seed, step, g, st);
}

}  // extern "C"
