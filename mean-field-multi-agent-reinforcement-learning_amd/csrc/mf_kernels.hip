// mf_kernels.hip -- mean-field pieces of the training loop, on device.
//
//  * mean-action pooling   senario_battle.py:141  former_act_prob = mean(one_hot(acts)) (float64)
//  * MF-Q target           algo/base.py:192-220   r + (1 - done) * Q_tgt(s', argmax Q_eval(s')) * gamma
//  * MF-AC returns         algo/ac.py:305-320     keep = keep * gamma + r[i], backwards per episode
// Each follows the reference's numpy dtype rules and operation order (-ffp-contract=off).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mfx_common.h"
#include "../../include/magent_amd.h"

namespace mfx {

// One workgroup per group row: histogram in LDS, then count / n in float64 (np.mean of one-hot
// rows sums exact 0/1 values, so the result is exactly count / n).
__global__ void __launch_bounds__(256) k_mean_action(const int32_t* __restrict__ acts, const int32_t* __restrict__ counts,
                                                     int rowcap, int n_action, double* __restrict__ out) {
    __shared__ int hist[256];
    const int b = blockIdx.x, n = counts[b];
    for (int k = threadIdx.x; k < n_action; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int a = acts[(size_t)b * rowcap + i];
        if (a >= 0 && a < n_action) atomicAdd(&hist[a], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n_action; k += blockDim.x)
        out[(size_t)b * n_action + k] = n ? (double)hist[k] / (double)n : __longlong_as_double(0x7FF8000000000000ll);
}

// One lane per sample.  np.argmax: first maximum, and the first NaN wins if any.
__global__ void __launch_bounds__(256) k_mfq_target(const float* __restrict__ e_q, const float* __restrict__ t_q,
                                                    const float* __restrict__ r, const uint8_t* __restrict__ done,
                                                    int M, int A, double gamma, double* __restrict__ out) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const float* row = e_q + (size_t)m * A;
    int best = 0;
    float bv = row[0];
    if (!isnan(bv)) {
        for (int k = 1; k < A; ++k) {
            const float x = row[k];
            if (isnan(x)) { best = k; break; }
            if (x > bv) { bv = x; best = k; }
        }
    }
    const double q = (double)t_q[(size_t)m * A + best];
    const double notdone = 1.0 - (done[m] ? 1.0 : 0.0);
    out[m] = (double)r[m] + (notdone * q) * gamma;
}

// One lane per episode: rewards[offsets[e] .. offsets[e+1]) are replaced by their discounted
// returns, bootstrapped from value[e] (algo/ac.py:312-320: keep = keep * gamma + r[i]; r[i] = keep).
// numpy1 = 1: the reference's NumPy-1 promotion (its TF1 era) -- np.float32 * python float is float64,
// so keep runs in float64 from the first step on and each r[i] is keep rounded to float32.
// numpy1 = 0: NEP 50 (NumPy 2) -- keep stays float32 and gamma is rounded to float32 first.
// Both pinned by tests/golden/algo_mfac_returns.npz (the reference's own loop, make_algo_fixtures.py).
__global__ void __launch_bounds__(256) k_mfac_returns(float* __restrict__ rew, const int64_t* __restrict__ offsets,
                                                      const float* __restrict__ value, int n_ep, double gamma,
                                                      int numpy1) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_ep) return;
    if (numpy1) {
        double keep = (double)value[e];
        for (int64_t i = offsets[e + 1] - 1; i >= offsets[e]; --i) {
            const double t = keep * gamma;
            keep = t + (double)rew[i];
            rew[i] = (float)keep;
        }
    } else {
        const float g = (float)gamma;
        float keep = value[e];
        for (int64_t i = offsets[e + 1] - 1; i >= offsets[e]; --i) {
            const float t = keep * g;
            keep = t + rew[i];
            rew[i] = keep;
        }
    }
}

}  // namespace mfx

extern "C" {

// Device pointers; stream may be null (the null stream).  acts [B][rowcap], counts [B] -> out [B][n_action]
MFX_API int mfx_mean_action(const int32_t* d_acts, const int32_t* d_counts, int B, int rowcap, int n_action,
                            double* d_out, void* stream) {
    if (n_action < 1 || n_action > 256) return mfx::fail("mean_action: 1 <= n_action <= 256");
    if (B == 0) return 0;
    mfx::k_mean_action<<<B, 256, 0, (hipStream_t)stream>>>(d_acts, d_counts, rowcap, n_action, d_out);
    MFX_HIP(hipGetLastError());
    return 0;
}

// e_q, t_q [M][A] f32, r [M] f32, done [M] u8 -> target [M] f64
MFX_API int mfx_mfq_target(const float* d_eq, const float* d_tq, const float* d_r, const uint8_t* d_done, int M, int A,
                           double gamma, double* d_out, void* stream) {
    if (A < 1) return mfx::fail("mfq_target: A must be >= 1");
    if (M == 0) return 0;
    mfx::k_mfq_target<<<(M + 255) / 256, 256, 0, (hipStream_t)stream>>>(d_eq, d_tq, d_r, d_done, M, A, gamma, d_out);
    MFX_HIP(hipGetLastError());
    return 0;
}

// rewards (in place) [offsets[n_ep]] f32, offsets [n_ep + 1] i64, value [n_ep] f32
MFX_API int mfx_mfac_returns(float* d_rew, const int64_t* d_offsets, const float* d_value, int n_ep, double gamma,
                             int numpy1, void* stream) {
    if (n_ep < 0) return mfx::fail("mfac_returns: n_ep must be >= 0");
    if (n_ep == 0) return 0;
    mfx::k_mfac_returns<<<(n_ep + 255) / 256, 256, 0, (hipStream_t)stream>>>(d_rew, d_offsets, d_value, n_ep, gamma,
                                                                             numpy1 != 0);
    MFX_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
