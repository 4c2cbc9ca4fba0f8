// Bit-exactness check of the cross-lane wave sum (observe.inc wave_sum): the permlane-swap + DPP form against the
// ds_bpermute butterfly (x += shfl_xor(x, o), o = 32 .. 1), on random f32 vectors of mixed magnitudes and signs.
// Build: hipcc --offload-arch=gfx950 -O3 wave_sum.hip -o wave_sum; prints mismatching lanes (0 expected) and timings.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

template <int kCtrl>
__device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), kCtrl, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_fast(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(q[0]) + __uint_as_float(q[1]);
    x += dpp<0x128>(x);     // row_ror:8
    x += dpp<0x124>(x);     // row_ror:4
    x += dpp<0x4E>(x);      // quad_perm [2,3,0,1]
    x += dpp<0xB1>(x);      // quad_perm [1,0,3,2]
    return x;
}
__device__ __forceinline__ float wave_sum_ref(float x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__global__ void k_check(const float* in, float* out, int n) {
    const int t = threadIdx.x & 63, w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= n) return;
    const float x = in[w * 64 + t];
    out[(w * 64 + t) * 2] = wave_sum_fast(x);
    out[(w * 64 + t) * 2 + 1] = wave_sum_ref(x);
}
// the DPP inclusive scan of step_big.inc (wave_incl_scan) against a serial prefix
template <int kCtrl, int kRows = 0xF>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, kRows, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += dpp_u32<0x111>(x);
    x += dpp_u32<0x112>(x);
    x += dpp_u32<0x114>(x);
    x += dpp_u32<0x118>(x);
    x += dpp_u32<0x142, 0xA>(x);
    x += dpp_u32<0x143, 0xC>(x);
    return x;
}
__global__ void k_scan(const uint32_t* in, uint32_t* out, int n) {
    const int t = threadIdx.x & 63, w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= n) return;
    out[w * 64 + t] = wave_incl_scan(in[w * 64 + t]);
}
template <bool kFast>
__global__ void k_chain(float* io, int iters) {
    float x = io[threadIdx.x];
    for (int i = 0; i < iters; ++i) x = (kFast ? wave_sum_fast(x) : wave_sum_ref(x)) * 0.015625f;
    io[threadIdx.x] = x;
}
int main() {
    const int n = 1 << 16;
    std::vector<float> h(n * 64);
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::uniform_int_distribution<int> ex(-30, 30);
    for (auto& v : h) v = std::ldexp(u(g), ex(g) / ((g() & 3) + 1));
    float *d_in, *d_out;
    hipMalloc(&d_in, h.size() * 4);
    hipMalloc(&d_out, h.size() * 8);
    hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    k_check<<<n / 4, 256>>>(d_in, d_out, n);
    std::vector<float> o(h.size() * 2);
    hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (size_t i = 0; i < h.size(); ++i)
        if (std::memcmp(&o[2 * i], &o[2 * i + 1], 4) != 0) ++bad;
    printf("wave_sum permlane/DPP vs butterfly: %ld mismatching lanes of %zu\n", bad, h.size());
    {
        std::vector<uint32_t> hi(h.size()), ho(h.size());
        for (auto& v : hi) v = g() & 0xFFFF;
        uint32_t *d_i, *d_o;
        hipMalloc(&d_i, hi.size() * 4);
        hipMalloc(&d_o, hi.size() * 4);
        hipMemcpy(d_i, hi.data(), hi.size() * 4, hipMemcpyHostToDevice);
        k_scan<<<n / 4, 256>>>(d_i, d_o, n);
        hipMemcpy(ho.data(), d_o, ho.size() * 4, hipMemcpyDeviceToHost);
        long sbad = 0;
        for (int w = 0; w < n; ++w) {
            uint32_t acc = 0;
            for (int l = 0; l < 64; ++l) { acc += hi[w * 64 + l]; if (ho[w * 64 + l] != acc) ++sbad; }
        }
        printf("wave_incl_scan DPP vs serial prefix: %ld mismatching lanes of %zu\n", sbad, hi.size());
        bad += sbad;
    }
    float* d_io;
    hipMalloc(&d_io, 256);
    hipMemcpy(d_io, h.data(), 256, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int f = 0; f < 2; ++f) {
        const int it = 1 << 16;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (f) k_chain<true><<<1, 64>>>(d_io, it); else k_chain<false><<<1, 64>>>(d_io, it);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("%s: %.1f ns per dependent wave sum\n", f ? "permlane/DPP" : "butterfly", ms * 1e6 / it);
        }
    }
    return bad ? 1 : 0;
}
