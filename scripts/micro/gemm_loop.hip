// The k_acnet view-layer loop alone (policy_gemm.h wg_gemm_i, MT = 16, K = 1184, 64 agents per 4-wave workgroup,
// two workgroups per CU) and variants of it, to see what the loop structure costs by itself:
//   mode 0  wg_gemm_i as k_acnet runs it (image chunk direct-to-LDS a chunk ahead, vmcnt(0) + barrier per chunk)
//   mode 1  the same loop body without the barrier (timing only: reads may be stale)
//   mode 2  without the image loads (LDS reused; timing only)
//   mode 3  neither (MFMAs + LDS reads only)
//   mode 4  mode 0 with waves 2-3 of each workgroup at s_setprio 1
//   mode 5  three chunk buffers, the image two chunks ahead (vmcnt leaves the newest chunk in flight)
//   mode 6  mode 5 with a bare s_barrier (after lgkmcnt(0)) in place of __syncthreads(), whose release fence makes
//           the compiler drain every load -- the chunk in flight too -- before the barrier
//   mode 7  mode 0 with the bare barrier
//   mode 8  mode 0 with 8-wave workgroups (128 agents, one per CU): half the image traffic per MFMA
//   mode 9  mode 8, waves 4-7 at s_setprio 1
// B operands come from registers (no view traffic).  Prints TF/s and the fraction of the f32 MFMA peak.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o gemm_loop scripts/micro/gemm_loop.hip && ./gemm_loop
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../mean-field-multi-agent-reinforcement-learning_amd/csrc/policy_gemm.h"

using namespace mfx;

template <int MODE, int NT = 256>
__device__ __forceinline__ void gemm_var(const float* __restrict__ img, int K, float* bsm, f32x4* acc, float vb) {
    constexpr int MT = 16, RW = img_row(MT), CF4 = 16 * RW / 4, G = MT / 4;
    const int tid = tid_x(), lane = tid & 63, h = lane >> 4, c = lane & 15, wid = tid >> 6;
    const int nchunk = (K + 15) / 16;
    constexpr bool kDma = MODE == 0 || MODE == 1 || MODE >= 4;
    constexpr bool kBar = MODE == 0 || MODE == 2 || MODE >= 4;
    constexpr bool kBare = MODE == 6 || MODE == 7, kDeep = MODE == 5 || MODE == 6;
    constexpr int NB = kDeep ? 3 : 2;
    auto issue = [&](int ch) {
        float* dst = bsm + (ch % NB) * kImgBuf;
        const float* src = img + (size_t)ch * CF4 * 4;
#pragma unroll
        for (int q = 0; q < CF4; q += NT)
            __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)(q + tid) * 4),
                                             (__attribute__((address_space(3))) void*)(dst + (q + wid * 64) * 4), 16, 0, 0);
    };
    const int cb = c * MT, sw = c * G / 16;
    auto read_row = [&](const float* cur, int kr, float* dst) {
        const float* src = cur + kr * RW + cb;
#pragma unroll
        for (int t4 = 0; t4 < G; ++t4) {
            const float4 x = reinterpret_cast<const float4*>(src)[(t4 + sw) % G];
            dst[4 * t4] = x.x; dst[4 * t4 + 1] = x.y; dst[4 * t4 + 2] = x.z; dst[4 * t4 + 3] = x.w;
        }
    };
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
    if (kDma) issue(0);
    if (kDeep) {
        issue(1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int ch = 0; ch < nchunk; ++ch) {
        const float* cur = bsm + (kDma ? (ch % NB) * kImgBuf : 0);
        if (kDeep) {
            if (ch + 2 < nchunk) issue(ch + 2);
        } else if (kDma && ch + 1 < nchunk) {
            issue(ch + 1);
        }
        float av[MT], an[MT];
        read_row(cur, 4 * h, av);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float v = vb + (float)(4 * ch + s);
            if (s + 1 < 4) read_row(cur, 4 * h + s + 1, an);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[t] = mfma4(av[t], v, acc[t]);
#pragma unroll
            for (int t = 0; t < MT; ++t) av[t] = an[t];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (kDeep) {
            if (ch + 2 < nchunk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (kDma) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (kBare) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        } else if (kBar) {
            __syncthreads();
        }
    }
}

template <int MODE>
__global__ void __launch_bounds__(512, 1) k_loop8(const float* __restrict__ img, int K, int tiles, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float bsm[];
    if (MODE == 9 && (threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);
    f32x4 acc[16];
    float sum = 0.f;
    for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        gemm_var<MODE, 512>(img, K, bsm, acc, (float)tile * 1e-3f);
#pragma unroll
        for (int t = 0; t < 16; ++t) sum += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
    }
    out[blockIdx.x * 512 + threadIdx.x] = sum;
}

template <int MODE>
__global__ void __launch_bounds__(256, 2) k_loop(const float* __restrict__ img, int K, int tiles, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float bsm[];
    if (MODE == 4 && (threadIdx.x >> 6) >= 2) __builtin_amdgcn_s_setprio(1);
    f32x4 acc[16];
    float sum = 0.f;
    for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        gemm_var<MODE>(img, K, bsm, acc, (float)tile * 1e-3f);
#pragma unroll
        for (int t = 0; t < 16; ++t) sum += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
    }
    out[blockIdx.x * 256 + threadIdx.x] = sum;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE>
void run(const float* img, int K, float* out, int grid, int tiles) {
    constexpr bool w8 = MODE >= 8;
    const size_t smem = w8 ? 160 * 1024 : 80 * 1024;
    const void* fn = w8 ? (const void*)k_loop8<MODE> : (const void*)k_loop<MODE>;
    CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    if (w8) { grid /= 2; tiles /= 2; }
    auto launch = [&] {
        if (w8) k_loop8<MODE><<<grid, 512, smem>>>(img, K, tiles, out);
        else k_loop<MODE><<<grid, 256, smem>>>(img, K, tiles, out);
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double flop = (double)tiles * (w8 ? 128 : 64) * ((K + 15) / 16 * 16) * 256 * 2;
    const double tf = flop / (best * 1e-3) / 1e12;
    printf("mode %d: grid %d tiles %d  %.3f ms  %.1f TF/s  frac %.3f\n", MODE, grid, tiles, best, tf, tf / 157.3);
}

int main() {
    const int K = 1184, tiles = 4096;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t n = img_floats(K, 16);
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    float *img, *out;
    CK(hipMalloc(&img, n * 4));
    CK(hipMalloc(&out, (size_t)2 * cus * 256 * 4));
    CK(hipMemcpy(img, h.data(), n * 4, hipMemcpyHostToDevice));
    const int grid = 2 * cus;
    run<0>(img, K, out, grid, tiles);
    run<0>(img, K, out, grid, tiles);
    run<5>(img, K, out, grid, tiles);
    run<1>(img, K, out, grid, tiles);
    run<2>(img, K, out, grid, tiles);
    run<3>(img, K, out, grid, tiles);
    run<4>(img, K, out, grid, tiles);
    run<0>(img, K, out, grid, tiles);
    run<5>(img, K, out, grid, tiles);
    run<6>(img, K, out, grid, tiles);
    run<7>(img, K, out, grid, tiles);
    run<8>(img, K, out, grid, tiles);
    run<9>(img, K, out, grid, tiles);
    run<8>(img, K, out, grid, tiles);
    run<0>(img, K, out, grid, tiles);
    return 0;
}
