// Measurement only (not on any product path):
// * the request -> completion round trip of a one-wave resident server polling coherent host memory, run
//   inside whatever process loaded the library, to separate the signalling floor from the drop-in kernel's
//   own costs (scripts/stamps_dropin.py);
// * the HBM write ceiling measured in the same process as the bench (mfx_store_ceiling): a write-only
//   float4 stream of a given byte count over a given device region, in the store shapes that reach the
//   card's highest write rate, so that bench.py can report the kernel's fraction of a ceiling measured on
//   the same box and run next to its nominal 8 TB/s fraction.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include "mfx_common.h"
#include "../../include/magent_amd.h"

namespace {
__global__ void k_diag_echo(const uint32_t* req, uint32_t* done, unsigned long long idle) {
    if (threadIdx.x != 0) return;
    uint32_t seq = 0;
    unsigned long long t0 = wall_clock64();
    for (uint32_t polls = 0; polls < (1u << 24); ++polls) {
        const uint32_t r = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (r == 0xFFFFFFFFu) break;
        if (r != seq) {
            seq = r;
            __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            t0 = wall_clock64();
            continue;
        }
        if (wall_clock64() - t0 > idle) break;
    }
}
// Write-only stream: each iteration a workgroup stores one contiguous chunk of kU x 4 KiB (kU float4 per lane, 1 KiB
// per wave-instruction).  kPersist: a grid of CUs x 8 workgroups strides over the region; else one workgroup per chunk
// (the shape torch's fill reaches ~6.9 TB/s with, profiles/r03_write_ceilings.txt).  kNt: nontemporal stores
// (k_rollout's observation stores are nt).
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <bool kNt, bool kPersist, int kU>
__global__ void __launch_bounds__(256) k_store_ceiling(f32x4_t* __restrict__ out, size_t n_chunks) {
    const f32x4_t v = {1.0f, (float)threadIdx.x, 2.0f, 3.0f};
    size_t c = blockIdx.x;
    const size_t stride = kPersist ? gridDim.x : n_chunks;
    for (; c < n_chunks; c += stride) {
        f32x4_t* p = out + c * 256 * kU + threadIdx.x;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (kNt) __builtin_nontemporal_store(v, p + 256 * u);
            else p[256 * u] = v;
        }
    }
}

template <bool kNt, bool kPersist, int kU>
hipError_t store_pass(f32x4_t* base, size_t chunks, int grid_p, hipStream_t st) {
    if (kPersist) {
        k_store_ceiling<kNt, true, kU><<<(unsigned)std::min<size_t>(chunks, (size_t)grid_p), 256, 0, st>>>(base, chunks);
        return hipGetLastError();
    }
    const size_t win = (size_t)1 << 20;                   // one-chunk-per-workgroup launches: <= 2^20 workgroups
    for (size_t off = 0; off < chunks; off += win) {
        const size_t n = std::min(chunks - off, win);
        k_store_ceiling<kNt, false, kU><<<(unsigned)n, 256, 0, st>>>(base + off * 256 * kU, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
}  // namespace

// Write `total_bytes` over the device region [d_buf, d_buf + region_bytes) (16-B aligned, wrapping: passes of
// at most region_bytes) in store shape `shape` (0..7: bit 0 nontemporal stores; bits 1-2: 0 / 1 / 2 = 4 / 8 / 16 KiB
// chunks, one workgroup per chunk, 3 = 4 KiB chunks on a persistent grid), on `stream`; *ms = the HIP-event time of
// all passes (synchronises).  The region's contents are overwritten.
extern "C" __attribute__((visibility("default"))) int mfx_store_ceiling(void* d_buf, size_t region_bytes,
                                                                         size_t total_bytes, int shape, void* stream,
                                                                         float* ms) {
    if (!d_buf || ((uintptr_t)d_buf & 15) || region_bytes < 16384 || shape < 0 || shape > 7 || !ms)
        return mfx::fail("store_ceiling: bad arguments (buffer %p, region %zu B, shape %d)", d_buf, region_bytes, shape);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int form = shape >> 1;
    const size_t chunk = form == 1 ? 8192 : form == 2 ? 16384 : 4096;
    const size_t region_chunks = region_bytes / chunk;
    const int grid_p = mfx::device_cus() * 8;
    hipEvent_t a, b;
    MFX_HIP(hipEventCreate(&a));
    MFX_HIP(hipEventCreate(&b));
    MFX_HIP(hipEventRecord(a, st));
    size_t left = total_bytes / chunk;
    f32x4_t* base = static_cast<f32x4_t*>(d_buf);
    while (left) {
        const size_t pass = left < region_chunks ? left : region_chunks;
        hipError_t e;
        switch (shape) {
            case 0: e = store_pass<false, false, 1>(base, pass, grid_p, st); break;
            case 1: e = store_pass<true, false, 1>(base, pass, grid_p, st); break;
            case 2: e = store_pass<false, false, 2>(base, pass, grid_p, st); break;
            case 3: e = store_pass<true, false, 2>(base, pass, grid_p, st); break;
            case 4: e = store_pass<false, false, 4>(base, pass, grid_p, st); break;
            case 5: e = store_pass<true, false, 4>(base, pass, grid_p, st); break;
            case 6: e = store_pass<false, true, 1>(base, pass, grid_p, st); break;
            default: e = store_pass<true, true, 1>(base, pass, grid_p, st); break;
        }
        MFX_HIP(e);
        left -= pass;
    }
    MFX_HIP(hipEventRecord(b, st));
    MFX_HIP(hipEventSynchronize(b));
    MFX_HIP(hipEventElapsedTime(ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 0;
}

// n round trips; *us = mean microseconds per round trip.  fence: an mfence after each request store.
extern "C" __attribute__((visibility("default"))) int mfx_diag_poll_rtt(int n, int fence, double* us) {
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return -1;
    uint32_t *h = nullptr, *d = nullptr;
    if (hipHostMalloc((void**)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return -1;
    if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) return -1;
    volatile uint32_t* hreq = h;
    volatile uint32_t* hdone = h + 64;
    *hreq = 0;
    *hdone = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    int dev = 0, khz = 100000;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    k_diag_echo<<<1, 64, 0, st>>>(d, d + 64, (unsigned long long)khz * 100);
    double total = 0;
    int rc = 0;
    for (uint32_t i = 1; i <= (uint32_t)n + 100; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        if (fence) { *hreq = i; __atomic_thread_fence(__ATOMIC_SEQ_CST); }
        else __atomic_store_n(const_cast<uint32_t*>(hreq), i, __ATOMIC_RELEASE);
        uint64_t k = 0;
        while (*hdone != i && ++k < (1ull << 27)) __builtin_ia32_pause();
        if (*hdone != i) { rc = -2; break; }
        if (i > 100) total += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    *hreq = 0xFFFFFFFFu;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    (void)hipStreamSynchronize(st);
    (void)hipHostFree(h);
    (void)hipStreamDestroy(st);
    *us = total / n;
    return rc;
}
