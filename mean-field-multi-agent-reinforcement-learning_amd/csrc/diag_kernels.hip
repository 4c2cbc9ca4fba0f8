// Diagnostics only (not on any product path): the request -> completion round trip of a one-wave
// resident server polling coherent host memory, run inside whatever process loaded the library, to
// separate the signalling floor from the drop-in kernel's own costs (scripts/stamps_dropin.py).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include "mfx_common.h"

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
}  // namespace

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
