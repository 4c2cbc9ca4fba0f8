// Request -> completion round trip through a resident one-wave server on MI355X, by where the request
// word lives: coherent host memory (the GPU polls across the bus) or fine-grained device memory the
// host writes through its BAR mapping (the GPU polls its own memory).  The completion word is in
// coherent host memory in both cases.  One wave, no barriers: lane 0 polls and answers.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>

__global__ void k_echo(const uint32_t* req, uint32_t* done, unsigned long long idle) {
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

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static int ping(const char* name, volatile uint32_t* hreq, const uint32_t* dreq, volatile uint32_t* hdone,
                uint32_t* ddone, hipStream_t st, unsigned long long idle) {
    *hreq = 0;
    *hdone = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    k_echo<<<1, 64, 0, st>>>(dreq, ddone, idle);
    CK(hipGetLastError());
    const int N = 20000;
    double total = 0;
    for (uint32_t i = 1; i <= N + 500; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        *hreq = i;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        for (uint64_t k = 0; *hdone != i; ++k) {
            __builtin_ia32_pause();
            if (k == (1ull << 25)) {
                printf("%s: request %u unanswered (done %u)\n", name, i, *hdone);
                *hreq = 0xFFFFFFFFu;
                return 1;
            }
        }
        if (i > 500) total += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    *hreq = 0xFFFFFFFFu;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(st));
    printf("%-40s %.2f us per round trip\n", name, total / N);
    return 0;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int dev = 0, khz = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    const unsigned long long idle = (unsigned long long)khz * 100;           // 100 ms
    uint32_t *h = nullptr, *d = nullptr;
    CK(hipHostMalloc((void**)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&d, h, 0));
    // request at h[0], completion at h[64] (another 256-B line)
    if (ping("request in coherent host memory", h, d, h + 64, d + 64, st, idle)) return 1;
    uint32_t* f = nullptr;
    CK(hipExtMallocWithFlags((void**)&f, 4096, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, f));
    uint32_t* fh = (uint32_t*)(at.hostPointer ? at.hostPointer : f);
    printf("fine-grained device memory: device %p host %p\n", (void*)f, (void*)at.hostPointer);
    fh[0] = 7;                             // a host store through that pointer (a fault ends the run here)
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    printf("host store to fine-grained device memory: read back %u\n", fh[0]);
    if (ping("request in fine-grained device memory", fh, f, h + 64, d + 64, st, idle)) return 1;
    return 0;
}
