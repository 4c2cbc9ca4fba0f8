// Round trip of one tiny launch on MI355X: host launch -> kernel publishes a word in host-mapped
// coherent memory -> host sees it (the floor of the drop-in's one-launch env.step()), against
// hipStreamSynchronize / hipEventSynchronize after the same launch.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>

__global__ void k_signal(uint32_t* word, uint32_t seq, int work) {
    __shared__ float acc[256];
    float x = threadIdx.x;
    for (int i = 0; i < work; ++i) x = x * 1.0001f + 0.5f;
    acc[threadIdx.x] = x;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(word, seq + (acc[5] < -1.0f), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint32_t *h = nullptr, *d = nullptr;
    CK(hipHostMalloc((void**)&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&d, h, 0));
    h[0] = 0;
    const int N = 20000;
    for (int work : {0, 2000}) {
        for (int mode = 0; mode < 3; ++mode) {
            uint32_t seq = 0;
            for (int i = 0; i < 200; ++i) { k_signal<<<1, 256, 0, st>>>(d, ++seq, work); CK(hipStreamSynchronize(st)); }
            hipEvent_t ev;
            CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            auto t0 = std::chrono::steady_clock::now();
            double launch_ns = 0;
            for (int i = 0; i < N; ++i) {
                auto a = std::chrono::steady_clock::now();
                k_signal<<<1, 256, 0, st>>>(d, ++seq, work);
                launch_ns += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - a).count();
                if (mode == 0) { while (*(volatile uint32_t*)h != seq) __builtin_ia32_pause(); }
                else if (mode == 1) CK(hipStreamSynchronize(st));
                else { CK(hipEventRecord(ev, st)); CK(hipEventSynchronize(ev)); }
            }
            CK(hipStreamSynchronize(st));
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
            printf("work %d  %-22s %.2f us per launch round trip (launch call %.2f us)\n", work,
                   mode == 0 ? "spin on mapped word" : mode == 1 ? "hipStreamSynchronize" : "hipEventSynchronize", us,
                   launch_ns / N / 1000.0);
            CK(hipEventDestroy(ev));
        }
    }
    return 0;
}
