// Write-bandwidth ceiling of the observation store pattern on one MI355X (diagnostic, not product).
//   hipcc --offload-arch=gfx950 -O3 write_ceiling.hip -o write_ceiling && ./write_ceiling
// Each wave streams `piece` bytes per iteration (the k_rollout obs flush is 1792 B: one 1 KiB
// dwordx4 store + one 768 B store), pieces of one workgroup's waves interleaved like the kernel's
// stream; persistent grid of `wgs` workgroups of 256 lanes.  nt = nontemporal stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool kNt>
__global__ void __launch_bounds__(256) k_write(f32x4* __restrict__ out, size_t n16, int piece16) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const size_t step = (size_t)gridDim.x * nw * piece16;
    f32x4 v = {1.0f, 2.0f, (float)lane, 0.0f};
    for (size_t base = ((size_t)blockIdx.x * nw + wid) * piece16; base + piece16 <= n16; base += step) {
        for (int i = lane; i < piece16; i += 64) {
            if (kNt) __builtin_nontemporal_store(v, out + base + i);
            else out[base + i] = v;
        }
    }
}

int main() {
    const size_t bytes = 4ull << 30, n16 = bytes / 16;
    f32x4* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int pieces[] = {112, 256, 1024, 4096};          // 16-B rows: 1792 B, 4 KiB, 16 KiB, 64 KiB
    const int per_cu[] = {2, 5, 8};
    for (int nt = 0; nt < 2; ++nt)
        for (int p : pieces)
            for (int k : per_cu) {
                const int wgs = cus * k;
                float best = 1e30f;
                for (int r = 0; r < 5; ++r) {
                    hipEventRecord(a);
                    if (nt) k_write<true><<<wgs, 256>>>(out, n16, p);
                    else k_write<false><<<wgs, 256>>>(out, n16, p);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    if (r && ms < best) best = ms;
                }
                printf("nt=%d piece=%6d B  wg/cu=%d  %.2f TB/s\n", nt, p * 16, k, bytes / (best * 1e-3) / 1e12);
            }
    return 0;
}
