// Which store shapes reach the fill ceiling? (diagnostic, not product)
//   hipcc --offload-arch=gfx950 -O3 write_shapes.hip -o write_shapes && ./write_shapes
// Every kernel writes the same 3.6 GB with 16-B stores; they differ in who writes what when:
//   chunkN_uU   : non-persistent grid, workgroup i writes the contiguous chunk i of N bytes; each lane
//                 U float4 per loop trip, a wave instruction = 1 KiB contiguous (lane-contiguous)
//   lanevecU    : non-persistent, each lane U consecutive float4 (lane stride U*16 B)
//   persist...  : the same chunks taken by a persistent grid (5 per CU): chunk b, b + grid, ...
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int kChunk16, int kU, bool kNt, bool kPersist>
__global__ void __launch_bounds__(256) k_chunks(f32x4* __restrict__ out, size_t n_chunks) {
    const f32x4 v = {1.0f, 2.0f, (float)threadIdx.x, 0.0f};
    for (size_t c = blockIdx.x; c < n_chunks; c += kPersist ? gridDim.x : n_chunks) {
        f32x4* base = out + c * kChunk16;
        for (int i = threadIdx.x; i < kChunk16; i += 256 * kU) {
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int k = i + u * 256;
                if (k < kChunk16) {
                    if (kNt) __builtin_nontemporal_store(v, base + k);
                    else base[k] = v;
                }
            }
        }
        if (!kPersist) break;
    }
}

template <int kU>
__global__ void __launch_bounds__(256) k_lanevec(f32x4* __restrict__ out, size_t n16) {
    const f32x4 v = {1.0f, 2.0f, (float)threadIdx.x, 0.0f};
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * kU;
#pragma unroll
    for (int u = 0; u < kU; ++u)
        if (i + u < n16) out[i + u] = v;
}

int main() {
    const size_t bytes = 3633ull << 20, n16 = bytes / 16;
    f32x4* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch) {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            (void)hipEventRecord(a);
            launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (r && ms < best) best = ms;
        }
        printf("%-28s %.2f TB/s\n", name, bytes / (best * 1e-3) / 1e12);
    };
#define CH(N16, U, NT)                                                                                      \
    timeit("chunk" #N16 "x16B_u" #U "_nt" #NT, [&] { k_chunks<N16, U, NT, false><<<(unsigned)(n16 / N16), 256>>>(out, n16 / N16); }); \
    timeit("persist" #N16 "x16B_u" #U "_nt" #NT, [&] { k_chunks<N16, U, NT, true><<<cus * 5, 256>>>(out, n16 / N16); });
    CH(256, 1, false)
    CH(1024, 4, false)
    CH(1024, 4, true)
    CH(4096, 4, false)
    CH(4096, 16, false)
    CH(448, 2, false)
    CH(448, 2, true)
    CH(896, 4, true)
    timeit("lanevec4", [&] { k_lanevec<4><<<(unsigned)(n16 / 1024), 256>>>(out, n16); });
    timeit("lanevec8", [&] { k_lanevec<8><<<(unsigned)(n16 / 2048), 256>>>(out, n16); });
    return 0;
}
