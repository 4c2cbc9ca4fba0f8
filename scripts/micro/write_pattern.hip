// Write-bandwidth ceiling of k_rollout's OWN store pattern (diagnostic, not product):
//   hipcc --offload-arch=gfx950 -O3 write_pattern.hip -o write_pattern && ./write_pattern
// Each workgroup (256 lanes, persistent grid of `per_cu` per CU) takes regions of `region` bytes (one
// group's view rows of one env: 128 agents x 4,732 B = 605,696 B), region b, b + grid, ...; inside a
// region its 4 waves stream 1792-B pieces, two consecutive pieces per wave per iteration, the waves
// interleaved (wave w takes pieces 2w, 2w+1, then 2w+8, ... -- obs_stream_battle).  nt: nontemporal.
// Also the round-1 micro's global round-robin of 1792-B pieces and a plain fill, for reference.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kPiece16 = 112;                    // 1792 B

template <bool kNt>
__device__ __forceinline__ void put(f32x4* p, f32x4 v) {
    if (kNt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool kNt>
__global__ void __launch_bounds__(256) k_regions(f32x4* __restrict__ out, size_t n_regions, size_t region16) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const f32x4 v = {1.0f, 2.0f, (float)lane, 0.0f};
    const size_t pieces = region16 / kPiece16;
    for (size_t r = blockIdx.x; r < n_regions; r += gridDim.x) {
        f32x4* base = out + r * region16;
        for (size_t p = (size_t)wid * 2; p < pieces; p += (size_t)nw * 2) {
            for (int k = 0; k < 2 && p + k < pieces; ++k) {
                f32x4* d = base + (p + k) * kPiece16;
                put<kNt>(d + lane, v);
                if (lane < kPiece16 - 64) put<kNt>(d + 64 + lane, v);
            }
        }
    }
}

template <bool kNt>
__global__ void __launch_bounds__(256) k_roundrobin(f32x4* __restrict__ out, size_t n16) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const f32x4 v = {1.0f, 2.0f, (float)lane, 0.0f};
    const size_t step = (size_t)gridDim.x * nw * kPiece16;
    for (size_t b = ((size_t)blockIdx.x * nw + wid) * kPiece16; b + kPiece16 <= n16; b += step) {
        put<kNt>(out + b + lane, v);
        if (lane < kPiece16 - 64) put<kNt>(out + b + 64 + lane, v);
    }
}

__global__ void __launch_bounds__(256) k_fill(f32x4* __restrict__ out, size_t n16) {
    const f32x4 v = {1.0f, 2.0f, 3.0f, 0.0f};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        out[i] = v;
}

int main() {
    const size_t region = 605696, n_regions = 6000, bytes = region * n_regions, n16 = bytes / 16;
    f32x4* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](auto launch) {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (r && ms < best) best = ms;
        }
        return bytes / (best * 1e-3) / 1e12;
    };
    printf("bytes per launch %.2f GB, %d CUs\n", bytes / 1e9, cus);
    for (int k : {5, 8}) {
        const int g = cus * k;
        printf("regions      nt=1 wg/cu=%d  %.2f TB/s\n", k, timeit([&] { k_regions<true><<<g, 256>>>(out, n_regions, region / 16); }));
        printf("regions      nt=0 wg/cu=%d  %.2f TB/s\n", k, timeit([&] { k_regions<false><<<g, 256>>>(out, n_regions, region / 16); }));
        printf("round-robin  nt=1 wg/cu=%d  %.2f TB/s\n", k, timeit([&] { k_roundrobin<true><<<g, 256>>>(out, n16); }));
    }
    printf("fill (grid-stride float4)       %.2f TB/s\n", timeit([&] { k_fill<<<cus * 8, 256>>>(out, n16); }));
    return 0;
}
