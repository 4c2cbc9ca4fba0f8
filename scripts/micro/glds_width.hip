// Where global_load_lds of 1 / 2 / 4 bytes writes in LDS (measured: 1 and 2 bytes land zero-extended, one dword per
// lane at base + 4 lane, not at base + lane x size): 64 lanes load word i (value 0x11110000 + i) with the
// given width into a 512-B LDS area pre-filled with 0xEE; the area is dumped as 32-bit words.
//   hipcc -O3 --offload-arch=gfx950 -o glds_width scripts/micro/glds_width.hip && ./glds_width
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int SZ>
__global__ void k(const unsigned* src, unsigned* out) {
    __shared__ unsigned buf[128];
    const int l = threadIdx.x;
    buf[l] = 0xEEEEEEEEu;
    buf[l + 64] = 0xEEEEEEEEu;
    __syncthreads();
    auto* d = (__attribute__((address_space(3))) void*)buf;
    if (SZ == 1) __builtin_amdgcn_global_load_lds((const void*)(src + l), d, 1, 0, 0);
    if (SZ == 2) __builtin_amdgcn_global_load_lds((const void*)(src + l), d, 2, 0, 0);
    if (SZ == 4) __builtin_amdgcn_global_load_lds((const void*)(src + l), d, 4, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    out[l] = buf[l];
    out[l + 64] = buf[l + 64];
}
int main() {
    unsigned h[64], *s, *o, r[128];
    for (int i = 0; i < 64; ++i) h[i] = 0x11110000u + i;
    hipMalloc(&s, 256); hipMalloc(&o, 512);
    hipMemcpy(s, h, 256, hipMemcpyHostToDevice);
    k<1><<<1, 64>>>(s, o); hipMemcpy(r, o, 512, hipMemcpyDeviceToHost);
    printf("size 1: %08x %08x %08x %08x | %08x %08x\n", r[0], r[1], r[2], r[3], r[16], r[64]);
    k<2><<<1, 64>>>(s, o); hipMemcpy(r, o, 512, hipMemcpyDeviceToHost);
    printf("size 2: %08x %08x %08x %08x | %08x %08x %08x\n", r[0], r[1], r[2], r[3], r[31], r[32], r[64]);
    k<4><<<1, 64>>>(s, o); hipMemcpy(r, o, 512, hipMemcpyDeviceToHost);
    printf("size 4: %08x %08x %08x %08x | %08x %08x\n", r[0], r[1], r[2], r[63], r[64], r[65]);
    return 0;
}
