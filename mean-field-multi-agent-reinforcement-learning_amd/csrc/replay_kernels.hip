// replay_kernels.hip -- the data path of the replay buffers (algo/tools.py:26-70 MetaBuffer, :118-173
// EpisodesBuffer, :218-362 MemoryGroup push / tight / sample) on device: every one of those operations
// moves whole rows of several columns (view 4,732 B, features, action, reward, terminal, mask, mean action)
// from one set of row positions to another -- a gather from a source index list (optionally modulo the
// source length, MetaBuffer.sample's idx % length) into consecutive destination rows (optionally a ring:
// MetaBuffer.append's wrap at max_len).  One launch moves every column of a batch of rows; the index
// lists themselves (the agent grouping, the reference's np.random draws) are computed by the caller.
// HBM-bound: 2 x the row bytes per row (read + write), coalesced dword / 16-B accesses along each row.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_common.h"
#include "../../include/magent_amd.h"

namespace mfx {

constexpr int kRowCols = 8;

struct RowCols {
    char* dst[kRowCols];
    const char* src[kRowCols];
    int64_t bytes[kRowCols];
    int n;
};

// Workgroup b copies rows b, b + grid, ...; each column with the widest access its alignment allows.
__global__ void __launch_bounds__(256) k_rows_copy(RowCols c, const int64_t* __restrict__ idx, int64_t src_mod,
                                                   int64_t dst_start, int64_t dst_cap, int64_t n) {
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        int64_t s = idx ? idx[i] : i;
        if (src_mod > 0) s = ((s % src_mod) + src_mod) % src_mod;
        const int64_t d = dst_cap > 0 ? (dst_start + i) % dst_cap : dst_start + i;
        for (int k = 0; k < c.n; ++k) {
            const int64_t b = c.bytes[k];
            const char* sp = c.src[k] + s * b;
            char* dp = c.dst[k] + d * b;
            if (((uintptr_t)sp | (uintptr_t)dp | (uintptr_t)b) % 16 == 0) {
                const uint4* s4 = reinterpret_cast<const uint4*>(sp);
                uint4* d4 = reinterpret_cast<uint4*>(dp);
                for (int64_t q = threadIdx.x; q < b / 16; q += blockDim.x) d4[q] = s4[q];
            } else if (((uintptr_t)sp | (uintptr_t)dp | (uintptr_t)b) % 4 == 0) {
                const uint32_t* s1 = reinterpret_cast<const uint32_t*>(sp);
                uint32_t* d1 = reinterpret_cast<uint32_t*>(dp);
                for (int64_t q = threadIdx.x; q < b / 4; q += blockDim.x) d1[q] = s1[q];
            } else {
                for (int64_t q = threadIdx.x; q < b; q += blockDim.x) dp[q] = sp[q];
            }
        }
    }
}

}  // namespace mfx

using namespace mfx;

extern "C" {

// For i in [0, n): row s = idx ? idx[i] : i (taken modulo src_mod when src_mod > 0) of every source column
// to row d = dst_start + i (modulo dst_cap when dst_cap > 0) of the destination column.  n_cols <= 8;
// row_bytes[k]: bytes per row of column k.  Destination rows of one call must be distinct (a ring shorter
// than n would make two rows race for a slot: the caller skips the rows a ring would overwrite).
MFX_API int mfx_rows_copy(int n_cols, void* const* dst, const void* const* src, const int64_t* row_bytes,
                          const int64_t* d_idx, int64_t src_mod, int64_t dst_start, int64_t dst_cap, int64_t n,
                          void* stream) {
    if (n_cols < 1 || n_cols > kRowCols) return fail("rows_copy: 1..%d columns, got %d", kRowCols, n_cols);
    if (n < 0 || (dst_cap > 0 && n > dst_cap)) return fail("rows_copy: %lld rows into a ring of %lld", (long long)n,
                                                           (long long)dst_cap);
    if (n == 0) return 0;
    RowCols c{};
    c.n = n_cols;
    for (int k = 0; k < n_cols; ++k) {
        if (!dst[k] || !src[k] || row_bytes[k] <= 0) return fail("rows_copy: column %d is empty", k);
        c.dst[k] = static_cast<char*>(dst[k]);
        c.src[k] = static_cast<const char*>(src[k]);
        c.bytes[k] = row_bytes[k];
    }
    const int grid = (int)(n < 65536 ? n : 65536);
    k_rows_copy<<<grid, 256, 0, (hipStream_t)stream>>>(c, d_idx, src_mod, dst_start, dst_cap, n);
    MFX_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
