// replay_kernels.hip -- the data path of the replay buffers (algo/tools.py:26-70 MetaBuffer, :118-173
// EpisodesBuffer, :218-362 MemoryGroup push / tight / sample) on device: every one of those operations
// moves whole rows of several columns (view 4,732 B, features, action, reward, terminal, mask, mean action)
// from one set of row positions to another -- a gather from a source index list (optionally modulo the
// source length, MetaBuffer.sample's idx % length) into consecutive destination rows (optionally a ring:
// MetaBuffer.append's wrap at max_len).  One launch moves every column of a batch of rows; the index
// lists themselves (the agent grouping, the reference's np.random draws) are computed by the caller.
// HBM-bound: 2 x the row bytes per row (read + write), coalesced dword / 16-B accesses along each row, one
// wave per row with its loads in flight ahead of its stores (scripts/bench_replay.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "mfx_common.h"
#include "../../include/magent_amd.h"

namespace mfx {

constexpr int kRowCols = 8;
#ifndef MFX_ROWS_PER_CU
#define MFX_ROWS_PER_CU 2            // k_rows_pipe workgroups per CU (A/B builds: make variant VFLAGS=-DMFX_ROWS_PER_CU=n)
#endif
constexpr int64_t kBigRow = 512;          // columns at least this wide get a per-column vector loop

struct RowCols {
    char* dst[kRowCols];
    const char* src[kRowCols];
    int64_t bytes[kRowCols];
    int n;
    // The narrow columns (feature rows, actions, rewards, flags, mean actions) are moved together: the lanes
    // of a wave take consecutive units of all of them at once -- unit u of column k is its
    // (u - ustart[k])-th dword when the column's rows are 4-B aligned (ubytes 4), else its byte (ubytes 1).
    // Wide columns (the view) have ubytes 0 and no units.
    int ustart[kRowCols + 1];
    int ubytes[kRowCols];
};

// dwords [0, nd) of one row: 20 loads per lane in flight before their stores (a 4,732-B view row in one pass)
constexpr int kCopyU4 = 20, kCopyU16 = 5;
__device__ __forceinline__ void row_copy4(const uint32_t* __restrict__ sp, uint32_t* __restrict__ dp, int64_t nd,
                                          int lane) {
    for (int64_t base = 0; base < nd; base += 64 * kCopyU4) {
        uint32_t r[kCopyU4];
#pragma unroll
        for (int u = 0; u < kCopyU4; ++u) {
            const int64_t q = base + lane + 64 * u;
            if (q < nd) r[u] = sp[q];
        }
#pragma unroll
        for (int u = 0; u < kCopyU4; ++u) {
            const int64_t q = base + lane + 64 * u;
            if (q < nd) dp[q] = r[u];
        }
    }
}

__device__ __forceinline__ void row_copy16(const uint4* __restrict__ sp, uint4* __restrict__ dp, int64_t nq, int lane) {
    for (int64_t base = 0; base < nq; base += 64 * kCopyU16) {
        uint4 r[kCopyU16];
#pragma unroll
        for (int u = 0; u < kCopyU16; ++u) {
            const int64_t q = base + lane + 64 * u;
            if (q < nq) r[u] = sp[q];
        }
#pragma unroll
        for (int u = 0; u < kCopyU16; ++u) {
            const int64_t q = base + lane + 64 * u;
            if (q < nq) dp[q] = r[u];
        }
    }
}

// The first out-of-range source index the row movers met: the workgroup whose compare-and-swap sets the flag
// stores the index (any int64, -1 included); read and cleared by mfx_rows_copy_error.  A bad row is skipped,
// never read.
__device__ unsigned int g_rows_bad_flag;
__device__ long long g_rows_bad_index;

__device__ __forceinline__ void rows_bad(int64_t raw) {
    if (atomicCAS(&g_rows_bad_flag, 0u, 1u) == 0u) g_rows_bad_index = (long long)raw;
}

// The source row of index raw: modulo src_mod when > 0 (the rings), else numpy's indexing of src_rows rows
// (-src_rows..-1 count from the end); -1 when out of range.
__device__ __forceinline__ int64_t rows_src(int64_t raw, int64_t src_mod, int64_t src_rows) {
    int64_t s = raw;
    if (src_mod > 0) { s %= src_mod; if (s < 0) s += src_mod; }
    else if (s < 0) s += src_rows;
    return (s < 0 || s >= src_rows) ? -1 : s;
}

// One wave per row (four rows per workgroup): row s = idx ? idx[i] : i (modulo src_mod) of every column to
// row d = dst_start + i (modulo dst_cap).  The narrow columns in one pass of unit loads, then each wide
// column with its loads issued ahead of its stores -- a row is ~5 KB, so a wave keeps 2 KB in flight.
// Source rows outside [0, src_rows) are skipped and reported (g_rows_bad).
__global__ void __launch_bounds__(256) k_rows_copy(RowCols c, const int64_t* __restrict__ idx, int64_t src_mod,
                                                   int64_t src_rows, int64_t dst_start, int64_t dst_cap, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += waves) {
        const int64_t raw = idx ? idx[i] : i;
        const int64_t s = rows_src(raw, src_mod, src_rows);
        if (s < 0) {
            if (lane == 0) rows_bad(raw);
            continue;
        }
        int64_t d = dst_start + i;
        if (dst_cap > 0 && d >= dst_cap) d %= dst_cap;
        for (int u = lane; u < c.ustart[kRowCols]; u += 64) {
            int k = 0;
            while (u >= c.ustart[k + 1]) ++k;
            const int64_t b = c.bytes[k], off = u - c.ustart[k];
            if (c.ubytes[k] == 4)
                *reinterpret_cast<uint32_t*>(c.dst[k] + d * b + 4 * off) =
                    *reinterpret_cast<const uint32_t*>(c.src[k] + s * b + 4 * off);
            else
                c.dst[k][d * b + off] = c.src[k][s * b + off];
        }
        for (int k = 0; k < c.n; ++k) {
            if (c.ubytes[k]) continue;
            const int64_t b = c.bytes[k];
            const char* sp = c.src[k] + s * b;
            char* dp = c.dst[k] + d * b;
            const uintptr_t al = (uintptr_t)sp | (uintptr_t)dp | (uintptr_t)b;
            if ((al & 15) == 0) {
                row_copy16(reinterpret_cast<const uint4*>(sp), reinterpret_cast<uint4*>(dp), b / 16, lane);
            } else if ((al & 3) == 0) {
                row_copy4(reinterpret_cast<const uint32_t*>(sp), reinterpret_cast<uint32_t*>(dp), b / 4, lane);
            } else {
                for (int64_t q = lane; q < b; q += 64) dp[q] = sp[q];
            }
        }
    }
}

// The same move, software-pipelined, for the common shape (MemoryGroup.sample, tight, push: at most one wide
// column, 4-B aligned, <= 64 x 4 kPipeQ + 3 dwords per row, and at most 64 narrow units): each wave keeps two rows in
// flight -- row k + 1's loads are issued before row k's stores, so the in-order vmcnt of gfx9 lets the stores
// of one row drain under the loads of the next instead of serialising load -> store per row -- and reads its row
// indices through scalar loads (the row is wave-uniform), which wait on lgkmcnt, not behind the data loads.
// The wide column moves in 16-B units at its rows' 4-B alignment (global_load / store_dwordx4 need only dword
// alignment on gfx950: one 1-KiB wave-instruction per 1 KiB of row, where dword units took four 256-B ones; +1.5 %,
// profiles/r06_replay_ab.txt), its last wdw % 4 dwords by single lanes.
constexpr int kPipeQ = 5;
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
struct PipeRow {
    int64_t s, d;
    bool ok;
    uint32_t u;                    // this lane's narrow unit (dword, or byte in the low 8 bits)
    u32x4a4 q[kPipeQ];             // this lane's 16-B units of the wide column
    uint32_t t;                    // this lane's tail dword
};

__global__ void __launch_bounds__(256) k_rows_pipe(RowCols c, int wk, int64_t wdw, const int64_t* __restrict__ idx,
                                                   int64_t src_mod, int64_t src_rows, int64_t dst_start,
                                                   int64_t dst_cap, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t W = (int64_t)gridDim.x * 4;
    const int64_t first = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int units = c.ustart[kRowCols];
    // this lane's narrow unit: column, byte offset, width (fixed for the whole launch)
    int uk = -1, uoff = 0, uw = 0;
    if (lane < units) {
        uk = 0;
        while (lane >= c.ustart[uk + 1]) ++uk;
        uw = c.ubytes[uk];
        uoff = (lane - c.ustart[uk]) * uw;
    }
    auto locate = [&](int64_t i, PipeRow& r) {
        r.ok = i < n;
        if (!r.ok) return;
        const int64_t raw = idx ? idx[i] : i;              // wave-uniform: a scalar load
        const int64_t s = rows_src(raw, src_mod, src_rows);
        if (s < 0) {
            if (lane == 0) rows_bad(raw);
            r.ok = false;
            return;
        }
        int64_t d = dst_start + i;
        if (dst_cap > 0 && d >= dst_cap) d %= dst_cap;
        r.s = s;
        r.d = d;
    };
    auto fetch = [&](PipeRow& r) {
        if (!r.ok) return;
        if (uk >= 0) {
            const char* sp = c.src[uk] + r.s * c.bytes[uk] + uoff;
            r.u = uw == 4 ? *reinterpret_cast<const uint32_t*>(sp) : (uint32_t)*reinterpret_cast<const uint8_t*>(sp);
        }
        if (wk >= 0) {
            const uint32_t* sp = reinterpret_cast<const uint32_t*>(c.src[wk] + r.s * c.bytes[wk]);
            const int64_t nq = wdw >> 2;
#pragma unroll
            for (int j = 0; j < kPipeQ; ++j) {
                const int64_t q = lane + 64 * j;
                if (q < nq) r.q[j] = reinterpret_cast<const u32x4a4*>(sp)[q];
            }
            if (lane < (wdw & 3)) r.t = sp[4 * nq + lane];
        }
    };
    auto put = [&](const PipeRow& r) {
        if (!r.ok) return;
        if (uk >= 0) {
            char* dp = c.dst[uk] + r.d * c.bytes[uk] + uoff;
            if (uw == 4) *reinterpret_cast<uint32_t*>(dp) = r.u;
            else *reinterpret_cast<uint8_t*>(dp) = (uint8_t)r.u;
        }
        if (wk >= 0) {
            uint32_t* dp = reinterpret_cast<uint32_t*>(c.dst[wk] + r.d * c.bytes[wk]);
            const int64_t nq = wdw >> 2;
#pragma unroll
            for (int j = 0; j < kPipeQ; ++j) {
                const int64_t q = lane + 64 * j;
                if (q < nq) reinterpret_cast<u32x4a4*>(dp)[q] = r.q[j];
            }
            if (lane < (wdw & 3)) dp[4 * nq + lane] = r.t;
        }
    };
    PipeRow a, b;
    int64_t i = first;
    locate(i, a);
    fetch(a);
    while (i < n) {
        const int64_t i1 = i + W;
        locate(i1, b);
        fetch(b);                                          // row i1 in flight ...
        put(a);                                            // ... while row i drains
        if (i1 >= n) break;
        const int64_t i2 = i1 + W;
        locate(i2, a);
        fetch(a);
        put(b);
        i = i2;
    }
}

}  // namespace mfx

using namespace mfx;

extern "C" {

// For i in [0, n): row s = idx ? idx[i] : i (taken modulo src_mod when src_mod > 0) of every source column
// to row d = dst_start + i (modulo dst_cap when dst_cap > 0) of the destination column.  n_cols <= 8;
// row_bytes[k]: bytes per row of column k.  Destination rows of one call must be distinct (a ring shorter
// than n would make two rows race for a slot: the caller skips the rows a ring would overwrite).
// src_rows: rows every source column holds; without src_mod an index in [-src_rows, 0) counts from the end (numpy's
// indexing); any other index outside [0, src_rows) skips its row and is reported by mfx_rows_copy_error.
MFX_API int mfx_rows_copy(int n_cols, void* const* dst, const void* const* src, const int64_t* row_bytes,
                          const int64_t* d_idx, int64_t src_mod, int64_t src_rows, int64_t dst_start, int64_t dst_cap,
                          int64_t n, void* stream) {
    if (n_cols < 1 || n_cols > kRowCols) return fail("rows_copy: 1..%d columns, got %d", kRowCols, n_cols);
    if (src_mod > src_rows) return fail("rows_copy: modulo %lld over %lld source rows", (long long)src_mod,
                                        (long long)src_rows);
    if (!d_idx && n > src_rows) return fail("rows_copy: %lld rows from %lld source rows", (long long)n,
                                            (long long)src_rows);
    if (n < 0 || (dst_cap > 0 && n > dst_cap)) return fail("rows_copy: %lld rows into a ring of %lld", (long long)n,
                                                           (long long)dst_cap);
    if (n == 0) return 0;
    RowCols c{};
    c.n = n_cols;
    int units = 0;
    for (int k = 0; k < n_cols; ++k) {
        if (!dst[k] || !src[k] || row_bytes[k] <= 0) return fail("rows_copy: column %d is empty", k);
        c.dst[k] = static_cast<char*>(dst[k]);
        c.src[k] = static_cast<const char*>(src[k]);
        c.bytes[k] = row_bytes[k];
        c.ustart[k] = units;
        if (row_bytes[k] >= kBigRow) {
            c.ubytes[k] = 0;
        } else {
            const bool a4 = (((uintptr_t)dst[k] | (uintptr_t)src[k] | (uintptr_t)row_bytes[k]) & 3) == 0;
            c.ubytes[k] = a4 ? 4 : 1;
            units += (int)(row_bytes[k] / c.ubytes[k]);
        }
    }
    for (int k = n_cols; k <= kRowCols; ++k) c.ustart[k] = units;
    // the pipelined form takes at most one wide column (4-B aligned, <= 64 x 4 kPipeQ + 3 dwords) and <= 64 units
    int wide = -1, n_wide = 0;
    for (int k = 0; k < n_cols; ++k)
        if (!c.ubytes[k]) { wide = k; ++n_wide; }
    const bool pipe = n_wide <= 1 && units <= 64 &&
                      (wide < 0 || ((((uintptr_t)dst[wide] | (uintptr_t)src[wide] | (uintptr_t)row_bytes[wide]) & 3) == 0 &&
                                    row_bytes[wide] / 4 <= 64 * 4 * kPipeQ + 3));
    const char* pe = getenv("MFX_ROWS_PIPE");              // 0: the one-row-per-wave form (tests)
    const int use_pipe = pe ? atoi(pe) : 1;
    const int64_t wgs = (n + 3) / 4;
    if (pipe && use_pipe) {
        // persistent-sized grid, each wave walking its rows two in flight
        static const int cus = [] {
            int dev = 0, n_cu = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
            return n_cu;
        }();
        // 2 workgroups per CU with the 16-B units: 0.573-0.577 of the HBM peak on the MF-Q sample against 0.565 at 4
        // and 0.49 at 8 (profiles/r06_replay_ab.txt; round 4 with dword units: 0.555-0.559 at 4, 0.464 / 0.520 at 7
        // / 14, 0.510-0.537 for the one-row-per-wave form; four rows loaded then stored, and nontemporal stores, lost:
        // profiles/r04_replay_ab.txt)
        const int64_t cap = (int64_t)cus * MFX_ROWS_PER_CU;
        const int grid = (int)(wgs < cap ? wgs : cap);
        const int64_t wdw = wide >= 0 ? row_bytes[wide] / 4 : 0;
        k_rows_pipe<<<grid, 256, 0, (hipStream_t)stream>>>(c, wide, wdw, d_idx, src_mod, src_rows, dst_start, dst_cap, n);
        MFX_HIP(hipGetLastError());
        return 0;
    }
    const int grid = (int)(wgs < 65536 ? wgs : 65536);
    k_rows_copy<<<grid, 256, 0, (hipStream_t)stream>>>(c, d_idx, src_mod, src_rows, dst_start, dst_cap, n);
    MFX_HIP(hipGetLastError());
    return 0;
}

// Synchronises `stream`; *bad_index = the first out-of-range source index any k_rows_copy met since the last
// call (-1: none), and the word is cleared.  Returns -1 (with the message) when one was met.
MFX_API int mfx_rows_copy_error(int64_t* bad_index, void* stream) {
    unsigned int flag = 0;
    long long h = -1;
    MFX_HIP(hipStreamSynchronize((hipStream_t)stream));
    MFX_HIP(hipMemcpyFromSymbol(&flag, HIP_SYMBOL(g_rows_bad_flag), sizeof(flag), 0, hipMemcpyDeviceToHost));
    *bad_index = -1;
    if (!flag) return 0;
    MFX_HIP(hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_rows_bad_index), sizeof(h), 0, hipMemcpyDeviceToHost));
    *bad_index = (int64_t)h;
    const unsigned int z = 0;
    MFX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rows_bad_flag), &z, sizeof(z), 0, hipMemcpyHostToDevice));
    return fail("rows_copy: source index %lld out of range (row skipped)", (long long)*bad_index);
}

}  // extern "C"
