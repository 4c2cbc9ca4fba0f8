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

constexpr int kRowCols = 12;
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
    // Columns with bit k set read source row idx[i] + shift_by instead of idx[i] (before the modulo):
    // MemoryGroup.sample's next-state columns at next_idx = (idx + 1) % nb_entries (tools.py:241), moved in the
    // same launch as the current-state columns -- rows idx and idx + 1 are adjacent in the ring.
    uint32_t shift;
    int64_t shift_by;
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
    if (src_mod > 0) {
        if ((uint64_t)raw <= 0xffffffffull && src_mod <= 0xffffffffll)   // the common case: a 32-bit remainder
            s = (uint32_t)raw % (uint32_t)src_mod;
        else { s %= src_mod; if (s < 0) s += src_mod; }
    }
    else if (s < 0) s += src_rows;
    return (s < 0 || s >= src_rows) ? -1 : s;
}

// Source rows of entry raw: s0 for the unshifted columns, s1 for the shifted ones; false (reported) when one
// is out of range.
__device__ __forceinline__ bool rows_src2(const RowCols& c, int64_t raw, int64_t src_mod, int64_t src_rows,
                                          int64_t& s0, int64_t& s1, int lane) {
    s0 = rows_src(raw, src_mod, src_rows);
    if (!c.shift) s1 = s0;
    else if (src_mod > 0 && c.shift_by >= 0 && c.shift_by < src_mod) {   // (s0 + shift) mod src_mod, no division
        s1 = s0 + c.shift_by;
        if (s1 >= src_mod) s1 -= src_mod;
    } else s1 = rows_src(raw + c.shift_by, src_mod, src_rows);
    if (s0 >= 0 && s1 >= 0) return true;
    if (lane == 0) rows_bad(s0 < 0 ? raw : raw + c.shift_by);
    return false;
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
        int64_t s0, s1;
        if (!rows_src2(c, raw, src_mod, src_rows, s0, s1, lane)) continue;
        int64_t d = dst_start + i;
        if (dst_cap > 0 && d >= dst_cap) d %= dst_cap;
        for (int u = lane; u < c.ustart[kRowCols]; u += 64) {
            int k = 0;
            while (u >= c.ustart[k + 1]) ++k;
            const int64_t b = c.bytes[k], off = u - c.ustart[k];
            const int64_t s = (c.shift >> k & 1) ? s1 : s0;
            if (c.ubytes[k] == 4)
                *reinterpret_cast<uint32_t*>(c.dst[k] + d * b + 4 * off) =
                    *reinterpret_cast<const uint32_t*>(c.src[k] + s * b + 4 * off);
            else
                c.dst[k][d * b + off] = c.src[k][s * b + off];
        }
        for (int k = 0; k < c.n; ++k) {
            if (c.ubytes[k]) continue;
            const int64_t b = c.bytes[k], s = (c.shift >> k & 1) ? s1 : s0;
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

// The same move, software-pipelined, for the common shapes (MemoryGroup.sample with its next-state columns, tight,
// push: at most two wide columns, 4-B aligned, <= 64 x 4 kPipeQ + 3 dwords per row, and at most 64 kPipeU narrow
// units): each wave keeps two rows in flight -- row k + 1's loads are issued before row k's stores, so the in-order
// vmcnt of gfx9 lets the stores of one row drain under the loads of the next instead of serialising load -> store
// per row -- and reads its row indices through scalar loads (the row is wave-uniform), which wait on lgkmcnt, not
// behind the data loads.  The wide columns move in 16-B units at their rows' 4-B alignment (global_load /
// store_dwordx4 need only dword alignment on gfx950: one 1-KiB wave-instruction per 1 KiB of row, where dword units
// took four 256-B ones; +1.5 %, profiles/r06_replay_ab.txt), their last dw % 4 dwords by single lanes.  A fused
// sample (view at idx and at idx + 1) reads 9.5 KB of adjacent ring rows per entry in one wave.
// kDepth rows in flight per wave: 3 and 4 measured no faster than 2 (profiles/r06_replay_ab.txt)
constexpr int kPipeQ = 5, kPipeW = 2, kPipeU = 2, kDepth = 2;
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
struct PipeWide {                  // the wide columns, resolved on the host (no dynamic indexing of RowCols)
    const char* src[kPipeW];       // nullptr when slot w is unused
    char* dst[kPipeW];
    int64_t bytes[kPipeW], dw[kPipeW];
    bool shifted[kPipeW];
};
template <int NW, int NU>
struct PipeRow {
    const char* us[NU];        // this lane's narrow unit source addresses (row chosen in locate: a select of
    const uint32_t* ws[NW];        // values -- a select between two fields of the row made the rows scratch-resident)
    int64_t d;
    bool ok;
    uint32_t u[NU];                // this lane's narrow units (dword, or byte in the low 8 bits)
    u32x4a4 q[NW][kPipeQ];         // this lane's 16-B units of the wide columns
    uint32_t t[NW];                // this lane's tail dwords
};

// NW wide columns (slots past the used ones are empty), NU narrow units per lane: compiled per shape, the one-wide
// one-unit form (tight, push, unfused samples) keeps round 6's 60 VGPRs.
template <int NW, int NU>
__global__ void __launch_bounds__(256) k_rows_pipe(RowCols c, PipeWide wd, const int64_t* __restrict__ idx,
                                                   int64_t src_mod, int64_t src_rows, int64_t dst_start,
                                                   int64_t dst_cap, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t W = (int64_t)gridDim.x * 4;
    const int64_t first = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int units = c.ustart[kRowCols];
    // this lane's narrow units lane + 64 j: column, width, shifted or not, base pointers (fixed for the launch)
    const char* usrc[NU];
    char* udst[NU];
    int64_t ub[NU];
    int uw[NU];
    bool ush[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) {
        const int u = lane + 64 * j;
        uw[j] = 0;
        usrc[j] = nullptr;
        udst[j] = nullptr;
        ub[j] = 0;
        ush[j] = false;
#pragma unroll
        for (int k = 0; k < kRowCols; ++k) {                // constant column indices: selects, not a scratch copy
            if (u >= c.ustart[k] && u < c.ustart[k + 1]) {
                uw[j] = c.ubytes[k];
                ub[j] = c.bytes[k];
                ush[j] = c.shift >> k & 1;
                usrc[j] = c.src[k] + (int64_t)(u - c.ustart[k]) * c.ubytes[k];
                udst[j] = c.dst[k] + (int64_t)(u - c.ustart[k]) * c.ubytes[k];
            }
        }
    }
    auto locate = [&](int64_t i, PipeRow<NW, NU>& r) {
        r.ok = i < n;
        if (!r.ok) return;
        const int64_t raw = idx ? idx[i] : i;              // wave-uniform: a scalar load
        int64_t s0, s1;
        r.ok = rows_src2(c, raw, src_mod, src_rows, s0, s1, lane);
#pragma unroll
        for (int j = 0; j < NU; ++j) r.us[j] = usrc[j] + (ush[j] ? s1 : s0) * ub[j];
#pragma unroll
        for (int w = 0; w < NW; ++w)
            r.ws[w] = reinterpret_cast<const uint32_t*>(wd.src[w] + (wd.shifted[w] ? s1 : s0) * wd.bytes[w]);
        int64_t d = dst_start + i;
        if (dst_cap > 0 && d >= dst_cap) d %= dst_cap;
        r.d = d;
    };
    auto fetch = [&](PipeRow<NW, NU>& r) {
        if (!r.ok) return;
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            if (!uw[j]) continue;
            const char* sp = r.us[j];
            r.u[j] = uw[j] == 4 ? *reinterpret_cast<const uint32_t*>(sp) : (uint32_t)*reinterpret_cast<const uint8_t*>(sp);
        }
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            if (!wd.src[w]) continue;
            const uint32_t* sp = r.ws[w];
            const int64_t nq = wd.dw[w] >> 2;
#pragma unroll
            for (int j = 0; j < kPipeQ; ++j) {
                const int64_t q = lane + 64 * j;
                if (q < nq) r.q[w][j] = reinterpret_cast<const u32x4a4*>(sp)[q];
            }
            if (lane < (wd.dw[w] & 3)) r.t[w] = sp[4 * nq + lane];
        }
    };
    auto put = [&](const PipeRow<NW, NU>& r) {
        if (!r.ok) return;
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            if (!uw[j]) continue;
            char* dp = udst[j] + r.d * ub[j];
            if (uw[j] == 4) *reinterpret_cast<uint32_t*>(dp) = r.u[j];
            else *reinterpret_cast<uint8_t*>(dp) = (uint8_t)r.u[j];
        }
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            if (!wd.src[w]) continue;
            uint32_t* dp = reinterpret_cast<uint32_t*>(wd.dst[w] + r.d * wd.bytes[w]);
            const int64_t nq = wd.dw[w] >> 2;
#pragma unroll
            for (int j = 0; j < kPipeQ; ++j) {
                const int64_t q = lane + 64 * j;
                if (q < nq) reinterpret_cast<u32x4a4*>(dp)[q] = r.q[w][j];
            }
            if (lane < (wd.dw[w] & 3)) dp[4 * nq + lane] = r.t[w];
        }
    };
    // kDepth rows in flight per wave: row i + (kDepth - 1) W is issued before row i's stores (slots rotate; the
    // unrolled loop keeps every slot index a constant, so the rows stay in registers)
    PipeRow<NW, NU> r[kDepth];
#pragma unroll
    for (int k = 0; k < kDepth - 1; ++k) {
        locate(first + k * W, r[k]);
        fetch(r[k]);
    }
    int64_t i = first;
    while (i < n) {
#pragma unroll
        for (int k = 0; k < kDepth; ++k) {
            PipeRow<NW, NU>& ahead = r[(k + kDepth - 1) % kDepth];
            locate(i + (kDepth - 1) * W, ahead);
            fetch(ahead);                                  // rows i + W .. in flight ...
            put(r[k]);                                     // ... while row i drains
            i += W;
            if (i >= n) break;
        }
    }
}

}  // namespace mfx

using namespace mfx;

extern "C" {

// For i in [0, n): row s = idx ? idx[i] : i (taken modulo src_mod when src_mod > 0) of every source column
// to row d = dst_start + i (modulo dst_cap when dst_cap > 0) of the destination column.  n_cols <= 12;
// row_bytes[k]: bytes per row of column k.  Destination rows of one call must be distinct (a ring shorter
// than n would make two rows race for a slot: the caller skips the rows a ring would overwrite).
// src_rows: rows every source column holds; without src_mod an index in [-src_rows, 0) counts from the end (numpy's
// indexing); any other index outside [0, src_rows) skips its row and is reported by mfx_rows_copy_error.
// Columns k with bit k of shift_mask set read row idx[i] + shift instead (before the modulo; their row is checked
// the same way): MemoryGroup.sample's next-state columns, (idx + 1) % nb_entries, in the same launch.
MFX_API int mfx_rows_copy_shift(int n_cols, void* const* dst, const void* const* src, const int64_t* row_bytes,
                                const int64_t* d_idx, int64_t src_mod, int64_t src_rows, int64_t dst_start,
                                int64_t dst_cap, int64_t n, uint32_t shift_mask, int64_t shift, void* stream) {
    if (n_cols < 1 || n_cols > kRowCols) return fail("rows_copy: 1..%d columns, got %d", kRowCols, n_cols);
    if (shift_mask >> n_cols) return fail("rows_copy: shift mask 0x%x names columns past %d", shift_mask, n_cols);
    if (src_mod > src_rows) return fail("rows_copy: modulo %lld over %lld source rows", (long long)src_mod,
                                        (long long)src_rows);
    if (!d_idx && n > src_rows) return fail("rows_copy: %lld rows from %lld source rows", (long long)n,
                                            (long long)src_rows);
    if (n < 0 || (dst_cap > 0 && n > dst_cap)) return fail("rows_copy: %lld rows into a ring of %lld", (long long)n,
                                                           (long long)dst_cap);
    if (n == 0) return 0;
    RowCols c{};
    c.n = n_cols;
    c.shift = shift_mask;
    c.shift_by = shift_mask ? shift : 0;
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
    // the pipelined form takes at most two wide columns (4-B aligned, <= 64 x 4 kPipeQ + 3 dwords) and <= 64 kPipeU
    // units
    PipeWide wd{};
    int n_wide = 0;
    bool wide_ok = true;
    for (int k = 0; k < n_cols; ++k) {
        if (c.ubytes[k]) continue;
        wide_ok = wide_ok && ((((uintptr_t)dst[k] | (uintptr_t)src[k] | (uintptr_t)row_bytes[k]) & 3) == 0) &&
                  row_bytes[k] / 4 <= 64 * 4 * kPipeQ + 3;
        if (n_wide < kPipeW) {
            wd.src[n_wide] = c.src[k];
            wd.dst[n_wide] = c.dst[k];
            wd.bytes[n_wide] = row_bytes[k];
            wd.dw[n_wide] = row_bytes[k] / 4;
            wd.shifted[n_wide] = shift_mask >> k & 1;
        }
        ++n_wide;
    }
    const bool pipe = n_wide <= kPipeW && wide_ok && units <= 64 * kPipeU;
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
        // Workgroups per CU (profiles/r06_replay_ab.txt): two wide columns (the fused sample, ~9.9 KB per entry) 2 --
        // 0.614 of the HBM peak against 0.604-0.608 at 3, 0.537 at 4, 0.527 at 1; one wide column (~5 KB per row) 3
        // -- 0.587-0.590 on the MF-Q columns against 0.569-0.575 at 2, 0.586 at 4, 0.448 at 1 (and 0.49 at 8; round
        // 4's dword units: 0.555-0.559 at 4, 0.464 / 0.520 at 7 / 14, 0.510-0.537 for the one-row-per-wave form; four
        // rows loaded then stored, and nontemporal stores, lost: profiles/r04_replay_ab.txt)
        const int per_cu = n_wide == 2 ? 2 : 3;
        const int64_t cap = (int64_t)cus * per_cu;
        const int grid = (int)(wgs < cap ? wgs : cap);
        auto* kern = n_wide == 2 ? (units > 64 ? k_rows_pipe<2, 2> : k_rows_pipe<2, 1>)
                                 : (units > 64 ? k_rows_pipe<1, 2> : k_rows_pipe<1, 1>);
        kern<<<grid, 256, 0, (hipStream_t)stream>>>(c, wd, d_idx, src_mod, src_rows, dst_start, dst_cap, n);
        MFX_HIP(hipGetLastError());
        return 0;
    }
    const int grid = (int)(wgs < 65536 ? wgs : 65536);
    k_rows_copy<<<grid, 256, 0, (hipStream_t)stream>>>(c, d_idx, src_mod, src_rows, dst_start, dst_cap, n);
    MFX_HIP(hipGetLastError());
    return 0;
}

// mfx_rows_copy_shift with no shifted column.
MFX_API int mfx_rows_copy(int n_cols, void* const* dst, const void* const* src, const int64_t* row_bytes,
                          const int64_t* d_idx, int64_t src_mod, int64_t src_rows, int64_t dst_start, int64_t dst_cap,
                          int64_t n, void* stream) {
    return mfx_rows_copy_shift(n_cols, dst, src, row_bytes, d_idx, src_mod, src_rows, dst_start, dst_cap, n, 0u, 0,
                               stream);
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
