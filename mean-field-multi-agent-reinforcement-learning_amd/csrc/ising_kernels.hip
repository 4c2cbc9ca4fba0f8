// ising_kernels.hip -- Ising spin lattice + tabular mean-field Q-learning on gfx950.
//
// Reference: examples/ising_model/Ising.py (_calc_mask :7-58, reset :79-99, reward :101-111,
// observation :113-119), multiagent/core.py (IsingWorld.step :99-125) and the MF-Q loop of
// main_MFQ_Ising.py (:55-67 Boltzmann exploration, :103-159 episode loop).
//
// Layout: R independent replicas of an L x L periodic lattice, N = L*L agents, agent i at
// row i / L, column i % L (Ising.py:81-90).  One workgroup per replica, one thread per spin (up
// to 1024 spins, Q in registers), or 1024 threads over the spins with Q in HBM (k_ising_mfq_big).
//   spins  u8  [R][N]        0 = down, 1 = up (global_state)
//   nbr    i16 [N][K]        neighbour ids of agent i in ascending id order (spin_mask == 1)
//   Q      f64 [R][N][K+1][2]
// All float64 arithmetic is the reference's own sequence of single IEEE operations
// (-ffp-contract=off).  exp() is the device libm; see DESIGN.md for why an ulp there cannot
// change an action in practice.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "ising_kernels.h"

namespace mfx {

constexpr int kIsingMaxK = 16;
constexpr int kIsingMaxN = 32767;      // int16 neighbour ids; 3 N bytes of LDS in k_ising_mfq_big

// ------------------------------------------------------------------ env step
// IsingMultiAgentEnv._step (environment.py:49-78): spin_i := action_i for every agent, then
// n_up / order parameter (core.py:110-116), then per agent observation (neighbour spins) and
// reward 0.5 * s_i * sum_j s_j in +-1 units (Ising.py:101-111), all on the NEW spins.
__global__ void __launch_bounds__(1024) k_ising_step(int N, int K, const int16_t* __restrict__ nbr,
                                                     uint8_t* __restrict__ spins, const int32_t* __restrict__ actions,
                                                     double* __restrict__ reward, uint8_t* __restrict__ obs,
                                                     int32_t* __restrict__ n_up, double* __restrict__ order) {
    extern __shared__ uint8_t sp[];                                   // [N] the new spins
    __shared__ int cnt;
    const int r = blockIdx.x;
    uint8_t* S = spins + (size_t)r * N;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    int mine = 0;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const uint8_t s = actions[(size_t)r * N + i] <= 0 ? 0 : 1;       // _set_action (:112-114)
        sp[i] = s;
        S[i] = s;
        mine += s;
    }
    atomicAdd(&cnt, mine);
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        int sum = 0;
        for (int k = 0; k < K; ++k) {
            const int j = nbr[i * K + k];
            obs[((size_t)r * N + i) * K + k] = sp[j];
            sum += sp[j] ? 1 : -1;
        }
        const double gi = sp[i] ? 1.0 : -1.0;
        const double local = (-0.5 * gi) * (double)sum;               // Ising.py:106-108
        reward[(size_t)r * N + i] = -local;
    }
    if (threadIdx.x == 0) {
        n_up[r] = cnt;
        const int down = N - cnt;
        order[r] = (double)(cnt > down ? cnt - down : down - cnt) / ((double)N + 0.0);
    }
}

// ------------------------------------------------------------------ Philox 4x32-10 (perf mode)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

__device__ __forceinline__ double philox_uniform(uint32_t seed, uint32_t rep, uint32_t t, uint32_t i) {
    uint32_t c[4] = {i, t, rep, 0x5EED1u};
    philox(c, seed, 0xA511E9B3u);
    const uint64_t bits = ((uint64_t)(c[0] >> 5) << 26) | (c[1] >> 6);   // 53 bits, like random_sample
    return (double)bits * (1.0 / 9007199254740992.0);
}

// ------------------------------------------------------------------ numpy's legacy MT19937 stream
// main_MFQ_Ising.py draws from numpy's legacy RandomState (numpy/random/mtrand.pyx over
// numpy/random/src/mt19937): RandomState(seed) = init_genrand(seed) (key[0] = seed, key[i] = 1812433253 *
// (key[i-1] ^ key[i-1] >> 30) + i), 624-word twists, tempered outputs.  Its consumption, pinned against numpy itself
// (tests/test_ising_cpu.py test_numpy_stream_model): random_sample = one double from two words (a >> 5, b >> 6);
// choice(2) = one word & 1 (a masked bounded draw of 1); choice(N, k, replace=False) = permutation(N)[:k], the
// legacy shuffle of arange(N): for i = N-1 .. 1, j = random_interval(i) -- one word per try, masked to the smallest
// 2^b - 1 >= i, retried while above i -- then swap(x[i], x[j]).
constexpr int kMtN = 624;
__device__ __forceinline__ uint32_t mt_next(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}
// random_sample's double from words p[0], p[1] (legacy random_standard_uniform / rk_double)
__device__ __forceinline__ double mt_uniform(const uint32_t* p) {
    const uint32_t a = p[0] >> 5, b = p[1] >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// One 256-lane workgroup per replica, the state in LDS: a twist in three passes of at most 227 lanes whose reads all
// precede their writes (a barrier between): i < 227 reads key[i + 1], key[i + 397] as they were; 227 <= i < 454
// reads key[i - 227] of the first pass; the rest reads key[i - 227] of the second and, for i = 623, key[0] of the
// first.  Each block of 624 words is tempered and stored in order: words[r][624 b ...] is the replica's stream from
// its first draw.  (One wave per replica ran each block ~2x longer: the block chain is the replica's latency.)
__global__ void __launch_bounds__(256) k_mt_words(uint32_t seed0, int r0, int n_blocks, uint32_t* __restrict__ words,
                                                  size_t stride) {
    __shared__ uint32_t mt[kMtN];
    const int r = blockIdx.x, t = threadIdx.x;
    if (t == 0) {
        uint32_t x = seed0 + (uint32_t)(r0 + r);
        mt[0] = x;
        for (int i = 1; i < kMtN; ++i) {
            x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
            mt[i] = x;
        }
    }
    __syncthreads();
    uint32_t* out = words + (size_t)r * stride;
    for (int b = 0; b < n_blocks; ++b) {
        uint32_t v = 0;
        if (t < 227) v = mt_next(mt[t], mt[t + 1], mt[t + 397]);
        __syncthreads();
        if (t < 227) mt[t] = v;
        __syncthreads();
        const int i2 = 227 + t;
        if (i2 < 454) v = mt_next(mt[i2], mt[i2 + 1], mt[i2 - 227]);
        __syncthreads();
        if (i2 < 454) mt[i2] = v;
        __syncthreads();
        const int i3 = 454 + t;
        if (i3 < kMtN) v = mt_next(mt[i3], mt[i3 == kMtN - 1 ? 0 : i3 + 1], mt[i3 - 227]);
        __syncthreads();
        if (i3 < kMtN) mt[i3] = v;
        __syncthreads();
        for (int i = t; i < kMtN; i += 256) out[(size_t)b * kMtN + i] = mt_temper(mt[i]);
    }
}

// One wave per replica: one episode of main_MFQ_Ising.py's draws over the replica's word stream -- env.reset's N
// spins (choice(2)), then per step the offset of its N uniforms (2 N words) and the act_group permutation's words.
// The permutation's draws are walked 64 words at a time (word j in lane j).  Word j serves draw m0 - a_j, a_j the
// draws accepted before it, and is taken iff (w_j & mask(m0 - a_j)) <= m0 - a_j.  a_j is solved as a fixed point over
// the lanes (a ballot and a lane count per pass, from a guess at the draw's acceptance rate): the recursion is
// triangular, so the fixed point is unique and pass k fixes lane k at the latest, and a decision changes only when its
// threshold falls between two guesses -- ~3.5 passes per chunk.  (A scalar walk over the 64 thresholds -- v_readlane,
// compare, add-carry -- measured 2.7x slower: every readlane waits on the VALU; a chunk that ends where the mask
// halves, 1.3x slower.)  The chunk ends at 64 words or at draw 1.  n_upd < N (act_rate < 1): lane 0 also applies the
// swaps to arange(N) in perm and the first
// n_upd entries set the step's act_group bits.
// The permutation's words come from an LDS ring of RB blocks of 64 words (the uniforms are never fetched: k_ising_mfq
// reads them): each step's blocks are fetched by direct-to-LDS loads (global_load_lds) while the step before walks.
// The ring is the kernel's occupancy -- one wave per replica, latency-bound, so the waves per CU are its rate: RB = 32
// (8 KB, 20 waves per CU) holds a step and the next at N = 400; RB = 24 (6 KB, 26 waves) holds the step and most of
// the next, and is the faster (+3 % at 16384 replicas); words outside the ring are read from memory.
template <int RB>
__global__ void __launch_bounds__(64) k_ising_scan(IsingScanArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[RB * 64];
    const int r = blockIdx.x, lane = threadIdx.x;
    const uint32_t* W = a.words + (size_t)r * a.wstride;
    const size_t cap = a.wstride;
    const int N = a.N, T = a.T, mw = (N + 31) >> 5;
    const bool perm = a.n_upd < N;
    uint16_t* x = perm ? a.perm + (size_t)r * N : nullptr;
    uint32_t* off = a.off + (size_t)r * (T + 1);
    bool over = false;
    auto fetch = [&](size_t b0, size_t b1) {                 // issue blocks [b0, b1) into the ring (async)
#pragma nounroll
        for (size_t b = b0; b < b1; ++b) {
            const size_t p = b * 64 + lane;
            // (a 1- or 2-byte LDS-DMA would not shrink the ring: gfx950 writes each lane's bytes zero-extended to a
            // dword at base + 4 lane -- scripts/micro/glds_width.hip)
            __builtin_amdgcn_global_load_lds((const void*)(W + (p < cap ? p : 0)),
                                             (__attribute__((address_space(3))) void*)(ring + (b % RB) * 64), 4, 0, 0);
        }
    };
    auto word = [&](size_t p, size_t blo, size_t bhi) -> uint32_t {
        if (p >= cap) { over = true; return 0u; }
        const size_t b = p >> 6;
        if (b >= blo && b < bhi) return ring[(b % RB) * 64 + (p & 63)];
        return W[p];
    };
    // the episode's first draw: after make_world's N choice(2) draws, or where the previous episode stopped
    size_t pos = a.prev_off ? a.prev_off[(size_t)r * (T + 1) + a.prev_steps[r]] : (size_t)N;
    for (int i = lane; i < N; i += 64) {
        const size_t p = pos + i;
        if (p >= cap) over = true;
        a.spins0[(size_t)r * N + i] = (uint8_t)((p < cap ? W[p] : 0u) & 1u);
    }
    pos += N;
    // [vlo, vhi): the blocks complete in the ring; [plo, phi): the blocks in flight.  A fetch may land in the slots of
    // blocks below phi - RB at any time, so those leave the valid range as it is issued.
    size_t vlo = 0, vhi = 0, plo = (pos + 2 * (size_t)N) >> 6, phi = (pos + 4 * (size_t)N + 127) >> 6;
    if (phi > plo + RB) phi = plo + RB;
    fetch(plo, phi);                                         // step 0's permutation starts at pos + 2 N
    for (int t = 0; t < T; ++t) {
        if (lane == 0) off[t] = (uint32_t)pos;
        pos += 2 * (size_t)N;                                 // the Boltzmann uniforms (k_ising_mfq reads them)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the blocks in flight have landed
        if (phi > plo) {
            if (plo <= vhi && plo >= vlo) { if (phi > vhi) vhi = phi; }
            else { vlo = plo; vhi = phi; }
            if (vhi > RB && vlo < vhi - RB) vlo = vhi - RB;
        }
        // step t + 1's permutation starts 3 N - 1 .. 4 N words past this one's and takes at most 2 N (+ one chunk of
        // read-ahead; a longer walk reads its tail from memory): in flight while this step walks, never more than
        // RB blocks above this step's first
        plo = (pos + 3 * (size_t)N - 1) >> 6;
        if (plo < vhi) plo = vhi;
        phi = (pos + 6 * (size_t)N + 127) >> 6;
        if (phi > (pos >> 6) + RB) phi = (pos >> 6) + RB;
        if (t + 1 < T && phi > plo) {
            fetch(plo, phi);
            if (phi > RB && vlo < phi - RB) vlo = phi - RB;
        } else {
            phi = plo;
        }
        const size_t blo = vlo, bhi = vhi;
        if (perm && lane == 0)
            for (int i = 0; i < N; ++i) x[i] = (uint16_t)i;
        int m = N - 1;                                       // random_interval(m), m = N-1 .. 1
        while (m >= 1) {
            const uint32_t w = word(pos + lane, blo, bhi);
            // the guess: lane j's share of accepted words at draw m's acceptance rate (m + 1) / (mask(m) + 1)
            const float q = (float)(m + 1) / ((float)(0xFFFFFFFFu >> __builtin_clz((uint32_t)m)) + 1.0f);
            int aj = (int)((float)lane * q), acc = 0;
            unsigned long long bal = 0;
            for (int it = 0; it <= 64; ++it) {
                const int mm = m - aj;                       // the draw word j serves, and its mask
                const uint32_t M = mm >= 1 ? (0xFFFFFFFFu >> __builtin_clz((uint32_t)mm)) : 0u;
                acc = (mm < 1 || (w & M) <= (uint32_t)mm) ? 1 : 0;
                bal = __ballot(acc);
                const int an = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                const bool settled = __ballot(an != aj) == 0ull;
                aj = an;
                if (settled) break;
            }
            const unsigned long long fin = __ballot(aj + acc >= m);   // the word accepting draw 1, and after
            const int used = fin ? __builtin_ctzll(fin) + 1 : 64;
            if (perm) {                                      // the swaps in draw order (lane 0, one by one)
                const int mm = m - aj;
                const uint32_t jv = mm >= 1 ? (w & (0xFFFFFFFFu >> __builtin_clz((uint32_t)mm))) : 0u;
                for (int l = 0; l < used; ++l) {
                    const int al = __builtin_amdgcn_readlane(acc, l), ml = __builtin_amdgcn_readlane(mm, l);
                    const int jl = __builtin_amdgcn_readlane((int)jv, l);
                    if (lane == 0 && al && ml >= 1) {
                        const uint16_t xi = x[ml], xj = x[jl];
                        x[ml] = xj;
                        x[jl] = xi;
                    }
                }
            }
            pos += used;
            m = fin ? 0 : m - __popcll(bal);
        }
        if (perm) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            uint32_t* mk = a.mask + ((size_t)r * T + t) * mw;
            for (int i = lane; i < mw; i += 64) mk[i] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            for (int p = lane; p < a.n_upd; p += 64) {
                const int v = x[p];
                atomicOr(&mk[v >> 5], 1u << (v & 31));
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) off[T] = (uint32_t)pos;
    if (__ballot(over) && lane == 0) atomicExch(a.err, 1);
}

// ------------------------------------------------------------------ fused MF-Q episode
// One workgroup = one replica = one run of main_MFQ_Ising.py's episode loop.  Thread i owns agent
// i's Q rows in registers.  The uniforms: numpy's stream generated on the device (words at woff[t] + 2 i:
// k_mt_words, k_ising_scan), host-uploaded u [T][N], or null = Philox; mask: [T][ceil(N/32)] act_group bits
// (null = all).
template <int KMAX>
__global__ void __launch_bounds__(1024) k_ising_mfq(IsingMfqArgs a) {
    __shared__ uint8_t sp[4096];
    __shared__ int cnt[2];
    const int r = blockIdx.x, N = a.N, K = a.K, i = threadIdx.x;
    const bool own = i < N;
    double q[KMAX + 1][2];
#pragma unroll
    for (int s = 0; s < KMAX + 1; ++s) { q[s][0] = 0.0; q[s][1] = 0.0; }
    int16_t nb[KMAX];
    for (int k = 0; k < K; ++k) nb[k] = own ? a.nbr[i * K + k] : 0;
    if (own) sp[i] = a.spins0[(size_t)r * N + i];
    if (i == 0) { cnt[0] = 0; cnt[1] = 0; }
    __syncthreads();
    double current_t = 0.3, max_order = 0.0;
    int done_ = 0, t = 0;
    const int words = (N + 31) >> 5;
    for (t = 0; t < a.T; ++t) {
        if (t % a.decay_gap == 0) current_t *= a.decay_rate;           // main_MFQ_Ising.py:108-112
        if (current_t < a.temperature) current_t = a.temperature;
        // ---- state = number of up neighbours (count_nonzero(obs == 1)), Boltzmann action (:55-67)
        int st = 0;
        int act = 0;
        if (own) {
            for (int k = 0; k < K; ++k) st += sp[nb[k]];
            double q0 = 0.0, q1 = 0.0;
#pragma unroll
            for (int s = 0; s < KMAX + 1; ++s) if (s == st) { q0 = q[s][0]; q1 = q[s][1]; }
            const double e0 = exp(q0 / current_t), e1 = exp(q1 / current_t);
            const double denom = e0 + e1;
            const double p0 = e0 / denom, p1 = e1 / denom;
            const double c0 = p0 / (p0 + p1);                          // cdf /= cdf[-1]
            const double u = a.words ? mt_uniform(a.words + (size_t)r * a.wstride + a.woff[(size_t)r * (a.T + 1) + t] + 2 * i)
                           : a.u ? a.u[((size_t)r * a.T + t) * N + i]
                                 : philox_uniform(a.seed, (uint32_t)r, (uint32_t)t, (uint32_t)i);
            act = (u >= c0) ? 1 : 0;                                   // searchsorted(side='right')
        }
        __syncthreads();                                               // every state read the old spins
        if (own) sp[i] = (uint8_t)act;
        if (i == 0) cnt[t & 1] = 0;
        __syncthreads();
        // ---- world.step: order parameter; reward on the new spins; Q update (:122-133)
        const int par = t & 1;
        if (own) {
            int sum = 0;
            for (int k = 0; k < K; ++k) sum += sp[nb[k]] ? 1 : -1;
            const double gi = act ? 1.0 : -1.0;
            const double rew = -((-0.5 * gi) * (double)sum);
            const bool upd = !a.mask || ((a.mask[((size_t)r * a.T + t) * words + (i >> 5)] >> (i & 31)) & 1u);
            if (upd) {
#pragma unroll
                for (int s = 0; s < KMAX + 1; ++s)
                    if (s == st) {
                        if (act) q[s][1] = q[s][1] + a.lr * (rew - q[s][1]);
                        else q[s][0] = q[s][0] + a.lr * (rew - q[s][0]);
                    }
            }
        }
        const unsigned long long up = __ballot(own && act);
        if ((i & 63) == 0) atomicAdd(&cnt[par], __popcll(up));
        __syncthreads();
        const int n_up = cnt[par], n_down = N - n_up;
        const double order = (double)(n_up > n_down ? n_up - n_down : n_down - n_up) / ((double)N + 0.0);
        if (i == 0) {
            if (a.order_out) a.order_out[(size_t)r * a.T + t] = order;
            if (a.nup_out) a.nup_out[(size_t)r * a.T + t] = n_up;
        }
        if (order > max_order) max_order = order;                      // :138-156 (same on all lanes)
        if (fabs(max_order - order) < 0.001) ++done_;
        else done_ = 0;
        if (done_ == 500 || t > a.T) { ++t; break; }
    }
    if (own) {
        double* Q = a.q_out + ((size_t)r * N + i) * (K + 1) * 2;
        for (int s = 0; s <= K; ++s) {
#pragma unroll
            for (int ss = 0; ss < KMAX + 1; ++ss)
                if (ss == s) { Q[2 * s] = q[ss][0]; Q[2 * s + 1] = q[ss][1]; }
        }
        if (a.spins_out) a.spins_out[(size_t)r * N + i] = sp[i];
    }
    if (i == 0 && a.steps_out) a.steps_out[r] = t;
}

// ------------------------------------------------------------------ fused MF-Q episode, large lattices
// N > 1024 (up to kIsingMaxN): one 1024-lane workgroup per replica, lane l owns agents l, l + 1024, ...
// The Q rows live in the output buffer (HBM, each row touched by its owner only) and the spins, the
// new spins and the step's states in LDS (3 N bytes).  Same float64 operation sequence as k_ising_mfq.
template <int KMAX>
__global__ void __launch_bounds__(1024) k_ising_mfq_big(IsingMfqArgs a) {
    extern __shared__ uint8_t lds[];
    __shared__ int cnt[2];
    const int r = blockIdx.x, N = a.N, K = a.K;
    uint8_t* sp = lds;                 // spins before the step
    uint8_t* nsp = lds + N;            // spins after the step (the actions)
    uint8_t* stl = lds + 2 * N;        // each agent's state (up-neighbour count) this step
    double* Q = a.q_out + (size_t)r * N * (K + 1) * 2;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        sp[i] = a.spins0[(size_t)r * N + i];
        for (int k = 0; k < 2 * (K + 1); ++k) Q[(size_t)i * (K + 1) * 2 + k] = 0.0;
    }
    if (threadIdx.x == 0) { cnt[0] = 0; cnt[1] = 0; }
    __syncthreads();
    double current_t = 0.3, max_order = 0.0;
    int done_ = 0, t = 0;
    const int words = (N + 31) >> 5;
    for (t = 0; t < a.T; ++t) {
        if (t % a.decay_gap == 0) current_t *= a.decay_rate;           // main_MFQ_Ising.py:108-112
        if (current_t < a.temperature) current_t = a.temperature;
        for (int i = threadIdx.x; i < N; i += blockDim.x) {            // state + Boltzmann action (:55-67)
            int st = 0;
            for (int k = 0; k < K; ++k) st += sp[a.nbr[i * K + k]];
            const double* qr = Q + ((size_t)i * (K + 1) + st) * 2;
            const double q0 = qr[0], q1 = qr[1];
            const double e0 = exp(q0 / current_t), e1 = exp(q1 / current_t);
            const double denom = e0 + e1;
            const double p0 = e0 / denom, p1 = e1 / denom;
            const double c0 = p0 / (p0 + p1);
            const double u = a.words ? mt_uniform(a.words + (size_t)r * a.wstride + a.woff[(size_t)r * (a.T + 1) + t] + 2 * i)
                           : a.u ? a.u[((size_t)r * a.T + t) * N + i]
                                 : philox_uniform(a.seed, (uint32_t)r, (uint32_t)t, (uint32_t)i);
            nsp[i] = (u >= c0) ? 1 : 0;
            stl[i] = (uint8_t)st;
        }
        const int par = t & 1;
        if (threadIdx.x == 0) cnt[par] = 0;
        __syncthreads();
        int ups = 0;
        for (int i = threadIdx.x; i < N; i += blockDim.x) {            // reward on the new spins, Q (:122-133)
            const int act = nsp[i];
            int sum = 0;
            for (int k = 0; k < K; ++k) sum += nsp[a.nbr[i * K + k]] ? 1 : -1;
            const double gi = act ? 1.0 : -1.0;
            const double rew = -((-0.5 * gi) * (double)sum);
            const bool upd = !a.mask || ((a.mask[((size_t)r * a.T + t) * words + (i >> 5)] >> (i & 31)) & 1u);
            if (upd) {
                double* q = Q + ((size_t)i * (K + 1) + stl[i]) * 2 + act;
                *q = *q + a.lr * (rew - *q);
            }
            ups += act;
        }
        atomicAdd(&cnt[par], ups);
        __syncthreads();
        for (int i = threadIdx.x; i < N; i += blockDim.x) sp[i] = nsp[i];
        const int n_up = cnt[par], n_down = N - n_up;
        const double order = (double)(n_up > n_down ? n_up - n_down : n_down - n_up) / ((double)N + 0.0);
        if (threadIdx.x == 0) {
            if (a.order_out) a.order_out[(size_t)r * a.T + t] = order;
            if (a.nup_out) a.nup_out[(size_t)r * a.T + t] = n_up;
        }
        if (order > max_order) max_order = order;                      // :138-156 (same on all lanes)
        if (fabs(max_order - order) < 0.001) ++done_;
        else done_ = 0;
        __syncthreads();                                               // sp complete before the next step
        if (done_ == 500 || t > a.T) { ++t; break; }
    }
    if (a.spins_out)
        for (int i = threadIdx.x; i < N; i += blockDim.x) a.spins_out[(size_t)r * N + i] = sp[i];
    if (threadIdx.x == 0 && a.steps_out) a.steps_out[r] = t;
}

hipError_t launch_ising_step(int R, int N, int K, const int16_t* nbr, uint8_t* spins, const int32_t* actions,
                             double* reward, uint8_t* obs, int32_t* n_up, double* order, hipStream_t st) {
    if (N > kIsingMaxN || K > kIsingMaxK) return hipErrorInvalidValue;
    const int threads = N >= 1024 ? 1024 : ((N + 63) / 64) * 64;
    k_ising_step<<<R, threads, N, st>>>(N, K, nbr, spins, actions, reward, obs, n_up, order);
    return hipGetLastError();
}

hipError_t launch_ising_mfq(const IsingMfqArgs& a, int R, hipStream_t st) {
    if (a.N > kIsingMaxN || a.K > kIsingMaxK) return hipErrorInvalidValue;
    if (a.N > 1024) {                  // Q rows in HBM, spins in LDS
        const size_t lds = 3 * (size_t)a.N;
        if (a.K <= 4) k_ising_mfq_big<4><<<R, 1024, lds, st>>>(a);
        else k_ising_mfq_big<kIsingMaxK><<<R, 1024, lds, st>>>(a);
        return hipGetLastError();
    }
    const int threads = ((a.N + 63) / 64) * 64;
    if (a.K <= 4)
        k_ising_mfq<4><<<R, threads, 0, st>>>(a);
    else
        k_ising_mfq<kIsingMaxK><<<R, threads, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t launch_mt_words(uint32_t seed0, int r0, int R, int n_blocks, uint32_t* words, size_t stride, hipStream_t st) {
    if (R < 1 || n_blocks < 1 || stride < (size_t)n_blocks * kMtN) return hipErrorInvalidValue;
    k_mt_words<<<R, 256, 0, st>>>(seed0, r0, n_blocks, words, stride);
    return hipGetLastError();
}

hipError_t launch_ising_scan(const IsingScanArgs& a, int R, hipStream_t st) {
    if (a.N < 1 || a.N > kIsingMaxN || a.T < 1 || (a.n_upd < a.N && (!a.mask || !a.perm))) return hipErrorInvalidValue;
    // the ring's blocks: 24 (26 waves per CU; 3.41e10 spin-steps/s against 3.32e10 with 32 at 16384 replicas)
    k_ising_scan<24><<<R, 64, 0, st>>>(a);
    return hipGetLastError();
}

}  // namespace mfx
