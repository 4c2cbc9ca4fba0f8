// ising_kernels.h -- launchers of the Ising lattice / tabular MF-Q kernels (ising_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfx {

struct IsingMfqArgs {              // one run of main_MFQ_Ising.py's episode loop per replica
    int N, K, T;                   // agents, neighbours per agent, max time steps
    const int16_t* nbr;            // [N][K]
    const uint8_t* spins0;         // [R][N] initial spins (after env.reset)
    const double* u;               // [R][T][N] uniforms (null: words or on-device Philox)
    const uint32_t* words;         // [R][wstride] numpy's MT19937 word stream (k_mt_words; null: u or Philox)
    const uint32_t* woff;          // [R][T + 1] word offset of each step's uniforms (k_ising_scan)
    size_t wstride;
    const uint32_t* mask;          // [R][T][ceil(N/32)] act_group bits (null: every agent)
    double temperature, lr, decay_rate;
    int decay_gap;
    uint32_t seed;                 // Philox key (perf mode)
    double* q_out;                 // [R][N][K+1][2]
    double* order_out;             // [R][T] order parameter after each step (nullable)
    int32_t* nup_out;              // [R][T] (nullable)
    uint8_t* spins_out;            // [R][N] (nullable)
    int32_t* steps_out;            // [R] steps executed before the early stop (nullable)
};

hipError_t launch_ising_step(int R, int N, int K, const int16_t* nbr, uint8_t* spins, const int32_t* actions,
                             double* reward, uint8_t* obs, int32_t* n_up, double* order, hipStream_t st);
hipError_t launch_ising_mfq(const IsingMfqArgs& a, int R, hipStream_t st);

// numpy's legacy RandomState stream on the device (main_MFQ_Ising.py's np.random): k_mt_words writes the first
// n_blocks * 624 tempered MT19937 words of RandomState(seed0 + r0 + r) to words[r][...] for r < R; k_ising_scan walks
// one episode of main_MFQ_Ising.py's draws over them.
hipError_t launch_mt_words(uint32_t seed0, int r0, int R, int n_blocks, uint32_t* words, size_t stride, hipStream_t st);
struct IsingScanArgs {
    int N, T, n_upd;               // agents, steps, act_group size (int(act_rate * N))
    const uint32_t* words;         // [R][wstride]
    size_t wstride;
    const uint32_t* prev_off;      // [R][T + 1] the previous episode's offsets (null: the first episode)
    const int32_t* prev_steps;     // [R] the previous episode's steps
    uint8_t* spins0;               // [R][N] env.reset's spins
    uint32_t* off;                 // [R][T + 1]
    uint32_t* mask;                // [R][T][ceil(N / 32)] act_group bits (n_upd < N), else null
    uint16_t* perm;                // [R][N] scratch (n_upd < N)
    int32_t* err;                  // set to 1 when a replica's walk runs past wstride
};
hipError_t launch_ising_scan(const IsingScanArgs& a, int R, hipStream_t st);

}  // namespace mfx
