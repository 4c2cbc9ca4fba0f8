// ising_kernels.h -- launchers of the Ising lattice / tabular MF-Q kernels (ising_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfx {

struct IsingMfqArgs {              // one run of main_MFQ_Ising.py's episode loop per replica
    int N, K, T;                   // agents, neighbours per agent, max time steps
    const int16_t* nbr;            // [N][K]
    const uint8_t* spins0;         // [R][N] initial spins (after env.reset)
    const double* u;               // [R][T][N] uniforms (null: on-device Philox)
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

}  // namespace mfx
