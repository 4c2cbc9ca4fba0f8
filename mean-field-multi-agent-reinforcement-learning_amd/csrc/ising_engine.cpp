// ising_engine.cpp -- host runtime + C ABI of the Ising lattice and tabular MF-Q kernels.
//
// The reference has no native layer here (everything is python: examples/ising_model and
// main_MFQ_Ising.py).  This ABI is what this repository's drop-in `examples.ising_model`
// package and `mfrl_amd.ising` bind through ctypes; host buffers in, host buffers out.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ising_kernels.h"
#include "mfx_common.h"
#include "../../include/magent_amd.h"

namespace mfx {

struct IsingEngine {
    int R = 1, N = 0, K = 0;
    hipStream_t stream = nullptr;
    DevBuf<int16_t> nbr;
    DevBuf<uint8_t> spins, obs, spins_out;
    DevBuf<int32_t> actions, n_up, steps;
    DevBuf<double> reward, order, q, u, order_t;
    DevBuf<uint32_t> mask;
    DevBuf<int32_t> nup_t;
    DevBuf<int32_t> err;
    // mfx_ising_mfq_run_stream's two pass slots: pass p's words are generated and walked (gen stream) into slot
    // p % 2 while pass p - 1's episode runs out of the other (stream)
    struct Slot {
        DevBuf<uint32_t> words, off[2], mask;
        DevBuf<uint16_t> perm;
        DevBuf<double> q, order_t;
        DevBuf<int32_t> nup_t, steps;
        hipEvent_t produced = nullptr, consumed = nullptr;
    } slot[2];
    hipStream_t gen = nullptr;
    ~IsingEngine() {
        for (auto& sl : slot) {
            if (sl.produced) (void)hipEventDestroy(sl.produced);
            if (sl.consumed) (void)hipEventDestroy(sl.consumed);
        }
        if (gen) (void)hipStreamDestroy(gen);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

}  // namespace mfx

using mfx::IsingEngine;

extern "C" {

// R replicas of an N-agent lattice whose neighbour table nbr[N][K] (ascending ids) comes from
// Ising.py:_calc_mask (computed by the python Scenario).
MFX_API int mfx_ising_create(int R, int N, int K, const int16_t* nbr, void** handle) {
    if (R < 1 || N < 1 || N > 32767 || K < 1 || K > 16) return mfx::fail("ising: need 1 <= N <= 32767, 1 <= K <= 16");
    try {
        auto* e = new IsingEngine();
        e->R = R; e->N = N; e->K = K;
        MFX_HIP_THROW(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
        e->nbr.ensure((size_t)N * K);
        MFX_HIP_THROW(hipMemcpy(e->nbr.p, nbr, sizeof(int16_t) * N * K, hipMemcpyHostToDevice));
        e->spins.ensure((size_t)R * N);
        MFX_HIP_THROW(hipMemset(e->spins.p, 0, (size_t)R * N));
        *handle = e;
        return 0;
    } catch (const std::exception& ex) {
        return mfx::fail("%s", ex.what());
    }
}

MFX_API int mfx_ising_destroy(void* h) { delete static_cast<IsingEngine*>(h); return 0; }

MFX_API int mfx_ising_set_spins(void* h, const uint8_t* spins) {
    auto* e = static_cast<IsingEngine*>(h);
    MFX_HIP(hipMemcpy(e->spins.p, spins, (size_t)e->R * e->N, hipMemcpyHostToDevice));
    return 0;
}

MFX_API int mfx_ising_get_spins(void* h, uint8_t* spins) {
    auto* e = static_cast<IsingEngine*>(h);
    MFX_HIP(hipMemcpy(spins, e->spins.p, (size_t)e->R * e->N, hipMemcpyDeviceToHost));
    return 0;
}

// One IsingMultiAgentEnv.step for every replica: actions [R][N] -> rewards [R][N] f64,
// observations [R][N][K] u8 (neighbour spins), n_up [R], order parameter [R].
MFX_API int mfx_ising_step(void* h, const int32_t* actions, double* reward, uint8_t* obs, int32_t* n_up,
                           double* order) {
    auto* e = static_cast<IsingEngine*>(h);
    const size_t RN = (size_t)e->R * e->N;
    try {
        e->actions.ensure(RN); e->reward.ensure(RN); e->obs.ensure(RN * e->K); e->n_up.ensure(e->R);
        e->order.ensure(e->R);
    } catch (const std::exception& ex) {
        return mfx::fail("%s", ex.what());
    }
    MFX_HIP(hipMemcpyAsync(e->actions.p, actions, sizeof(int32_t) * RN, hipMemcpyHostToDevice, e->stream));
    MFX_HIP(mfx::launch_ising_step(e->R, e->N, e->K, e->nbr.p, e->spins.p, e->actions.p, e->reward.p, e->obs.p,
                                   e->n_up.p, e->order.p, e->stream));
    MFX_HIP(hipMemcpyAsync(reward, e->reward.p, sizeof(double) * RN, hipMemcpyDeviceToHost, e->stream));
    MFX_HIP(hipMemcpyAsync(obs, e->obs.p, RN * e->K, hipMemcpyDeviceToHost, e->stream));
    MFX_HIP(hipMemcpyAsync(n_up, e->n_up.p, sizeof(int32_t) * e->R, hipMemcpyDeviceToHost, e->stream));
    MFX_HIP(hipMemcpyAsync(order, e->order.p, sizeof(double) * e->R, hipMemcpyDeviceToHost, e->stream));
    MFX_HIP(hipStreamSynchronize(e->stream));
    return 0;
}

// The whole tabular MF-Q episode of main_MFQ_Ising.py for every replica, starting from the
// current spins.  u: host [R][T][N] uniforms or null (Philox, `seed`); mask: host
// [R][T][ceil(N/32)] act_group bits or null (act_rate 1).  Outputs (host, nullable except q):
// q [R][N][K+1][2], order [R][T], n_up [R][T], steps [R]; spins are updated in place.
MFX_API int mfx_ising_mfq_run(void* h, int T, double temperature, double lr, double decay_rate, int decay_gap,
                              const double* u, const uint32_t* mask, unsigned seed, double* q, double* order,
                              int32_t* n_up, int32_t* steps) {
    auto* e = static_cast<IsingEngine*>(h);
    const int R = e->R, N = e->N, K = e->K, words = (N + 31) / 32;
    if (T < 1) return mfx::fail("ising mfq: T must be >= 1");
    if (decay_gap < 1) return mfx::fail("ising mfq: decay_gap must be >= 1");
    mfx::IsingMfqArgs a{};
    try {
        if (u) {
            e->u.ensure((size_t)R * T * N);
            MFX_HIP_THROW(hipMemcpyAsync(e->u.p, u, sizeof(double) * R * T * N, hipMemcpyHostToDevice, e->stream));
        }
        if (mask) {
            e->mask.ensure((size_t)R * T * words);
            MFX_HIP_THROW(hipMemcpyAsync(e->mask.p, mask, sizeof(uint32_t) * R * T * words, hipMemcpyHostToDevice,
                                         e->stream));
        }
        e->q.ensure((size_t)R * N * (K + 1) * 2);
        e->order_t.ensure((size_t)R * T);
        e->nup_t.ensure((size_t)R * T);
        e->steps.ensure(R);
        e->spins_out.ensure((size_t)R * N);
    } catch (const std::exception& ex) {
        return mfx::fail("%s", ex.what());
    }
    a.N = N; a.K = K; a.T = T; a.nbr = e->nbr.p; a.spins0 = e->spins.p;
    a.u = u ? e->u.p : nullptr; a.mask = mask ? e->mask.p : nullptr;
    a.temperature = temperature; a.lr = lr; a.decay_rate = decay_rate; a.decay_gap = decay_gap; a.seed = seed;
    a.q_out = e->q.p; a.order_out = e->order_t.p; a.nup_out = e->nup_t.p; a.spins_out = e->spins_out.p;
    a.steps_out = e->steps.p;
    MFX_HIP(mfx::launch_ising_mfq(a, R, e->stream));
    MFX_HIP(hipMemcpyAsync(e->spins.p, e->spins_out.p, (size_t)R * N, hipMemcpyDeviceToDevice, e->stream));
    MFX_HIP(hipMemcpyAsync(q, e->q.p, sizeof(double) * R * N * (K + 1) * 2, hipMemcpyDeviceToHost, e->stream));
    if (order) MFX_HIP(hipMemcpyAsync(order, e->order_t.p, sizeof(double) * R * T, hipMemcpyDeviceToHost, e->stream));
    if (n_up) MFX_HIP(hipMemcpyAsync(n_up, e->nup_t.p, sizeof(int32_t) * R * T, hipMemcpyDeviceToHost, e->stream));
    if (steps) MFX_HIP(hipMemcpyAsync(steps, e->steps.p, sizeof(int32_t) * R, hipMemcpyDeviceToHost, e->stream));
    MFX_HIP(hipStreamSynchronize(e->stream));
    return 0;
}

// main_MFQ_Ising.py with its numpy stream generated on the device (k_mt_words, k_ising_scan): replica r is the
// script run with seed seed0 + r -- RandomState(seed0 + r), make_world's N discarded choice(2) draws, then per
// episode env.reset's N spins and per step the N Boltzmann uniforms and the act_group permutation
// (choice(N, int(act_rate N), replace=False)) -- for `episodes` episodes in sequence on the one stream, each until
// its own early stop (-epi).  Nothing is read back between episodes: the next episode's first draw is found on the
// device from the steps the previous one ran.  Outputs (host; nullable except q), per episode:
// q [E][R][N][K+1][2], order [E][R][T], n_up [E][R][T], steps [E][R]; the spins end as the last episode left them.
MFX_API int mfx_ising_mfq_run_stream(void* h, int T, double temperature, double lr, double decay_rate, int decay_gap,
                                     double act_rate, unsigned seed0, int episodes, double* q, double* order,
                                     int32_t* n_up, int32_t* steps) {
    auto* e = static_cast<IsingEngine*>(h);
    const int R = e->R, N = e->N, K = e->K, mw = (N + 31) / 32;
    if (T < 1 || episodes < 1) return mfx::fail("ising mfq stream: T and episodes must be >= 1");
    if (decay_gap < 1) return mfx::fail("ising mfq stream: decay_gap must be >= 1");
    if (!(act_rate >= 0.0 && act_rate <= 1.0)) return mfx::fail("ising mfq stream: act_rate must be in [0, 1]");
    const int n_upd = (int)(act_rate * N);                  // int(act_rate * n_agents), main_MFQ_Ising.py:126
    // words per replica: make_world's N, then per episode N spins and per step 2 N uniforms + the permutation's
    // draws (N - 1 accepted words plus rejections: ~0.5 N expected, bounded here by 2 N -- a walk past the end sets
    // the error word) + one chunk of read-ahead (k_ising_scan reads 64 words at a time; its prefetch clamps at the stride)
    const size_t per = (size_t)N + (size_t)episodes * ((size_t)N + (size_t)T * 4 * N) + 320;
    const size_t blocks_z = (per + 623) / 624;
    const size_t W = blocks_z * 624;
    // the per-step word offsets (k_ising_scan's off, k_ising_mfq's woff, the next episode's prev_off) are 32-bit
    if (W > (size_t)UINT32_MAX)
        return mfx::fail("ising mfq stream: %zu words per replica (episodes x T x 4 N) exceed the 32-bit word offsets; "
                         "run fewer episodes per call or mode 'host'", W);
    const int blocks = (int)blocks_z;
    // replicas per pass: a slot's word streams within 64 GB and a third of the free memory.  Big passes: the walk
    // is one latency-bound wave per replica, so a pass's walk takes about as long whatever its replicas -- 16384
    // replicas at 2000 steps: 3.41e10 spin-steps/s in 16-GB passes, 3.86e10 in 64-GB ones (MFX_ISING_PASS_GB: A/B only)
    const char* pg = getenv("MFX_ISING_PASS_GB");
    size_t pass_bytes = (size_t)64 << 30;
    {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr / 3 < pass_bytes) pass_bytes = std::max<size_t>(fr / 3, (size_t)1 << 30);
    }
    if (pg) pass_bytes = (size_t)std::max(1, atoi(pg)) << 30;
    const int Rb = (int)std::max<size_t>(1, std::min<size_t>((size_t)R, pass_bytes / (W * 4)));
    const int P = (R + Rb - 1) / Rb;                           // passes
    const size_t QR = (size_t)N * (K + 1) * 2;
    try {
        for (int k = 0; k < std::min(P, 2); ++k) {
            auto& sl = e->slot[k];
            sl.words.ensure((size_t)Rb * W);
            for (auto& o : sl.off) o.ensure((size_t)Rb * (T + 1));
            if (n_upd < N) { sl.perm.ensure((size_t)Rb * N); sl.mask.ensure((size_t)Rb * T * mw); }
            sl.q.ensure((size_t)Rb * QR);
            sl.order_t.ensure((size_t)Rb * T);
            sl.nup_t.ensure((size_t)Rb * T);
            sl.steps.ensure(Rb);
            if (!sl.produced) MFX_HIP_THROW(hipEventCreateWithFlags(&sl.produced, hipEventDisableTiming));
            if (!sl.consumed) MFX_HIP_THROW(hipEventCreateWithFlags(&sl.consumed, hipEventDisableTiming));
        }
        if (!e->gen) MFX_HIP_THROW(hipStreamCreateWithFlags(&e->gen, hipStreamNonBlocking));
        e->err.ensure(1);
        e->spins_out.ensure((size_t)R * N);
    } catch (const std::exception& ex) {
        return mfx::fail("%s", ex.what());
    }
    MFX_HIP(hipMemsetAsync(e->err.p, 0, sizeof(int32_t), e->stream));
    hipStream_t gs = e->gen;                                         // the generation's own stream
    {   // the gen stream starts after the error word is cleared
        hipEvent_t ready = e->slot[0].consumed;
        MFX_HIP(hipEventRecord(ready, e->stream));
        MFX_HIP(hipStreamWaitEvent(e->gen, ready, 0));
    }
    auto scan = [&](IsingEngine::Slot& sl, int r0, int nr, int ep, hipStream_t st) -> hipError_t {
        mfx::IsingScanArgs sa{};
        sa.N = N; sa.T = T; sa.n_upd = n_upd; sa.words = sl.words.p; sa.wstride = W;
        sa.prev_off = ep ? sl.off[(ep - 1) & 1].p : nullptr;
        sa.prev_steps = ep ? sl.steps.p : nullptr;
        sa.spins0 = e->spins.p + (size_t)r0 * N;
        sa.off = sl.off[ep & 1].p;
        sa.mask = n_upd < N ? sl.mask.p : nullptr;
        sa.perm = n_upd < N ? sl.perm.p : nullptr;
        sa.err = e->err.p;
        return mfx::launch_ising_scan(sa, nr, st);
    };
    // pass p's generation and first walk (gen stream), into slot p % 2 once pass p - 2 has released it
    auto produce = [&](int p) -> hipError_t {
        auto& sl = e->slot[p & 1];
        const int r0 = p * Rb, nr = std::min(Rb, R - r0);
        hipError_t err;
        if (p >= 2 && (err = hipStreamWaitEvent(gs, sl.consumed, 0)) != hipSuccess) return err;
        if ((err = mfx::launch_mt_words(seed0, r0, nr, blocks, sl.words.p, W, gs)) != hipSuccess) return err;
        if ((err = scan(sl, r0, nr, 0, gs)) != hipSuccess) return err;
        return hipEventRecord(sl.produced, gs);
    };
    MFX_HIP(produce(0));
    if (P > 1) MFX_HIP(produce(1));
    for (int p = 0; p < P; ++p) {
        auto& sl = e->slot[p & 1];
        const int r0 = p * Rb, nr = std::min(Rb, R - r0);
        MFX_HIP(hipStreamWaitEvent(e->stream, sl.produced, 0));
        for (int ep = 0; ep < episodes; ++ep) {
            if (ep) MFX_HIP(scan(sl, r0, nr, ep, e->stream));       // (after the previous episode's early stop)
            mfx::IsingMfqArgs a{};
            a.N = N; a.K = K; a.T = T; a.nbr = e->nbr.p; a.spins0 = e->spins.p + (size_t)r0 * N;
            a.words = sl.words.p; a.woff = sl.off[ep & 1].p; a.wstride = W;
            a.mask = n_upd < N ? sl.mask.p : nullptr;
            a.temperature = temperature; a.lr = lr; a.decay_rate = decay_rate; a.decay_gap = decay_gap;
            a.q_out = sl.q.p; a.order_out = sl.order_t.p; a.nup_out = sl.nup_t.p;
            a.spins_out = e->spins_out.p + (size_t)r0 * N; a.steps_out = sl.steps.p;
            MFX_HIP(mfx::launch_ising_mfq(a, nr, e->stream));
            const size_t er = (size_t)ep * R + r0;               // this pass's rows of episode ep's outputs
            MFX_HIP(hipMemcpyAsync(q + er * QR, sl.q.p, sizeof(double) * nr * QR, hipMemcpyDeviceToHost, e->stream));
            if (order)
                MFX_HIP(hipMemcpyAsync(order + er * T, sl.order_t.p, sizeof(double) * nr * T, hipMemcpyDeviceToHost,
                                       e->stream));
            if (n_up)
                MFX_HIP(hipMemcpyAsync(n_up + er * T, sl.nup_t.p, sizeof(int32_t) * nr * T, hipMemcpyDeviceToHost,
                                       e->stream));
            if (steps)
                MFX_HIP(hipMemcpyAsync(steps + er, sl.steps.p, sizeof(int32_t) * nr, hipMemcpyDeviceToHost, e->stream));
        }
        MFX_HIP(hipEventRecord(sl.consumed, e->stream));
        if (p + 2 < P) MFX_HIP(produce(p + 2));
    }
    MFX_HIP(hipMemcpyAsync(e->spins.p, e->spins_out.p, (size_t)R * N, hipMemcpyDeviceToDevice, e->stream));
    int32_t err = 0;
    MFX_HIP(hipMemcpyAsync(&err, e->err.p, sizeof(err), hipMemcpyDeviceToHost, e->stream));
    MFX_HIP(hipStreamSynchronize(e->stream));
    if (err) return mfx::fail("ising mfq stream: a replica's draws ran past its %zu generated words", W);
    return 0;
}

}  // extern "C"
