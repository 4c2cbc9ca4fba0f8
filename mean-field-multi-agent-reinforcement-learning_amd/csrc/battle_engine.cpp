// battle_engine.cpp -- host runtime of the Battle engine + its C ABI.
//
// The C ABI is the reference's own (runtime_api.h:118-181: env_* / gridworld_*), so the
// reference python wrapper (gridworld.py, via ctypes) and this repository's drop-in
// `magent` package both bind it unchanged.  Those calls work on env 0 and move data
// through host buffers.  The batched device API (mfx_battle_*) drives all E envs of an
// engine with device pointers and never leaves HBM.  See include/magent_amd.h.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <fstream>
#include <sstream>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "battle_kernels.h"
#include "battle_layout.h"
#include "mfx_common.h"
#include "../../include/magent_amd.h"

namespace mfx {

// The queue kernels (k_rollout_bigq) hand work between the workgroups of one launch.  Each env lives on one XCD, an
// XCD's work of a launch completes with any one of the launch's workgroups resident there, and a workgroup leaves as
// soon as its XCD's work is done (rollout_big.inc xcd_done); the pipelined few-env form also claims stepper roles and
// takes back unclaimed items from waiting workgroups (few_rollout).  So neither needs its whole grid co-resident.
// The large-env form still runs one launch at a time per process and device (this lock: each such launch waits for
// the previous one's completion event on its device) -- its grid fills every CU, and two of them dispatched at once
// would split the chip between two copies of the same observation stream for no gain.
class BigqSerial {
  public:
    explicit BigqSerial(hipStream_t st) : st_(st), lock_(mu()) {
        if (hipGetDevice(&dev_) != hipSuccess || dev_ < 0 || dev_ >= kDevs) dev_ = -1;
        else if (has()[dev_]) err_ = hipStreamWaitEvent(st_, ev()[dev_], 0);
    }
    ~BigqSerial() {
        if (dev_ < 0) return;
        if (!ev()[dev_] && hipEventCreateWithFlags(&ev()[dev_], hipEventDisableTiming) != hipSuccess) return;
        if (hipEventRecord(ev()[dev_], st_) == hipSuccess) has()[dev_] = true;
    }
    hipError_t status() const { return err_; }

  private:
    static constexpr int kDevs = 64;
    static std::mutex& mu() { static std::mutex m; return m; }
    static hipEvent_t* ev() { static hipEvent_t e[kDevs] = {}; return e; }
    static bool* has() { static bool h[kDevs] = {}; return h; }
    hipStream_t st_;
    std::lock_guard<std::mutex> lock_;
    int dev_ = -1;
    hipError_t err_ = hipSuccess;
};

// ------------------------------------------------------------------ host-side ranges
struct HostRange {                                  // Range.h:14-113
    int w = 0, h = 0, count = 0, x1 = 0, y1 = 0, x2 = 0, y2 = 0;
    std::vector<uint8_t> in;
    std::vector<int> dx, dy;
};

static HostRange circle_range(float radius, float inner, int parity) {   // Range.h:171-215
    const double eps = 1e-8;
    HostRange r;
    int width = 2 * (int)(radius + eps) + parity;
    const int center = (int)radius;
    if (width % 2 != parity) width++;
    r.w = r.h = width;
    r.in.assign((size_t)width * width, 0);
    const double delta = parity == 0 ? 0.5 : 0;
    for (int i = 0; i < width; i++)
        for (int j = 0; j < width; j++) {
            const double ddx = std::fabs(j - center + delta), ddy = std::fabs(i - center + delta);
            const double dis = std::sqrt(ddx * ddx + ddy * ddy);
            if (dis < radius + eps && dis > inner - eps) {
                r.in[(size_t)i * width + j] = 1;
                r.dx.push_back(j - center);
                r.dy.push_back(i - center);
            }
        }
    r.count = (int)r.dx.size();
    r.x1 = r.y1 = -center;
    r.x2 = r.y2 = width - center - 1;
    return r;
}

static HostRange sector_range(float angle, float radius, int parity) {   // Range.h:121-166
    const double PI = 3.1415926536, eps = 0.00001;
    HostRange r;
    const int height = (int)(radius + 0.5);
    int width = (int)(2 * radius * std::sin(angle / 2 * (PI / 180)) + 0.5);
    if (width % 2 != parity) width--;
    r.w = width; r.h = height;
    r.in.assign((size_t)std::max(0, width * height), 0);
    for (int i = 0; i < height; i++)
        for (int j = 0; j < width; j++) {
            const double ddx = std::fabs(j - (width - 1) / 2.0), ddy = std::fabs((double)(height - i));
            const double dis = std::sqrt(ddx * ddx + ddy * ddy);
            if (dis < radius + 0.2 + eps && ddx / ddy < std::tan(angle / 2 * PI / 180) + eps) {
                r.in[(size_t)i * width + j] = 1;
                r.dx.push_back(j - width / 2);
                r.dy.push_back(i - height);
            }
        }
    r.count = (int)r.dx.size();
    r.x1 = -width / 2; r.y1 = -height; r.x2 = (width - 1) / 2; r.y2 = -1;
    return r;
}

struct AgentTypeSpec {                               // AgentType.cc:28-131
    std::string name;
    int width = 1, length = 1;
    float speed = 1, hp = 1, view_radius = 1, view_angle = 360, attack_radius = 0, attack_angle = 0;
    float hear_radius = 0, speak_radius = 0;
    int speak_ability = 0;
    float damage = 0, trace = 0, eat_ability = 0, step_recover = 0, kill_supply = 0, food_supply = 0;
    bool attack_in_group = false, can_absorb = false;
    float step_reward = 0, kill_reward = 0, dead_penalty = 0, attack_penalty = 0;
    HostRange view, attack, move;
    int turn_base = 0, attack_base = 0, n_action = 0;
};

// ------------------------------------------------------------------ the engine
class BattleEngine {
public:
    // --- configuration (GridWorld.cc:126-155)
    int W = 0, H = 0, emb = 0;
    bool minimap = false, food = false, turn = false, goal = false;
    bool large_map = false; int n_sep = 8;
    uint32_t rng_init = 1;                          // seed(0) -> state 1 (GridWorld.cc:31)
    std::map<std::string, AgentTypeSpec> types;
    std::vector<std::string> group_types;
    struct Sym { int group, index; };
    struct Node { int op; std::vector<int> raw; };
    struct Rule { int on; std::vector<int> recv; std::vector<float> val; bool terminal; };
    std::vector<Sym> syms; std::vector<Node> nodes; std::vector<Rule> rules;

    // --- device
    int E = 1;
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool stream_set = false;                          // a caller-provided stream (may be the null stream)
    GameParams gp{};
    GameParams* d_gp = nullptr;
    State s{};
    uint32_t* d_sort = nullptr;
    int32_t* d_err = nullptr;
    bool allocated = false;
    // render (RenderGenerator.cc): config.json + video_<file>.txt frames of env 0
    std::string render_dir;
    int file_ct = 0, frame_ct = 0, frame_per_file = 10000;
    bool first_render = true;
    int max_ids = 0;                                 // upper bound of id_counter over envs
    std::vector<int> group_ub;                       // upper bound of grp_n per group
    int pending_ub = 0;                              // upper bound of queued actions
    int acts_since_step[kMaxGroups] = {};            // set_action calls per group since the last step
    // drop-in staging (env 0, host buffers)
    DevBuf<float> st_view, st_feat, st_f32;
    // Drop-in host cache (env 0).  The reference call sequence asks the same state many times per step
    // (get_num before every getter, both groups' observations, ids / rewards / alive of both groups);
    // every state change bumps `epoch`, and a getter fetches everything it may be asked next for the
    // current epoch in ONE device-to-host transfer into pinned memory with ONE stream sync: two syncs
    // per training-loop step (observations + ids before the actions, done + rewards / alive / positions
    // after the step) instead of one or two per call.
    uint64_t epoch = 1, n_ep = 0, obs_ep = 0, info_ep = 0;
    int hn[kMaxGroups] = {};                 // group sizes of env 0 (valid when n_ep == epoch)
    size_t obs_rows = 0, info_rows = 0;      // rows per group of the staging layouts below
    bool obs_packed = false;                 // one env: pin_obs holds views|features per group packed
    size_t obs_pack_off[kMaxGroups] = {};    //   at these float offsets
    DevBuf<uint8_t> st_info;                 // env 0's record (k_get_env0): header, then per group
                                             //   ids i32 | reward f32 | pos 2 x i32 | alive u8, x rows
    PinBuf<uint8_t> pin_obs, pin_info;       // host copies: views + features, info, in the same layouts
    PinBuf<int32_t> pin_act;                 // [G][rows] actions on their way to the device
    hipEvent_t act_ev[kMaxGroups] = {};      // that copy of group g has left pin_act
    const uint8_t* info_src = nullptr;       // the record the getters answer from (pin_info or pin_fast)
    size_t info_src_rows = 0;                //   and its rows per group
    // Fast drop-in step (k_dropin_step, battle/dropin.inc): set_action and clear_dead are deferred and
    // env.step() is ONE launch that also leaves the records of the post-step and post-clear_dead states
    // and the next observation in host-mapped memory.  Deferred work runs for real (flush_deferred)
    // before anything else reads or changes the device state.
    bool fast_enabled = fast_default();      // MFX_DROPIN_FAST=0: the per-call path (A/B, tests)
    static bool fast_default() {
        const char* v = getenv("MFX_DROPIN_FAST");
        return !v || atoi(v) != 0;
    }
    bool defer_act[kMaxGroups] = {};         // group g's actions wait in pin_fact
    int defer_n[kMaxGroups] = {};
    bool defer_clear = false;                // clear_dead waits for the next k_dropin_step
    uint64_t spec_ep = 0;                    // epoch at which the step record / the observation blocks apply
    bool obs_fast = false;                   // the observation cache is pin_fast's blocks
    MappedBuf<uint8_t> pin_fast;             // rec_step | per group view block, feature block
    MappedBuf<int32_t> pin_fact;             // [G][fact_rows] deferred actions
    MappedBuf<uint32_t> pin_flag;            // [2] k_dropin_step's completion words (coherent)
    uint32_t fast_seq = 0;                   // sequence number of the last k_dropin_step request
    uint32_t obs_seq = 0;                    // the request whose observation the cache holds
    // Resident server (engines on their own stream, MFX_DROPIN_RESIDENT != 0): one k_dropin_step launch
    // keeps env 0 in LDS and answers every env.step() posted in the mailbox (battle_layout.h
    // DropinMailbox) -- no launch, no install per step.  It leaves after a stop request (quiesce(),
    // before anything else touches the stream or the state) or after res_idle_us without a request,
    // and is relaunched by the next step.
    bool res_enabled = env_flag("MFX_DROPIN_RESIDENT", true);
    bool res_live = false;                   // a server was launched and not asked to stop
    bool fast_res = false;                   // the last request went to the resident server
    int res_relaunch = 0;                    // relaunches after an idle exit (statistics)
    MappedBuf<DropinMailbox> mbox;
    uint32_t mail_tag[kMaxGroups] = {};      // tag of group g's actions in mbox->acts (~0: not there)
    size_t mail_stride[kMaxGroups] = {};     //   and the per-group stride they were written with
    int ensure_mbox() {
        if (mbox.p) return 0;
        try { mbox.ensure(1, hipHostMallocCoherent); } catch (const HipFailure& f) { return fail("%s", f.what()); }
        memset(mbox.p, 0, sizeof(DropinMailbox));
        return 0;
    }
    DropinArgs res_da{};                     // the arguments of the live server (relaunch)
    static bool env_flag(const char* name, bool dflt) {
        const char* v = getenv(name);
        return v ? atoi(v) != 0 : dflt;
    }
    size_t fast_rows = 0, fact_rows = 0;
    size_t fast_rec = 0, fast_view[kMaxGroups] = {}, fast_feat[kMaxGroups] = {}, fast_set_bytes = 0;
    std::vector<void*> retired;              // outgrown pin_fast blocks (views may outlive them), freed last
    std::vector<uint8_t> clr_rec;            // the record after a deferred clear_dead (host-built)
    DevBuf<int> st_i32, st_xs, st_ys, st_dirs;
    DevBuf<uint8_t> st_u8;
    // fused rollout (bench / throughput path)
    bool rollout_ready = false;
    bool ro_big = false;                     // large envs: k_observe + k_rollout_big, state in HBM
    bool ro_small_e = false;                 // LDS-sized envs on the large-env path: few envs (small_e_max)
    // Batches of at most this many LDS-sized envs take the queue kernel (MFX_SMALL_E overrides)
    static int small_e_max() {
        const char* v = getenv("MFX_SMALL_E");
        return v ? atoi(v) : kSmallEMax;
    }
    RolloutArgs ra{};
    DevBuf<float> ro_view[kMaxGroups], ro_feat[kMaxGroups], ro_rewards, ro_return;
    DevBuf<float> ro_mm;                     // large envs: next observation's minimap   [E][G][169]
    DevBuf<uint32_t> ro_info;                //             and per-id hp/max | group     [E][cap]
    DevBuf<uint32_t> ro_sort;                //             band-ordered moves            [E][acap]
    DevBuf<uint32_t> ro_items;               //             observation work items        [2][E*G*slots]
    DevBuf<int32_t> ro_cnt;                  //             their counters                [split][2][2]
    int ro_item_grid = 0;                    //             persistent grid of k_observe_items
    // large envs, queue-driven (k_rollout_bigq, default): one launch per ro_sub steps of every env
    bool ro_bigq = false;
    bool ro_bigq_want = true;                // MFX_BIG_FUSED=0 at rollout_init: the two-stream pipeline (A/B)
    DevBuf<uint32_t> ro_q_items, ro_q_si;    // [2][kXcds][list cap] tagged items; [E] next step index
    DevBuf<uint8_t> ro_snap;                 // few_pipe: [E][2] observation snapshots
    DevBuf<int32_t> ro_q_step;               // few_pipe: [kXcds] stepper claims
    DevBuf<int32_t> ro_q_cnt, ro_q_left, ro_q_done;
    int ro_q_grid = 0, ro_qpar = 0;
    uint32_t ro_qlaunch = 0;                 // launches so far (item tags)
    // Large envs on the queue kernel (not pipelined): the envs run in ro_qchunks consecutive launches per block of
    // steps, each over one chunk of envs with queues of its own.  One launch over all envs slows past ~2048 envs at
    // 256x256 (0.80 of the HBM roofline at 2048, 0.77 at 2560, 0.71 at 3072, 0.62-0.64 at 4096, ~0.3 MB of env state
    // each); 4096 envs as two launches of 2048 run at 0.79, while 3072 as two of 1536 gain nothing (0.711 vs 0.714):
    // so the chunks are at least kBigqChunkBytes of state (2048 envs at 256x256) -- floor(state / kBigqChunkBytes)
    // of them (profiles/r05_bigq_chunks.txt).
    static constexpr int kMaxQChunks = 8;
    static constexpr size_t kBigqChunkBytes = (size_t)2048 * 312648;
    int ro_qchunks = 1;
    int ro_qc_e0[kMaxQChunks + 1] = {};
    int ro_qc_par[kMaxQChunks] = {};
    uint32_t ro_qc_launch[kMaxQChunks] = {};
    State ro_qc_s[kMaxQChunks];
    RolloutArgs ro_qc_ra[kMaxQChunks];
    DevBuf<RolloutCtx> ro_qc_ctx;
    static uint32_t qtag(uint32_t launch) { return launch % 63u + 1u; }   // 6 tag bits (rollout_big.inc), never 0
    bool ro_prep_stale = true;               // ro_mm / ro_info / items lag the state (per-call calls since)
    DevBuf<int32_t> ro_actions, ro_eplen, ro_tx, ro_ty;
    DevBuf<double> ro_mean, ro_stats;
    DevBuf<unsigned long long> ro_steps;
    DevBuf<int32_t> ro_work;                 // k_rollout work-queue counters (2)
    DevBuf<int32_t> ro_cls_cnt, ro_cls_list; // k_rollout work queue (weight-class lists)
    uint64_t ro_launch = 0;                  // launches so far (queue phase = ro_launch % 6)
    DevBuf<uint4> ro_image;                  // reset image (k_reset_image)
    DevBuf<uint4> ro_walls;                  // its cells without the agents (RolloutArgs::wall_image)
    bool cells_stale = false;                // State::cells lags the fused rollout (sync_cells)
    bool walls_after_init = false;           // walls added after rollout_init: not in the rollout's cells
    DevBuf<RolloutCtx> ro_ctx;               // device copy of {s, ra} read by k_rollout
    RolloutCtx ro_ctx_host{};
    int ro_grid = 0, ro_cap = 0;
    // fused rollout: consecutive steps of each env per k_rollout launch (env image kept in LDS between
    // them; the launch's ramp-up / tail and the install / write-back are paid once per ro_sub steps)
    int ro_sub = 1;                          // 0: chosen per path and batch (sub_steps)
    // large-env path: the envs split into ro_split independent sub-batches, each a pipeline
    // (k_observe_items -> k_rollout_big) on its own stream, so one sub-batch's latency-bound step
    // overlaps the other's HBM-bound observation.  Each item launch takes a third of the chip's
    // k_observe_items slots, leaving room for the other stream's step.  Measured at 256x256 / 4096
    // agents, 1024 envs (profiles/r01_big_sweeps.txt): 2 streams / 1/3 grid / 64-agent items best.
    static constexpr int kBigSplit = 2, kItemGridDiv = 3, kItemRows = 64;
    static constexpr int kBigqRows = 512;         // agents per k_rollout_bigq observation item (64: 9.6e8, 256: 1.06e9, 384-512: 1.08e9, 1024: 1.04e9; profiles/r02_bigq_sweeps.txt)
    static constexpr bool kPipeDefault = false;   // measured slower than the fused step
    // Batches of at most kSmallEMax LDS-sized envs run on k_rollout_bigq (64x64 / 256 agents, one MI355X,
    // profiles/r03_small_e_sweep.txt, r03_crossover.txt): 8 envs 0.0435 vs 0.0944 ms per step (k_rollout),
    // 64 envs 0.050 vs 0.121, 1024 envs 3.00e8 vs 2.59e8 agent-steps/s; k_rollout wins from 2048 envs on
    // (4.0e8 vs 3.2e8).  16-agent items: 0.0435 ms per step at 8 envs vs 0.0461 (32), 0.0497 (64), 0.0441 (8).
    static constexpr int kSmallEMax = 1024;
    static constexpr int kSmallERows = 16;
    // the pipelined few-env stepper: wave 0 alone steps envs of up to this many agents (k_rollout's threshold)
    static constexpr int kFewWaveMax = 64;
    // steps per launch: at most 64 (k_rollout, the queue kernel's item lists); the pipelined few-env form's lists
    // are sized for kMaxPipeSub (its item words' 6 step bits only guard the hand-off, modulo 64)
    static constexpr int kMaxSub = 64, kMaxPipeSub = 1024;
    static constexpr int kPipeStepPerCu = 4, kPipeObsPerCu = 2;
    int ro_split = kBigSplit;
    hipStream_t ro_str[kMaxSplit] = {};
    hipEvent_t ro_ev[kMaxSplit + 1] = {};
    State ro_sub_s[kMaxSplit];
    RolloutArgs ro_sub_ra[kMaxSplit];
    int ro_sub_n[kMaxSplit] = {};            // envs of sub-batch k
    int sub_envs(int k) const { return ro_sub_n[k]; }
    DevBuf<RolloutCtx> ro_sub_ctx;
    // observation/step pipeline (LDS-sized envs): k_rollout_obs on ro_str[0] observes every env
    // from one copy of the per-env state while k_rollout<.., kSplit> steps the same envs from it
    // and writes the other copy (tw); the copies trade places after every launch.
    bool ro_pipe = false;
    State tw{};                              // the other copy (the kTwin fields below)
    int tw_cap = -1, tw_E = -1;
    int ro_par = 0;                          // 0: s is ro_pipe_ctx[0].s
    int ro_obs_grid = 0;
    DevBuf<RolloutCtx> ro_pipe_ctx;          // [2]: {s, ra, tw} and {tw, ra, s} as planned
    RolloutCtx ro_pipe_host[2] = {};

    ~BattleEngine() {
        (void)quiesce();
        for (void* p : retired) (void)hipHostFree(p);
#ifdef MFX_STAMPS
        if (hst_n)
            fprintf(stderr, "[magent_amd stamps] fast_step host us: enter->posted %.2f posted->record %.2f record->return %.2f (%ld steps)\n",
                    hst[0] / hst_n, hst[1] / hst_n, hst[2] / hst_n, hst_n);
#endif
        for (auto& x : act_ev) if (x) (void)hipEventDestroy(x);
        release();
        for (auto& x : ro_str) if (x) (void)hipStreamDestroy(x);
        for (auto& x : ro_ev) if (x) (void)hipEventDestroy(x);
        if (own_stream && stream) (void)hipStreamDestroy(stream);
    }

    // envs [e0, e0 + n) of s / ra as a batch of their own (every per-env array offset by e0)
    State sub_state(int e0, int n) const {
        State q = s;
        const size_t G = (size_t)n_groups(), c = (size_t)s.cap, a = (size_t)s.acap, cn = (size_t)s.cells_n;
        q.E = n;
        q.cells += e0 * cn; q.xy += e0 * c; q.hp += e0 * c; q.next_r += e0 * c; q.last_r += e0 * c;
        q.last_act += e0 * c; q.op_obj += e0 * c; q.meta += e0 * c; q.grp_ids += e0 * G * c;
        q.grp_n += e0 * G; q.grp_dead += e0 * G; q.grp_reward += e0 * G; q.id_counter += e0; q.rng += e0;
        q.rid += e0 * c; q.rid_off += e0;
        q.atk += e0 * a; q.n_atk += e0; q.mov += e0 * a; q.n_mov += e0; q.done += e0;
        if (q.food) q.food += e0 * cn;
        q.idx_mark += e0;
        return q;
    }
    // The queue kernel's view of env chunk k (envs [e0, e0 + n)): every per-env array from e0, the chunk's own
    // queue lists and counters (rollout_plan sizes them: q_list_cap per list of one chunk).
    RolloutArgs chunk_args(int e0, int k) const {
        RolloutArgs q = ra;
        const int G = n_groups();
        const size_t rc = (size_t)ra.rowcap;
        for (int g = 0; g < G; g++) {
            const TypeParams& T = gp.type[g];
            q.view[g] += e0 * rc * T.view_w * T.view_h * gp.n_ch;
            q.feat[g] += e0 * rc * gp.feat_size[g];
        }
        q.actions += e0 * G * rc; q.rewards += e0 * G * rc; q.mean_act += (size_t)e0 * G * ra.mean_stride;
        q.ep_return += (size_t)e0 * G; q.ep_len += e0; q.stats += (size_t)e0 * 4; q.agent_steps += e0;
        if (q.obs_mm) { q.obs_mm += (size_t)e0 * G * 169; q.obs_info += (size_t)e0 * s.cap; }
        q.env_base = e0;
        if (q.big_sort) q.big_sort += (size_t)e0 * s.acap;
        q.q_items += (size_t)k * 2 * kXcds * ra.q_list_cap;
        q.q_cnt += (size_t)k * 2 * kXcds * kObsCntPad;
        q.q_left += e0; q.q_si += e0;
        return q;
    }
    // Bytes of one env's state a large-env step and its observation items cycle through (cells, the per-slot arrays,
    // the group lists, the action buffers, the observation's minimap and info words, the move sort buffer).
    size_t env_state_bytes() const {
        const size_t c = (size_t)s.cap, a = (size_t)s.acap, G = (size_t)n_groups();
        return (size_t)s.cells_n * 2 + c * (4 + 4 + 4 + 4 + 1 + 4 + 1 + 2 + 4) + G * c * 2 + 3 * a * 4 + G * 169 * 4;
    }
    RolloutArgs sub_args(int e0, int k) const {
        RolloutArgs q = ra;
        const int G = n_groups();
        const size_t rc = (size_t)ra.rowcap;
        for (int g = 0; g < G; g++) {
            const TypeParams& T = gp.type[g];
            q.view[g] += e0 * rc * T.view_w * T.view_h * gp.n_ch;
            q.feat[g] += e0 * rc * gp.feat_size[g];
        }
        q.actions += e0 * G * rc; q.rewards += e0 * G * rc; q.mean_act += (size_t)e0 * G * ra.mean_stride;
        q.ep_return += (size_t)e0 * G; q.ep_len += e0; q.stats += (size_t)e0 * 4; q.agent_steps += e0;
        if (q.obs_mm) { q.obs_mm += (size_t)e0 * G * 169; q.obs_info += (size_t)e0 * s.cap; }
        q.env_base = e0;
        if (q.big_sort) q.big_sort += (size_t)e0 * s.acap;
        if (q.obs_items) {   // sub-batch k's lists: obs_lists x obs_list_stride items from (e0 + kXcds k) env slots
            const size_t slots = (size_t)G * ((ra.rowcap + ra.obs_item_rows - 1) / ra.obs_item_rows);
            q.obs_items += ((size_t)e0 + (size_t)kXcds * k) * slots;
            q.obs_cnt += 2 * kXcds * kObsCntPad * k;
            const int n = sub_envs(k);
            q.obs_list_stride = (size_t)((n + ra.obs_lists - 1) / ra.obs_lists) * slots;
        }
        return q;
    }

    void release() {
        for (void* p : {(void*)s.cells, (void*)s.xy, (void*)s.hp, (void*)s.next_r, (void*)s.last_r,
                        (void*)s.last_act, (void*)s.op_obj, (void*)s.meta, (void*)s.grp_ids, (void*)s.grp_n,
                        (void*)s.grp_dead, (void*)s.grp_reward, (void*)s.id_counter, (void*)s.rng, (void*)s.atk,
                        (void*)s.n_atk, (void*)s.mov, (void*)s.n_mov, (void*)s.done, (void*)s.idx_mark, (void*)s.food,
                        (void*)s.rid, (void*)s.rid_off, (void*)d_sort, (void*)d_gp,
                        (void*)d_err})
            if (p) (void)hipFree(p);
        s = State{}; d_sort = nullptr; d_gp = nullptr; d_err = nullptr; allocated = false;
        free_twin();
    }

    // The per-env fields k_rollout reads and writes back (the pipeline keeps two copies of them).
    template <class F> static void twin_fields(State& a, State& b, F&& f) {
        f(a.xy, b.xy); f(a.hp, b.hp); f(a.next_r, b.next_r); f(a.last_r, b.last_r); f(a.last_act, b.last_act);
        f(a.op_obj, b.op_obj); f(a.meta, b.meta); f(a.grp_ids, b.grp_ids); f(a.grp_n, b.grp_n);
        f(a.grp_dead, b.grp_dead); f(a.grp_reward, b.grp_reward); f(a.id_counter, b.id_counter); f(a.rng, b.rng);
    }
    void free_twin() {
        State none{};
        twin_fields(tw, none, [](auto& p, auto&) { if (p) (void)hipFree(p); p = nullptr; });
        tw_cap = tw_E = -1;
        ro_par = 0;
    }
    void alloc_twin() {
        if (tw_cap == s.cap && tw_E == E) return;
        free_twin();
        const size_t c = (size_t)s.cap, G = (size_t)n_groups();
        alloc(tw.xy, E * c); alloc(tw.hp, E * c); alloc(tw.next_r, E * c); alloc(tw.last_r, E * c);
        alloc(tw.last_act, E * c); alloc(tw.op_obj, E * c); alloc(tw.meta, E * c); alloc(tw.grp_ids, E * G * c);
        alloc(tw.grp_n, E * G); alloc(tw.grp_dead, E * G); alloc(tw.grp_reward, E * G); alloc(tw.id_counter, E);
        alloc(tw.rng, E);
        tw_cap = s.cap; tw_E = E;
    }
    // s with tw's copies of the twin fields
    State twin_state() const {
        State t = s, x = tw;
        twin_fields(t, x, [](auto& a, auto& b) { a = b; });
        return t;
    }
    void swap_twin() { twin_fields(s, tw, [](auto& a, auto& b) { std::swap(a, b); }); }

    int n_groups() const { return (int)group_types.size(); }
    AgentTypeSpec& gtype(int g) { return types.at(group_types.at(g)); }
    int group2channel(int g) const { return (food ? 2 : 1) + g * (minimap ? 3 : 2); }
    int feature_size(int g) {
        int f = emb + gtype(g).n_action + 1;
        if (goal) f += 2;
        if (minimap) f += 2;
        return f;
    }

    // ------------------------------------------------------------------ config
    int set_config(const char* key, void* p) {
        MFX_CHECK(quiesce());
        touch();
        if (!strcmp(key, "map_width")) W = *(int*)p;
        else if (!strcmp(key, "map_height")) H = *(int*)p;
        else if (!strcmp(key, "food_mode")) food = *(bool*)p;
        else if (!strcmp(key, "turn_mode")) turn = *(bool*)p;
        else if (!strcmp(key, "minimap_mode")) minimap = *(bool*)p;
        else if (!strcmp(key, "goal_mode")) goal = *(bool*)p;
        else if (!strcmp(key, "embedding_size")) emb = *(int*)p;
        else if (!strcmp(key, "render_dir")) render_dir = (const char*)p;
        else if (!strcmp(key, "seed")) {
            const unsigned long sv = (unsigned long)(long)*(int*)p;
            const uint64_t x = sv % 2147483647UL;
            rng_init = x ? (uint32_t)x : 1u;
            if (allocated) {
                std::vector<uint32_t> h((size_t)E, rng_init);
                MFX_HIP(hipMemcpyAsync(s.rng, h.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice, stream));
                MFX_HIP(hipStreamSynchronize(stream));
            }
        } else return fail("invalid argument in set_config: %s", key);
        return 0;
    }

    int register_type(const char* name, int n, const char** keys, const float* values) {
        MFX_CHECK(quiesce());
        touch();
        if (types.count(name)) return fail("duplicated name of agent type: %s", name);
        AgentTypeSpec t;
        t.name = name;
        for (int i = 0; i < n; i++) {
            const char* k = keys[i];
            const float v = values[i];
#define MFX_I(f) if (!strcmp(k, #f)) { t.f = (int)(v + 0.5); continue; }
#define MFX_F(f) if (!strcmp(k, #f)) { t.f = v; continue; }
#define MFX_B(f) if (!strcmp(k, #f)) { t.f = (bool)(int)(v + 0.5); continue; }
            MFX_I(width) MFX_I(length) MFX_F(speed) MFX_F(hp) MFX_F(view_radius) MFX_F(view_angle)
            MFX_F(attack_radius) MFX_F(attack_angle) MFX_F(hear_radius) MFX_F(speak_radius)
            MFX_I(speak_ability) MFX_F(damage) MFX_F(trace) MFX_F(eat_ability) MFX_F(step_recover)
            MFX_F(kill_supply) MFX_F(food_supply) MFX_B(attack_in_group) MFX_B(can_absorb)
            MFX_F(step_reward) MFX_F(kill_reward) MFX_F(dead_penalty) MFX_F(attack_penalty)
#undef MFX_I
#undef MFX_F
#undef MFX_B
            // accepted and then recomputed from the body size (AgentType.cc:117-120)
            if (!strcmp(k, "view_x_offset") || !strcmp(k, "view_y_offset") || !strcmp(k, "att_x_offset") ||
                !strcmp(k, "att_y_offset") || !strcmp(k, "turn_x_offset") || !strcmp(k, "turn_y_offset"))
                continue;
            return fail("invalid agent config in register_agent_type: %s", k);
        }
        if (t.width < 1 || t.length < 1 || t.width > 8 || t.length > 8)
            return fail("agent bodies must be 1..8 cells wide and long");
        const int parity = t.width % 2;
        if (t.view_angle >= 180) {
            if (std::fabs(t.view_angle - 360) > 1e-5) return fail("only angle = 360 when angle > 180");
            t.view = circle_range(t.view_radius, 0, parity);
        } else t.view = sector_range(t.view_angle, t.view_radius, parity);
        if (t.attack_angle >= 180) {
            if (std::fabs(t.attack_angle - 360) > 1e-5) return fail("only angle = 360 when angle > 180");
            t.attack = circle_range(t.attack_radius, t.width / 2.0f, parity);
        } else t.attack = sector_range(t.attack_angle, t.attack_radius, parity);
        t.move = circle_range(t.speed, 0, 1);
        t.turn_base = t.move.count;
        t.attack_base = turn ? t.turn_base + 2 : t.turn_base;      // AgentType.cc:118-122 (turn at register)
        t.n_action = t.attack_base + t.attack.count;
        if (t.view.w * t.view.h > kMaxViewCells || t.view.w <= 0 || t.view.h <= 0)
            return fail("view range too large (max %d cells)", kMaxViewCells);
        if (t.move.count > kMaxRangeCount || t.attack.count > kMaxRangeCount)
            return fail("move/attack range too large (max %d cells)", kMaxRangeCount);
        types.emplace(t.name, std::move(t));
        return 0;
    }

    int new_group(const char* type_name, int* group) {
        MFX_CHECK(quiesce());
        touch();
        if (!types.count(type_name)) return fail("invalid name of agent type in new_group: %s", type_name);
        if (n_groups() >= kMaxGroups) return fail("at most %d groups", kMaxGroups);
        if (allocated) return fail("new_group after the first reset is not supported");
        *group = n_groups();
        group_types.push_back(type_name);
        return 0;
    }

    // ------------------------------------------------------------------ reward DSL
    // The common rule form handled by RuleParams (k_step / k_rollout without the interpreter).
    bool simple_rule(const Rule& R) const {
        if (R.on < 0 || R.on >= (int)nodes.size()) return false;
        const Node& N = nodes[R.on];
        if (N.op != kEvAttack && N.op != kEvKill && N.op != kEvCollide) return false;
        if (N.raw.size() < 2) return false;
        const int sa = N.raw[0], sb = N.raw[1];
        if (sa < 0 || sb < 0 || sa >= (int)syms.size() || sb >= (int)syms.size()) return false;
        if (syms[sa].index != -1 || syms[sb].index != -1 || syms[sa].group == syms[sb].group) return false;
        if ((int)R.recv.size() > kMaxRecv) return false;
        for (int x : R.recv)
            if (x != sa && x != sb) return false;
        return true;
    }

    // related_symbols / infer_map of a node (GridWorld::collect_related_symbol, RewardEngine.cc:68-101):
    // std::set / std::map keyed by AgentSymbol*, i.e. ordered by symbol number; map insertion keeps
    // the first entry for a key.
    int node_symbols(int ni, std::set<int>& rel, std::map<int, int>& infer, int depth) const {
        if (ni < 0 || ni >= (int)nodes.size() || depth > kMaxNodes)
            return fail("reward DSL: bad event node %d", ni);
        const Node& N = nodes[ni];
        const auto need = [&](size_t k) { return N.raw.size() >= k; };
        switch (N.op) {
            case kEvAnd: case kEvOr: {
                if (!need(2)) return fail("reward DSL: malformed node %d", ni);
                std::set<int> r0, r1; std::map<int, int> m0, m1;
                MFX_CHECK(node_symbols(N.raw[0], r0, m0, depth + 1));
                MFX_CHECK(node_symbols(N.raw[1], r1, m1, depth + 1));
                rel.insert(r0.begin(), r0.end()); rel.insert(r1.begin(), r1.end());
                infer.insert(m0.begin(), m0.end()); infer.insert(m1.begin(), m1.end());
                return 0;
            }
            case kEvNot: {
                if (!need(1)) return fail("reward DSL: malformed node %d", ni);
                std::set<int> r0; std::map<int, int> m0;
                MFX_CHECK(node_symbols(N.raw[0], r0, m0, depth + 1));
                rel.insert(r0.begin(), r0.end()); infer.insert(m0.begin(), m0.end());
                return 0;
            }
            case kEvKill: case kEvCollide: case kEvAttack:
                if (!need(2)) return fail("reward DSL: malformed node %d", ni);
                rel.insert(N.raw[0]); rel.insert(N.raw[1]);
                infer.insert(std::make_pair(N.raw[0], N.raw[1]));
                return 0;
            case kEvAt: case kEvIn: case kEvDie: case kEvInALine:
                if (!need(N.op == kEvAt ? 3 : N.op == kEvIn ? 5 : 1)) return fail("reward DSL: malformed node %d", ni);
                rel.insert(N.raw[0]);
                return 0;
            case kEvAlign:
                // reads counter_x / counter_y, which the reference allocates and never fills
                // (GridWorld.cc:99-100, :1039-1050 commented out): no defined result to reproduce
                return fail("reward DSL: 'align' reads uninitialised engine memory in the reference; not supported");
            default:
                return fail("reward DSL: invalid event op %d", N.op);
        }
    }

    int post_order(int ni, std::vector<int>& out, int depth) const {
        if (depth > kMaxNodes) return fail("reward DSL: event graph too deep");
        if (std::find(out.begin(), out.end(), ni) != out.end()) return 0;
        const Node& N = nodes[ni];
        if (N.op == kEvAnd || N.op == kEvOr) {
            MFX_CHECK(post_order(N.raw[0], out, depth + 1));
            MFX_CHECK(post_order(N.raw[1], out, depth + 1));
        } else if (N.op == kEvNot) {
            MFX_CHECK(post_order(N.raw[0], out, depth + 1));
        }
        out.push_back(ni);
        return 0;
    }

    // GridWorld::init_reward_description (RewardEngine.cc:105-208) into a DslProgram.
    int compile_dsl(DslProgram& P) const {
        P = DslProgram{};
        if ((int)syms.size() > kMaxSyms) return fail("reward DSL: at most %d agent symbols", kMaxSyms);
        if ((int)nodes.size() > kMaxNodes) return fail("reward DSL: at most %d event nodes", kMaxNodes);
        const int G = n_groups();
        for (size_t i = 0; i < syms.size(); i++) {
            if (syms[i].group < 0 || syms[i].group >= G) return fail("reward DSL: symbol %zu has no valid group", i);
            if (syms[i].index < -2) return fail("reward DSL: symbol %zu has a bad index", i);
            P.sym[i] = DslSym{syms[i].group, syms[i].index};
        }
        auto sym_ok = [&](int x) { return x >= 0 && x < (int)syms.size(); };
        for (size_t i = 0; i < nodes.size(); i++) {
            const Node& N = nodes[i];
            DslNode& D = P.node[i];
            D = DslNode{N.op, -1, -1, 0, 0, 0, 0};
            const auto raw = [&](size_t k) { return k < N.raw.size() ? N.raw[k] : -1; };
            D.a = raw(0); D.b = raw(1);
            switch (N.op) {
                case kEvAnd: case kEvOr: case kEvNot:
                    if (D.a < 0 || D.a >= (int)nodes.size() || (N.op != kEvNot && (D.b < 0 || D.b >= (int)nodes.size())))
                        return fail("reward DSL: node %zu has a bad input", i);
                    break;
                case kEvKill: case kEvCollide: case kEvAttack:
                    if (!sym_ok(D.a) || !sym_ok(D.b)) return fail("reward DSL: node %zu has a bad symbol", i);
                    if (syms[D.b].index == -2)       // assert(!symbol_input[1]->is_all()) (RewardEngine.cc:221)
                        return fail("reward DSL: the object of attack/kill/collide cannot be a whole group");
                    break;
                case kEvAt:
                    if (!sym_ok(D.a)) return fail("reward DSL: node %zu has a bad symbol", i);
                    D.i0 = raw(1); D.i1 = raw(2);
                    break;
                case kEvIn:
                    if (!sym_ok(D.a)) return fail("reward DSL: node %zu has a bad symbol", i);
                    D.i0 = raw(1); D.i1 = raw(2); D.i2 = raw(3); D.i3 = raw(4);
                    break;
                case kEvDie:
                    if (!sym_ok(D.a)) return fail("reward DSL: node %zu has a bad symbol", i);
                    break;
                case kEvInALine:
                    if (!sym_ok(D.a) || syms[D.a].index != -2)      // assert(is_all()) (RewardEngine.cc:260)
                        return fail("reward DSL: in_a_line needs a whole-group symbol");
                    break;
                default:
                    break;                     // reported by node_symbols when a rule uses it
            }
        }
        P.n_rules = (int)rules.size();
        for (size_t r = 0; r < rules.size(); r++) {
            const Rule& R = rules[r];
            DslRule& D = P.rule[r];
            std::set<int> rel;
            std::map<int, int> infer;
            MFX_CHECK(node_symbols(R.on, rel, infer, 0));
            // input symbols: first the inferable subjects with their objects, then the rest
            std::vector<int> in, inf;
            std::set<int> added;
            for (int x : rel) {
                if (added.count(x)) continue;
                auto it = infer.find(x);
                if (it != infer.end()) {
                    in.push_back(x); inf.push_back(it->second);
                    added.insert(x); added.insert(it->second);
                }
            }
            for (int x : rel)
                if (!added.count(x)) { in.push_back(x); inf.push_back(-1); }
            if ((int)in.size() > kMaxSyms) return fail("reward rule %zu: too many symbols", r);
            D.n_in = (int)in.size();
            for (size_t k = 0; k < in.size(); k++) { D.in_sym[k] = (int8_t)in[k]; D.infer[k] = (int8_t)inf[k]; }
            std::vector<int> post;
            MFX_CHECK(post_order(R.on, post, 0));
            D.n_post = (int)post.size();
            for (size_t k = 0; k < post.size(); k++) D.post[k] = (int8_t)post[k];
            if ((int)R.recv.size() > kMaxRecv) return fail("reward rule %zu: too many receivers", r);
            D.n_recv = (int)R.recv.size();
            D.terminal = R.terminal;
            for (size_t k = 0; k < R.recv.size(); k++) {
                const int x = R.recv[k];
                if (!sym_ok(x)) return fail("reward rule %zu: bad receiver", r);
                // a receiver is bound only if the event involves it (RewardEngine.cc:191-193)
                if (syms[x].index != -2 && !rel.count(x))
                    return fail("reward rule %zu: receiver %d is not involved in the triggering event", r, x);
                D.recv[k] = (int8_t)x;
                D.val[k] = R.val[k];
            }
        }
        return 0;
    }

    // ------------------------------------------------------------------ compile
    int build_params() {
        const int G = n_groups();
        if (W <= 0 || H <= 0) return fail("map_width/map_height not set");
        if (W > 0xFFFF || H > 0xFFFF) return fail("map too large");
        if (G == 0) return fail("no groups");
        GameParams p{};
        p.W = W; p.H = H; p.n_groups = G; p.minimap = minimap; p.emb = emb;
        p.turn_mode = turn; p.food_mode = food;
        p.n_ch = group2channel(G);
        if ((long)W * H > 99 * 99) { large_map = true; n_sep = (long)W * H > 1000 * 1000 ? 16 : 8; }  // sticky
        p.large_map = large_map; p.n_sep = n_sep; p.band_w = (W + n_sep - 1) / n_sep;
        for (int g = 0; g < G; g++) {
            AgentTypeSpec& t = gtype(g);
            TypeParams& T = p.type[g];
            T.hp = t.hp; T.damage = t.damage; T.step_recover = t.step_recover; T.kill_supply = t.kill_supply;
            T.step_reward = t.step_reward; T.kill_reward = t.kill_reward; T.dead_penalty = t.dead_penalty;
            T.attack_penalty = t.attack_penalty; T.attack_in_group = t.attack_in_group;
            T.can_absorb = t.can_absorb;
            T.n_action = t.n_action; T.turn_base = t.turn_base; T.attack_base = t.attack_base;
            T.n_move = t.move.count; T.n_attack = t.attack.count;
            T.view_w = t.view.w; T.view_h = t.view.h;
            T.view_x1 = t.width / 2 + t.view.x1;     // eye = pos + view offset (Map.cc:146-149)
            T.view_y1 = t.length / 2 + t.view.y1;
            T.att_x_off = t.width / 2; T.att_y_off = t.length / 2;
            T.body_w = t.width; T.body_h = t.length;
            T.view_off_x = t.width / 2; T.view_off_y = t.length / 2;
            T.view_lt_x = t.view.x1; T.view_lt_y = t.view.y1;
            T.eat_ability = t.eat_ability; T.food_supply = t.food_supply;
            for (int i = 0; i < t.move.count; i++) { T.move_dx[i] = (int8_t)t.move.dx[i]; T.move_dy[i] = (int8_t)t.move.dy[i]; }
            for (int i = 0; i < t.attack.count; i++) { T.att_dx[i] = (int8_t)t.attack.dx[i]; T.att_dy[i] = (int8_t)t.attack.dy[i]; }
            for (int i = 0; i < t.view.w * t.view.h; i++) {
                T.view_mask[i] = t.view.in[i];
                if (t.view.in[i]) T.view_bits[i >> 5] |= 1u << (i & 31);
            }
            p.feat_size[g] = feature_size(g);
        }
        // reward rules: the common form (one attack/kill/collide event between 'any' agents of two
        // groups, receivers among its subject/object) runs data-parallel (RuleParams); anything else
        // goes through the DSL interpreter (DslProgram), rule order preserved either way.
        if ((int)rules.size() > kMaxRules) return fail("at most %d reward rules", kMaxRules);
        bool simple = true;
        for (size_t r = 0; r < rules.size() && simple; r++) simple = simple_rule(rules[r]);
        p.n_rules = 0;
        p.dsl = 0;
        if (simple) {
            p.n_rules = (int)rules.size();
            for (size_t r = 0; r < rules.size(); r++) {
                const Rule& R = rules[r];
                const Node& N = nodes[R.on];
                const int sa = N.raw[0], sb = N.raw[1];
                RuleParams& RP = p.rules[r];
                RP.op = N.op == kEvAttack ? kOpAttack : (N.op == kEvKill ? kOpKill : kOpCollide);
                RP.subj_group = syms[sa].group; RP.obj_group = syms[sb].group;
                RP.n_recv = (int)R.recv.size(); RP.terminal = R.terminal;
                for (size_t k = 0; k < R.recv.size(); k++) {
                    RP.recv_is_obj[k] = R.recv[k] == sb;
                    RP.val[k] = R.val[k];
                }
            }
        } else {
            MFX_CHECK(compile_dsl(p.prog));
            p.dsl = 1;
        }
        p.record_events = first_render ? 0 : 1;
        p.par_step = 1;
        // kill_supply != 0 keeps the parallel forms: the per-call step's wave attack models it (<= 64 attackers),
        // every other attack falls back to the serial walk inside the step (step_env_core)
        // (round 5 stepped them serially throughout: forest 74 -> 30 us per step, r06_generic_step_times.jsonl).
        // Bodies larger than 1x1 keep them too (the per-call step's move_wave_body / attack_wave<.., true>) unless an
        // attack cell can fall on the attacker's own body: a self-hit would have to kill its attacker at its own turn,
        // which the fixed point's "alive at its turn" test does not model (circle ranges exclude the body).
        for (int g = 0; g < p.n_groups; g++) {
            const TypeParams& T = p.type[g];
            bool self_hit = false;
            for (int k = 0; k < T.n_attack; k++) {
                const int cx = T.att_x_off + T.att_dx[k], cy = T.att_y_off + T.att_dy[k];
                self_hit = self_hit || (cx >= 0 && cx < T.body_w && cy >= 0 && cy < T.body_h);
            }
            p.par_step &= !self_hit && !T.can_absorb;     // absorption: the serial move (do_move_one)
        }
        // turn and food mode run on k_step<.., kBody>'s wave forms (the other kernels walk them serially)
        gp = p;
        return 0;
    }

    template <class T> static void alloc(T*& ptr, size_t n) {
        MFX_HIP_THROW(hipMalloc(&ptr, sizeof(T) * std::max<size_t>(n, 1)));
    }

    // (Re)allocate per-agent arrays with a new capacity, preserving contents row by row.
    template <class T> void grow(T*& ptr, size_t rows, size_t old_cap, size_t new_cap) {
        T* np;
        alloc(np, rows * new_cap);
        if (ptr && old_cap)
            MFX_HIP_THROW(hipMemcpy2DAsync(np, new_cap * sizeof(T), ptr, old_cap * sizeof(T), old_cap * sizeof(T),
                                           rows, hipMemcpyDeviceToDevice, stream));
        MFX_HIP_THROW(hipStreamSynchronize(stream));
        if (ptr) (void)hipFree(ptr);
        ptr = np;
    }

    void ensure_capacity(int need_ids, int need_actions) {
        if ((need_ids > s.cap || need_actions > s.acap) && quiesce() != 0) throw HipFailure("resident server: stop failed");
        const int G = n_groups();
        if (need_ids > s.cap) {
            int nc = std::max(64, s.cap);
            while (nc < need_ids) nc *= 2;
            if (nc > kCellFood) nc = kCellFood;        // ids stay below the cell codes
            const int oc = s.cap;
            grow(s.xy, E, oc, nc); grow(s.hp, E, oc, nc); grow(s.next_r, E, oc, nc); grow(s.last_r, E, oc, nc);
            grow(s.last_act, E, oc, nc); grow(s.op_obj, E, oc, nc); grow(s.meta, E, oc, nc);
            grow(s.grp_ids, (size_t)E * G, oc, nc);
            grow(s.rid, E, oc, nc);
            s.cap = nc;
            MFX_HIP_THROW(launch_rid_fill(s, oc, stream));   // new slots: slot == id until renumbered
            MFX_HIP_THROW(hipStreamSynchronize(stream));
        }
        if (need_actions > s.acap) {
            int na = std::max(128, s.acap);
            while (na < need_actions) na *= 2;
            const int oa = s.acap;
            grow(s.atk, E, oa, na); grow(s.mov, E, oa, na); grow(d_sort, E, oa, na);
            if (s.ev) (void)hipFree(s.ev);
            alloc(s.ev, 1 + (size_t)3 * na);
            MFX_HIP_THROW(hipMemset(s.ev, 0, sizeof(int32_t)));
            s.acap = na;
        }
    }

    int reset() {
        MFX_CHECK(flush_deferred());
        touch();
        for (int g = 0; g < kMaxGroups; g++) acts_since_step[g] = 0;
        ro_prep_stale = true;
        MFX_CHECK(build_params());
        try {
            const int G = n_groups();
            if (!allocated) {
                MFX_HIP_THROW(hipGetDevice(&device));
                if (!stream_set) { MFX_HIP_THROW(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)); own_stream = true; }
                s.E = E;
                s.cells_n = W * H;
                alloc(s.cells, (size_t)E * W * H);
                alloc(s.grp_n, (size_t)E * G); alloc(s.grp_dead, (size_t)E * G); alloc(s.grp_reward, (size_t)E * G);
                alloc(s.id_counter, E); alloc(s.rng, E); alloc(s.n_atk, E); alloc(s.n_mov, E); alloc(s.done, E);
                alloc(s.idx_mark, E); alloc(s.rid_off, E);
                if (food) alloc(s.food, (size_t)E * W * H);
                MFX_HIP_THROW(hipMemset(s.grp_reward, 0, sizeof(float) * E * G));   // Group ctor
                alloc(d_gp, 1); alloc(d_err, 1);
                MFX_HIP_THROW(hipMemset(d_err, 0, sizeof(int32_t)));
                s.err = d_err;
                std::vector<uint32_t> h((size_t)E, rng_init);
                MFX_HIP_THROW(hipMemcpy(s.rng, h.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice));
                group_ub.assign(G, 0);
                allocated = true;
                ensure_capacity(64, 128);
            } else if (s.cells_n != W * H) {
                return fail("map size changed after the first reset");
            }
            if (food && !s.food) alloc(s.food, (size_t)E * W * H);
            MFX_HIP_THROW(hipMemcpyAsync(d_gp, &gp, sizeof(GameParams), hipMemcpyHostToDevice, stream));
            MFX_HIP_THROW(launch_reset(d_gp, s, stream));
            cells_stale = false;
            next_file();                              // GridWorld.cc:102
            max_ids = 0;
            std::fill(group_ub.begin(), group_ub.end(), 0);
            pending_ub = 0;
            return 0;
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
    }

    // same placement for every env (host arrays)
    int add_agents(int group, int n, const char* method, const int* xs, const int* ys, const int* dirs) {
        MFX_CHECK(flush_deferred());
        touch();
        ro_prep_stale = true;
        if (!allocated) return fail("add_agents before reset");
        if (group >= n_groups() || group < -1) return fail("invalid group handle in add_agents: %d", group);
        MFX_CHECK(sync_cells());
        if (group < 0 && rollout_ready) walls_after_init = true;
        int m, count;
        std::vector<int> hx, hy, hd;
        if (!strcmp(method, "custom")) {
            m = 0; count = n;
            hx.assign(xs, xs + n); hy.assign(ys, ys + n);
            if (group >= 0) {                                  // GridWorld.cc:259-261
                hd.assign((size_t)n, kDirNorth);
                for (int i = 0; i < n && dirs; i++) {
                    if (dirs[i] >= 4) return fail("invalid direction in GridWorld::add_agent");
                    hd[i] = dirs[i];
                }
            }
        } else if (!strcmp(method, "random")) {
            m = 1; count = n;
        } else if (!strcmp(method, "fill")) {
            m = 2; count = std::max(0, xs[2]) * std::max(0, xs[3]);
            hx.assign(xs, xs + (turn && group >= 0 ? 5 : 4));   // {x, y, w, h, dir} (GridWorld.cc:270-273)
            if (turn && group >= 0 && (hx[4] < 0 || hx[4] >= 4)) return fail("invalid direction in GridWorld::add_agent");
        } else return fail("unsupported method in add_agents: %s", method);
        try {
            if (group >= 0) {
                ensure_capacity(max_ids + count, 0);
                max_ids += count;
                group_ub[group] += count;
            }
            if (hx.empty()) hx.push_back(0);
            if (hy.empty()) hy.push_back(0);
            if (hd.empty()) hd.push_back(kDirNorth);
            st_xs.ensure(hx.size()); st_ys.ensure(hy.size()); st_dirs.ensure(hd.size());
            MFX_HIP_THROW(hipMemcpyAsync(st_xs.p, hx.data(), sizeof(int) * hx.size(), hipMemcpyHostToDevice, stream));
            MFX_HIP_THROW(hipMemcpyAsync(st_ys.p, hy.data(), sizeof(int) * hy.size(), hipMemcpyHostToDevice, stream));
            MFX_HIP_THROW(hipMemcpyAsync(st_dirs.p, hd.data(), sizeof(int) * hd.size(), hipMemcpyHostToDevice, stream));
            MFX_HIP_THROW(launch_add_agents(d_gp, s, group, n, m, st_xs.p, st_ys.p, st_dirs.p, 0, stream));
            MFX_HIP_THROW(hipStreamSynchronize(stream));   // host vectors go out of scope
            return check_err();
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
    }

    // GridWorld::set_goal (GridWorld.cc:729-740): "random" only, goals never read back.
    int set_goal(int group, const char* method) {
        MFX_CHECK(flush_deferred());
        touch();
        if (strcmp(method, "random")) return fail("invalid goal type in GridWorld::set_goal");
        if (!allocated || group < 0 || group >= n_groups()) return fail("set_goal: bad state or group");
        MFX_HIP(launch_set_goal_random(d_gp, s, group, stream));
        MFX_HIP(hipStreamSynchronize(stream));
        return 0;
    }

    int check_err() {
        MFX_CHECK(quiesce());
        int32_t h = 0;
        MFX_HIP(hipMemcpyAsync(&h, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        MFX_HIP(hipStreamSynchronize(stream));
        if (h) {
            MFX_HIP(hipMemsetAsync(d_err, 0, sizeof(int32_t), stream));
            static const char* msg[] = {"", "", "agent capacity exceeded", "no blank position for random placement",
                                        "output row capacity smaller than the group", "invalid action id",
                                        "action buffer overflow", "move claim table outside the step scratch"};
            return fail("device error %d: %s", h, h > 0 && h < 8 ? msg[h] : "unknown");
        }
        return 0;
    }

    void touch() { ++epoch; }                // any state change of env 0 (drop-in host cache)

    int report_err(int32_t h) {
        if (!h) return 0;
        MFX_CHECK(quiesce());
        MFX_HIP(hipMemsetAsync(d_err, 0, sizeof(int32_t), stream));
        static const char* msg[] = {"", "", "agent capacity exceeded", "no blank position for random placement",
                                    "output row capacity smaller than the group", "invalid action id",
                                    "action buffer overflow", "move claim table outside the step scratch"};
        return fail("device error %d: %s", h, h > 0 && h < 8 ? msg[h] : "unknown");
    }

    // env 0's record (k_get_env0): 64-B header (group sizes, error word, done), then per group
    // ids | rewards | positions | alive, info_rows rows each
    static constexpr size_t kInfoRowBytes = 4 + 4 + 8 + 1;
    size_t info_region() const { return ((info_rows * kInfoRowBytes) + 15) & ~(size_t)15; }
    size_t info_off(int g, int what) const {         // in the record at info_src
        const size_t r = info_src_rows;
        const size_t base = 64 + (size_t)g * (((r * kInfoRowBytes) + 15) & ~(size_t)15);
        if (what == kGetId) return base;
        if (what == kGetReward) return base + r * 4;
        if (what == kGetPos) return base + r * 8;
        return base + r * 16;                                        // kGetAlive
    }
    const int32_t* info_hdr() const { return reinterpret_cast<const int32_t*>(info_src); }

    // Queue the record's launch and its one copy to pinned memory (no sync).
    int queue_info() {
        const int G = n_groups();
        size_t rows = 1;
        for (int g = 0; g < G; g++) rows = std::max(rows, (size_t)std::max(group_ub[g], 1));
        try {
            if (rows > info_rows) info_rows = rows;
            st_info.ensure(64 + (size_t)G * info_region());
            pin_info.ensure(64 + (size_t)G * info_region());
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        MFX_HIP(launch_get_env0(d_gp, s, st_info.p, (int)info_rows, stream));
        MFX_HIP(hipMemcpyAsync(pin_info.p, st_info.p, 64 + (size_t)G * info_region(), hipMemcpyDeviceToHost, stream));
        return 0;
    }

    // after the sync that follows queue_info (or k_dropin_step): this epoch's group sizes and info are
    // on the host, in the record at src
    int take_info(const uint8_t* src = nullptr, size_t rows = 0) {
        info_src = src ? src : pin_info.p;
        info_src_rows = src ? rows : info_rows;
        for (int g = 0; g < n_groups(); g++) hn[g] = info_hdr()[g];
        n_ep = info_ep = epoch;
        return report_err(info_hdr()[kMaxGroups]);
    }

    int ensure_info() {
        if (info_ep == epoch) return 0;
        MFX_CHECK(flush_deferred());
        MFX_CHECK(queue_info());
        MFX_HIP(hipStreamSynchronize(stream));
        return take_info();
    }
    int ensure_counts() { return n_ep == epoch ? 0 : ensure_info(); }

    int num_env0(int g) {
        if (!allocated) return 0;
        if (ensure_counts() != 0) return 0;
        return hn[g];
    }

    size_t obs_off_view(int g) const { return (size_t)g * obs_rows * obs_row_bytes(); }
    size_t obs_row_bytes() const {
        size_t b = 0;
        for (int g = 0; g < n_groups(); g++) {
            const TypeParams& T = gp.type[g];
            b = std::max(b, (size_t)4 * ((size_t)T.view_w * T.view_h * gp.n_ch + gp.feat_size[g]));
        }
        return (b + 15) & ~(size_t)15;
    }

    // views + features of every group of env 0 (and the info of the same epoch) in one transfer
    int ensure_obs() {
        if (obs_ep == epoch) return 0;
        MFX_CHECK(flush_deferred());
        MFX_CHECK(ensure_counts());
        obs_fast = false;
        const int G = n_groups();
        int rowcap = 4;
        for (int g = 0; g < G; g++) rowcap = std::max(rowcap, group_ub[g]);
        rowcap = (rowcap + 3) & ~3;
        size_t vmax = 0, fmax = 0;
        for (int g = 0; g < G; g++) {
            const TypeParams& T = gp.type[g];
            vmax = std::max(vmax, (size_t)T.view_w * T.view_h * gp.n_ch);
            fmax = std::max(fmax, (size_t)gp.feat_size[g]);
        }
        try {
            obs_rows = std::max(obs_rows, (size_t)rowcap);
            st_view.ensure((size_t)G * E * rowcap * (vmax + fmax));   // (+ fmax: the packed one-env layout)
            st_feat.ensure((size_t)G * E * rowcap * fmax);
            pin_obs.ensure((size_t)G * obs_rows * obs_row_bytes());
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        obs_packed = E == 1;
        if (obs_packed) {
            // one env: every group's views, each followed by its features, back to back in the
            // staging buffer and in pin_obs -- one copy for all of it
            size_t off = 0;
            for (int g = 0; g < G; g++) {
                const TypeParams& T = gp.type[g];
                const size_t VF = (size_t)T.view_w * T.view_h * gp.n_ch, F = gp.feat_size[g];
                obs_pack_off[g] = off;
                if (!hn[g]) continue;
                float* dv = st_view.p + off;
                MFX_CHECK(observe(g, dv, dv + (size_t)hn[g] * VF, rowcap));
                off += (size_t)hn[g] * (VF + F);
            }
            if (off) MFX_HIP(hipMemcpyAsync(pin_obs.p, st_view.p, sizeof(float) * off, hipMemcpyDeviceToHost, stream));
        } else {
            for (int g = 0; g < G; g++) {
                if (!hn[g]) continue;
                const TypeParams& T = gp.type[g];
                const size_t VF = (size_t)T.view_w * T.view_h * gp.n_ch, F = gp.feat_size[g];
                float* dv = st_view.p + (size_t)g * E * rowcap * vmax;
                float* df = st_feat.p + (size_t)g * E * rowcap * fmax;
                MFX_CHECK(observe(g, dv, df, rowcap));
                uint8_t* hv = pin_obs.p + obs_off_view(g);
                MFX_HIP(hipMemcpyAsync(hv, dv, sizeof(float) * hn[g] * VF, hipMemcpyDeviceToHost, stream));
                MFX_HIP(hipMemcpyAsync(hv + sizeof(float) * obs_rows * VF, df, sizeof(float) * hn[g] * F,
                                       hipMemcpyDeviceToHost, stream));
            }
        }
        MFX_CHECK(queue_info());                 // this epoch's ids (and the error word) ride along
        MFX_HIP(hipStreamSynchronize(stream));
        obs_ep = epoch;
        return take_info();
    }

    // ------------------------------------------------------------------ batched device API
    // The fused rollout keeps the cells in LDS only; rebuild State::cells before the per-call path
    // (or anything else that reads them) runs after rollout steps.
    int sync_cells() {
        if (!cells_stale) return 0;
        MFX_HIP(launch_rebuild_cells(d_gp, s, ro_walls.p, stream));
        cells_stale = false;
        return 0;
    }

    int observe(int g, float* d_view, float* d_feat, int rowcap) {
        if (!allocated || g < 0 || g >= n_groups()) return fail("observe: bad state or group");
        MFX_CHECK(flush_deferred());
        MFX_CHECK(sync_cells());
        MFX_HIP(launch_observe(gp, d_gp, s, g, group_ub[g], d_view, d_feat, rowcap, stream));
        return 0;
    }
    int set_action(int g, const int* d_actions, int rowcap) {
        MFX_CHECK(flush_deferred());
        touch();
        if (g >= 0 && g < kMaxGroups) acts_since_step[g]++;
        if (!allocated || g < 0 || g >= n_groups()) return fail("set_action: bad state or group");
        pending_ub += group_ub[g];
        try { ensure_capacity(0, pending_ub); } catch (const HipFailure& f) { return fail("%s", f.what()); }
        MFX_HIP(launch_set_action(d_gp, s, g, d_actions, rowcap, stream));
        return 0;
    }
    // A group's set_action called twice before a step: the serial forms (see State::serial_step).
    void begin_step() {
        s.serial_step = 0;
        for (int g = 0; g < kMaxGroups; g++) { s.serial_step |= acts_since_step[g] > 1; acts_since_step[g] = 0; }
    }
    int step(int* d_done) {
        MFX_CHECK(flush_deferred());
        touch();
        ro_prep_stale = true;
        if (!allocated) return fail("step before reset");
        MFX_CHECK(sync_cells());
        begin_step();
        const hipError_t le = launch_step(gp, d_gp, s, max_ids, d_sort, stream);
        s.serial_step = 0;
        MFX_HIP(le);
        pending_ub = 0;
        if (d_done) MFX_HIP(hipMemcpyAsync(d_done, s.done, sizeof(int32_t) * E, hipMemcpyDeviceToDevice, stream));
        return 0;
    }
    int get(int g, int what, void* d_out, int rowcap) {
        if (!allocated || g < 0 || g >= n_groups()) return fail("get: bad state or group");
        MFX_CHECK(flush_deferred());
        MFX_HIP(launch_get(d_gp, s, g, what, d_out, rowcap, stream));
        return 0;
    }
    int clear_dead() {
        MFX_CHECK(flush_deferred());
        touch();
        ro_prep_stale = true;
        if (!allocated) return fail("clear_dead before reset");
        MFX_HIP(launch_clear_dead(d_gp, s, stream));
        return 0;
    }

    // ------------------------------------------------------------------ fused rollout
    // Template placement per group (host arrays, applied in group order at every episode start),
    // followed by an immediate reset + placement of every env.
    int rollout_init(const int* tmpl_n, const int* const* xs, const int* const* ys, int max_steps, float eps,
                     uint32_t seed, int stagger) {
        MFX_CHECK(flush_deferred());
        const int G = n_groups();
        if (!allocated) MFX_CHECK(reset());
        int total = 0, rowcap = 4, tcap = 1;
        for (int g = 0; g < G; g++) { total += tmpl_n[g]; rowcap = std::max(rowcap, tmpl_n[g]); tcap = std::max(tcap, tmpl_n[g]); }
        rowcap = (rowcap + 3) & ~3;                      // 16-B aligned rows (4 * 1183 floats)
        for (int g = 0; g < G; g++) {
            if (gtype(g).n_action > 64) return fail("rollout: n_action must be <= 64");
            if (gp.type[g].view_w != gp.type[0].view_w || gp.type[g].view_h != gp.type[0].view_h)
                return fail("rollout: every group must share one view size; use the per-call API");
        }
        if (gp.dsl) return fail("rollout: reward rules outside the attack/kill/collide form need the per-call API");
        if (turn || food) return fail("rollout: turn_mode / food_mode need the per-call API");
        for (int g = 0; g < G; g++)
            if (gp.type[g].body_w != 1 || gp.type[g].body_h != 1) return fail("rollout: 1x1 bodies only; use the per-call API");
        for (int g = 0; g < G; g++)
            if (gp.type[g].can_absorb) return fail("rollout: can_absorb types need the per-call API");
        try {
            ensure_capacity(total, total);
            {
                const char* fv = getenv("MFX_BIG_FUSED");
                ro_bigq_want = !(fv && atoi(fv) == 0);
            }
            const size_t smem = rollout_smem_bytes(gp, s.cells_n, s.cap, s.acap, rowcap);
            // envs too large for one workgroup's LDS run k_observe + k_rollout_big with the state in HBM
            ro_big = smem > 160 * 1024;
            if (ro_big && (!gp.par_step || big_step_smem_bytes(gp, s.cap, s.acap, true) > 160 * 1024))
                return fail("rollout: env too large for the fused kernels (%zu bytes of LDS); use the per-call API", smem);
            // few envs (configs[3]: 8 per GPU): one workgroup per env would leave the chip idle and put each
            // env's whole observation on one CU; the queue kernel spreads every env's observation over many
            // workgroups (small items) and steps it in HBM, like the large envs
            ro_small_e = !ro_big && battle_shape(gp) && n_groups() == 2 && gp.par_step && E <= small_e_max() &&
                         big_step_smem_bytes(gp, s.cap, s.acap, true) <= 160 * 1024;
            if (ro_small_e) ro_big = true;
            std::vector<int> hx((size_t)G * tcap, 0), hy((size_t)G * tcap, 0);
            for (int g = 0; g < G; g++)
                for (int i = 0; i < tmpl_n[g]; i++) { hx[(size_t)g * tcap + i] = xs[g][i]; hy[(size_t)g * tcap + i] = ys[g][i]; }
            ro_tx.ensure(hx.size()); ro_ty.ensure(hy.size());
            MFX_HIP_THROW(hipMemcpy(ro_tx.p, hx.data(), sizeof(int) * hx.size(), hipMemcpyHostToDevice));
            MFX_HIP_THROW(hipMemcpy(ro_ty.p, hy.data(), sizeof(int) * hy.size(), hipMemcpyHostToDevice));
            RolloutArgs a{};
            for (int g = 0; g < G; g++) {
                const TypeParams& T = gp.type[g];
                ro_view[g].ensure((size_t)E * rowcap * T.view_w * T.view_h * gp.n_ch);
                ro_feat[g].ensure((size_t)E * rowcap * gp.feat_size[g]);
                a.view[g] = ro_view[g].p; a.feat[g] = ro_feat[g].p;
                a.tmpl_n[g] = tmpl_n[g];
            }
            int na = 0;
            for (int g = 0; g < G; g++) na = std::max(na, gtype(g).n_action);
            ro_actions.ensure((size_t)E * G * rowcap); ro_rewards.ensure((size_t)E * G * rowcap);
            ro_mean.ensure((size_t)E * G * na); ro_return.ensure((size_t)E * G); ro_eplen.ensure(E);
            ro_stats.ensure((size_t)E * 4); ro_steps.ensure(E);
            MFX_HIP_THROW(hipMemset(ro_return.p, 0, sizeof(float) * E * G));
            MFX_HIP_THROW(hipMemset(ro_mean.p, 0, sizeof(double) * ro_mean.n));   // former_act_prob = 0 at step 0
            // stagger episode phases over envs: env e's first episode is cut at max_steps - e*max_steps/E,
            // so after max_steps steps the batch cycles through every phase of an episode uniformly
            std::vector<int32_t> phase((size_t)E);
            for (int e = 0; e < E; e++) phase[e] = stagger ? (int32_t)((long long)e * max_steps / E) : 0;
            MFX_HIP_THROW(hipMemcpy(ro_eplen.p, phase.data(), sizeof(int32_t) * E, hipMemcpyHostToDevice));
            MFX_HIP_THROW(hipMemset(ro_stats.p, 0, sizeof(double) * E * 4));
            MFX_HIP_THROW(hipMemset(ro_steps.p, 0, sizeof(unsigned long long) * E));
            a.rowcap = rowcap; a.actions = ro_actions.p; a.rewards = ro_rewards.p; a.mean_act = ro_mean.p;
            a.mean_stride = na;
            a.ep_return = ro_return.p; a.ep_len = ro_eplen.p; a.stats = ro_stats.p; a.agent_steps = ro_steps.p;
            a.tmpl_x = ro_tx.p; a.tmpl_y = ro_ty.p; a.tmpl_cap = tcap;
            a.max_steps = max_steps; a.policy_seed = seed; a.step_index = 0; a.eps = eps;
            ra = a;
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        MFX_CHECK(reset());
        for (int g = 0; g < G; g++) MFX_CHECK(add_agents(g, tmpl_n[g], "custom", xs[g], ys[g], nullptr));
        MFX_CHECK(rollout_plan());
        rollout_ready = true;
        walls_after_init = false;
        return 0;
    }

    // Reset image, work queue and persistent grid for the current capacity.
    int rollout_plan() {
        ro_prep_stale = true;                    // the large-env observation inputs follow the new plan
        try {
            ro_work.ensure(4);                   // [0..1] k_rollout, [2..3] k_rollout_obs
            MFX_HIP_THROW(hipMemsetAsync(ro_work.p, 0, 4 * sizeof(int32_t), stream));
            ro_image.ensure((rollout_reset_image_bytes(gp, s.cells_n, s.cap) + 15) / 16);
            // queue for the next launch: every env in class 0 in index order, other counts zero
            ro_cls_cnt.ensure(3 * 8); ro_cls_list.ensure((size_t)2 * 8 * E);
            const int qp = (int)(ro_launch % 6);
            std::vector<int32_t> cnt(3 * 8, 0), idx((size_t)E);
            cnt[(qp % 3) * 8] = E;
            for (int e = 0; e < E; e++) idx[e] = e;
            MFX_HIP_THROW(hipMemcpy(ro_cls_cnt.p, cnt.data(), sizeof(int32_t) * cnt.size(), hipMemcpyHostToDevice));
            MFX_HIP_THROW(hipMemcpy(ro_cls_list.p + (size_t)(qp & 1) * 8 * E, idx.data(), sizeof(int32_t) * E,
                                    hipMemcpyHostToDevice));
            ra.work = ro_work.p; ra.work_sel = 0; ra.reset_image = ro_image.p;
            ra.cls_cnt = ro_cls_cnt.p; ra.cls_list = ro_cls_list.p; ra.cls_stride = E;
            MFX_HIP_THROW(launch_reset_image(gp, d_gp, s, ra, ro_image.p, stream));
            {   // the walls of the reset image (agents removed), shared by every env's install
                std::vector<uint16_t> cells((size_t)s.cells_n);
                MFX_HIP_THROW(hipStreamSynchronize(stream));
                MFX_HIP_THROW(hipMemcpy(cells.data(), ro_image.p, cells.size() * 2, hipMemcpyDeviceToHost));
                for (auto& c : cells) if (c < kCellFood) c = kCellEmpty;
                ro_walls.ensure((cells.size() * 2 + 15) / 16);
                MFX_HIP_THROW(hipMemcpy(ro_walls.p, cells.data(), cells.size() * 2, hipMemcpyHostToDevice));
                ra.wall_image = ro_walls.p;
            }
            ra.renumber = 0;
            ra.lds_step = 0;
            ra.few_pipe = 0;
            if (ro_big) {
                ro_grid = E;
                ro_sort.ensure((size_t)E * s.acap);
                ra.big_sort = ro_sort.p;
                // envs too large for LDS: clear_dead renumbers the slots to the list order (dense per-slot
                // arrays); LDS-sized envs (few-env path) keep slot == id, as k_rollout assumes
                const char* rn = getenv("MFX_RENUMBER");       // A/B only: 0 = off, 2 = no identity fast path
                ra.renumber = ro_small_e ? 0 : (rn ? std::min(std::max(atoi(rn), 0), 2) : 1);
                // few LDS-sized envs: each env is staged in LDS for its step (big_env_step)
                const char* ls = getenv("MFX_LDS_STEP");                   // A/B only: 0 = the step in HBM
                ra.lds_step = ro_small_e && !(ls && atoi(ls) == 0);
                if (battle_shape(gp)) {
                    ro_mm.ensure((size_t)E * n_groups() * 169);
                    ro_info.ensure((size_t)E * s.cap);
                    ra.obs_mm = ro_mm.p; ra.obs_info = ro_info.p;
                    const int R = kItemRows;
                    const size_t slots = (size_t)(ra.rowcap + R - 1) / R;
                    // per sub-batch of n envs: obs_lists lists of ceil(n / obs_lists) envs' items each,
                    // i.e. at most n + kXcds env slots
                    const size_t par_stride = ((size_t)E + (size_t)kXcds * kMaxSplit) * n_groups() * slots;
                    ro_items.ensure(2 * par_stride);
                    ro_cnt.ensure(2 * kXcds * kObsCntPad * kMaxSplit);
                    ra.obs_lists = kXcds;                           // one list per XCD (profiles/r02_xcd_items_ab.txt)
                    ra.obs_items = ro_items.p; ra.obs_cnt = ro_cnt.p;
                    ra.obs_par_stride = par_stride; ra.obs_item_rows = R;
                    MFX_HIP_THROW(observe_items_grid(gp, R, &ro_item_grid));
                    ro_item_grid = std::max(1, ro_item_grid / kItemGridDiv);
                    if (ro_item_grid >= kXcds) ro_item_grid -= ro_item_grid % kXcds;   // as many per XCD
                    // the queue-driven kernel: item words hold 13 env bits and 6 chunk bits
                    const char* rv = getenv("MFX_BIGQ_ROWS");                  // sweeps only
                    const int Rq = rv && atoi(rv) > 0 ? atoi(rv) : (ro_small_e ? kSmallERows : kBigqRows);
                    const int chunks = (ra.rowcap + Rq - 1) / Rq;
                    ro_bigq = ro_bigq_want && E <= 8192 && chunks <= 64 && n_groups() == 2 &&
                              bigq_smem_bytes(gp, s.cap, s.acap, Rq, ra.lds_step) <= 160 * 1024;
                    if (ro_bigq) MFX_HIP_THROW(bigq_grid(gp, s.cap, s.acap, Rq, ra.lds_step, &ro_q_grid));
                    ro_bigq = ro_bigq && ro_q_grid > 0;          // (0: not one SPX device of 8 XCDs)
                    if (ro_bigq) {
                        // few envs with the env staged in LDS: the pipelined form (a stepper workgroup per env
                        // steps while the items observe its snapshot) while the steppers leave at least 3 of 4
                        // of every XCD's workgroups to the items
                        const char* fp = getenv("MFX_FEW_PIPE");                // A/B only: 0 = off
                        ra.few_pipe = ra.lds_step && E <= ro_q_grid / 4 && !(fp && atoi(fp) == 0) &&
                                      bigq_smem_bytes(gp, s.cap, s.acap, Rq, true, true) <= 160 * 1024;
                        if (ra.few_pipe) {
                            // (the stepper's scratch for the items it takes back follows its LDS layout)
                            int pg = 0;
                            MFX_HIP_THROW(bigq_grid(gp, s.cap, s.acap, Rq, true, &pg, true));
                            ra.few_pipe = E <= std::min(ro_q_grid, pg) / 4;
                            // (the pipe grid only when the pipelined form stays: the queue-step form keeps its
                            // full grid)
                            if (ra.few_pipe) ro_q_grid = std::min(ro_q_grid, pg);
                        }
                        // env chunks (not pipelined): envs per launch by the state bytes one launch cycles through
                        ro_qchunks = 1;
                        if (!ra.few_pipe) {
                            const char* qc = getenv("MFX_BIGQ_CHUNK");         // A/B and tests: envs per launch
                            if (qc) {
                                const long long want = atoll(qc);
                                if (want > 0 && want < E)
                                    ro_qchunks = (int)std::min<long long>(kMaxQChunks, (E + want - 1) / want);
                            } else {
                                const size_t k = (size_t)E * env_state_bytes() / kBigqChunkBytes;
                                ro_qchunks = (int)std::max<size_t>(1, std::min<size_t>(kMaxQChunks, k));
                            }
                        }
                        for (int k = 0; k <= ro_qchunks; ++k) ro_qc_e0[k] = (int)((long long)E * k / ro_qchunks);
                        const int qmax = (E + ro_qchunks - 1) / ro_qchunks;
                        // per list and parity: one filing per env and step of a launch (<= 64 steps; the
                        // pipelined form kMaxPipeSub) (+ the tickets workgroups hold past the last filing: two
                        // per workgroup); one such set per env chunk
                        const size_t lcap = (size_t)((qmax + kXcds - 1) / kXcds) * (ra.few_pipe ? kMaxPipeSub : 64) *
                                            (size_t)(n_groups() * chunks) + 2 * (size_t)ro_q_grid;
                        ro_q_items.ensure(2 * kXcds * lcap * ro_qchunks);
                        ro_q_cnt.ensure(2 * kXcds * kObsCntPad * ro_qchunks);
                        ro_q_left.ensure(E); ro_q_si.ensure(E); ro_q_done.ensure(kObsCntPad);
                        MFX_HIP_THROW(hipMemsetAsync(ro_q_items.p, 0, ro_q_items.n * sizeof(uint32_t), stream));
                        MFX_HIP_THROW(hipMemsetAsync(ro_q_done.p, 0, kObsCntPad * sizeof(int32_t), stream));
                        ra.q_items = ro_q_items.p; ra.q_cnt = ro_q_cnt.p; ra.q_left = ro_q_left.p;
                        ra.q_si = ro_q_si.p; ra.q_done = ro_q_done.p; ra.q_list_cap = lcap;
                        ra.obs_item_rows = Rq;
                        if (ra.few_pipe) {
                            // (at most 64: attack_wave / move_wave give each attacker and mover one lane)
                            ra.few_wave_max = kFewWaveMax;
                            ra.few_snap_bytes = few_snap_bytes(s.cells_n, s.cap, n_groups());
                            ro_snap.ensure((size_t)E * 2 * ra.few_snap_bytes);
                            ro_q_step.ensure(kXcds);
                            ra.few_snap = ro_snap.p; ra.q_step = ro_q_step.p;
                            // one workgroup per CU while that leaves 3 of 4 to the items: the stepper then has its
                            // CU to itself (8 envs 0.0222 -> 0.0219 ms per step, profiles/r04_few_grid_ab.txt)
                            int dev = 0, cus = 0;
                            if (hipGetDevice(&dev) == hipSuccess &&
                                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                                cus % kXcds == 0 && 4 * E <= cus)
                                ro_q_grid = std::min(ro_q_grid, cus);
                        }
                        const char* qg = getenv("MFX_BIGQ_GRID");               // sweeps only
                        // (a multiple of kXcds: every XCD's list needs workgroups of its own)
                        if (qg && atoi(qg) > 0)
                            ro_q_grid = std::min(ro_q_grid, std::max(kXcds, atoi(qg) - atoi(qg) % kXcds));
                    }
                } else {
                    ro_bigq = false;
                }
                const int K = std::min(ro_split, E);
                ro_sub_ctx.ensure(K);
                std::vector<RolloutCtx> subs(K);
                for (int k = 0; k < K; k++) {
                    const int e0 = (int)((long long)E * k / K), e1 = (int)((long long)E * (k + 1) / K);
                    ro_sub_n[k] = e1 - e0;
                    ro_sub_s[k] = sub_state(e0, e1 - e0);
                    ro_sub_ra[k] = sub_args(e0, k);
                    subs[k].s = ro_sub_s[k]; subs[k].ra = ro_sub_ra[k];
                    if (!ro_str[k]) MFX_HIP_THROW(hipStreamCreateWithFlags(&ro_str[k], hipStreamNonBlocking));
                }
                for (auto& x : ro_ev) if (!x) MFX_HIP_THROW(hipEventCreateWithFlags(&x, hipEventDisableTiming));
                MFX_HIP_THROW(hipMemcpyAsync(ro_sub_ctx.p, subs.data(), sizeof(RolloutCtx) * K, hipMemcpyHostToDevice,
                                             stream));
            } else {
                const char* pv = getenv("MFX_ROLLOUT_PIPE");
                ro_pipe = pv ? atoi(pv) != 0 : kPipeDefault;
                if (ro_pipe) {
                    MFX_HIP_THROW(rollout_grid(gp, s, ra.rowcap, 1, kPipeStepPerCu, &ro_grid));
                    MFX_HIP_THROW(rollout_obs_grid(gp, s, ra.rowcap, kPipeObsPerCu, &ro_obs_grid));
                    alloc_twin();
                    ro_par = 0;
                    ro_pipe_host[0].s = s; ro_pipe_host[0].ra = ra; ro_pipe_host[0].w = twin_state();
                    ro_pipe_host[1].s = twin_state(); ro_pipe_host[1].ra = ra; ro_pipe_host[1].w = s;
                    ro_pipe_ctx.ensure(2);
                    MFX_HIP_THROW(hipMemcpyAsync(ro_pipe_ctx.p, ro_pipe_host, sizeof(ro_pipe_host), hipMemcpyHostToDevice,
                                                 stream));
                    if (!ro_str[0]) MFX_HIP_THROW(hipStreamCreateWithFlags(&ro_str[0], hipStreamNonBlocking));
                    for (auto& x : ro_ev) if (!x) MFX_HIP_THROW(hipEventCreateWithFlags(&x, hipEventDisableTiming));
                } else {
                    MFX_HIP_THROW(rollout_grid(gp, s, ra.rowcap, 0, 0, &ro_grid));
                }
            }
            ro_cap = s.cap;
            ro_ctx.ensure(1);
            ro_ctx_host.s = s; ro_ctx_host.ra = ra; ro_ctx_host.w = s;
            MFX_HIP_THROW(hipMemcpyAsync(ro_ctx.p, &ro_ctx_host, sizeof(RolloutCtx), hipMemcpyHostToDevice, stream));
            if (ro_big && ro_bigq && !ra.few_pipe) {
                ro_qc_ctx.ensure(ro_qchunks);
                std::vector<RolloutCtx> qc(ro_qchunks);
                for (int k = 0; k < ro_qchunks; ++k) {
                    const int e0 = ro_qc_e0[k], n = ro_qc_e0[k + 1] - e0;
                    ro_qc_s[k] = ro_qchunks > 1 ? sub_state(e0, n) : s;
                    ro_qc_ra[k] = ro_qchunks > 1 ? chunk_args(e0, k) : ra;
                    qc[k].s = ro_qc_s[k]; qc[k].ra = ro_qc_ra[k]; qc[k].w = ro_qc_s[k];
                    ro_qc_par[k] = 0;
                    ro_qc_launch[k] = ro_qlaunch;
                }
                MFX_HIP_THROW(hipMemcpyAsync(ro_qc_ctx.p, qc.data(), sizeof(RolloutCtx) * ro_qchunks, hipMemcpyHostToDevice,
                                             stream));
            }
            MFX_HIP_THROW(hipStreamSynchronize(stream));
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        return 0;
    }

    int rollout_step(int n_steps) {
        MFX_CHECK(flush_deferred());
        touch();
        if (!rollout_ready) return fail("rollout_step before rollout_init");
        if (walls_after_init) return fail("rollout: walls added after rollout_init are not part of the rollout's episodes");
        {
            const State& planned = ro_pipe ? ro_pipe_host[ro_par].s : ro_ctx_host.s;
            if (s.cap != ro_cap || memcmp(&planned, &s, sizeof(State)) != 0) MFX_CHECK(rollout_plan());
        }
        if (ro_big && ro_bigq && ra.few_pipe) {
            // the pipelined few-env form: every launch files and observes its own items (parity 0, a fresh tag),
            // the steppers claimed per XCD; q_left must read 0 (no items outstanding) at a launch start
            MFX_CHECK(sync_cells());
            const size_t lst = (size_t)kXcds * kObsCntPad;
            if (ro_prep_stale) {
                ro_qlaunch++;
                MFX_HIP(hipMemsetAsync(ro_q_items.p, 0, ro_q_items.n * sizeof(uint32_t), stream));
                MFX_HIP(hipMemsetAsync(ro_q_done.p, 0, kObsCntPad * sizeof(int32_t), stream));
                MFX_HIP(hipMemsetAsync(ro_q_left.p, 0, (size_t)E * sizeof(int32_t), stream));
            }
            ro_prep_stale = false;
            for (int i = 0; i < n_steps;) {
                const int k = std::min(sub_steps(), n_steps - i);
                // a slot whose item its stepper took back keeps the stolen mark if no holder reached it before the
                // launch ended (k_rollout_bigq: bigq_wait / few_steal): clear the lists when the tag comes round
                if (qtag(ro_qlaunch) == 1)
                    MFX_HIP(hipMemsetAsync(ro_q_items.p, 0, ro_q_items.n * sizeof(uint32_t), stream));
                // (both parities: parity 1 holds the per-XCD done counts, k_rollout_bigq xcd_done)
                MFX_HIP(hipMemsetAsync(ro_q_cnt.p, 0, 2 * lst * sizeof(int32_t), stream));
                MFX_HIP(hipMemsetAsync(ro_q_step.p, 0, kXcds * sizeof(int32_t), stream));
                // (no BigqSerial: the pipelined form completes with one workgroup of its grid per XCD, and its grid
                // -- one or two workgroups per CU, at most half of an XCD's slots -- never holds a whole XCD)
                MFX_HIP(launch_rollout_bigq(gp, d_gp, s, ro_ctx.p, ra.obs_item_rows, ra.step_index, k, 0,
                                            qtag(ro_qlaunch), qtag(ro_qlaunch + 1), ro_q_grid,
                                            ra.lds_step, stream, true));
                ro_qlaunch++;
                ro_launch++;
                ra.step_index += k;
                i += k;
            }
            return 0;
        }
        if (ro_big && ro_bigq) {
            MFX_CHECK(sync_cells());
            const size_t lst = (size_t)kXcds * kObsCntPad;           // counters of one parity
            if (ro_prep_stale) {
                // Re-seed after per-call calls: the last launch's filings for the next launch (never
                // consumed) still hold the live tag in the slots past the new, smaller filing count --
                // clear every slot and move to a fresh tag, so no stale word can pass for an item.
#ifndef MFX_AB_R2_RESEED                 // A/B only: the round-2 re-seed, which the regression test must catch
                MFX_HIP(hipMemsetAsync(ro_q_items.p, 0, ro_q_items.n * sizeof(uint32_t), stream));
#endif
                MFX_HIP(hipMemsetAsync(ro_q_cnt.p, 0, ro_q_cnt.n * sizeof(int32_t), stream));
                MFX_HIP(hipMemsetAsync(ro_q_done.p, 0, kObsCntPad * sizeof(int32_t), stream));
                for (int c = 0; c < ro_qchunks; ++c) {
                    ro_qc_par[c] = 0;
#ifndef MFX_AB_R2_RESEED
                    ro_qc_launch[c]++;
#endif
                    MFX_HIP(launch_bigq_seed(d_gp, ro_qc_s[c], ro_qc_ra[c], 0, qtag(ro_qc_launch[c]), ra.step_index,
                                             stream));
                }
            }
            ro_prep_stale = false;
            // chunk after chunk, each through every launch of the n steps (the envs are independent; within a
            // chunk the launches chain as one batch's would)
            for (int c = 0; c < ro_qchunks; ++c) {
                int32_t* cnt = ro_q_cnt.p + (size_t)c * 2 * lst;
                uint32_t si = ra.step_index;
                for (int i = 0; i < n_steps;) {
                    const int k = std::min(sub_steps(), n_steps - i);
                    MFX_HIP(hipMemsetAsync(cnt + (ro_qc_par[c] ^ 1) * lst, 0, lst * sizeof(int32_t), stream));
                    BigqSerial serial(stream);
                    MFX_HIP(serial.status());
                    MFX_HIP(launch_rollout_bigq(gp, d_gp, ro_qc_s[c], ro_qc_ctx.p + c, ra.obs_item_rows, si, k,
                                                ro_qc_par[c], qtag(ro_qc_launch[c]), qtag(ro_qc_launch[c] + 1),
                                                ro_q_grid, ra.lds_step, stream));
                    ro_qc_par[c] ^= 1;
                    ro_qc_launch[c]++;
                    ro_launch++;
                    si += k;
                    i += k;
                }
            }
            ra.step_index += n_steps;
            return 0;
        }
        if (ro_big) {
            MFX_CHECK(sync_cells());
            const int K = std::min(ro_split, E);
            if (ra.obs_mm && ro_prep_stale) {
                if (ra.obs_items)
                    MFX_HIP(hipMemsetAsync(ro_cnt.p, 0, sizeof(int32_t) * 2 * kXcds * kObsCntPad * kMaxSplit, stream));
                for (int k = 0; k < K; k++)
                    MFX_HIP(launch_obs_prep(d_gp, ro_sub_s[k], ro_sub_ra[k], (int)(ra.step_index & 1), stream));
            }
            ro_prep_stale = false;
            // fork: every sub-batch stream waits for the caller's stream, the caller joins them all
            MFX_HIP(hipEventRecord(ro_ev[kMaxSplit], stream));
            for (int k = 0; k < K; k++) MFX_HIP(hipStreamWaitEvent(ro_str[k], ro_ev[kMaxSplit], 0));
            for (int i = 0; i < n_steps; i++) {
                for (int k = 0; k < K; k++) {
                    const State& q = ro_sub_s[k];
                    const RolloutArgs& qa = ro_sub_ra[k];
                    if (qa.obs_items) {
                        MFX_HIP(launch_observe_items(gp, d_gp, q, qa, (int)(ra.step_index & 1), ro_item_grid,
                                                     ro_str[k]));
                    } else {                           // generic (non-Battle-shape) observation
                        for (int g = 0; g < n_groups(); g++)
                            MFX_HIP(launch_observe(gp, d_gp, q, g, qa.rowcap, qa.view[g], qa.feat[g], qa.rowcap,
                                                   ro_str[k]));
                    }
                    MFX_HIP(launch_rollout_big(gp, d_gp, q, ro_sub_ctx.p + k, ra.step_index, ra.lds_step, ro_str[k]));
                }
                ro_launch++;
                ra.step_index++;
            }
            for (int k = 0; k < K; k++) {
                MFX_HIP(hipEventRecord(ro_ev[k], ro_str[k]));
                MFX_HIP(hipStreamWaitEvent(stream, ro_ev[k], 0));
            }
            return 0;
        }
        if (ro_pipe) {
            for (int i = 0; i < n_steps; i++) {
                const RolloutCtx* c = ro_pipe_ctx.p + ro_par;
                const int qp = (int)(ro_launch % 6);
                MFX_HIP(hipEventRecord(ro_ev[kMaxSplit], stream));
                MFX_HIP(hipStreamWaitEvent(ro_str[0], ro_ev[kMaxSplit], 0));
                MFX_HIP(launch_rollout_obs(gp, d_gp, s, c, ra.rowcap, ra.work_sel, qp, ro_obs_grid, ro_str[0]));
                MFX_HIP(launch_rollout(gp, d_gp, s, c, ra.rowcap, ra.step_index, ra.work_sel, qp, ro_grid, 1, 1, stream));
                MFX_HIP(hipEventRecord(ro_ev[0], ro_str[0]));
                MFX_HIP(hipStreamWaitEvent(stream, ro_ev[0], 0));
                swap_twin();                     // the written copy is the state now
                ro_par ^= 1;
                ro_launch++;
                ra.step_index++;
                ra.work_sel ^= 1;
                cells_stale = true;
            }
            return 0;
        }
        for (int i = 0; i < n_steps;) {
            const int k = std::min(sub_steps(), n_steps - i);
            MFX_HIP(launch_rollout(gp, d_gp, s, ro_ctx.p, ra.rowcap, ra.step_index, ra.work_sel, (int)(ro_launch % 6),
                                   ro_grid, 0, k, stream));
            ro_launch++;
            ra.step_index += k;
            ra.work_sel ^= 1;
            cells_stale = true;
            i += k;
        }
        return 0;
    }

    // A learned policy's launches (include/magent_amd.h mfx_battle_rollout_policy_step): mode 2 observes every
    // env into the rollout buffers; mode 1 acts with the actions in the rollout's action buffer (the
    // policy's forward on that observation), steps, and observes the new state.  The fused k_rollout only.
    int rollout_policy_step(int mode) {
        MFX_CHECK(flush_deferred());
        touch();
        if (!rollout_ready) return fail("rollout_policy_step before rollout_init");
        if (mode != 1 && mode != 2) return fail("rollout_policy_step: mode %d (1 step, 2 observe)", mode);
        if (walls_after_init) return fail("rollout: walls added after rollout_init are not part of the rollout's episodes");
        {
            const State& planned = ro_pipe ? ro_pipe_host[ro_par].s : ro_ctx_host.s;
            if (s.cap != ro_cap || memcmp(&planned, &s, sizeof(State)) != 0) MFX_CHECK(rollout_plan());
        }
        if (ro_big || ro_pipe)
            return fail("rollout_policy_step: a learned policy steps on the fused k_rollout (LDS-sized envs; batches of "
                        "more than %d envs or MFX_SMALL_E=0; MFX_ROLLOUT_PIPE=0)", small_e_max());
        MFX_HIP(launch_rollout_mode(gp, d_gp, s, ro_ctx.p, ra.rowcap, ra.step_index, ra.work_sel, (int)(ro_launch % 6),
                                    ro_grid, mode, stream));
        ro_launch++;
        if (mode == 1) ra.step_index++;
        ra.work_sel ^= 1;
        cells_stale = true;
        return 0;
    }

    // Synchronise and report the device error word and, on the queue-driven large-env kernel, its queue
    // error word: 0 if neither is set.
    int rollout_check() {
        if (!rollout_ready) return fail("rollout_check before rollout_init");
        if (ro_big && ro_bigq) {
            int32_t w[kObsCntPad] = {};
            MFX_HIP(hipMemcpyAsync(w, ro_q_done.p, sizeof(w), hipMemcpyDeviceToHost, stream));
            MFX_HIP(hipStreamSynchronize(stream));
            static const char* msg[] = {"", "", "a wait without progress (stalled queue)", "a ticket past the list",
                                        "a workgroup outside XCDs 0-7 (not one SPX device)",
                                        "hand-off guard: an item saw a step counter other than its own"};
            if (w[2]) return fail("rollout: k_rollout_bigq error %d: %s", w[2], w[2] > 0 && w[2] < 6 ? msg[w[2]] : "?");
        }
        return check_err();
    }

    // Which kernels rollout_step runs (include/magent_amd.h mfx_battle_rollout_path).
    int rollout_path() const {
        if (!rollout_ready) return -1;
        if (ro_big) return ro_bigq ? 3 : 2;
        return ro_pipe ? 1 : 0;
    }

    // Steps per launch: ro_sub, or with ro_sub 0 (mfx_battle_rollout_set_substeps(game, 0)) the measured best of the
    // path (profiles/r04_substeps_auto.txt, one MI355X): the pipelined few-env stepper kMaxPipeSub -- a launch ends
    // with its slowest env's steps (the envs step independently inside it), and a longer launch averages each env's
    // heavy early-episode steps with its light ones: 8 envs 0.0356 -> 0.0285 ms per step from 20 to 64 steps per
    // launch --, in practice the whole rollout_step(n) as one launch; k_rollout below 96 envs per CU 2 (its workgroups'
    // heaviest units end the launch: 8192 envs 0.556 -> 0.594 of peak, 16384 0.62 -> 0.63), else 20 (32768
    // envs 0.75 at 5, 0.77 at 20; the bench's 131072, 0.84-0.86); the large-env queue kernel 20.
    int sub_steps() const {
        // (one step per launch: the two-kernel observation / step pipeline and the large-env two-stream pipeline --
        // rollout_step launches those per step whatever ro_sub says)
        if (ro_pipe || (ro_big && !ro_bigq)) return 1;
        const bool pipe = ro_big && ro_bigq && ra.few_pipe;
        if (ro_sub > 0) return std::min(ro_sub, pipe ? kMaxPipeSub : kMaxSub);
        if (ro_big) return pipe ? kMaxPipeSub : 20;
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return E < 96 * cus ? 2 : 20;
    }

    // Lanes over which the rollout sums a group's rewards of an env with n agents (the order the episode
    // returns follow): k_rollout's wave 0 up to 64 agents, else its workgroup; the step of the large-env
    // and few-env queue paths (big_env_step) 512 lanes; the pipelined few-env stepper (few_env_step) k_rollout's
    // team forms: wave 0 up to 64 agents, else its 512-lane workgroup.
    int rollout_sum_lanes(int n) const {
        if (!rollout_ready) return -1;
        if (ro_big && ro_bigq && ra.few_pipe) return n <= ra.few_wave_max ? 64 : 512;
        if (ro_big) return 512;                       // kBigRolloutThreads (battle/rollout_big.inc)
        return n <= 64 ? 64 : 256;
    }

    int rollout_info(int* grid, int* lds_bytes) {
        if (!rollout_ready) return fail("rollout_info before rollout_init");
        *grid = ro_grid;
        *lds_bytes = (int)(ro_big ? big_step_smem_bytes(gp, s.cap, s.acap, true, ra.lds_step)
                                  : rollout_smem_bytes(gp, s.cells_n, s.cap, s.acap, ra.rowcap));
        return 0;
    }

    int rollout_buffer(const char* name, int group, void** ptr, size_t* bytes) {
        if (!rollout_ready) return fail("rollout_buffer before rollout_init");
        const int G = n_groups();
        if (group < 0 || group >= G) return fail("bad group");
        const TypeParams& T = gp.type[group];
        const size_t rc = ra.rowcap;
        if (!strcmp(name, "view")) { *ptr = ra.view[group]; *bytes = E * rc * T.view_w * T.view_h * gp.n_ch * 4; }
        else if (!strcmp(name, "feature")) { *ptr = ra.feat[group]; *bytes = E * rc * gp.feat_size[group] * 4; }
        else if (!strcmp(name, "actions")) { *ptr = ra.actions; *bytes = (size_t)E * G * rc * 4; }
        else if (!strcmp(name, "rewards")) { *ptr = ra.rewards; *bytes = (size_t)E * G * rc * 4; }
        else if (!strcmp(name, "mean_action")) { *ptr = ra.mean_act; *bytes = ro_mean.n * 8; }
        else if (!strcmp(name, "episode_return")) { *ptr = ra.ep_return; *bytes = (size_t)E * G * 4; }
        else if (!strcmp(name, "stats")) { *ptr = ra.stats; *bytes = (size_t)E * 4 * 8; }
        else if (!strcmp(name, "agent_steps")) { *ptr = ra.agent_steps; *bytes = (size_t)E * 8; }
        else if (!strcmp(name, "group_num")) { *ptr = s.grp_n; *bytes = (size_t)E * G * 4; }
        else return fail("unknown rollout buffer %s", name);
        return 0;
    }

    // ------------------------------------------------------------------ drop-in (env 0, host buffers)
    // The fast step applies to one env whose config the fused rollout supports and whose image plus
    // step / observation scratch fits one workgroup's LDS.
    size_t fast_rows_now() const {
        size_t r = 4;
        for (int g = 0; g < n_groups(); g++) r = std::max(r, (size_t)group_ub[g]);
        return (r + 3) & ~(size_t)3;
    }
    bool fast_dropin_ok() const {
        if (!fast_enabled || E != 1 || !allocated || gp.dsl || turn || food) return false;
        for (int g = 0; g < n_groups(); g++) {
            const TypeParams& T = gp.type[g];
            if (T.body_w != 1 || T.body_h != 1 || T.view_w != gp.type[0].view_w || T.view_h != gp.type[0].view_h)
                return false;
        }
        return dropin_smem_bytes(gp, s.cells_n, s.cap, s.acap, (int)fast_rows_now()) <= 160 * 1024;
    }
    // Run deferred set_action / clear_dead for real, in call order (clear_dead came first).
    // Stop the resident server (if one may be running) and wait until it has left: its LDS image
    // must not outlive a change made by anything else, and nothing else may wait behind it.
    int quiesce() {
        if (!res_live) return 0;
        res_live = false;
        DropinMailbox* mb = mbox.p;
        mb->cmd = kDropinStop;
        __atomic_store_n(&mb->req, ++fast_seq, __ATOMIC_RELEASE);
        MFX_HIP(hipStreamSynchronize(stream));
        return 0;
    }
    int flush_deferred() {
        MFX_CHECK(quiesce());
        bool acts = false;
        for (int g = 0; g < kMaxGroups; g++) acts |= defer_act[g];
        spec_ep = 0;
        if (!defer_clear && !acts) return 0;
        if (defer_clear) {
            defer_clear = false;
            MFX_HIP(launch_clear_dead(d_gp, s, stream));
        }
        for (int g = 0; g < n_groups(); g++) {
            if (!defer_act[g]) continue;
            defer_act[g] = false;
            const int rowcap = std::max(group_ub[g], 1);
            try { st_i32.ensure((size_t)E * rowcap); } catch (const HipFailure& f) { return fail("%s", f.what()); }
            if (defer_n[g])
                MFX_HIP(hipMemcpyAsync(st_i32.p, pin_fact.p + (size_t)g * fact_rows, sizeof(int) * defer_n[g],
                                       hipMemcpyHostToDevice, stream));
            MFX_HIP(launch_set_action(d_gp, s, g, st_i32.p, rowcap, stream));
        }
        if (acts) MFX_HIP(hipStreamSynchronize(stream));   // pin_fact may be rewritten next
        return 0;
    }
    // set_action deferred: the actions wait in host-mapped memory for the step's launch.
    int fast_set_action(int g, const int* actions) {
        if (defer_act[g]) MFX_CHECK(flush_deferred());      // a second call for the group before a step
        const int n = num_env0(g);
        const size_t rows = fast_rows_now();
        try {
            if (fact_rows < rows || pin_fact.n < (size_t)n_groups() * rows) {
                MFX_CHECK(flush_deferred());
                MFX_HIP_THROW(hipStreamSynchronize(stream));
                fact_rows = std::max(fact_rows, rows);
                pin_fact.ensure((size_t)n_groups() * fact_rows, hipHostMallocCoherent);
            }
            pending_ub += group_ub[g];
            ensure_capacity(0, pending_ub);
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        if (n) memcpy(pin_fact.p + (size_t)g * fact_rows, actions, sizeof(int) * n);
        // the resident server also finds them in its mailbox, tagged with the request that will carry
        // them (read in the same poll as the request, battle/dropin.inc dropin_wait)
        mail_tag[g] = ~0u;
        if (res_enabled && own_stream && env_flag("MFX_DROPIN_MAIL", false) &&
            (size_t)n_groups() * fact_rows <= (size_t)kMailActs) {
            bool ok = true;
            for (int i = 0; i < n && ok; i++) ok = (uint32_t)actions[i] <= 0xFFFFu;
            if (ok) {
                if (ensure_mbox() != 0) return -1;
                const uint32_t tag = (fast_seq + 1) & 0xFFFFu;
                uint32_t* d = mbox.p->acts + (size_t)g * fact_rows;
                for (int i = 0; i < n; i++) d[i] = (tag << 16) | (uint32_t)actions[i];
                mail_tag[g] = tag;
                mail_stride[g] = fact_rows;
            }
        }
        acts_since_step[g]++;
        defer_act[g] = true;
        defer_n[g] = n;
        const int keep_n = n_ep == epoch;
        touch();
        ro_prep_stale = true;
        spec_ep = 0;
        if (keep_n) n_ep = epoch;                           // group sizes do not change
        return 0;
    }
    // env.step(): one k_dropin_step launch and one sync.
#ifdef MFX_STAMPS
    // diagnostic build: host-side split of env.step() (enter -> request posted -> record seen -> return)
    double hst[3] = {0, 0, 0};
    long hst_n = 0;
    std::chrono::steady_clock::time_point hst_t0, hst_t1;
#endif
    int fast_step(int* done) {
#ifdef MFX_STAMPS
        hst_t0 = std::chrono::steady_clock::now();
#endif
        touch();
        ro_prep_stale = true;
        MFX_CHECK(sync_cells());
        const int G = n_groups();
        const size_t rows = fast_rows_now();
        DropinArgs da{};
        try {
            const size_t rec = (64 + (size_t)G * (((rows * kInfoRowBytes) + 15) & ~(size_t)15) + 255) & ~(size_t)255;
            // rec | observation set 0 | set 1: request k writes set k & 1, so the arrays a caller got
            // from get_observation (mfx_env_observation_view) stay intact through the next step
            size_t off = rec;
            size_t vo[kMaxGroups], fo[kMaxGroups];
            for (int g = 0; g < G; g++) {
                const TypeParams& T = gp.type[g];
                vo[g] = off; off = (off + rows * T.view_w * T.view_h * gp.n_ch * 4 + 255) & ~(size_t)255;
                fo[g] = off; off = (off + rows * gp.feat_size[g] * 4 + 255) & ~(size_t)255;
            }
            const size_t set_bytes = off - rec;
            off += set_bytes;
            if (pin_fast.n < off || (res_live && (int)rows != res_da.rows)) {
                if (quiesce() != 0) throw HipFailure("quiesce failed");
                MFX_HIP_THROW(hipStreamSynchronize(stream));   // the last launch may still write it
                if (pin_fast.n < off && pin_fast.p) {           // callers may still hold views of it
                    retired.push_back(pin_fast.p);
                    pin_fast.p = pin_fast.d = nullptr;
                    pin_fast.n = 0;
                }
                pin_fast.ensure(off, hipHostMallocCoherent);
            }
            fast_set_bytes = set_bytes;
            if (!pin_flag.p) {
                pin_flag.ensure(2, hipHostMallocCoherent);
                pin_flag.p[0] = pin_flag.p[1] = 0;
            }
            fast_rows = rows;
            fast_rec = rec;
            for (int g = 0; g < G; g++) { fast_view[g] = vo[g]; fast_feat[g] = fo[g]; }
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        for (int g = 0; g < G; g++) {
            da.acts[g] = defer_act[g] ? pin_fact.d + (size_t)g * fact_rows : nullptr;
            da.n_acts[g] = defer_act[g] ? defer_n[g] : 0;
            da.view[g] = reinterpret_cast<float*>(pin_fast.d + fast_view[g]);
            da.feat[g] = reinterpret_cast<float*>(pin_fast.d + fast_feat[g]);
        }
        da.pending_clear = defer_clear;
        da.obs_alt = fast_set_bytes / sizeof(float);
        da.rows = (int)rows;
        da.rec_step = pin_fast.d;
        da.flag = pin_flag.d;
        begin_step();
        fast_res = res_enabled && own_stream && !s.serial_step;
        if (fast_res) {
            MFX_CHECK(ensure_mbox());
            DropinMailbox* mb = mbox.p;
            const uint32_t seq = ++fast_seq;
            bool tagged = true;
            for (int g = 0; g < G; g++)
                if (defer_act[g] && (mail_tag[g] != (seq & 0xFFFFu) || mail_stride[g] != fact_rows)) tagged = false;
            mb->cmd = kDropinStep;
            mb->pending_clear = defer_clear;
            for (int g = 0; g < kMaxGroups; g++) mb->n_acts[g] = g < G && defer_act[g] ? defer_n[g] : -1;
            mb->tagged = tagged;
            mb->act_stride = (int32_t)std::max<size_t>(fact_rows, 1);
            // a server that left on its idle timeout wrote the last request it answered into done[3]
            // on its way out: relaunch it at once (wait_fast's stream query would notice ~100 us later)
            if (res_live && __atomic_load_n(&mb->done[3], __ATOMIC_ACQUIRE) == seq - 1) res_live = false;
            __atomic_store_n(&mb->req, seq, __ATOMIC_RELEASE);
            if (!res_live) {
                for (int g = 0; g < G; g++) da.acts[g] = pin_fact.d + (size_t)g * fact_rows;
                da.mb = mbox.d;
                da.seq = seq - 1;
                da.idle = res_idle_ticks();
                {   // MFX_DROPIN_MAIL=1: poll the tagged actions with the header (just the words they need)
                    const size_t words = 16 + (size_t)G * fact_rows;
                    da.mail_passes = words <= 256 ? 1 : words <= (size_t)kMailWords ? 2 : 0;
                    if (!env_flag("MFX_DROPIN_MAIL", false)) da.mail_passes = 0;   // measured neutral: off
                }
                da.variant = res_variant();
                res_da = da;
                MFX_HIP(launch_dropin_step(gp, d_gp, s, da, stream));
                res_live = true;
            }
        } else {
            MFX_CHECK(quiesce());
            da.seq = ++fast_seq;
            const hipError_t le = launch_dropin_step(gp, d_gp, s, da, stream);
            MFX_HIP(le);
        }
        s.serial_step = 0;
        obs_seq = fast_seq;
#ifdef MFX_STAMPS
        hst_t1 = std::chrono::steady_clock::now();
#endif
        MFX_CHECK(wait_fast(0, fast_seq));        // the records; the observation is still being written
#ifdef MFX_STAMPS
        const auto hst_t2 = std::chrono::steady_clock::now();
#endif
        defer_clear = false;
        for (int g = 0; g < kMaxGroups; g++) defer_act[g] = false;
        pending_ub = 0;
        MFX_CHECK(take_info(pin_fast.p, rows));
        *done = info_hdr()[kMaxGroups + 1];
        spec_ep = epoch;
#ifdef MFX_STAMPS
        const auto hst_t3 = std::chrono::steady_clock::now();
        hst[0] += std::chrono::duration<double, std::micro>(hst_t1 - hst_t0).count();
        hst[1] += std::chrono::duration<double, std::micro>(hst_t2 - hst_t1).count();
        hst[2] += std::chrono::duration<double, std::micro>(hst_t3 - hst_t2).count();
        hst_n++;
#endif
        return 0;
    }
    // Spin on k_dropin_step's completion word `which` (0 records, 1 observation) of request `seq`.
    // The stream is polled now and then, so a failed or faulted launch is reported instead of awaited;
    // a resident server that left on its idle timeout before seeing the request is launched again.
    int wait_fast(int which, uint32_t seq) {
        const bool res = fast_res;
        volatile uint32_t* f = res ? &mbox.p->done[which] : pin_flag.p + which;
        // the stream is queried every ~100 us of waiting (a query costs microseconds; polling it by
        // iteration count delayed the detection of the word)
        const auto t_start = std::chrono::steady_clock::now();
        auto t_next = t_start + std::chrono::microseconds(100);
        for (uint32_t k = 1, relaunched = 0;; k++) {
            if (*f == seq) break;
            if ((k & 63) == 0 && std::chrono::steady_clock::now() >= t_next) {
                t_next = std::chrono::steady_clock::now() + std::chrono::microseconds(100);
                if (t_next - t_start > std::chrono::seconds(20))
                    return fail("k_dropin_step: request %u unanswered after 20 s (word %d = %u)", seq, which, *f);
                const hipError_t q = hipStreamQuery(stream);
                if (q == hipSuccess) {
                    if (*f == seq) break;
                    if (res && res_live && seq == fast_seq && relaunched < 2) {
                        DropinArgs da = res_da;      // the request is still posted: serve it
                        da.seq = seq - 1;
                        MFX_HIP(launch_dropin_step(gp, d_gp, s, da, stream));
                        relaunched++;
                        res_relaunch++;
                        continue;
                    }
                    return fail("k_dropin_step finished without publishing word %d", which);
                }
                if (q != hipErrorNotReady) return fail("k_dropin_step: %s", hipGetErrorString(q));
            }
            __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return 0;
    }
    static int res_variant() {
        static const int v = getenv("MFX_DROPIN_VARIANT") ? atoi(getenv("MFX_DROPIN_VARIANT")) : 0;
        return v;
    }
    static long long res_idle_us() {                       // (read each time: tests change it)
        const char* v = getenv("MFX_DROPIN_IDLE_US");
        return v ? std::max(1, atoi(v)) : 2000;
    }
    unsigned long long res_idle_ticks() const {
        int dev = 0, khz = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
            khz <= 0)
            khz = 100000;                                  // gfx9: 100 MHz
        return (unsigned long long)res_idle_us() * (unsigned long long)khz / 1000ull;
    }
    // clear_dead right after a fast step: deferred; the step's launch already left what the getters
    // and get_observation ask next.
    int fast_clear_dead() {
        defer_clear = true;
        touch();
        ro_prep_stale = true;
        spec_ep = 0;
        // the record after clear_dead, from the step's record (clear_dead_env): the alive rows in
        // order, reward = next_r + group reward = step_reward + 0
        const size_t rows = fast_rows, region = ((rows * kInfoRowBytes) + 15) & ~(size_t)15;
        clr_rec.resize(fast_rec);
        const uint8_t* src = pin_fast.p;
        uint8_t* dst = clr_rec.data();
        memcpy(dst, src, 64);
        int32_t* hdr = reinterpret_cast<int32_t*>(dst);
        for (int g = 0; g < n_groups(); g++) {
            const int n = std::min(hdr[g], (int)rows);
            const uint8_t* b = src + 64 + (size_t)g * region;
            uint8_t* o = dst + 64 + (size_t)g * region;
            const int32_t* ids = reinterpret_cast<const int32_t*>(b);
            const int32_t* pos = reinterpret_cast<const int32_t*>(b + rows * 8);
            const uint8_t* alive = b + rows * 16;
            int32_t* oids = reinterpret_cast<int32_t*>(o);
            float* orew = reinterpret_cast<float*>(o + rows * 4);
            int32_t* opos = reinterpret_cast<int32_t*>(o + rows * 8);
            uint8_t* oalive = o + rows * 16;
            volatile float zero = 0.0f;
            const float r = gp.type[g].step_reward + zero;
            int k = 0;
            for (int i = 0; i < n; i++) {
                if (!alive[i]) continue;
                oids[k] = ids[i]; orew[k] = r; opos[2 * k] = pos[2 * i]; opos[2 * k + 1] = pos[2 * i + 1]; oalive[k] = 1;
                k++;
            }
            hdr[g] = k;
        }
        MFX_CHECK(take_info(dst, rows));
        obs_fast = true;
        obs_ep = epoch;
        return 0;
    }

    int host_observe(int g, float** bufs) {
        if (!allocated) return fail("get_observation before reset");
        if (g < 0 || g >= n_groups()) return fail("get_observation: bad group %d", g);
        MFX_CHECK(ensure_obs());
        const int n = hn[g];
        if (n == 0) return 0;
        const TypeParams& T = gp.type[g];
        const size_t VF = (size_t)T.view_w * T.view_h * gp.n_ch, F = gp.feat_size[g];
        if (obs_fast) {
            MFX_CHECK(wait_fast(1, obs_seq));
            const size_t o = (obs_seq & 1) ? fast_set_bytes : 0;
            memcpy(bufs[0], pin_fast.p + o + fast_view[g], sizeof(float) * n * VF);
            memcpy(bufs[1], pin_fast.p + o + fast_feat[g], sizeof(float) * n * F);
            return 0;
        }
        if (obs_packed) {
            const float* hv = reinterpret_cast<const float*>(pin_obs.p) + obs_pack_off[g];
            memcpy(bufs[0], hv, sizeof(float) * n * VF);
            memcpy(bufs[1], hv + (size_t)n * VF, sizeof(float) * n * F);
            return 0;
        }
        const uint8_t* hv = pin_obs.p + obs_off_view(g);
        memcpy(bufs[0], hv, sizeof(float) * n * VF);
        memcpy(bufs[1], hv + sizeof(float) * obs_rows * VF, sizeof(float) * n * F);
        return 0;
    }
    // get_observation without the copy: host pointers to env 0's observation of group g, written by
    // the drop-in step into pinned memory (the set of the last request; the next request writes the
    // other set, so they stay valid until the step after next).  1: not available (the caller copies
    // through host_observe).
    int observation_view(int g, float** view, float** feat, int* n, int* rows) {
        if (!allocated) return fail("get_observation before reset");
        if (g < 0 || g >= n_groups()) return fail("get_observation: bad group %d", g);
        MFX_CHECK(ensure_obs());
        if (!obs_fast) return 1;
        MFX_CHECK(wait_fast(1, obs_seq));
        const size_t o = (obs_seq & 1) ? fast_set_bytes : 0;
        *view = reinterpret_cast<float*>(pin_fast.p + o + fast_view[g]);
        *feat = reinterpret_cast<float*>(pin_fast.p + o + fast_feat[g]);
        *n = hn[g];
        *rows = (int)fast_rows;
        return 0;
    }
    // No sync: the actions go out of pinned memory (one region per group, reused once the previous
    // copy from it has left), the launch is queued, device errors surface at the next cache fetch.
    int host_set_action(int g, const int* actions) {
        if (!allocated) return fail("set_action before reset");
        if (g < 0 || g >= n_groups()) return fail("set_action: bad group %d", g);
        if (fast_dropin_ok()) return fast_set_action(g, actions);
        const int n = num_env0(g);
        const int rowcap = std::max(group_ub[g], 1);
        try {
            st_i32.ensure((size_t)E * rowcap);
            if (pin_act.n < (size_t)n_groups() * rowcap) {
                MFX_HIP_THROW(hipStreamSynchronize(stream));            // no copy may be in flight
                pin_act.ensure((size_t)n_groups() * rowcap);
            }
            if (!act_ev[g]) MFX_HIP_THROW(hipEventCreateWithFlags(&act_ev[g], hipEventDisableTiming));
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        const size_t stride = pin_act.n / n_groups();
        int32_t* pa = pin_act.p + (size_t)g * stride;
        MFX_HIP(hipEventSynchronize(act_ev[g]));
        if (n) {
            memcpy(pa, actions, sizeof(int) * n);
            MFX_HIP(hipMemcpyAsync(st_i32.p, pa, sizeof(int) * n, hipMemcpyHostToDevice, stream));
            MFX_HIP(hipEventRecord(act_ev[g], stream));
        }
        const int keep_n = n_ep == epoch;
        MFX_CHECK(set_action(g, st_i32.p, rowcap));   // a state change: last_act feeds the features
        if (keep_n) n_ep = epoch;                     // group sizes do not change
        return 0;
    }
    int host_step(int* done) {
        if (!allocated) return fail("step before reset");
        if (fast_dropin_ok()) return fast_step(done);
        MFX_CHECK(step(nullptr));
        MFX_CHECK(queue_info());                   // done + rewards / alive / positions in one transfer
        MFX_HIP(hipStreamSynchronize(stream));
        *done = info_hdr()[kMaxGroups + 1];
        return take_info();
    }
    // clear_dead without a sync: with this epoch's alive flags at hand, the new group sizes are known.
    int host_clear_dead() {
        if (spec_ep != 0 && spec_ep == epoch) return fast_clear_dead();
        const int G = n_groups();
        int nn[kMaxGroups] = {};
        const bool known = allocated && info_ep == epoch && n_ep == epoch;
        if (known)
            for (int g = 0; g < G; g++) {
                const uint8_t* al = info_src + info_off(g, kGetAlive);
                for (int i = 0; i < hn[g]; i++) nn[g] += al[i] != 0;
            }
        MFX_CHECK(clear_dead());
        if (known) { for (int g = 0; g < G; g++) hn[g] = nn[g]; n_ep = epoch; }
        return 0;
    }
    int host_get(int g, int what, void* out, size_t elem_bytes) {
        if (g < 0 || g >= n_groups()) return fail("get: bad group %d", g);
        const int n = num_env0(g);
        if (n == 0) return 0;
        if (what == kGetId || what == kGetReward || what == kGetPos || what == kGetAlive) {
            MFX_CHECK(ensure_info());
            memcpy(out, info_src + info_off(g, what), elem_bytes * n);
            return 0;
        }
        const int rowcap = std::max(group_ub[g], 1);
        st_u8.ensure((size_t)E * rowcap * elem_bytes);
        MFX_CHECK(get(g, what, st_u8.p, rowcap));
        MFX_HIP(hipMemcpyAsync(out, st_u8.p, elem_bytes * n, hipMemcpyDeviceToHost, stream));
        MFX_HIP(hipStreamSynchronize(stream));
        return check_err();
    }

    // One call per getter of the drop-in wrapper (mfx_env_get_rows): the group's size n, and for what 0 id /
    // 1 reward / 2 alive / 3 pos the n rows copied into out when n <= cap (what -1: the size only).
    int get_rows(int g, int what, void* out, int cap) {
        MFX_CHECK(sync_cells());
        if (g < 0 || g >= n_groups()) return fail("get_rows: bad group %d", g);
        if (what < -1 || what > 3) return fail("get_rows: bad field %d", what);
        if (!allocated) return 0;
        MFX_CHECK(ensure_counts());
        const int n = hn[g];
        if (what < 0 || n == 0 || n > cap) return n;
        static const int field[4] = {kGetId, kGetReward, kGetAlive, kGetPos};
        static const size_t bytes[4] = {4, 4, 1, 8};
        MFX_CHECK(host_get(g, field[what], out, bytes[what]));
        return n;
    }

    int get_info(int group, const char* name, void* buf) {   // GridWorld.cc:777-978
        int* ib = (int*)buf;
        const int G = n_groups();
        const bool need_group = strcmp(name, "both_attack") != 0;
        if (need_group && (group < 0 || group >= G)) return fail("invalid group %d for get_info(%s)", group, name);
        if (!strcmp(name, "num")) { if (!allocated) { ib[0] = 0; return 0; } ib[0] = num_env0(group); return 0; }
        if (!strcmp(name, "id")) return host_get(group, kGetId, buf, 4);
        if (!strcmp(name, "pos")) return host_get(group, kGetPos, buf, 8);
        if (!strcmp(name, "alive")) return host_get(group, kGetAlive, buf, 1);
        AgentTypeSpec& t = gtype(group);
        if (!strcmp(name, "action_space")) { ib[0] = t.n_action; return 0; }
        if (!strcmp(name, "view_space")) { ib[0] = t.view.h; ib[1] = t.view.w; ib[2] = group2channel(G); return 0; }
        if (!strcmp(name, "feature_space")) { ib[0] = feature_size(group); return 0; }
        if (!strcmp(name, "attack_base")) { ib[0] = t.attack_base; return 0; }
        if (!strcmp(name, "view2attack")) {
            for (int i = 0; i < t.view.w * t.view.h; i++) ib[i] = -1;
            for (int i = 0; i < t.attack.count; i++)
                ib[(t.attack.dy[i] - t.view.y1) * t.view.w + (t.attack.dx[i] - t.view.x1)] = i;
            return 0;
        }
        if (!strcmp(name, "both_attack")) { ib[0] = 0; return 0; }   // statistics are compiled off (GridWorld.cc:501)
        if (!strcmp(name, "mean_info")) return mean_info(group, (float*)buf);
        return fail("unsupported info name in get_info: %s", name);
    }

    // ---- rendering (GridWorld.cc:1023-1033, RenderGenerator.cc): frames of env 0
    void next_file() { file_ct++; frame_ct = 0; }

    void start_recording() {                      // events are kept once first_render is false
        if (!first_render) return;
        first_render = false;
        gp.record_events = 1;
        if (allocated) MFX_HIP_THROW(hipMemcpy(d_gp, &gp, sizeof(GameParams), hipMemcpyHostToDevice));
    }

    std::vector<int> attack_events() {            // (id, x, y) triples of the last step
        std::vector<int> ev;
        if (first_render || !allocated) return ev;
        MFX_HIP_THROW(hipStreamSynchronize(stream));
        int n = 0;
        MFX_HIP_THROW(hipMemcpy(&n, s.ev, sizeof(int), hipMemcpyDeviceToHost));
        ev.resize((size_t)3 * n);
        if (n) MFX_HIP_THROW(hipMemcpy(ev.data(), s.ev + 1, sizeof(int) * ev.size(), hipMemcpyDeviceToHost));
        return ev;
    }

    static std::string rgba(int r, int g, int b, float alpha) {
        std::stringstream ss;
        ss << "\"rgba(" << r << "," << g << "," << b << "," << alpha << ")\"";
        return ss.str();
    }

    template <class T> static void json(std::ofstream& os, const char* key, T value, bool last = false) {
        os << "\"" << key << "\": " << value;
        os << (last ? "" : ",") << std::endl;
    }

    void gen_config() {                           // RenderGenerator.cc:58-111
        static const int colors[4][3] = {{192, 64, 64}, {64, 64, 192}, {64, 192, 64}, {64, 64, 64}};
        std::ofstream f(render_dir + "/" + "config.json");
        f << "{" << std::endl;
        json(f, "width", W);
        json(f, "height", H);
        json(f, "static-file", "\"static.map\"");
        json(f, "obstacle-style", rgba(127, 127, 127, 1));
        json(f, "dynamic-file-directory", "\".\"");
        json(f, "attack-style", rgba(63, 63, 63, 0.8f));
        json(f, "minimap-width", 300);
        json(f, "minimap-height", 250);
        f << "\"group\" : [" << std::endl;
        const int G = n_groups();
        for (int i = 0; i < G; i++) {
            const AgentTypeSpec& t = gtype(i);
            const int* c = colors[i];
            f << "{" << std::endl;
            json(f, "height", t.length);
            json(f, "width", t.width);
            json(f, "style", rgba(c[0], c[1], c[2], 1));
            json(f, "anchor", "[0, 0]");
            json(f, "max-speed", (int)t.speed);
            json(f, "speed-style", rgba(c[0], c[1], c[2], 0.01f));
            json(f, "vision-radius", t.view_radius);
            json(f, "vision-angle", t.view_angle);
            json(f, "vision-style", rgba(c[0], c[1], c[2], 0.2f));
            json(f, "attack-radius", t.attack_radius);
            json(f, "attack-angle", t.attack_angle);
            json(f, "attack-style", rgba(c[0], c[1], c[2], 0.1f));
            json(f, "broadcast-radius", 1, true);
            f << (i == G - 1 ? "}" : "},") << std::endl;
        }
        f << "]" << std::endl;
        f << "}" << std::endl;
    }

    int render() {                                // GridWorld::render + RenderGenerator::render_a_frame
        if (render_dir.empty()) return 0;
        MFX_CHECK(flush_deferred());
        if (render_dir == "___debug___") return 0;   // the reference prints the map to stdout
        try {
            if (first_render) { start_recording(); gen_config(); }
            const int G = n_groups();
            std::ofstream fout(render_dir + "/" + "video_" + std::to_string(file_ct) + ".txt",
                               frame_ct == 0 ? std::ios::out : std::ios::app);
            if (frame_ct == 0) {
                std::vector<int> walls(2 * (size_t)W * H + 2);
                get_info_global(-1, "walls_info", walls.data());
                fout << "W" << " " << walls[0] << std::endl;
                for (int i = 1; i <= walls[0]; i++) fout << walls[2 * i] << " " << walls[2 * i + 1] << std::endl;
            }
            std::vector<int> ev = attack_events();
            // can_absorb groups: only their absorbed agents are drawn (RenderGenerator.cc:129-160)
            std::vector<std::vector<int>> absorbed((size_t)G);
            int num_agents = 0;
            for (int i = 0; i < G && allocated; i++) {
                const int n = num_env0(i);
                num_agents += n;
                if (!gtype(i).can_absorb || !n) continue;
                absorbed[i].resize(n);
                MFX_CHECK(host_get(i, kGetAbsorbed, absorbed[i].data(), 4));
                for (int j = 0; j < n; j++) num_agents -= absorbed[i][j] ? 0 : 1;
            }
            fout << "F" << " " << num_agents << " " << (int)(ev.size() / 3) << " " << 0 << std::endl;
            for (int i = 0; i < G && allocated; i++) {
                const int n = num_env0(i);
                if (!n) continue;
                std::vector<int> ids(n), pos(2 * (size_t)n), dir(n);
                std::vector<float> hp(n);
                MFX_CHECK(host_get(i, kGetId, ids.data(), 4));
                MFX_CHECK(host_get(i, kGetPos, pos.data(), 8));
                MFX_CHECK(host_get(i, kGetHp, hp.data(), 4));
                MFX_CHECK(host_get(i, kGetDir, dir.data(), 4));
                const float max_hp = gtype(i).hp;
                static const int dir2angle[] = {0, 90, 180, 270};   // RenderGenerator.cc:148
                for (int j = 0; j < n; j++) {
                    if (!absorbed[i].empty() && !absorbed[i][j]) continue;
                    int h = std::max(0, int(100 * hp[j] / max_hp));
                    h = std::min(h, 100);
                    fout << ids[j] << " " << h << " " << dir2angle[dir[j] & 3] << " " << pos[2 * j] << " "
                         << pos[2 * j + 1] << " " << i << std::endl;
                }
            }
            for (size_t k = 0; k < ev.size(); k += 3)
                fout << 0 << " " << ev[k] << " " << ev[k + 1] << " " << ev[k + 2] << std::endl;
            if (frame_ct++ > frame_per_file) { frame_ct = 0; file_ct++; }
        } catch (const HipFailure& f) {
            return fail("%s", f.what());
        }
        return 0;
    }

    // ---- get_info extras (GridWorld.cc:811-954), env 0, from the device state
    std::vector<int> group_pos(int g) {              // x, y per agent in group order (dead included)
        const int n = num_env0(g);
        std::vector<int> pos((size_t)2 * std::max(n, 1));
        if (n > 0 && host_get(g, kGetPos, pos.data(), 8) != 0) throw HipFailure("get pos");
        pos.resize((size_t)2 * n);
        return pos;
    }

    int mean_info(int group, float* out) {           // GridWorld.cc:832-853
        MFX_CHECK(flush_deferred());
        const int n = num_env0(group), na = gtype(group).n_action;
        if (n == 0) return fail("mean_info of an empty group");          // the reference asserts
        std::vector<int> pos = group_pos(group), act((size_t)n);
        MFX_CHECK(host_get(group, kGetLastAct, act.data(), 4));
        float sum_x = 0, sum_y = 0;
        std::vector<int> counter((size_t)na, 0);
        for (int i = 0; i < n; i++) {
            sum_x += (float)pos[2 * i];
            sum_y += (float)pos[2 * i + 1];
            if (act[i] >= 0 && act[i] < na) counter[act[i]]++;   // before the first set_action the
        }                                                         // reference indexes out of range
        out[0] = sum_x / (float)n;
        out[1] = sum_y / (float)n;
        for (int k = 0; k < na; k++) out[2 + k] = (float)(1.0 * counter[k] / n);
        return 0;
    }

    // Keys the python wrapper asks with group -1 (gridworld.py:526-636).
    int get_info_global(int group, const char* name, void* buf) {
        MFX_CHECK(sync_cells());
        int* ib = (int*)buf;
        float* fb = (float*)buf;
        const int G = n_groups();
        if (!strcmp(name, "global_minimap")) {       // GridWorld.cc:807-830
            const int vh = (int)lround(fb[0]), vw = (int)lround(fb[1]);
            if (vh <= 0 || vw <= 0) return fail("global_minimap: bad size %d x %d", vh, vw);
            memset(fb, 0, sizeof(float) * vh * vw * G);
            const int sh = (H + vh - 1) / vh, sw = (W + vw - 1) / vw;
            for (int i = 0; i < G; i++) {
                // the reference computes (i - group + n_group) % n_group in size_t; group -1 -> (i+1) % n
                const size_t ch = ((size_t)i - (size_t)(long)group + (size_t)G) % (size_t)G;
                std::vector<int> pos = allocated ? group_pos(i) : std::vector<int>();
                const size_t n = pos.size() / 2;
                for (size_t j = 0; j < n; j++) fb[((size_t)(pos[2 * j + 1] / sh) * vw + pos[2 * j] / sw) * G + ch] += 1.0f;
                for (int y = 0; y < vh; y++)
                    for (int x = 0; x < vw; x++) fb[((size_t)y * vw + x) * G + ch] /= (float)n;
            }
            return 0;
        }
        if (!strcmp(name, "walls_info")) {           // GridWorld.cc:854-863, Map.cc:621-627 (scan order)
            std::vector<uint16_t> cells((size_t)W * H);
            if (allocated) MFX_HIP(hipMemcpy(cells.data(), s.cells, cells.size() * 2, hipMemcpyDeviceToHost));
            int n = 0;
            for (int c = 0; c < W * H; c++)
                if (allocated && cells[c] == kCellWall) { ++n; ib[2 * n] = c % W; ib[2 * n + 1] = c / W; }
            ib[0] = n;
            return 0;
        }
        if (!strcmp(name, "render_window_info")) {   // GridWorld.cc:864-896
            const int x1 = ib[0], y1 = ib[1], x2 = ib[2], y2 = ib[3];
            int ct = 1;
            for (int i = 0; i < G; i++) {
                std::vector<int> pos = allocated ? group_pos(i) : std::vector<int>();
                std::vector<int> ids(pos.size() / 2), absorbed;
                if (!ids.empty()) MFX_CHECK(host_get(i, kGetId, ids.data(), 4));
                if (!ids.empty() && gtype(i).can_absorb) {          // GridWorld.cc:905-906
                    absorbed.resize(ids.size());
                    MFX_CHECK(host_get(i, kGetAbsorbed, absorbed.data(), 4));
                }
                for (size_t j = 0; j < ids.size(); j++) {
                    const int x = pos[2 * j], y = pos[2 * j + 1];
                    if (x < x1 || x > x2 || y < y1 || y > y2) continue;
                    if (!absorbed.empty() && !absorbed[j]) continue;
                    ib[4 * ct] = ids[j]; ib[4 * ct + 1] = x; ib[4 * ct + 2] = y; ib[4 * ct + 3] = i;
                    ct++;
                }
            }
            ib[0] = ct - 1;
            ib[1] = (int)(attack_events().size() / 3);
            start_recording();                        // GridWorld.cc:882
            return 0;
        }
        if (!strcmp(name, "attack_event")) {         // GridWorld.cc:919-926
            std::vector<int> ev = attack_events();
            std::copy(ev.begin(), ev.end(), ib);
            return 0;
        }
        if (!strcmp(name, "groups_info")) {          // GridWorld.cc:934-949
            static const int colors[4][3] = {{192, 64, 64}, {64, 64, 192}, {64, 192, 64}, {64, 64, 64}};
            for (int i = 0; i < G; i++) {
                ib[5 * i] = 1; ib[5 * i + 1] = 1;     // 1 x 1 bodies (width, length)
                for (int k = 0; k < 3; k++) ib[5 * i + 2 + k] = colors[i][k];
            }
            return 0;
        }
        return get_info(group, name, buf);
    }
};

}  // namespace mfx

using mfx::BattleEngine;

// ============================================================================ C ABI
#define MFX_ENV(h) static_cast<BattleEngine*>(h)
#define MFX_GUARD(expr)                                                          \
    try {                                                                        \
        return (expr);                                                           \
    } catch (const std::exception& ex) {                                         \
        return mfx::fail("%s", ex.what());                                       \
    }

extern "C" {

// ---- reference runtime_api.h:118-181 ------------------------------------------------
MFX_API int env_new_game(void** game, const char* name) {
    if (strcmp(name, "GridWorld") != 0) return mfx::fail("invalid name of game: %s", name);
    MFX_GUARD((*game = new BattleEngine(), 0));
}
MFX_API int env_delete_game(void* game) { delete MFX_ENV(game); return 0; }
MFX_API int env_config_game(void* game, const char* name, void* value) { MFX_GUARD(MFX_ENV(game)->set_config(name, value)); }
MFX_API int env_reset(void* game) { MFX_GUARD(MFX_ENV(game)->reset()); }
MFX_API int env_get_observation(void* game, int group, float** buffer) { MFX_GUARD(MFX_ENV(game)->host_observe(group, buffer)); }
// get_observation without the copy (the drop-in fast step): pointers to env 0's observation of the
// group in engine-owned pinned memory (n rows of blocks of `rows`), valid until the step after next or
// the engine's deletion.  Returns 1 when the observation is not held that way (use env_get_observation).
MFX_API int mfx_env_observation_view(void* game, int group, float** view, float** feature, int* n, int* rows) {
    MFX_GUARD(MFX_ENV(game)->observation_view(group, view, feature, n, rows));
}
MFX_API int env_set_action(void* game, int group, const int* actions) { MFX_GUARD(MFX_ENV(game)->host_set_action(group, actions)); }
MFX_API int env_step(void* game, int* done) { MFX_GUARD(MFX_ENV(game)->host_step(done)); }
MFX_API int env_get_reward(void* game, int group, float* buffer) {
    MFX_GUARD(MFX_ENV(game)->host_get(group, mfx::kGetReward, buffer, 4));
}
MFX_API int env_get_info(void* game, int group, const char* name, void* buffer) {
    MFX_GUARD(MFX_ENV(game)->get_info_global(group, name, buffer));
}
// The drop-in wrapper's getters in one FFI call each where the reference's wrapper makes two
// (gridworld.py get_agent_id / get_reward / get_alive / get_pos: env_get_info("num"), then env_get_info(name) or
// env_get_reward): returns the group's size n and, when n <= cap, copies its n rows of field `what` (0 id int32,
// 1 reward float32, 2 alive uint8, 3 pos int32 pairs; -1: the size only) into out.  -1 on error.
MFX_API int mfx_env_get_rows(void* game, int group, int what, void* out, int cap) {
    MFX_GUARD(MFX_ENV(game)->get_rows(group, what, out, cap));
}
MFX_API int env_render(void* game) { MFX_GUARD(MFX_ENV(game)->render()); }
MFX_API int env_render_next_file(void* game) { MFX_GUARD((MFX_ENV(game)->next_file(), 0)); }

MFX_API int gridworld_register_agent_type(void* game, const char* name, int n, const char** keys, float* values) {
    MFX_GUARD(MFX_ENV(game)->register_type(name, n, keys, values));
}
MFX_API int gridworld_new_group(void* game, const char* agent_type_name, int* group) {
    MFX_GUARD(MFX_ENV(game)->new_group(agent_type_name, group));
}
MFX_API int gridworld_add_agents(void* game, int group, int n, const char* method, const int* pos_x, const int* pos_y,
                                 const int* dir) {
    MFX_GUARD(MFX_ENV(game)->add_agents(group, n, method, pos_x, pos_y, dir));
}
MFX_API int gridworld_clear_dead(void* game) { MFX_GUARD(MFX_ENV(game)->host_clear_dead()); }
MFX_API int gridworld_set_goal(void* game, int group, const char* method, const int* linear_buffer) {
    (void)linear_buffer;
    MFX_GUARD(MFX_ENV(game)->set_goal(group, method));
}
MFX_API int gridworld_define_agent_symbol(void* game, int no, int group, int index) {
    BattleEngine* e = MFX_ENV(game);
    if (no < 0) return mfx::fail("bad symbol number");
    if ((size_t)no >= e->syms.size()) e->syms.resize(no + 1);
    e->syms[no] = {group, index};
    return 0;
}
MFX_API int gridworld_define_event_node(void* game, int no, int op, int* inputs, int n_inputs) {
    BattleEngine* e = MFX_ENV(game);
    if (no < 0) return mfx::fail("bad event node number");
    if ((size_t)no >= e->nodes.size()) e->nodes.resize(no + 1);
    e->nodes[no].op = op;
    e->nodes[no].raw.assign(inputs, inputs + n_inputs);
    return 0;
}
// The reference python passes only 6 of these 7 arguments (gridworld.py:719-722);
// auto_value is never read (it only matters for OP_ALIGN, RewardEngine.cc:252).
MFX_API int gridworld_add_reward_rule(void* game, int on, int* receiver, float* value, int n_receiver, bool is_terminal,
                                      bool auto_value) {
    (void)auto_value;
    BattleEngine* e = MFX_ENV(game);
    BattleEngine::Rule r;
    r.on = on;
    r.recv.assign(receiver, receiver + n_receiver);
    r.val.assign(value, value + n_receiver);
    r.terminal = is_terminal;
    e->rules.push_back(std::move(r));
    return 0;
}

// ---- batched device API (include/magent_amd.h) ---------------------------------------
MFX_API int mfx_battle_set_num_envs(void* game, int n_envs) {
    BattleEngine* e = MFX_ENV(game);
    if (e->allocated) return mfx::fail("set_num_envs must precede the first reset");
    if (n_envs < 1) return mfx::fail("n_envs must be >= 1");
    e->E = n_envs;
    return 0;
}
MFX_API int mfx_battle_set_stream(void* game, void* stream) {
    BattleEngine* e = MFX_ENV(game);
    MFX_CHECK(e->quiesce());
    if (e->own_stream && e->stream) { (void)hipStreamSynchronize(e->stream); (void)hipStreamDestroy(e->stream); }
    e->stream = (hipStream_t)stream;
    e->own_stream = false;
    e->stream_set = true;
    return 0;
}
MFX_API int mfx_battle_observe(void* game, int group, float* d_view, float* d_feature, int rowcap) {
    MFX_GUARD(MFX_ENV(game)->observe(group, d_view, d_feature, rowcap));
}
MFX_API int mfx_battle_set_action(void* game, int group, const int* d_actions, int rowcap) {
    MFX_GUARD(MFX_ENV(game)->set_action(group, d_actions, rowcap));
}
MFX_API int mfx_battle_step(void* game, int* d_done) { MFX_GUARD(MFX_ENV(game)->step(d_done)); }
MFX_API int mfx_battle_get(void* game, int group, int what, void* d_out, int rowcap) {
    MFX_GUARD(MFX_ENV(game)->get(group, what, d_out, rowcap));
}
MFX_API int mfx_battle_clear_dead(void* game) { MFX_GUARD(MFX_ENV(game)->clear_dead()); }
MFX_API int mfx_battle_sync(void* game) {
    BattleEngine* e = MFX_ENV(game);
    if (!e->allocated) return 0;
    MFX_CHECK(e->quiesce());
    MFX_HIP(hipStreamSynchronize(e->stream));
    return e->check_err();
}
MFX_API int mfx_battle_rollout_init(void* game, const int* tmpl_n, const int* const* xs, const int* const* ys,
                                    int max_steps, float eps, unsigned seed, int stagger) {
    MFX_GUARD(MFX_ENV(game)->rollout_init(tmpl_n, xs, ys, max_steps, eps, seed, stagger));
}
MFX_API int mfx_battle_rollout_step(void* game, int n_steps) { MFX_GUARD(MFX_ENV(game)->rollout_step(n_steps)); }
MFX_API int mfx_battle_rollout_buffer(void* game, const char* name, int group, void** ptr, size_t* bytes) {
    MFX_GUARD(MFX_ENV(game)->rollout_buffer(name, group, ptr, bytes));
}
// Copy a rollout buffer (see rollout_buffer names) to dst (host or device pointer),
// asynchronously on the engine stream; `bytes` may be smaller than the buffer.
MFX_API int mfx_battle_rollout_copy(void* game, const char* name, int group, void* dst, size_t bytes) {
    BattleEngine* e = MFX_ENV(game);
    void* src = nullptr;
    size_t n = 0;
    MFX_CHECK(e->rollout_buffer(name, group, &src, &n));
    if (bytes > n) return mfx::fail("rollout_copy: %zu bytes requested, buffer has %zu", bytes, n);
    MFX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, e->stream));
    return 0;
}
// The same for bytes [offset, offset + bytes) of the buffer (e.g. one env's rows).
MFX_API int mfx_battle_rollout_copy_at(void* game, const char* name, int group, size_t offset, void* dst, size_t bytes) {
    BattleEngine* e = MFX_ENV(game);
    void* src = nullptr;
    size_t n = 0;
    MFX_CHECK(e->rollout_buffer(name, group, &src, &n));
    if (offset > n || bytes > n - offset)
        return mfx::fail("rollout_copy_at: bytes [%zu, %zu) outside the buffer (%zu)", offset, offset + bytes, n);
    MFX_HIP(hipMemcpyAsync(dst, static_cast<const char*>(src) + offset, bytes, hipMemcpyDefault, e->stream));
    return 0;
}
// Diagnostic build only: route k_rollout phase stamps ([E][16] u64 s_memtime) to d_buf.
MFX_API int mfx_battle_set_stamp_buffer(void* d_buf) {
    MFX_HIP(mfx::set_stamp_buffer((unsigned long long*)d_buf));
    return 0;
}
// Launch geometry of the fused rollout: persistent grid (workgroups) and LDS bytes per workgroup.
MFX_API int mfx_battle_rollout_info(void* game, int* grid, int* lds_bytes) {
    MFX_GUARD(MFX_ENV(game)->rollout_info(grid, lds_bytes));
}

// Synchronise; -1 and the message if a device error was raised or (k_rollout_bigq) the in-launch work
// queue reported an error.
MFX_API int mfx_battle_rollout_check(void* game) {
    MFX_GUARD(MFX_ENV(game)->rollout_check());
}
// A learned policy's launches: mode 2 observes every env, mode 1 acts with the action buffer, steps, observes.
MFX_API int mfx_battle_rollout_policy_step(void* game, int mode) {
    MFX_GUARD(MFX_ENV(game)->rollout_policy_step(mode));
}
// The kernels rollout_step runs: 0 k_rollout, 1 k_rollout_obs + k_rollout (pipeline), 2 k_observe_items +
// k_rollout_big (large-env pipeline), 3 k_rollout_bigq.
MFX_API int mfx_battle_rollout_path(void* game, int* path) {
    const int p = MFX_ENV(game)->rollout_path();
    if (p < 0) return mfx::fail("rollout_path before rollout_init");
    *path = p;
    return 0;
}

// Lanes over which the rollout sums a group's rewards of an env with n_agents agents (the summation order
// the episode returns follow; the oracle replay restates it).
MFX_API int mfx_battle_rollout_sum_lanes(void* game, int n_agents, int* lanes) {
    const int l = MFX_ENV(game)->rollout_sum_lanes(n_agents);
    if (l < 0) return mfx::fail("rollout_sum_lanes before rollout_init");
    *lanes = l;
    return 0;
}

// Steps per k_rollout launch (1..64; up to 1024 on the pipelined few-env path, the others run 64 at most): every
// env runs that many consecutive steps while its image stays
// in LDS; the large-env queue kernel k_rollout_bigq runs that many steps of every env per launch (its
// item lists hold one filing per env and step of a launch: lcap in rollout_plan, hence <= 64).
// rollout_step(n) results are identical for any value (the last step's buffers, the same state); only
// the launch count changes.  Ignored by the two pipelines (one step per launch).  0: chosen per path and batch
// (BattleEnv::sub_steps); mfx_battle_rollout_get_substeps reports the value in force.
MFX_API int mfx_battle_rollout_set_substeps(void* game, int n_sub) {
    if (n_sub < 0 || n_sub > 1024) return mfx::fail("rollout_set_substeps: %d not in 0..1024", n_sub);
    MFX_ENV(game)->ro_sub = n_sub;
    return 0;
}

MFX_API int mfx_battle_rollout_get_substeps(void* game, int* n_sub) {
    if (!MFX_ENV(game)->rollout_ready) return mfx::fail("rollout_get_substeps before rollout_init");
    *n_sub = MFX_ENV(game)->sub_steps();
    return 0;
}

MFX_API int mfx_battle_rollout_rowcap(void* game, int* rowcap) {
    *rowcap = MFX_ENV(game)->ra.rowcap;
    return 0;
}
MFX_API int mfx_battle_rollout_mean_stride(void* game, int* stride) {
    *stride = MFX_ENV(game)->ra.mean_stride;
    return 0;
}
// The inputs of group g's observation view that can be non-zero (Map::extract_view, Map.cc:130-218): every channel
// of a cell inside the view range, only the minimap channels (group2channel(k) + 2, GridWorld.cc:396-409) of a cell
// outside it.  mask[n], n = view_h * view_w * n_ch (the view's NHWC order): 1 = may be non-zero, 0 = always 0.
MFX_API int mfx_battle_view_support(void* game, int group, uint8_t* mask, int n) {
    BattleEngine* e = MFX_ENV(game);
    if (group < 0 || group >= e->n_groups()) return mfx::fail("view_support: bad group");
    if (!e->allocated) {                     // (once allocated, gp is the parameter set the device runs on)
        try {
            MFX_CHECK(e->build_params());
        } catch (const std::exception& ex) {
            return mfx::fail("%s", ex.what());
        }
    }
    const mfx::TypeParams& T = e->gp.type[group];
    const int NC = e->gp.n_ch, cells = T.view_w * T.view_h;
    if (n != cells * NC) return mfx::fail("view_support: %d entries, the view has %d", n, cells * NC);
    for (int c = 0; c < cells; c++)
        for (int ch = 0; ch < NC; ch++) {
            bool mm = false;
            for (int k = 0; e->minimap && k < e->n_groups(); k++) mm = mm || ch == e->group2channel(k) + 2;
            mask[c * NC + ch] = (uint8_t)(T.view_mask[c] || mm);
        }
    return 0;
}
MFX_API int mfx_battle_group_capacity(void* game, int group, int* cap) {
    BattleEngine* e = MFX_ENV(game);
    if (group < 0 || group >= e->n_groups()) return mfx::fail("bad group");
    *cap = e->allocated ? e->group_ub[group] : 0;
    return 0;
}

}  // extern "C"
