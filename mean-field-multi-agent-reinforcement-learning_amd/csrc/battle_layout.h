// battle_layout.h -- HBM layout of a batch of Battle gridworlds (shared host/device).
//
// One engine holds E independent environments with identical configuration (map size,
// agent types, reward rules).  All per-env state is struct-of-arrays in HBM with a fixed
// per-env stride, so a workgroup that owns env e touches only its own slabs:
//
//   cells     u16 [E][H*W]    0xFFFF empty, 0xFFFE wall, else the occupying agent's slot
//   agents (indexed by slot, slots are dense 0..id_counter-1).  A slot is the agent's id
//   (GridWorld.cc:184) until the large-env rollout renumbers the slots to the list order at a
//   clear_dead (clear_dead_renumber, battle/rollout_big.inc); the id itself is always rid[slot]
//     rid       u16 [E][cap]   the reference's agent id of the slot (features, get_agent_id, keys)
//     xy        u32 [E][cap]   x | y << 16
//     hp        f32 [E][cap]
//     next_r    f32 [E][cap]   Agent::next_reward  (GridWorld.h:248)
//     last_r    f32 [E][cap]   Agent::last_reward
//     last_act  u8  [E][cap]   Agent::last_action  (initially n_action, GridWorld.h:145) in bits 0-6
//                              | bit7 Agent::absorbed (GridWorld.h:196-197; can_absorb types only)
//     op_obj    i32 [E][cap]   id of Agent::op_obj or -1
//     meta      u8  [E][cap]   bit0 dead | bits1-2 last_op | bit3 involved (reward DSL, transient)
//                              | bits4-5 group | bits6-7 direction ^ 3 (0 = NORTH, turn_mode)
//   groups
//     grp_ids   u16 [E][G][cap] the ordered agent vector of each group (Group::agents)
//     grp_n, grp_dead i32 [E][G];  grp_reward f32 [E][G]
//   id_counter i32 [E] slots in use, rid_off i32 [E] the reference's id_counter minus id_counter
//   (0 unless renumbered), rng u32 [E] (minstd_rand0 state, GridWorld.h:106)
//   pending actions since the last step (GridWorld::set_action, GridWorld.cc:430-496)
//     atk u32 [E][acap] = id << 8 | attack index      n_atk i32 [E]
//     mov u32 [E][acap] = id << 16 | move index << 8 | bucket (0xFF = boundary buffer)
//                                                     n_mov i32 [E]
#pragma once
#include <stdint.h>

namespace mfx {

constexpr int kMaxGroups = 4;
constexpr int kMaxViewCells = 32 * 32;
constexpr int kMaxRangeCount = 64;
constexpr int kMaxRules = 8;
constexpr int kMaxRecv = 8;
constexpr int kMaxSyms = 16;        // reward DSL: agent symbols, event nodes (RewardEngine.h)
constexpr int kMaxNodes = 32;
constexpr uint16_t kCellEmpty = 0xFFFF;
constexpr uint16_t kCellWall = 0xFFFE;
constexpr uint16_t kCellFood = 0xFFFD;   // food_mode: a food slot (amount in State::food); ids stay below
constexpr uint32_t kBucketBoundary = 0xFF;
constexpr int kMaxSplit = 8;              // large-env rollout: most sub-batches (streams)

// last_op encoding in meta bits 1-2
enum : uint32_t { kOpNull = 0, kOpAttack = 1, kOpKill = 2, kOpCollide = 3 };
// reference EventOp numbering (grid_def.h:17-23), used by the reward-rule ABI
enum : int { kEvAnd = 0, kEvOr = 1, kEvNot = 2, kEvKill = 3, kEvAt = 4, kEvIn = 5, kEvCollide = 6, kEvAttack = 7,
             kEvDie = 8, kEvInALine = 9, kEvAlign = 10 };

struct TypeParams {                 // AgentType (AgentType.h:17-52), the fields the path reads
    float hp, damage, step_recover, kill_supply;
    float step_reward, kill_reward, dead_penalty, attack_penalty;
    int attack_in_group, can_absorb;           // can_absorb: Map.cc:352-356, GridWorld.cc:362/:638/:905
    int n_action, turn_base, attack_base;
    int n_move, n_attack;
    int view_w, view_h, view_x1, view_y1;      // view window relative to the agent (NORTH)
    int att_x_off, att_y_off;
    int body_w, body_h;                        // width x length cells from pos (NORTH, Map.cc:75-97)
    int view_off_x, view_off_y, view_lt_x, view_lt_y;   // turn_mode: eye offset and window corner (rela)
    float eat_ability, food_supply;            // food_mode (Map.cc:289-303, AgentType.h)
    int8_t move_dx[kMaxRangeCount], move_dy[kMaxRangeCount];
    int8_t att_dx[kMaxRangeCount], att_dy[kMaxRangeCount];
    uint8_t view_mask[kMaxViewCells];          // Range::is_in, row-major [view_h][view_w]
    uint32_t view_bits[kMaxViewCells / 32];    // the same mask, one bit per cell
};

struct RuleParams {                 // RewardRule on one binary event between two 'any' symbols
    int op;                         // kOpAttack / kOpKill / kOpCollide
    int subj_group, obj_group;
    int n_recv;
    int recv_is_obj[kMaxRecv];
    float val[kMaxRecv];
    int terminal;
};

// The general reward DSL (RewardEngine.cc:105-443), compiled on the host into the reference's
// own inference plan (init_reward_description) and interpreted by one lane per env (k_step<true>).
struct DslSym { int group, index; };                 // index -1 any, -2 all, >= 0 fixed
struct DslNode {                                     // op (kEv*); a, b: node or symbol numbers;
    int op, a, b, i0, i1, i2, i3;                    // i0..i3: AT (x, y) / IN (x1, y1, x2, y2)
};
struct DslRule {
    int n_in;                                        // DFS levels (RewardRule::input_symbols)
    int8_t in_sym[kMaxSyms], infer[kMaxSyms];        // infer: symbol bound from op_obj, or -1
    int n_post;                                      // the `on` subtree, children before parents
    int8_t post[kMaxNodes];
    int n_recv, terminal;
    int8_t recv[kMaxRecv];
    float val[kMaxRecv];
};
struct DslProgram {
    int n_rules;
    DslSym sym[kMaxSyms];
    DslNode node[kMaxNodes];
    DslRule rule[kMaxRules];
};

struct GameParams {
    int W, H, n_groups, minimap, emb, n_ch;
    int large_map, n_sep, band_w;
    int n_rules;
    int record_events;              // 1 once rendering started: k_step records env 0's attack events
    int par_step;                   // 1: attack / move resolution may run in parallel (every
                                    //    kill_supply == 0, so a kill never changes the killer's hp)
    int dsl;                        // 1: reward rules outside the RuleParams form run through `prog`
    int turn_mode, food_mode;       // GridWorld.cc:138-147 (serial / generic paths only)
    int feat_size[kMaxGroups];
    TypeParams type[kMaxGroups];    // per group (Group::type)
    RuleParams rules[kMaxRules];
    DslProgram prog;
};

struct State {                      // device pointers; every array is [E][stride]
    int E, cap, acap, cells_n;      // cells_n = H*W
    uint16_t* cells;
    uint32_t* xy;
    float* hp;
    float* next_r;
    float* last_r;
    uint8_t* last_act;
    int32_t* op_obj;
    uint8_t* meta;
    uint16_t* grp_ids;              // [E][G][cap]
    int32_t* grp_n;                 // [E][G]
    int32_t* grp_dead;              // [E][G]
    float* grp_reward;              // [E][G]
    int32_t* id_counter;            // [E] slots in use
    uint16_t* rid;                  // [E][cap] reference id of each slot
    int32_t* rid_off;               // [E] next id add_agents hands out (GridWorld::id_counter) - id_counter
    uint32_t* rng;                  // [E]
    uint32_t* atk;                  // [E][acap]
    int32_t* n_atk;                 // [E]
    uint32_t* mov;                  // [E][acap]
    int32_t* n_mov;                 // [E]
    int32_t* done;                  // [E]
    float* food;                    // [E][H*W] food amount where cells == kCellFood (food_mode only)
    int32_t* idx_mark;              // [E] id_counter at the last clear_dead: Agent::index is the list
                                    //     position for ids below it, else 0 (GridWorld.h:139, :718)
    int32_t* err;                   // [1] sticky device-side error code
    int32_t* ev;                    // [1 + 3 * acap] env 0's attack events of the last step (render):
                                    //   count, then (attacker id, target x, target y) in shuffle order
    int serial_step;                // this step runs the serial forms: a group's set_action was called
                                    //   more than once since the last step, so an agent may appear twice
                                    //   in the action buffers (the parallel forms take one entry per agent)
};

// Arguments of the drop-in single-env step (k_dropin_step, battle/dropin.inc).
// The resident drop-in server's mailbox (k_dropin_step with DropinArgs::mb set), in coherent host
// memory.  The host writes a request's fields, then `req` (release); the kernel answers in `done`,
// on its own 128-B line so that the two sides do not write one line.
enum : int32_t { kDropinStop = 0, kDropinStep = 1 };
// the request line and the tagged actions: one 16-B load per lane of wave 0, two passes (512 words)
constexpr int kMailWords = 512, kMailActs = kMailWords - 16;
struct DropinMailbox {
    uint32_t req;                        // word 0: sequence number of the latest request
    int32_t cmd;                         // 1: kDropinStep / kDropinStop
    int32_t pending_clear;               // 2: a clear_dead is deferred from the previous step
    int32_t n_acts[kMaxGroups];          // 3-6: deferred set_action lengths, -1: no call for the group
    int32_t tagged;                      // 7: the actions are in acts[], each word (req & 0xFFFF) << 16 | action
    int32_t act_stride;                  // 8: words per group in acts[]
    int32_t pad0[7];
    uint32_t acts[kMailActs];            // words 16..511: group g's actions from g * act_stride
    uint32_t done[4];                    // [0] records written, [1] observation written, [2] unused,
                                         // [3] the kernel has left (the last request it saw)
    int32_t pad1[28];
};

struct DropinArgs {
    const int32_t* acts[kMaxGroups];     // deferred set_action buffers (host-mapped), null: none
    int n_acts[kMaxGroups];              //   and their lengths (group sizes after the deferred clear)
    int pending_clear;                   // a clear_dead is deferred from the previous step
    int rows;                            // rows per group of the records and observation blocks
    uint8_t* rec_step;                   // record after the step          (host-mapped)
    float* view[kMaxGroups];             // [rows][VH*VW*NC] per group     (host-mapped), set 0
    float* feat[kMaxGroups];             // [rows][F]
    size_t obs_alt;                      // floats from set 0 to set 1: request seq writes set seq & 1
    uint32_t* flag;                      // [2] host-mapped coherent words: seq once the record is
    uint32_t seq;                        //   written, seq once the observation is
    // resident server (mb != null): the launch installs env 0 once and then answers every request
    // posted in mb (acts[g] fixed, lengths and the clear flag from the mailbox, completion words
    // mb->done) until a kDropinStop request or `idle` wall-clock ticks without one.  seq = the last
    // request already answered; flag is unused.
    DropinMailbox* mb;
    unsigned long long idle;
    int mail_passes;                     // 16-B loads per lane and poll: 1 or 2 (header + tagged actions,
                                         // 256 / 512 words), 0: the header only (actions read after)
    int variant;                         // diagnostics (MFX_DROPIN_VARIANT): bit 1 answers requests
                                         // without doing the step (timing only),
                                         // bit 3 writes the record in system-scope stores and publishes
                                         // it without the system fence
};

// Arguments of the fused rollout step (k_rollout): one launch = one step of the
// reference training loop (senario_battle.play, :96-171) for every env, with the
// synthetic rush policy of SURVEY.md 8(d) on device.  All pointers are [E][...] slabs.
struct RolloutArgs {
    float* view[kMaxGroups];        // [E][rowcap][VH*VW*NC]   get_observation views
    float* feat[kMaxGroups];        // [E][rowcap][F]          get_observation features
    int rowcap;                     // rows per env in every per-agent output (>= max group size)
    int32_t* actions;               // [E][G][rowcap]  actions taken this step
    float* rewards;                 // [E][G][rowcap]  get_reward after the step
    double* mean_act;               // [E][G][mean_stride] former_act_prob (senario_battle.py:141); group g
    int mean_stride;                //   fills its first n_action(g) entries; stride = max n_action
    float* ep_return;               // [E][G]  running episode return (sum of rewards)
    int32_t* ep_len;                // [E]     steps into the current episode
    double* stats;                  // [E][4]  finished episodes, sum final return g0, g1, kills
    unsigned long long* agent_steps;// [E]     agents present at get_observation, summed
    const int32_t* tmpl_x;          // [G][tmpl_cap] placement re-applied at each episode start
    const int32_t* tmpl_y;
    int tmpl_n[kMaxGroups];
    int tmpl_cap;
    int max_steps;                  // episode cap (play(max_steps=400))
    uint32_t policy_seed;
    uint32_t step_index;            // global step counter (policy RNG stream)
    float eps;                      // random-action probability of the rush policy
    int32_t* cls_cnt;               // [3][8] envs per weight class: launch L reads [L % 3], appends to
                                    //   [(L + 1) % 3] and zeroes [(L + 2) % 3]  (L = queue phase)
    int32_t* cls_list;              // [2][8][cls_stride] env indices per class, read [L % 2], written
    int cls_stride;                 //   [(L + 1) % 2]
    int32_t* work;                  // [2] env work-queue counters; launch k uses work[k & 1]
    int work_sel;                   //     and zeroes the other one for launch k + 1
    const uint4* reset_image;       // LDS image of the env right after reset + template placement,
                                    // followed by int32 [grp_n[kMaxGroups], id_counter]
    int env_base;                   // index of env 0 of this (sub-)batch in the whole batch (policy keys)
    uint32_t* big_sort;             // large envs: [E][acap] band-ordered move buffer of k_rollout_big
    int renumber;                   // large envs: clear_dead renumbers the slots to the list order, so
                                    //   the per-slot arrays of the live agents stay dense (rid keeps ids);
                                    //   2: without the identity fast path (A/B only)
    int lds_step;                   // few LDS-sized envs on the queue kernel: big_env_step stages the env in
                                    //   LDS for the step and writes it back (BigLayout::img)
    float* obs_mm;                  // large envs (k_rollout_big): [E][G][VH*VW] minimap density and
    uint32_t* obs_info;             //   [E][cap] packed hp/max | group << 31 of the NEXT observation,
                                    //   computed once per env at the end of the step (obs_prep_env)
    uint32_t* obs_items;            //   [2][obs_lists][obs_list_stride] observation work items (env << 12 |
                                    //   group << 10 | chunk) by step parity, filed by obs_file_items into
                                    //   list e % obs_lists (one list per XCD: the items of an env are taken
                                    //   by workgroups of one XCD, whose L2 then holds that env's cells)
    int32_t* obs_cnt;               //   [2][obs_lists][kObsCntPad] per parity and list: items filed, items
                                    //   taken (k_observe_items)
    size_t obs_par_stride;          //   items per parity region of obs_items
    size_t obs_list_stride;         //   items per list
    int obs_lists;                  //   1 or kXcds
    int obs_item_rows;              //   agents per item
    uint32_t* q_items;              // large envs, k_rollout_bigq: [2][kXcds][q_list_cap] tagged work items
    int32_t* q_cnt;                 //   [2][kXcds][kObsCntPad] items filed, items taken
    int32_t* q_left;                //   [E] items of the env's current step not yet observed
    uint32_t* q_si;                 //   [E] the env's next step index
    int32_t* q_done;                //   [kObsCntPad] 0: env-steps done (monotone), 2: stuck-queue error word
    size_t q_list_cap;              //   items per list and parity
    int few_pipe;                   // few LDS-sized envs on the queue kernel, pipelined: one stepper workgroup
    int few_wave_max;               // few_pipe: the stepper's wave team (wave 0 alone) up to this many agents, else the workgroup
                                    //   per env keeps it in LDS for the whole launch and steps it while the
                                    //   item workers observe the state the step started from, out of a
                                    //   per-env snapshot (few_snap, 2 parities) -- k_rollout_bigq<true>
    uint8_t* few_snap;              //   [E][2][few_snap_bytes] (snap_layout)
    size_t few_snap_bytes;
    int32_t* q_step;                //   [kXcds] stepper roles claimed per XCD this launch (zeroed per launch)
    const uint4* wall_image;        // [H*W] u16 cells of that image with the agents removed: every
                                    // install rebuilds the cells from it plus the agents' positions, so
                                    // per-env cells are neither read nor written back (State::cells is
                                    // rebuilt on demand, BattleEngine::sync_cells)
};

// XCDs of the MI355X (workgroup i of a launch runs on XCD i % kXcds) and the int32 pad of one
// item-list counter pair (its own 64-B line)
constexpr int kXcds = 8, kObsCntPad = 16;

// Everything k_rollout reads besides GameParams, resident in HBM (uploaded when it changes); the
// kernel re-reads it per env through scalar loads instead of pinning ~80 SGPRs for the launch.
// s: the state a launch reads; w: where k_rollout writes each env back.  The fused step has
// w == s; the observation/step pipeline (k_rollout_obs beside k_rollout<.., kSplit>) reads one
// copy of the per-env state and writes the other, so that both kernels of a launch see the state
// before the step.
struct RolloutCtx {
    State s;
    RolloutArgs ra;
    State w;
};

// last_act bit 7: the agent was absorbed (Map::do_move's can_absorb collision)
constexpr uint32_t kLastActAbsorbed = 0x80u;
__host__ __device__ inline uint32_t last_action(uint32_t la) { return la & 0x7Fu; }
__host__ __device__ inline bool is_absorbed(uint32_t la) { return (la & kLastActAbsorbed) != 0u; }

// meta helpers
__host__ __device__ inline uint32_t meta_dead(uint32_t m) { return m & 1u; }
__host__ __device__ inline uint32_t meta_op(uint32_t m) { return (m >> 1) & 3u; }
__host__ __device__ inline uint32_t meta_group(uint32_t m) { return (m >> 4) & 3u; }
__host__ __device__ inline uint32_t meta_make(uint32_t dead, uint32_t op, uint32_t g) {
    return dead | (op << 1) | (g << 4);
}
// Direction (grid_def.h:15): EAST 0, SOUTH 1, WEST 2, NORTH 3; stored xor 3 so that every meta
// built without direction bits faces NORTH.
enum : int { kDirEast = 0, kDirSouth = 1, kDirWest = 2, kDirNorth = 3 };
__host__ __device__ inline int meta_dir(uint32_t m) { return (int)(((m >> 6) & 3u) ^ 3u); }
__host__ __device__ inline uint32_t meta_set_dir(uint32_t m, int dir) {
    return (m & 0x3Fu) | ((((uint32_t)dir ^ 3u) & 3u) << 6);
}
__host__ __device__ inline uint32_t meta_keep_dir(uint32_t fresh, uint32_t old) { return fresh | (old & 0xC0u); }

}  // namespace mfx
