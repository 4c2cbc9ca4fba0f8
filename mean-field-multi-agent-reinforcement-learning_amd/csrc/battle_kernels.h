// battle_kernels.h -- host-side launchers of the Battle kernels (battle_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "battle_layout.h"

namespace mfx {

enum GetWhat : int { kGetNum = 0, kGetReward = 1, kGetId = 2, kGetAlive = 3, kGetPos = 4, kGetHp = 5, kGetLastAct = 6, kGetDir = 7, kGetAbsorbed = 8 };

size_t observe_smem_bytes(const GameParams& gp, int g, int cells_in_lds, int cells_n, int cap);
size_t step_smem_bytes(const GameParams& gp, int cells_n, int n_ids, int acap, int cap);

hipError_t launch_reset(const GameParams* d_gp, const State& s, hipStream_t st);
hipError_t launch_rid_fill(const State& s, int from, hipStream_t st);   // rid[e][i] = i for i >= from
hipError_t launch_add_agents(const GameParams* d_gp, const State& s, int group, int n, int method,
                             const int* d_xs, const int* d_ys, const int* d_dirs, int per_env_stride, hipStream_t st);
hipError_t launch_set_goal_random(const GameParams* d_gp, const State& s, int g, hipStream_t st);
hipError_t launch_rebuild_cells(const GameParams* d_gp, const State& s, const void* walls, hipStream_t st);
hipError_t launch_observe(const GameParams& gp, const GameParams* d_gp, const State& s, int g, int max_n,
                          float* d_view, float* d_feat, int rowcap, hipStream_t st);
bool battle_shape(const GameParams& gp);     // the Battle fast-path shape (is_battle_shape)
hipError_t launch_obs_prep(const GameParams* d_gp, const State& s, const RolloutArgs& ra, int par, hipStream_t st);
hipError_t launch_observe_items(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutArgs& ra,
                                int par, int grid, hipStream_t st);
hipError_t observe_items_grid(const GameParams& gp, int rows, int* grid);
hipError_t launch_set_action(const GameParams* d_gp, const State& s, int g, const int* d_actions, int rowcap,
                             hipStream_t st);
hipError_t launch_step(const GameParams& gp, const GameParams* d_gp, const State& s, int max_ids,
                       uint32_t* d_sort_scratch, hipStream_t st);
hipError_t launch_clear_dead(const GameParams* d_gp, const State& s, hipStream_t st);
hipError_t set_stamp_buffer(unsigned long long* d_buf);
size_t rollout_smem_bytes(const GameParams& gp, int cells_n, int cap, int acap, int rows);
hipError_t launch_rollout(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                          int rows, uint32_t step_index, int work_sel, int qphase, int grid, int split,
                          int n_sub, hipStream_t st);
hipError_t launch_rollout_mode(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                               int rows, uint32_t step_index, int work_sel, int qphase, int grid, int mode,
                               hipStream_t st);
size_t rollout_obs_smem_bytes(const GameParams& gp, int cells_n, int cap, int rows);
hipError_t launch_rollout_obs(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                              int rows, int work_sel, int qphase, int grid, hipStream_t st);
hipError_t rollout_obs_grid(const GameParams& gp, const State& s, int rows, int per_cu_want, int* grid);
size_t big_step_smem_bytes(const GameParams& gp, int cap, int acap, bool rollout, bool lds_env = false);
hipError_t launch_rollout_big(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                              uint32_t step_index, bool lds_env, hipStream_t st);
hipError_t rollout_grid(const GameParams& gp, const State& s, int rows, int split, int per_cu_want, int* grid);
// large envs, one queue-driven launch per n_sub steps (k_rollout_bigq)
// lds_env: the few-env path stages each env in LDS for its step (RolloutArgs::lds_step)
size_t bigq_smem_bytes(const GameParams& gp, int cap, int acap, int rows, bool lds_env, bool pipe = false);
hipError_t bigq_grid(const GameParams& gp, int cap, int acap, int rows, bool lds_env, int* grid, bool pipe = false);
hipError_t launch_bigq_seed(const GameParams* d_gp, const State& s, const RolloutArgs& ra, int par, uint32_t tag,
                            uint32_t step_index, hipStream_t st);
// pipe: the pipelined few-env form (RolloutArgs::few_pipe: one stepper workgroup per env, k_rollout_bigq<true>)
hipError_t launch_rollout_bigq(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutCtx* d_ctx,
                               int rows, uint32_t si0, int n_sub, int par, uint32_t tag_cur, uint32_t tag_next,
                               int grid, bool lds_env, hipStream_t st, bool pipe = false);
size_t few_snap_bytes(int cells_n, int cap, int G);
size_t rollout_reset_image_bytes(const GameParams& gp, int cells_n, int cap);
hipError_t launch_reset_image(const GameParams& gp, const GameParams* d_gp, const State& s, const RolloutArgs& ra,
                              uint4* d_image, hipStream_t st);
size_t dropin_smem_bytes(const GameParams& gp, int cells_n, int cap, int acap, int rows);
hipError_t launch_dropin_step(const GameParams& gp, const GameParams* d_gp, const State& s, const DropinArgs& da,
                              hipStream_t st);
hipError_t launch_get_env0(const GameParams* d_gp, const State& s, uint8_t* d_out, int rows, hipStream_t st);
hipError_t launch_get(const GameParams* d_gp, const State& s, int g, int what, void* d_out, int rowcap,
                      hipStream_t st);

}  // namespace mfx
