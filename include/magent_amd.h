/*
 * magent_amd.h -- C ABI of the MI355X-native Battle / Ising mean-field engine (libmagent.so).
 *
 * Part 1 is the reference's own ABI, symbol for symbol: the 18 GridWorld entry points of
 * examples/battle_model/src/runtime_api.h:20-55 (implemented at runtime_api.cc:15-169), so
 * the reference python wrapper examples/battle_model/python/magent/gridworld.py (ctypes, no
 * argtypes) and c_lib.py:13-31 bind this library unchanged.  Those calls act on env 0 and move
 * data through caller-owned host buffers, exactly like the reference.  On one env whose config the
 * fused kernels take, set_action and clear_dead are deferred and env_step is one request to a
 * resident k_dropin_step workgroup (a mailbox in coherent host memory; MFX_DROPIN_RESIDENT=0: one
 * launch per step) that also leaves the getters' record and the next observation in pinned memory;
 * any other call first stops the server and runs the deferred work (MFX_DROPIN_FAST=0: one launch
 * per call).
 *
 * Part 2 is this library's batched device API: E envs per engine, every buffer in HBM.
 * Part 3 covers the Ising lattice / tabular MF-Q (the reference's examples/ising_model and
 * main_MFQ_Ising.py are pure python; there is no reference ABI to mirror).
 * Part 4 covers the mean-field training-loop kernels.
 *
 * Conventions: every function returns 0 on success and -1 on failure (message on stderr and in
 * mfx_last_error()); the reference returns 0 and aborts on fatal errors instead.  "d_" pointers
 * are device pointers, the others host pointers.  Streams are hipStream_t passed as void*.
 */
#ifndef MAGENT_AMD_H
#define MAGENT_AMD_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- part 1: reference ABI */
/* runtime_api.h:20 env_new_game -- name must be "GridWorld" (DiscreteSnake is out of scope) */
int env_new_game(void **game, const char *name);
/* runtime_api.h:21 */
int env_delete_game(void *game);
/* runtime_api.h:22 -- keys of GridWorld::set_config (GridWorld.cc:126-155): map_width,
 * map_height (int*), minimap_mode, food_mode, turn_mode, goal_mode (bool*), embedding_size (int*),
 * render_dir (char*), seed (int*) -- every key the reference accepts */
int env_config_game(void *game, const char *key, void *value);
/* runtime_api.h:25 */
int env_reset(void *game);
/* runtime_api.h:26 -- bufs[0] = float[n][view_h][view_w][n_ch], bufs[1] = float[n][feature] */
int env_get_observation(void *game, int group, float **bufs);
/* runtime_api.h:27 -- actions int32[n] in group-vector order */
int env_set_action(void *game, int group, const int *actions);
/* runtime_api.h:28 */
int env_step(void *game, int *done);
/* runtime_api.h:29 -- float[n] */
int env_get_reward(void *game, int group, float *buffer);
/* runtime_api.h:32 -- num, id, pos, alive, action_space, view_space, feature_space,
 * view2attack, attack_base, both_attack, global_minimap, mean_info, walls_info,
 * render_window_info, attack_event, groups_info (GridWorld.cc:777-978) */
int env_get_info(void *game, int group, const char *name, void *buffer);
/* runtime_api.h:35-36 -- RenderGenerator's frame files: config.json + video_<n>.txt of env 0
 * (RenderGenerator.cc), byte-identical to the reference build's; only the websocket server and the
 * JS viewer are out of scope */
int env_render(void *game);
int env_render_next_file(void *game);
/* runtime_api.h:42 -- AgentType reflection keys (AgentType.cc:63-101) */
int gridworld_register_agent_type(void *game, const char *name, int n, const char **keys, float *values);
/* runtime_api.h:43 */
int gridworld_new_group(void *game, const char *agent_type_name, int *group);
/* runtime_api.h:44-45 -- method "custom" | "random" | "fill"; group -1 = walls */
int gridworld_add_agents(void *game, int group, int n, const char *method, const int *pos_x, const int *pos_y,
                         const int *dir);
/* runtime_api.h:48 */
int gridworld_clear_dead(void *game);
/* runtime_api.h:49 -- "random" only (GridWorld.cc:729-740): advances the engine LCG like the
 * reference, goals are never read back */
int gridworld_set_goal(void *game, int group, const char *method, const int *linear_buffer);
/* runtime_api.h:52-55 -- the full reward DSL (RewardEngine.cc:14-443): and / or / not over
 * attack / kill / collide / at / in / die / in_a_line events, 'any' / 'all' / fixed-index symbols,
 * group receivers, terminal rules.  Rules of the one-event attack/kill/collide form run
 * data-parallel, the rest through a one-lane interpreter; 'align' fails loudly (the reference
 * never fills the counters it reads).  The reference python passes 6 arguments to the
 * 7-parameter add_reward_rule; auto_value is never read (RewardEngine.cc:252, OP_ALIGN only). */
int gridworld_define_agent_symbol(void *game, int no, int group, int index);
int gridworld_define_event_node(void *game, int no, int op, int *inputs, int n_inputs);
int gridworld_add_reward_rule(void *game, int on, int *receiver, float *value, int n_receiver, bool is_terminal,
                              bool auto_value);
/* Extension of env_get_observation (runtime_api.h:26) for the drop-in python: the same views and
 * features of env 0 (n agents), as pointers into engine-owned pinned memory the drop-in step wrote
 * them to (no copy), in blocks of `rows` agents that stay at those addresses until the group
 * outgrows them; valid until the step after next or env_delete_game.  Returns 1 (nothing set) when
 * the observation is not held that way -- call env_get_observation then. */
int mfx_env_observation_view(void *game, int group, float **view, float **feature, int *n, int *rows);
/* Extension of env_get_info("num") + env_get_info("id" / "alive" / "pos") / env_get_reward (runtime_api.h:29, :32)
 * for the drop-in python: one call per getter.  Returns the group's agent count n and, when n <= cap, copies
 * its n rows of field `what` (0 id int32, 1 reward float32, 2 alive uint8, 3 pos int32 x 2; -1: the count only)
 * into out; -1 on error. */
int mfx_env_get_rows(void *game, int group, int what, void *out, int cap);

/* ---------------------------------------------------------------- part 2: batched Battle */
/* Before the first env_reset: make the engine hold n_envs identical envs. */
int mfx_battle_set_num_envs(void *game, int n_envs);
/* Launch everything on this hipStream_t (may be the null stream). */
int mfx_battle_set_stream(void *game, void *stream);
/* Per-call API on device buffers; per-agent arrays are [E][rowcap][...]. */
int mfx_battle_observe(void *game, int group, float *d_view, float *d_feature, int rowcap);
int mfx_battle_set_action(void *game, int group, const int *d_actions, int rowcap);
int mfx_battle_step(void *game, int *d_done);
/* what: 0 num ([E]), 1 reward (f32), 2 id (i32), 3 alive (u8), 4 pos (i32 x2), 5 hp (f32) */
int mfx_battle_get(void *game, int group, int what, void *d_out, int rowcap);
int mfx_battle_clear_dead(void *game);
/* Wait for the stream and report any device-side error (capacity, bad action, ...). */
int mfx_battle_sync(void *game);
/* Upper bound of a group's size (rows needed per env). */
int mfx_battle_group_capacity(void *game, int group, int *cap);
/* Fused rollout: one launch per training-loop step for all envs (obs for every group, on-device
 * rush policy, set_action, step, reward, mean action, clear_dead, restart at done / max_steps).
 * tmpl_n[G], xs[G][tmpl_n[g]], ys[...]: placement re-applied at every episode start. */
int mfx_battle_rollout_init(void *game, const int *tmpl_n, const int *const *xs, const int *const *ys,
                            int max_steps, float eps, unsigned seed, int stagger);
int mfx_battle_rollout_step(void *game, int n_steps);
/* Steps per launch (1..64, up to 1024 on the pipelined few-env path; default 1; 0 = chosen per path and batch
 * size): k_rollout runs each env's steps
 * back to back with its image resident in LDS; the large-env queue kernel (k_rollout_bigq) runs every env's
 * steps in one launch.  rollout_step(n) gives identical results for every value.  get: the value in force. */
int mfx_battle_rollout_set_substeps(void *game, int n_sub);
int mfx_battle_rollout_get_substeps(void *game, int *n_sub);
/* names: view, feature, actions, rewards, mean_action, episode_return, stats, agent_steps, group_num */
int mfx_battle_rollout_buffer(void *game, const char *name, int group, void **d_ptr, size_t *bytes);
int mfx_battle_rollout_copy(void *game, const char *name, int group, void *dst, size_t bytes);
/* bytes [offset, offset + bytes) of a rollout buffer (e.g. one env's rows), async on the engine stream */
int mfx_battle_rollout_copy_at(void *game, const char *name, int group, size_t offset, void *dst, size_t bytes);
int mfx_battle_rollout_rowcap(void *game, int *rowcap);
/* Doubles per [env][group] row of the rollout's mean-action buffer (the largest n_action of the groups). */
int mfx_battle_rollout_mean_stride(void *game, int *stride);
/* Persistent grid (workgroups per launch) and dynamic LDS bytes per workgroup of the fused rollout. */
int mfx_battle_rollout_info(void *game, int *grid, int *lds_bytes);
/* Synchronises the engine stream; -1 (message in mfx_last_error) if a device error was raised or, on the
 * large-env queue kernel k_rollout_bigq, its work queue reported an error (a stall, a workgroup outside
 * XCDs 0-7, or the hand-off guard: an item that saw a step counter other than its own). */
int mfx_battle_rollout_check(void *game);
/* The kernels rollout_step runs: 0 k_rollout, 1 k_rollout_obs + k_rollout (pipeline), 2 k_observe_items +
 * k_rollout_big (large-env pipeline), 3 k_rollout_bigq. */
int mfx_battle_rollout_path(void *game, int *path);
/* Lanes over which the rollout sums a group's rewards of an env with n_agents agents: the summation order of
 * the episode returns (64: one wave, 256 / 512: a workgroup's lane-strided partials, then wave sums). */
int mfx_battle_rollout_sum_lanes(void *game, int n_agents, int *lanes);
/* A learned policy in the loop (the fused k_rollout path: batches of LDS-sized envs larger than the few-env
 * threshold): mode 2 writes every env's observation into the rollout buffers; mode 1 takes the actions in
 * the rollout's action buffer (a policy forward on that observation, e.g. mfx_qnet_act_rollout), runs
 * set_action / step / reward / mean action / clear_dead / restart and writes the next observation.  The
 * mean-action buffer then holds each group's former_act_prob (zeros at an episode's first step). */
int mfx_battle_rollout_policy_step(void *game, int mode);
/* The inputs of group `group`'s observation view that can be non-zero (Map.cc:130-218): mask[n] (n = view_h *
 * view_w * n_ch, NHWC) = 1 for every channel of a cell inside the view range and for the minimap channels of the
 * cells outside it, else 0 (never written: always zero). */
int mfx_battle_view_support(void *game, int group, uint8_t *mask, int n);
/* Diagnostic build only (libmagent_stamps.so): per-phase s_memtime stamps [E][16]. */
int mfx_battle_set_stamp_buffer(void *d_buf);

/* ---------------------------------------------------------------- part 3: Ising MF-Q */
int mfx_ising_create(int replicas, int n_agents, int k, const int16_t *nbr, void **handle);
int mfx_ising_destroy(void *handle);
int mfx_ising_set_spins(void *handle, const uint8_t *spins);
int mfx_ising_get_spins(void *handle, uint8_t *spins);
/* IsingMultiAgentEnv.step for every replica (environment.py:49-78) */
int mfx_ising_step(void *handle, const int32_t *actions, double *reward, uint8_t *obs, int32_t *n_up,
                   double *order);
/* The episode loop of main_MFQ_Ising.py (:84-159) in one launch per batch of replicas. */
int mfx_ising_mfq_run(void *handle, int T, double temperature, double lr, double decay_rate, int decay_gap,
                      const double *u, const uint32_t *mask, unsigned seed, double *q, double *order,
                      int32_t *n_up, int32_t *steps);
/* main_MFQ_Ising.py with its numpy RandomState stream generated on the device (MT19937, numpy's legacy draws: the
 * Boltzmann uniforms and the act_group permutation): replica r runs the script with seed seed0 + r for `episodes`
 * episodes in sequence on one stream (-epi), each until its early stop; outputs per episode (host, nullable except
 * q): q [E][R][N][K+1][2], order [E][R][T], n_up [E][R][T], steps [E][R]. */
int mfx_ising_mfq_run_stream(void *handle, int T, double temperature, double lr, double decay_rate, int decay_gap,
                             double act_rate, unsigned seed0, int episodes, double *q, double *order, int32_t *n_up,
                             int32_t *steps);

/* ---------------------------------------------------------------- part 4: mean-field kernels */
/* senario_battle.py:141 */
int mfx_mean_action(const int32_t *d_acts, const int32_t *d_counts, int B, int rowcap, int n_action, double *d_out,
                    void *stream);
/* algo/base.py:192-220 */
int mfx_mfq_target(const float *d_eq, const float *d_tq, const float *d_r, const uint8_t *d_done, int M, int A,
                   double gamma, double *d_out, void *stream);
/* algo/ac.py:305-320 -- numpy1 = 1: the reference's NumPy-1 promotion (float64 running return, the
 * default of the python wrapper); 0: NEP-50 (float32), as the same lines run under NumPy 2 */
int mfx_mfac_returns(float *d_rew, const int64_t *d_offsets, const float *d_value, int n_ep, double gamma,
                     int numpy1, void *stream);

/* ---------------------------------------------------------------- part 5: policy forward */
/* The Q network of ValueNet._construct_net (algo/base.py:123-183) and its greedy act (:228-254), forward
 * only, f32 MFMA (csrc/policy_kernels.hip); the Battle view (13 x 13 x 7), features F <= 256, n_action <= 32.
 * Weights: one float32 blob of n_floats in the layout mfx_qnet_blob_size reports (18 offsets: w1 b1 w2 b2
 * wd bd we be wp1 bp1 wp2 bp2 w2d b2d wo bo wq bq, every matrix [K][N] row-major, K padded to 4). */
int mfx_qnet_blob_size(int feature, int n_action, int use_mf, size_t *n_floats, size_t *offsets);
int mfx_qnet_create(int view_h, int view_w, int n_ch, int feature, int n_action, int use_mf, void **handle);
int mfx_qnet_destroy(void *handle);
int mfx_qnet_set_weights(void *handle, const float *d_blob, size_t n_floats, void *stream);
/* n agents: view [n][1183], feature [n][F], prob [n][A] (mean field, else null) -> q [n][A], act [n] */
int mfx_qnet_forward(void *handle, const float *d_view, const float *d_feat, const float *d_prob, int n, float *d_q,
                     int32_t *d_act, void *stream);
/* group g of a rollout batch -> the rollout's action buffer (live rows); d_rows: E * rowcap ints scratch, d_total:
 * 1 + ceil(E / 64) ints (the row count, then per-64-env chunk totals) -- one buffer of E * rowcap + 1 + ceil(E / 64)
 * ints with d_total = d_rows + E * rowcap is the usual layout */
int mfx_qnet_act_rollout(void *handle, const float *d_view, const float *d_feat, const int32_t *d_counts,
                         const double *d_mean, int mean_stride, int E, int G, int g, int rowcap, int32_t *d_rows,
                         int32_t *d_total, int32_t *d_act, void *stream);
/* (the row count stays on the device: the kernels are launched for E * rowcap rows and read *d_total) */

/* The compact row list the act_rollout calls build: d_rows[i] = e * rowcap + j over envs e, j < min(counts[e][g],
 * rowcap), in env order; d_total[0] = the row count (d_total: 1 + ceil(E / 64) ints). */
int mfx_rollout_rows(const int32_t *d_counts, int E, int G, int g, int rowcap, int32_t *d_rows, int32_t *d_total,
                     void *stream);

/* The actor-critic network of ActorCritic._create_network (algo/ac.py:48-98) / MFAC._create_network (:219-276)
 * and its act, tf.multinomial(log(policy)) (:43-46, :213-217), forward only, f32 MFMA
 * (csrc/acnet_kernels.hip); views of view_floats <= 4096 floats (flattened NHWC), features <= 256,
 * 2 <= n_action <= 32.  Weights: one float32 blob in the layout mfx_acnet_blob_size reports (19 offsets: wv bv
 * we be wd0 wd1 bd wp bp wval bval wep bep wdp bdp wvd bvd wvo bvo, every matrix [K][N] row-major, K padded to
 * 4; the 512-wide dense layer split by output halves).  The draw of row r of group g at step t is the first
 * action whose running f32 sum of the clipped policy exceeds u * (its f32 total), u = a 24-bit counter hash of
 * (seed, t, g, r) (tests/acnet_ref.py restates it). */
int mfx_acnet_blob_size(int view_floats, int feature, int n_action, int use_mf, size_t *n_floats, size_t *offsets);
int mfx_acnet_create(int view_floats, int feature, int n_action, int use_mf, void **handle);
int mfx_acnet_destroy(void *handle);
int mfx_acnet_set_weights(void *handle, const float *d_blob, size_t n_floats, void *stream);
/* The view inputs that can be non-zero, mask[n] (n = view_floats; e.g. mfx_battle_view_support), or null for the dense
 * order: later forwards run the view layer over the supported inputs only, bit-identical when the others are zero
 * (the caller's contract).  input_support_size: the inputs the view layer runs over (0 = dense). */
int mfx_acnet_set_input_support(void *handle, const uint8_t *mask, int n, void *stream);
int mfx_acnet_input_support_size(void *handle, int *k);
/* n agents: view [n][view_floats], feature [n][F], prob [n][A] float32 (the MF value head; else null) ->
 * policy [n][A], value [n], act [n] (each may be null); row i drawn with (seed, step, group 0, row i) */
int mfx_acnet_forward(void *handle, const float *d_view, const float *d_feat, const float *d_prob, int n,
                      float *d_policy, float *d_value, int32_t *d_act, uint32_t seed, uint32_t step, void *stream);
/* group g of a rollout batch -> sampled actions in the rollout's action buffer (live rows; row j of env e drawn
 * with (seed, step, g, e * rowcap + j)); d_rows / d_total as mfx_qnet_act_rollout's; nothing is read back */
int mfx_acnet_act_rollout(void *handle, const float *d_view, const float *d_feat, const int32_t *d_counts, int E,
                          int G, int g, int rowcap, int32_t *d_rows, int32_t *d_total, int32_t *d_act, uint32_t seed,
                          uint32_t step, void *stream);

/* ---------------------------------------------------------------- part 6: replay rows */
/* The data path of the replay buffers (algo/tools.py:26-362): for i < n, row idx[i] (or i; modulo src_mod
 * when > 0) of every source column -> row dst_start + i (modulo dst_cap when > 0) of its destination column;
 * n_cols <= 12, row_bytes per column; one launch (csrc/replay_kernels.hip).  src_rows: rows of every source
 * column -- without src_mod an index in [-src_rows, 0) counts from the end, as numpy's indexing does; any other
 * index outside [0, src_rows) (the reference's numpy indexing raises IndexError) skips the row and is reported by
 * mfx_rows_copy_error (synchronising; -1 and *bad_index when one was met, -1 included, then cleared). */
int mfx_rows_copy(int n_cols, void *const *dst, const void *const *src, const int64_t *row_bytes, const int64_t *d_idx,
                  int64_t src_mod, int64_t src_rows, int64_t dst_start, int64_t dst_cap, int64_t n, void *stream);
/* The same move with the columns whose bit is set in shift_mask reading source row idx[i] + shift (before the
 * modulo, checked the same way): MemoryGroup.sample's next-state columns at next_idx = (idx + 1) % nb_entries
 * (algo/tools.py:239-262) in the launch of the current-state columns.  mfx_rows_copy = shift_mask 0. */
int mfx_rows_copy_shift(int n_cols, void *const *dst, const void *const *src, const int64_t *row_bytes,
                        const int64_t *d_idx, int64_t src_mod, int64_t src_rows, int64_t dst_start, int64_t dst_cap,
                        int64_t n, uint32_t shift_mask, int64_t shift, void *stream);
int mfx_rows_copy_error(int64_t *bad_index, void *stream);

/* ---------------------------------------------------------------- measurement */
/* The HBM write ceiling on this device, measured in-process beside the bench (csrc/diag_kernels.hip): total_bytes
 * of float4 stores over the device region [d_buf, d_buf + region_bytes), wrapping; shape 0..7: bit 0 = nontemporal
 * stores, bits 1-2 = 4 / 8 / 16 KiB chunks, one workgroup per chunk, or (3) 4 KiB chunks on a persistent grid;
 * *ms = HIP-event time (synchronises). */
int mfx_store_ceiling(void *d_buf, size_t region_bytes, size_t total_bytes, int shape, void *stream, float *ms);

/* ---------------------------------------------------------------- library */
const char *mfx_last_error(void);
const char *mfx_build_info(void);
int mfx_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MAGENT_AMD_H */
