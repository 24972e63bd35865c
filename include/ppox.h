/*
 * ppox.h — C ABI of libppox.so, the MI355X (gfx950) hot path of the PPO +
 * exploration training loop (BoogaQ/PPO-exploration drop-in).
 *
 * Conventions (every entry point):
 *   - plain pointers + sizes; every array pointer is a DEVICE pointer unless
 *     the parameter name ends in _host;
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream);
 *     the call only enqueues work on it: no allocation, no host sync, so every
 *     entry point is hipGraph-capturable;
 *   - return 0 on success, PPOX_EINVAL on a rejected argument, or
 *     -(hipError_t) when a launch fails; ppox_last_error() describes the most
 *     recent failure on the calling thread;
 *   - the library never allocates; scratch comes from caller workspaces.
 *
 * Rollout arrays are STEP-MAJOR, element (t, n) at t*N + n, exactly the
 * reference's (buffer_size, n_envs) layout (buffer.py:153-161).  Minibatch
 * indices are the reference's ENV-MAJOR flat indices i = n*T + t
 * (swap_and_flatten, buffer.py:41-52); kernels map i -> (t = i % T, n = i / T)
 * so the rollout is never physically flattened.
 *
 * The reference has no FFI: each function below replaces a Python/numpy/torch
 * site, cited as file:line relative to the reference repository.
 */
#ifndef PPOX_H
#define PPOX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPOX_OK 0
#define PPOX_EINVAL (-1000)

/* Library identification and error reporting. */
const char* ppox_version(void);
const char* ppox_last_error(void);

/* ---------------------------------------------------------------------------
 * K1  GAE(lambda) backward scan.
 * Replaces RolloutStorage.compute_returns_and_advantages (buffer.py:203-230).
 *   rewards, values : (T, N) f32        dones : (T, N) u8 — done flag stored by
 *   add() at step t (the reference's `masks`, ppo.py:192)
 *   last_value : (N,) f32 — V(s_{T-1}) as passed by ppo.py:196
 *   last_done  : (N,) u8  — dones of the last env step (ppo.py:196)
 * Output advantages/returns (T, N) f32 are BIT-IDENTICAL to the reference:
 * f32 gamma*next_value, float64 carry, returns = adv + values in f32.
 * -------------------------------------------------------------------------*/
int ppox_gae(const float* rewards, const float* values, const uint8_t* dones,
             const float* last_value, const uint8_t* last_done, int64_t T, int64_t N,
             double gamma, double lam, float* advantages, float* returns, void* stream);

/* Two reward streams.  Replaces IntrinsicStorage.compute_returns_and_advantages
 * (buffer.py:321-362): extrinsic stream as ppox_gae; intrinsic stream is
 * non-episodic (no done mask) and computed in f32 with f32(int_gamma*lam). */
int ppox_gae_dual(const float* rewards, const float* values, const uint8_t* dones,
                  const float* last_value, const uint8_t* last_done,
                  const float* int_rewards, const float* int_values, const float* last_int_value,
                  int64_t T, int64_t N, double gamma, double int_gamma, double lam,
                  float* advantages, float* returns, float* int_advantages, float* int_returns,
                  void* stream);


/* ---------------------------------------------------------------------------
 * K2/K3  Running moments and observation normalisation.
 * Replace RunningMeanStd.update/update_from_moments (util.py:20-44) and
 * BaseAlgorithm.normalize_obs (ppo.py:111-118).  State (mean, var: float64
 * per feature) lives on the device; `count` is the host-side float the
 * reference keeps in Python (util.py:18), passed by value (the caller adds
 * `rows` to it afterwards, exactly like util.py:40-44).
 * -------------------------------------------------------------------------*/
/* u8 batch (rows, cols) with row stride (bytes): exact integer column sums;
 * optional batch_mean/batch_var outputs (nullable); mean/var nullable together
 * (moments only).  Workspace: ppox_rms_u8_workspace_bytes(rows, cols). */
int64_t ppox_rms_u8_workspace_bytes(int64_t rows, int64_t cols);
int ppox_rms_update_u8(const uint8_t* x, int64_t rows, int64_t cols, int64_t row_stride,
                       double* mean, double* var, double count, void* workspace,
                       int64_t workspace_bytes, double* batch_mean, double* batch_var, void* stream);
/* f32 batch: numpy's own summation order (bit-identical batch moments). */
int ppox_rms_update_f32(const float* x, int64_t rows, int64_t cols, int64_t row_stride,
                        double* mean, double* var, double count, void* stream);
/* int_rew_rms.update(r); r /= sqrt(var) + 1e-8  (ppo.py:396-398), in place on (n,) f32. */
int ppox_rms_scale_int_rewards(float* int_rewards, int64_t n, double* mean, double* var,
                               double count, void* stream);
/* out (rows, cols) f32 = f32(clip((x - mean) / sqrt(var + 1e-10), -5, 5)) computed in f64. */
int ppox_normalize_obs_u8(const uint8_t* x, int64_t rows, int64_t cols, int64_t row_stride,
                          const double* mean, const double* var, float* out, void* stream);
int ppox_normalize_obs_f32(const float* x, int64_t rows, int64_t cols, int64_t row_stride,
                           const double* mean, const double* var, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * K4  Fused PPO minibatch loss (ppo.py:216-238; RND ppo.py:428-460; ICM policy
 * part ppo.py:668-692) and the collect-time categorical head (models.py:30-41).
 * Minibatch rows come from the network outputs (logits (B, A), values (B,),
 * int_values (B,) or NULL for one stream) and from the rollout through the
 * env-major indices idx (B,) — never a gathered copy of the scalar fields.
 * adv_stats (device, [4] f64): mean, unbiased std of the minibatch advantages
 * (and of the intrinsic ones) — see ppox_minibatch_adv_stats.
 * -------------------------------------------------------------------------*/
#define PPOX_LOSS_PARTIALS 64
/* Per-minibatch advantage mean / unbiased std (ppo.py:219) for every slice
 * [k*batch, (k+1)*batch) of the epoch permutation; stats_out [n_mb][4]. */
int ppox_minibatch_adv_stats(const float* advantages, const float* int_advantages,
                             const int64_t* perm, int64_t total, int64_t batch_size,
                             int64_t T, int64_t N, double* stats_out, void* stream);
/* Forward partial sums -> partials [PPOX_LOSS_PARTIALS][8] f64 (sum-reducible
 * across data-parallel ranks). */
int ppox_ppo_loss_partials(const float* logits, const float* values, const float* int_values,
                           int64_t B, int32_t A, const int64_t* idx, int64_t T, int64_t N,
                           const int32_t* actions, const float* old_logp, const float* old_values,
                           const float* advantages, const float* returns,
                           const float* old_int_values, const float* int_advantages,
                           const float* int_returns, const double* adv_stats, float clip,
                           double* partials, void* stream);
/* Backward: dL/dlogits (B, A), dL/dvalues (B,), dL/dint_values (B,) for the loss
 * scale * (policy + ent_coef*entropy + vf_coef*value [+ int_vf_coef*int_value]),
 * means taken over B_global rows.  loss_accum (nullable, [8] f64) += this
 * minibatch's [policy, value, entropy, total, int_value, 1]. */
int ppox_ppo_loss_backward(const float* logits, const float* values, const float* int_values,
                           int64_t B, int32_t A, const int64_t* idx, int64_t T, int64_t N,
                           const int32_t* actions, const float* old_logp, const float* old_values,
                           const float* advantages, const float* returns,
                           const float* old_int_values, const float* int_advantages,
                           const float* int_returns, const double* adv_stats, float clip,
                           const double* partials, int64_t B_global, float ent_coef,
                           float vf_coef, float int_vf_coef, float scale, float* dlogits,
                           float* dvalues, float* dint_values, double* loss_accum, void* stream);
/* Box action spaces (models.py:40-46, 66-71: Normal(tanh(mu), exp(action_log_std)),
 * per-dimension surrogate, ppo.py:216-238).  mu = actor pre-activations (B, D);
 * actions / old_logp are the rollout's (T, N, D) step-major arrays.  log_prob,
 * ratio and surrogate run in f64 (the reference's f64 actions promote them,
 * buffer.py:156); clip is the Python float clip_range.  The backward also
 * returns dL/d(action_log_std) (D,) = the fixed-order sum of
 * dlog_std_partials [PPOX_LOSS_PARTIALS][D] f64 (caller workspace). */
int ppox_ppo_box_loss_partials(const float* mu, const float* log_std, const float* values,
                               const float* int_values, int64_t B, int32_t D, const int64_t* idx,
                               int64_t T, int64_t N, const float* actions, const float* old_logp,
                               const float* old_values, const float* advantages,
                               const float* returns, const float* old_int_values,
                               const float* int_advantages, const float* int_returns,
                               const double* adv_stats, double clip, double* partials,
                               void* stream);
int ppox_ppo_box_loss_backward(const float* mu, const float* log_std, const float* values,
                               const float* int_values, int64_t B, int32_t D, const int64_t* idx,
                               int64_t T, int64_t N, const float* actions, const float* old_logp,
                               const float* old_values, const float* advantages,
                               const float* returns, const float* old_int_values,
                               const float* int_advantages, const float* int_returns,
                               const double* adv_stats, double clip, const double* partials,
                               int64_t B_global, float ent_coef, float vf_coef, float int_vf_coef,
                               float scale, float* dmu, double* dlog_std_partials, float* dlog_std,
                               float* dvalues, float* dint_values, double* loss_accum,
                               void* stream);
/* a ~ Normal(tanh(mu), exp(log_std)) per dimension (Philox + Box-Muller), f32
 * log_prob(a) (models.py:42-45). */
int ppox_normal_sample(const float* mu, const float* log_std, int64_t N, int32_t D,
                       int64_t env_offset, uint64_t seed, int64_t counter, float* actions,
                       float* log_probs, void* stream);
/* a ~ Categorical(probs=softmax(logits)) (Philox, counter-based), log_prob(a). */
int ppox_categorical_sample(const float* logits, int64_t N, int32_t A, int64_t env_offset,
                            uint64_t seed, int64_t counter, int32_t* actions, float* log_probs,
                            void* stream);
/* The same draw with the Philox counter read from the device: counter = *counter_base +
 * counter_off (a graph-captured collect step keeps its counters in device memory and
 * advances them with ppox_counters_add; ppo.py:174-194 draws one action per env per step). */
int ppox_categorical_sample_dc(const float* logits, int64_t N, int32_t A, int64_t env_offset,
                               uint64_t seed, const int64_t* counter_base, int64_t counter_off,
                               int32_t* actions, float* log_probs, void* stream);

/* ---------------------------------------------------------------------------
 * K8  SimHash count bonus (buffer.py:188-200, RolloutStorage(sim_hash=True)).
 * keys[n] = sign bits of A @ obs[n] (A: 16 x D f64 row-major, bit b <- row b).
 * apply: for the local envs [offset, offset + n_local) of the step's n_total
 * keys (global env order), rewards[i] += beta / sqrt(count) with the count the
 * reference's sequential dictionary update gives that env; then counts (65,536
 * u32, replicated per rank) += every key of the step.
 * -------------------------------------------------------------------------*/
#define PPOX_SIMHASH_KEYS 65536
int ppox_simhash_keys(const float* obs, int64_t N, int64_t D, int64_t obs_stride,
                      const double* A, int32_t* keys, void* stream);
int ppox_simhash_apply(const int32_t* keys_all, int64_t n_total, int64_t offset, int64_t n_local,
                       uint32_t* counts, double beta, float* rewards, void* stream);

/* ---------------------------------------------------------------------------
 * K5  Minibatch gather (buffer.py:41-52, 256-267): dst[r] = rollout row of the
 * env-major index idx[r]; rows of row_bytes at src_row_stride (step-major).
 * -------------------------------------------------------------------------*/
/* dst[i] = (float)src[i], n a multiple of 16, 16B-aligned (the ICM encoder's float input). */
int ppox_u8_to_f32(const void* src, int64_t n, float* dst, void* stream);
int ppox_gather_rows(const void* src, int64_t T, int64_t N, int64_t row_bytes,
                     int64_t src_row_stride, const int64_t* idx, int64_t nrows, void* dst,
                     void* stream);

/* ---------------------------------------------------------------------------
 * Optimiser over flat buffers: clip_grad_norm_ + Adam.step (ppo.py:241-244).
 * ppox_grad_sumsq writes PPOX_NORM_PARTIALS f64 partial sums of g^2 (caller may
 * sum-reduce them across ranks only if grads are NOT yet all-reduced — normally
 * they are, and the partials are used as-is).
 * -------------------------------------------------------------------------*/
#define PPOX_NORM_PARTIALS 256
int ppox_grad_sumsq(const float* grads, int64_t n, double* partials, void* stream);
/* Bench timing of an entry point's main kernel (bench.py): arm a (timing-enabled) hipEvent_t; an entry point that
 * ends in a reduce of its kernel's partial slabs (the weight gradients) records it on its stream just before that
 * reduce; ppox_ktime_take returns 1 if one did (and disarms). */
void ppox_ktime_arm(void* event);
int ppox_ktime_take(void);
int ppox_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                   const double* norm_partials, float max_norm, double lr, double beta1,
                   double beta2, double eps, int64_t step, float* total_norm_out, void* stream);
/* ppox_adam_step that also records the amax partials of the NatureCNN weights it updates (round 6: the
 * weight packing's amax pass folded into the Adam step).  ranges (host): PPOX_WMAX_TENSORS element offsets
 * into params, then as many counts (0: none) — conv1, conv2, conv3, fc and the heads' hidden-layer weight,
 * in ppox_nature_pack_all's order; amax_out (16B-aligned, PPOX_WMAX_TENSORS x PPOX_WMAX_SLOTS uint32, zeroed
 * beforehand: ppox_nature_pack_all_wmax's amax_next) gets per slot the maximum |p| after the update (f32 bits,
 * atomicMax: order-free, deterministic).  Params, moments and total_norm_out bitwise ppox_adam_step's. */
#define PPOX_WMAX_TENSORS 5
#define PPOX_WMAX_SLOTS 256
int ppox_adam_step_wmax(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                        const double* norm_partials, float max_norm, double lr, double beta1, double beta2,
                        double eps, int64_t step, float* total_norm_out, const int64_t* ranges,
                        uint32_t* amax_out, void* stream);

/* ---------------------------------------------------------------------------
 * Synthetic device environments (replace SB3 SubprocVecEnv + gym/ALE, env.py:7-12).
 * Philox4x32-10 keyed by seed, counter (block, env_offset + n, step, action).
 * -------------------------------------------------------------------------*/
int ppox_atari_env_reset(uint8_t* obs, int64_t N, int64_t env_offset, uint64_t seed,
                         float* ep_ret, int32_t* ep_len, void* stream);
int ppox_atari_env_step(const uint8_t* obs_in, uint8_t* obs_out, const int32_t* actions,
                        int64_t N, int64_t env_offset, uint64_t seed, int64_t step,
                        float p_reward, float p_done, float* rewards, uint8_t* dones,
                        float* ep_ret, int32_t* ep_len, float* done_ret, int32_t* done_len,
                        void* stream);
/* step = *step_base + step_off, read on the device (graph-captured collect). */
int ppox_atari_env_step_dc(const uint8_t* obs_in, uint8_t* obs_out, const int32_t* actions,
                           int64_t N, int64_t env_offset, uint64_t seed, const int64_t* step_base,
                           int64_t step_off, float p_reward, float p_done, float* rewards,
                           uint8_t* dones, float* ep_ret, int32_t* ep_len, float* done_ret,
                           int32_t* done_len, void* stream);
/* counters[i] += delta for i < n (n <= 64): advances device-resident step counters. */
int ppox_counters_add(int64_t* counters, int32_t n, int64_t delta, void* stream);
int ppox_vec_env_reset(float* obs, int64_t N, int32_t D, int64_t env_offset, uint64_t seed,
                       float* ep_ret, int32_t* ep_len, void* stream);
int ppox_vec_env_step(float* obs, const int32_t* actions, int64_t N, int32_t D,
                      int64_t env_offset, uint64_t seed, int64_t step, float p_done,
                      int32_t max_len, float* rewards, uint8_t* dones, float* ep_ret,
                      int32_t* ep_len, float* done_ret, int32_t* done_len, void* stream);

/* ---------------------------------------------------------------------------
 * K6  NatureCNN convolutions (checkpoint models-checkpoint.py:52-58) and their
 * backward, as fp32 MFMA implicit GEMMs (v_mfma_f32_32x32x2_f32).
 *   layer 1: x = uint8 frames (batch, 4, 84, 84) [or rollout rows through idx:
 *            sample b = step-major row (idx[b] % T, idx[b] / T) of a (T, N_env, ...)
 *            array] -> y (batch, 20, 20, 32) f32 NHWC
 *   layer 2: x (batch, 20, 20, 32) NHWC -> y (batch, 9, 9, 64) NHWC
 *   layer 3: x (batch, 9, 9, 64) NHWC -> y (batch, 64, 7, 7) NCHW (Flatten order)
 * Forward fuses + bias and ReLU.  Weights are PyTorch [co][ci][ky][kx]; the
 * kernels read copies packed by ppox_nature_pack_weights (once per optimizer
 * step): wp1 [256][32], wp2 [512][64], wp3 [576][64] (forward), wpd2 [4][256][32],
 * wpd3 [576][64] (dgrad; nullable if no backward is needed).
 * -------------------------------------------------------------------------*/
int ppox_nature_pack_weights(const float* w1, const float* w2, const float* w3, float* wp1,
                             float* wp2, float* wp3, float* wpd2, float* wpd3, void* stream);
int ppox_nature_conv_fwd(int32_t layer, const void* x, int64_t batch, const int64_t* idx,
                         int64_t T, int64_t N_env, int64_t x_sample_stride, const float* wp,
                         const float* bias, float* y, void* stream);
/* grad_in (NHWC, layer input shape) = conv_transpose(grad_out NHWC, W) * (prev_act > 0):
 * the ReLU backward of the previous layer is fused (prev_act = its NHWC output). */
int ppox_nature_conv_dgrad(int32_t layer, const float* grad_out, int64_t batch, const float* wpd,
                           const float* prev_act, float* grad_in, void* stream);
/* dW (PyTorch layout) and db from the layer input x (as in ppox_nature_conv_fwd) and
 * the ReLU-masked output grad (NHWC), in two launches: ppox_nature_conv_wgrad writes
 * split-K partial slabs (over output pixels) into a workspace of
 * ppox_nature_wgrad_workspace_bytes(layer, batch); ppox_nature_wgrad_reduce sums
 * them in a fixed order (deterministic) into dw [co][ci][ky][kx] and db. */
int64_t ppox_nature_wgrad_splits(int32_t layer, int64_t batch);
int64_t ppox_nature_wgrad_workspace_bytes(int32_t layer, int64_t batch);
int ppox_nature_conv_wgrad(int32_t layer, const void* x, int64_t batch, const int64_t* idx,
                           int64_t T, int64_t N_env, int64_t x_sample_stride,
                           const float* grad_out, void* workspace, int64_t workspace_bytes,
                           void* stream);
int ppox_nature_wgrad_reduce(int32_t layer, int64_t batch, const void* workspace, float* dw,
                             float* db, void* stream);
/* (batch, 64, 7, 7) NCHW grad of the trunk output -> NHWC, times (act > 0). */
int ppox_nchw_to_nhwc_relu_grad(const float* grad, const float* act, int64_t batch, float* out,
                                void* stream);

/* SB3 VecNormalize (the reference's env wrapper, env.py:10-11: VecNormalize(env,
 * norm_reward=True); stable_baselines3 0.x, not vendored — restated, parity unpinned):
 * observations: f32(clip((x - mean) / sqrt(var + eps), -clip, clip)) in f64 (obs_rms
 * updated with ppox_rms_update_f32 first); rewards, in place: ret = ret * gamma + r,
 * ret_rms.update(ret) (float64 pairwise moments, Chan merge; skipped when update = 0),
 * r = clip(r / sqrt(ret_rms.var + eps), -clip, clip), ret[dones] = 0.  n <= 524288. */
int ppox_normalize_obs_f32_ex(const float* x, int64_t rows, int64_t cols, int64_t row_stride,
                              const double* mean, const double* var, double eps, double clip,
                              float* out, void* stream);
int ppox_vecnorm_reward(float* rewards, const uint8_t* dones, double* ret, int64_t n, double gamma,
                        double* mean, double* var, double count, double eps, double clip,
                        int32_t update, void* stream);

/* NatureCNN hidden layer Linear(3136, 512) + ReLU (.ipynb_checkpoints/models-checkpoint.py:58-59)
 * on the split-f16 GEMM (see the K6 split section below for the arithmetic and the amax slots):
 * weights packed (once per optimizer step) by ppox_nature_fc_pack into ppox_nature_fc_pack_elems()
 * uint16 each for the forward (W^T) and the dgrad (W) operand.  amax_h3 / amax_df: the slots of
 * the A operand (required); amax_g3 / amax_f: the slots the dgrad / forward record g3's / f's
 * amax into (nullable).  relu_bits (dgrad, nullable): h3's ReLU bitmask from the conv3 split forward,
 * used instead of h3.
 * Both run in NHWC feature order: h3 is the split conv3 forward's NHWC output (batch, 7, 7, 64)
 * and W is packed through the permutation f = p * 64 + c <- Flatten feature c * 49 + p.
 * fwd: f = relu(h3 @ W^T + b); dgrad: g3 (NHWC (B,7,7,64)) = (df @ W) * (h3 > 0)
 * (df = dL/df already ReLU-masked) — the trunk's ReLU backward fused. */
int64_t ppox_nature_fc_pack_elems(void);
/* All weight packings of one optimizer step in a single launch (any output may be null):
 * wpd2 = f32 conv2 dgrad ([(ky,kx,co)][ci]); q1..q3 / qd2, qd3 = split forms (as
 * ppox_nature_pack_split); qfc_fwd / qfc_dgrad = fc split forms (as ppox_nature_fc_pack).
 * With q2 / q3 / qfc_dgrad the tails also get the PX output bounds (the column l1-norms of the
 * packed matrix and, from b2 / b3 — nullable: a PX output bounded without them comes out NaN —
 * the bias bound), read by the producers of the PX planes h2, h3 and g3 (below).
 * zero (nullable, 16B-aligned): zero_words uint32 set to 0 before the packing kernels finish —
 * the next pass's amax table, so a training step needs no fill launch of its own. */
int ppox_nature_pack_all(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                         const float* b3, const float* wfc, float* wpd2, uint16_t* q1, uint16_t* q2, uint16_t* q3,
                         uint16_t* qd2, uint16_t* qd3, uint16_t* qfc_fwd, uint16_t* qfc_dgrad, const float* wh,
                         uint16_t* qh_fwd, uint16_t* qh_dgrad, uint32_t* zero, int64_t zero_words, void* stream);
/* ppox_nature_pack_all with the weights' amax partials given (round 6): amax_in (nullable) = the partials
 * ppox_adam_step_wmax recorded for exactly these weights, unchanged since — then ONE launch (no amax pass;
 * the packed forms bitwise what ppox_nature_pack_all writes, but for the tails' amax partials, which hold the
 * step's slot partition of the same maximum); null: the amax pass as ppox_nature_pack_all.  amax_next (nullable, != amax_in): PPOX_WMAX_TENSORS x PPOX_WMAX_SLOTS uint32 zeroed
 * on the way (the buffer the next ppox_adam_step_wmax records into). */
int ppox_nature_pack_all_wmax(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                              const float* b3, const float* wfc, float* wpd2, uint16_t* q1, uint16_t* q2,
                              uint16_t* q3, uint16_t* qd2, uint16_t* qd3, uint16_t* qfc_fwd, uint16_t* qfc_dgrad,
                              const float* wh, uint16_t* qh_fwd, uint16_t* qh_dgrad, const uint32_t* amax_in,
                              uint32_t* amax_next, uint32_t* zero, int64_t zero_words, void* stream);
/* conv1 -> conv2 on H1P, the split-f16 operand form of conv1's output h1 (Conv2d(4, 32, 8, 4) + ReLU
 * of models-checkpoint.py:52-53): per pixel (NHWC) its 32 channels' high f16 plane then their low
 * plane, h1 * 2^E = hi + lo (128 B per pixel, the size of the f32 form), E derived by
 * ppox_nature_pack_all (b1 required with q1) from the bound |h1| <= 255 max_c (sum |W1[c]| + |b1[c]|)
 * and kept in q1's tail, so the producer splits its output in its epilogue and the consumers read
 * the planes as they lie (no amax pass, no split in the consumers).
 *   conv1_fwd_planes:  as ppox_nature_conv_fwd_split(1, ...) writing h1p (batch x 400 x 64 uint16)
 *   conv2_fwd_planes:  as ppox_nature_conv_fwd_split(2, ...) reading h1p (q1: its exponent)
 *   conv2_wgrad_planes: dW2 [64][32][4][4] and db2 of Conv2d(32, 64, 4, 2) from h1p and the output
 *                      grad g2 (NHWC f32, amax_g its slots): one workgroup per CU over whole samples
 *                      (the direct form: the H1P image and the G rows of a sample in LDS, no
 *                      im2col), slabs in the workspace (ppox_nature_conv2_wgrad_planes_workspace_bytes)
 *                      summed in a fixed order.  Replaces the Conv2d weight / bias autograd of
 *                      models-checkpoint.py:54 in the training backward of ppo.py:241. */
/* PX (round 4): the H1P form generalised to the trunk's other split operands.  An f32 tensor of
 * NHWC rows is stored in the same bytes as, per aligned run of 32 elements, the 32 high f16 then
 * the 32 low f16 of its values times 2^E (element e's halves at uint16 2 (e & ~31) + (e & 31) and
 * + 32).  A producer writes its output this way (y_exp_out / g3_exp_out non-null: E from the bound
 * amax(input) * max column l1-norm of its weights + max |bias|, stored to that int) and its
 * consumers read the planes as they lie (x_exp / g_exp / h3_exp: the int holding E):
 *   h2 — conv2 forward (conv2_fwd_planes, y_exp_out; amax_x = h1's slots) -> conv3 forward
 *        (conv_fwd_split(3, x_exp)) and conv3 weight gradient (conv_wgrad_split(3, x_exp));
 *   h3 — conv3 forward (conv_fwd_split(3, y_exp_out)) -> fc forward (fc_fwd[_splitk], h3_exp) and
 *        fc weight gradient (fc_wgrad, h3_exp);
 *   g3 — fc dgrad (fc_dgrad, g3_exp_out; relu_bits required) -> conv3 dgrad
 *        (conv_dgrad_split(3, g_exp); relu_bits required) and conv3 weight gradient (g_exp);
 *   g2 — conv3 dgrad (conv_dgrad_split(3, y_exp_out), round 5) -> conv2 dgrad (conv_dgrad_split(2,
 *        g_exp): the direct form) and conv2 weight gradient (conv2_wgrad_planes(g_exp)).
 * Null exponents select the f32 operands.  conv1_fwd_planes records h1's amax into amax_y
 * (nullable): the start of h2's bound. */
int ppox_nature_conv1_fwd_planes(const void* x, int64_t batch, const int64_t* idx, int64_t T, int64_t N_env,
                                 int64_t x_sample_stride, const uint16_t* wq1, const float* bias, uint16_t* h1p,
                                 uint32_t* amax_y, uint32_t* relu_bits, void* stream);
int ppox_nature_conv2_fwd_planes(const uint16_t* h1p, const uint16_t* q1, int64_t batch, const uint16_t* wq2,
                                 const float* bias, float* y, const uint32_t* amax_x, uint32_t* amax_y,
                                 uint32_t* relu_bits, int* y_exp_out, void* stream);
int64_t ppox_nature_conv2_wgrad_planes_workspace_bytes(int64_t batch);
int ppox_nature_conv2_wgrad_planes(const uint16_t* h1p, const uint16_t* q1, int64_t batch, const float* grad_out,
                                   void* workspace, int64_t workspace_bytes, float* dw, float* db,
                                   const uint32_t* amax_g, const int* g_exp, void* stream);
/* The heads' hidden layer Linear(512, 512) + ReLU (models-checkpoint.py:62-66 extra_layer; the
 * forward of forward() / evaluate and its autograd in ppo.py:216-238) on the split-f16 GEMM, with
 * wh (512 x 512) packed by ppox_nature_pack_all into qh_fwd / qh_dgrad of
 * ppox_head_hidden_pack_elems() uint16 each.
 *   fwd:   e = relu(f wh^T + b)                         (amax_f: f's slots, required)
 *   dgrad: df = (f > 0) ? df + de wh : 0, in place       (df holds the heads' other input grads;
 *          the ReLU backward of the fc layer fused; amax_df: df's slots to record, nullable)
 *   wgrad: dw (512 x 512) = de^T f, split-K slabs in the workspace
 *          (ppox_head_hidden_wgrad_workspace_bytes(rows)) summed in a fixed order; rows 0 writes
 *          a zero gradient. */
int64_t ppox_head_hidden_pack_elems(void);
int ppox_head_hidden_fwd(const float* f, int64_t rows, const uint16_t* q_fwd, const float* bias, float* e,
                         const uint32_t* amax_f, void* stream);
/* fwd split over K for small batches (as ppox_nature_fc_fwd_splitk; workspace
 * ppox_head_hidden_fwd_splitk_workspace_bytes(rows)); with value != NULL the reduce also runs the
 * critic head Linear(512, 1) on each finished row (models-checkpoint.py:72, 85 critic_ext):
 * value = e w_critic^T + b_critic, bitwise as ppox_skinny_linear. */
int64_t ppox_head_hidden_fwd_splitk_workspace_bytes(int64_t rows);
int ppox_head_hidden_fwd_splitk(const float* f, int64_t rows, const uint16_t* q_fwd, const float* bias,
                                void* workspace, int64_t workspace_bytes, float* e, const uint32_t* amax_f,
                                const float* w_critic, const float* b_critic, float* value, void* stream);
int ppox_head_hidden_dgrad(const float* de, int64_t rows, const uint16_t* q_dgrad, const float* f, float* df,
                           const uint32_t* amax_de, uint32_t* amax_df, void* stream);
/* The heads' backward to the fc output in one launch (round 5; replaces ppox_head_dgrad_outer +
 * ppox_head_hidden_dgrad for a net without the intrinsic head): de = (e > 0) dv w_critic (bitwise
 * ppox_head_dgrad_outer's de) and df = (f > 0) (dout w_actor + de W) with W the hidden layer
 * (q_dgrad: its ppox_nature_pack_all dgrad form), f32 (rows x 512); both amax recorded.  w_actor, e, f,
 * df, de and q_dgrad 16-B aligned; w_critic any float alignment (its offset in the flat parameter
 * buffer follows the action count).  Reference:
 * models-checkpoint.py:72, 80-85 (actor, extra_layer, critic_ext) backward, ppo.py:241. */
int ppox_head_backward(const float* dout, const float* w_actor, const float* dv, const float* w_critic, const float* e,
                       const float* f, const uint16_t* q_dgrad, int64_t rows, int64_t h, int64_t n_out, float* df,
                       float* de, uint32_t* amax_de, uint32_t* amax_df, void* stream);
int64_t ppox_head_hidden_wgrad_workspace_bytes(int64_t rows);
int ppox_head_hidden_wgrad(const float* de, int64_t rows, const float* f, void* workspace, int64_t workspace_bytes,
                           float* dw, const uint32_t* amax_de, const uint32_t* amax_f, void* stream);
int ppox_nature_fc_pack(const float* w, uint16_t* q_fwd, uint16_t* q_dgrad, void* stream);
int ppox_nature_fc_fwd(const float* h3, int64_t batch, const uint16_t* q_fwd, const float* bias, float* f,
                       const uint32_t* amax_h3, uint32_t* amax_f, const int* h3_exp, void* stream);
/* df_exp (nullable): df is given as PX planes (ppox_px_split) with that exponent; amax_df stays
 * required (the PX g3 bound) */
int ppox_nature_fc_dgrad(const float* df, int64_t batch, const uint16_t* q_dgrad, const float* h3, float* g3,
                         const uint32_t* amax_df, uint32_t* amax_g3, const uint32_t* relu_bits, int* g3_exp_out,
                         const int* df_exp, void* stream);
/* fc forward (as ppox_nature_fc_fwd) split over K for small batches: 2-8 K-ranges per (128-row
 * tile, 64-column block) so the grid fills the chip, partial products into the workspace
 * (ppox_nature_fc_fwd_splitk_workspace_bytes(batch)), then one fixed-order reduce adding the
 * partials, the bias and the ReLU.  Replaces the same site (models-checkpoint.py:58-59).  With
 * logits != NULL the reduce also runs the actor head Linear(512, n_actions) on each finished row
 * (n_actions 1..8, w_actor 16B-aligned; models-checkpoint.py:60-61): logits = f w_actor^T + b_actor,
 * bitwise as ppox_skinny_linear. */
int64_t ppox_nature_fc_fwd_splitk_workspace_bytes(int64_t batch);
int ppox_nature_fc_fwd_splitk(const float* h3, int64_t batch, const uint16_t* q_fwd, const float* bias,
                              void* workspace, int64_t workspace_bytes, float* f, const uint32_t* amax_h3,
                              uint32_t* amax_f, const float* w_actor, const float* b_actor, int32_t n_actions,
                              float* logits, const int* h3_exp, void* stream);
/* fc weight gradient dW (512 x 3136, the weight's Flatten order) = df^T @ h3 over the batch,
 * split-f16 (fp32-class; amax_df, amax_h3: the operands' slots), deterministic: df (batch, 512) is dL/df already ReLU-masked, h3 the
 * NHWC (batch, 7, 7, 64) conv3 output of the split forward.  Replaces the library GEMM of
 * torch.nn.Linear's backward (reference: models-checkpoint.py:58-59 trained by ppo.py:236-238).
 * batch 0 writes a zero gradient.  workspace: ppox_nature_fc_wgrad_workspace_bytes(batch).  h3_exp /
 * df_exp (nullable): that operand is given as PX planes with that exponent (its amax then unused). */
int64_t ppox_nature_fc_wgrad_workspace_bytes(int64_t batch);
int ppox_nature_fc_wgrad(const float* df, int64_t batch, const float* h3, void* workspace,
                         int64_t workspace_bytes, float* dw, const uint32_t* amax_df, const uint32_t* amax_h3,
                         const int* h3_exp, const int* df_exp, void* stream);
/* PX planes of an f32 tensor x (n % 32 == 0, as laid out in memory) whose amax slots are recorded:
 * y (n int16 = the same bytes) = its two f16 planes at E = the split scale of amax (what a split
 * GEMM takes for x as an f32 operand); *exp_out = E.  The fc layer's df for the fc dgrad and weight
 * gradient, which otherwise split it in registers once per tile (round 4). */
int ppox_px_split(const float* x, int64_t n, const uint32_t* amax, uint16_t* y, int* exp_out, void* stream);

/* ES-NSRA (evolution_strategies.py:103-384, csrc/es.hip), float64 throughout.
 * ppox_es_noise: eps[p][j] ~ N(0,1) for members member0..member0+P-1 of a generation
 *   (the population draw of :167-177; Philox, shard-invariant).
 * ppox_es_env_noise: the synthetic env's shared noise table xi[T][D].
 * ppox_es_evaluate: episode return of each perturbed policy w + sigma*eps[p] (eps null:
 *   w itself, P = 1) — :147-195 evaluate/_get_rewards with the arctan MLP of :50-63 (two
 *   hidden layers <= 64, D <= 32, A <= 8, Box/tanh head); bc (nullable, P x 2): final
 *   state[0:2] (get_behavior_char :248-271).
 * ppox_es_update: out[j] = sum_p coef[p] * eps[p][j], fixed order (the P^T r of :237-242). */
int ppox_es_noise(int64_t P, int64_t n_params, int64_t member0, int64_t generation, uint64_t seed,
                  double* eps, void* stream);
int ppox_es_env_noise(int32_t T, int32_t D, uint64_t env_seed, double* xi, void* stream);
int ppox_es_evaluate(const double* w, const double* eps, double sigma, int64_t P, int32_t D, int32_t H1,
                     int32_t H2, int32_t A, int32_t T, uint64_t env_seed, const double* xi,
                     double* fitness, double* bc, void* stream);
int64_t ppox_es_update_workspace_bytes(int64_t P, int64_t n_params);
int ppox_es_update(const double* eps, const double* coef, int64_t P, int64_t n_params,
                   double* workspace, int64_t workspace_bytes, double* out, void* stream);

/* NatureCNN head backward (explicit training backward of CnnActorCritic, replacing the
 * autograd of nn.ReLU / Linear(H, 1) at .ipynb_checkpoints/models-checkpoint.py:60-87):
 * grad = act > 0 ? grad : 0 in place (n % 4 == 0); out[b][j] = dv[b] * w[j] * (act[b][j] > 0)
 * (amax: out's split-f16 amax slots to record, nullable). */
int ppox_relu_backward_(float* grad, const float* act, int64_t n, void* stream);
/* as ppox_relu_backward_, also recording max |grad| into amax (split-f16 slots, below): the fc
 * output grad df that the split fc dgrad / weight gradient take as an operand */
int ppox_relu_backward_amax_(float* grad, const float* act, int64_t n, uint32_t* amax, void* stream);
/* Column-reduction gradients of the NatureCNN heads (models-checkpoint.py:60-87; the
 * explicit backward of models.CnnActorCritic) in one pass over f, e, de, df (rows x h):
 * w_actor (A x h) = dout^T f, b_actor = sum dout, w_critic (h) = dv^T e, b_critic = sum dv,
 * b_extra = sum de, b_fc = sum df; with ie != NULL also the intrinsic head's
 * w_critic_int = div^T ie, b_critic_int = sum div, b_int_extra = sum die.  Outputs are
 * overwritten.  h <= 512, A <= 18.  Workspace: ppox_head_grads_workspace_bytes.  relu_df != 0:
 * df is first masked by the fc layer's ReLU, df = f > 0 ? df : 0, IN PLACE (the nn.ReLU backward
 * of models-checkpoint.py:57, fused), its max |df| recorded into amax_df (nullable).  df_planes
 * (nullable, relu_df == 0, h % 32 == 0; round 6): df's PX planes written in the same pass, bitwise
 * ppox_px_split(df, df_planes_amax, df_planes, df_planes_exp) — the fc dgrad / weight gradient's
 * operand without a pass of its own. */
int64_t ppox_head_grads_workspace_bytes(int64_t rows, int64_t h, int64_t n_actions, int32_t intrinsic);
int ppox_head_grads(const float* f, const float* e, const float* dout, const float* dv, const float* de,
                    const float* df, const float* ie, const float* div, const float* die, int64_t rows, int64_t h,
                    int64_t n_actions, void* workspace, float* w_actor, float* b_actor, float* w_critic,
                    float* b_critic, float* b_extra, float* b_fc, float* w_critic_int, float* b_critic_int,
                    float* b_int_extra, int32_t relu_df, uint32_t* amax_df, uint16_t* df_planes,
                    const uint32_t* df_planes_amax, int32_t* df_planes_exp, void* stream);
/* Skinny heads (models-checkpoint.py:60-87 actor / critic Linear layers, n_out <= 8):
 * ppox_skinny_linear: y (rows x n_out) = x (rows x h) w^T + bias, one wave per row;
 * ppox_skinny_dgrad:  d (rows x h) = g (rows x n_out) w (n_out x h) — overwritten. */
int ppox_skinny_linear(const float* x, const float* w, const float* bias, int64_t rows, int64_t h, int64_t n_out,
                       float* y, void* stream);
int ppox_skinny_dgrad(const float* g, const float* w, int64_t rows, int64_t h, int64_t n_out, float* d,
                      void* stream);
int ppox_outer_relu_backward(const float* dv, const float* w, const float* act, int64_t rows, int64_t h,
                             float* out, uint32_t* amax, void* stream);
/* ppox_skinny_dgrad (df = dout w_actor) and ppox_outer_relu_backward (de = dv w_critic (e > 0), amax_de
 * nullable) of the first head in one launch, bitwise the same results (models-checkpoint.py:60-87). */
int ppox_head_dgrad_outer(const float* dout, const float* w_actor, const float* dv, const float* w_critic,
                          const float* e, int64_t rows, int64_t h, int64_t n_out, float* df, float* de,
                          uint32_t* amax_de, void* stream);

/* ---------------------------------------------------------------------------
 * K6, split-f16 forms (csrc/conv_split.hip, csrc/conv.hip): the same ops, layouts and
 * fused epilogues as above, on the f16 matrix cores (v_mfma_f32_32x32x16_f16).  Every f32
 * operand x is scaled by a power of two 2^E per tensor (max|x| 2^E in [2^14, 2^15)) and split
 * by round-to-nearest into two fp16 planes, x 2^E = h + l + r with |r| <= 2^-24 |x 2^E|; a
 * product keeps the three terms hA hB + hA lB + lA hB (the dropped lA lB <= 2^-22 |ab|), large
 * and small terms accumulated separately in f32, and the result is unscaled exactly.  The
 * uint8 frames of layer 1 are exact in one plane (two products).  Accuracy: fp32-class (error
 * vs fp64 at or below the f32-MFMA kernels', tests/test_kernels_gpu.py).
 *
 * Operand scales.  A tensor's "amax slots" are ppox_amax_slots() uint32 (16-B aligned) holding
 * the f32 bits of max |x| spread over the slots (the consumer takes their maximum).  The caller
 * zeroes them before the tensor is produced; the kernels that produce an operand of a later
 * split GEMM record into the slots passed as amax_y / amax_out (nullable: not recorded), and
 * ppox_amax records any other tensor's (n % 4 == 0).  Weights carry their own scale: the
 * packers write it after the planes of ppox_nature_split_pack_elems(which) elements (which =
 * 1, 2, 3: forward weights of that layer; 12, 13: dgrad weights of conv2 / conv3).
 * Replaces the same reference sites as the f32 forms.  One layout difference: the split
 * conv3 forward writes its output NHWC, y (batch, 7, 7, 64) — feature p * 64 + c instead
 * of the reference's Flatten feature c * 49 + p — which the split fc layer above consumes
 * (its weights are packed through that permutation).
 * -------------------------------------------------------------------------*/
int32_t ppox_amax_slots(void);
int ppox_amax(const float* x, int64_t n, uint32_t* amax, void* stream);
int64_t ppox_nature_split_pack_elems(int32_t which);
int ppox_nature_pack_split(const float* w1, const float* w2, const float* w3, uint16_t* q1,
                           uint16_t* q2, uint16_t* q3, uint16_t* qd2, uint16_t* qd3, void* stream);
/* amax_x: slots of x (layers 2, 3; null for layer 1's frames); amax_y: y's slots (nullable);
 * relu_bits (nullable): y's ReLU bitmask, bit c % 32 of uint32 word p * (C / 32) + c / 32 set iff
 * channel c of output pixel p (n * P + oy * OW + ox) is > 0 — batch * P * C / 32 words (8-B
 * aligned), read by the next layer's split dgrad (conv1's by conv2's, conv2's by conv3's) and, for
 * conv3, by the fc dgrad */
int ppox_nature_conv_fwd_split(int32_t layer, const void* x, int64_t batch, const int64_t* idx,
                               int64_t T, int64_t N_env, int64_t x_sample_stride,
                               const uint16_t* wq, const float* bias, float* y, const uint32_t* amax_x,
                               uint32_t* amax_y, uint32_t* relu_bits, const int* x_exp, int* y_exp_out,
                               void* stream);
/* dgrad (as ppox_nature_conv_dgrad) of conv2/conv3 with split weights (which = 12, 13);
 * amax_g: grad_out's slots, amax_out: grad_in's (nullable).  The ReLU mask of the layer below
 * comes from relu_bits (that layer's split forward's bitmask) when non-null, else from prev_act.
 * PX (round 5): layer 3 with y_exp_out writes g2 as its planes (E from amax(g3) x the dgrad
 * matrix's column norms, which ppox_nature_pack_all records for wqd; relu_bits required); layer 2
 * with g_exp reads those planes and runs the direct class-wise form (models-checkpoint.py:55
 * backward: per input-pixel parity class an implicit GEMM over its 4 taps x 64 channels; relu_bits
 * = conv1's bitmask required, grad_in f32). */
int ppox_nature_conv_dgrad_split(int32_t layer, const float* grad_out, int64_t batch,
                                 const uint16_t* wqd, const float* prev_act, float* grad_in,
                                 const uint32_t* amax_g, uint32_t* amax_out, const uint32_t* relu_bits,
                                 const int* g_exp, int* y_exp_out, void* stream);
/* dW [co][ci][ky][kx] and db (as ppox_nature_conv_wgrad + ppox_nature_wgrad_reduce, in one
 * call): split-K slabs into a workspace of ppox_nature_wgrad_split_workspace_bytes(layer,
 * batch), reduced in a fixed order (deterministic).  x: u8 frames (layer 1, samples
 * x_sample_stride bytes apart; amax_x null) or NHWC f32; grad_out: ReLU-masked NHWC output
 * grad (amax_g its slots). */
int64_t ppox_nature_wgrad_split_workspace_bytes(int32_t layer, int64_t batch);
int ppox_nature_conv_wgrad_split(int32_t layer, const void* x, int64_t batch,
                                 int64_t x_sample_stride, const float* grad_out, void* workspace,
                                 int64_t workspace_bytes, float* dw, float* db, const uint32_t* amax_x,
                                 const uint32_t* amax_g, const int* x_exp, const int* g_exp, void* stream);

/* conv1 split wgrad with the minibatch gather fused: sample n is env-major row idx[n]
 * (i = env * T + step) of the step-major (T, N_env, 4, 84, 84) uint8 rollout frames x.
 * Replaces ppox_gather_rows + ppox_nature_conv_wgrad_split(1, ...) on the minibatch
 * observations of buffer.py:97-109 / models-checkpoint.py:52-58 (Conv2d(4, 32, 8, 4) backward). */
int ppox_nature_conv_wgrad_split_idx(int32_t layer, const void* x, int64_t batch, const int64_t* idx,
                                     int64_t T, int64_t N_env, const float* grad_out, void* workspace,
                                     int64_t workspace_bytes, float* dw, float* db, const uint32_t* amax_g,
                                     void* stream);

/* ---------------------------------------------------------------------------
 * K11 ICM on image observations (csrc/icm.hip): the IntrinsicCuriosityModule of
 * models.py:270-320 with uint8 frame-stack rows of K bytes (K % 32 == 0), Discrete actions
 * (n_actions <= 32, int32) and feature size 32.  Replaces the torch Linear / LeakyReLU /
 * Embedding / cross_entropy / mse_loss forward + autograd of ppo.py:629-630 (collect) and
 * ppo.py:684-699 (train).  "seg" is the ICM's parameter segment after state_encoder[0].weight:
 * b1, W2, b2 (state_encoder), Wf1, bf1, Wf2, bf2 (forward_model), Wi1, bi1, Wi2, bi2
 * (inverse_model), Wae (action_encoder) contiguous in that (module) order,
 * ppox_icm_param_elems(n_actions) floats; the gradient segment has the same layout.
 * The encoder's Linear(K, 32) runs split-bf16 (fp32-class, as K6); everything deterministic.
 *   ppox_icm_pack_w1:    W1 (32 x K f32, K % 64 == 0) -> ppox_icm_w1_pack_elems(K) uint16: its two
 *                        f16 planes (row n times 2^E[n]) in the forward's fragment order, then E[32].
 *   ppox_icm_encode:     pre1 = x W1^T + b1, phi = leaky(pre1) W2^T + b2 for `rows` frame rows
 *                        (idx != NULL: env-major rollout rows of the step-major (T, N_env, ...)
 *                        frames, as ppox_nature_conv_fwd_split); rowno (nullable, uint32 per
 *                        row) = the frame row read.  workspace: ppox_icm_encode_workspace_bytes.
 *   ppox_icm_pair_backward: pairs (row j, row j + 1) of a minibatch of B rows with features
 *                        phi (B x 32): the inverse / forward models, both losses (means over
 *                        n_pairs_global pairs, weights 1 - beta / beta) and their backward.
 *                        actions of row j: actions[rowno ? rowno[j] : j] (actions NULL, with a
 *                        pair list: the B floats after phi, ppox_icm_scatter_positions' layout).
 *                        pairs: the first rows of the evaluated pairs (NULL: all j < B - 1, n_pairs
 *                        = B - 1; a listed B - 1 has no pair and is skipped, n_pairs <= B).
 *                        dS[j] / dN[j + 1] (B x 32) = dL/dphi through a pair's first / second
 *                        row (with pairs == NULL every row of both is written; with a list, dS
 *                        and dN are zeroed first).  partials: ppox_icm_partials_bytes(rows, n_actions).
 *   ppox_icm_scatter_positions: world > 1 — this rank's `rows` features phi (rows x 32) and actions
 *                        (actions[rowno[i]]) at their minibatch positions pos[i] of
 *                        fa = [B x 32 | B actions as f32], zero elsewhere (for one all-reduce).
 *   ppox_icm_row_backward: dphi = dS + dN (dN nullable) of minibatch row pos[i] (pos nullable)
 *                        -> g1 = dL/dpre1 in fragment order (f32) + per-column max |g1| of each
 *                        32-row block (ppox_icm_g1_pack_elems(rows) uint16)
 *                        + partials of db1, dW2, db2.
 *   ppox_icm_grad_reduce: partials -> grad_seg (overwritten) and, loss_accum != NULL,
 *                        loss_accum[0] += this call's share of (1 - beta) CE + beta MSE.
 *   ppox_icm_enc_wgrad:  dW1 (32 x K, overwritten) = g1^T x over the rows read by encode.
 *   ppox_icm_int_reward: collect: int_rewards = clamp(mean((forward_model(phi_s, a) - phi_n)^2),
 *                        -5, 5), rewards = (1 - eta) rewards + eta int_rewards (in place). */
int64_t ppox_icm_param_elems(int32_t n_actions);
int64_t ppox_icm_w1_pack_elems(int64_t K);
int ppox_icm_pack_w1(const float* w1, int64_t K, uint16_t* q, void* stream);
int64_t ppox_icm_encode_workspace_bytes(int64_t rows, int64_t K);
int ppox_icm_encode(const void* x, int64_t rows, const int64_t* idx, int64_t T, int64_t N_env, int64_t K,
                    const uint16_t* q, const float* seg, void* workspace, float* pre1, float* phi, uint32_t* rowno,
                    void* stream);
int64_t ppox_icm_partials_bytes(int64_t rows, int32_t n_actions);
int64_t ppox_icm_g1_pack_elems(int64_t rows);
int ppox_icm_pair_backward(const float* phi, int64_t B, const int32_t* actions, const uint32_t* rowno,
                           const int64_t* pairs, int64_t n_pairs, int64_t n_pairs_global, int32_t n_actions,
                           float beta, const float* seg, float* dS, float* dN, float* partials, void* stream);
int ppox_icm_scatter_positions(const float* phi, const int32_t* actions, const uint32_t* rowno, const int64_t* pos,
                               int64_t rows, int64_t B, float* fa, void* stream);
int ppox_icm_row_backward(const float* dS, const float* dN, const int64_t* pos, int64_t rows, const float* pre1,
                          const float* seg, int32_t n_actions, uint16_t* g1q, float* partials, void* stream);
int ppox_icm_grad_reduce(const float* partials, int64_t rows, int64_t n_pairs, int32_t n_actions, float beta,
                         int64_t n_pairs_global, float* grad_seg, double* loss_accum, void* stream);
int ppox_icm_enc_wgrad(const void* x, const uint32_t* rowno, int64_t rows, int64_t K, const uint16_t* g1q,
                       float* dw1, void* stream);
int ppox_icm_int_reward(const float* phi_s, const float* phi_n, const int32_t* actions, int64_t N,
                        int32_t n_actions, const float* seg, float eta, float* rewards, float* int_rewards,
                        void* stream);

/* Data-parallel exchange (world > 1; replaces the per-minibatch torch.distributed all-reduces around the
 * sharded update, ppo.py:241-244 — the reference is single-process).  The one exception to "never
 * allocates": ppox_dp_comm_init creates the RCCL communicator, a stream and two events.
 *   ppox_dp_load:       resolve RCCL from the library at rccl_path (the one the process already loaded).
 *   ppox_dp_unique_id:  rank 0: the communicator id (ppox_dp_unique_id_bytes() bytes, host) every rank
 *                       then passes to ppox_dp_comm_init (a collective call).
 *   ppox_dp_all_reduce: in-place SUM of count elements (dtype 0 float32, 1 float64) on the communicator's
 *                       stream after the work already on `stream`; wait != 0: `stream` waits for it.
 *   ppox_dp_wait:       `stream` waits for every reduction issued so far. */
int ppox_dp_load(const char* rccl_path);
int ppox_dp_unique_id_bytes(void);
int ppox_dp_unique_id(uint8_t* id_host);
int ppox_dp_comm_init(const uint8_t* id_host, int32_t world, int32_t rank, int32_t device, void** comm_out);
int ppox_dp_comm_destroy(void* comm);
int ppox_dp_all_reduce(void* comm, void* buf, int64_t count, int32_t dtype, int32_t wait, void* stream);
int ppox_dp_wait(void* comm, void* stream);

/* Stream ordering for the backward's fork / join (the reference has one stream): an event created with
 * hipEventCreateWithFlags(flags | hipEventDisableTiming); ppox_stream_order records it on record_stream and
 * makes wait_stream wait for it. */
int ppox_event_create(uint32_t flags, void** event_out);
int ppox_event_destroy(void* event);
int ppox_stream_order(void* event, void* record_stream, void* wait_stream);

#ifdef __cplusplus
}
#endif
#endif /* PPOX_H */
