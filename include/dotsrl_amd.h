/*
 * dotsrl_amd.h — C-ABI of the MI355X (gfx950) PPO/GRPO actor-learner hot path.
 *
 * Drop-in boundary for the numeric core behind verl's DataParallelPPOActor / RayPPOTrainer
 * (rednote-hilab/dots.rl @ 2025-09-19, paths relative to that tree). Every entry point replaces one
 * reference interface (cited per function). Rules of the boundary:
 *   - plain pointers + sizes; all buffers are device memory allocated by the caller (PyTorch-ROCm
 *     storage in the Python host); the library never allocates, frees or synchronises;
 *   - `stream` is a hipStream_t (passed as void*); every call only enqueues work on it, so the
 *     calls are hipGraph-capturable;
 *   - return 0 on success, a negative DRL_ERR_* code otherwise; drl_last_error() describes the last
 *     failure on the calling thread. No C++ exception crosses the boundary.
 *   - tensors are row-major and contiguous unless a leading dimension (`ld*`) is given.
 */
#ifndef DOTSRL_AMD_H_
#define DOTSRL_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: drl_ppo_loss_params gained policy_loss, cov_ratio, clip_cov_lb, clip_cov_ub, ppo_kl_coef, cov_seed (a caller
 * built against version 2 passes a shorter struct); drl_gemm (operand layouts, fp32 epilogues, stream-K) */
#define DRL_ABI_VERSION 8

/* ld_vt value selecting the key-blocked V^T cache layout (B, Hkv, ceil(cap / 32), D, 32) wherever a V^T
 * operand with a leading dimension ld_vt is taken (flash / decode attention, the rope and decode-projection
 * cache writers): element (d, key) of a (sequence, KV head) panel sits at (key / 32) * 32 * D + d * 32 +
 * key % 32, and cap is the K capacity of the same call (ld_k or Tk). */
#define DRL_VT_BLOCKED (-32)

#define DRL_OK 0
#define DRL_ERR_INVALID (-1)     /* bad argument (shape, dtype, null pointer, alignment) */
#define DRL_ERR_HIP (-2)         /* a HIP runtime call failed */
#define DRL_ERR_UNSUPPORTED (-3) /* valid request this build does not implement */
#define DRL_ERR_WORKSPACE (-4)   /* workspace too small */

typedef enum drl_dtype {
  DRL_I64 = 0,
  DRL_I32 = 1,
  DRL_U8 = 2, /* also torch.bool */
  DRL_F32 = 3,
  DRL_BF16 = 4,
} drl_dtype;

/* loss_agg_mode of core_algos.agg_loss (verl/trainer/ppo/core_algos.py:703-736) */
typedef enum drl_agg_mode {
  DRL_AGG_TOKEN_MEAN = 0,
  DRL_AGG_SEQ_MEAN_TOKEN_SUM = 1,
  DRL_AGG_SEQ_MEAN_TOKEN_MEAN = 2,
  DRL_AGG_SEQ_MEAN_TOKEN_SUM_NORM = 3,
} drl_agg_mode;

/* kl_penalty types (verl/trainer/ppo/core_algos.py:1272-1307) */
typedef enum drl_kl_type {
  DRL_KL_NONE = -1, /* use_kl_loss = False */
  DRL_KL_K1 = 0,    /* "kl" / "k1" */
  DRL_KL_ABS = 1,   /* "abs" */
  DRL_KL_K2 = 2,    /* "mse" / "k2" */
  DRL_KL_K3 = 3,    /* "low_var_kl" / "k3" */
} drl_kl_type;


const char* drl_last_error(void);
int drl_abi_version(void);
/* Number of compute units of the current device (grid sizing); <0 on error. */
int drl_device_cu_count(void);

/* ------------------------------------------------------------------------------------------------
 * K1 — fused per-micro-batch actor loss, forward + backward in ONE launch.
 * Replaces the eager chain of DataParallelPPOActor.update_policy (verl/workers/actor/dp_actor.py:419-466):
 *   compute_policy_loss_vanilla (core_algos.py:815-889) + agg_loss(entropy) + kl_penalty + agg_loss(kld)
 *   + `loss * loss_scale_factor` + loss.backward() down to d loss / d log_prob and d loss / d entropy.
 * Inputs (B, R) float32, response_mask (B, R) of `mask_dtype` (I64/I32/U8/F32).
 * entropy may be NULL (entropy_coeff must then be 0); ref_log_prob may be NULL (kl_type must be NONE).
 * out_scalars: device float[DRL_PPO_OUT_N], see the enum. dlog_prob / dentropy may be NULL.
 * workspace: drl_ppo_loss_workspace_bytes(B, R) bytes whose first 256 bytes are ZERO before the first call
 * (hipMemset once at allocation); every call leaves them zero again, so a workspace reused by calls on one
 * stream needs no per-call memset. Use it for K1 only (drl_agg_loss keeps its own).
 * ---------------------------------------------------------------------------------------------- */
typedef struct drl_ppo_loss_params {
  float clip_ratio_low;    /* actor.clip_ratio_low (defaults to clip_ratio) */
  float clip_ratio_high;   /* actor.clip_ratio_high */
  float clip_ratio_c;      /* actor.clip_ratio_c (dual clip, > 1) */
  float entropy_coeff;     /* actor.entropy_coeff; 0 = term absent (dp_actor.py:441-447) */
  float kl_loss_coef;      /* actor.kl_loss_coef */
  float loss_scale_factor; /* 1 / gradient_accumulation (dp_actor.py:415-417) */
  int32_t loss_agg_mode;   /* drl_agg_mode */
  int32_t kl_type;         /* drl_kl_type; NONE = use_kl_loss False */
  /* optional, token-mean only: device double = sum(response_mask) of this call's tokens (e.g. the per-row
   * counts the rollout's response-mask step already has, summed over the micro-batch). When given, K1
   * runs as ONE pass (the mask is read once, in the loss pass) instead of the count pass + loss pass.
   * NULL = K1 counts the mask itself. */
  const double* token_count;
  /* policy loss (actor.policy_loss.loss_mode, get_policy_loss_fn core_algos.py:68-83): DRL_POLICY_VANILLA =
   * compute_policy_loss_vanilla (PPO clip + dual clip, :815-889), DRL_POLICY_GPG = compute_policy_loss_gpg
   * (pg = -log_prob * advantages, :957-975; clipfrac / ppo_kl / clipfrac_lower reported as 0),
   * DRL_POLICY_GSPO = compute_policy_loss_gspo (:892-954: the row's mean log-ratio as every token's ratio, clamped
   * at 10, PPO clip without dual clip, pg aggregated seq-mean-token-mean whatever loss_agg_mode is;
   * pg_clipfrac_lower 0), DRL_POLICY_GEO_MEAN = compute_policy_loss_geo_mean (:1143-1210, GMPO: log-ratios clipped
   * to [-clip_ratio_low, clip_ratio_high] toward sign(A), geometric-mean ratio and mean advantage per row, pg =
   * mean over rows). The two sequence-level losses run as three small launches (per-row sums, per-token terms,
   * row fold) instead of K1's stream, and ignore token_count and clip_ratio_c.
   * DRL_POLICY_CLIP_COV = compute_policy_loss_clip_cov (:978-1069) and DRL_POLICY_KL_COV = compute_policy_loss_kl_cov
   * (:1072-1140): token covariances (A - mean A)(log_prob - mean log_prob) over the micro-batch select tokens by a
   * one-workgroup radix select — kl_cov: the max(1, int(n_valid * cov_ratio)) largest (lowest flat index first
   * among equal values) get -A r + ppo_kl_coef |log_prob - old| (ratio r = exp(log_prob - old), unclamped);
   * clip_cov: of the valid, not already clipped tokens with clip_cov_lb < cov < clip_cov_ub, min(max(1,
   * int(cov_ratio * sum(mask))), #candidates) get their clipped loss zeroed — the reference draws that subset with
   * torch.randperm, here the candidates with the smallest fmix32(flat index ^ seed) (a uniformly random subset on
   * cov_seed; every candidate when they fit). */
  int32_t policy_loss;
  float cov_ratio;    /* policy_loss.clip_cov_ratio / kl_cov_ratio */
  float clip_cov_lb;  /* policy_loss.clip_cov_lb */
  float clip_cov_ub;  /* policy_loss.clip_cov_ub */
  float ppo_kl_coef;  /* policy_loss.ppo_kl_coef */
  uint64_t cov_seed;  /* clip_cov's subset draw */
} drl_ppo_loss_params;

enum { DRL_POLICY_VANILLA = 0, DRL_POLICY_GPG = 1, DRL_POLICY_GSPO = 2, DRL_POLICY_GEO_MEAN = 3, DRL_POLICY_CLIP_COV = 4,
       DRL_POLICY_KL_COV = 5 };

enum {
  DRL_PPO_OUT_PG_LOSS = 0,
  DRL_PPO_OUT_PG_CLIPFRAC = 1,
  DRL_PPO_OUT_PPO_KL = 2,
  DRL_PPO_OUT_PG_CLIPFRAC_LOWER = 3,
  DRL_PPO_OUT_ENTROPY_LOSS = 4, /* agg_loss(entropy) when entropy != NULL, else 0 */
  DRL_PPO_OUT_KL_LOSS = 5,      /* agg_loss(kld) when kl_type != NONE, else 0 */
  DRL_PPO_OUT_LOSS = 6,         /* (pg - c_ent*ent + c_kl*kl) * loss_scale_factor — the value backpropagated */
  DRL_PPO_OUT_MASK_COUNT = 7,   /* sum(response_mask) */
  DRL_PPO_OUT_N = 8
};

size_t drl_ppo_loss_workspace_bytes(int64_t B, int64_t R);
int drl_ppo_loss_fwd_bwd(const float* old_log_prob, const float* log_prob, const float* advantages,
                         const void* response_mask, int32_t mask_dtype, const float* entropy,
                         const float* ref_log_prob, int64_t B, int64_t R, const drl_ppo_loss_params* params,
                         float* out_scalars, float* dlog_prob, float* dentropy, void* workspace,
                         size_t workspace_bytes, void* stream);

/* kl_penalty elementwise (core_algos.py:1272-1307): out[n] = kl(logprob[n], ref_logprob[n]). */
int drl_kl_penalty(const float* log_prob, const float* ref_log_prob, int64_t n, int32_t kl_type, float* out,
                   void* stream);

/* agg_loss forward (core_algos.py:703-736), used for the driver-side entropy metric
 * (ray_trainer.py:1215). out: device float[1]. */
size_t drl_agg_loss_workspace_bytes(int64_t B, int64_t R);
int drl_agg_loss(const float* loss_mat, const void* loss_mask, int32_t mask_dtype, int64_t B, int64_t R,
                 int32_t loss_agg_mode, float* out, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------
 * K2 — log-prob of labels and entropy over the vocabulary, from logits (one pass, online softmax).
 * Replaces logprobs_from_logits / entropy_from_logits (verl/utils/torch_functional.py:64-160) as called
 * from _forward_micro_batch (dp_actor.py:198-211, 263-272) after `logits.div_(temperature)`.
 * logits: (N, V) F32 or BF16 with row stride ld (elements). Math in float32; outputs float32
 * (the flash-attn cross-entropy semantics of torch_functional.py:81-100).
 * entropy / lse_out may be NULL. lse_out keeps logsumexp(logits/T) for the backward.
 * ---------------------------------------------------------------------------------------------- */
int drl_logprob_entropy_fwd(const void* logits, int32_t logits_dtype, int64_t N, int64_t V, int64_t ld,
                            const int64_t* labels, float temperature, float* log_prob, float* entropy,
                            float* lse_out, void* stream);
/* rollout.calculate_log_probs (vllm_rollout_spmd.py:350-395 `rollout_log_probs`; compared with the actor's
 * old_log_probs by ray_trainer.py:1221-1225 -> utils/debug/metrics.py:63-108): out[n * ld_out + c] =
 * log softmax(logits[n] / T)[tokens[n * ld_tok + c]] with c = *dev_step (0 when dev_step is NULL), the
 * temperature applied as drl_logprob_entropy_fwd applies it. One launch per decode step, graph-capturable. */
int drl_token_logprob(const void* logits, int32_t logits_dtype, int64_t N, int64_t V, int64_t ld, const int64_t* tokens,
                      int64_t ld_tok, const int64_t* dev_step, float temperature, float* out, int64_t ld_out,
                      void* stream);
/* d logits = (dlogp*(onehot - p) - dent*p*(log p + H)) / T   (experimental/torch_functional.py:40-72)
 * dlog_prob / dentropy may be NULL (treated as 0). dlogits (N, V) of dlogits_dtype (F32/BF16), row stride
 * ld_out; dlogits may alias logits (in-place backward, torch_functional.py:81 inplace_backward). */
int drl_logprob_entropy_bwd(const void* logits, int32_t logits_dtype, int64_t N, int64_t V, int64_t ld,
                            const int64_t* labels, float temperature, const float* dlog_prob,
                            const float* dentropy, const float* lse, const float* entropy, void* dlogits,
                            int32_t dlogits_dtype, int64_t ld_out, void* stream);

/* ------------------------------------------------------------------------------------------------
 * K3 — GRPO outcome advantage (core_algos.py:260-324), computed on device.
 * group_offsets[G+1] / group_members[B] is the CSR of uid -> rows in order of first appearance
 * (built on the host from DataProto.non_tensor_batch["uid"]). advantages/returns (B, R) float32.
 * ---------------------------------------------------------------------------------------------- */
size_t drl_grpo_workspace_bytes(int64_t B);
int drl_grpo_outcome_advantage(const float* token_level_rewards, const void* response_mask, int32_t mask_dtype,
                               const int32_t* row_group, const int32_t* group_offsets,
                               const int32_t* group_members, int64_t B, int64_t R, int64_t G, float epsilon,
                               int32_t norm_adv_by_std, float* advantages, float* returns, void* workspace,
                               size_t workspace_bytes, void* stream);

/* K3 generalised to the other group-outcome estimators (same CSR of uid groups):
 * DRL_ADV_RLOO = compute_rloo_outcome_advantage (core_algos.py:444-493),
 * DRL_ADV_REINFORCE_PP_BASELINE = compute_reinforce_plus_plus_baseline_outcome_advantage (core_algos.py:392-441:
 * group-mean baseline, then masked_whiten over the batch, times the mask; needs
 * drl_group_outcome_advantage_workspace_bytes(B)),
 * DRL_ADV_OPO = compute_opo_outcome_advantage (core_algos.py:495-546: length-weighted group baseline; needs the
 * workspace above for the response lengths),
 * DRL_ADV_GPG = compute_gpg_outcome_advantage (core_algos.py:624-684: alpha * (s - group mean), alpha = B / max(#nonzero
 * scores, 1), f_norm = 1),
 * DRL_ADV_GRPO_PASSK = compute_grpo_passk_outcome_advantage (core_algos.py:327-386: the best sample of a group gets
 * r_max - r_second_max, divided by std + epsilon when norm_adv_by_std; every group must have >= 2 samples).
 * epsilon / norm_adv_by_std apply to GRPO and GRPO_PASSK only. */
enum { DRL_ADV_GRPO = 0, DRL_ADV_RLOO = 1, DRL_ADV_REINFORCE_PP_BASELINE = 2, DRL_ADV_OPO = 3, DRL_ADV_GPG = 4,
       DRL_ADV_GRPO_PASSK = 5 };
size_t drl_group_outcome_advantage_workspace_bytes(int64_t B);
int drl_group_outcome_advantage(const float* token_level_rewards, const void* response_mask, int32_t mask_dtype,
                                const int32_t* row_group, const int32_t* group_offsets, const int32_t* group_members,
                                int64_t B, int64_t R, int64_t G, int32_t estimator, float epsilon,
                                int32_t norm_adv_by_std, float* advantages, float* returns, void* workspace,
                                size_t workspace_bytes, void* stream);

/* REINFORCE++ (core_algos.py:550-586): returns = masked discounted reward-to-go (a masked token resets the
 * carry), advantages = masked_whiten(returns) * mask. workspace: drl_gae_workspace_bytes(B, R). */
/* ReMax (core_algos.py:588-621): returns = reverse cumulative sum of rewards * mask along the response, advantages
 * = returns - reward_baselines[b] * mask; reward_baselines (B) float32 (the greedy baseline's scores). */
int drl_remax_advantage_return(const float* token_level_rewards, const float* reward_baselines, const void* response_mask,
                               int32_t mask_dtype, int64_t B, int64_t R, float* advantages, float* returns, void* stream);
int drl_reinforce_pp_advantage_return(const float* token_level_rewards, const void* response_mask, int32_t mask_dtype,
                                      int64_t B, int64_t R, float gamma, float* advantages, float* returns,
                                      void* workspace, size_t workspace_bytes, void* stream);

/* K5 — GAE + masked_whiten (core_algos.py:208-256, torch_functional.py:206-223). values (B, R) of
 * values_dtype: F32, or BF16 = the critic's autocast output as the reference stores it (then gamma * V(t+1)
 * is rounded to bf16 as the reference's bf16 tensor arithmetic does). */
size_t drl_gae_workspace_bytes(int64_t B, int64_t R);
int drl_gae_advantage_return(const float* token_level_rewards, const void* values, int32_t values_dtype,
                             const void* response_mask, int32_t mask_dtype, int64_t B, int64_t R, float gamma,
                             float lam, float* advantages, float* returns, void* workspace, size_t workspace_bytes,
                             void* stream);

/* ------------------------------------------------------------------------------------------------
 * K6 — critic: clipped value loss, forward + backward in one launch (after a row-count pre-pass).
 * Replaces compute_value_loss (verl/trainer/ppo/core_algos.py:1230-1269) + `vf_loss * loss_scale_factor`
 * + loss.backward() down to d loss / d vpreds (verl/workers/critic/dp_critic.py:218-245) and the
 * critic/vpred_mean metric (masked_mean, torch_functional.py:171-185).
 * vpreds / values (B, R) of value_dtype (F32, or BF16 = the reference critic's autocast output: the clip
 * bounds values -/+ cliprange are rounded to bf16 as the reference's bf16 tensor arithmetic does);
 * returns (B, R) float32; out_scalars device float[DRL_VALUE_OUT_N]; dvpreds (B, R) float32 or NULL.
 * ---------------------------------------------------------------------------------------------- */
typedef struct drl_value_loss_params {
  float cliprange_value;   /* critic.cliprange_value */
  float loss_scale_factor; /* 1 / gradient_accumulation (dp_critic.py:236-238) */
  int32_t loss_agg_mode;   /* drl_agg_mode (critic.loss_agg_mode) */
  int32_t pad;
} drl_value_loss_params;

enum {
  DRL_VALUE_OUT_VF_LOSS = 0,     /* 0.5 * agg_loss(max(vf_losses1, vf_losses2)) */
  DRL_VALUE_OUT_VF_CLIPFRAC = 1, /* masked_mean(vf_losses2 > vf_losses1) */
  DRL_VALUE_OUT_VPRED_MEAN = 2,  /* masked_mean(vpreds) */
  DRL_VALUE_OUT_LOSS = 3,        /* vf_loss * loss_scale_factor — the value backpropagated */
  DRL_VALUE_OUT_MASK_COUNT = 4,
  DRL_VALUE_OUT_N = 8
};

size_t drl_value_loss_workspace_bytes(int64_t B, int64_t R);
int drl_value_loss_fwd_bwd(const void* vpreds, const void* values, int32_t value_dtype, const float* returns,
                           const void* response_mask, int32_t mask_dtype, int64_t B, int64_t R,
                           const drl_value_loss_params* params, float* out_scalars, float* dvpreds, void* workspace,
                           size_t workspace_bytes, void* stream);

/* Critic value head (HF GenericForTokenClassification.score = Linear(H, 1, bias=True), the critic the
 * reference loads with AutoModelForTokenClassification, dp_critic.py:57-145): values[n] = hidden[n, :] . w
 * + b, fp32 accumulation, written as out_dtype (BF16 = the reference's autocast output). hidden (N, H)
 * row stride ld_h, weight (H) and bias (1, may be NULL) in `dt` (BF16 / F32). H % 8 (bf16) / 4 (fp32). */
int drl_value_head_fwd(const void* hidden, int64_t ld_h, const void* weight, const void* bias, int32_t dt, int64_t N,
                       int64_t H, void* values, int32_t out_dtype, void* stream);
/* Backward: dhidden[n, :] = dvalues[n] * w (in `dt`, may be NULL); dweight[k] += sum_n dvalues[n] hidden[n, k]
 * and dbias[0] += sum_n dvalues[n] (fp32 gradient buffers, accumulated in place; either may be NULL);
 * deterministic (fixed-order partials). workspace: drl_value_head_bwd_workspace_bytes(N, H) bytes. */
size_t drl_value_head_bwd_workspace_bytes(int64_t N, int64_t H);
int drl_value_head_bwd(const void* hidden, int64_t ld_h, const void* weight, int32_t dt, const float* dvalues,
                       int64_t N, int64_t H, void* dhidden, int64_t ld_dh, float* dweight, float* dbias,
                       void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------
 * K4 — decode-step token selection over the vocabulary (HF generate semantics that HFRollout
 * delegates to, verl/workers/rollout/hf_rollout.py:112-124). Two launches per decode step.
 * logits (N, V) F32/BF16 (row stride ld). unfinished (N) int32 in/out: rows already finished emit
 * pad_token_id (HF: next = next*unfinished + pad*(1-unfinished)) and a row hitting any eos id
 * becomes finished. The chosen token is written to out_tokens[n*ld_out] (int64) — pass a column
 * of the `responses` tensor to fill it in place. temperature <= 0 or do_sample == 0 -> greedy
 * (argmax, first index on ties = torch.argmax; row slices across workgroups, then one thread per row).
 * Sampling: z = logit / temperature (fp32, HF TemperatureLogitsWarper), then top-k (top_k > 0: tokens
 * below the k-th largest z dropped, ties kept, HF TopKLogitsWarper) and top-p (top_p < 1: the nucleus of
 * HF TopPLogitsWarper over the top-k survivors — a token is kept iff the softmax mass of the tokens above
 * it is < top_p; ties at the cut kept) as one cut per row (a third launch, one workgroup per row,
 * deterministic radix select), then the categorical draw over the kept tokens as a two-level race of
 * exponential clocks — softmax(z)-distributed like HF's torch.multinomial (whose one-sample path is the
 * same race, argmax p_i / E_i): the row is cut into slices of 2048 tokens; slice s races with key
 * ln(sum_{kept i in s} exp z_i) - ln(E_s), then the tokens i of the winning slice race with key
 * z_i - ln(E_i). E = -ln(1 - v), v = ((w >> 8) + 0.5) / 2^24, w = word (c & 3) of Philox4x32-10(key = seed,
 * counter = ((row_base + n) << 32 | c >> 2), offset = decode step) with c = i for tokens and
 * c = 2^33 + s for slices (counter low word 2^31 | s >> 2).
 * workspace: drl_select_tokens_workspace_bytes(N, V) bytes, 8-byte aligned, zero-filled before the first
 * call; every call leaves its greedy maxima zeroed again (one in-flight call per workspace).
 * ---------------------------------------------------------------------------------------------- */
typedef struct drl_sampling_params {
  int32_t do_sample;
  float temperature;
  int32_t top_k;
  float top_p;
  uint64_t seed;
  uint64_t offset;
  int64_t row_base;
  int64_t pad_token_id;
  const int64_t* eos_ids; /* device int64[n_eos]; may be NULL when n_eos == 0 */
  int32_t n_eos;
  /* optional device int64 scalar s (graph-captured decode loops): when non-NULL the Philox offset is
   * offset + s and the token is written to out_tokens[n * ld_out + s]. */
  const int64_t* dev_step;
} drl_sampling_params;

size_t drl_select_tokens_workspace_bytes(int64_t N, int64_t V);
int drl_select_tokens(const void* logits, int32_t logits_dtype, int64_t N, int64_t V, int64_t ld,
                      const drl_sampling_params* params, int32_t* unfinished, int64_t* out_tokens,
                      int64_t ld_out, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Rollout bookkeeping (A4/A5).
 * get_response_mask (torch_functional.py:226-246): mask[b,t] = 1 up to and including the first eos.
 * compute_position_id_with_mask (utils/model.py:219): pos = clip(cumsum(mask)-1, 0).
 * response positions (hf_rollout.py:151-155): pos[b, P+t] = pos[b, P-1] + 1 + t.
 * ---------------------------------------------------------------------------------------------- */
int drl_response_mask(const int64_t* responses, int64_t B, int64_t R, int64_t ld, const int64_t* eos_ids,
                      int32_t n_eos, void* mask_out, int32_t mask_dtype, int64_t ld_out, void* stream);
int drl_position_ids(const void* attention_mask, int32_t mask_dtype, int64_t B, int64_t T, int64_t* position_ids,
                     void* stream);
int drl_response_position_ids(int64_t* position_ids, int64_t B, int64_t P, int64_t R, void* stream);

/* ------------------------------------------------------------------------------------------------
 * A15 — optimizer step on a flat fp32 master buffer: clip_grad_norm_ + skip-if-non-finite + AdamW
 * (dp_actor.py:282-298; torch.optim.AdamW semantics, fsdp_workers.py:454-459).
 * drl_grad_norm: out_norm[0] = ||grads||_2 (device float).
 * drl_adamw_step: applies clip coef min(1, max_norm/(norm+1e-6)) from device `norm`; if norm is not
 * finite the step is skipped (params/moments untouched). Optionally writes a bf16 compute copy.
 * ---------------------------------------------------------------------------------------------- */
size_t drl_grad_norm_workspace_bytes(int64_t n);
int drl_grad_norm(const float* grads, int64_t n, float* out_norm, void* workspace, size_t workspace_bytes,
                  void* stream);
typedef struct drl_adamw_params {
  float lr;
  float beta1;
  float beta2;
  float eps;
  float weight_decay;
  int32_t step;       /* 1-based step count after this update */
  float max_grad_norm; /* <= 0: no clipping */
} drl_adamw_params;
int drl_adamw_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, uint16_t* params_bf16,
                   int64_t n, const drl_adamw_params* hp, const float* grad_norm, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Transformer-layer kernels of the actor / reference / rollout model (HF Qwen2 semantics as the
 * reference runs them inside _forward_micro_batch, dp_actor.py:90-280, and HF generate,
 * hf_rollout.py:112-124). `dt` is the element type of the activations (DRL_BF16 in production,
 * DRL_F32 for the parity model); the residual stream and norm weights are always float32.
 * ---------------------------------------------------------------------------------------------- */
/* qkv (B,T,(Hq+2Hkv)*D) -> RoPE'd q in grouped layout (B,Hkv,Hq/Hkv,T,D), RoPE'd k and v written at
 * key offset koff of (B,Hkv,Tk,D) buffers (the KV cache when decoding). cos/sin: (maxpos, D/2) fp32.
 * koff_dev (optional device int64 scalar) replaces koff — graph-captured decode steps; an out-of-range
 * device offset writes nothing. Optional head-dim-major copies for the fused attention kernels, row
 * stride ld_t over positions: qt (B,Hkv,G,D,ld_t), kt and vt (B,Hkv,D,ld_t); v may be NULL when vt
 * is given. */
int drl_rope_qkv_fwd(const void* qkv, int32_t dt, const int64_t* position_ids, const float* cos_t, const float* sin_t,
                     int64_t maxpos, int64_t B, int64_t T, int64_t Hq, int64_t Hkv, int64_t D, void* q, void* k,
                     void* v, int64_t Tk, int64_t koff, const int64_t* koff_dev, void* qt, void* kt, void* vt,
                     int64_t ld_t, void* stream);
/* drl_rope_qkv_fwd over a packed qkv (remove-padding / prefix-sharing passes): the qkv row of position (b, t) is
 * row src_row[b * T + t] of qkv (a negative entry: a zero row, the pad positions pad_input leaves zero), so the
 * packed rows are never scattered into a padded (B * T) copy first. src_row NULL: drl_rope_qkv_fwd.
 * q_skip (B,) int32, optional (ABI 7): q rows t < (q_skip[b] & ~31) are left unwritten — pass the q_start of
 * drl_flash_attn_fwd / _bwd, whose kernels never read those query tiles (prefix sharing's copies). */
int drl_rope_qkv_fwd_rows(const void* qkv, const int64_t* src_row, int32_t dt, const int64_t* position_ids,
                          const float* cos_t, const float* sin_t, int64_t maxpos, int64_t B, int64_t T, int64_t Hq,
                          int64_t Hkv, int64_t D, void* q, void* k, void* v, int64_t Tk, int64_t koff,
                          const int64_t* koff_dev, void* qt, void* kt, void* vt, int64_t ld_t, const int32_t* q_skip,
                          void* stream);
int drl_rope_qkv_bwd(const void* dq, const void* dk, const void* dv, int32_t dt, const int64_t* position_ids,
                     const float* cos_t, const float* sin_t, int64_t maxpos, int64_t B, int64_t T, int64_t Hq,
                     int64_t Hkv, int64_t D, void* dqkv, void* stream);
/* fp32 scores (B,Hkv,G,Tq,Tk) -> probs of type dt: softmax(scale*s) over keys j with
 * j <= q+qoff && key_valid[b,j] (causal + key padding, HF semantics: a query with no allowed key is
 * uniform over all Tk keys, as HF's additive finfo.min mask makes it). */
int drl_masked_softmax_fwd(const float* scores, void* probs, int32_t dt, const uint8_t* key_valid, int64_t ld_valid,
                           int64_t B, int64_t HG, int64_t Tq, int64_t Tk, int64_t qoff, float scale, void* stream);
/* dscores = probs * (dprobs - rowsum(probs*dprobs)) * scale  (rows x Tk; dprobs fp32) */
int drl_masked_softmax_bwd(const void* probs, const float* dprobs, void* dscores, int32_t dt, int64_t rows, int64_t Tk,
                           float scale, void* stream);
/* x_out = x_in (+ delta); y = w * x_out * rsqrt(mean(x_out^2) + eps)  (Qwen2RMSNorm); rstd saved. */
int drl_add_rmsnorm_fwd(const float* x_in, const void* delta, float* x_out, const float* weight, void* y, int32_t dt,
                        float* rstd, int64_t N, int64_t H, float eps, void* stream);
size_t drl_rmsnorm_bwd_workspace_bytes(int64_t N, int64_t H);
/* dx += d norm(x)/dx . dy ; dw += sum_rows dy * xhat */
int drl_rmsnorm_bwd(const float* x, const float* weight, const float* rstd, const void* dy, int32_t dt, float* dx,
                    float* dw, int64_t N, int64_t H, void* workspace, size_t workspace_bytes, void* stream);
/* drl_rmsnorm_bwd with the residual gradient passed through: dx = dx_in + d norm(x)/dx . dy (dx_in NULL: zero;
 * dx_in == dx: in place), and, when dx_bf16 is not NULL, its bf16 rounding written in the same pass (the operand of
 * the next dgrad, and the gradient of a bf16 residual delta). Workspace as drl_rmsnorm_bwd. */
int drl_rmsnorm_bwd_ex(const float* x, const float* weight, const float* rstd, const void* dy, int32_t dt,
                       const float* dx_in, float* dx, void* dx_bf16, float* dw, int64_t N, int64_t H, void* workspace,
                       size_t workspace_bytes, void* stream);
/* gate_up (N, 2I) -> out (N, I) = silu(gate) * up ; backward -> d gate_up */
int drl_swiglu_fwd(const void* gate_up, void* out, int32_t dt, int64_t N, int64_t I, void* stream);
int drl_swiglu_bwd(const void* gate_up, const void* dout, void* dgate_up, int32_t dt, int64_t N, int64_t I,
                   void* stream);

/* ---- decode attention (rollout engine; replaces the per-token attention of HF generate,
 *      hf_rollout.py:112-124 -> Qwen2Attention with the KV cache).
 * q (B, Hkv, G, D) for one new token; k/v cache (B, Hkv, Tk, D), keys [0, L) used; a key j is attended iff
 * key_valid[b*ld_valid + j] && j <= qpos, where qpos = *qpos_ptr if qpos_ptr != NULL (device scalar, for
 * graph capture) else qpos. out (B, Hkv, G, D) == (B, Hq*D). A row with no allowed key writes zeros.
 * With a workspace of drl_decode_attention_workspace_bytes(B, Hkv, G, D, L) and fewer (b, kv head) pairs
 * than CUs, the key range is split over more workgroups (split-K + fixed-order merge); otherwise a single
 * pass per (b, kv head) runs. */
size_t drl_decode_attention_workspace_bytes(int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t L);
int drl_decode_attention(const void* q, const void* k_cache, const void* v_cache, int32_t dt, const uint8_t* key_valid,
                         int64_t ld_valid, const int64_t* qpos_ptr, int64_t qpos, int64_t B, int64_t Hkv, int64_t G,
                         int64_t D, int64_t Tk, int64_t L, float scale, void* out, void* workspace,
                         size_t workspace_bytes, void* stream);

/* ---- fused attention forward on MFMA (full-sequence passes: old / ref log-probs, training forward;
 *      replaces the eager q k^T -> masked softmax -> p v of HF Qwen2 attention under dp_actor.py:90-280).
 * q (B,Hkv,G,Tq,D) bf16 (grouped layout of drl_rope_qkv_fwd), k (B,Hkv,ld_k,D) of which keys [0,Tk)
 * are used (ld_k > Tk: a KV cache), vt (B,Hkv,D,ld_vt) (V
 * transposed, ld_vt >= Tk, multiple of 8), key_valid (B, ld_valid) u8 with 4-byte aligned rows.
 * Query t attends to key j iff j <= t + qoff && key_valid[b, j]; out (B,Tq,Hkv*G*D) bf16 (the o_proj
 * input layout). lse (optional, (B,Hkv,G,Tq) fp32) = log sum_j exp(scale * s_tj) over allowed keys.
 * A query row with no allowed key writes zeros and lse = -inf. bf16, head_dim 64 or 128, G <= 8.
 * q_start (optional, (B,) int32): the 32-query tiles of row b wholly below q_start[b] are skipped and their out /
 * lse rows left unwritten — the shared-prompt copies under prefix sharing, which nothing reads. */
int drl_flash_attn_fwd(const void* q, const void* k, const void* vt, int32_t dt, const uint8_t* key_valid,
                       int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t Tq, int64_t Tk,
                       int64_t ld_k, int64_t ld_vt, int64_t qoff, const int32_t* q_start, float scale, void* out,
                       float* lse, void* stream);
/* drl_flash_attn_fwd writing packed rows (remove-padding / prefix sharing, forward-only passes): out_row (B*Tq,)
 * int64 gives the out row of query (b, t) — out is (rows, Hkv*G*D) — and a negative entry skips the query's output
 * (pads; the shared-prompt copies, whose packed row is their leader's). The packed copy the o_proj reads is then
 * written by the attention itself, with no padded (B, Tq) output and no row copy after it. out_row NULL:
 * drl_flash_attn_fwd. */
int drl_flash_attn_fwd_rows(const void* q, const void* k, const void* vt, int32_t dt, const uint8_t* key_valid,
                            int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t Tq, int64_t Tk,
                            int64_t ld_k, int64_t ld_vt, int64_t qoff, const int32_t* q_start, float scale, void* out,
                            const int64_t* out_row, float* lse, void* stream);
/* Decode attention on MFMA over a cache with V head-dim-major: q (B,Hkv,G,D) bf16 (one token), k_cache
 * (B,Hkv,ld_k,D), vt_cache (B,Hkv,D,ld_vt); keys j < L with key_valid[b, j] && j <= qpos (device scalar
 * *qpos_ptr when non-NULL). out (B,Hkv,G,D), or with out_mbt > 0 the (B, Hq*D) panel fragment-packed for
 * drl_decode_gemm (out_mbt >= B/32 blocks). G <= 32, head_dim 64 or 128. Same semantics as
 * drl_decode_attention (the VALU kernel over a row-major V cache used by the fp32 parity model).
 * q and both caches 16-byte aligned, ld_vt % 8 == 0 (32-key blocks are fetched with whole 16-byte loads).
 * Small batches split the keys over workgroups (partial softmax states merged in split order by the last
 * arriving split): workspace of drl_decode_attention_vt_workspace_bytes(B, Hkv, D, L) bytes (0 = none
 * needed), 256-byte aligned, zero-filled before the first call and left zeroed by every call. */
size_t drl_decode_attention_vt_workspace_bytes(int64_t B, int64_t Hkv, int64_t D, int64_t L);
/* Graphed decode step prologue (hf_rollout.py:112-124's per-token bookkeeping for a device step counter): with
 * t = *t_dev, for every row b: x[b, :] = float(embed[responses[b, t - 1], :]) (bf16 embedding (V, H) -> fp32
 * residual stream), positions[b] = last_pos[b] + t, key_valid[b, t + prompt_len - 1] = 1; then *kpos =
 * t + prompt_len - 1, *t_cur = t and *t_dev = t + 1 (the last workgroup, after every row has read t_dev).
 * workspace: drl_decode_step_prologue_workspace_bytes() bytes, zero-filled once (left zeroed by every call).
 * x_mbt > 0 (ABI 8): x is the fused-norm decode's packed fp32 residual (drl_decode_gemm_resid), x_mbt token blocks;
 * 0: x row-major (B, H). */
size_t drl_decode_step_prologue_workspace_bytes(void);
int drl_decode_step_prologue(const int64_t* responses, int64_t ld_responses, int64_t* t_dev, int64_t* t_cur,
                             const int64_t* last_pos, int64_t prompt_len, const void* embed, int32_t dt, int64_t V,
                             int64_t H, int64_t B, float* x, int64_t* positions, int64_t* kpos, uint8_t* key_valid,
                             int64_t ld_valid, void* workspace, size_t workspace_bytes, int64_t x_mbt, void* stream);
/* Tuning hook (tools/kernel_bench.py): force waves per workgroup (2/4/8/16) and key splits; 0 = automatic. */
void drl_decode_attention_set_plan(int32_t waves, int32_t splits);
/* Tuning hook of the decode attention's work placement (ABI 8): rows per column tile of the prompt-group kernel
 * (1..32 / G; 0 = 32 / G), workgroup -> XCD map of both kernels (0 = units round-robin over the XCDs, 1 = a contiguous
 * eighth of the cache rows per XCD) and the prompt-group kernel's own-block schedule (1 = balanced over the waves,
 * 0 = by block class, -1 = automatic). Results are identical for every plan. */
void drl_decode_group_set_plan(int32_t rows_per_tile, int32_t xcd_map, int32_t balanced);
/* Tuning hook of the fused attention backward (head_dim 64): 0 = dQ over one query tile per workgroup (default),
 * 1 = two query tiles per workgroup (K / V fragments in registers), 2 = two tiles re-reading them. Same bits. */
void drl_flash_attn_bwd_set_variant(int32_t variant);
/* Tuning hook for forced plans (set_plan waves != 0): 1 = register-lean key loop (one block in flight per
 * wave, fragments read from LDS); 2..4 = that many blocks in flight per wave (4 and 8 waves, D = 64; else 2);
 * 5 = the register-lean loop with 2 blocks in flight (8 waves, D = 64). Results are identical. */
void drl_decode_attention_set_variant(int32_t variant);
/* Prompt groups (the n samples of one prompt, hf_rollout.py's repeated prompts / vLLM's shared prefix): with
 * group > 1, sequences b = p * group + r share one prompt, and keys j < shared_keys (a multiple of 32, <= L) are
 * read from cache row p — K and V^T — where the rollout prefilled each distinct prompt once; keys j >= shared_keys
 * from row b. key_valid is always row b's own (every row holds its prompt's mask: row p < B / group is itself a
 * sample of prompt p / group). group 1 and shared_keys 0: every row reads its own keys. With at least half a
 * workgroup per CU of (prompt, KV head, 32 / G rows) tiles, one workgroup takes a tile's rows together and loads each
 * shared block once for them; its result equals the per-row kernel's at the same wave count without key splits
 * (8 waves at head_dim 64, 4 at 128; drl_decode_attention_set_plan forces both). Contract: the rows of a group have
 * identical key_valid bytes below shared_keys (the rollout copies the prompt's mask to every row). */
int drl_decode_attention_vt(const void* q, const void* k_cache, const void* vt_cache, int32_t dt,
                            const uint8_t* key_valid, int64_t ld_valid, const int64_t* qpos_ptr, int64_t qpos,
                            int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t ld_k, int64_t ld_vt, int64_t L,
                            int64_t group, int64_t shared_keys, float scale, void* out, int64_t out_mbt,
                            void* workspace, size_t workspace_bytes, void* stream);
/* Backward of drl_flash_attn_fwd for Tq == Tk == T, qoff = 0 (the training forward), recomputing P from lse:
 * q (B,Hkv,G,T,D), k / v (B,Hkv,T,D) row-major, kt (B,Hkv,D,ld_t) head-dim-major copy of k (written by
 * drl_rope_qkv_fwd), o and dout (B,T,Hkv*G*D), lse from the forward. delta: (B,Hkv,G,T) fp32 scratch.
 * Outputs dq (B,Hkv,G,T,D), dk / dv (B,Hkv,T,D) bf16 (the drl_rope_qkv_bwd inputs). T and ld_t multiples
 * of 8; head_dim 64. Deterministic (the G heads' dK/dV partials are summed in a fixed order). q_start (optional,
 * (B,) int32, as in the forward): dout is zero on the skipped query tiles — their dq rows are written as zeros and
 * contribute nothing to dk / dv (not read: o, dout, lse of those rows may hold anything). */
int drl_flash_attn_bwd(const void* q, const void* k, const void* kt, const void* v, const void* o, const void* dout,
                       const float* lse, int32_t dt, const uint8_t* key_valid, int64_t ld_valid, int64_t B,
                       int64_t Hkv, int64_t G, int64_t D, int64_t T, int64_t ld_t, const int32_t* q_start, float scale,
                       float* delta, void* dq, void* dk, void* dv, void* stream);
/* drl_flash_attn_bwd with o packed (rows, Hkv*G*D) — the forward's drl_flash_attn_fwd_rows output — read through
 * o_row (B*T,) (the same map; a negative entry reads row 0: those rows' dout is zero, so delta = 0 either way). dout
 * stays padded (B, T, Hkv*G*D). o_row NULL: drl_flash_attn_bwd. */
int drl_flash_attn_bwd_rows(const void* q, const void* k, const void* kt, const void* v, const void* o,
                            const int64_t* o_row, const void* dout, const float* lse, int32_t dt,
                            const uint8_t* key_valid, int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D,
                            int64_t T, int64_t ld_t, const int32_t* q_start, float scale, float* delta, void* dq,
                            void* dk, void* dv, void* stream);

/* A21 fused lm_head + log-prob + entropy (MFMA; logits never written). Replaces FusedLinearForPPO.forward
 * (verl/utils/experimental/torch_functional.py:20-37, :153-216) and the Triton linear_cross_entropy forward
 * (verl/utils/kernel/linear_cross_entropy.py:41-84 -> kernels.py:507-696) for reduction "none".
 * hidden (N, ld_h) bf16, weight (V, H) bf16 row-major, labels (N) int64 in [0, V); H % 64 == 0, 16-B aligned
 * operands. z = hidden W^T / temperature in fp32 (no bf16 rounding of the logits: the Triton kernel's
 * numerics); outputs (each may be NULL) logp[t] = z[t, label] - lse[t], entropy[t] = lse[t] - sum_v p z,
 * lse[t] (natural log), all fp32. workspace: drl_linear_logprob_workspace_bytes(N, H, V) bytes, any content.
 * Deterministic (fixed tile order, fixed-order merges). */
size_t drl_linear_logprob_workspace_bytes(int64_t N, int64_t H, int64_t V);
int drl_linear_logprob_fwd(const void* hidden, int64_t ld_h, const void* weight, const int64_t* labels, int32_t dt,
                           int64_t N, int64_t H, int64_t V, float temperature, float* logp, float* entropy,
                           float* lse, void* workspace, size_t workspace_bytes, void* stream);
/* A21 backward, d_logits stage (the reference's BackwardEnum._Total_Separate, kernels.py:1378-1480 ->
 * efficient_entropy_backward_kernel_general_d_logits; semantics torch_functional.py:40-72): recomputes z and
 * writes d_logits TRANSPOSED, dlogits_t (V, ld_dl) bf16 with ld_dl >= N:
 *   d z[t, v] = (dlogp[t] (1[v == label] - p) - dentropy[t] p (log p + entropy[t])) / temperature.
 * dentropy may be NULL (no entropy gradient; entropy then unused). d_hidden = dlogits_t^T W and
 * d_W = dlogits_t hidden are library GEMMs on the caller side. */
int drl_linear_logprob_dlogits(const void* hidden, int64_t ld_h, const void* weight, const int64_t* labels, int32_t dt,
                               int64_t N, int64_t H, int64_t V, float temperature, const float* dlogp,
                               const float* dentropy, const float* lse, const float* entropy, void* dlogits_t,
                               int64_t ld_dl, void* stream);

/* K4 fused with the lm_head (decode): token selection straight from hidden (N, ld_h) bf16 and the lm_head
 * weight (V, H) bf16 without writing the (N, V) logits — drl_select_tokens' semantics on the bf16 logits
 * bf16(hidden W^T), greedy only (argmax, lowest index on ties; do_sample returns DRL_ERR_UNSUPPORTED: the
 * two-level draw races inside one slice of the logits row), the same params / unfinished / EOS bookkeeping. workspace: drl_linear_select_tokens_workspace_bytes(N)
 * bytes, 8-byte aligned, zero-filled before the first call and left zeroed by every call. H % 64 == 0. */
size_t drl_linear_select_tokens_workspace_bytes(int64_t N);
int drl_linear_select_tokens(const void* hidden, int64_t ld_h, const void* weight, int32_t dt, int64_t N, int64_t H,
                             int64_t V, const drl_sampling_params* params, int32_t* unfinished, int64_t* out_tokens,
                             int64_t ld_out, void* workspace, size_t workspace_bytes, void* stream);

/* ---- Decode-step projections on fragment-packed operands (csrc/decode_gemm.hip). Replace the per-token
 * nn.Linear / RMSNorm / rotary calls of HF generate (hf_rollout.py:112-124 -> modeling_qwen2) for 1..512
 * token rows. Packed layout of an activation panel (M rows, K columns, MBT 32-row blocks, MBT >= M/32):
 * element (m, k) at ((k/16 * MBT + m/32) * 64 + ((k/8) & 1) * 32 + m % 32) * 8 + k % 8; rows >= M must hold
 * zeros (allocate zero-filled, never write them). */
typedef enum drl_decode_epilogue {
  DRL_DECODE_PARTIAL = 0, /* fp32 partial sums per K slice: partials (ksplit, M, N) */
  DRL_DECODE_SWIGLU = 1,  /* W = [gate | up] packed with swiglu=1: bf16(bf16(silu(g)) * u) packed (MBT, N/2) */
  DRL_DECODE_RESID = 2,   /* drl_decode_norm_plan only: the residual producer drl_decode_gemm_resid */
  DRL_DECODE_ROPE = 3     /* drl_decode_norm_plan only: the norm consumer drl_decode_qkv_rope_norm */
} drl_decode_epilogue;
/* ksplit (K slices = partial sums the consumer adds) and mbt (token blocks the packed panels need). */
int drl_decode_gemm_plan(int64_t M, int64_t N, int64_t K, int32_t epilogue, int32_t* ksplit, int32_t* mbt);
/* Tuning hook (tools/kernel_bench.py): force 32-row token blocks per workgroup (1, 2) and k16 steps per wave
 * (1, 2, 4, 7, 14; 19 with one block); 0 = automatic. */
void drl_decode_gemm_set_plan(int32_t mb, int32_t ksw);
/* 192..512 rows run the MFMA-tiled form (2-D wave tiles over weight rows x tokens) for the partial and qkv + RoPE
 * projections: mode 1 (default); 0 = never (A/B tuning); 2 = tiled with one K slice (tests). */
void drl_decode_gemm_set_tiled(int32_t mode);
/* Tuning hook: most K slices (partial sums) of a tiled decode GEMM plan, 1..16 (default 4). Schedule only. */
void drl_decode_gemm_set_max_splits(int32_t ks);
/* Tuning hook: force tiled configuration `config` (-1 = planner) and the smallest M of the tiled path (0 = 192). */
void drl_decode_gemm_force_tiled(int32_t config, int32_t min_rows);
/* Elements of the packed copy of W (N, K) bf16 (swiglu: W = [gate | up], blocks interleave 16 + 16 rows). */
size_t drl_decode_pack_weight_elems(int64_t N, int64_t K, int32_t swiglu);
int drl_decode_pack_weight(const void* w, int64_t ld, int64_t N, int64_t K, int32_t swiglu, void* packed, void* stream);
/* y = x W^T with x packed (M rows), W packed; K % 64 == 0, 1 <= M <= 512. PARTIAL writes fp32 partials,
 * SWIGLU writes the activation packed for the down projection. */
int drl_decode_gemm(const void* x_packed, const void* w_packed, int64_t M, int64_t N, int64_t K, int32_t epilogue,
                    float* partials, void* out_packed, void* stream);
/* Packed copy of qkv_proj.weight (N = (Hq + 2 Hkv) head_dim rows) in rotation pairs: every 32-row block
 * holds 16 consecutive head-dim rows and their RoPE partners head_dim/2 further (drl_decode_qkv_rope). */
int drl_decode_pack_weight_rope(const void* w, int64_t ld, int64_t N, int64_t K, int64_t head_dim, void* packed,
                                void* stream);
/* qkv_proj + bias + rotary embedding of one decode token per sequence in ONE launch (replaces
 * drl_decode_gemm + drl_decode_rope): qkv = bf16(x W^T + bias), q/k rotated as drl_rope_qkv_fwd, q written
 * (M, Hkv, G, D), k to k_cache (M, Hkv, Tk, D) row *koff_dev, v to vt_cache (M, Hkv, D, ld_vt) column
 * *koff_dev. x packed (M rows, K % 64 == 0), W packed by drl_decode_pack_weight_rope. */
int drl_decode_qkv_rope(const void* x_packed, const void* w_packed, const void* bias, const int64_t* position_ids,
                        const float* cos_t, const float* sin_t, int64_t maxpos, int64_t M, int64_t K, int64_t Hq,
                        int64_t Hkv, int64_t D, void* q, void* k_cache, void* vt_cache, int64_t Tk, int64_t ld_vt,
                        const int64_t* koff_dev, void* stream);
/* x_out = x_in + bf16(sum of nsplit partials (nsplit, M, H)) (partials may be NULL: no delta), y = bf16(w *
 * x_out * rsqrt(mean(x_out^2) + eps)) packed with mbt blocks, or row-major (M, H) when mbt == 0
 * (drl_add_rmsnorm_fwd semantics). H % 8 == 0. y_packed (ABI 8, may be NULL): the same y written a second time,
 * packed with packed_mbt blocks (the decode lm_head's operand beside a row-major y). */
int drl_decode_rmsnorm(const float* x_in, const float* partials, int32_t nsplit, float* x_out, const float* weight,
                       void* y, int64_t M, int64_t H, int64_t mbt, float eps, void* y_packed, int64_t packed_mbt,
                       void* stream);
/* One decode token per sequence: qkv = bf16(sum of nsplit partials (nsplit, B, (Hq+2Hkv)D) + bias), then
 * drl_rope_qkv_fwd's rotation: q (B, Hkv, G, D), k_cache (B, Hkv, Tk, D) row koff, V into vt_cache
 * (B, Hkv, D, ld_vt) column koff and/or v_cache (B, Hkv, Tk, D); koff_dev (device int64) overrides koff. */
int drl_decode_rope(const float* partials, int32_t nsplit, const void* bias, const int64_t* position_ids,
                    const float* cos_t, const float* sin_t, int64_t maxpos, int64_t B, int64_t Hq, int64_t Hkv,
                    int64_t D, void* q, void* k_cache, void* v_cache, void* vt_cache, int64_t Tk, int64_t ld_vt,
                    int64_t koff, const int64_t* koff_dev, void* stream);
/* ---- Fused-norm decode step (ABI 8; 1..128 rows by default): the decoder layer's two RMSNorms folded into the
 * consumer GEMMs' prologue, so a layer is five launches (qkv + RoPE, attention, o_proj, gate_up + SwiGLU, down_proj)
 * instead of seven. Replaces, per decode token of HF generate (hf_rollout.py:112-124 -> modeling_qwen2), the
 * residual adds of Qwen2DecoderLayer and Qwen2RMSNorm (input_layernorm / post_attention_layernorm) with the same
 * rounding: x += bf16(o) in fp32, y = bf16(w * (x * rsqrt(mean(x^2) + eps))). The fp32 residual stream x_resid is
 * kept packed: element (m, k) at the packed-activation offset above (fp32 elements), x_mbt token blocks, rows >= M
 * zero. */
/* Plan query: epilogue DRL_DECODE_RESID (ksplit: K slices of the residual producer, config: its k16 steps per wave),
 * DRL_DECODE_SWIGLU (the gate_up consumer) or DRL_DECODE_ROPE (the qkv consumer; N = (Hq + 2 Hkv) D), config: the
 * consumer's kernel configuration; mbt: the token blocks of every packed panel of the step. DRL_ERR_UNSUPPORTED when
 * the shape takes the unfused path (more rows than the fused form's limit, K > 4096). */
int drl_decode_norm_plan(int64_t M, int64_t N, int64_t K, int32_t epilogue, int32_t* ksplit, int32_t* mbt,
                         int32_t* config);
/* Tuning hook: force consumer configuration `config` (-1 = planner), the fused form's row limit (0 = 128) and the most
 * K slices of the residual producer (0 = the partial-sum planner's choice; 1 = whole K where a shape allows). */
void drl_decode_norm_set_plan(int32_t config, int32_t max_rows, int32_t resid_max_splits);
/* Bytes of zeroed arrival counters drl_decode_gemm_resid needs (0 when the shape is not on the fused path). */
size_t drl_decode_resid_counter_bytes(int64_t M, int64_t N, int64_t K);
/* o_proj / down_proj of the fused-norm step: x_resid (packed fp32, x_mbt blocks, N columns) += bf16(x W^T) in place,
 * the K slices summed in slice order by the slice that arrives last (no grid barrier). partials: ksplit x M x N fp32
 * scratch; counters: drl_decode_resid_counter_bytes zero-filled bytes, left zeroed by every call. */
int drl_decode_gemm_resid(const void* x_packed, const void* w_packed, int64_t M, int64_t N, int64_t K, float* x_resid,
                          int64_t x_mbt, float* partials, void* counters, size_t counter_bytes, void* stream);
/* gate_up + SwiGLU of the fused-norm step: y = RMSNorm(x_resid) with norm_weight (K fp32) computed per workgroup in
 * the prologue, then drl_decode_gemm's SWIGLU epilogue (out packed, N/2 columns). */
int drl_decode_gemm_norm(const float* x_resid, const float* norm_weight, float eps, const void* w_packed, int64_t M,
                         int64_t N, int64_t K, void* out_packed, void* stream);
/* qkv + bias + RoPE + cache writes of the fused-norm step: drl_decode_qkv_rope on RMSNorm(x_resid). */
int drl_decode_qkv_rope_norm(const float* x_resid, const float* norm_weight, float eps, const void* w_packed,
                             const void* bias, const int64_t* position_ids, const float* cos_t, const float* sin_t,
                             int64_t maxpos, int64_t M, int64_t K, int64_t Hq, int64_t Hkv, int64_t D, void* q,
                             void* k_cache, void* vt_cache, int64_t Tk, int64_t ld_vt, const int64_t* koff_dev,
                             void* stream);
/* The model's final norm of the fused-norm step (Qwen2Model.norm): y = bf16(w * x * rsqrt(mean(x^2) + eps)) from the
 * packed residual, y packed (y_mbt blocks) or row-major (M, H) when y_mbt == 0. */
int drl_decode_final_norm(const float* x_resid, int64_t x_mbt, const float* weight, void* y, int64_t M, int64_t H,
                          int64_t y_mbt, float eps, void* y_packed, int64_t packed_mbt, void* stream);
/* The decode step's lm_head at <= 64 rows (ABI 8; replaces nn.Linear lm_head of HF generate's per-token forward,
 * hf_rollout.py:112-124): logits (M, ld) bf16 = bf16(h W^T) with h the packed final-norm output (mbt blocks from
 * drl_decode_lm_head_plan) and W packed by drl_decode_pack_weight (V rows). K = 896. One workgroup per CU holds the h
 * panel in LDS and streams its own contiguous range of the packed weight (no cross-workgroup dependence). */
int drl_decode_lm_head_plan(int64_t M, int64_t V, int64_t K, int32_t* mbt);
/* Tuning hook: the decode lm_head's (waves per workgroup, weight loads in flight per wave) configuration 0..5
 * (-1 = automatic). */
void drl_decode_lm_head_set_config(int32_t config);
int drl_decode_lm_head(const void* h_packed, int64_t mbt, const void* w_packed, int64_t M, int64_t V, int64_t K,
                       void* logits, int64_t ld, void* stream);



/* ------------------------------------------------------------------------------------------------
 * Every transformer GEMM of the actor's passes (csrc/gemm_sk.hip): the forward projections, their dgrad and their
 * wgrad — replaces hipBLASLt behind nn.Linear's forward AND its autograd backward in HF Qwen2 / Llama under the
 * reference's FSDP autocast (dp_actor.py:110; loss.backward() at dp_actor.py:466): dx = dy W (F.linear's grad_input),
 * dW += dy^T x (grad_weight, accumulated over micro-batches in fp32 as FSDP's fp32 gradient).
 *   C(m, n) (+)= sum_k A(m, k) B(n, k),  A(m, k) = a[m*lda + k] (DRL_LAYOUT_K) or a[k*lda + m] (DRL_LAYOUT_T),
 *                                        B(n, k) = b[n*ldb + k] (DRL_LAYOUT_K) or b[k*ldb + n] (DRL_LAYOUT_T).
 * bf16 operands, fp32 accumulation (a layout-K A operand over 2 GB runs as one launch, its buffer descriptor
 * rebased per tile). c_dtype DRL_BF16 epilogues
 * (bias / SwiGLU need both operands layout K): PLAIN c (M, N) = bf16(acc); BIAS c = bf16(acc + bias) (addmm: one
 * rounding); SWIGLU: B = [gate | up] (N = 2I rows), c (M, I) = bf16(bf16(silu(g)) * u) with g, u the bf16-rounded
 * gate / up sums, c2 (M, 2I) = [g | u] when not NULL (the backward's saved activation); DRL_F32 (plain epilogue): c = acc, or c += acc when beta != 0. K % 64 == 0 unless both
 * operands are layout T (then any K: the k tail reads as zeros). A / B 16-byte aligned, ld % 8 == 0, each operand
 * < 2 GB. DRL_GEMM_SWIGLU_BWD (drl_gemm only): the down_proj dgrad fused with the SwiGLU backward (swiglu_bwd's
 * math on d a = bf16(acc)): A = dy layout K, B = W_down layout T, c2 = gu (M, 2N) read, c = dgu (M, 2N) written.
 * Work is split stream-K over at most one workgroup per CU; split tiles are summed in a fixed order
 * (bit-reproducible). workspace: drl_gemm_workspace_bytes() bytes, 16-byte aligned, zeroed once at allocation
 * (every call leaves its flag words zero again); calls sharing a workspace must be ordered on one stream. */
enum { DRL_GEMM_PLAIN = 0, DRL_GEMM_BIAS = 1, DRL_GEMM_SWIGLU = 2, DRL_GEMM_SWIGLU_BWD = 3 };
enum { DRL_LAYOUT_K = 0, DRL_LAYOUT_T = 1 };
int drl_gemm(const void* a, int64_t lda, int32_t a_layout, const void* b, int64_t ldb, int32_t b_layout, void* c,
             int64_t ldc, int32_t c_dtype, int32_t beta, int64_t M, int64_t N, int64_t K, const void* bias,
             int32_t epilogue, void* c2, int64_t ldc2, void* workspace, int64_t workspace_bytes, void* stream);
int64_t drl_gemm_workspace_bytes(void);
/* Tuning hook of drl_gemm: grid (0 = CU count), M-tiles per rasterization group, dp_mode (0 automatic: whole-tile
 * rounds while they fill the grid, stream-K for the last one or two; 1 = all stream-K; 2 = whole tiles only),
 * min_iters (minimum k-tile pairs per workgroup of an all-stream-K grid, 0 = 2). Schedule only, same result. */
void drl_gemm_set_sk_tuning(int32_t grid, int32_t group, int32_t dp_mode, int32_t min_iters);
/* Measurement hook (never set in the product path), bit flags, 0 = normal: 1 = whole tiles skip their epilogue (no
 * output written), to time the main loop and the per-tile fixed cost apart; 2 = the plain epilogue stages but does not
 * store; 4 = the epilogue's barriers only; 8 = slice-major split-K workgroup order; 16 = layout-T operands past 2 GB as
 * a host loop of K-block launches; 32 = full-width tiles for the last tile column of N % 256 in (0, 128] (the
 * half-width path off: same results bit for bit). */
void drl_gemm_set_debug(int32_t flags);
/* (flags bit 8: all-split-K grids in slice-major workgroup order instead of tile-major — schedule only, the same
 * bits; bit 16: a layout-T operand past 2 GB as the host loop of K-block launches; both for A/B measurement.) */
/* The decomposition drl_gemm would launch for one (M, N, K, epilogue) over `cus` CUs under the current tuning (host
 * arithmetic only, no device): info[0] mode (1 stream-K, 2 whole tiles, 3 uniform split-K), info[1] split-K slices
 * per split tile, info[2] workgroups, info[3] tiles dealt whole, info[4] first split workgroup (tail split-K).
 * Per launch: an operand past the 2 GB buffer range (K blocks of a layout-T operand) is several launches. */
int drl_gemm_plan(int64_t M, int64_t N, int64_t K, int32_t epilogue, int32_t cus, int32_t* info);


/* Row gather / scatter of the remove-padding passes (flash_attn.bert_padding unpad_input / pad_input /
 * index_first_axis under dp_actor.py:119-247, dp_critic.py:69-107 with use_remove_padding=True): for i < n_rows,
 * row src_idx[i] (or i when NULL) of src -> row dst_idx[i] (or i) of dst, row_bytes each (a multiple of 16, rows
 * 16-byte aligned); a negative index skips the row. */
int drl_copy_rows(const void* src, int64_t ld_src_bytes, const int64_t* src_idx, void* dst, int64_t ld_dst_bytes,
                  const int64_t* dst_idx, int64_t n_rows, int64_t row_bytes, void* stream);
/* The gather of drl_copy_rows that writes every destination row: row i of dst (i < n_rows) = row src_idx[i] of src,
 * or zeros where src_idx[i] < 0 (pad_input's zero pad rows without a memset of the padded buffer first). */
int drl_gather_rows(const void* src, int64_t ld_src_bytes, const int64_t* src_idx, void* dst, int64_t ld_dst_bytes,
                    int64_t n_rows, int64_t row_bytes, void* stream);
/* Row sums of prefix sharing (the adjoint of a gather in which K padded positions read one packed row — a prompt
 * token shared by the samples of one prompt; the reference runs every sample's copy, dp_actor.py:119-247): for
 * j < m, dst[dst_idx[j] (or j)] = sum over k < K of src[src_idx[k * m + j]] (an index < 0 adds nothing; a
 * negative dst index skips the row), fp32 accumulation in k order, dt DRL_BF16 or DRL_F32; ld_src / ld_dst in
 * elements, rows 16-byte aligned, cols a multiple of 16 bytes. */
int drl_sum_rows(const void* src, int64_t ld_src, const int64_t* src_idx, int64_t K, void* dst, int64_t ld_dst,
                 const int64_t* dst_idx, int64_t m, int64_t cols, int32_t dt, void* stream);



/* out (C,) fp32 += column sums of x (N, C) bf16 (row stride ld): the qkv bias gradient, dqkv summed over tokens
 * (replaces the autograd of `+ bias` in Qwen2Attention's q/k/v Linear). Deterministic (fixed order). */
size_t drl_colsum_bf16_workspace_bytes(int64_t N, int64_t C);
int drl_colsum_bf16_acc(const void* x, int64_t ld, int64_t N, int64_t C, float* out, void* workspace,
                        size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DOTSRL_AMD_H_ */
