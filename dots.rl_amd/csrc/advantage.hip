// K3 — GRPO outcome advantage and K5 — GAE + masked_whiten, on device.
// References: verl/trainer/ppo/core_algos.py:208-256 (GAE), 260-324 (GRPO);
// verl/utils/torch_functional.py:171-223 (masked_mean / masked_var / masked_whiten).
// The reference runs both as Python loops on the driver CPU (core_algos.py:297-324); here the scores
// are row sums of the (B, R) rewards in HBM, the group statistics come from a host-built CSR of the uid
// groups (order of first appearance, the order torch.stack sees them), and the (B, R) outputs are
// written in one coalesced pass.
#include "common.h"

namespace drl {
namespace {

// scores[b] = token_level_rewards[b, :].sum(-1), one wave per row
__global__ __launch_bounds__(256) void row_sum_kernel(const float* x, int64_t B, int64_t R, float* out) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float s = 0.f;
  for (int64_t t = lane; t < R; t += 64) s += x[row * R + t];
  s = wave_sum(s);
  if (lane == 0) out[row] = s;
}

// scores[b] = rewards row sum and lens[b] = response_mask row sum (OPO's response lengths), one wave per row
template <int MDT>
__global__ __launch_bounds__(256) void row_sum_len_kernel(const float* x, const void* mask, int64_t B, int64_t R,
                                                          float* out, float* lens) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float s = 0.f, l = 0.f;
  for (int64_t t = lane; t < R; t += 64) {
    s += x[row * R + t];
    l += mask_at<MDT>(mask, row * R + t);
  }
  s = wave_sum(s);
  l = wave_sum(l);
  if (lane == 0) { out[row] = s; lens[row] = l; }
}

// per row: group mean/std over the CSR members (float32, torch.mean / unbiased torch.std), then
// advantages[b, t] = returns[b, t] = norm_score[b] * mask[b, t]
// estimator: DRL_ADV_GRPO (core_algos.py:260-324), DRL_ADV_RLOO (core_algos.py:444-493: n > 1 ->
// s * n / (n - 1) - mean * n / (n - 1), a single sample keeps its score), DRL_ADV_REINFORCE_PP_BASELINE
// (core_algos.py:392-441: s - group mean, then masked_whiten over the batch by the caller's second kernel),
// DRL_ADV_OPO (core_algos.py:495-546: s - sum(len * s) / sum(len) over the group, 0 baseline for a single
// sample), DRL_ADV_GPG (core_algos.py:624-684: alpha * (s - group mean), alpha = B / max(#nonzero scores, 1)
// over the batch, f_norm = 1), DRL_ADV_GRPO_PASSK (core_algos.py:327-386: the group's best sample gets
// r_max - r_second_max (/ (std + eps)), every other sample 0; groups of >= 2 samples, checked by the host).
template <int MDT>
__global__ __launch_bounds__(256) void grpo_write_kernel(const float* scores, const void* mask, const int32_t* row_group,
                                                         const int32_t* off, const int32_t* mem, int64_t B, int64_t R,
                                                         float eps, int norm_by_std, float* adv, float* ret,
                                                         int estimator, const float* lens) {
  const int64_t row = blockIdx.x;
  __shared__ float s_val;
  __shared__ float s_cnt[4];
  float alpha = 1.f;
  if (estimator == DRL_ADV_GPG) {  // torch.count_nonzero(scores) over the batch, then B / max(m, 1)
    float c = 0.f;
    for (int64_t i = threadIdx.x; i < B; i += blockDim.x) c += scores[i] != 0.f ? 1.f : 0.f;
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = c;
    __syncthreads();
    const float m = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
    alpha = static_cast<float>(B) / fmaxf(m, 1.f);
  }
  if (threadIdx.x == 0) {
    const int g = row_group[row];
    const int b = off[g], e = off[g + 1], n = e - b;
    float mean = 0.f, stdv = 1.f;
    if (n > 1) {
      float sum = 0.f;
      for (int k = b; k < e; ++k) sum += scores[mem[k]];
      mean = sum / static_cast<float>(n);
      float ss = 0.f;
      for (int k = b; k < e; ++k) {
        const float d = scores[mem[k]] - mean;
        ss += d * d;
      }
      stdv = sqrtf(ss / static_cast<float>(n - 1));
    }
    const float sc = scores[row];
    if (estimator == DRL_ADV_OPO) {
      float bsl = 0.f;
      if (n > 1) {
        float num = 0.f, den = 0.f;
        for (int k = b; k < e; ++k) {
          num += lens[mem[k]] * scores[mem[k]];
          den += lens[mem[k]];
        }
        bsl = num / den;
      }
      s_val = sc - bsl;
    } else if (estimator == DRL_ADV_GPG) {
      s_val = alpha * (sc - mean) / 1.0f;
    } else if (estimator == DRL_ADV_GRPO_PASSK) {
      // torch.topk(rewards, 2): the best member (lowest position on ties: then r_max == r_second, advantage 0
      // whichever member holds it) and the runner-up value
      int kbest = b;
      for (int k = b + 1; k < e; ++k)
        if (scores[mem[k]] > scores[mem[kbest]]) kbest = k;
      float second = -INFINITY;
      for (int k = b; k < e; ++k)
        if (k != kbest) second = fmaxf(second, scores[mem[k]]);
      float a_best = scores[mem[kbest]] - second;
      if (norm_by_std) a_best = a_best / (stdv + eps);
      s_val = mem[kbest] == row ? a_best : 0.f;
    } else if (estimator == DRL_ADV_RLOO) {
      const float fn = static_cast<float>(n), fn1 = static_cast<float>(n - 1);
      s_val = n > 1 ? (sc * fn) / fn1 - (mean * fn) / fn1 : sc;
    } else if (estimator == DRL_ADV_REINFORCE_PP_BASELINE) {
      s_val = sc - mean;
    } else {
      s_val = norm_by_std ? (sc - mean) / (stdv + eps) : sc - mean;
    }
  }
  __syncthreads();
  const float v = s_val;
  for (int64_t t = threadIdx.x; t < R; t += blockDim.x) {
    const float o = v * mask_at<MDT>(mask, row * R + t);
    adv[row * R + t] = o;
    if (ret) ret[row * R + t] = o;
  }
}

// GAE reverse scan, one thread per row (core_algos.py:237-256); also emits returns = adv + values.
// VDT = DRL_BF16: values are the critic's bf16 output (dp_critic.py:192): the reference's `gamma * nextvalues`
// is then bf16 tensor arithmetic (rounded to bf16); everything else promotes to fp32 against the fp32 rewards.
template <int MDT, int VDT>
__global__ __launch_bounds__(256) void gae_scan_kernel(const float* r, const void* vals, const void* mask, int64_t B,
                                                       int64_t R, float gamma, float lam, float* adv, float* ret) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (row >= B) return;
  float nextvalues = 0.f, lastgaelam = 0.f;
  for (int64_t t = R - 1; t >= 0; --t) {
    const int64_t i = row * R + t;
    const float m = mask_at<MDT>(mask, i);
    const float vi = VDT == DRL_BF16 ? bf16_to_f32(static_cast<const uint16_t*>(vals)[i]) : static_cast<const float*>(vals)[i];
    float gv = gamma * nextvalues;
    if (VDT == DRL_BF16) gv = bf16_to_f32(f32_to_bf16(gv));
    const float delta = r[i] + gv - vi;
    const float lg = delta + gamma * lam * lastgaelam;
    nextvalues = vi * m + (1.f - m) * nextvalues;
    lastgaelam = lg * m + (1.f - m) * lastgaelam;
    adv[i] = lastgaelam;
    ret[i] = lastgaelam + vi;
  }
}

// REINFORCE++ discounted return scan, one thread per row (core_algos.py:573-578): running = r + gamma *
// running, returns[t] = running, then running *= mask[t] (a masked token resets the carry); adv starts as a
// copy of the returns and is whitened + masked in place by masked_whiten_kernel.
template <int MDT>
__global__ __launch_bounds__(256) void rfpp_scan_kernel(const float* r, const void* mask, int64_t B, int64_t R,
                                                        float gamma, float* adv, float* ret) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (row >= B) return;
  float running = 0.f;
  for (int64_t t = R - 1; t >= 0; --t) {
    const int64_t i = row * R + t;
    running = r[i] + gamma * running;
    ret[i] = running;
    adv[i] = running;
    running = running * mask_at<MDT>(mask, i);
  }
}

// ReMax (core_algos.py:588-621), one thread per row: returns = reverse cumsum of rewards * mask (float32, from
// the last token), advantages = returns - baseline[b] * mask.
template <int MDT>
__global__ __launch_bounds__(256) void remax_scan_kernel(const float* r, const float* baseline, const void* mask,
                                                         int64_t B, int64_t R, float* adv, float* ret) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (row >= B) return;
  const float bl = baseline[row];
  float running = 0.f;
  for (int64_t t = R - 1; t >= 0; --t) {
    const int64_t i = row * R + t;
    const float m = mask_at<MDT>(mask, i);
    running += r[i] * m;
    ret[i] = running;
    adv[i] = running - bl * m;
  }
}

// masked_whiten over the whole (B, R) tensor in place: mean, unbiased var, (x - mean) * rsqrt(var + 1e-8).
// One workgroup (the tensor is one PPO batch of advantages, a few MB); three ordered passes.
template <int MDT>
__global__ __launch_bounds__(1024) void masked_whiten_kernel(float* x, const void* mask, int64_t n, int* err,
                                                             float* copy = nullptr, int times_mask = 0) {
  __shared__ double red[16][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double s = 0.0, c = 0.0;
  for (int64_t i = tid; i < n; i += 1024) {
    const float m = mask_at<MDT>(mask, i);
    s += (m != 0.f) ? static_cast<double>(x[i]) * m : 0.0;
    c += m;
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (lane == 0) { red[wave][0] = s; red[wave][1] = c; }
  __syncthreads();
  double S = 0, C = 0;
  for (int w = 0; w < 16; ++w) { S += red[w][0]; C += red[w][1]; }
  __syncthreads();
  const float mean = static_cast<float>(S / (C + 1e-8));
  double q = 0.0;
  for (int64_t i = tid; i < n; i += 1024) {
    const float m = mask_at<MDT>(mask, i);
    const double d = static_cast<double>(x[i] - mean);
    q += (m != 0.f) ? d * d * m : 0.0;
  }
  q = wave_sum(q);
  if (lane == 0) red[wave][0] = q;
  __syncthreads();
  double Q = 0;
  for (int w = 0; w < 16; ++w) Q += red[w][0];
  if (tid == 0 && (C == 0.0 || C == 1.0)) *err = 1;  // the reference raises ValueError
  const double var = Q / (C + 1e-8) * (C / (C - 1.0));
  const float rs = static_cast<float>(1.0 / sqrt(var + 1e-8));
  for (int64_t i = tid; i < n; i += 1024) {
    float v = (x[i] - mean) * rs;
    if (times_mask) v *= mask_at<MDT>(mask, i);  // RF++-baseline: masked_whiten(...) * response_mask
    x[i] = v;
    if (copy) copy[i] = v;
  }
}

}  // namespace
}  // namespace drl

extern "C" {

size_t drl_grpo_workspace_bytes(int64_t B) { return drl::round_up(static_cast<size_t>(B) * sizeof(float), 256); }

int drl_grpo_outcome_advantage(const float* rewards, const void* mask, int32_t mdt, const int32_t* row_group,
                               const int32_t* group_offsets, const int32_t* group_members, int64_t B, int64_t R,
                               int64_t G, float epsilon, int32_t norm_adv_by_std, float* advantages, float* returns,
                               void* workspace, size_t workspace_bytes, void* stream) {
  return drl_group_outcome_advantage(rewards, mask, mdt, row_group, group_offsets, group_members, B, R, G, DRL_ADV_GRPO,
                                     epsilon, norm_adv_by_std, advantages, returns, workspace, workspace_bytes, stream);
}

size_t drl_group_outcome_advantage_workspace_bytes(int64_t B) {
  return 2 * drl::round_up(static_cast<size_t>(B) * sizeof(float), 256) + 256;
}

int drl_group_outcome_advantage(const float* rewards, const void* mask, int32_t mdt, const int32_t* row_group,
                                const int32_t* group_offsets, const int32_t* group_members, int64_t B, int64_t R,
                                int64_t G, int32_t estimator, float epsilon, int32_t norm_adv_by_std,
                                float* advantages, float* returns, void* workspace, size_t workspace_bytes,
                                void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(estimator >= DRL_ADV_GRPO && estimator <= DRL_ADV_GRPO_PASSK, "unknown group estimator %d", estimator);
  DRL_CHECK_ARG((estimator != DRL_ADV_REINFORCE_PP_BASELINE && estimator != DRL_ADV_OPO) ||
                    workspace_bytes >= drl_group_outcome_advantage_workspace_bytes(B),
                "workspace too small for the whitening pass / the response lengths");
  DRL_CHECK_ARG(rewards && mask && row_group && group_offsets && group_members && advantages, "NULL input");
  DRL_CHECK_ARG(B >= 1 && R >= 1 && G >= 1 && G <= B, "bad shape B=%lld R=%lld G=%lld", (long long)B, (long long)R,
                (long long)G);
  DRL_CHECK_ARG(mdt == DRL_I64 || mdt == DRL_I32 || mdt == DRL_U8 || mdt == DRL_F32, "bad mask dtype");
  if (workspace == nullptr || workspace_bytes < drl_grpo_workspace_bytes(B))
    return fail(DRL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* scores = static_cast<float*>(workspace);
  int* err = reinterpret_cast<int*>(static_cast<char*>(workspace) + round_up(static_cast<size_t>(B) * sizeof(float), 256));
  float* lens = reinterpret_cast<float*>(static_cast<char*>(workspace) + round_up(static_cast<size_t>(B) * sizeof(float), 256) + 256);
  if (estimator == DRL_ADV_REINFORCE_PP_BASELINE) DRL_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  if (estimator != DRL_ADV_OPO) {
    hipLaunchKernelGGL(row_sum_kernel, dim3((B + 3) / 4), dim3(256), 0, s, rewards, B, R, scores);
    DRL_LAUNCH_CHECK();
  }
#define DRL_GRPO(MDT)                                                                                              \
  if (estimator == DRL_ADV_OPO)                                                                                    \
    hipLaunchKernelGGL(row_sum_len_kernel<MDT>, dim3((B + 3) / 4), dim3(256), 0, s, rewards, mask, B, R, scores,    \
                       lens);                                                                                      \
  hipLaunchKernelGGL(grpo_write_kernel<MDT>, dim3(B), dim3(256), 0, s, scores, mask, row_group, group_offsets,       \
                     group_members, B, R, epsilon, norm_adv_by_std, advantages,                                   \
                     estimator == DRL_ADV_REINFORCE_PP_BASELINE ? nullptr : returns, estimator, lens);             \
  if (estimator == DRL_ADV_REINFORCE_PP_BASELINE)                                                                  \
    hipLaunchKernelGGL(masked_whiten_kernel<MDT>, dim3(1), dim3(1024), 0, s, advantages, mask, B * R, err, returns, 1)
  switch (mdt) {
    case DRL_I64: DRL_GRPO(DRL_I64); break;
    case DRL_I32: DRL_GRPO(DRL_I32); break;
    case DRL_U8: DRL_GRPO(DRL_U8); break;
    default: DRL_GRPO(DRL_F32); break;
  }
#undef DRL_GRPO
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_gae_workspace_bytes(int64_t B, int64_t R) {
  (void)B;
  (void)R;
  return 256;
}

int drl_gae_advantage_return(const float* rewards, const void* values, int32_t values_dtype, const void* mask,
                             int32_t mdt, int64_t B, int64_t R, float gamma, float lam, float* advantages,
                             float* returns, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(rewards && values && mask && advantages && returns, "NULL input");
  DRL_CHECK_ARG(values_dtype == DRL_F32 || values_dtype == DRL_BF16, "values dtype must be F32 or BF16");
  DRL_CHECK_ARG(B >= 1 && R >= 1, "bad shape");
  DRL_CHECK_ARG(mdt == DRL_I64 || mdt == DRL_I32 || mdt == DRL_U8 || mdt == DRL_F32, "bad mask dtype");
  if (workspace == nullptr || workspace_bytes < drl_gae_workspace_bytes(B, R))
    return fail(DRL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  int* err = static_cast<int*>(workspace);
  DRL_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
#define DRL_GAE(MDT)                                                                                               \
  if (values_dtype == DRL_BF16)                                                                                    \
    hipLaunchKernelGGL((gae_scan_kernel<MDT, DRL_BF16>), dim3((B + 255) / 256), dim3(256), 0, s, rewards, values,  \
                       mask, B, R, gamma, lam, advantages, returns);                                               \
  else                                                                                                             \
    hipLaunchKernelGGL((gae_scan_kernel<MDT, DRL_F32>), dim3((B + 255) / 256), dim3(256), 0, s, rewards, values,   \
                       mask, B, R, gamma, lam, advantages, returns);                                               \
  hipLaunchKernelGGL(masked_whiten_kernel<MDT>, dim3(1), dim3(1024), 0, s, advantages, mask, B * R, err)
  switch (mdt) {
    case DRL_I64: DRL_GAE(DRL_I64); break;
    case DRL_I32: DRL_GAE(DRL_I32); break;
    case DRL_U8: DRL_GAE(DRL_U8); break;
    default: DRL_GAE(DRL_F32); break;
  }
#undef DRL_GAE
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_reinforce_pp_advantage_return(const float* rewards, const void* mask, int32_t mdt, int64_t B, int64_t R,
                                      float gamma, float* advantages, float* returns, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(rewards && mask && advantages && returns, "NULL input");
  DRL_CHECK_ARG(B >= 1 && R >= 1, "bad shape");
  DRL_CHECK_ARG(mdt == DRL_I64 || mdt == DRL_I32 || mdt == DRL_U8 || mdt == DRL_F32, "bad mask dtype");
  if (workspace == nullptr || workspace_bytes < drl_gae_workspace_bytes(B, R))
    return fail(DRL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  int* err = static_cast<int*>(workspace);
  DRL_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
#define DRL_RFPP(MDT)                                                                                             \
  hipLaunchKernelGGL(rfpp_scan_kernel<MDT>, dim3((B + 255) / 256), dim3(256), 0, s, rewards, mask, B, R, gamma,     \
                     advantages, returns);                                                                         \
  hipLaunchKernelGGL(masked_whiten_kernel<MDT>, dim3(1), dim3(1024), 0, s, advantages, mask, B * R, err, nullptr, 1)
  switch (mdt) {
    case DRL_I64: DRL_RFPP(DRL_I64); break;
    case DRL_I32: DRL_RFPP(DRL_I32); break;
    case DRL_U8: DRL_RFPP(DRL_U8); break;
    default: DRL_RFPP(DRL_F32); break;
  }
#undef DRL_RFPP
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_remax_advantage_return(const float* rewards, const float* reward_baselines, const void* mask, int32_t mdt,
                               int64_t B, int64_t R, float* advantages, float* returns, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(rewards && reward_baselines && mask && advantages && returns, "NULL input");
  DRL_CHECK_ARG(B >= 1 && R >= 1, "bad shape");
  DRL_CHECK_ARG(mdt == DRL_I64 || mdt == DRL_I32 || mdt == DRL_U8 || mdt == DRL_F32, "bad mask dtype");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(static_cast<unsigned>((B + 255) / 256));
  switch (mdt) {
    case DRL_I64: hipLaunchKernelGGL(remax_scan_kernel<DRL_I64>, g, dim3(256), 0, s, rewards, reward_baselines, mask, B, R, advantages, returns); break;
    case DRL_I32: hipLaunchKernelGGL(remax_scan_kernel<DRL_I32>, g, dim3(256), 0, s, rewards, reward_baselines, mask, B, R, advantages, returns); break;
    case DRL_U8: hipLaunchKernelGGL(remax_scan_kernel<DRL_U8>, g, dim3(256), 0, s, rewards, reward_baselines, mask, B, R, advantages, returns); break;
    default: hipLaunchKernelGGL(remax_scan_kernel<DRL_F32>, g, dim3(256), 0, s, rewards, reward_baselines, mask, B, R, advantages, returns); break;
  }
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
