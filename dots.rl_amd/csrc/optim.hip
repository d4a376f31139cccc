// A15 — optimizer step on the flat fp32 master buffer: global grad norm, clip, skip-if-non-finite, AdamW,
// and the bf16 compute copy refreshed in the same pass.
// References: verl/workers/actor/dp_actor.py:282-298 (_optimizer_step: clip_grad_norm_, finite check,
// step), verl/workers/fsdp_workers.py:454-459 (AdamW hyper-parameters); torch.optim.AdamW semantics
// (decoupled weight decay, lerp first moment, bias-corrected denominator) and
// torch.nn.utils.clip_grad_norm_ (coef = max_norm / (norm + 1e-6), clamped to 1).
// HBM-bound: the step reads param+grad+m+v (16 B) and writes param+m+v (+bf16 copy) (12-14 B) per element.
#include "common.h"

namespace drl {
namespace {

constexpr int kThreads = 256;

struct NormHeader {
  unsigned ticket;
  unsigned pad[3];
};

__global__ __launch_bounds__(kThreads) void sumsq_kernel(const float* g, int64_t n, double* partials, NormHeader* hdr,
                                                         float* out_norm) {
  const int64_t n4 = n / 4;
  double acc = 0.0;
  float facc = 0.f;
  int cnt = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * kThreads) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    facc = fmaf(v.x, v.x, facc);
    facc = fmaf(v.y, v.y, facc);
    facc = fmaf(v.z, v.z, facc);
    facc = fmaf(v.w, v.w, facc);
    if (++cnt == 64) { acc += facc; facc = 0.f; cnt = 0; }
  }
  for (int64_t i = n4 * 4 + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * kThreads)
    facc = fmaf(g[i], g[i], facc);
  acc += facc;
  acc = wave_sum(acc);
  __shared__ double red[kThreads / kWave];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) store_sc1(partials + blockIdx.x, red[0] + red[1] + red[2] + red[3]);
  if (last_block_ticket(&hdr->ticket)) {
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (unsigned b = 0; b < gridDim.x; ++b) s += load_sc1(partials + b);
      *out_norm = static_cast<float>(sqrt(s));
    }
  }
}

struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  uint16_t* pbf;
  int64_t n;
  float lr, beta1, beta2, eps, wd, step_size, bc2_sqrt, max_norm;
  const float* norm;
};

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float coef, const AdamArgs& a) {
  g *= coef;
  p = p * (1.f - a.lr * a.wd);
  m = m + (1.f - a.beta1) * (g - m);  // torch.lerp(m, g, 1 - beta1) with weight < 0.5
  v = v * a.beta2 + (1.f - a.beta2) * (g * g);
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + (-a.step_size) * (m / denom);
}

__global__ __launch_bounds__(kThreads) void adamw_kernel(AdamArgs a) {
  float coef = 1.f;
  if (a.norm) {
    const float nrm = *a.norm;
    if (!isfinite(nrm)) return;  // dp_actor.py:292-297: non-finite grad norm -> skip the step
    if (a.max_norm > 0.f) coef = fminf(a.max_norm / (nrm + 1e-6f), 1.f);
  }
  const int64_t n4 = a.n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<float4*>(a.p)[i];
    const float4 g = reinterpret_cast<const float4*>(a.g)[i];
    float4 m = reinterpret_cast<float4*>(a.m)[i];
    float4 v = reinterpret_cast<float4*>(a.v)[i];
    adam_one(p.x, g.x, m.x, v.x, coef, a);
    adam_one(p.y, g.y, m.y, v.y, coef, a);
    adam_one(p.z, g.z, m.z, v.z, coef, a);
    adam_one(p.w, g.w, m.w, v.w, coef, a);
    reinterpret_cast<float4*>(a.p)[i] = p;
    reinterpret_cast<float4*>(a.m)[i] = m;
    reinterpret_cast<float4*>(a.v)[i] = v;
    if (a.pbf) {
      const uint32_t lo = static_cast<uint32_t>(f32_to_bf16(p.x)) | (static_cast<uint32_t>(f32_to_bf16(p.y)) << 16);
      const uint32_t hi = static_cast<uint32_t>(f32_to_bf16(p.z)) | (static_cast<uint32_t>(f32_to_bf16(p.w)) << 16);
      reinterpret_cast<uint2*>(a.pbf)[i] = make_uint2(lo, hi);
    }
  }
  for (int64_t i = n4 * 4 + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < a.n; i += stride) {
    adam_one(a.p[i], a.g[i], a.m[i], a.v[i], coef, a);
    if (a.pbf) a.pbf[i] = f32_to_bf16(a.p[i]);
  }
}

int grid_for(int64_t n4) {
  const int64_t want = (n4 + kThreads - 1) / kThreads;
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(want, static_cast<int64_t>(cu_count()) * 8)));
}

}  // namespace
}  // namespace drl

extern "C" {

size_t drl_grad_norm_workspace_bytes(int64_t n) {
  (void)n;
  return drl::round_up(sizeof(drl::NormHeader), 256) + static_cast<size_t>(drl::cu_count()) * 8 * sizeof(double);
}

int drl_grad_norm(const float* grads, int64_t n, float* out_norm, void* workspace, size_t workspace_bytes,
                  void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(grads && out_norm, "NULL input");
  DRL_CHECK_ARG(n >= 1, "empty gradient");
  DRL_CHECK_ARG(aligned16(grads), "grads not 16-byte aligned");
  if (workspace == nullptr || workspace_bytes < drl_grad_norm_workspace_bytes(n))
    return fail(DRL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* hdr = static_cast<NormHeader*>(workspace);
  auto* partials = reinterpret_cast<double*>(static_cast<char*>(workspace) + round_up(sizeof(NormHeader), 256));
  DRL_HIP(hipMemsetAsync(hdr, 0, sizeof(NormHeader), s));
  const int grid = grid_for(n / 4 + 1);
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid), dim3(kThreads), 0, s, grads, n, partials, hdr, out_norm);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_adamw_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, uint16_t* params_bf16,
                   int64_t n, const drl_adamw_params* hp, const float* grad_norm, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && hp, "NULL input");
  DRL_CHECK_ARG(n >= 1 && hp->step >= 1, "bad size/step");
  DRL_CHECK_ARG(aligned16(params) && aligned16(grads) && aligned16(exp_avg) && aligned16(exp_avg_sq) &&
                    (params_bf16 == nullptr || (reinterpret_cast<uintptr_t>(params_bf16) & 7u) == 0),
                "buffers not aligned");
  AdamArgs a{};
  a.p = params; a.g = grads; a.m = exp_avg; a.v = exp_avg_sq; a.pbf = params_bf16; a.n = n;
  a.lr = hp->lr; a.beta1 = hp->beta1; a.beta2 = hp->beta2; a.eps = hp->eps; a.wd = hp->weight_decay;
  const double bc1 = 1.0 - std::pow(static_cast<double>(hp->beta1), hp->step);
  const double bc2 = 1.0 - std::pow(static_cast<double>(hp->beta2), hp->step);
  a.step_size = static_cast<float>(static_cast<double>(hp->lr) / bc1);
  a.bc2_sqrt = static_cast<float>(std::sqrt(bc2));
  a.max_norm = hp->max_grad_norm;
  a.norm = grad_norm;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n / 4 + 1)), dim3(kThreads), 0, s, a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
