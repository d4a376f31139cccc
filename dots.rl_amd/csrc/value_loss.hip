// K6 — critic: fused clipped value loss (forward + backward in one launch) and the scalar value head.
// References: verl/trainer/ppo/core_algos.py:1230-1269 (compute_value_loss), 703-736 (agg_loss),
// verl/utils/torch_functional.py:136-142 (clip_by_value), 163-185 (masked_mean);
// verl/workers/critic/dp_critic.py:57-145 (values = score(h)[:, -R-1:-1]), 206-245 (loss * loss_scale_factor,
// backward, critic/vf_loss, vf_clipfrac, vpred_mean). The value head is HF GenericForTokenClassification's
// `score` Linear(H, 1, bias=True) (the critic the reference builds with AutoModelForTokenClassification).
//
// vpreds / values arrive in the critic's output dtype (bf16 under the reference's autocast, or fp32):
// clip bounds are `values -/+ cliprange` rounded to that dtype (bf16 tensor - python float stays bf16),
// the squared errors are fp32 against fp32 returns, exactly the reference's promotion order. Tokens are
// few (micro-batch x R): one thread per token, grid-stride, per-workgroup partials folded by the last
// workgroup in a fixed order (bitwise reproducible). token-mean needs sum(mask) before any gradient, so a
// row-count pre-pass (one wave per row) runs first and every workgroup sums the B row counts itself, in
// the same fixed order.
#include "common.h"

namespace drl {
namespace {

constexpr int kThreads = 256;
constexpr int kParts = 4;  // loss sum, clipfrac sum, masked vpred sum, mask count

struct Header {
  unsigned ticket;
  unsigned pad[7];
};

template <int DT>
__device__ __forceinline__ float ld_val(const void* p, int64_t i) {
  if constexpr (DT == DRL_BF16) return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
  else return static_cast<const float*>(p)[i];
}
// value in the tensor's dtype (python-float arithmetic on a bf16 tensor rounds back to bf16)
template <int DT>
__device__ __forceinline__ float round_dt(float x) {
  if constexpr (DT == DRL_BF16) return bf16_to_f32(f32_to_bf16(x));
  else return x;
}

template <int MDT>
__global__ __launch_bounds__(256) void vl_row_count_kernel(const void* mask, int64_t B, int64_t R, float* rowcnt) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float c = 0.f;
  for (int64_t t = lane; t < R; t += 64) c += mask_at<MDT>(mask, row * R + t);
  c = wave_sum(c);
  if (lane == 0) rowcnt[row] = c;
}

struct VArgs {
  const void* vpreds;
  const void* values;
  const float* returns;
  const void* mask;
  const float* rowcnt;
  float* dv;
  float* out;
  Header* hdr;
  double* partials;
  int64_t B, R;
  float clip, lsf;
  int mode;
};

template <int VDT, int MDT>
__global__ __launch_bounds__(kThreads) void value_loss_kernel(VArgs a) {
  __shared__ double red[kThreads / kWave][kParts];
  __shared__ float s_total;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t N = a.B * a.R;
  const bool tm = a.mode == DRL_AGG_TOKEN_MEAN, smtm = a.mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN;
  if (tm) {  // sum(mask) in a fixed order (same in every workgroup): wave 0 reduces the row counts
    if (wave == 0) {
      double c = 0.0;
      for (int64_t b = lane; b < a.B; b += 64) c += a.rowcnt[b];
      c = wave_sum(c);
      if (lane == 0) s_total = static_cast<float>(c);
    }
    __syncthreads();
  }
  const float inv_dtm = tm ? 1.0f / (s_total + 1e-8f) : 0.f;
  const float inv_B = 1.0f / static_cast<float>(a.B), inv_R = 1.0f / static_cast<float>(a.R);
  float s_loss = 0.f, s_clip = 0.f, s_v = 0.f, s_cnt = 0.f;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + tid; t < N;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const float v = ld_val<VDT>(a.vpreds, t);
    const float old = ld_val<VDT>(a.values, t);
    const float ret = a.returns[t];
    const float m = mask_at<MDT>(a.mask, t);
    const bool mb = m != 0.f;
    // clip_by_value = torch.max(torch.min(x, values + c), values - c), bounds in the value dtype
    // (the python-float cliprange takes the tensor's dtype first: torch's bf16 tensor-scalar arithmetic as the
    // golden vectors record it; a no-op for fp32)
    const float cv = round_dt<VDT>(a.clip);
    const float hi = round_dt<VDT>(old + cv), lo = round_dt<VDT>(old - cv);
    const float y = fminf(v, hi);
    const float gy = v < hi ? 1.f : (v == hi ? 0.5f : 0.f);  // torch.minimum splits ties
    const float vc = fmaxf(y, lo);
    const float gc = y > lo ? 1.f : (y == lo ? 0.5f : 0.f);
    const float e1 = v - ret, e2 = vc - ret;
    const float l1 = e1 * e1, l2 = e2 * e2;
    const float lmax = fmaxf(l1, l2);
    const float w1 = l1 > l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
    // d max(l1, l2) / d vpred
    const float dl = w1 * (2.f * e1) + (1.f - w1) * (2.f * e2) * (gy * gc);
    float rc_inv = smtm ? 1.0f / a.rowcnt[t / a.R] : 0.f;
    float w;  // d agg / d loss_mat
    if (tm) w = mb ? inv_dtm * m : 0.f;
    else if (a.mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM) w = inv_B * m;
    else if (smtm) w = m * (inv_B * rc_inv);
    else w = inv_R * m;
    float val;  // forward contribution (core_algos.py:716-733 op order)
    if (tm) val = mb ? lmax * m : 0.f;
    else if (smtm) val = (lmax * m) * rc_inv;
    else val = lmax * m;
    s_loss += val;
    s_clip += (mb && l2 > l1) ? m : 0.f;
    s_v += mb ? v * m : 0.f;
    s_cnt += m;
    if (a.dv) a.dv[t] = a.lsf * 0.5f * (w * dl);
  }
  const float vals[kParts] = {s_loss, s_clip, s_v, s_cnt};
#pragma unroll
  for (int k = 0; k < kParts; ++k) {
    const double r = wave_sum(static_cast<double>(vals[k]));
    if (lane == 0) red[wave][k] = r;
  }
  __syncthreads();
  if (tid < kParts)
    store_sc1(a.partials + tid * gridDim.x + blockIdx.x, red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid]);
  if (last_block_ticket(&a.hdr->ticket)) {
#pragma unroll
    for (int k = 0; k < kParts; ++k) {
      double r = 0.0;
      for (unsigned g = tid; g < gridDim.x; g += kThreads) r += load_sc1(a.partials + k * gridDim.x + g);
      r = wave_sum(r);
      if (lane == 0) red[wave][k] = r;
    }
    __syncthreads();
    if (tid == 0) {
      double r[kParts];
      for (int k = 0; k < kParts; ++k) r[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
      const double dm = static_cast<double>(static_cast<float>(r[3]) + 1e-8f);
      double agg;
      if (a.mode == DRL_AGG_TOKEN_MEAN) agg = r[0] / dm;
      else if (a.mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM || a.mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) agg = r[0] / static_cast<double>(a.B);
      else agg = r[0] / static_cast<double>(a.R);
      const double vf_loss = 0.5 * agg;
      a.out[DRL_VALUE_OUT_VF_LOSS] = static_cast<float>(vf_loss);
      a.out[DRL_VALUE_OUT_VF_CLIPFRAC] = static_cast<float>(r[1] / dm);
      // masked_mean over a bf16 tensor: the masked sum is a bf16 tensor (rounded), the quotient by the fp32
      // (mask.sum() + 1e-8) promotes to fp32
      a.out[DRL_VALUE_OUT_VPRED_MEAN] = VDT == DRL_BF16
          ? round_dt<VDT>(static_cast<float>(r[2])) / static_cast<float>(dm)
          : static_cast<float>(r[2] / dm);
      a.out[DRL_VALUE_OUT_LOSS] = static_cast<float>(vf_loss * a.lsf);
      a.out[DRL_VALUE_OUT_MASK_COUNT] = static_cast<float>(r[3]);
    }
  }
}

struct Layout {
  size_t partials, rowcnt, total;
};
int vl_grid(int64_t N) {
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(static_cast<int64_t>(cu_count()) * 4,
                                                                 (N + kThreads - 1) / kThreads)));
}
Layout vl_layout(int64_t B, int64_t R) {
  Layout L{};
  L.partials = round_up(sizeof(Header), 256);
  L.rowcnt = round_up(L.partials + static_cast<size_t>(vl_grid(B * R)) * kParts * sizeof(double), 256);
  L.total = round_up(L.rowcnt + static_cast<size_t>(B) * sizeof(float), 256);
  return L;
}

template <int VDT, int MDT>
int vl_launch(VArgs a, hipStream_t s) {
  const bool need_rows = a.mode == DRL_AGG_TOKEN_MEAN || a.mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN;
  if (need_rows) {
    hipLaunchKernelGGL(vl_row_count_kernel<MDT>, dim3((a.B + 3) / 4), dim3(256), 0, s, a.mask, a.B, a.R,
                       const_cast<float*>(a.rowcnt));
    DRL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL((value_loss_kernel<VDT, MDT>), dim3(vl_grid(a.B * a.R)), dim3(kThreads), 0, s, a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

template <int VDT>
int vl_dispatch_mask(VArgs a, int mdt, hipStream_t s) {
  switch (mdt) {
    case DRL_I64: return vl_launch<VDT, DRL_I64>(a, s);
    case DRL_I32: return vl_launch<VDT, DRL_I32>(a, s);
    case DRL_U8: return vl_launch<VDT, DRL_U8>(a, s);
    default: return vl_launch<VDT, DRL_F32>(a, s);
  }
}

// ---------------------------------------------------------------------------------- value head
// values[n] = dot(h[n, :], w) + b, fp32 accumulation, one wave per row, 16-B loads (8 bf16 / 4 fp32 per lane).
template <int HDT>
__global__ __launch_bounds__(256) void value_head_fwd_kernel(const void* h, int64_t ld, const void* w, const void* b,
                                                             int64_t N, int64_t H, void* out, int odt) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  float acc = 0.f;
  if constexpr (HDT == DRL_BF16) {
    const uint16_t* hr = static_cast<const uint16_t*>(h) + row * ld;
    const uint16_t* wr = static_cast<const uint16_t*>(w);
    for (int64_t k = lane * 8; k < H; k += 512) {
      const uint4 hv = *reinterpret_cast<const uint4*>(hr + k);
      const uint4 wv = *reinterpret_cast<const uint4*>(wr + k);
      const uint32_t hx[4] = {hv.x, hv.y, hv.z, hv.w}, wx[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc = fmaf(__uint_as_float(hx[j] << 16), __uint_as_float(wx[j] << 16), acc);
        acc = fmaf(__uint_as_float(hx[j] & 0xffff0000u), __uint_as_float(wx[j] & 0xffff0000u), acc);
      }
    }
  } else {
    const float* hr = static_cast<const float*>(h) + row * ld;
    const float* wr = static_cast<const float*>(w);
    for (int64_t k = lane * 4; k < H; k += 256) {
      const float4 hv = *reinterpret_cast<const float4*>(hr + k);
      const float4 wv = *reinterpret_cast<const float4*>(wr + k);
      acc = fmaf(hv.x, wv.x, acc); acc = fmaf(hv.y, wv.y, acc);
      acc = fmaf(hv.z, wv.z, acc); acc = fmaf(hv.w, wv.w, acc);
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float bias = b == nullptr ? 0.f
                                    : (HDT == DRL_BF16 ? bf16_to_f32(*static_cast<const uint16_t*>(b))
                                                       : *static_cast<const float*>(b));
    const float v = acc + bias;
    if (odt == DRL_BF16) static_cast<uint16_t*>(out)[row] = f32_to_bf16(v);
    else static_cast<float*>(out)[row] = v;
  }
}

// dh[n, k] = dv[n] * w[k] (written in h's dtype); per-workgroup column partials of sum_n dv[n] h[n, k] and
// sum_n dv[n] (bias) over the workgroup's kRowsBwd rows -> partials[wg][H + 1].
constexpr int kRowsBwd = 64;
template <int HDT>
__global__ __launch_bounds__(256) void value_head_bwd_kernel(const void* h, int64_t ld, const void* w, const float* dv,
                                                             int64_t N, int64_t H, void* dh, int64_t ld_dh,
                                                             float* partials) {
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kRowsBwd;
  const int64_t r1 = min(N, r0 + kRowsBwd);
  float* part = partials + static_cast<int64_t>(blockIdx.x) * (H + 1);
  for (int64_t k = threadIdx.x; k < H; k += blockDim.x) {
    const float wk = HDT == DRL_BF16 ? bf16_to_f32(static_cast<const uint16_t*>(w)[k]) : static_cast<const float*>(w)[k];
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const float g = dv[r];
      float hv;
      if constexpr (HDT == DRL_BF16) {
        hv = bf16_to_f32(static_cast<const uint16_t*>(h)[r * ld + k]);
        if (dh) static_cast<uint16_t*>(dh)[r * ld_dh + k] = f32_to_bf16(g * wk);
      } else {
        hv = static_cast<const float*>(h)[r * ld + k];
        if (dh) static_cast<float*>(dh)[r * ld_dh + k] = g * wk;
      }
      s = fmaf(g, hv, s);
    }
    part[k] = s;
  }
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += 64) s += dv[r];
    s = wave_sum(s);
    if (threadIdx.x == 0) part[H] = s;
  }
}

// dw[k] += sum over workgroups (fixed order) of partials[g][k]; db[0] += the bias column
__global__ __launch_bounds__(256) void value_head_wgrad_kernel(const float* partials, int64_t G, int64_t H, float* dw,
                                                               float* db) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k > H) return;
  float s = 0.f;
  for (int64_t g = 0; g < G; ++g) s += partials[g * (H + 1) + k];
  if (k < H) { if (dw) dw[k] += s; }
  else if (db) db[0] += s;
}

}  // namespace
}  // namespace drl

extern "C" {

size_t drl_value_loss_workspace_bytes(int64_t B, int64_t R) { return drl::vl_layout(B, R).total; }

int drl_value_loss_fwd_bwd(const void* vpreds, const void* values, int32_t value_dtype, const float* returns,
                           const void* response_mask, int32_t mask_dtype, int64_t B, int64_t R,
                           const drl_value_loss_params* p, float* out_scalars, float* dvpreds, void* workspace,
                           size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(p != nullptr, "params is NULL");
  DRL_CHECK_ARG(B >= 1 && R >= 1, "bad shape B=%lld R=%lld", (long long)B, (long long)R);
  DRL_CHECK_ARG(vpreds && values && returns && response_mask && out_scalars, "NULL input");
  DRL_CHECK_ARG(value_dtype == DRL_F32 || value_dtype == DRL_BF16, "value dtype must be F32 or BF16, got %d",
                value_dtype);
  DRL_CHECK_ARG(p->loss_agg_mode >= 0 && p->loss_agg_mode <= 3, "Invalid loss_agg_mode: %d", p->loss_agg_mode);
  DRL_CHECK_ARG(mask_dtype == DRL_I64 || mask_dtype == DRL_I32 || mask_dtype == DRL_U8 || mask_dtype == DRL_F32,
                "unsupported mask dtype %d", mask_dtype);
  const Layout L = vl_layout(B, R);
  if (workspace == nullptr || workspace_bytes < L.total)
    return fail(DRL_ERR_WORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, L.total);
  auto* ws = static_cast<char*>(workspace);
  VArgs a{};
  a.vpreds = vpreds; a.values = values; a.returns = returns; a.mask = response_mask;
  a.rowcnt = reinterpret_cast<const float*>(ws + L.rowcnt);
  a.dv = dvpreds; a.out = out_scalars;
  a.hdr = reinterpret_cast<Header*>(ws);
  a.partials = reinterpret_cast<double*>(ws + L.partials);
  a.B = B; a.R = R;
  a.clip = p->cliprange_value; a.lsf = p->loss_scale_factor; a.mode = p->loss_agg_mode;
  hipStream_t s = static_cast<hipStream_t>(stream);
  DRL_HIP(hipMemsetAsync(ws, 0, sizeof(Header), s));
  return value_dtype == DRL_BF16 ? vl_dispatch_mask<DRL_BF16>(a, mask_dtype, s)
                                 : vl_dispatch_mask<DRL_F32>(a, mask_dtype, s);
}

int drl_value_head_fwd(const void* hidden, int64_t ld_h, const void* weight, const void* bias, int32_t dt, int64_t N,
                       int64_t H, void* values, int32_t out_dtype, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(hidden && weight && values, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "dtype must be BF16 or F32");
  DRL_CHECK_ARG(out_dtype == DRL_BF16 || out_dtype == DRL_F32, "out dtype must be BF16 or F32");
  DRL_CHECK_ARG(N >= 0 && H >= 1 && ld_h >= H, "bad shape N=%lld H=%lld ld=%lld", (long long)N, (long long)H,
                (long long)ld_h);
  const int vec = dt == DRL_BF16 ? 8 : 4;
  DRL_CHECK_ARG(H % vec == 0 && ld_h % vec == 0 && aligned16(hidden) && aligned16(weight),
                "H and ld_h must be multiples of %d and the rows 16-byte aligned", vec);
  if (N == 0) return DRL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dt == DRL_BF16)
    hipLaunchKernelGGL(value_head_fwd_kernel<DRL_BF16>, dim3((N + 3) / 4), dim3(256), 0, s, hidden, ld_h, weight, bias,
                       N, H, values, out_dtype);
  else
    hipLaunchKernelGGL(value_head_fwd_kernel<DRL_F32>, dim3((N + 3) / 4), dim3(256), 0, s, hidden, ld_h, weight, bias,
                       N, H, values, out_dtype);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_value_head_bwd_workspace_bytes(int64_t N, int64_t H) {
  return static_cast<size_t>((N + drl::kRowsBwd - 1) / drl::kRowsBwd) * static_cast<size_t>(H + 1) * sizeof(float);
}

int drl_value_head_bwd(const void* hidden, int64_t ld_h, const void* weight, int32_t dt, const float* dvalues,
                       int64_t N, int64_t H, void* dhidden, int64_t ld_dh, float* dweight, float* dbias,
                       void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(hidden && weight && dvalues, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "dtype must be BF16 or F32");
  DRL_CHECK_ARG(N >= 0 && H >= 1 && ld_h >= H && (dhidden == nullptr || ld_dh >= H), "bad shape");
  if (N == 0) return DRL_OK;
  const size_t need = drl_value_head_bwd_workspace_bytes(N, H);
  if (workspace == nullptr || workspace_bytes < need)
    return fail(DRL_ERR_WORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t G = (N + kRowsBwd - 1) / kRowsBwd;
  float* part = static_cast<float*>(workspace);
  if (dt == DRL_BF16)
    hipLaunchKernelGGL(value_head_bwd_kernel<DRL_BF16>, dim3(G), dim3(256), 0, s, hidden, ld_h, weight, dvalues, N, H,
                       dhidden, ld_dh, part);
  else
    hipLaunchKernelGGL(value_head_bwd_kernel<DRL_F32>, dim3(G), dim3(256), 0, s, hidden, ld_h, weight, dvalues, N, H,
                       dhidden, ld_dh, part);
  DRL_LAUNCH_CHECK();
  hipLaunchKernelGGL(value_head_wgrad_kernel, dim3((H + 1 + 255) / 256), dim3(256), 0, s, part, G, H, dweight, dbias);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
