// A4/A5 — rollout bookkeeping on device: response mask from EOS, position ids from the attention mask,
// response-position continuation. References: verl/utils/torch_functional.py:226-246 (get_response_mask),
// verl/utils/model.py:219 (compute_position_id_with_mask), verl/workers/rollout/hf_rollout.py:151-160.
#include "common.h"

namespace drl {
namespace {

// mask[b, t] = 1 for t <= first eos position (inclusive), else 0. One wave per row.
template <int ODT>
__global__ __launch_bounds__(256) void response_mask_kernel(const int64_t* resp, int64_t B, int64_t R, int64_t ld,
                                                            const int64_t* eos, int n_eos, void* out, int64_t ld_out) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  int64_t first = R;  // first eos index in the row
  for (int64_t base = 0; base < R && first == R; base += 64) {
    const int64_t t = base + lane;
    bool hit = false;
    if (t < R) {
      const int64_t v = resp[row * ld + t];
      for (int k = 0; k < n_eos; ++k) hit |= (v == eos[k]);
    }
    const unsigned long long b = __ballot(hit);
    if (b) first = base + __builtin_ctzll(b);
  }
  for (int64_t t = lane; t < R; t += 64) {
    const int64_t m = t <= first ? 1 : 0;
    if constexpr (ODT == DRL_I64) static_cast<int64_t*>(out)[row * ld_out + t] = m;
    else if constexpr (ODT == DRL_I32) static_cast<int32_t*>(out)[row * ld_out + t] = static_cast<int32_t>(m);
    else if constexpr (ODT == DRL_U8) static_cast<uint8_t*>(out)[row * ld_out + t] = static_cast<uint8_t>(m);
    else static_cast<float*>(out)[row * ld_out + t] = static_cast<float>(m);
  }
}

// position_ids = clip(cumsum(mask, -1) - 1, 0). One wave per row, 64-wide inclusive scans.
template <int MDT>
__global__ __launch_bounds__(256) void position_ids_kernel(const void* mask, int64_t B, int64_t T, int64_t* pos) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  int64_t carry = 0;
  for (int64_t base = 0; base < T; base += 64) {
    const int64_t t = base + lane;
    int64_t v = t < T ? static_cast<int64_t>(mask_at<MDT>(mask, row * T + t)) : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t x = __shfl_up(v, o, kWave);
      if (lane >= o) v += x;
    }
    const int64_t c = carry + v - 1;
    if (t < T) pos[row * T + t] = c < 0 ? 0 : c;
    carry += __shfl(v, 63, kWave);
  }
}

// position_ids[b, P + t] = position_ids[b, P - 1] + 1 + t  for a (B, P + R) buffer
__global__ __launch_bounds__(256) void response_pos_kernel(int64_t* pos, int64_t B, int64_t P, int64_t R) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B * R) return;
  const int64_t b = i / R, t = i % R;
  pos[b * (P + R) + P + t] = pos[b * (P + R) + P - 1] + 1 + t;
}

}  // namespace
}  // namespace drl

extern "C" {

int drl_response_mask(const int64_t* responses, int64_t B, int64_t R, int64_t ld, const int64_t* eos_ids,
                      int32_t n_eos, void* mask_out, int32_t odt, int64_t ld_out, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(responses && mask_out, "NULL input");
  DRL_CHECK_ARG(n_eos == 0 || eos_ids, "n_eos > 0 but eos_ids is NULL");
  DRL_CHECK_ARG(B >= 0 && R >= 1 && ld >= R && ld_out >= R, "bad shape");
  if (B == 0) return DRL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid((B + 3) / 4);
  switch (odt) {
    case DRL_I64: hipLaunchKernelGGL(response_mask_kernel<DRL_I64>, grid, dim3(256), 0, s, responses, B, R, ld, eos_ids, n_eos, mask_out, ld_out); break;
    case DRL_I32: hipLaunchKernelGGL(response_mask_kernel<DRL_I32>, grid, dim3(256), 0, s, responses, B, R, ld, eos_ids, n_eos, mask_out, ld_out); break;
    case DRL_U8: hipLaunchKernelGGL(response_mask_kernel<DRL_U8>, grid, dim3(256), 0, s, responses, B, R, ld, eos_ids, n_eos, mask_out, ld_out); break;
    case DRL_F32: hipLaunchKernelGGL(response_mask_kernel<DRL_F32>, grid, dim3(256), 0, s, responses, B, R, ld, eos_ids, n_eos, mask_out, ld_out); break;
    default: return fail(DRL_ERR_INVALID, "bad mask dtype %d", odt);
  }
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_position_ids(const void* mask, int32_t mdt, int64_t B, int64_t T, int64_t* pos, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(mask && pos, "NULL input");
  DRL_CHECK_ARG(B >= 0 && T >= 1, "bad shape");
  if (B == 0) return DRL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid((B + 3) / 4);
  switch (mdt) {
    case DRL_I64: hipLaunchKernelGGL(position_ids_kernel<DRL_I64>, grid, dim3(256), 0, s, mask, B, T, pos); break;
    case DRL_I32: hipLaunchKernelGGL(position_ids_kernel<DRL_I32>, grid, dim3(256), 0, s, mask, B, T, pos); break;
    case DRL_U8: hipLaunchKernelGGL(position_ids_kernel<DRL_U8>, grid, dim3(256), 0, s, mask, B, T, pos); break;
    case DRL_F32: hipLaunchKernelGGL(position_ids_kernel<DRL_F32>, grid, dim3(256), 0, s, mask, B, T, pos); break;
    default: return fail(DRL_ERR_INVALID, "bad mask dtype %d", mdt);
  }
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_response_position_ids(int64_t* pos, int64_t B, int64_t P, int64_t R, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(pos, "NULL input");
  DRL_CHECK_ARG(B >= 0 && P >= 1 && R >= 0, "bad shape");
  if (B == 0 || R == 0) return DRL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(response_pos_kernel, dim3((B * R + 255) / 256), dim3(256), 0, s, pos, B, P, R);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
