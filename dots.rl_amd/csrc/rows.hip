// Row gather / scatter for the remove-padding (varlen) passes: the reference's unpad_input / pad_input /
// index_first_axis (flash_attn.bert_padding, used by dp_actor.py:119-247 and dp_critic.py:69-107 when
// use_remove_padding=True) — copies whole rows between a padded (B*T, C) layout and a packed (nnz, C) one through a
// row index map. One wave per row, 16-B lanes; an index < 0 skips the row.
#include "common.h"

namespace drl {
namespace {

// ZERO: a negative source index writes a zero row (the gather writes every destination row, so the caller's
// buffer needs no memset first); otherwise a negative index skips the row
template <bool ZERO>
__global__ __launch_bounds__(256) void copy_rows_kernel(const uint8_t* src, int64_t ld_src, const int64_t* src_idx,
                                                        uint8_t* dst, int64_t ld_dst, const int64_t* dst_idx, int64_t n,
                                                        int64_t row_bytes) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t s = src_idx ? src_idx[i] : i;
  const int64_t d = dst_idx ? dst_idx[i] : i;
  if (d < 0 || (!ZERO && s < 0)) return;
  uint4* dp = reinterpret_cast<uint4*>(dst + d * ld_dst);
  if (ZERO && s < 0) {
    for (int64_t c = threadIdx.x & 63; c < row_bytes / 16; c += 64) dp[c] = uint4{0u, 0u, 0u, 0u};
    return;
  }
  const uint4* sp = reinterpret_cast<const uint4*>(src + s * ld_src);
  for (int64_t c = threadIdx.x & 63; c < row_bytes / 16; c += 64) dp[c] = sp[c];
}

// dst[dst_idx[j]] = sum over k < K of src[src_idx[k * m + j]] (index < 0: no term), fp32 accumulation in k order:
// the gradient of a packed row that K padded positions read (a prompt token shared by a group's samples). One wave
// per output row, 16-B lanes (8 bf16 / 4 fp32 elements).
template <typename T>
__global__ __launch_bounds__(256) void sum_rows_kernel(const T* src, int64_t ld_src, const int64_t* src_idx,
                                                       int64_t K, T* dst, int64_t ld_dst, const int64_t* dst_idx,
                                                       int64_t m, int64_t cols) {
  constexpr int E = 16 / sizeof(T);
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (j >= m) return;
  const int64_t d = dst_idx ? dst_idx[j] : j;
  if (d < 0) return;
  for (int64_t c = (threadIdx.x & 63) * E; c < cols; c += 64 * E) {
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    for (int64_t k = 0; k < K; ++k) {
      const int64_t s = src_idx[k * m + j];
      if (s < 0) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(src + s * ld_src + c);
      if constexpr (sizeof(T) == 2) {
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += bf16_to_f32(h[e]);
      } else {
        const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += f[e];
      }
    }
    uint4 o;
    if constexpr (sizeof(T) == 2) {
      uint16_t* h = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
      for (int e = 0; e < E; ++e) h[e] = f32_to_bf16(acc[e]);
    } else {
      float* f = reinterpret_cast<float*>(&o);
#pragma unroll
      for (int e = 0; e < E; ++e) f[e] = acc[e];
    }
    *reinterpret_cast<uint4*>(dst + d * ld_dst + c) = o;
  }
}

}  // namespace
}  // namespace drl

extern "C" int drl_sum_rows(const void* src, int64_t ld_src, const int64_t* src_idx, int64_t K, void* dst,
                            int64_t ld_dst, const int64_t* dst_idx, int64_t m, int64_t cols, int32_t dt,
                            void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(src && dst && src_idx && K >= 1 && m >= 0 && cols >= 1, "NULL operand or empty shape");
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "bf16 or fp32 rows");
  const int64_t e = dt == DRL_BF16 ? 8 : 4;
  DRL_CHECK_ARG(cols % e == 0 && ld_src % e == 0 && ld_dst % e == 0 && ld_src >= cols && ld_dst >= cols &&
                    aligned16(src) && aligned16(dst),
                "16-byte aligned rows of 16-byte multiples");
  if (m == 0) return DRL_OK;
  const dim3 grid(static_cast<unsigned>((m + 3) / 4));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dt == DRL_BF16)
    hipLaunchKernelGGL(sum_rows_kernel<uint16_t>, grid, dim3(256), 0, s, static_cast<const uint16_t*>(src), ld_src,
                       src_idx, K, static_cast<uint16_t*>(dst), ld_dst, dst_idx, m, cols);
  else
    hipLaunchKernelGGL(sum_rows_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(src), ld_src, src_idx,
                       K, static_cast<float*>(dst), ld_dst, dst_idx, m, cols);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

extern "C" int drl_copy_rows(const void* src, int64_t ld_src_bytes, const int64_t* src_idx, void* dst,
                             int64_t ld_dst_bytes, const int64_t* dst_idx, int64_t n_rows, int64_t row_bytes,
                             void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(src && dst && n_rows >= 0 && row_bytes >= 16 && row_bytes % 16 == 0, "rows of 16-byte multiples");
  DRL_CHECK_ARG(aligned16(src) && aligned16(dst) && ld_src_bytes % 16 == 0 && ld_dst_bytes % 16 == 0 &&
                ld_src_bytes >= row_bytes && ld_dst_bytes >= row_bytes, "16-byte aligned rows");
  if (n_rows == 0) return DRL_OK;
  hipLaunchKernelGGL(copy_rows_kernel<false>, dim3(static_cast<unsigned>((n_rows + 3) / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(src), ld_src_bytes, src_idx,
                     static_cast<uint8_t*>(dst), ld_dst_bytes, dst_idx, n_rows, row_bytes);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

extern "C" int drl_gather_rows(const void* src, int64_t ld_src_bytes, const int64_t* src_idx, void* dst,
                               int64_t ld_dst_bytes, int64_t n_rows, int64_t row_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(src && dst && src_idx && n_rows >= 0 && row_bytes >= 16 && row_bytes % 16 == 0,
                "rows of 16-byte multiples, a source index map");
  DRL_CHECK_ARG(aligned16(src) && aligned16(dst) && ld_src_bytes % 16 == 0 && ld_dst_bytes % 16 == 0 &&
                ld_src_bytes >= row_bytes && ld_dst_bytes >= row_bytes, "16-byte aligned rows");
  if (n_rows == 0) return DRL_OK;
  hipLaunchKernelGGL(copy_rows_kernel<true>, dim3(static_cast<unsigned>((n_rows + 3) / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(src), ld_src_bytes, src_idx,
                     static_cast<uint8_t*>(dst), ld_dst_bytes, nullptr, n_rows, row_bytes);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}
