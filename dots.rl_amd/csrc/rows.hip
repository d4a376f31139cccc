// Row gather / scatter for the remove-padding (varlen) passes: the reference's unpad_input / pad_input /
// index_first_axis (flash_attn.bert_padding, used by dp_actor.py:119-247 and dp_critic.py:69-107 when
// use_remove_padding=True) — copies whole rows between a padded (B*T, C) layout and a packed (nnz, C) one through a
// row index map. One wave per row, 16-B lanes; an index < 0 skips the row.
#include "common.h"

namespace drl {
namespace {

__global__ __launch_bounds__(256) void copy_rows_kernel(const uint8_t* src, int64_t ld_src, const int64_t* src_idx,
                                                        uint8_t* dst, int64_t ld_dst, const int64_t* dst_idx, int64_t n,
                                                        int64_t row_bytes) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t s = src_idx ? src_idx[i] : i;
  const int64_t d = dst_idx ? dst_idx[i] : i;
  if (s < 0 || d < 0) return;
  const uint4* sp = reinterpret_cast<const uint4*>(src + s * ld_src);
  uint4* dp = reinterpret_cast<uint4*>(dst + d * ld_dst);
  for (int64_t c = threadIdx.x & 63; c < row_bytes / 16; c += 64) dp[c] = sp[c];
}

}  // namespace
}  // namespace drl

extern "C" int drl_copy_rows(const void* src, int64_t ld_src_bytes, const int64_t* src_idx, void* dst,
                             int64_t ld_dst_bytes, const int64_t* dst_idx, int64_t n_rows, int64_t row_bytes,
                             void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(src && dst && n_rows >= 0 && row_bytes >= 16 && row_bytes % 16 == 0, "rows of 16-byte multiples");
  DRL_CHECK_ARG(aligned16(src) && aligned16(dst) && ld_src_bytes % 16 == 0 && ld_dst_bytes % 16 == 0 &&
                ld_src_bytes >= row_bytes && ld_dst_bytes >= row_bytes, "16-byte aligned rows");
  if (n_rows == 0) return DRL_OK;
  hipLaunchKernelGGL(copy_rows_kernel, dim3(static_cast<unsigned>((n_rows + 3) / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(src), ld_src_bytes, src_idx,
                     static_cast<uint8_t*>(dst), ld_dst_bytes, dst_idx, n_rows, row_bytes);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}
