// Attention kernels of the rollout engine.
//
// decode_attention: one new query token per sequence against the KV cache, grouped-query attention
// (G = Hq / Hkv query heads per KV head, 7 for Qwen2.5-0.5B). Replaces the per-step (q K^T, softmax, P V)
// of HF generate's attention (hf_rollout.py:112-124 -> Qwen2 attention over the KV cache).
// Keys allowed: key_valid[b, j] && j <= qpos (HF: the attention mask grows by one valid key per step).
//
// HBM-bound: every (sequence, KV head) streams its K and V rows once (2 * L * D * 2 B) and nothing else
// of size leaves the chip. One workgroup per (sequence, KV head); a key row is split over TPK = D / 8
// lanes holding 8 contiguous elements (one 16-B load each for K and V), so a wave reads 64 / TPK whole
// rows per instruction, fully coalesced. Each lane group keeps an independent online softmax (running
// max m, sum l, and o[G][8]) over the keys it visits; groups are merged with shuffles inside the wave and
// through LDS across waves at the end. Loads for kUnroll keys are issued before their math.
// Split-K: the key range is cut into chunks of one pass (KPB * kUnroll keys) over grid.y, so every
// workgroup issues all of its loads at once and the whole grid keeps HBM busy; the chunks' partial
// (m, l, o) go to a workspace and decode_merge_kernel combines them in a fixed order.
#include "common.h"

namespace drl {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxG = 8;  // query heads per KV head handled by one workgroup
constexpr int kUnroll = 4;

template <typename E>
struct Vec8;  // 8 contiguous elements <-> fp32
template <>
struct Vec8<uint16_t> {
  static __device__ __forceinline__ void load(const uint16_t* p, float v[8]) {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(ww[e] << 16);
      v[2 * e + 1] = __uint_as_float(ww[e] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float v[8]) {
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = static_cast<uint32_t>(f32_to_bf16(v[2 * e])) | (static_cast<uint32_t>(f32_to_bf16(v[2 * e + 1])) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float v[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float v[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// q (B, Hkv, G, D); k/v cache (B, Hkv, Tk, D); out (B, Hkv, G, D) == (B, Hq*D) for one token
template <int D>
constexpr int keys_per_split() { return (kThreads / (D / 8)) * kUnroll; }

template <typename E, int D, int G>
__global__ __launch_bounds__(kThreads) void decode_attention_kernel(const E* q, const E* kc, const E* vc,
                                                                    const uint8_t* valid, int64_t ld_valid,
                                                                    const int64_t* qpos_ptr, int64_t qpos_const,
                                                                    int64_t Hkv, int64_t Tk, int64_t L, float scale,
                                                                    E* out, float* part) {
  constexpr int TPK = D / 8;           // lanes per key row
  constexpr int KPB = kThreads / TPK;  // keys per workgroup per pass
  constexpr int NW = kThreads / kWave;
  __shared__ float s_m[NW][G], s_l[NW][G];
  __shared__ float s_o[NW][G][D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = lane % TPK;  // which 8-element slice of the row
  const int grp = tid / TPK;   // key lane group within the workgroup
  const int64_t bg = blockIdx.x;  // b * Hkv + h
  const int64_t b = bg / Hkv;
  const int64_t qpos = qpos_ptr ? *qpos_ptr : qpos_const;
  const int64_t kstop = min(L, qpos + 1);
  const int64_t k_lo = part ? static_cast<int64_t>(blockIdx.y) * keys_per_split<D>() : 0;
  const int64_t kend = part ? min(kstop, k_lo + keys_per_split<D>()) : kstop;
  const float sl2 = scale * 1.4426950408889634f;  // softmax in the exp2 domain
  float qv[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    Vec8<E>::load(q + (bg * G + g) * D + sub * 8, qv[g]);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[g][e] *= sl2;
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[g][e] = 0.f;
  }
  const E* kb = kc + bg * Tk * D + sub * 8;
  const E* vb = vc + bg * Tk * D + sub * 8;
  const uint8_t* vrow = valid + b * ld_valid;
  for (int64_t j0 = k_lo + grp; j0 < kend; j0 += static_cast<int64_t>(KPB) * kUnroll) {
    float kv[kUnroll][8], vv[kUnroll][8];
    bool ok[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t j = j0 + static_cast<int64_t>(u) * KPB;
      ok[u] = j < kend && vrow[j];
      if (ok[u]) {
        Vec8<E>::load(kb + j * D, kv[u]);
        Vec8<E>::load(vb + j * D, vv[u]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) kv[u][e] = vv[u][e] = 0.f;
      }
    }
    // one online-softmax update for the kUnroll keys together: a single rescale of (l, o) per head
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float s[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float acc = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(qv[g][e], kv[u][e], acc);
        s[u] = acc;
      }
      // full dot products: sum over the TPK lanes of each key (all lanes of a group agree on ok[u])
#pragma unroll
      for (int sh = 1; sh < TPK; sh <<= 1) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) s[u] += __shfl_xor(s[u], sh, kWave);
      }
      float mx = m[g];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) mx = ok[u] ? fmaxf(mx, s[u]) : mx;
      if (mx != -INFINITY) {
        const float alpha = __builtin_amdgcn_exp2f(m[g] - mx);  // m = -inf -> 0
        m[g] = mx;
        float lsum = l[g] * alpha;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[g][e] *= alpha;
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          const float p = ok[u] ? __builtin_amdgcn_exp2f(s[u] - mx) : 0.f;
          lsum += p;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[g][e] = fmaf(p, vv[u][e], o[g][e]);
        }
        l[g] = lsum;
      }
    }
  }
  // merge the lane groups of this wave (lanes with equal `sub` are TPK apart)
#pragma unroll
  for (int sh = TPK; sh < kWave; sh <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float m2 = __shfl_xor(m[g], sh, kWave);
      const float l2 = __shfl_xor(l[g], sh, kWave);
      const float mn = fmaxf(m[g], m2);
      const float a1 = m[g] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[g] - mn);
      const float a2 = m2 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m2 - mn);
      m[g] = mn;
      l[g] = l[g] * a1 + l2 * a2;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[g][e] = o[g][e] * a1 + __shfl_xor(o[g][e], sh, kWave) * a2;
    }
  }
  if (lane < TPK) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (sub == 0) { s_m[wave][g] = m[g]; s_l[wave][g] = l[g]; }
#pragma unroll
      for (int e = 0; e < 8; ++e) s_o[wave][g][sub * 8 + e] = o[g][e];
    }
  }
  __syncthreads();
  // final merge across waves: thread -> (g, 8-element slice); a row with no allowed key writes zeros.
  // Split-K: the chunk's unnormalised partial (m, l, o[D]) goes to part[((bg * G + g) * nsplit + y) * (D + 2)].
  for (int item = tid; item < G * TPK; item += kThreads) {
    const int g = item / TPK, sl = item % TPK;
    float mm = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) mm = fmaxf(mm, s_m[w][g]);
    float ll = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float a = s_m[w][g] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s_m[w][g] - mm);
      ll = fmaf(s_l[w][g], a, ll);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(s_o[w][g][sl * 8 + e], a, acc[e]);
    }
    if (part) {
      float* pp = part + ((bg * G + g) * gridDim.y + blockIdx.y) * (D + 2);
      if (sl == 0) { pp[0] = mm; pp[1] = ll; }
#pragma unroll
      for (int e = 0; e < 8; ++e) pp[2 + sl * 8 + e] = acc[e];
      continue;
    }
    const float inv = ll > 0.f ? 1.f / ll : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    Vec8<E>::store(out + (bg * G + g) * D + sl * 8, acc);
  }
}

// combine the nsplit partials of each (sequence, KV head, query head) in chunk order
template <typename E, int D>
__global__ __launch_bounds__(kThreads) void decode_merge_kernel(const float* part, int64_t rows, int nsplit, E* out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;  // (row, d)
  if (i >= rows * D) return;
  const int64_t r = i / D, d = i % D;  // r = bg * G + g
  float mm = -INFINITY;
  for (int y = 0; y < nsplit; ++y) mm = fmaxf(mm, part[(r * nsplit + y) * (D + 2)]);
  float ll = 0.f, acc = 0.f;
  for (int y = 0; y < nsplit; ++y) {
    const float* pp = part + (r * nsplit + y) * (D + 2);
    const float a = pp[0] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(pp[0] - mm);
    ll = fmaf(pp[1], a, ll);
    acc = fmaf(pp[2 + d], a, acc);
  }
  const float o = ll > 0.f ? acc / ll : 0.f;
  if constexpr (sizeof(E) == 2) out[i] = f32_to_bf16(o);
  else out[i] = o;
}

}  // namespace
}  // namespace drl

namespace drl {
namespace {
int64_t keys_per_split_rt(int64_t D) {
  switch (D) {
    case 16: return keys_per_split<16>();
    case 32: return keys_per_split<32>();
    case 64: return keys_per_split<64>();
    default: return keys_per_split<128>();
  }
}
}  // namespace
}  // namespace drl

extern "C" {

size_t drl_decode_attention_workspace_bytes(int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t L) {
  if (B < 1 || Hkv < 1 || G < 1 || L < 1 || D < 16) return 0;
  const int64_t nsplit = (L + drl::keys_per_split_rt(D) - 1) / drl::keys_per_split_rt(D);
  return nsplit > 1 ? static_cast<size_t>(B * Hkv * G * nsplit * (D + 2)) * sizeof(float) : 0;
}

int drl_decode_attention(const void* q, const void* k_cache, const void* v_cache, int32_t dt, const uint8_t* key_valid,
                         int64_t ld_valid, const int64_t* qpos_ptr, int64_t qpos, int64_t B, int64_t Hkv, int64_t G,
                         int64_t D, int64_t Tk, int64_t L, float scale, void* out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(q && k_cache && v_cache && key_valid && out, "NULL input");
  DRL_CHECK_ARG(B >= 1 && Hkv >= 1 && G >= 1 && G <= kMaxG && L >= 1 && L <= Tk && ld_valid >= L, "bad shape");
  DRL_CHECK_ARG(D == 64 || D == 128 || D == 16 || D == 32, "head_dim must be 16, 32, 64 or 128");
  DRL_CHECK_ARG(aligned16(q) && aligned16(k_cache) && aligned16(v_cache) && aligned16(out),
                "16-B aligned buffers needed");
  hipStream_t s = static_cast<hipStream_t>(stream);
  // split-K only when one workgroup per (sequence, KV head) cannot fill the CUs (small decode batches):
  // with a full grid the single pass is faster (measured 70 us vs 114 us at B=512, L=640) and the
  // workspace is not touched.
  const size_t need = drl_decode_attention_workspace_bytes(B, Hkv, G, D, L);
  const bool split = need > 0 && workspace != nullptr && workspace_bytes >= need && B * Hkv < cu_count();
  const int64_t nsplit = split ? (L + keys_per_split_rt(D) - 1) / keys_per_split_rt(D) : 1;
  float* part = split ? static_cast<float*>(workspace) : nullptr;
#define DRL_DA(E, DD, GG)                                                                                          \
  do {                                                                                                             \
    hipLaunchKernelGGL((decode_attention_kernel<E, DD, GG>), dim3(B * Hkv, nsplit), dim3(kThreads), 0, s,          \
                       static_cast<const E*>(q), static_cast<const E*>(k_cache), static_cast<const E*>(v_cache),   \
                       key_valid, ld_valid, qpos_ptr, qpos, Hkv, Tk, L, scale, static_cast<E*>(out), part);        \
    if (split)                                                                                                     \
      hipLaunchKernelGGL((decode_merge_kernel<E, DD>), dim3((B * Hkv * GG * DD + kThreads - 1) / kThreads),        \
                         dim3(kThreads), 0, s, part, B * Hkv * GG, static_cast<int>(nsplit), static_cast<E*>(out)); \
  } while (0)
#define DRL_DA_G(E, DD)               \
  switch (G) {                        \
    case 1: DRL_DA(E, DD, 1); break;  \
    case 2: DRL_DA(E, DD, 2); break;  \
    case 3: DRL_DA(E, DD, 3); break;  \
    case 4: DRL_DA(E, DD, 4); break;  \
    case 5: DRL_DA(E, DD, 5); break;  \
    case 6: DRL_DA(E, DD, 6); break;  \
    case 7: DRL_DA(E, DD, 7); break;  \
    default: DRL_DA(E, DD, 8); break; \
  }
#define DRL_DA_D(E)                  \
  switch (D) {                       \
    case 16: DRL_DA_G(E, 16) break;  \
    case 32: DRL_DA_G(E, 32) break;  \
    case 64: DRL_DA_G(E, 64) break;  \
    default: DRL_DA_G(E, 128) break; \
  }
  if (dt == DRL_BF16) {
    DRL_DA_D(uint16_t)
  } else if (dt == DRL_F32) {
    DRL_DA_D(float)
  } else {
    return fail(DRL_ERR_INVALID, "dtype must be BF16 or F32");
  }
#undef DRL_DA_D
#undef DRL_DA_G
#undef DRL_DA
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
