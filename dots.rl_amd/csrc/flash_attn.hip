// Fused causal + key-padding attention forward on MFMA (gfx950 v_mfma_f32_32x32x16_bf16) for the
// full-sequence passes of the actor / reference model: old and ref log-probs (dp_actor.py:300-359 ->
// Qwen2 attention) and, with the LSE it saves, the training forward. Scores and probabilities never
// touch HBM: per 32-query tile the kernel streams the (b, kv-head)'s K and V once per query head.
//
// Orientation (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand"): each wave
// computes S^T = K Q^T for 32 keys x 32 queries, so a lane holds 16 keys of ONE query (lane & 31) and
// the online softmax over keys is lane-local (16 registers + one xor-32 shuffle). The fp32 S^T
// registers converted to bf16 are directly the B operand of O^T += V^T P^T (no LDS round trip); V is
// read transposed (vt: (B, Hkv, D, ld_vt)), so the A operand of that product is two 8-B loads per
// k-step. O^T's lane is again one query, so the rescale by exp(m_old - m_new) is a per-lane scalar.
//
// Grid: x = 32-query tile (longest causal rows first), y = b * Hkv + kv head; block = G waves, wave g =
// query head g of the group, so the G waves of a workgroup walk the same K / V rows (L1 reuse).
// Mask (HF semantics for every row that has an allowed key): key j is allowed for query t iff
// j <= t + qoff && key_valid[b, j]. A row with no allowed key (only left-padding query rows) writes
// zeros and LSE = -inf: those rows feed nothing that reaches the loss (no valid query attends to a pad
// key), so their value is unobservable; HF's uniform row is not reproduced there.
#include "common.h"

namespace drl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

struct FlashArgs {
  const uint16_t* q;   // (B, Hkv, G, Tq, D)
  const uint16_t* k;   // (B, Hkv, ld_k, D), keys [0, Tk) used
  const uint16_t* vt;  // (B, Hkv, D, ld_vt)
  const uint8_t* valid;
  int64_t ld_valid;
  uint16_t* out;  // (B, Tq, Hkv, G, D)
  float* lse;     // (B, Hkv, G, Tq) natural-log LSE of the scaled scores, or nullptr
  int64_t Hkv, G, Tq, Tk, ld_k, ld_vt, qoff;
  float scale_log2;  // softmax scale * log2(e)
};

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint16_t to_bf16_bits(float f) { return f32_to_bf16(f); }

template <int D>
__global__ __launch_bounds__(512) void flash_fwd_kernel(FlashArgs a) {
  constexpr int KS = D / 16;  // k-steps of S^T = K Q^T over the head dim
  constexpr int MT = D / 32;  // 32-row tiles of O^T over the head dim
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int qi = lane & 31, h = lane >> 5;
  const int64_t bh = blockIdx.y;
  const int64_t b = bh / a.Hkv;
  const int64_t ntiles = (a.Tq + 31) / 32;
  const int64_t t0 = (ntiles - 1 - static_cast<int64_t>(blockIdx.x)) * 32;
  const int64_t tq = t0 + qi;
  const bool qvalid = tq < a.Tq;

  bf16x8 qf[KS];
  {
    const uint16_t* qrow = a.q + ((bh * a.G + g) * a.Tq + (qvalid ? tq : 0)) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 v = *reinterpret_cast<const u16x8*>(qrow + 16 * s);
      if (!qvalid) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[s] = as_bf16x8(v);
    }
  }
  f32x16 o[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) o[mt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;

  const uint16_t* kbase = a.k + bh * a.ld_k * D;
  const uint16_t* vtbase = a.vt + bh * D * a.ld_vt;
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  const int64_t kmax = min(a.Tk, t0 + 31 + a.qoff + 1);  // causal limit of the tile's last query
  const int64_t qpos = tq + a.qoff;

  for (int64_t k0 = 0; k0 < kmax; k0 += 32) {
    // ---- S^T (32 keys x 32 queries): A = K rows (lane & 31 = key), B = Q fragments
    f32x16 st = f32x16{};
    {
      const int64_t key = k0 + qi;
      const bool kin = key < a.Tk;
      const uint16_t* krow = kbase + (kin ? key : 0) * D + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        u16x8 kv = *reinterpret_cast<const u16x8*>(krow + 16 * s);
        if (!kin) kv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kv), qf[s], st, 0, 0, 0);
      }
    }
    // ---- mask + scale; register r holds key k0 + (r & 3) + 8 * (r >> 2) + 4h of query tq
    float x[16];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t kb = k0 + 8 * c + 4 * h;
      uint32_t vb;
      if (kb + 3 < a.Tk) {
        vb = *reinterpret_cast<const uint32_t*>(vrow + kb);
      } else {
        vb = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) vb |= (kb + j < a.Tk ? static_cast<uint32_t>(vrow[kb + j]) : 0u) << (8 * j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * c + j;
        const bool ok = ((vb >> (8 * j)) & 0xffu) != 0u && kb + j <= qpos;
        x[r] = ok ? st[r] * a.scale_log2 : -INFINITY;
        mx = fmaxf(mx, x[r]);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
    const float mn = fmaxf(m, mx);
    const float alpha = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    float ps = 0.f;
    u16x8 pb[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = (mn == -INFINITY || x[r] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(x[r] - mn);
      ps += p;
      pb[r >> 3][r & 7] = to_bf16_bits(p);
    }
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) o[mt] *= alpha;
    // ---- O^T += V^T P^T; k-step s: element j of lane half h is key k0 + 16s + 8(j>>2) + 4h + (j&3)
    const bool tail = k0 + 32 > a.Tk;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const uint16_t* vtrow = vtbase + static_cast<int64_t>(32 * mt + qi) * a.ld_vt;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int64_t ka = k0 + 16 * s + 4 * h, kb2 = ka + 8;
        u16x4 lo = *reinterpret_cast<const u16x4*>(vtrow + ka);
        u16x4 hi = *reinterpret_cast<const u16x4*>(vtrow + kb2);
        if (tail) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (ka + j >= a.Tk) lo[j] = 0;
            if (kb2 + j >= a.Tk) hi[j] = 0;
          }
        }
        const u16x8 vv = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(vv), as_bf16x8(pb[s]), o[mt], 0, 0, 0);
      }
    }
  }
  // ---- finalize: O^T register r of tile mt = head-dim row 32mt + (r & 3) + 8(r >> 2) + 4h of query tq
  const float lt = lsum + __shfl_xor(lsum, 32, kWave);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (!qvalid) return;
  uint16_t* orow = a.out + (((b * a.Tq + tq) * a.Hkv + (bh % a.Hkv)) * a.G + g) * D;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u16x4 w = u16x4{to_bf16_bits(o[mt][4 * c] * inv), to_bf16_bits(o[mt][4 * c + 1] * inv),
                            to_bf16_bits(o[mt][4 * c + 2] * inv), to_bf16_bits(o[mt][4 * c + 3] * inv)};
      *reinterpret_cast<u16x4*>(orow + 32 * mt + 8 * c + 4 * h) = w;
    }
  }
  if (a.lse != nullptr && h == 0)
    a.lse[(bh * a.G + g) * a.Tq + tq] = lt > 0.f ? (m + __builtin_amdgcn_logf(lt)) * 0.6931471805599453f : -INFINITY;
}

}  // namespace
}  // namespace drl

extern "C" {

int drl_flash_attn_fwd(const void* q, const void* k, const void* vt, int32_t dt, const uint8_t* key_valid,
                       int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t Tq, int64_t Tk,
                       int64_t ld_k, int64_t ld_vt, int64_t qoff, float scale, void* out, float* lse, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(q && k && vt && key_valid && out, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "flash attention runs on bf16 operands");
  DRL_CHECK_ARG(D == 64 || D == 128, "head_dim must be 64 or 128");
  DRL_CHECK_ARG(B >= 1 && Hkv >= 1 && G >= 1 && G <= 8 && Tq >= 1 && Tk >= 1 && qoff >= 0, "bad shape");
  DRL_CHECK_ARG(ld_vt >= Tk && ld_vt % 8 == 0, "ld_vt must be >= Tk and a multiple of 8");
  DRL_CHECK_ARG(ld_k >= Tk, "ld_k < Tk");
  DRL_CHECK_ARG(ld_valid >= Tk && ld_valid % 4 == 0 && (reinterpret_cast<uintptr_t>(key_valid) & 3u) == 0,
                "key_valid rows must be 4-byte aligned");
  DRL_CHECK_ARG(aligned16(q) && aligned16(k) && aligned16(vt) && (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                "misaligned operand");
  FlashArgs a{static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k), static_cast<const uint16_t*>(vt),
              key_valid, ld_valid, static_cast<uint16_t*>(out), lse, Hkv, G, Tq, Tk, ld_k, ld_vt, qoff,
              scale * 1.4426950408889634f};
  const dim3 grid(static_cast<unsigned>((Tq + 31) / 32), static_cast<unsigned>(B * Hkv));
  const dim3 block(static_cast<unsigned>(64 * G));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (D == 64) hipLaunchKernelGGL(flash_fwd_kernel<64>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(flash_fwd_kernel<128>, grid, block, 0, s, a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
