// Transformer-layer kernels of the Qwen2 actor / reference / rollout model (everything that is not a
// GEMM; GEMMs run on drl_gemm, csrc/gemm_sk.hip): fused QKV split + RoPE + grouped-query re-layout (fwd / bwd),
// masked softmax over attention scores (fwd / bwd), residual-add + RMSNorm (fwd / bwd), SwiGLU (fwd / bwd).
// Semantics follow HF Qwen2 (Qwen2RMSNorm fp32 variance, rotate_half RoPE, SiLU(gate) * up, causal +
// key-padding attention mask) as the reference runs it (verl/workers/actor/dp_actor.py:90-280 model call).
// All are HBM-bound streaming kernels: 16-B vector loads, fp32 math, one pass.
#include "common.h"

namespace drl {
namespace {

// element I/O: E = uint16_t (bf16) or float
__device__ __forceinline__ float ldf(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
__device__ __forceinline__ float ldf(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ void stf(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
__device__ __forceinline__ void stf(float* p, int64_t i, float v) { p[i] = v; }
template <typename E>
__device__ __forceinline__ float rnd(float v) {  // round through E (models a separate E-typed op)
  if constexpr (sizeof(E) == 2) return bf16_to_f32(f32_to_bf16(v));
  else return v;
}

// ------------------------------------------------------------------------------------------ RoPE + QKV
// qkv (B, T, (Hq + 2 Hkv) * D) bf16 ->
//   q  (B, Hkv, G, T, D)   G = Hq / Hkv query heads per KV head, rotated
//   k  (B, Hkv, Tk, D) at key offset koff (the KV cache when decoding), rotated
//   v  (B, Hkv, Tk, D) at key offset koff
// cos/sin tables (maxpos, D/2) fp32 indexed by position_ids (B, T). One thread per (b, t, head, pair).
template <typename E>
struct RopeArgs {
  const E* qkv;
  const int64_t* pos;
  const float* cos_t;
  const float* sin_t;
  E* q;
  E* k;
  E* v;
  int64_t B, T, Hq, Hkv, D, Tk, koff, maxpos;
  const int64_t* koff_dev;  // device key offset (graph-captured decode) overriding koff when non-NULL
  // optional head-dim-major copies for the fused attention kernels (row stride ld_t over key positions):
  // qt (B, Hkv, G, D, ld_t), kt / vt (B, Hkv, D, ld_t)
  E* qt;
  E* kt;
  E* vt;
  int64_t ld_t;
  // optional source row of each (b, t) in qkv (packed rows: remove-padding / prefix sharing), < 0 = a zero row;
  // NULL: row b * T + t
  const int64_t* src_row;
  // optional (B,): q rows t < (q_skip[b] & ~31) are not written (prefix sharing's copies: the fused attention skips
  // those query tiles — drl_flash_attn_fwd / bwd q_start — and never reads them)
  const int32_t* q_skip;
};

template <typename E>
__device__ __forceinline__ int64_t rope_q_skip(const RopeArgs<E>& a, int64_t b) {
  return a.q_skip ? static_cast<int64_t>(a.q_skip[b] & ~31) : 0;
}

// the qkv row of (b, t): its packed row through src_row (a pad reads row 0 and is zeroed by its caller)
template <typename E>
__device__ __forceinline__ const E* rope_src(const RopeArgs<E>& a, int64_t bt, int64_t Hall, int64_t h, bool& zero) {
  int64_t r = bt;
  zero = false;
  if (a.src_row) {
    r = a.src_row[bt];
    zero = r < 0;
    r = zero ? 0 : r;
  }
  return a.qkv + (r * Hall + h) * a.D;
}

template <typename E>
__global__ __launch_bounds__(256) void rope_qkv_fwd_kernel(RopeArgs<E> a) {
  const int64_t half = a.D / 2;
  const int64_t Hall = a.Hq + 2 * a.Hkv;
  const int64_t n = a.B * a.T * Hall * half;
  const int64_t G = a.Hq / a.Hkv;
  const int64_t koff = a.koff_dev ? *a.koff_dev : a.koff;
  if (koff < 0 || koff + a.T > a.Tk) return;  // device offset out of range: write nothing
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t j = i % half;
    const int64_t h = (i / half) % Hall;
    const int64_t bt = i / (half * Hall);
    const int64_t t = bt % a.T, b = bt / a.T;
    if (h < a.Hq && t < rope_q_skip(a, b)) continue;
    bool zero;
    const E* src = rope_src(a, bt, Hall, h, zero);
    const float x1 = zero ? 0.f : ldf(src, j), x2 = zero ? 0.f : ldf(src, j + half);
    if (h < a.Hq + a.Hkv) {
      int64_t p = a.pos[b * a.T + t];
      p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
      const float c = a.cos_t[p * half + j], s = a.sin_t[p * half + j];
      // rotate_half: out1 = x1*cos - x2*sin ; out2 = x2*cos + x1*sin
      // explicit contraction: identical rounding in every kernel that rotates
      const float o1 = fmaf(x1, c, -(x2 * s)), o2 = fmaf(x2, c, x1 * s);
      E* dst;
      E* dstt;  // transposed copy (nullptr: not requested)
      if (h < a.Hq) {
        const int64_t g = h / G, hi = h % G;
        dst = a.q + (((b * a.Hkv + g) * G + hi) * a.T + t) * a.D;
        dstt = a.qt ? a.qt + ((b * a.Hkv + g) * G + hi) * a.D * a.ld_t + t : nullptr;
      } else {
        dst = a.k + ((b * a.Hkv + (h - a.Hq)) * a.Tk + koff + t) * a.D;
        dstt = a.kt ? a.kt + (b * a.Hkv + (h - a.Hq)) * a.D * a.ld_t + koff + t : nullptr;
      }
      stf(dst, j, o1);
      stf(dst, j + half, o2);
      if (dstt) {
        stf(dstt, j * a.ld_t, o1);
        stf(dstt, (j + half) * a.ld_t, o2);
      }
    } else {
      if (a.vt != nullptr) {
        E* dst = a.vt + (b * a.Hkv + (h - a.Hq - a.Hkv)) * vt_panel(a.ld_t, a.D, a.Tk);
        stf(dst, vt_index(j, koff + t, a.ld_t, a.D), x1);  // exact: x1 is the element (or 0 for a pad row)
        stf(dst, vt_index(j + half, koff + t, a.ld_t, a.D), x2);
      }
      if (a.v != nullptr) {
        E* dst = a.v + ((b * a.Hkv + (h - a.Hq - a.Hkv)) * a.Tk + koff + t) * a.D;
        stf(dst, j, x1);
        stf(dst, j + half, x2);
      }
    }
  }
}

// Tiled form for full sequences that also want head-dim-major copies: one workgroup per (64-position
// tile, head, sequence) rotates the tile, writes the row-major output, and writes the transposed copy
// through an LDS tile so each head-dim row gets 64 contiguous positions (coalesced) instead of one
// 2-byte store per position. Same results as rope_qkv_fwd_kernel.
constexpr int kRopeTile = 64;

template <typename E>
__global__ __launch_bounds__(256) void rope_qkv_fwd_tiled_kernel(RopeArgs<E> a) {
  __shared__ __attribute__((aligned(16))) E tile[128][kRopeTile + 8];
  const int half = static_cast<int>(a.D / 2);
  const int64_t Hall = a.Hq + 2 * a.Hkv;
  const int64_t G = a.Hq / a.Hkv;
  const int64_t h = blockIdx.y, b = blockIdx.z;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kRopeTile;
  const int64_t koff = a.koff_dev ? *a.koff_dev : a.koff;
  if (koff < 0 || koff + a.T > a.Tk) return;
  const bool is_q = h < a.Hq, is_k = !is_q && h < a.Hq + a.Hkv;
  if (is_q && t0 + kRopeTile <= rope_q_skip(a, b)) return;  // a q tile no attention kernel reads
  E* rowdst;   // row-major destination base of this (b, head), indexed [pos][D]
  E* tdst;     // head-dim-major destination base, indexed [d * ld_t + pos]
  int64_t pos0;  // position offset of t = 0 in the destinations
  if (is_q) {
    const int64_t g = h / G, hi = h % G;
    rowdst = a.q + ((b * a.Hkv + g) * G + hi) * a.T * a.D;
    tdst = a.qt ? a.qt + ((b * a.Hkv + g) * G + hi) * a.D * a.ld_t : nullptr;
    pos0 = 0;
  } else if (is_k) {
    rowdst = a.k + (b * a.Hkv + (h - a.Hq)) * a.Tk * a.D;
    tdst = a.kt ? a.kt + (b * a.Hkv + (h - a.Hq)) * a.D * a.ld_t : nullptr;
    pos0 = koff;
  } else {
    rowdst = a.v ? a.v + (b * a.Hkv + (h - a.Hq - a.Hkv)) * a.Tk * a.D : nullptr;
    tdst = a.vt ? a.vt + (b * a.Hkv + (h - a.Hq - a.Hkv)) * vt_panel(a.ld_t, a.D, a.Tk) : nullptr;
    pos0 = koff;
  }
  const int rows_per_pass = 256 / half;
  for (int p = threadIdx.x / half; p < kRopeTile; p += rows_per_pass) {
    const int j = threadIdx.x % half;
    const int64_t t = t0 + p;
    if (t >= a.T) break;
    bool zero;
    const E* src = rope_src(a, b * a.T + t, Hall, h, zero);
    float o1 = zero ? 0.f : ldf(src, j), o2 = zero ? 0.f : ldf(src, j + half);
    if (is_q || is_k) {
      int64_t ps = a.pos[b * a.T + t];
      ps = ps < 0 ? 0 : (ps >= a.maxpos ? a.maxpos - 1 : ps);
      const float c = a.cos_t[ps * half + j], s = a.sin_t[ps * half + j];
      const float x1 = o1, x2 = o2;
      o1 = fmaf(x1, c, -(x2 * s));
      o2 = fmaf(x2, c, x1 * s);
    }
    if (rowdst) {
      stf(rowdst + (pos0 + t) * a.D, j, o1);
      stf(rowdst + (pos0 + t) * a.D, j + half, o2);
    }
    if (tdst) {
      E e1, e2;
      stf(&e1, 0, o1);
      stf(&e2, 0, o2);
      tile[j][p] = e1;
      tile[j + half][p] = e2;
    }
  }
  if (tdst == nullptr) return;
  __syncthreads();
  // transposed rows: D rows x 64 positions, 16 positions (one or two 16-B pieces) per thread
  constexpr int kPer = 16;
  const int nvalid = static_cast<int>(min<int64_t>(kRopeTile, a.T - t0));
  for (int it = threadIdx.x; it < a.D * (kRopeTile / kPer); it += 256) {
    const int d = it / (kRopeTile / kPer), c = it % (kRopeTile / kPer);
    const int64_t p0 = pos0 + t0 + c * kPer;  // first position of this thread's piece
    E* dst = tdst + vt_index(d, p0, a.ld_t, a.D);
    // the 16 positions are contiguous unless the key-blocked layout splits them over two 32-key blocks
    const bool contig = a.ld_t != DRL_VT_BLOCKED || (p0 & 31) + kPer <= 32;
    const bool aligned = ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) && sizeof(E) == 2;
    if (contig && aligned && c * kPer + kPer <= nvalid) {
      const uint4* srcv = reinterpret_cast<const uint4*>(&tile[d][c * kPer]);
      uint4* dv = reinterpret_cast<uint4*>(dst);
      dv[0] = srcv[0];
      dv[1] = srcv[1];
    } else {
      for (int e = 0; e < kPer && c * kPer + e < nvalid; ++e) tdst[vt_index(d, p0 + e, a.ld_t, a.D)] = tile[d][c * kPer + e];
    }
  }
}

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
// 4-element vector load / store with the fp32 compute conversion (8 B for bf16, 16 B for fp32)
__device__ __forceinline__ void ld4(const uint16_t* p, float (&f)[4]) {
  const u16x4 v = *reinterpret_cast<const u16x4*>(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) f[e] = bf16_to_f32(v[e]);
}
__device__ __forceinline__ void ld4(const float* p, float (&f)[4]) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
__device__ __forceinline__ void st4(uint16_t* p, const float (&f)[4]) {
  *reinterpret_cast<u16x4*>(p) = u16x4{f32_to_bf16(f[0]), f32_to_bf16(f[1]), f32_to_bf16(f[2]), f32_to_bf16(f[3])};
}
__device__ __forceinline__ void st4(float* p, const float (&f)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
}

template <typename E>
__global__ __launch_bounds__(256) void rope_qkv_fwd_tiled4_kernel(RopeArgs<E> a) {
  __shared__ __attribute__((aligned(16))) E tile[128][kRopeTile + 8];
  const int half = static_cast<int>(a.D / 2);
  const int64_t Hall = a.Hq + 2 * a.Hkv;
  const int64_t G = a.Hq / a.Hkv;
  const int64_t h = blockIdx.y, b = blockIdx.z;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kRopeTile;
  const int64_t koff = a.koff_dev ? *a.koff_dev : a.koff;
  if (koff < 0 || koff + a.T > a.Tk) return;
  const bool is_q = h < a.Hq, is_k = !is_q && h < a.Hq + a.Hkv;
  if (is_q && t0 + kRopeTile <= rope_q_skip(a, b)) return;  // a q tile no attention kernel reads
  E* rowdst;   // row-major destination base of this (b, head), indexed [pos][D]
  E* tdst;     // head-dim-major destination base, indexed [d * ld_t + pos]
  int64_t pos0;  // position offset of t = 0 in the destinations
  if (is_q) {
    const int64_t g = h / G, hi = h % G;
    rowdst = a.q + ((b * a.Hkv + g) * G + hi) * a.T * a.D;
    tdst = a.qt ? a.qt + ((b * a.Hkv + g) * G + hi) * a.D * a.ld_t : nullptr;
    pos0 = 0;
  } else if (is_k) {
    rowdst = a.k + (b * a.Hkv + (h - a.Hq)) * a.Tk * a.D;
    tdst = a.kt ? a.kt + (b * a.Hkv + (h - a.Hq)) * a.D * a.ld_t : nullptr;
    pos0 = koff;
  } else {
    rowdst = a.v ? a.v + (b * a.Hkv + (h - a.Hq - a.Hkv)) * a.Tk * a.D : nullptr;
    tdst = a.vt ? a.vt + (b * a.Hkv + (h - a.Hq - a.Hkv)) * vt_panel(a.ld_t, a.D, a.Tk) : nullptr;
    pos0 = koff;
  }
  // 4 consecutive head-dim pairs per thread: 8-B (bf16) / 16-B (fp32) loads and stores instead of 2-B ones
  const int tpr = half / 4, rows_per_pass = 256 / tpr;
  const int j0 = 4 * (threadIdx.x % tpr);
  for (int p = threadIdx.x / tpr; p < kRopeTile; p += rows_per_pass) {
    const int64_t t = t0 + p;
    if (t >= a.T) break;
    bool zero;
    const E* src = rope_src(a, b * a.T + t, Hall, h, zero);
    float o1[4], o2[4];
    ld4(src + j0, o1);
    ld4(src + j0 + half, o2);
    if (zero) {  // a pad position of the packed source: zeros, as pad_input leaves them (select after the load)
#pragma unroll
      for (int e = 0; e < 4; ++e) o1[e] = o2[e] = 0.f;
    }
    if (is_q || is_k) {
      int64_t ps = a.pos[b * a.T + t];
      ps = ps < 0 ? 0 : (ps >= a.maxpos ? a.maxpos - 1 : ps);
      const float4 c = *reinterpret_cast<const float4*>(a.cos_t + ps * half + j0);
      const float4 sn = *reinterpret_cast<const float4*>(a.sin_t + ps * half + j0);
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x1 = o1[e], x2 = o2[e];
        o1[e] = fmaf(x1, cc[e], -(x2 * ss[e]));
        o2[e] = fmaf(x2, cc[e], x1 * ss[e]);
      }
    }
    if (rowdst) {
      st4(rowdst + (pos0 + t) * a.D + j0, o1);
      st4(rowdst + (pos0 + t) * a.D + j0 + half, o2);
    }
    if (tdst) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        E e1, e2;
        stf(&e1, 0, o1[e]);
        stf(&e2, 0, o2[e]);
        tile[j0 + e][p] = e1;
        tile[j0 + e + half][p] = e2;
      }
    }
  }
  if (tdst == nullptr) return;
  __syncthreads();
  // transposed rows: D rows x 64 positions, 16 positions (one or two 16-B pieces) per thread
  constexpr int kPer = 16;
  const int nvalid = static_cast<int>(min<int64_t>(kRopeTile, a.T - t0));
  for (int it = threadIdx.x; it < a.D * (kRopeTile / kPer); it += 256) {
    const int d = it / (kRopeTile / kPer), c = it % (kRopeTile / kPer);
    const int64_t p0 = pos0 + t0 + c * kPer;  // first position of this thread's piece
    E* dst = tdst + vt_index(d, p0, a.ld_t, a.D);
    // the 16 positions are contiguous unless the key-blocked layout splits them over two 32-key blocks
    const bool contig = a.ld_t != DRL_VT_BLOCKED || (p0 & 31) + kPer <= 32;
    const bool aligned = ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) && sizeof(E) == 2;
    if (contig && aligned && c * kPer + kPer <= nvalid) {
      const uint4* srcv = reinterpret_cast<const uint4*>(&tile[d][c * kPer]);
      uint4* dv = reinterpret_cast<uint4*>(dst);
      dv[0] = srcv[0];
      dv[1] = srcv[1];
    } else {
      for (int e = 0; e < kPer && c * kPer + e < nvalid; ++e) tdst[vt_index(d, p0 + e, a.ld_t, a.D)] = tile[d][c * kPer + e];
    }
  }
}

// backward: dq (B,Hkv,G,T,D), dk/dv (B,Hkv,T,D) -> dqkv (B,T,(Hq+2Hkv)*D) with the inverse rotation
template <typename E>
__global__ __launch_bounds__(256) void rope_qkv_bwd_kernel(RopeArgs<E> a, const E* dq, const E* dk, const E* dv,
                                                           E* dqkv) {
  const int64_t half = a.D / 2;
  const int64_t Hall = a.Hq + 2 * a.Hkv;
  const int64_t n = a.B * a.T * Hall * half;
  const int64_t G = a.Hq / a.Hkv;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t j = i % half;
    const int64_t h = (i / half) % Hall;
    const int64_t bt = i / (half * Hall);
    const int64_t t = bt % a.T, b = bt / a.T;
    E* dst = dqkv + bt * Hall * a.D + h * a.D;
    if (h < a.Hq + a.Hkv) {
      const E* src;
      if (h < a.Hq) {
        const int64_t g = h / G, hi = h % G;
        src = dq + (((b * a.Hkv + g) * G + hi) * a.T + t) * a.D;
      } else {
        src = dk + ((b * a.Hkv + (h - a.Hq)) * a.T + t) * a.D;
      }
      int64_t p = a.pos[b * a.T + t];
      p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
      const float c = a.cos_t[p * half + j], s = a.sin_t[p * half + j];
      const float g1 = ldf(src, j), g2 = ldf(src, j + half);
      // transpose of [[c, -s], [s, c]]
      stf(dst, j, g1 * c + g2 * s);
      stf(dst, j + half, g2 * c - g1 * s);
    } else {
      const E* src = dv + ((b * a.Hkv + (h - a.Hq - a.Hkv)) * a.T + t) * a.D;
      dst[j] = src[j];
      dst[j + half] = src[j + half];
    }
  }
}

// 4 consecutive head-dim pairs per lane (8-B / 16-B accesses; the index arithmetic once per 4 pairs). Same
// per-element math as rope_qkv_bwd_kernel.
template <typename E>
__global__ __launch_bounds__(256) void rope_qkv_bwd4_kernel(RopeArgs<E> a, const E* dq, const E* dk, const E* dv,
                                                            E* dqkv) {
  const int64_t half = a.D / 2, q4 = half / 4;
  const int64_t Hall = a.Hq + 2 * a.Hkv;
  const int64_t n = a.B * a.T * Hall * q4;
  const int64_t G = a.Hq / a.Hkv;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t j0 = 4 * (i % q4);
    const int64_t h = (i / q4) % Hall;
    const int64_t bt = i / (q4 * Hall);
    const int64_t t = bt % a.T, b = bt / a.T;
    E* dst = dqkv + bt * Hall * a.D + h * a.D;
    float g1[4], g2[4];
    if (h < a.Hq + a.Hkv) {
      const E* src;
      if (h < a.Hq) {
        const int64_t g = h / G, hi = h % G;
        src = dq + (((b * a.Hkv + g) * G + hi) * a.T + t) * a.D;
      } else {
        src = dk + ((b * a.Hkv + (h - a.Hq)) * a.T + t) * a.D;
      }
      int64_t p = a.pos[b * a.T + t];
      p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
      const float4 c4 = *reinterpret_cast<const float4*>(a.cos_t + p * half + j0);
      const float4 s4 = *reinterpret_cast<const float4*>(a.sin_t + p * half + j0);
      const float c[4] = {c4.x, c4.y, c4.z, c4.w}, sn[4] = {s4.x, s4.y, s4.z, s4.w};
      ld4(src + j0, g1);
      ld4(src + j0 + half, g2);
      float o1[4], o2[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // transpose of [[c, -s], [s, c]]
        o1[e] = g1[e] * c[e] + g2[e] * sn[e];
        o2[e] = g2[e] * c[e] - g1[e] * sn[e];
      }
      st4(dst + j0, o1);
      st4(dst + j0 + half, o2);
    } else {
      const E* src = dv + ((b * a.Hkv + (h - a.Hq - a.Hkv)) * a.T + t) * a.D;
      ld4(src + j0, g1);
      ld4(src + j0 + half, g2);
      st4(dst + j0, g1);
      st4(dst + j0 + half, g2);
    }
  }
}

// ------------------------------------------------------------------------------------------ softmax
// Rows of attention scores S (rows, Tk) bf16 laid out (B, Hkv, G, Tq, Tk). Row r: q = r % Tq, b = r / (Hkv G Tq).
// allowed(key j) = valid[b, j] && j <= q + qoff; a row with no allowed key is uniform (HF finfo.min mask)
// P = softmax(S * scale) written as bf16 (in place allowed). One wave per row.
template <typename E>
struct SoftmaxArgs {
  const float* s;  // fp32 scores (hipBLASLt bf16 x bf16 -> fp32)
  E* p;
  const uint8_t* valid;  // (B, ld_valid) 0/1
  int64_t rows, Tq, Tk, HG, qoff, ld_valid;
  float scale;
};

template <typename E>
__global__ __launch_bounds__(256) void masked_softmax_fwd_kernel(SoftmaxArgs<E> a) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.rows) return;
  const int64_t q = row % a.Tq;
  const int64_t b = row / (a.HG * a.Tq);
  const int64_t qpos = q + a.qoff;
  const float* src = a.s + row * a.Tk;
  E* dst = a.p + row * a.Tk;
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  const float sl2 = a.scale * 1.4426950408889634f;  // exp(x*scale) = exp2(x*scale*log2e)
  float m = -INFINITY;
  for (int64_t j = lane; j < a.Tk; j += 64) {
    if (j <= qpos && vrow[j]) m = fmaxf(m, ldf(src, j) * sl2);
  }
  m = wave_max(m);
  if (m == -INFINITY) {
    // no allowed key (a left-padded query): HF adds finfo.min to every masked score, which makes the
    // row uniform over all Tk keys; its output only ever reaches padded positions
    const float u = 1.f / static_cast<float>(a.Tk);
    for (int64_t j = lane; j < a.Tk; j += 64) stf(dst, j, u);
    return;
  }
  float sum = 0.f;
  for (int64_t j = lane; j < a.Tk; j += 64) {
    if (j <= qpos && vrow[j]) sum += __builtin_amdgcn_exp2f(ldf(src, j) * sl2 - m);
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  for (int64_t j = lane; j < a.Tk; j += 64) {
    const bool ok = j <= qpos && vrow[j];
    const float e = ok ? __builtin_amdgcn_exp2f(ldf(src, j) * sl2 - m) * inv : 0.f;
    stf(dst, j, e);
  }
}

// Single-pass variants for rows of up to kRegCols keys: the row lives in registers (lane l holds columns
// 4l + 256k .. +3), so S / dP are read from HBM once with 16-B loads and P / dS written once.
constexpr int kRegChunks = 16;                 // 16 x 256 columns
constexpr int64_t kRegCols = kRegChunks * 256;  // 4096 keys

__device__ __forceinline__ void ld4f(const float* p, int64_t j, int64_t n, bool vec, float v[4]) {
  if (vec && j + 3 < n) {
    const float4 q = *reinterpret_cast<const float4*>(p + j);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = j + e < n ? p[j + e] : 0.f;
  }
}
template <typename E>
__device__ __forceinline__ void ld4e(const E* p, int64_t j, int64_t n, bool vec, float v[4]) {
  if constexpr (sizeof(E) == 2) {
    if (vec && j + 3 < n) {
      const uint2 q = *reinterpret_cast<const uint2*>(p + j);
      v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
      v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
      return;
    }
  } else {
    if (vec && j + 3 < n) {
      const float4 q = *reinterpret_cast<const float4*>(p + j);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      return;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = j + e < n ? ldf(p, j + e) : 0.f;
}
template <typename E>
__device__ __forceinline__ void st4e(E* p, int64_t j, int64_t n, bool vec, const float v[4]) {
  if constexpr (sizeof(E) == 2) {
    if (vec && j + 3 < n) {
      const uint32_t lo = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      const uint32_t hi = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      *reinterpret_cast<uint2*>(p + j) = make_uint2(lo, hi);
      return;
    }
  } else {
    if (vec && j + 3 < n) {
      *reinterpret_cast<float4*>(p + j) = make_float4(v[0], v[1], v[2], v[3]);
      return;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (j + e < n) stf(p, j + e, v[e]);
}

template <typename E>
__global__ __launch_bounds__(256) void masked_softmax_fwd_reg_kernel(SoftmaxArgs<E> a) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.rows) return;
  const int64_t q = row % a.Tq, b = row / (a.HG * a.Tq), qpos = q + a.qoff, Tk = a.Tk;
  const bool vec = (Tk & 3) == 0;
  const float* src = a.s + row * Tk;
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  const float sl2 = a.scale * 1.4426950408889634f;
  const int nchunk = static_cast<int>((Tk + 255) / 256);
  float v[kRegChunks][4];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < kRegChunks; ++k) {
    if (k < nchunk) {
      const int64_t j = 256 * k + 4 * lane;
      ld4f(src, j, Tk, vec, v[k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t jj = j + e;
        const bool ok = jj < Tk && jj <= qpos && vrow[jj];
        v[k][e] = ok ? v[k][e] * sl2 : -INFINITY;
        m = fmaxf(m, v[k][e]);
      }
    }
  }
  m = wave_max(m);
  E* dst = a.p + row * Tk;
  if (m == -INFINITY) {  // no allowed key: uniform row (HF finfo.min mask)
    const float u = 1.f / static_cast<float>(Tk);
    const float uu[4] = {u, u, u, u};
#pragma unroll
    for (int k = 0; k < kRegChunks; ++k)
      if (k < nchunk) st4e(dst, 256 * k + 4 * lane, Tk, vec, uu);
    return;
  }
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kRegChunks; ++k) {
    if (k < nchunk) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[k][e] = __builtin_amdgcn_exp2f(v[k][e] - m);  // exp2(-inf) = 0 for masked keys
        sum += v[k][e];
      }
    }
  }
  const float inv = 1.f / wave_sum(sum);
#pragma unroll
  for (int k = 0; k < kRegChunks; ++k) {
    if (k < nchunk) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] *= inv;
      st4e(dst, 256 * k + 4 * lane, Tk, vec, v[k]);
    }
  }
}

// dS = P * (dP - sum_j P dP) * scale: P (E), dP fp32 -> dS (E). One wave per row.
template <typename E>
__global__ __launch_bounds__(256) void masked_softmax_bwd_kernel(const E* p, const float* dp, E* ds, int64_t rows,
                                                                 int64_t Tk, float scale) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const E* pr = p + row * Tk;
  const float* dr = dp + row * Tk;
  E* sr = ds + row * Tk;
  if (Tk <= kRegCols) {
    const bool vec = (Tk & 3) == 0;
    const int nchunk = static_cast<int>((Tk + 255) / 256);
    float pv[kRegChunks][4], dv[kRegChunks][4];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < kRegChunks; ++k) {
      if (k < nchunk) {
        const int64_t j = 256 * k + 4 * lane;
        ld4e(pr, j, Tk, vec, pv[k]);
        ld4f(dr, j, Tk, vec, dv[k]);
#pragma unroll
        for (int e = 0; e < 4; ++e) dot += pv[k][e] * dv[k][e];
      }
    }
    dot = wave_sum(dot);
#pragma unroll
    for (int k = 0; k < kRegChunks; ++k) {
      if (k < nchunk) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dv[k][e] = pv[k][e] * (dv[k][e] - dot) * scale;
        st4e(sr, 256 * k + 4 * lane, Tk, vec, dv[k]);
      }
    }
    return;
  }
  float dot = 0.f;
  for (int64_t j = lane; j < Tk; j += 64) dot += ldf(pr, j) * dr[j];
  dot = wave_sum(dot);
  for (int64_t j = lane; j < Tk; j += 64) stf(sr, j, ldf(pr, j) * (dr[j] - dot) * scale);
}

// ------------------------------------------------------------------------------------------ RMSNorm
// x_out = x_in (+ delta) (fp32 residual stream; x_out may alias x_in or be NULL = no write);
// y = w * x * rsqrt(mean(x^2) + eps) as E; rstd (N) saved for backward. One wave per row.
template <typename E>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_kernel(const float* x_in, const E* delta, float* x_out,
                                                              const float* w, E* y, float* rstd, int64_t N, int64_t H,
                                                              float eps) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* xr = x_in + row * H;
  float* xo = x_out ? x_out + row * H : nullptr;
  float ss = 0.f;
  for (int64_t j = lane * 4; j < H; j += 256) {
    float4 v = *reinterpret_cast<const float4*>(xr + j);
    if (delta) {
      v.x += ldf(delta, row * H + j);
      v.y += ldf(delta, row * H + j + 1);
      v.z += ldf(delta, row * H + j + 2);
      v.w += ldf(delta, row * H + j + 3);
    }
    if (xo) *reinterpret_cast<float4*>(xo + j) = v;
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / static_cast<float>(H) + eps);
  if (lane == 0 && rstd) rstd[row] = r;
  const float* xs = xo ? xo : xr;
  for (int64_t j = lane * 4; j < H; j += 256) {
    float4 v = *reinterpret_cast<const float4*>(xs + j);
    if (delta && !xo) {
      v.x += ldf(delta, row * H + j);
      v.y += ldf(delta, row * H + j + 1);
      v.z += ldf(delta, row * H + j + 2);
      v.w += ldf(delta, row * H + j + 3);
    }
    const float4 ww = *reinterpret_cast<const float4*>(w + j);
    stf(y, row * H + j, ww.x * (v.x * r));
    stf(y, row * H + j + 1, ww.y * (v.y * r));
    stf(y, row * H + j + 2, ww.z * (v.z * r));
    stf(y, row * H + j + 3, ww.w * (v.w * r));
  }
}

// bf16-output form for H % 128 == 0 (Qwen2: 896): one wave per row, each lane owns the column pairs
// 2*lane + 128*k; the row is read once (x, delta) and kept in registers for the normalisation, so the decode
// step's 64-row norm is one dependent memory round trip instead of two.
template <int K>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_vec_kernel(const float* x_in, const uint16_t* delta, float* x_out,
                                                                  const float* w, uint16_t* y, float* rstd, int64_t N,
                                                                  float eps) {
  constexpr int H = 128 * K;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  float2 v[K];
  uint32_t d[K];
  // every load of the row issued before the first use (a null test on delta inside the loop made hipcc wait for
  // all loads in flight before each delta load: K dependent round trips per row)
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = *reinterpret_cast<const float2*>(x_in + row * H + 2 * lane + 128 * k);
  if (delta) {
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = *reinterpret_cast<const uint32_t*>(delta + row * H + 2 * lane + 128 * k);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      v[k].x += bf16_to_f32(static_cast<uint16_t>(d[k] & 0xffffu));
      v[k].y += bf16_to_f32(static_cast<uint16_t>(d[k] >> 16));
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (x_out) *reinterpret_cast<float2*>(x_out + row * H + 2 * lane + 128 * k) = v[k];
    ss += v[k].x * v[k].x + v[k].y * v[k].y;
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / static_cast<float>(H) + eps);
  if (lane == 0 && rstd) rstd[row] = r;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float2 ww = *reinterpret_cast<const float2*>(w + 2 * lane + 128 * k);
    const uint32_t o = static_cast<uint32_t>(f32_to_bf16(ww.x * (v[k].x * r))) |
                       (static_cast<uint32_t>(f32_to_bf16(ww.y * (v[k].y * r))) << 16);
    *reinterpret_cast<uint32_t*>(y + row * H + 2 * lane + 128 * k) = o;
  }
}

// dx += rstd * (w*dy - xhat * mean(xhat * w*dy)) ; dw partials per block (fixed order) -> dw_part (grid, H)
template <typename E>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const float* x, const float* w, const float* rstd,
                                                          const E* dy, const float* dx_in, float* dx, uint16_t* dx_lp,
                                                          float* dw_part, int64_t N, int64_t H) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  extern __shared__ float s_dw[];  // 4 waves x H
  for (int64_t j = threadIdx.x; j < 4 * H; j += blockDim.x) s_dw[j] = 0.f;
  __syncthreads();
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + wave; row < N; row += static_cast<int64_t>(gridDim.x) * 4) {
    const float r = rstd[row];
    const float* xr = x + row * H;
    float dot = 0.f;
    for (int64_t j = lane; j < H; j += 64) dot += (w[j] * ldf(dy, row * H + j)) * (xr[j] * r);
    dot = wave_sum(dot) / static_cast<float>(H);
    for (int64_t j = lane; j < H; j += 64) {
      const float g = ldf(dy, row * H + j);
      const float xh = xr[j] * r;
      const float d = (dx_in ? dx_in[row * H + j] : 0.f) + r * (w[j] * g - xh * dot);
      dx[row * H + j] = d;
      if (dx_lp) dx_lp[row * H + j] = f32_to_bf16(d);
      s_dw[wave * H + j] += g * xh;
    }
  }
  __syncthreads();
  for (int64_t j = threadIdx.x; j < H; j += blockDim.x)
    dw_part[blockIdx.x * H + j] = s_dw[j] + s_dw[H + j] + s_dw[2 * H + j] + s_dw[3 * H + j];
}

// two adjacent elements (j even; the launcher checks the alignment)
__device__ __forceinline__ float2 ldf2(const uint16_t* p, int64_t j) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(p + j);
  return make_float2(bf16_to_f32(static_cast<uint16_t>(u & 0xffffu)), bf16_to_f32(static_cast<uint16_t>(u >> 16)));
}
__device__ __forceinline__ float2 ldf2(const float* p, int64_t j) { return *reinterpret_cast<const float2*>(p + j); }

// Vectorised form for H % 128 == 0 (Qwen2: 896): one wave per row, each lane owns the column pairs
// 2*lane + 128*k; the row's x, dy and dx_in stay in registers between the dot product and the update (one read).
// Each wave takes its rows two at a time (rows r and r + stride of its grid-stride sequence, every load of both
// issued before the first reduction: one dependent round trip per pair; the grid is 2 workgroups per CU, so a
// row at a time left 8 rows' loads in flight per CU), accumulating dw in the sequence's order. 264 -> 233 us at the
// update pass's 82144 rows (profiles/r05_rmsnorm_bwd_ab.txt); deterministic, not bit-identical to the row-at-a-time
// form (hipcc contracts the mul/add chains into FMAs differently).
template <typename E, int K>
__global__ __launch_bounds__(256) void rmsnorm_bwd_vec_kernel(const float* x, const float* w, const float* rstd,
                                                              const E* dy, const float* dx_in, float* dx,
                                                              uint16_t* dx_lp, float* dw_part, int64_t N) {
  constexpr int H = 128 * K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ float2 s_dw[4][64 * K];
  float2 wv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wv[k] = *reinterpret_cast<const float2*>(w + 2 * lane + 128 * k);
  float2 acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = make_float2(0.f, 0.f);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 4;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + wave; row < N; row += 2 * stride) {
    const bool two = row + stride < N;
    int64_t rr[2] = {row, two ? row + stride : row};
    float r[2];
    float2 xv[2][K], gv[2][K], dv[2][K];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      r[q] = rstd[rr[q]];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t j = rr[q] * H + 2 * lane + 128 * k;
        xv[q][k] = *reinterpret_cast<const float2*>(x + j);
        gv[q][k] = ldf2(dy, j);
        dv[q][k] = dx_in ? *reinterpret_cast<const float2*>(dx_in + j) : make_float2(0.f, 0.f);
      }
    }
    float dot[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      dot[q] = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k)
        dot[q] += (wv[k].x * gv[q][k].x) * (xv[q][k].x * r[q]) + (wv[k].y * gv[q][k].y) * (xv[q][k].y * r[q]);
    }
    dot[0] = wave_sum(dot[0]) / static_cast<float>(H);
    dot[1] = wave_sum(dot[1]) / static_cast<float>(H);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1 && !two) break;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t j = rr[q] * H + 2 * lane + 128 * k;
        const float xh0 = xv[q][k].x * r[q], xh1 = xv[q][k].y * r[q];
        float2 d = dv[q][k];
        d.x += r[q] * (wv[k].x * gv[q][k].x - xh0 * dot[q]);
        d.y += r[q] * (wv[k].y * gv[q][k].y - xh1 * dot[q]);
        *reinterpret_cast<float2*>(dx + j) = d;
        if (dx_lp)  // the bf16 copy the next dgrad consumes, in the same pass
          *reinterpret_cast<uint32_t*>(dx_lp + j) = static_cast<uint32_t>(f32_to_bf16(d.x)) |
                                                    (static_cast<uint32_t>(f32_to_bf16(d.y)) << 16);
        acc[k].x += gv[q][k].x * xh0;
        acc[k].y += gv[q][k].y * xh1;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) s_dw[wave][lane + 64 * k] = acc[k];
  __syncthreads();
  for (int j = threadIdx.x; j < 64 * K; j += blockDim.x) {
    const float2 a = s_dw[0][j], b = s_dw[1][j], c = s_dw[2][j], d = s_dw[3][j];
    const int col = 2 * (j % 64) + 128 * (j / 64);
    dw_part[blockIdx.x * H + col] = (a.x + b.x) + (c.x + d.x);
    dw_part[blockIdx.x * H + col + 1] = (a.y + b.y) + (c.y + d.y);
  }
}

// Column sums of a bf16 (N, C) matrix (the qkv bias gradient = dqkv summed over tokens), phase 1: workgroup
// (64-column stripe, row slice) -> fp32 partials (slices, C); thread = 8 columns (one 16-B load) x every 32nd row
// of the slice, combined in LDS in a fixed order. Phase 2 is colsum_kernel (fixed slice order): deterministic.
__global__ __launch_bounds__(256) void colsum_bf16_partial_kernel(const uint16_t* x, int64_t ld, int64_t N, int64_t C,
                                                                  int64_t rows_per_slice, float* part) {
  __shared__ float red[32][65];
  const int t = threadIdx.x, cg = t & 7, rl = t >> 3;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * 64 + cg * 8;
  const int64_t r_begin = static_cast<int64_t>(blockIdx.y) * rows_per_slice;
  const int64_t r_end = min(N, r_begin + rows_per_slice);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 + 7 < C) {
    for (int64_t r = r_begin + rl; r < r_end; r += 32) {
      const uint4 u = *reinterpret_cast<const uint4*>(x + r * ld + c0);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += __uint_as_float(w[e] << 16);
        acc[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
      }
    }
  } else {
    for (int64_t r = r_begin + rl; r < r_end; r += 32)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < C) acc[e] += __uint_as_float(static_cast<uint32_t>(x[r * ld + c0 + e]) << 16);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][cg * 8 + e] = acc[e];
  __syncthreads();
  if (t < 64) {
    const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + t;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) v += red[k][t];
    if (c < C) part[static_cast<int64_t>(blockIdx.y) * C + c] = v;
  }
}

// dw[j] += sum over blocks of dw_part[:, j]: 16 columns x 16 block-slices per workgroup (many
// workgroups, short dependent chains), slices combined in a fixed order
__global__ __launch_bounds__(256) void colsum_kernel(const float* part, int64_t nb, int64_t H, float* out) {
  __shared__ float red[16][16];
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 16 + c;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (j < H) {
    int64_t b = sl;
    for (; b + 48 < nb; b += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += part[(b + 16 * u) * H + j];
    }
    for (; b < nb; b += 16) s[0] += part[b * H + j];
  }
  red[sl][c] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (sl == 0 && j < H) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][c];
    out[j] += t;
  }
}

// ------------------------------------------------------------------------------------------ SwiGLU
// gu (N, 2I) = [gate | up] -> a (N, I) = silu(gate) * up   (two E-typed ops, as F.silu then * in the model)
// 4 consecutive columns per thread (I % 4 == 0 on the vector path).
template <typename E>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const E* gu, E* out, int64_t N, int64_t I) {
  const int64_t n4 = N * I / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t row = (4 * i) / I, c = (4 * i) % I;
    float g[4], u[4], o[4];
    ld4e(gu, row * 2 * I + c, row * 2 * I + I, true, g);
    ld4e(gu, row * 2 * I + I + c, row * 2 * I + 2 * I, true, u);
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = rnd<E>(silu_fast(g[e])) * u[e];
    st4e(out, 4 * i, N * I, true, o);
  }
}

// d gate = da * up * silu'(gate), d up = da * silu(gate)   ->   dgu (N, 2I)
template <typename E>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const E* gu, const E* da, E* dgu, int64_t N, int64_t I) {
  const int64_t n4 = N * I / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t row = (4 * i) / I, c = (4 * i) % I;
    float g[4], u[4], d[4], dg[4], du[4];
    ld4e(gu, row * 2 * I + c, row * 2 * I + I, true, g);
    ld4e(gu, row * 2 * I + I + c, row * 2 * I + 2 * I, true, u);
    ld4e(da, 4 * i, N * I, true, d);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sig = sigmoid_fast(g[e]);
      dg[e] = rnd<E>(d[e] * u[e]) * (sig * (1.f + g[e] * (1.f - sig)));
      du[e] = d[e] * rnd<E>(g[e] * sig);
    }
    st4e(dgu, row * 2 * I + c, row * 2 * I + I, true, dg);
    st4e(dgu, row * 2 * I + I + c, row * 2 * I + 2 * I, true, du);
  }
}

// bf16 fast path (I % 8 == 0, 16-B aligned rows): 8 columns per lane = one 16-B load of gate, one of up and
// one 16-B store per lane (1 KiB per wave instruction), rows found with a 32-bit division by I / 8 instead
// of the 64-bit div/mod of the generic path, two independent groups in flight per lane. Same math and
// rounding as swiglu_fwd_kernel / swiglu_bwd_kernel.
__device__ __forceinline__ void unpack8(const uint4 q, float v[8]) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(w[e] << 16);
    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float v[8]) {
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    w[e] = static_cast<uint32_t>(f32_to_bf16(v[2 * e])) | (static_cast<uint32_t>(f32_to_bf16(v[2 * e + 1])) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(256) void swiglu_fwd_bf16x8_kernel(const uint16_t* gu, uint16_t* out, uint32_t n8,
                                                                uint32_t i8) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += 2 * stride) {
    uint4 gq[2], uq[2];
    bool on[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t j = i + k * stride;
      on[k] = j < n8;
      const uint32_t row = on[k] ? j / i8 : 0, c = on[k] ? j - row * i8 : 0;
      const uint16_t* base = gu + (static_cast<size_t>(row) * 2 * i8 + c) * 8;
      if (on[k]) {
        gq[k] = *reinterpret_cast<const uint4*>(base);
        uq[k] = *reinterpret_cast<const uint4*>(base + static_cast<size_t>(i8) * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (!on[k]) continue;
      float g[8], u[8], o[8];
      unpack8(gq[k], g);
      unpack8(uq[k], u);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rnd<uint16_t>(silu_fast(g[e])) * u[e];
      *reinterpret_cast<uint4*>(out + static_cast<size_t>(i + k * stride) * 8) = pack8(o);
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_bf16x8_kernel(const uint16_t* gu, const uint16_t* da, uint16_t* dgu,
                                                                uint32_t n8, uint32_t i8) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const uint32_t row = i / i8, c = i - row * i8;
    const size_t gbase = (static_cast<size_t>(row) * 2 * i8 + c) * 8;
    const uint4 gq = *reinterpret_cast<const uint4*>(gu + gbase);
    const uint4 uq = *reinterpret_cast<const uint4*>(gu + gbase + static_cast<size_t>(i8) * 8);
    const uint4 dq = *reinterpret_cast<const uint4*>(da + static_cast<size_t>(i) * 8);
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(gq, g);
    unpack8(uq, u);
    unpack8(dq, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sig = sigmoid_fast(g[e]);
      dg[e] = rnd<uint16_t>(d[e] * u[e]) * (sig * (1.f + g[e] * (1.f - sig)));
      du[e] = d[e] * rnd<uint16_t>(g[e] * sig);
    }
    *reinterpret_cast<uint4*>(dgu + gbase) = pack8(dg);
    *reinterpret_cast<uint4*>(dgu + gbase + static_cast<size_t>(i8) * 8) = pack8(du);
  }
}

int grid_stride(int64_t n, int threads = 256) {
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + threads - 1) / threads, static_cast<int64_t>(cu_count()) * 16)));
}

}  // namespace
}  // namespace drl

#define DRL_E_DISPATCH(dt, ...)                                   \
  do {                                                          \
    if ((dt) == DRL_BF16) { using E = uint16_t; __VA_ARGS__; }  \
    else if ((dt) == DRL_F32) { using E = float; __VA_ARGS__; } \
    else return ::drl::fail(DRL_ERR_INVALID, "dtype must be BF16 or F32"); \
  } while (0)

extern "C" {

int drl_rope_qkv_fwd(const void* qkv, int32_t dt, const int64_t* position_ids, const float* cos_t, const float* sin_t,
                     int64_t maxpos, int64_t B, int64_t T, int64_t Hq, int64_t Hkv, int64_t D, void* q, void* k,
                     void* v, int64_t Tk, int64_t koff, const int64_t* koff_dev, void* qt, void* kt, void* vt,
                     int64_t ld_t, void* stream) {
  return drl_rope_qkv_fwd_rows(qkv, nullptr, dt, position_ids, cos_t, sin_t, maxpos, B, T, Hq, Hkv, D, q, k, v, Tk,
                               koff, koff_dev, qt, kt, vt, ld_t, nullptr, stream);
}

int drl_rope_qkv_fwd_rows(const void* qkv, const int64_t* src_row, int32_t dt, const int64_t* position_ids,
                          const float* cos_t, const float* sin_t, int64_t maxpos, int64_t B, int64_t T, int64_t Hq,
                          int64_t Hkv, int64_t D, void* q, void* k, void* v, int64_t Tk, int64_t koff,
                          const int64_t* koff_dev, void* qt, void* kt, void* vt, int64_t ld_t, const int32_t* q_skip,
                          void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(qkv && position_ids && cos_t && sin_t && q && k && (v || vt), "NULL input");
  DRL_CHECK_ARG((qt == nullptr && kt == nullptr && vt == nullptr) || (ld_t >= Tk && ld_t >= T) ||
                    (ld_t == DRL_VT_BLOCKED && qt == nullptr && kt == nullptr),
                "ld_t too small (DRL_VT_BLOCKED only for a vt cache alone)");
  DRL_CHECK_ARG(B >= 1 && T >= 1 && Hq >= 1 && Hkv >= 1 && Hq % Hkv == 0 && D % 2 == 0, "bad shape");
  DRL_CHECK_ARG(koff >= 0 && koff + T <= Tk, "key offset out of range");
  const int64_t n = B * T * (Hq + 2 * Hkv) * (D / 2);
  DRL_E_DISPATCH(dt, {
    RopeArgs<E> a{static_cast<const E*>(qkv), position_ids, cos_t, sin_t, static_cast<E*>(q), static_cast<E*>(k),
                  static_cast<E*>(v), B, T, Hq, Hkv, D, Tk, koff, maxpos, koff_dev, static_cast<E*>(qt),
                  static_cast<E*>(kt), static_cast<E*>(vt), ld_t, src_row, q_skip};
    const bool vec4 = D % 8 == 0 && 256 % (D / 8) == 0 && aligned16(qkv) && aligned16(cos_t) && aligned16(sin_t) &&
                      (q == nullptr || aligned16(q)) && (k == nullptr || aligned16(k)) && (v == nullptr || aligned16(v));
    if ((qt || kt || vt) && T >= 16 && D <= 128 && D % 2 == 0 && 256 % (D / 2) == 0) {
      const dim3 grid(static_cast<unsigned>((T + kRopeTile - 1) / kRopeTile), static_cast<unsigned>(Hq + 2 * Hkv),
                      static_cast<unsigned>(B));
      if (vec4)
        hipLaunchKernelGGL(rope_qkv_fwd_tiled4_kernel<E>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), a);
      else
        hipLaunchKernelGGL(rope_qkv_fwd_tiled_kernel<E>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), a);
    } else {
      hipLaunchKernelGGL(rope_qkv_fwd_kernel<E>, dim3(grid_stride(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                         a);
    }
  });
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_rope_qkv_bwd(const void* dq, const void* dk, const void* dv, int32_t dt, const int64_t* position_ids,
                     const float* cos_t, const float* sin_t, int64_t maxpos, int64_t B, int64_t T, int64_t Hq,
                     int64_t Hkv, int64_t D, void* dqkv, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(dq && dk && dv && position_ids && cos_t && sin_t && dqkv, "NULL input");
  DRL_CHECK_ARG(B >= 1 && T >= 1 && Hq % Hkv == 0 && D % 2 == 0, "bad shape");
  const int64_t n = B * T * (Hq + 2 * Hkv) * (D / 2);
  DRL_E_DISPATCH(dt, {
    RopeArgs<E> a{nullptr, position_ids, cos_t, sin_t, nullptr, nullptr, nullptr, B, T, Hq, Hkv, D, T, 0, maxpos};
    if (D % 8 == 0 && aligned16(dq) && aligned16(dk) && aligned16(dv) && aligned16(dqkv) && aligned16(cos_t) &&
        aligned16(sin_t))
      hipLaunchKernelGGL(rope_qkv_bwd4_kernel<E>, dim3(grid_stride(n / 4)), dim3(256), 0,
                         static_cast<hipStream_t>(stream), a, static_cast<const E*>(dq), static_cast<const E*>(dk),
                         static_cast<const E*>(dv), static_cast<E*>(dqkv));
    else
      hipLaunchKernelGGL(rope_qkv_bwd_kernel<E>, dim3(grid_stride(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                         a, static_cast<const E*>(dq), static_cast<const E*>(dk), static_cast<const E*>(dv),
                         static_cast<E*>(dqkv));
  });
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_masked_softmax_fwd(const float* scores, void* probs, int32_t dt, const uint8_t* key_valid, int64_t ld_valid,
                           int64_t B, int64_t HG, int64_t Tq, int64_t Tk, int64_t qoff, float scale, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(scores && probs && key_valid, "NULL input");
  DRL_CHECK_ARG(B >= 1 && HG >= 1 && Tq >= 1 && Tk >= 1 && ld_valid >= Tk && qoff >= 0 && qoff + Tq <= Tk, "bad shape");
  const int64_t rows = B * HG * Tq;
  DRL_E_DISPATCH(dt, {
    SoftmaxArgs<E> a{scores, static_cast<E*>(probs), key_valid, rows, Tq, Tk, HG, qoff, ld_valid, scale};
    if (Tk <= kRegCols)
      hipLaunchKernelGGL(masked_softmax_fwd_reg_kernel<E>, dim3((rows + 3) / 4), dim3(256), 0,
                         static_cast<hipStream_t>(stream), a);
    else
      hipLaunchKernelGGL(masked_softmax_fwd_kernel<E>, dim3((rows + 3) / 4), dim3(256), 0,
                         static_cast<hipStream_t>(stream), a);
  });
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_masked_softmax_bwd(const void* probs, const float* dprobs, void* dscores, int32_t dt, int64_t rows, int64_t Tk,
                           float scale, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(probs && dprobs && dscores && rows >= 0 && Tk >= 1, "bad input");
  if (rows == 0) return DRL_OK;
  DRL_E_DISPATCH(dt, hipLaunchKernelGGL(masked_softmax_bwd_kernel<E>, dim3((rows + 3) / 4), dim3(256), 0,
                                        static_cast<hipStream_t>(stream), static_cast<const E*>(probs), dprobs,
                                        static_cast<E*>(dscores), rows, Tk, scale));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_add_rmsnorm_fwd(const float* x_in, const void* delta, float* x_out, const float* weight, void* y, int32_t dt,
                        float* rstd, int64_t N, int64_t H, float eps, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_in && weight && y, "NULL input");
  DRL_CHECK_ARG(N >= 0 && H >= 4 && H % 4 == 0, "bad shape (H %% 4 == 0 required)");
  if (N == 0) return DRL_OK;
  auto al = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
  if (dt == DRL_BF16 && H == 896 && al(x_in, 8) && al(x_out, 8) && al(weight, 8) && al(delta, 4) && al(y, 4)) {
    hipLaunchKernelGGL(add_rmsnorm_fwd_vec_kernel<7>, dim3((N + 3) / 4), dim3(256), 0, static_cast<hipStream_t>(stream),
                       x_in, static_cast<const uint16_t*>(delta), x_out, weight, static_cast<uint16_t*>(y), rstd, N, eps);
    DRL_LAUNCH_CHECK();
    return DRL_OK;
  }
  DRL_E_DISPATCH(dt, hipLaunchKernelGGL(add_rmsnorm_fwd_kernel<E>, dim3((N + 3) / 4), dim3(256), 0,
                                        static_cast<hipStream_t>(stream), x_in, static_cast<const E*>(delta), x_out,
                                        weight, static_cast<E*>(y), rstd, N, H, eps));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_rmsnorm_bwd_workspace_bytes(int64_t N, int64_t H) {
  (void)N;
  return static_cast<size_t>(drl::cu_count()) * 2 * static_cast<size_t>(H) * sizeof(float);
}

int drl_rmsnorm_bwd(const float* x, const float* weight, const float* rstd, const void* dy, int32_t dt, float* dx,
                    float* dw, int64_t N, int64_t H, void* workspace, size_t workspace_bytes, void* stream) {
  return drl_rmsnorm_bwd_ex(x, weight, rstd, dy, dt, dx, dx, nullptr, dw, N, H, workspace, workspace_bytes, stream);
}

int drl_rmsnorm_bwd_ex(const float* x, const float* weight, const float* rstd, const void* dy, int32_t dt,
                       const float* dx_in, float* dx, void* dx_bf16, float* dw, int64_t N, int64_t H, void* workspace,
                       size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x && weight && rstd && dy && dx && dw, "NULL input");
  uint16_t* dx_lp = static_cast<uint16_t*>(dx_bf16);
  DRL_CHECK_ARG(N >= 1 && H >= 1 && 4 * H * sizeof(float) <= 64 * 1024, "bad shape");
  const int grid = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(cu_count()) * 2, (N + 3) / 4));
  if (workspace == nullptr || workspace_bytes < static_cast<size_t>(grid) * H * sizeof(float))
    return fail(DRL_ERR_WORKSPACE, "workspace too small");
  float* part = static_cast<float*>(workspace);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = H == 896 && (reinterpret_cast<uintptr_t>(x) & 7u) == 0 && (reinterpret_cast<uintptr_t>(dx) & 7u) == 0 &&
                   (reinterpret_cast<uintptr_t>(dx_in) & 7u) == 0 && (reinterpret_cast<uintptr_t>(dx_lp) & 3u) == 0 &&
                   (reinterpret_cast<uintptr_t>(weight) & 7u) == 0 &&
                   (reinterpret_cast<uintptr_t>(dy) & (dt == DRL_BF16 ? 3u : 7u)) == 0;
  if (vec) {
    DRL_E_DISPATCH(dt, hipLaunchKernelGGL((rmsnorm_bwd_vec_kernel<E, 7>), dim3(grid), dim3(256), 0, s, x, weight, rstd,
                                          static_cast<const E*>(dy), dx_in, dx, dx_lp, part, N));
  } else {
    DRL_E_DISPATCH(dt, hipLaunchKernelGGL(rmsnorm_bwd_kernel<E>, dim3(grid), dim3(256), 4 * H * sizeof(float), s, x,
                                          weight, rstd, static_cast<const E*>(dy), dx_in, dx, dx_lp, part, N, H));
  }
  DRL_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_kernel, dim3((H + 15) / 16), dim3(256), 0, s, part, static_cast<int64_t>(grid), H, dw);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_colsum_bf16_workspace_bytes(int64_t N, int64_t C) {
  (void)N;
  return static_cast<size_t>(16) * static_cast<size_t>(C) * sizeof(float);
}

int drl_colsum_bf16_acc(const void* x, int64_t ld, int64_t N, int64_t C, float* out, void* workspace,
                        size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x && out && N >= 1 && C >= 1 && ld >= C && ld % 8 == 0 && aligned16(x), "bad colsum input");
  if (workspace == nullptr || workspace_bytes < drl_colsum_bf16_workspace_bytes(N, C))
    return fail(DRL_ERR_WORKSPACE, "colsum workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t slices = std::min<int64_t>(16, (N + 31) / 32);
  const int64_t per = (N + slices - 1) / slices;
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(colsum_bf16_partial_kernel, dim3(static_cast<unsigned>((C + 63) / 64), static_cast<unsigned>(slices)),
                     dim3(256), 0, s, static_cast<const uint16_t*>(x), ld, N, C, per, part);
  DRL_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_kernel, dim3(static_cast<unsigned>((C + 15) / 16)), dim3(256), 0, s, part, slices, C, out);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_swiglu_fwd(const void* gate_up, void* out, int32_t dt, int64_t N, int64_t I, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(gate_up && out && N >= 0 && I >= 4 && I % 4 == 0, "bad input (I %% 4 == 0 required)");
  if (N == 0) return DRL_OK;
  if (dt == DRL_BF16 && I % 8 == 0 && N * I / 8 < (int64_t(1) << 31) && aligned16(gate_up) && aligned16(out)) {
    const uint32_t n8 = static_cast<uint32_t>(N * I / 8);
    hipLaunchKernelGGL(swiglu_fwd_bf16x8_kernel, dim3(grid_stride((n8 + 1) / 2)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(gate_up),
                       static_cast<uint16_t*>(out), n8, static_cast<uint32_t>(I / 8));
    DRL_LAUNCH_CHECK();
    return DRL_OK;
  }
  DRL_E_DISPATCH(dt, hipLaunchKernelGGL(swiglu_fwd_kernel<E>, dim3(grid_stride(N * I / 4)), dim3(256), 0,
                                        static_cast<hipStream_t>(stream), static_cast<const E*>(gate_up),
                                        static_cast<E*>(out), N, I));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_swiglu_bwd(const void* gate_up, const void* dout, void* dgate_up, int32_t dt, int64_t N, int64_t I,
                   void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(gate_up && dout && dgate_up && N >= 0 && I >= 4 && I % 4 == 0, "bad input (I %% 4 == 0 required)");
  if (N == 0) return DRL_OK;
  if (dt == DRL_BF16 && I % 8 == 0 && N * I / 8 < (int64_t(1) << 31) && aligned16(gate_up) && aligned16(dout) &&
      aligned16(dgate_up)) {
    const uint32_t n8 = static_cast<uint32_t>(N * I / 8);
    hipLaunchKernelGGL(swiglu_bwd_bf16x8_kernel, dim3(grid_stride(n8)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint16_t*>(gate_up), static_cast<const uint16_t*>(dout),
                       static_cast<uint16_t*>(dgate_up), n8, static_cast<uint32_t>(I / 8));
    DRL_LAUNCH_CHECK();
    return DRL_OK;
  }
  DRL_E_DISPATCH(dt, hipLaunchKernelGGL(swiglu_bwd_kernel<E>, dim3(grid_stride(N * I / 4)), dim3(256), 0,
                                        static_cast<hipStream_t>(stream), static_cast<const E*>(gate_up),
                                        static_cast<const E*>(dout), static_cast<E*>(dgate_up), N, I));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
