// K2 — log-prob of the label + entropy over the vocabulary (forward and backward), and
// K4 — decode-step token selection (greedy / temperature sampling) over the vocabulary.
//
// Both stream one (N, V) logits row per workgroup (V = 151,936 for Qwen2.5: 297 KiB bf16 per row),
// 8 bf16 / 4 f32 per lane per 16-B load, and keep all softmax state in registers with an online
// (running max) formulation, so the logits are read exactly once in the forward and once in the
// backward (which writes d logits in the same pass). HBM-bound: ~2V bytes per row forward.
// References: verl/utils/torch_functional.py:64-160 (logprobs / entropy), experimental/torch_functional.py
// :40-72 (backward formula), workers/rollout/hf_rollout.py:112-124 (HF generate greedy / sampling).
#include "common.h"

namespace drl {
namespace {

constexpr int kThreads = 256;

template <int DT>
struct Elem;
template <>
struct Elem<DRL_BF16> {
  static constexpr int kVec = 8;
  using T = uint16_t;
  __device__ static float get(const void* p, int64_t i) { return bf16_to_f32(static_cast<const uint16_t*>(p)[i]); }
  __device__ static void load_vec(const void* p, int64_t i, float v[8]) {
    const uint4 q = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
};
template <>
struct Elem<DRL_F32> {
  static constexpr int kVec = 4;
  using T = float;
  __device__ static float get(const void* p, int64_t i) { return static_cast<const float*>(p)[i]; }
  __device__ static void load_vec(const void* p, int64_t i, float v[4]) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
};

// logits / temperature. The logprob path mirrors `logits.div_(temperature)` (dp_actor.py:195,263), which
// runs in the logits' dtype, so a bf16 row is rounded back to bf16 after the division; the sampler
// mirrors HF's TemperatureLogitsWarper on fp32 scores (no rounding). Division, not a reciprocal
// multiply, to keep the reference's rounding.
template <int DT>
__device__ __forceinline__ float scale_logit(float x, float temp, bool apply, bool round_bf16 = true) {
  if (!apply) return x;
  const float z = x / temp;
  if constexpr (DT == DRL_BF16) return round_bf16 ? bf16_to_f32(f32_to_bf16(z)) : z;
  else return z;
}

// merge two online-softmax states (max m, sum_e s = sum exp(z-m), sum_ez t = sum exp(z-m)*z)
__device__ __forceinline__ void merge_state(float& m, float& s, float& t, float m2, float s2, float t2) {
  const float mn = fmaxf(m, m2);
  const float a = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m - mn) * 1.4426950408889634f);
  const float b = (m2 == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m2 - mn) * 1.4426950408889634f);
  s = s * a + s2 * b;
  t = t * a + t2 * b;
  m = mn;
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr int kUnroll = 4;  // 16-B loads in flight per lane per step

__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * kLog2e); }

template <bool WANT_T>
__device__ __forceinline__ void online_update(const float* v, int n, float& m, float& s, float& t) {
  float mx = -INFINITY;
  for (int k = 0; k < n; ++k) mx = fmaxf(mx, v[k]);
  if (mx > m) {
    const float sc = (m == -INFINITY) ? 0.f : fast_exp(m - mx);
    s *= sc;
    if (WANT_T) t *= sc;
    m = mx;
  }
  for (int k = 0; k < n; ++k) {
    const float e = fast_exp(v[k] - m);
    s += e;
    if (WANT_T) t = fmaf(e, v[k], t);
  }
}

template <int DT, bool WANT_T, bool ROUND = true>
__device__ __forceinline__ void row_softmax_state(const void* row, int64_t V, bool vec, float inv_t, bool apply_t,
                                                  float& m, float& s, float& t) {
  constexpr int kV = Elem<DT>::kVec;
  m = -INFINITY; s = 0.f; t = 0.f;
  const int tid = threadIdx.x;
  int64_t done = 0;
  if (vec) {
    const int64_t nfull = V / kV;  // vectors in the row
    const int64_t nsteps = nfull / (kThreads * kUnroll);
    for (int64_t st = 0; st < nsteps; ++st) {
      float v[kUnroll][kV];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        Elem<DT>::load_vec(row, ((st * kUnroll + u) * kThreads + tid) * kV, v[u]);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
        for (int k = 0; k < kV; ++k) v[u][k] = scale_logit<DT>(v[u][k], inv_t, apply_t, ROUND);
      }
      online_update<WANT_T>(&v[0][0], kUnroll * kV, m, s, t);
    }
    for (int64_t c = nsteps * kUnroll * kThreads + tid; c < nfull; c += kThreads) {
      float v[kV];
      Elem<DT>::load_vec(row, c * kV, v);
#pragma unroll
      for (int k = 0; k < kV; ++k) v[k] = scale_logit<DT>(v[k], inv_t, apply_t, ROUND);
      online_update<WANT_T>(v, kV, m, s, t);
    }
    done = nfull * kV;
  }
  for (int64_t i = done + tid; i < V; i += kThreads) {
    const float z = scale_logit<DT>(Elem<DT>::get(row, i), inv_t, apply_t, ROUND);
    online_update<WANT_T>(&z, 1, m, s, t);
  }
  // wave then block merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, kWave), s2 = __shfl_xor(s, o, kWave), t2 = WANT_T ? __shfl_xor(t, o, kWave) : 0.f;
    merge_state(m, s, t, m2, s2, t2);
  }
  __shared__ float sm[kThreads / kWave][3];
  const int lane = tid & 63, wave = tid >> 6;
  if (lane == 0) { sm[wave][0] = m; sm[wave][1] = s; sm[wave][2] = t; }
  __syncthreads();
  m = sm[0][0]; s = sm[0][1]; t = sm[0][2];
#pragma unroll
  for (int w = 1; w < kThreads / kWave; ++w) merge_state(m, s, t, sm[w][0], sm[w][1], sm[w][2]);
  __syncthreads();
}

template <int DT>
__global__ __launch_bounds__(kThreads) void logprob_fwd_kernel(const void* logits, int64_t V, int64_t ld,
                                                               const int64_t* labels, float inv_t, int apply_t,
                                                               bool vec, float* logp, float* ent, float* lse_out) {
  const int64_t r = blockIdx.x;
  const void* row = static_cast<const typename Elem<DT>::T*>(logits) + r * ld;
  float m, s, t;
  if (ent) row_softmax_state<DT, true>(row, V, vec, inv_t, apply_t, m, s, t);
  else row_softmax_state<DT, false>(row, V, vec, inv_t, apply_t, m, s, t);
  if (threadIdx.x == 0) {
    const float lse = m + logf(s);
    const int64_t y = labels[r];
    const float zy = scale_logit<DT>(Elem<DT>::get(row, y), inv_t, apply_t);
    logp[r] = zy - lse;
    if (ent) ent[r] = lse - t / s;
    if (lse_out) lse_out[r] = lse;
  }
}

// rollout.calculate_log_probs: log p(token) of the token the decode step just selected, under the actor's
// compute_log_prob definition (logits / temperature as logprob_fwd_kernel), read from out-of-band token columns
// (the graph-captured decode loop: column *dev_step of tokens / out)
template <int DT>
__global__ __launch_bounds__(kThreads) void token_logprob_kernel(const void* logits, int64_t V, int64_t ld,
                                                                 const int64_t* tokens, int64_t ld_tok,
                                                                 const int64_t* dev_step, float inv_t, int apply_t,
                                                                 bool vec, float* out, int64_t ld_out) {
  const int64_t r = blockIdx.x;
  const void* row = static_cast<const typename Elem<DT>::T*>(logits) + r * ld;
  float m, s, t;
  row_softmax_state<DT, false>(row, V, vec, inv_t, apply_t, m, s, t);
  if (threadIdx.x == 0) {
    const int64_t col = dev_step ? *dev_step : 0;
    const int64_t y = tokens[r * ld_tok + col];
    const float lse = m + logf(s);
    out[r * ld_out + col] = (y >= 0 && y < V) ? scale_logit<DT>(Elem<DT>::get(row, y), inv_t, apply_t) - lse : -INFINITY;
  }
}

template <int DT, int ODT>
__global__ __launch_bounds__(kThreads) void logprob_bwd_kernel(const void* logits, int64_t V, int64_t ld,
                                                               const int64_t* labels, float inv_t, int apply_t,
                                                               bool vec, const float* dlogp, const float* dent,
                                                               const float* lse, const float* ent, void* dlogits,
                                                               int64_t ld_out) {
  constexpr int kV = Elem<DT>::kVec;
  const int64_t r = blockIdx.x;
  const void* row = static_cast<const typename Elem<DT>::T*>(logits) + r * ld;
  const float gl = dlogp ? dlogp[r] : 0.f;
  const float ge = dent ? dent[r] : 0.f;
  const float L = lse[r];
  const float H = ent ? ent[r] : 0.f;
  const int64_t y = labels[r];
  // d/dz of (gl*logp + ge*H) = gl*(onehot - p) - ge*p*(log p + H); d/dx = that / T
  auto grad = [&](float x, int64_t i) -> float {
    const float z = scale_logit<DT>(x, inv_t, apply_t);
    const float lp = z - L;
    const float p = fast_exp(lp);
    float g = -gl * p - ge * p * (lp + H);
    if (i == y) g += gl;
    return apply_t ? g / inv_t : g;
  };
  auto store = [&](int64_t i, float g) {
    if constexpr (ODT == DRL_BF16) static_cast<uint16_t*>(dlogits)[r * ld_out + i] = f32_to_bf16(g);
    else static_cast<float*>(dlogits)[r * ld_out + i] = g;
  };
  const int tid = threadIdx.x;
  auto store_vec = [&](int64_t c, const float* g) {
    if constexpr (ODT == DRL_BF16) {
      uint32_t w[kV / 2];
#pragma unroll
      for (int k = 0; k < kV / 2; ++k)
        w[k] = static_cast<uint32_t>(f32_to_bf16(g[2 * k])) | (static_cast<uint32_t>(f32_to_bf16(g[2 * k + 1])) << 16);
      if constexpr (kV == 8)
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(dlogits) + r * ld_out + c * kV) = make_uint4(w[0], w[1], w[2], w[3]);
      else
        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(dlogits) + r * ld_out + c * kV) = make_uint2(w[0], w[1]);
    } else {
#pragma unroll
      for (int k = 0; k < kV; k += 4)
        *reinterpret_cast<float4*>(static_cast<float*>(dlogits) + r * ld_out + c * kV + k) =
            make_float4(g[k], g[k + 1], g[k + 2], g[k + 3]);
    }
  };
  if (vec) {
    const int64_t nfull = V / kV;
    const int64_t nsteps = nfull / (kThreads * kUnroll);
    for (int64_t st = 0; st < nsteps; ++st) {
      float v[kUnroll][kV];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) Elem<DT>::load_vec(row, ((st * kUnroll + u) * kThreads + tid) * kV, v[u]);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t c = (st * kUnroll + u) * kThreads + tid;
        float g[kV];
#pragma unroll
        for (int k = 0; k < kV; ++k) g[k] = grad(v[u][k], c * kV + k);
        store_vec(c, g);
      }
    }
    for (int64_t c = nsteps * kUnroll * kThreads + tid; c < nfull; c += kThreads) {
      float v[kV];
      Elem<DT>::load_vec(row, c * kV, v);
      float g[kV];
#pragma unroll
      for (int k = 0; k < kV; ++k) g[k] = grad(v[k], c * kV + k);
      store_vec(c, g);
    }
    for (int64_t i = nfull * kV + tid; i < V; i += kThreads) store(i, grad(Elem<DT>::get(row, i), i));
  } else {
    for (int64_t i = tid; i < V; i += kThreads) store(i, grad(Elem<DT>::get(row, i), i));
  }
}

// ------------------------------------------------------------------------------------------------ K4

// Philox4x32-10 block (seed = key, counter (c0,c1) | offset (c2,c3)); four 32-bit outputs
__device__ __forceinline__ uint4 philox4(uint64_t seed, uint64_t offset, uint64_t counter) {
  uint32_t c0 = static_cast<uint32_t>(counter), c1 = static_cast<uint32_t>(counter >> 32);
  uint32_t c2 = static_cast<uint32_t>(offset), c3 = static_cast<uint32_t>(offset >> 32);
  uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
    const uint32_t n0 = static_cast<uint32_t>(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n1 = static_cast<uint32_t>(p1);
    const uint32_t n2 = static_cast<uint32_t>(p0 >> 32) ^ c3 ^ k1;
    const uint32_t n3 = static_cast<uint32_t>(p0);
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

// Sampling: the categorical draw as a race of exponential clocks (race_key, common.h), run in two levels.
// The row is cut into fixed slices of kSlice tokens. Pass 1 reduces every slice to its mass
// (m_s = max kept logit, l_s = sum over kept tokens of exp((x_i - m_s) / T)); pass 2 races the slices with
// keys ln(mass_s) - ln(E_s) (one Philox word per slice), then races the tokens of the winning slice only.
// The min of independent clocks E_i / p_i over a slice is an Exp(mass_s) clock, so this is the flat race's
// distribution (softmax(z) over the kept tokens) exactly, while the per-token Philox + log work — which made
// the flat race VALU-bound at ~1.3 TB/s — is spent on kSlice tokens per row instead of V.

constexpr int kSlice = 2048;  // tokens per slice: one wave's stream in pass 1 (32 per lane)

// (key, index) -> one u64 whose unsigned max is torch.argmax: order-preserving key bits (NaN = maximum)
// in the high word, ~index in the low word (ties -> lowest index)
__device__ __forceinline__ uint64_t pack_key(float key, int64_t idx) {
  uint32_t b = __float_as_uint(key);
  b = isnan(key) ? 0xFFFFFFFFu : ((b & 0x80000000u) ? ~b : (b | 0x80000000u));
  return (static_cast<uint64_t>(b) << 32) | (0xFFFFFFFFu - static_cast<uint32_t>(idx));
}

__device__ __forceinline__ uint64_t max_u64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t other = (static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(v >> 32), o, kWave)) << 32) |
                           __shfl_xor(static_cast<uint32_t>(v), o, kWave);
    v = max_u64(v, other);
  }
  return v;
}

// workgroup max; every thread gets the result (LDS slot array owned by the caller's call site)
__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t* s_slot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_max_u64(v);
  if (lane == 0) s_slot[wave] = v;
  __syncthreads();
  v = s_slot[0];
#pragma unroll
  for (int w = 1; w < kThreads / kWave; ++w) v = max_u64(v, s_slot[w]);
  return v;
}

struct SelectArgs {
  const void* logits;
  int64_t V, ld, ld_out, chunk;  // chunk: elements per workgroup slice of the greedy pass (multiple of 8)
  bool vec;
  int do_sample;
  float temp;
  uint64_t seed, offset;
  int64_t row_base, pad;
  const int64_t* eos;
  int n_eos;
  int32_t* unfinished;
  int64_t* out;
  const int64_t* dev_step;
  unsigned long long* best;  // (N) greedy running max per row; zero on entry, reset to zero by the finish kernel
  const float* thr;          // (N) top-k / top-p cut on z = logit / T (tokens below it never win), or nullptr
  float2* mass;              // (N, S) sampling slice masses (m_s, l_s)
  int64_t S;                 // slices per row, ceil(V / kSlice)
};

// Greedy: best packed logit over [blockIdx.x * chunk, ...) of row blockIdx.y, merged into best[r] with one
// atomic max (a handful of VALU ops per token: HBM-bound).
template <int DT>
__global__ __launch_bounds__(kThreads) void select_slice_kernel(SelectArgs a) {
  const int64_t r = blockIdx.y;
  const int tid = threadIdx.x;
  const void* row = static_cast<const typename Elem<DT>::T*>(a.logits) + r * a.ld;
  const int64_t begin = static_cast<int64_t>(blockIdx.x) * a.chunk;
  const int64_t end = begin + a.chunk < a.V ? begin + a.chunk : a.V;
  uint64_t best = 0;
  int64_t done = begin;
  if (a.vec) {
    const int64_t vend = begin + (end - begin) / 8 * 8;
    for (int64_t i = begin + 8 * tid; i < vend; i += 8 * kThreads) {
      float v[8];
      Elem<DT>::load_vec(row, i, v);
      if constexpr (DT == DRL_F32) Elem<DT>::load_vec(row, i + 4, v + 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) best = max_u64(best, pack_key(v[k], i + k));
    }
    done = vend;
  }
  for (int64_t i = done + tid; i < end; i += kThreads) best = max_u64(best, pack_key(Elem<DT>::get(row, i), i));
  __shared__ uint64_t s_best[kThreads / kWave];
  best = block_max_u64(best, s_best);
  if (tid == 0)
    __hip_atomic_fetch_max(a.best + r, static_cast<unsigned long long>(best), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Sampling pass 1: wave w of workgroup (x, r) reduces slice s = 4x + w of row r to (m_s, l_s) over the kept
// tokens (z = x / T >= thr[r]); l_s = 0 for a slice with no kept token. 32 tokens per lane held in
// registers: one max, then one exp2 per token — no Philox, no log.
template <int DT, bool FILTER>
__global__ __launch_bounds__(kThreads) void select_mass_kernel(SelectArgs a) {
  constexpr int kV = Elem<DT>::kVec, kPer = kSlice / kWave;
  const int64_t r = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int64_t s = static_cast<int64_t>(blockIdx.x) * (kThreads / kWave) + (threadIdx.x >> 6);
  if (s >= a.S) return;  // no barrier in this kernel
  const void* row = static_cast<const typename Elem<DT>::T*>(a.logits) + r * a.ld;
  const int64_t begin = s * kSlice;
  float v[kPer];
  if (a.vec && begin + kSlice <= a.V) {
#pragma unroll
    for (int j = 0; j < kPer / kV; ++j) Elem<DT>::load_vec(row, begin + (j * kWave + lane) * kV, v + j * kV);
  } else {
#pragma unroll
    for (int j = 0; j < kPer / kV; ++j)
#pragma unroll
      for (int k = 0; k < kV; ++k) {
        const int64_t i = begin + (j * kWave + lane) * kV + k;
        v[j * kV + k] = i < a.V ? Elem<DT>::get(row, i) : -INFINITY;
      }
  }
  const bool apply_t = a.temp != 1.0f;
  if constexpr (FILTER) {
    const float cut = a.thr[r];
#pragma unroll
    for (int k = 0; k < kPer; ++k) v[k] = scale_logit<DT>(v[k], a.temp, apply_t, false) >= cut ? v[k] : -INFINITY;
  }
  float m = v[0];
#pragma unroll
  for (int k = 1; k < kPer; ++k) m = fmaxf(m, v[k]);
  m = wave_max(m);
  float l = 0.f;
  if (m != -INFINITY) {
    const float c = kLog2e / a.temp, mc = m * c;  // exp((x - m) / T) = exp2(x c - m c)
#pragma unroll
    for (int k = 0; k < kPer; ++k) l += __builtin_amdgcn_exp2f(fmaf(v[k], c, -mc));
  }
  l = wave_sum(l);
  if (lane == 0) a.mass[r * a.S + s] = make_float2(m, l);
}

// Sampling pass 2, one workgroup per row: race the slices (key ln(mass_s) - ln(E_s), E_s from Philox word
// s & 3 of counter (row << 32 | 2^31 | s >> 2) — disjoint from the token counters i >> 2 < 2^30), then race
// the kept tokens of the winning slice (token keys z_i - ln(E_i) on counter (row << 32 | i >> 2), word i & 3),
// then the finished-row / eos bookkeeping of select_finish_kernel.
template <int DT, bool FILTER>
__global__ __launch_bounds__(kThreads) void select_pick_kernel(SelectArgs a) {
  const int64_t r = blockIdx.x;
  const int tid = threadIdx.x;
  const uint64_t off = a.offset + (a.dev_step ? static_cast<uint64_t>(*a.dev_step) : 0ull);
  const uint64_t ctr_row = static_cast<uint64_t>(a.row_base + r) << 32;
  const bool apply_t = a.temp != 1.0f;
  __shared__ uint64_t s_slot[2][kThreads / kWave];
  uint64_t best = 0;
  for (int64_t s = tid; s < a.S; s += kThreads) {
    const float2 ms = a.mass[r * a.S + s];
    float key = -INFINITY;
    if (!(ms.y <= 0.f)) {  // NaN mass races (and wins) like a NaN token in the flat race
      const uint4 p = philox4(a.seed, off, ctr_row | 0x80000000ull | static_cast<uint64_t>(s >> 2));
      const uint32_t w[4] = {p.x, p.y, p.z, p.w};
      const float lnmass = scale_logit<DT>(ms.x, a.temp, apply_t, false) + 0.6931471805599453f * __builtin_amdgcn_logf(ms.y);
      key = race_key(lnmass, w[s & 3]);
    }
    best = max_u64(best, pack_key(key, s));
  }
  best = block_max_u64(best, s_slot[0]);
  const int64_t win = static_cast<int64_t>(0xFFFFFFFFu - static_cast<uint32_t>(best));
  const void* row = static_cast<const typename Elem<DT>::T*>(a.logits) + r * a.ld;
  const float cut = FILTER ? a.thr[r] : -INFINITY;
  auto key_of = [&](float x, uint32_t bits) -> float {
    const float z = scale_logit<DT>(x, a.temp, apply_t, false);
    return (!FILTER || z >= cut) ? race_key(z, bits) : -INFINITY;
  };
  const int64_t begin = win * kSlice;
  const int64_t end = begin + kSlice < a.V ? begin + kSlice : a.V;
  best = 0;
  static_assert(kSlice == 8 * kThreads, "one 8-token group per thread");
  if (a.vec && end - begin == kSlice) {
    const int64_t i = begin + 8 * tid;
    float v[8];
    Elem<DT>::load_vec(row, i, v);
    if constexpr (DT == DRL_F32) Elem<DT>::load_vec(row, i + 4, v + 4);
    const uint4 p0 = philox4(a.seed, off, ctr_row | static_cast<uint64_t>(i >> 2));
    const uint4 p1 = philox4(a.seed, off, ctr_row | static_cast<uint64_t>((i >> 2) + 1));
    const uint32_t bits[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) best = max_u64(best, pack_key(key_of(v[k], bits[k]), i + k));
  } else {
    for (int64_t i = begin + tid; i < end; i += kThreads) {
      const uint4 p = philox4(a.seed, off, ctr_row | static_cast<uint64_t>(i >> 2));
      const uint32_t w[4] = {p.x, p.y, p.z, p.w};
      best = max_u64(best, pack_key(key_of(Elem<DT>::get(row, i), w[i & 3]), i));
    }
  }
  best = block_max_u64(best, s_slot[1]);
  if (tid == 0) {
    const int64_t choice = static_cast<int64_t>(0xFFFFFFFFu - static_cast<uint32_t>(best));
    const bool alive = a.unfinished ? a.unfinished[r] != 0 : true;
    const int64_t tok = alive ? choice : a.pad;
    a.out[r * a.ld_out + (a.dev_step ? *a.dev_step : 0)] = tok;
    if (a.unfinished && alive) {
      for (int k = 0; k < a.n_eos; ++k)
        if (tok == a.eos[k]) { a.unfinished[r] = 0; break; }
    }
  }
}

// One thread per row: decode the winning index, reset best[r], apply the finished-row / eos bookkeeping.
__global__ __launch_bounds__(kThreads) void select_finish_kernel(SelectArgs a, int64_t N) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (r >= N) return;
  const uint64_t b = a.best[r];
  a.best[r] = 0;
  const int64_t choice = static_cast<int64_t>(0xFFFFFFFFu - static_cast<uint32_t>(b));
  const bool alive = a.unfinished ? a.unfinished[r] != 0 : true;
  const int64_t tok = alive ? choice : a.pad;
  a.out[r * a.ld_out + (a.dev_step ? *a.dev_step : 0)] = tok;
  if (a.unfinished && alive) {
    for (int k = 0; k < a.n_eos; ++k)
      if (tok == a.eos[k]) { a.unfinished[r] = 0; break; }
  }
}

// Top-k / top-p (HF TopKLogitsWarper then TopPLogitsWarper, after TemperatureLogitsWarper) as one cut per
// row on z = logit / T: one workgroup per row, radix select over order-preserving 32-bit keys, 8-bit digits,
// LDS histograms with integer atomics (so the cut is deterministic, identical in graph replay and eager).
//   top-k: the k-th largest z (all ties with it kept, as `scores < topk[..., -1]` removes only smaller ones);
//   top-p: over the top-k survivors, masses e = exp(z - max) in 2^40 fixed point; the cut is the value of the
//   last token (descending) whose strictly-higher mass is < top_p * sum — the nucleus of
//   `cumsum(softmax(sorted ascending)) <= 1 - top_p` removed; ties at the cut are all kept (HF's sort order
//   decides among them). thr[r] = max of the two cuts; the sampler skips tokens with z < thr[r].
__device__ __forceinline__ uint32_t order_key(float z) {
  const uint32_t b = __float_as_uint(z);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int DT>
__global__ __launch_bounds__(kThreads) void select_threshold_kernel(SelectArgs a, int top_k, float top_p) {
  const int64_t r = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const void* row = static_cast<const typename Elem<DT>::T*>(a.logits) + r * a.ld;
  const int64_t V = a.V;
  auto zat = [&](int64_t i) { return scale_logit<DT>(Elem<DT>::get(row, i), a.temp, a.temp != 1.0f, false); };
  __shared__ unsigned long long hist[256];
  __shared__ float s_red[kThreads / kWave];
  __shared__ unsigned long long s_u64[kThreads / kWave];
  __shared__ uint32_t s_prefix;
  __shared__ unsigned long long s_target;

  // radix select: find the key of the element where the (count or mass) from the top crosses `target`
  // (returned prefix = full 32-bit key). weight(i) = 1 (top-k) or fixed-point mass (top-p).
  auto radix = [&](auto weight, unsigned long long target, uint32_t lo_key) -> uint32_t {
    uint32_t prefix = 0;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      for (int b = tid; b < 256; b += kThreads) hist[b] = 0;
      __syncthreads();
      for (int64_t i = tid; i < V; i += kThreads) {
        const float z = zat(i);
        const uint32_t k = order_key(z);
        if (k < lo_key) continue;
        if (pass > 0 && (k >> (shift + 8)) != prefix) continue;
        const unsigned long long w = weight(z);
        if (w) atomicAdd(&hist[(k >> shift) & 0xFFu], w);
      }
      __syncthreads();
      if (tid == 0) {
        unsigned long long above = 0;
        int b = 255;
        for (; b > 0; --b) {
          if (above + hist[b] >= target) break;
          above += hist[b];
        }
        s_prefix = (prefix << 8) | static_cast<uint32_t>(b);
        s_target = target - above;
      }
      __syncthreads();
      prefix = s_prefix;
      target = s_target;
      __syncthreads();
    }
    return prefix;
  };

  uint32_t cut_key = 0;
  if (top_k > 0 && top_k < V)
    cut_key = radix([](float) { return 1ull; }, static_cast<unsigned long long>(top_k), 0u);
  if (top_p < 1.0f) {
    // max z (the top token always survives top-k)
    float m = -INFINITY;
    for (int64_t i = tid; i < V; i += kThreads) m = fmaxf(m, zat(i));
    m = wave_max(m);
    if (lane == 0) s_red[wave] = m;
    __syncthreads();
    m = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
    const float scale = 1099511627776.0f;  // 2^40 fixed point: exact, associative integer sums
    const uint32_t kk = cut_key;
    auto mass = [&](float z) -> unsigned long long {
      return order_key(z) >= kk ? static_cast<unsigned long long>(__expf(z - m) * scale) : 0ull;
    };
    unsigned long long tot = 0;
    for (int64_t i = tid; i < V; i += kThreads) tot += mass(zat(i));
    tot = wave_sum_u64(tot);
    if (lane == 0) s_u64[wave] = tot;
    __syncthreads();
    tot = s_u64[0] + s_u64[1] + s_u64[2] + s_u64[3];
    // keep j iff mass strictly above j < top_p * total: the cut token is where the running mass from the top
    // first reaches that target (a token exactly at it is the last one kept)
    unsigned long long target = static_cast<unsigned long long>(static_cast<double>(top_p) * static_cast<double>(tot));
    if (target < 1) target = 1;
    const uint32_t pk = radix(mass, target, kk);
    cut_key = pk > cut_key ? pk : cut_key;
  }
  if (tid == 0) const_cast<float*>(a.thr)[r] = cut_key ? key_value(cut_key) : -INFINITY;
}

bool rows_aligned(const void* p, int64_t ld, int dt) {
  const int64_t esz = dt == DRL_BF16 ? 2 : 4;
  return aligned16(p) && ((ld * esz) % 16 == 0);
}

}  // namespace
}  // namespace drl

extern "C" {

int drl_logprob_entropy_fwd(const void* logits, int32_t dt, int64_t N, int64_t V, int64_t ld, const int64_t* labels,
                            float temperature, float* log_prob, float* entropy, float* lse_out, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(logits && labels && log_prob, "NULL input");
  DRL_CHECK_ARG(N >= 0 && V >= 1 && ld >= V, "bad shape N=%lld V=%lld ld=%lld", (long long)N, (long long)V, (long long)ld);
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "logits dtype must be F32 or BF16");
  DRL_CHECK_ARG(temperature > 0.f, "temperature must be > 0");
  DRL_CHECK_ARG(N <= 0x7fffffff, "too many rows");
  if (N == 0) return DRL_OK;
  const bool vec = rows_aligned(logits, ld, dt);
  const float inv_t = temperature;  // kernels divide by it
  const int apply_t = temperature != 1.0f;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dt == DRL_BF16)
    hipLaunchKernelGGL(logprob_fwd_kernel<DRL_BF16>, dim3(N), dim3(kThreads), 0, s, logits, V, ld, labels, inv_t,
                       apply_t, vec, log_prob, entropy, lse_out);
  else
    hipLaunchKernelGGL(logprob_fwd_kernel<DRL_F32>, dim3(N), dim3(kThreads), 0, s, logits, V, ld, labels, inv_t,
                       apply_t, vec, log_prob, entropy, lse_out);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_token_logprob(const void* logits, int32_t dt, int64_t N, int64_t V, int64_t ld, const int64_t* tokens,
                      int64_t ld_tok, const int64_t* dev_step, float temperature, float* out, int64_t ld_out,
                      void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(logits && tokens && out, "NULL input");
  DRL_CHECK_ARG(N >= 0 && V >= 1 && ld >= V && ld_tok >= 1 && ld_out >= 1, "bad shape");
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "logits dtype must be F32 or BF16");
  DRL_CHECK_ARG(temperature > 0.f, "temperature must be > 0");
  DRL_CHECK_ARG(N <= 0x7fffffff, "too many rows");
  if (N == 0) return DRL_OK;
  const bool vec = rows_aligned(logits, ld, dt);
  const int apply_t = temperature != 1.0f;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dt == DRL_BF16)
    hipLaunchKernelGGL(token_logprob_kernel<DRL_BF16>, dim3(N), dim3(kThreads), 0, s, logits, V, ld, tokens, ld_tok,
                       dev_step, temperature, apply_t, vec, out, ld_out);
  else
    hipLaunchKernelGGL(token_logprob_kernel<DRL_F32>, dim3(N), dim3(kThreads), 0, s, logits, V, ld, tokens, ld_tok,
                       dev_step, temperature, apply_t, vec, out, ld_out);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_logprob_entropy_bwd(const void* logits, int32_t dt, int64_t N, int64_t V, int64_t ld, const int64_t* labels,
                            float temperature, const float* dlog_prob, const float* dentropy, const float* lse,
                            const float* entropy, void* dlogits, int32_t odt, int64_t ld_out, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(logits && labels && lse && dlogits, "NULL input");
  DRL_CHECK_ARG(dentropy == nullptr || entropy != nullptr, "dentropy needs the forward entropy");
  DRL_CHECK_ARG(N >= 0 && V >= 1 && ld >= V && ld_out >= V, "bad shape");
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "logits dtype must be F32 or BF16");
  DRL_CHECK_ARG(odt == DRL_BF16 || odt == DRL_F32, "dlogits dtype must be F32 or BF16");
  DRL_CHECK_ARG(temperature > 0.f, "temperature must be > 0");
  DRL_CHECK_ARG(dlogits != logits || (dt == odt && ld == ld_out), "in-place backward needs identical layout");
  if (N == 0) return DRL_OK;
  const bool vec = rows_aligned(logits, ld, dt) && rows_aligned(dlogits, ld_out, odt) &&
                   (dt == DRL_BF16 ? 8 : 4) % (odt == DRL_BF16 ? 4 : 4) == 0;
  const float inv_t = temperature;  // kernels divide by it
  const int apply_t = temperature != 1.0f;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define DRL_BWD(DT, ODT)                                                                                      \
  hipLaunchKernelGGL((logprob_bwd_kernel<DT, ODT>), dim3(N), dim3(kThreads), 0, s, logits, V, ld, labels, inv_t, \
                     apply_t, vec, dlog_prob, dentropy, lse, entropy, dlogits, ld_out)
  if (dt == DRL_BF16 && odt == DRL_BF16) DRL_BWD(DRL_BF16, DRL_BF16);
  else if (dt == DRL_BF16) DRL_BWD(DRL_BF16, DRL_F32);
  else if (odt == DRL_BF16) DRL_BWD(DRL_F32, DRL_BF16);
  else DRL_BWD(DRL_F32, DRL_F32);
#undef DRL_BWD
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

// best (N x u64) + the top-k / top-p cut (N x f32, padded to 8 B) + the sampling slice masses (N x S x float2)
size_t drl_select_tokens_workspace_bytes(int64_t N, int64_t V) {
  if (N <= 0 || V <= 0) return 0;
  const int64_t S = (V + drl::kSlice - 1) / drl::kSlice;
  return static_cast<size_t>(N) * 16 + static_cast<size_t>(N) * static_cast<size_t>(S) * 8;
}

int drl_select_tokens(const void* logits, int32_t dt, int64_t N, int64_t V, int64_t ld,
                      const drl_sampling_params* p, int32_t* unfinished, int64_t* out_tokens, int64_t ld_out,
                      void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(logits && p && out_tokens, "NULL input");
  DRL_CHECK_ARG(N >= 0 && V >= 1 && ld >= V && V < (int64_t(1) << 32), "bad shape");
  DRL_CHECK_ARG(dt == DRL_BF16 || dt == DRL_F32, "logits dtype must be F32 or BF16");
  DRL_CHECK_ARG(p->n_eos == 0 || p->eos_ids != nullptr, "n_eos > 0 but eos_ids is NULL");
  const bool sample = p->do_sample && p->temperature > 0.f;
  const bool filter = sample && ((p->top_k > 0 && p->top_k < V) || p->top_p < 1.0f);
  DRL_CHECK_ARG(!sample || (p->top_p > 0.f && p->top_p <= 1.0f), "top_p must be in (0, 1], got %f", p->top_p);
  if (N == 0) return DRL_OK;
  DRL_CHECK_ARG(N <= 65535, "too many rows for one launch");
  if (!workspace || workspace_bytes < drl_select_tokens_workspace_bytes(N, V) || (reinterpret_cast<uintptr_t>(workspace) & 7u))
    return fail(DRL_ERR_WORKSPACE, "select workspace: need %zu 8-byte aligned bytes", drl_select_tokens_workspace_bytes(N, V));
  SelectArgs a{};
  a.logits = logits; a.V = V; a.ld = ld; a.ld_out = ld_out; a.vec = rows_aligned(logits, ld, dt);
  a.do_sample = sample; a.temp = sample ? p->temperature : 1.0f;
  a.seed = p->seed; a.offset = p->offset; a.row_base = p->row_base; a.pad = p->pad_token_id;
  a.eos = p->eos_ids; a.n_eos = p->n_eos; a.unfinished = unfinished; a.out = out_tokens;
  a.dev_step = p->dev_step;
  a.best = static_cast<unsigned long long*>(workspace);
  a.thr = filter ? reinterpret_cast<const float*>(static_cast<char*>(workspace) + static_cast<size_t>(N) * 8) : nullptr;
  a.S = (V + kSlice - 1) / kSlice;
  a.mass = reinterpret_cast<float2*>(static_cast<char*>(workspace) + static_cast<size_t>(N) * 16);
  // slices per row: ~4 workgroups per CU over the whole launch, >= 2048 elements per slice
  const int64_t want = (4 * static_cast<int64_t>(cu_count()) + N - 1) / N;
  const int64_t max_slices = (V + 2047) / 2048;
  const int64_t slices = want < 1 ? 1 : (want > max_slices ? max_slices : want);
  a.chunk = ((V + slices - 1) / slices + 7) / 8 * 8;
  const dim3 grid(static_cast<unsigned>((V + a.chunk - 1) / a.chunk), static_cast<unsigned>(N));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (filter) {
    const int k = (p->top_k > 0 && p->top_k < V) ? p->top_k : 0;
    if (dt == DRL_BF16)
      hipLaunchKernelGGL(select_threshold_kernel<DRL_BF16>, dim3(static_cast<unsigned>(N)), dim3(kThreads), 0, s, a, k,
                         p->top_p);
    else
      hipLaunchKernelGGL(select_threshold_kernel<DRL_F32>, dim3(static_cast<unsigned>(N)), dim3(kThreads), 0, s, a, k,
                         p->top_p);
    DRL_LAUNCH_CHECK();
  }
  if (sample) {
    const dim3 g1(static_cast<unsigned>((a.S + kThreads / kWave - 1) / (kThreads / kWave)), static_cast<unsigned>(N));
    const dim3 g2(static_cast<unsigned>(N));
#define DRL_SAMPLE(DT, F)                                                                   \
  do {                                                                                      \
    hipLaunchKernelGGL((select_mass_kernel<DT, F>), g1, dim3(kThreads), 0, s, a);           \
    DRL_LAUNCH_CHECK();                                                                     \
    hipLaunchKernelGGL((select_pick_kernel<DT, F>), g2, dim3(kThreads), 0, s, a);           \
  } while (0)
    if (dt == DRL_BF16) { if (filter) DRL_SAMPLE(DRL_BF16, true); else DRL_SAMPLE(DRL_BF16, false); }
    else { if (filter) DRL_SAMPLE(DRL_F32, true); else DRL_SAMPLE(DRL_F32, false); }
#undef DRL_SAMPLE
    DRL_LAUNCH_CHECK();
    return DRL_OK;
  }
  if (dt == DRL_BF16) hipLaunchKernelGGL((select_slice_kernel<DRL_BF16>), grid, dim3(kThreads), 0, s, a);
  else hipLaunchKernelGGL((select_slice_kernel<DRL_F32>), grid, dim3(kThreads), 0, s, a);
  DRL_LAUNCH_CHECK();
  hipLaunchKernelGGL(select_finish_kernel, dim3(static_cast<unsigned>((N + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     s, a, N);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
