// K1 — fused actor loss (vanilla PPO clip + dual clip, entropy bonus, KL-to-ref), forward AND backward,
// one pass over HBM. Replaces dp_actor.py:419-466 (+ core_algos.py:703-736, 815-889, 1272-1307).
//
// Layout: the (B, R) float32 inputs are flattened to N = B*R tokens in 1024-token chunks, 4 tokens per lane
// (16-B nontemporal loads/stores, 1 KiB per wave-instruction per stream). Chunks are dealt to the workgroups
// grid-stride (chunk = base + u * grid): at any moment the whole grid sweeps one window of every stream, which
// keeps DRAM pages open; 2 workgroups per CU with 2 chunks in flight per lane (measured on K1's exact shape,
// tools/probes/k1_stream_probe.hip: 6.1 TB/s vs 5.4 TB/s for contiguous per-workgroup runs at 4 per CU).
// token-mean needs the global mask count before any gradient can be written. K1a streams ONLY the mask
// (8 B/token for int64), writes it back as a 1-bit image (N/8 bytes, one 64-bit ballot per wave and
// element slot) and folds the count (fixed order, last workgroup); K1b reads that count, the other inputs and the
// bit image (1/8 B/token instead of 8) and writes the gradients: 36.25 B/token of traffic for 36 B/token
// of algorithmic bytes, no grid barrier. A caller that already holds sum(mask) (params.token_count) skips
// K1a: K1b then reads the mask itself and the whole fwd+bwd is one streaming pass. The other modes know their gradient weights up front
// (seq-mean-token-mean gets per-row counts from a small pre-pass) and run K1b alone. Forward scalars:
// per-workgroup partials (double) reduced by the last workgroup in a fixed order, so the results are
// bitwise reproducible run to run.
#include "common.h"

namespace drl {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = kThreads * 4;  // 1024 tokens: one workgroup iteration, 16 mask words (4 waves x 4 slots)
constexpr int kNumPartials = 8;
#ifndef DRL_K1_PACK_U
#define DRL_K1_PACK_U 4
#endif
#ifndef DRL_K1_U
#define DRL_K1_U 1
#endif
#ifndef DRL_K1_PIPE
#define DRL_K1_PIPE 1
#endif

// every K1 byte is touched once: nontemporal (streaming) loads and stores keep it out of the caches'
// way (measured on the 5-read/2-write shape: 5.16 -> 5.49 TB/s, tools/hbm_probe.hip)
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef long long nt_i2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ nt_f4 ldnt(const float* p) { return __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p)); }
__device__ __forceinline__ nt_i2 ldnt(const int64_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const nt_i2*>(p)); }
__device__ __forceinline__ void stnt(float* p, nt_f4 v) { __builtin_nontemporal_store(v, reinterpret_cast<nt_f4*>(p)); }


// Zero before the first call (the caller zeroes the workspace once at allocation); K1b's last workgroup
// zeroes it again after every other workgroup has finished with it, so a workspace reused on one stream
// needs no per-call memset (a fill kernel + a kernel boundary, ~6 us per call). Every read of a header
// field is an agent-scope atomic (sc1: never served from a stale L2 line of another XCD), every write a
// write-through atomic store or RMW.
struct Header {
  unsigned ticket;
  unsigned nonbinary;  // some mask value is not 0/1: K1b reads the original mask instead of the bits
  unsigned pack_ticket;
  unsigned pad;
  double mask_total;   // token-mean: sum(mask), reduced by K1a's last workgroup in a fixed order
  double pad2;         // 32 B: one fill on the stream
};

struct Args {
  const float* old_lp;
  const float* lp;
  const float* adv;
  const void* mask;
  const float* ent;
  const float* ref;
  const float* rowcnt;               // seq-mean-token-mean: sum(mask) per row
  const unsigned long long* bits;    // token-mean: packed mask (nullptr: read `mask`)
  const double* token_count;         // token-mean: caller-provided sum(mask) (one-pass form), or nullptr
  float* dlp;
  float* dent;
  float* out;
  Header* hdr;
  double* partials;                  // gridDim.x * kNumPartials
  int64_t N, B, R;
  float lo, hi, clip_c, ent_coef, kl_coef, lsf;
  int mode, kl;
  int policy;  // DRL_POLICY_*
};

template <int MDT, bool NT = true>
__device__ __forceinline__ void load_mask4(const void* m, int64_t t, int64_t N, float v[4]) {
  if (t + 3 < N) {
    if constexpr (MDT == DRL_I64) {
      const int64_t* p = static_cast<const int64_t*>(m) + t;
      nt_i2 a, b;
      if constexpr (NT) { a = ldnt(p); b = ldnt(p + 2); }
      else { a = *reinterpret_cast<const nt_i2*>(p); b = *reinterpret_cast<const nt_i2*>(p + 2); }
      v[0] = static_cast<float>(a.x); v[1] = static_cast<float>(a.y);
      v[2] = static_cast<float>(b.x); v[3] = static_cast<float>(b.y);
    } else if constexpr (MDT == DRL_I32) {
      const int4 a = *reinterpret_cast<const int4*>(static_cast<const int32_t*>(m) + t);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else if constexpr (MDT == DRL_U8) {
      const uint32_t a = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(m) + t);
      v[0] = a & 0xff; v[1] = (a >> 8) & 0xff; v[2] = (a >> 16) & 0xff; v[3] = a >> 24;
    } else {
      const nt_f4 a = ldnt(static_cast<const float*>(m) + t);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (t + j < N) ? mask_at<MDT>(m, t + j) : 0.f;
  }
}

// 4 mask values at t (all inside N), unguarded. int64 -> float through the low word unless some lane holds a
// value outside int32 (then the exact 64-bit conversion, wave-uniform branch): the general conversion costs
// ~10 VALU instructions per value, a third of K1's per-token work
template <int MDT>
__device__ __forceinline__ void load_mask4_full(const void* m, int64_t t, float v[4]) {
  if constexpr (MDT == DRL_I64) {
    const int64_t* p = static_cast<const int64_t*>(m) + t;
    const nt_i2 a = ldnt(p), b = ldnt(p + 2);
    const long long x[4] = {a.x, a.y, b.x, b.y};
    bool big = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) big |= x[j] != static_cast<long long>(static_cast<int32_t>(x[j]));
    if (__builtin_expect(__any(big), 0)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = static_cast<float>(x[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = static_cast<float>(static_cast<int32_t>(x[j]));
    }
  } else if constexpr (MDT == DRL_I32) {
    const int4 a = *reinterpret_cast<const int4*>(static_cast<const int32_t*>(m) + t);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else if constexpr (MDT == DRL_U8) {
    const uint32_t a = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(m) + t);
    v[0] = a & 0xff; v[1] = (a >> 8) & 0xff; v[2] = (a >> 16) & 0xff; v[3] = a >> 24;
  } else {
    const nt_f4 a = ldnt(static_cast<const float*>(m) + t);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
}

__device__ __forceinline__ void load4(const float* p, int64_t t, int64_t N, float v[4]) {
  if (t + 3 < N) {
    const nt_f4 a = ldnt(p + t);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (t + j < N) ? p[t + j] : 0.f;
  }
}

__device__ __forceinline__ void store4(float* p, int64_t t, int64_t N, const float v[4]) {
  if (t + 3 < N) {
    stnt(p + t, nt_f4{v[0], v[1], v[2], v[3]});
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (t + j < N) p[t + j] = v[j];
  }
}

#ifndef DRL_K1_FASTEXP
#define DRL_K1_FASTEXP 1
#endif
// exp of the clamped K3 log-ratio (|x| <= 20; no decision is taken on its value): v_exp_f32(x * log2 e) is within ~|x| * 2^-24 relative of the
// correctly rounded value (<= 1.2e-6 at the clamp, ~1e-7 for the usual |x| < 1), 2 VALU instructions
// instead of ocml's ~10 (range reduction + ldexp + overflow selects)
__device__ __forceinline__ float k1_exp(float x) {
#if DRL_K1_FASTEXP
  return __expf(x);
#else
  return expf(x);
#endif
}

// kl_penalty value and d/d logprob (core_algos.py:1272-1307)
__device__ __forceinline__ void kl_term(int kl, float lp, float ref, float& val, float& dval) {
  switch (kl) {
    case DRL_KL_K1: val = lp - ref; dval = 1.f; break;
    case DRL_KL_ABS: {
      const float d = lp - ref;
      val = fabsf(d);
      dval = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      break;
    }
    case DRL_KL_K2: {
      const float d = lp - ref;
      val = 0.5f * (d * d);
      dval = d;
      break;
    }
    case DRL_KL_K3: {
      const float raw = ref - lp;
      const float k = fminf(fmaxf(raw, -20.f), 20.f);
      const float g1 = (raw >= -20.f && raw <= 20.f) ? 1.f : 0.f;
      const float r = k1_exp(k);
      const float kld = (r - k) - 1.f;
      val = fminf(fmaxf(kld, -10.f), 10.f);
      const float g2 = (kld >= -10.f && kld <= 10.f) ? 1.f : 0.f;
      dval = -(r - 1.f) * g1 * g2;
      break;
    }
    default: val = 0.f; dval = 0.f;
  }
}

// K1a (token-mean only): stream the mask once; per 1024-token chunk store one 64-bit ballot per wave and
// element slot (N/8 bytes in total) and accumulate sum(mask) per workgroup; the last workgroup folds the
// per-workgroup counts in a fixed order into the header.
template <int MDT>
__global__ __launch_bounds__(kThreads) void mask_pack_kernel(const void* mask, int64_t N, unsigned long long* bits,
                                                             double* counts, Header* hdr) {
  constexpr int kU = DRL_K1_PACK_U;  // chunks in flight per lane (2 x 16-B loads each for an int64 mask)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t nchunks = (N + kChunk - 1) / kChunk;
  float cnt = 0.f;
  double dcnt = 0.0;
  bool nonbin = false;
  const int64_t G = gridDim.x;
  for (int64_t c0 = blockIdx.x; c0 < nchunks; c0 += G * kU) {
    float m[kU][4];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t t = (c0 + u * G) * kChunk + tid * 4;
      if (c0 + u * G < nchunks) load_mask4<MDT>(mask, t, N, m[u]);
      else m[u][0] = m[u][1] = m[u][2] = m[u][3] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t cu = c0 + u * G;
      unsigned long long mine = 0;  // lane j (< 4) stores the wave's ballot of element slot j
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cnt += m[u][j];
        nonbin |= (m[u][j] != 0.f && m[u][j] != 1.f);
        const unsigned long long b = __ballot(m[u][j] != 0.f);
        mine = lane == j ? b : mine;
      }
      // the wave's 4 words are contiguous: one 32-B store instead of four single-lane ones
      if (lane < 4 && cu < nchunks) bits[cu * 16 + wave * 4 + lane] = mine;
    }
    if (cnt >= 8388608.f) { dcnt += cnt; cnt = 0.f; }  // keep float partials exact
  }
  dcnt += cnt;
  if (__any(nonbin) && lane == 0) atomicOr(&hdr->nonbinary, 1u);
  dcnt = wave_sum(dcnt);
  __shared__ double red[kThreads / kWave];
  if (lane == 0) red[wave] = dcnt;
  __syncthreads();
  if (tid == 0) store_sc1(counts + blockIdx.x, red[0] + red[1] + red[2] + red[3]);
  // the last workgroup folds the per-workgroup counts (fixed order) so K1b reads one value
  if (last_block_ticket(&hdr->pack_ticket)) {
    double v = 0.0;
    for (unsigned g = tid; g < gridDim.x; g += kThreads) v += load_sc1(counts + g);
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    if (tid == 0) store_sc1(&hdr->mask_total, red[0] + red[1] + red[2] + red[3]);
  }
}

// K1b: per-token loss terms, gradients and the workgroup's partial sums. Grid-stride 1024-token chunks,
// DRL_K1_U in flight per workgroup; 4 tokens per lane per chunk.
// FMODE / FKL: the aggregation mode and KL type fixed at compile time for the hot configurations
// (kRuntime = read from Args), so the per-token math carries no mode branches. The chunk loop itself is
// instantiated per (mask source, entropy present, KL present) and runs branch-free over the chunks that lie
// wholly inside N: a bounds-checked load is a branch, and hipcc waits vmcnt(0) at the join of every such
// branch, which serialised the 6-7 loads per chunk (measured 0.54 -> see DESIGN.md §4).
constexpr int kRuntime = -2;

struct Chunk {
  float m[4], old[4], lp[4], A[4], en[4], rf[4];
};

struct Sums {
  float pg = 0.f, clip = 0.f, kl = 0.f, cliplow = 0.f, ent = 0.f, kld = 0.f, cnt = 0.f;
};

// FULL: the chunk lies wholly inside N (no bounds checks, no branches); else every access is guarded
template <int MDT, bool BITS, bool ENT, bool KL, bool FULL>
__device__ __forceinline__ void load_chunk(const Args& a, int64_t c, int64_t N, int tid, int lane, int wave, Chunk& k) {
  const int64_t t = c * kChunk + tid * 4;
  if constexpr (FULL) {
    if constexpr (BITS) {
      // the wave's four 64-bit ballots (32 contiguous bytes, the same address on every lane)
      const nt_i2* bp = reinterpret_cast<const nt_i2*>(a.bits + c * 16 + wave * 4);
      const nt_i2 b0 = bp[0], b1 = bp[1];
      const unsigned long long w[4] = {static_cast<unsigned long long>(b0.x), static_cast<unsigned long long>(b0.y),
                                       static_cast<unsigned long long>(b1.x), static_cast<unsigned long long>(b1.y)};
#pragma unroll
      for (int j = 0; j < 4; ++j) k.m[j] = ((w[j] >> lane) & 1ull) ? 1.f : 0.f;
    } else {
      load_mask4_full<MDT>(a.mask, t, k.m);
    }
    const nt_f4 o = ldnt(a.old_lp + t), l = ldnt(a.lp + t), A = ldnt(a.adv + t);
    k.old[0] = o.x; k.old[1] = o.y; k.old[2] = o.z; k.old[3] = o.w;
    k.lp[0] = l.x; k.lp[1] = l.y; k.lp[2] = l.z; k.lp[3] = l.w;
    k.A[0] = A.x; k.A[1] = A.y; k.A[2] = A.z; k.A[3] = A.w;
    if constexpr (ENT) {
      const nt_f4 e = ldnt(a.ent + t);
      k.en[0] = e.x; k.en[1] = e.y; k.en[2] = e.z; k.en[3] = e.w;
    }
    if constexpr (KL) {
      const nt_f4 r = ldnt(a.ref + t);
      k.rf[0] = r.x; k.rf[1] = r.y; k.rf[2] = r.z; k.rf[3] = r.w;
    }
  } else {
    const int64_t tt = c * kChunk < N ? t : N;  // past the end: every load4 takes its bounds path and yields 0
    if (BITS && c * kChunk < N) {
#pragma unroll
      for (int j = 0; j < 4; ++j) k.m[j] = ((a.bits[c * 16 + wave * 4 + j] >> lane) & 1ull) ? 1.f : 0.f;
    } else {
      load_mask4<MDT>(a.mask, tt, N, k.m);
    }
    load4(a.old_lp, tt, N, k.old);
    load4(a.lp, tt, N, k.lp);
    load4(a.adv, tt, N, k.A);
    if constexpr (ENT) load4(a.ent, tt, N, k.en);
    if constexpr (KL) load4(a.ref, tt, N, k.rf);
  }
}

// per-token loss terms + gradients of one chunk (past the end, t >= N: nothing counted or stored)
template <int MODE, int KLT, bool ENT, bool KL, bool FULL>
__device__ __forceinline__ void process_chunk(const Args& a, const Chunk& k, int64_t c, int64_t N, int tid,
                                              float inv_denom_tm, Sums& S) {
  const int mode = MODE != kRuntime ? MODE : a.mode;
  const int kl = KLT != kRuntime ? KLT : a.kl;
  const float inv_B = 1.0f / static_cast<float>(a.B), inv_R = 1.0f / static_cast<float>(a.R);
  const bool tm = mode == DRL_AGG_TOKEN_MEAN, smtm = mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN;
  const int64_t t = c * kChunk + tid * 4;
  const float* m = k.m;
  const float* old = k.old;
  const float* lp = k.lp;
  const float* A = k.A;
  float g_lp[4], g_en[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool valid = FULL || t + j < N;
    // compute_policy_loss_vanilla, float32 with the reference's op order
    const float raw = lp[j] - old[j];
    const float nkl = fminf(fmaxf(raw, -20.f), 20.f);
    const float gate = (raw >= -20.f && raw <= 20.f) ? 1.f : 0.f;
    const float ratio = expf(nkl);  // exact: the clip / tie decisions on ratio must match torch.exp
    const float negA = -A[j];
    const float L1 = negA * ratio;
    const float rc = fminf(fmaxf(ratio, a.lo), a.hi);
    const float gc = (ratio >= a.lo && ratio <= a.hi) ? 1.f : 0.f;
    const float L2 = negA * rc;
    const float C1 = fmaxf(L1, L2);
    const float w1 = L1 > L2 ? 1.f : (L1 == L2 ? 0.5f : 0.f);  // torch.maximum splits ties
    const float dC1 = (w1 + (1.f - w1) * gc) * negA;
    const float L3 = negA * a.clip_c;
    const float C2 = fminf(L3, C1);
    const float wc = C1 < L3 ? 1.f : (C1 == L3 ? 0.5f : 0.f);
    const bool neg = A[j] < 0.f;
    const bool gpg = a.policy == DRL_POLICY_GPG;  // uniform per launch
    // GPG (core_algos.py:957-975): pg = -log_prob * advantages, d pg / d log_prob = -A
    const float pg = gpg ? (-lp[j]) * A[j] : (neg ? C2 : C1);
    const float dpg = gpg ? -A[j] : (neg ? wc * dC1 : dC1) * ratio * gate;

    const float mj = valid ? m[j] : 0.f;
    const bool mb = mj != 0.f;
    // d agg / d loss_mat of this token, and its forward contribution
    float rc_inv = 0.f;
    if (smtm) rc_inv = 1.0f / a.rowcnt[valid ? (t + j) / a.R : 0];
    float w;
    if (tm) w = mb ? inv_denom_tm * mj : 0.f;
    else if (mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM) w = inv_B * mj;
    else if (smtm) w = mj * (inv_B * rc_inv);
    else w = inv_R * mj;
    // token-mean sums where(mask, x, 0) * mask; the seq modes x * mask (core_algos.py:716-733)
    auto agg_val = [&](float x) -> float {
      if (tm) return mb ? x * mj : 0.f;
      if (smtm) return (x * mj) * rc_inv;
      return x * mj;
    };
    if (valid) {
      S.pg += agg_val(pg);
      S.cnt += mj;
      if (!gpg) {  // GPG reports clipfrac / ppo_kl / clipfrac_lower as 0
        S.clip += (mb && L2 > L1) ? mj : 0.f;
        S.kl += mb ? -nkl * mj : 0.f;
        S.cliplow += (mb && C1 > L3 && neg) ? mj : 0.f;
      }
    }
    float gl = w * dpg;
    if constexpr (KL) {
      float kv, dk;
      kl_term(kl, lp[j], k.rf[j], kv, dk);
      if (valid) S.kld += agg_val(kv);
      gl += a.kl_coef * (w * dk);
    }
    if constexpr (ENT) {
      if (valid) S.ent += agg_val(k.en[j]);
    }
    g_lp[j] = a.lsf * gl;
    g_en[j] = a.ent_coef != 0.f ? a.lsf * (-a.ent_coef * w) : 0.f;
  }
  if constexpr (FULL) {
    if (a.dlp != nullptr) stnt(a.dlp + t, nt_f4{g_lp[0], g_lp[1], g_lp[2], g_lp[3]});
    if (a.dent != nullptr) stnt(a.dent + t, nt_f4{g_en[0], g_en[1], g_en[2], g_en[3]});
  } else {
    if (a.dlp != nullptr) store4(a.dlp, t, N, g_lp);
    if (a.dent != nullptr) store4(a.dent, t, N, g_en);
  }
}

// the workgroup's chunks: blockIdx.x, +G, +2G, ...; kU full chunks loaded before any is computed, then the
// remainder (at most kU - 1 full chunks and the partial last chunk) one at a time
template <int MDT, int MODE, int KLT, bool BITS, bool ENT, bool KL>
__device__ __forceinline__ void stream_chunks(const Args& a, float inv_denom_tm, Sums& S) {
  constexpr int kU = DRL_K1_U;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t N = a.N, G = gridDim.x;
  const int64_t nfull = N / kChunk, nchunks = (N + kChunk - 1) / kChunk;
  int64_t c0 = blockIdx.x;
  auto load_group = [&](int64_t c, Chunk* ck) {
#pragma unroll
    for (int u = 0; u < kU; ++u) load_chunk<MDT, BITS, ENT, KL, true>(a, c + u * G, N, tid, lane, wave, ck[u]);
  };
  auto process_group = [&](int64_t c, const Chunk* ck) {
#pragma unroll
    for (int u = 0; u < kU; ++u) process_chunk<MODE, KLT, ENT, KL, true>(a, ck[u], c + u * G, N, tid, inv_denom_tm, S);
  };
#if DRL_K1_PIPE
  // software pipeline, ping-pong register sets: the next group's loads are in flight while this group computes
  if (c0 + (kU - 1) * G < nfull) {
    Chunk x[kU], y[kU];
    load_group(c0, x);
    for (;;) {
      int64_t cn = c0 + G * kU;
      bool more = cn + (kU - 1) * G < nfull;
      if (more) load_group(cn, y);
      process_group(c0, x);
      c0 = cn;
      if (!more) break;
      cn = c0 + G * kU;
      more = cn + (kU - 1) * G < nfull;
      if (more) load_group(cn, x);
      process_group(c0, y);
      c0 = cn;
      if (!more) break;
    }
  }
#else
  for (; c0 + (kU - 1) * G < nfull; c0 += G * kU) {
    Chunk ck[kU];
    load_group(c0, ck);
    process_group(c0, ck);
  }
#endif
  for (; c0 < nchunks; c0 += G) {
    Chunk ck;
    if (c0 < nfull) {
      load_chunk<MDT, BITS, ENT, KL, true>(a, c0, N, tid, lane, wave, ck);
      process_chunk<MODE, KLT, ENT, KL, true>(a, ck, c0, N, tid, inv_denom_tm, S);
    } else {
      load_chunk<MDT, BITS, ENT, KL, false>(a, c0, N, tid, lane, wave, ck);
      process_chunk<MODE, KLT, ENT, KL, false>(a, ck, c0, N, tid, inv_denom_tm, S);
    }
  }
}

template <int MDT, int MODE, int KLT, bool BITS>
__device__ __forceinline__ void stream_dispatch(const Args& a, bool has_ent, bool has_kl, float inv_denom_tm, Sums& S) {
  if constexpr (KLT == DRL_KL_NONE) {
    if (has_ent) stream_chunks<MDT, MODE, KLT, BITS, true, false>(a, inv_denom_tm, S);
    else stream_chunks<MDT, MODE, KLT, BITS, false, false>(a, inv_denom_tm, S);
  } else if constexpr (KLT != kRuntime) {
    if (has_ent) stream_chunks<MDT, MODE, KLT, BITS, true, true>(a, inv_denom_tm, S);
    else stream_chunks<MDT, MODE, KLT, BITS, false, true>(a, inv_denom_tm, S);
  } else {
    if (has_ent && has_kl) stream_chunks<MDT, MODE, KLT, BITS, true, true>(a, inv_denom_tm, S);
    else if (has_ent) stream_chunks<MDT, MODE, KLT, BITS, true, false>(a, inv_denom_tm, S);
    else if (has_kl) stream_chunks<MDT, MODE, KLT, BITS, false, true>(a, inv_denom_tm, S);
    else stream_chunks<MDT, MODE, KLT, BITS, false, false>(a, inv_denom_tm, S);
  }
}

template <int MDT, int FMODE, int FKL>
__global__ __launch_bounds__(kThreads) void ppo_loss_kernel(Args a) {
  __shared__ double red[kThreads / kWave][kNumPartials];
  const int mode = FMODE != kRuntime ? FMODE : a.mode;
  const int kl = FKL != kRuntime ? FKL : a.kl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  float cnt_total = 0.f;
  bool use_bits = false;
  if (mode == DRL_AGG_TOKEN_MEAN && a.token_count != nullptr) {
    cnt_total = static_cast<float>(*a.token_count);  // one-pass form: the caller's count, mask read here
  } else if (mode == DRL_AGG_TOKEN_MEAN && a.bits != nullptr) {
    // global mask count, folded by the pack kernel's last workgroup
    cnt_total = static_cast<float>(load_sc1(&a.hdr->mask_total));
    use_bits = __hip_atomic_load(&a.hdr->nonbinary, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  }
  const float denom_tm = cnt_total + 1e-8f;       // masked_mean: sum / (mask.sum() + 1e-8)
  const float inv_denom_tm = 1.0f / denom_tm;     // upstream / D once, then * mask (MeanBackward style)
  const bool has_ent = a.ent != nullptr, has_kl = kl != DRL_KL_NONE;
  Sums S;
  if (use_bits) stream_dispatch<MDT, FMODE, FKL, true>(a, has_ent, has_kl, inv_denom_tm, S);
  else stream_dispatch<MDT, FMODE, FKL, false>(a, has_ent, has_kl, inv_denom_tm, S);
  const float s_pg = S.pg, s_clip = S.clip, s_kl = S.kl, s_cliplow = S.cliplow, s_ent = S.ent, s_kld = S.kld,
              s_cnt = S.cnt;

  // ---- workgroup partials -> the last workgroup reduces all of them in a fixed order
  const float vals[kNumPartials] = {s_pg, s_clip, s_kl, s_cliplow, s_ent, s_kld, s_cnt, 0.f};
#pragma unroll
  for (int k = 0; k < kNumPartials; ++k) {
    const double v = wave_sum(static_cast<double>(vals[k]));
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  if (tid < kNumPartials) store_sc1(a.partials + tid * gridDim.x + blockIdx.x, red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid]);
  if (last_block_ticket(&a.hdr->ticket)) {
#pragma unroll
    for (int k = 0; k < kNumPartials; ++k) {
      double v = 0.0;
      for (unsigned g = tid; g < gridDim.x; g += kThreads) v += load_sc1(a.partials + k * gridDim.x + g);
      v = wave_sum(v);
      if (lane == 0) red[wave][k] = v;
    }
    __syncthreads();
    if (tid == 0) {
      double r[kNumPartials];
      for (int k = 0; k < kNumPartials; ++k) r[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
      const double cnt = r[6];
      const double dm = static_cast<double>(static_cast<float>(cnt) + 1e-8f);
      auto agg = [&](double s) -> double {
        if (mode == DRL_AGG_TOKEN_MEAN) return s / dm;
        if (mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM || mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) return s / static_cast<double>(a.B);
        return s / static_cast<double>(a.R);
      };
      const double pg_loss = agg(r[0]);
      const double ent_loss = has_ent ? agg(r[4]) : 0.0;
      const double kl_loss = has_kl ? agg(r[5]) : 0.0;
      double total = pg_loss;
      if (a.ent_coef != 0.f) total -= ent_loss * a.ent_coef;
      if (has_kl) total += kl_loss * a.kl_coef;
      a.out[DRL_PPO_OUT_PG_LOSS] = static_cast<float>(pg_loss);
      a.out[DRL_PPO_OUT_PG_CLIPFRAC] = static_cast<float>(r[1] / dm);
      a.out[DRL_PPO_OUT_PPO_KL] = static_cast<float>(r[2] / dm);
      a.out[DRL_PPO_OUT_PG_CLIPFRAC_LOWER] = static_cast<float>(r[3] / dm);
      a.out[DRL_PPO_OUT_ENTROPY_LOSS] = static_cast<float>(ent_loss);
      a.out[DRL_PPO_OUT_KL_LOSS] = static_cast<float>(kl_loss);
      a.out[DRL_PPO_OUT_LOSS] = static_cast<float>(total * a.lsf);
      a.out[DRL_PPO_OUT_MASK_COUNT] = static_cast<float>(cnt);
      // every other workgroup has taken its ticket, i.e. is past its last header read: leave the header zero
      __hip_atomic_store(&a.hdr->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.hdr->pack_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.hdr->nonbinary, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      store_sc1(&a.hdr->mask_total, 0.0);
    }
  }
}

// sum(mask) per row, one wave per row (seq-mean-token-mean pre-pass)
template <int MDT>
__global__ __launch_bounds__(256) void row_count_kernel(const void* mask, int64_t B, int64_t R, float* rowcnt) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float c = 0.f;
  for (int64_t t = lane; t < R; t += 64) c += mask_at<MDT>(mask, row * R + t);
  c = wave_sum(c);
  if (lane == 0) rowcnt[row] = c;
}

#ifndef DRL_K1_WG_PER_CU
#define DRL_K1_WG_PER_CU 2
#endif
#ifndef DRL_K1_PACK_WG_PER_CU
#define DRL_K1_PACK_WG_PER_CU 4
#endif
int max_grid() { return cu_count() * (DRL_K1_WG_PER_CU > DRL_K1_PACK_WG_PER_CU ? DRL_K1_WG_PER_CU : DRL_K1_PACK_WG_PER_CU); }

struct Layout {
  size_t partials, rowcnt, counts, bits, seqrow, seqpart, seqsel, total;
};

Layout ws_layout(int64_t B, int64_t R) {
  Layout L{};
  const size_t grid = static_cast<size_t>(max_grid());
  const size_t nchunks = static_cast<size_t>((B * R + kChunk - 1) / kChunk);
  L.partials = round_up(sizeof(Header), 256);
  L.rowcnt = round_up(L.partials + grid * kNumPartials * sizeof(double), 256);
  L.counts = round_up(L.rowcnt + static_cast<size_t>(B) * sizeof(float), 256);
  L.bits = round_up(L.counts + grid * sizeof(double), 256);
  L.seqrow = round_up(L.bits + nchunks * 16 * sizeof(unsigned long long), 256);
  L.seqpart = round_up(L.seqrow + static_cast<size_t>(B) * 8 * sizeof(float), 256);
  L.seqsel = round_up(L.seqpart + static_cast<size_t>(B) * kNumPartials * sizeof(double), 256);
  L.total = round_up(L.seqsel + 256, 256);
  return L;
}

template <int MDT>
int launch(Args a, const Layout& L, char* ws, hipStream_t s) {
  if (a.mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) {
    hipLaunchKernelGGL(row_count_kernel<MDT>, dim3((a.B + 3) / 4), dim3(256), 0, s, a.mask, a.B, a.R,
                       const_cast<float*>(a.rowcnt));
    DRL_LAUNCH_CHECK();
  }
  const int64_t nchunks = (a.N + kChunk - 1) / kChunk;
  if (a.mode == DRL_AGG_TOKEN_MEAN && (a.dlp != nullptr || a.dent != nullptr) && a.token_count == nullptr) {
    auto* bits = reinterpret_cast<unsigned long long*>(ws + L.bits);
    auto* counts = reinterpret_cast<double*>(ws + L.counts);
    const int g1 = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(cu_count()) * DRL_K1_PACK_WG_PER_CU,
                                                      (nchunks + DRL_K1_PACK_U - 1) / DRL_K1_PACK_U));
    hipLaunchKernelGGL(mask_pack_kernel<MDT>, dim3(g1), dim3(kThreads), 0, s, a.mask, a.N, bits, counts, a.hdr);
    DRL_LAUNCH_CHECK();
    a.bits = bits;
  }
  // one chunk per workgroup until the grid reaches DRL_K1_WG_PER_CU workgroups per CU
  const int grid = static_cast<int>(std::max<int64_t>(
      1, std::min<int64_t>(static_cast<int64_t>(cu_count()) * DRL_K1_WG_PER_CU, nchunks)));
  if (a.mode == DRL_AGG_TOKEN_MEAN && a.kl == DRL_KL_K3)
    hipLaunchKernelGGL((ppo_loss_kernel<MDT, DRL_AGG_TOKEN_MEAN, DRL_KL_K3>), dim3(grid), dim3(kThreads), 0, s, a);
  else if (a.mode == DRL_AGG_TOKEN_MEAN && a.kl == DRL_KL_NONE)
    hipLaunchKernelGGL((ppo_loss_kernel<MDT, DRL_AGG_TOKEN_MEAN, DRL_KL_NONE>), dim3(grid), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL((ppo_loss_kernel<MDT, kRuntime, kRuntime>), dim3(grid), dim3(kThreads), 0, s, a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

__global__ __launch_bounds__(256) void kl_penalty_kernel(const float* lp, const float* ref, int64_t n, int kl, float* out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float v, d;
    kl_term(kl, lp[i], ref[i], v, d);
    out[i] = v;
  }
}

// agg_loss forward: weighted partial sums per workgroup, last workgroup finishes (fixed order).
template <int MDT>
__global__ __launch_bounds__(256) void agg_loss_kernel(const float* x, const void* mask, int64_t B, int64_t R,
                                                       int mode, const float* rowcnt, double* partials, Header* hdr,
                                                       float* out) {
  const int64_t N = B * R;
  double s = 0.0, c = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < N;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float m = mask_at<MDT>(mask, i);
    float v;
    if (mode == DRL_AGG_TOKEN_MEAN) v = m != 0.f ? x[i] * m : 0.f;
    else if (mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) v = (x[i] * m) / rowcnt[i / R];
    else v = x[i] * m;
    s += v;
    c += m;
  }
  s = wave_sum(s);
  c = wave_sum(c);
  __shared__ double red[4][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red[wave][0] = s; red[wave][1] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    store_sc1(partials + 2 * blockIdx.x, red[0][0] + red[1][0] + red[2][0] + red[3][0]);
    store_sc1(partials + 2 * blockIdx.x + 1, red[0][1] + red[1][1] + red[2][1] + red[3][1]);
  }
  if (last_block_ticket(&hdr->ticket) && threadIdx.x == 0) {
    double S = 0.0, C = 0.0;
    for (unsigned b = 0; b < gridDim.x; ++b) { S += load_sc1(partials + 2 * b); C += load_sc1(partials + 2 * b + 1); }
    double r;
    if (mode == DRL_AGG_TOKEN_MEAN) r = S / static_cast<double>(static_cast<float>(C) + 1e-8f);
    else if (mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM || mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) r = S / static_cast<double>(B);
    else r = S / static_cast<double>(R);
    *out = static_cast<float>(r);
  }
}

template <int MDT>
int launch_agg(const float* x, const void* mask, int64_t B, int64_t R, int mode, char* ws, size_t off_part,
               size_t off_row, float* out, hipStream_t s) {  // workspace offsets from ws_layout()
  float* rowcnt = reinterpret_cast<float*>(ws + off_row);
  if (mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) {
    hipLaunchKernelGGL(row_count_kernel<MDT>, dim3((B + 3) / 4), dim3(256), 0, s, mask, B, R, rowcnt);
    DRL_LAUNCH_CHECK();
  }
  const int grid = static_cast<int>(std::min<int64_t>(max_grid(), (B * R + 255) / 256));
  hipLaunchKernelGGL(agg_loss_kernel<MDT>, dim3(grid), dim3(256), 0, s, x, mask, B, R, mode, rowcnt,
                     reinterpret_cast<double*>(ws + off_part), reinterpret_cast<Header*>(ws), out);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

// ------------------------------------------------------------------------------------------------------------
// Sequence-level policy losses: GSPO (core_algos.py:892-954) and GMPO geo_mean (core_algos.py:1143-1210), composed
// with the entropy bonus / KL term / loss scale of dp_actor.py:419-466 like K1. Their pg terms need per-row sums
// before any token's gradient, so they run as three small launches instead of K1's stream: (S1) per-row sums,
// one wave per row; (S2) one workgroup per row: per-token loss terms, d loss / d log_prob, d loss / d entropy and
// the row's partial forward sums; (S3) one workgroup folds the rows' partials in row order (deterministic).
// rowstat[b] = {sum(mask), sum(nak * mask), sum(nak_min * mask), sum(A * mask)}, nak = log_prob - old_log_prob.
struct SeqArgs {
  const float* old_lp;
  const float* lp;
  const float* adv;
  const void* mask;
  const float* ent;
  const float* ref;
  float* dlp;
  float* dent;
  float* out;
  float* rowstat;   // (B, 8)
  double* rowpart;  // (B, kNumPartials)
  unsigned* sel;    // covariance selection: {key threshold, flat-index cutoff at the threshold, take-all flag}
  float cov_ratio, cov_lb, cov_ub, ppo_kl_coef;
  uint32_t cov_seed;
  int64_t B, R;
  float lo, hi;          // GSPO: 1 - clip_ratio_low, 1 + clip_ratio_high (ratio space)
  float llo, lhi;        // GMPO: clip_ratio_low, clip_ratio_high (log-ratio space)
  float ent_coef, kl_coef, lsf;
  int mode, kl, policy;
};

// GMPO: nak clipped toward sign(A) (value) and d value / d nak (torch.min / torch.clamp backward)
__device__ __forceinline__ void geo_clip(float nak, float A, float llo, float lhi, float& v, float& d) {
  const float sg = A > 0.f ? 1.f : (A < 0.f ? -1.f : 0.f);
  const float ncl = fminf(fmaxf(nak, -llo), lhi);
  const float gc = (nak >= -llo && nak <= lhi) ? 1.f : 0.f;
  const float x = sg * nak, y = sg * ncl;
  v = sg * fminf(x, y);
  const float wa = x < y ? 1.f : (x == y ? 0.5f : 0.f);
  d = sg * sg * (wa + (1.f - wa) * gc);
}

// ---- clip_cov / kl_cov token selection (core_algos.py:978-1140). Both rank tokens by the covariance
// cov = (A - mean A) (log_prob - mean log_prob) over the batch:
//   kl_cov: means over the valid tokens (plain means of the selected entries); the k = max(1, int(n_valid *
//   kl_cov_ratio)) largest covariances (torch.topk; equal values at the k-th taken lowest flat index first)
//   get the loss -A r + ppo_kl_coef |log_prob - old|;
//   clip_cov: masked means (sum(x m) / (sum(m) + 1e-8)); candidates are valid tokens with lb < cov < ub that the
//   PPO clip did not already clip; min(clip_num, #candidates) of them (clip_num = max(int(clip_cov_ratio *
//   sum(m)), 1)) get corr = 0. The reference draws that subset with torch.randperm; here it is the candidates
//   with the smallest keys of a bijective 32-bit hash of (flat index ^ seed): uniformly random subsets, a
//   different draw (all candidates when they fit, which is deterministic in both).
__device__ __forceinline__ uint32_t cov_hash(uint32_t i, uint32_t seed) {  // murmur3 fmix32: a bijection
  uint32_t h = i ^ seed;
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t fkey(float v) {  // order-preserving key of a float
  const uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

struct CovSel {
  float mean_a, mean_lp;
  uint32_t thr, cut;  // threshold key, flat-index cutoff among keys equal to it
  int all;            // take every eligible token (clip_cov: the candidates fit into clip_num)
  int none;           // nothing selected
};

// batch means from the per-row sums (fixed order; every caller computes the same values)
__device__ __forceinline__ void cov_means(const SeqArgs& a, float& mean_a, float& mean_lp, float& n_valid,
                                          float& msum) {
  float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t b = 0; b < a.B; ++b) {
    const float* r = a.rowstat + 8 * b;
    s[0] += r[4]; s[1] += r[5]; s[2] += r[6]; s[3] += r[0]; s[4] += r[3]; s[5] += r[7];
  }
  n_valid = s[0];
  msum = s[3];
  if (a.policy == DRL_POLICY_KL_COV) { mean_a = s[1] / s[0]; mean_lp = s[2] / s[0]; }
  else { mean_a = s[4] / (s[3] + 1e-8f); mean_lp = s[5] / (s[3] + 1e-8f); }
}

// eligibility and ranking key of token i (larger key = picked first)
__device__ __forceinline__ bool cov_key(const SeqArgs& a, float mean_a, float mean_lp, int64_t i, float A, float lpv,
                                        float nak, float r, float m, uint32_t& key) {
  if (!(m > 0.f)) return false;
  const float c = (A - mean_a) * (lpv - mean_lp);
  if (a.policy == DRL_POLICY_KL_COV) { key = fkey(c); return true; }
  const float negA = -A;
  const float L1 = negA * r, L2 = negA * fminf(fmaxf(r, a.lo), a.hi);
  if (L2 > L1) return false;  // clip_by_origin
  if (!(c < a.cov_ub && c > a.cov_lb)) return false;
  key = ~cov_hash(static_cast<uint32_t>(i), a.cov_seed);  // smallest hash first
  return true;
}

__device__ __forceinline__ CovSel cov_selection(const SeqArgs& a) {
  CovSel cs{};
  float nv, msum;
  cov_means(a, cs.mean_a, cs.mean_lp, nv, msum);
  cs.thr = a.sel[0]; cs.cut = a.sel[1]; cs.all = static_cast<int>(a.sel[2] & 1u); cs.none = static_cast<int>(a.sel[2] >> 1);
  return cs;
}

__device__ __forceinline__ bool cov_picked(const SeqArgs& a, const CovSel& cs, int64_t i, float A, float lpv, float nak,
                                           float r, float m) {
  if (cs.none) return false;
  uint32_t key;
  if (!cov_key(a, cs.mean_a, cs.mean_lp, i, A, lpv, nak, r, m, key)) return false;
  if (cs.all) return true;
  return key > cs.thr || (key == cs.thr && static_cast<uint32_t>(i) <= cs.cut);
}

// One workgroup: the k-th largest key over the eligible tokens by an 8-bit radix select (4 passes, integer LDS
// histograms: deterministic), then the flat-index cutoff among the tokens equal to it (contiguous thread ranges +
// an exclusive scan). Writes sel = {threshold, cutoff, flags}.
__global__ __launch_bounds__(256) void cov_select_kernel(SeqArgs a, const void* mask, int mdt) {
  const int tid = threadIdx.x;
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_need;
  __shared__ unsigned s_cnt[256];
  float mean_a, mean_lp, nv, msum;
  cov_means(a, mean_a, mean_lp, nv, msum);
  const int64_t N = a.B * a.R;
  auto mask_of = [&](int64_t i) -> float {
    switch (mdt) {
      case DRL_I64: return mask_at<DRL_I64>(mask, i);
      case DRL_I32: return mask_at<DRL_I32>(mask, i);
      case DRL_U8: return mask_at<DRL_U8>(mask, i);
      default: return mask_at<DRL_F32>(mask, i);
    }
  };
  auto key_at = [&](int64_t i, uint32_t& key) -> bool {
    const float lpv = a.lp[i], nak = lpv - a.old_lp[i];
    return cov_key(a, mean_a, mean_lp, i, a.adv[i], lpv, nak, expf(nak), mask_of(i), key);
  };
  // how many to take
  unsigned cnt = 0;
  for (int64_t i = tid; i < N; i += 256) { uint32_t k; cnt += key_at(i, k) ? 1u : 0u; }
  s_cnt[tid] = cnt;
  __syncthreads();
  if (tid == 0) {
    unsigned tot = 0;
    for (int t = 0; t < 256; ++t) tot += s_cnt[t];
    unsigned need;
    if (a.policy == DRL_POLICY_KL_COV) {
      const unsigned kk = static_cast<unsigned>(static_cast<double>(nv) * static_cast<double>(a.cov_ratio));
      need = nv > 0.f ? (kk > 1u ? kk : 1u) : 0u;
    } else {
      const unsigned cn = static_cast<unsigned>(static_cast<double>(a.cov_ratio) * static_cast<double>(msum));
      need = cn > 1u ? cn : 1u;
    }
    unsigned flags = 0;
    if (need == 0 || tot == 0) flags = 2u;             // none
    else if (need >= tot) flags = 1u;                  // all eligible
    a.sel[2] = flags;
    s_need = (flags == 0) ? need : 0u;
  }
  __syncthreads();
  unsigned need = s_need;
  if (need == 0) return;  // uniform
  // radix select of the need-th largest key
  uint32_t prefix = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    hist[tid] = 0;
    __syncthreads();
    for (int64_t i = tid; i < N; i += 256) {
      uint32_t k;
      if (!key_at(i, k)) continue;
      if (pass > 0 && (k >> (shift + 8)) != prefix) continue;
      atomicAdd(&hist[(k >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned above = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (above + hist[b] >= need) break;
        above += hist[b];
      }
      s_prefix = (prefix << 8) | static_cast<uint32_t>(b);
      s_need = need - above;
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    __syncthreads();
  }
  // prefix = threshold key; take `need` of the tokens equal to it, lowest flat index first
  const int64_t per = (N + 255) / 256, lo = tid * per, hi = lo + per < N ? lo + per : N;
  unsigned eq = 0;
  for (int64_t i = lo; i < hi; ++i) { uint32_t k; eq += (key_at(i, k) && k == prefix) ? 1u : 0u; }
  s_cnt[tid] = eq;
  __syncthreads();
  if (tid == 0) {
    unsigned run = 0;
    for (int t = 0; t < 256; ++t) { const unsigned c = s_cnt[t]; s_cnt[t] = run; run += c; }
  }
  __syncthreads();
  const unsigned before = s_cnt[tid];
  if (before < need && before + eq >= need) {
    unsigned seen = before;
    for (int64_t i = lo; i < hi; ++i) {
      uint32_t k;
      if (key_at(i, k) && k == prefix && ++seen == need) { a.sel[1] = static_cast<unsigned>(i); break; }
    }
  }
  if (tid == 0) a.sel[0] = prefix;
}

template <int MDT>
__global__ __launch_bounds__(256) void seq_row_kernel(SeqArgs a) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.B) return;
  float c = 0.f, sk = 0.f, sm = 0.f, sa = 0.f, nv = 0.f, sav = 0.f, slv = 0.f, slm = 0.f;
  for (int64_t t = lane; t < a.R; t += 64) {
    const int64_t i = row * a.R + t;
    const float m = mask_at<MDT>(a.mask, i);
    const float nak = a.lp[i] - a.old_lp[i];
    c += m;
    sk += nak * m;
    if (a.policy == DRL_POLICY_GEO_MEAN) {
      float v, d;
      geo_clip(nak, a.adv[i], a.llo, a.lhi, v, d);
      sm += v * m;
    }
    sa += a.adv[i] * m;
    slm += a.lp[i] * m;
    if (m > 0.f) { nv += 1.f; sav += a.adv[i]; slv += a.lp[i]; }  // kl_cov: plain means over the valid tokens
  }
  c = wave_sum(c); sk = wave_sum(sk); sm = wave_sum(sm); sa = wave_sum(sa);
  nv = wave_sum(nv); sav = wave_sum(sav); slv = wave_sum(slv); slm = wave_sum(slm);
  if (lane == 0) {
    float* r = a.rowstat + 8 * row;
    r[0] = c; r[1] = sk; r[2] = sm; r[3] = sa; r[4] = nv; r[5] = sav; r[6] = slv; r[7] = slm;
  }
}

template <int MDT>
__global__ __launch_bounds__(256) void seq_token_kernel(SeqArgs a) {
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float s_cnt[4];
  __shared__ double red[4][kNumPartials];
  // sum(mask) over the whole micro-batch (token-mean weights), the same fixed order in every workgroup
  float c = 0.f;
  for (int64_t b = tid; b < a.B; b += 256) c += a.rowstat[8 * b];
  c = wave_sum(c);
  if (lane == 0) s_cnt[wave] = c;
  __syncthreads();
  const float cnt = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
  const float inv_denom_tm = 1.0f / (cnt + 1e-8f);
  const float rowcnt = a.rowstat[8 * row];
  const float inv_B = 1.0f / static_cast<float>(a.B), inv_R = 1.0f / static_cast<float>(a.R);
  const bool tm = a.mode == DRL_AGG_TOKEN_MEAN, smtm = a.mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN;
  const bool gspo = a.policy == DRL_POLICY_GSPO;
  const bool cov = a.policy == DRL_POLICY_CLIP_COV || a.policy == DRL_POLICY_KL_COV;
  // per-row scalars
  float ratio = 1.f, gate = 1.f, geo_scale = 0.f, pg_row = 0.f;
  CovSel cs{};
  if (cov) {
    cs = cov_selection(a);
  } else if (gspo) {  // seq log-ratio = sum(nak * mask) / clamp(len, 1), clamped at 10 (clamp passes the gradient at 10)
    const float seq_kl = a.rowstat[8 * row + 1] / fmaxf(rowcnt, 1.f);
    gate = seq_kl <= 10.f ? 1.f : 0.f;
    ratio = expf(fminf(seq_kl, 10.f));
  } else {  // GMPO: exp(mean clipped log-ratio), mean advantage; pg_row = -adv * ratio
    const float msum = rowcnt + 1e-8f;
    ratio = expf(a.rowstat[8 * row + 2] / msum);
    const float adv = a.rowstat[8 * row + 3] / msum;
    pg_row = -adv * ratio;
    geo_scale = ((-adv * ratio) / msum) * inv_B;  // d pg_loss / d nak_min_t = geo_scale * mask_t
  }
  float S[kNumPartials] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t t = tid; t < a.R; t += 256) {
    const int64_t i = row * a.R + t;
    const float mj = mask_at<MDT>(a.mask, i);
    const bool mb = mj != 0.f;
    const float lpv = a.lp[i], A = a.adv[i];
    const float nak = lpv - a.old_lp[i];
    float w;  // d agg / d loss_mat for the entropy / KL terms (loss_agg_mode)
    if (tm) w = mb ? inv_denom_tm * mj : 0.f;
    else if (a.mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM) w = inv_B * mj;
    else if (smtm) w = mj * (inv_B * (1.0f / rowcnt));
    else w = inv_R * mj;
    auto agg_val = [&](float x) -> float {
      if (tm) return mb ? x * mj : 0.f;
      if (smtm) return (x * mj) * (1.0f / rowcnt);
      return x * mj;
    };
    float dpg;
    if (cov) {  // token-level: ratio = exp(log_prob - old) unclamped, pg aggregated by loss_agg_mode
      const float r = expf(nak);
      const float negA = -A;
      const float L1 = negA * r;
      const bool picked = cov_picked(a, cs, i, A, lpv, nak, r, mj);
      if (a.policy == DRL_POLICY_KL_COV) {  // picked tokens: -A r + ppo_kl_coef |nak|
        const float pg = picked ? L1 + a.ppo_kl_coef * fabsf(nak) : L1;
        dpg = w * (negA * r + (picked ? a.ppo_kl_coef * (nak > 0.f ? 1.f : (nak < 0.f ? -1.f : 0.f)) : 0.f));
        S[0] += agg_val(pg);
        S[2] += mb ? fabsf(nak) * mj : 0.f;  // ppo_kl reported as masked_mean(|nak|)
      } else {  // clip_cov: PPO clip (no dual clip), picked tokens' loss zeroed (corr = 0)
        const float rc = fminf(fmaxf(r, a.lo), a.hi);
        const float gc = (r >= a.lo && r <= a.hi) ? 1.f : 0.f;
        const float L2 = negA * rc;
        const float corr = picked ? 0.f : 1.f;
        const float pg = fmaxf(L1, L2) * corr;
        const float w1 = L1 > L2 ? 1.f : (L1 == L2 ? 0.5f : 0.f);
        dpg = w * corr * ((w1 + (1.f - w1) * gc) * negA * r);
        S[0] += agg_val(pg);
        S[1] += (mb && picked) ? mj : 0.f;  // pg_clipfrac = masked_mean(corr == 0)
        S[2] += mb ? -nak * mj : 0.f;
      }
    } else if (gspo) {  // PPO clip on the sequence ratio, no dual clip; pg aggregated seq-mean-token-mean
      const float negA = -A;
      const float L1 = negA * ratio;
      const float rc = fminf(fmaxf(ratio, a.lo), a.hi);
      const float gc = (ratio >= a.lo && ratio <= a.hi) ? 1.f : 0.f;
      const float L2 = negA * rc;
      const float pg = fmaxf(L1, L2);
      const float w1 = L1 > L2 ? 1.f : (L1 == L2 ? 0.5f : 0.f);
      dpg = (mj * (inv_B * (1.0f / rowcnt))) * ((w1 + (1.f - w1) * gc) * negA * ratio * gate);
      S[0] += (pg * mj) * (1.0f / rowcnt);
      S[1] += (mb && L2 > L1) ? mj : 0.f;
    } else {
      float v, d;
      geo_clip(nak, A, a.llo, a.lhi, v, d);
      dpg = geo_scale * mj * d;
      const float ncl = fminf(fmaxf(nak, -a.llo), a.lhi);
      const bool clipped = nak != ncl;
      S[1] += (mb && clipped && A > 0.f) ? mj : 0.f;
      S[3] += (mb && clipped && A < 0.f) ? mj : 0.f;
    }
    if (!cov) S[2] += mb ? -nak * mj : 0.f;
    S[6] += mj;
    float gl = dpg;
    if (a.kl != DRL_KL_NONE) {
      float kv, dk;
      kl_term(a.kl, lpv, a.ref[i], kv, dk);
      S[5] += agg_val(kv);
      gl += a.kl_coef * (w * dk);
    }
    if (a.ent != nullptr) S[4] += agg_val(a.ent[i]);
    if (a.dlp != nullptr) a.dlp[i] = a.lsf * gl;
    if (a.dent != nullptr) a.dent[i] = a.ent_coef != 0.f ? a.lsf * (-a.ent_coef * w) : 0.f;
  }
  if (!gspo && !cov && tid == 0) S[0] = pg_row;  // GMPO: one sequence-level term per row
#pragma unroll
  for (int k = 0; k < kNumPartials; ++k) {
    const double v = wave_sum(static_cast<double>(S[k]));
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  if (tid < kNumPartials) a.rowpart[row * kNumPartials + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

__global__ __launch_bounds__(256) void seq_final_kernel(SeqArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double red[4][kNumPartials];
#pragma unroll
  for (int k = 0; k < kNumPartials; ++k) {
    double v = 0.0;
    for (int64_t b = tid; b < a.B; b += 256) v += a.rowpart[b * kNumPartials + k];
    v = wave_sum(v);
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  if (tid != 0) return;
  double r[kNumPartials];
  for (int k = 0; k < kNumPartials; ++k) r[k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  const double cnt = r[6];
  const double dm = static_cast<double>(static_cast<float>(cnt) + 1e-8f);
  auto agg = [&](double x) -> double {
    if (a.mode == DRL_AGG_TOKEN_MEAN) return x / dm;
    if (a.mode == DRL_AGG_SEQ_MEAN_TOKEN_SUM || a.mode == DRL_AGG_SEQ_MEAN_TOKEN_MEAN) return x / static_cast<double>(a.B);
    return x / static_cast<double>(a.R);
  };
  const bool cov = a.policy == DRL_POLICY_CLIP_COV || a.policy == DRL_POLICY_KL_COV;
  // GSPO: seq-mean of token-means; GMPO: mean over rows; clip_cov / kl_cov: agg_loss(loss_agg_mode)
  const double pg_loss = cov ? agg(r[0]) : r[0] / static_cast<double>(a.B);
  const bool has_ent = a.ent != nullptr, has_kl = a.kl != DRL_KL_NONE;
  const double ent_loss = has_ent ? agg(r[4]) : 0.0;
  const double kl_loss = has_kl ? agg(r[5]) : 0.0;
  double total = pg_loss;
  if (a.ent_coef != 0.f) total -= ent_loss * a.ent_coef;
  if (has_kl) total += kl_loss * a.kl_coef;
  a.out[DRL_PPO_OUT_PG_LOSS] = static_cast<float>(pg_loss);
  a.out[DRL_PPO_OUT_PG_CLIPFRAC] = static_cast<float>(r[1] / dm);
  a.out[DRL_PPO_OUT_PPO_KL] = static_cast<float>(r[2] / dm);
  a.out[DRL_PPO_OUT_PG_CLIPFRAC_LOWER] = static_cast<float>(r[3] / dm);
  a.out[DRL_PPO_OUT_ENTROPY_LOSS] = static_cast<float>(ent_loss);
  a.out[DRL_PPO_OUT_KL_LOSS] = static_cast<float>(kl_loss);
  a.out[DRL_PPO_OUT_LOSS] = static_cast<float>(total * a.lsf);
  a.out[DRL_PPO_OUT_MASK_COUNT] = static_cast<float>(cnt);
}

template <int MDT>
int launch_seq(const SeqArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(seq_row_kernel<MDT>, dim3(static_cast<unsigned>((a.B + 3) / 4)), dim3(256), 0, s, a);
  DRL_LAUNCH_CHECK();
  if (a.policy == DRL_POLICY_CLIP_COV || a.policy == DRL_POLICY_KL_COV) {
    hipLaunchKernelGGL(cov_select_kernel, dim3(1), dim3(256), 0, s, a, a.mask, MDT);
    DRL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(seq_token_kernel<MDT>, dim3(static_cast<unsigned>(a.B)), dim3(256), 0, s, a);
  DRL_LAUNCH_CHECK();
  hipLaunchKernelGGL(seq_final_kernel, dim3(1), dim3(256), 0, s, a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // namespace
}  // namespace drl

extern "C" {

size_t drl_ppo_loss_workspace_bytes(int64_t B, int64_t R) { return drl::ws_layout(B, R).total; }

int drl_ppo_loss_fwd_bwd(const float* old_log_prob, const float* log_prob, const float* advantages,
                         const void* response_mask, int32_t mask_dtype, const float* entropy,
                         const float* ref_log_prob, int64_t B, int64_t R, const drl_ppo_loss_params* p,
                         float* out_scalars, float* dlog_prob, float* dentropy, void* workspace,
                         size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(p != nullptr, "params is NULL");
  DRL_CHECK_ARG(B >= 1 && R >= 1, "bad shape B=%lld R=%lld", (long long)B, (long long)R);
  DRL_CHECK_ARG(old_log_prob && log_prob && advantages && response_mask && out_scalars, "NULL input");
  DRL_CHECK_ARG(p->loss_agg_mode >= 0 && p->loss_agg_mode <= 3, "bad loss_agg_mode %d", p->loss_agg_mode);
  DRL_CHECK_ARG(p->kl_type >= DRL_KL_NONE && p->kl_type <= DRL_KL_K3, "bad kl_type %d", p->kl_type);
  DRL_CHECK_ARG(p->kl_type == DRL_KL_NONE || ref_log_prob != nullptr, "kl_type set but ref_log_prob is NULL");
  DRL_CHECK_ARG(p->entropy_coeff == 0.f || entropy != nullptr, "entropy_coeff != 0 but entropy is NULL");
  DRL_CHECK_ARG(p->policy_loss != DRL_POLICY_VANILLA || p->clip_ratio_c > 1.f,
                "clip_ratio_c must be > 1.0 (dual-clip PPO), got %f", p->clip_ratio_c);
  DRL_CHECK_ARG(p->policy_loss >= DRL_POLICY_VANILLA && p->policy_loss <= DRL_POLICY_KL_COV, "bad policy_loss %d",
                p->policy_loss);
  DRL_CHECK_ARG(mask_dtype == DRL_I64 || mask_dtype == DRL_I32 || mask_dtype == DRL_U8 || mask_dtype == DRL_F32,
                "unsupported mask dtype %d", mask_dtype);
  const void* ptrs[] = {old_log_prob, log_prob, advantages, response_mask, entropy, ref_log_prob, dlog_prob, dentropy};
  for (const void* q : ptrs) DRL_CHECK_ARG(q == nullptr || aligned16(q), "tensor base not 16-byte aligned");
  const Layout L = ws_layout(B, R);
  if (workspace == nullptr || workspace_bytes < L.total)
    return fail(DRL_ERR_WORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, L.total);

  auto* ws = static_cast<char*>(workspace);
  if (p->policy_loss >= DRL_POLICY_GSPO) {
    SeqArgs q{};
    q.old_lp = old_log_prob; q.lp = log_prob; q.adv = advantages; q.mask = response_mask;
    q.ent = entropy; q.ref = p->kl_type == DRL_KL_NONE ? nullptr : ref_log_prob;
    q.dlp = dlog_prob; q.dent = dentropy; q.out = out_scalars;
    q.rowstat = reinterpret_cast<float*>(ws + L.seqrow);
    q.rowpart = reinterpret_cast<double*>(ws + L.seqpart);
    q.B = B; q.R = R;
    q.lo = static_cast<float>(1.0 - static_cast<double>(p->clip_ratio_low));
    q.hi = static_cast<float>(1.0 + static_cast<double>(p->clip_ratio_high));
    q.llo = p->clip_ratio_low; q.lhi = p->clip_ratio_high;
    q.ent_coef = p->entropy_coeff; q.kl_coef = p->kl_loss_coef; q.lsf = p->loss_scale_factor;
    q.mode = p->loss_agg_mode; q.kl = p->kl_type; q.policy = p->policy_loss;
    q.sel = reinterpret_cast<unsigned*>(ws + L.seqsel);
    q.cov_ratio = p->cov_ratio; q.cov_lb = p->clip_cov_lb; q.cov_ub = p->clip_cov_ub; q.ppo_kl_coef = p->ppo_kl_coef;
    q.cov_seed = static_cast<uint32_t>(p->cov_seed ^ (p->cov_seed >> 32));
    DRL_CHECK_ARG(p->policy_loss < DRL_POLICY_CLIP_COV || p->cov_ratio > 0.f, "clip_cov / kl_cov ratio must be > 0");
    DRL_CHECK_ARG(B * R < (int64_t(1) << 32), "clip_cov / kl_cov: more than 2^32 tokens");
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (mask_dtype) {
      case DRL_I64: return launch_seq<DRL_I64>(q, s);
      case DRL_I32: return launch_seq<DRL_I32>(q, s);
      case DRL_U8: return launch_seq<DRL_U8>(q, s);
      default: return launch_seq<DRL_F32>(q, s);
    }
  }
  Args a{};
  a.old_lp = old_log_prob; a.lp = log_prob; a.adv = advantages; a.mask = response_mask;
  a.ent = entropy; a.ref = p->kl_type == DRL_KL_NONE ? nullptr : ref_log_prob;
  a.rowcnt = reinterpret_cast<const float*>(ws + L.rowcnt);
  a.bits = nullptr;
  a.dlp = dlog_prob; a.dent = dentropy; a.out = out_scalars;
  a.hdr = reinterpret_cast<Header*>(ws);
  a.partials = reinterpret_cast<double*>(ws + L.partials);
  a.N = B * R; a.B = B; a.R = R;
  // python computes 1 - cliprange_low in double; torch.clamp then casts the bound to float32
  a.lo = static_cast<float>(1.0 - static_cast<double>(p->clip_ratio_low));
  a.hi = static_cast<float>(1.0 + static_cast<double>(p->clip_ratio_high));
  a.clip_c = p->clip_ratio_c; a.ent_coef = p->entropy_coeff; a.kl_coef = p->kl_loss_coef;
  a.lsf = p->loss_scale_factor; a.mode = p->loss_agg_mode; a.kl = p->kl_type;
  a.token_count = p->loss_agg_mode == DRL_AGG_TOKEN_MEAN ? p->token_count : nullptr;
  a.policy = p->policy_loss;

  hipStream_t s = static_cast<hipStream_t>(stream);  // the header is zero on entry (see Header)
  switch (mask_dtype) {
    case DRL_I64: return launch<DRL_I64>(a, L, ws, s);
    case DRL_I32: return launch<DRL_I32>(a, L, ws, s);
    case DRL_U8: return launch<DRL_U8>(a, L, ws, s);
    default: return launch<DRL_F32>(a, L, ws, s);
  }
}

int drl_kl_penalty(const float* log_prob, const float* ref_log_prob, int64_t n, int32_t kl_type, float* out,
                   void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(log_prob && ref_log_prob && out, "NULL input");
  DRL_CHECK_ARG(kl_type >= DRL_KL_K1 && kl_type <= DRL_KL_K3, "bad kl_type %d", kl_type);
  if (n <= 0) return DRL_OK;
  const int grid = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(cu_count()) * 8, (n + 255) / 256));
  hipLaunchKernelGGL(kl_penalty_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), log_prob,
                     ref_log_prob, n, kl_type, out);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_agg_loss_workspace_bytes(int64_t B, int64_t R) { return drl_ppo_loss_workspace_bytes(B, R); }

int drl_agg_loss(const float* loss_mat, const void* loss_mask, int32_t mdt, int64_t B, int64_t R, int32_t mode,
                 float* out, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(loss_mat && loss_mask && out, "NULL input");
  DRL_CHECK_ARG(B >= 1 && R >= 1, "bad shape");
  DRL_CHECK_ARG(mode >= 0 && mode <= 3, "bad loss_agg_mode %d", mode);
  const Layout L = ws_layout(B, R);
  const size_t off_part = L.partials, off_row = L.rowcnt;
  if (workspace == nullptr || workspace_bytes < L.total) return fail(DRL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* ws = static_cast<char*>(workspace);
  DRL_HIP(hipMemsetAsync(ws, 0, sizeof(Header), s));
  switch (mdt) {
    case DRL_I64: return launch_agg<DRL_I64>(loss_mat, loss_mask, B, R, mode, ws, off_part, off_row, out, s);
    case DRL_I32: return launch_agg<DRL_I32>(loss_mat, loss_mask, B, R, mode, ws, off_part, off_row, out, s);
    case DRL_U8: return launch_agg<DRL_U8>(loss_mat, loss_mask, B, R, mode, ws, off_part, off_row, out, s);
    case DRL_F32: return launch_agg<DRL_F32>(loss_mat, loss_mask, B, R, mode, ws, off_part, off_row, out, s);
    default: return fail(DRL_ERR_INVALID, "bad mask dtype %d", mdt);
  }
}

}  // extern "C"
