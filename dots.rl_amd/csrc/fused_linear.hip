// A21 — fused lm_head + log-prob + entropy on MFMA (gfx950 v_mfma_f32_32x32x16_bf16), replacing
// FusedLinearForPPO (verl/utils/experimental/torch_functional.py:20-216) and the Triton
// linear_cross_entropy (verl/utils/kernel/linear_cross_entropy.py:41-117, kernels.py:507-696 forward,
// kernels.py:1378-1586 backward) behind model.fused_kernel_options.impl_backend.
//
// Forward: logits z = (h W^T) / T are produced tile by tile in fp32 accumulators and consumed in
// registers: each lane keeps an online (max, sum exp, sum exp * z) per token over the vocabulary rows it
// sees, and the one lane holding z[label] writes it out. The (N, V) logits never reach HBM (bf16 logits
// of a 4096-row micro-batch would be 1.24 GB written and read back). A small merge kernel folds the
// per-chunk statistics: lse, entropy = lse - sum p z, logp = z[label] - lse.
// Backward (the reference's BackwardEnum._Total_Separate): the same GEMM core recomputes z and writes
// d_logits^T (V, N) bf16 = ((dlogp (onehot - p) - dent p (log p + H)) / T); d_hidden and d_W are then two
// library GEMMs (d_W accumulated in place into the fp32 gradient).
//
// Tile: 256 vocabulary rows x 256 tokens per workgroup step, K (= hidden size) in 64-wide steps staged
// global -> LDS by global_load_lds (two buffers, one barrier per step). Orientation (as the attention kernels):
// C = W h^T, so a lane's accumulator column is ONE token and its 16 registers are 16 vocabulary rows —
// the softmax statistics are lane-local, no cross-lane reduction per tile. 8 waves = 4 (vocab) x 2
// (tokens); a wave owns 64 vocab rows x 128 tokens = 2 x 4 MFMA blocks (128 accumulator registers).
// A workgroup walks a chunk of consecutive vocabulary tiles for one token tile (statistics stay in
// registers across the chunk); chunks x token tiles fill the chip.
// LDS image: [256 rows][64] bf16 per operand, 16-B unit u of row r stored at u ^ ((r >> 1) & 7): the 8
// lanes of a row write 8 distinct units and the 16 lanes of a fragment read (rows r..r+15, one unit)
// cover all 64 banks once.
#include <algorithm>

#include "common.h"

namespace drl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr int kBV = 256, kBT = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kTileU16 = 256 * kBK;            // one operand tile in LDS (32 KB)
constexpr int kLdsU16 = 2 * 2 * kTileU16;       // 2 buffers x (A, B) = 128 KB

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ uint16_t to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }
__device__ __forceinline__ int swz(int row, int unit) { return row * kBK + 8 * (unit ^ ((row >> 1) & 7)); }

struct FlArgs {
  const uint16_t* h;  // (N, ld_h) bf16 hidden rows
  int64_t ld_h;
  const uint16_t* w;  // (V, H) bf16 lm_head weight, row-major
  const int64_t* labels;
  int64_t N, H, V;
  float inv_t;     // 1 / temperature
  float l2e_t;     // log2(e) / temperature
  int tok_tiles, tiles_per_chunk, nchunks, vtiles;
  // forward
  float* part;     // (nchunks, 3, N): max (log2 units), sum exp2, sum exp2 * z
  float* zlab;     // (N) z[label]
  // backward
  const float* dlogp;
  const float* dent;  // nullptr: no entropy gradient
  const float* lse;
  const float* ent;
  uint16_t* dlt;      // (V, ld_dl) bf16 d_logits^T
  int64_t ld_dl;
  // token selection (decode): greedy argmax over the bf16 logits
  const int64_t* dev_step;
  unsigned long long* best;  // (N) packed (key, ~index) running max, zero between calls
};

constexpr int MODE_LOGPROB = 0, MODE_DLOGITS = 1, MODE_SELECT = 2;

// order-preserving (key, ~index) packing of csrc/vocab.hip: unsigned max == torch.argmax (first index on ties)
__device__ __forceinline__ uint64_t pack_key(float key, int64_t idx) {
  uint32_t b = __float_as_uint(key);
  b = isnan(key) ? 0xFFFFFFFFu : ((b & 0x80000000u) ? ~b : (b | 0x80000000u));
  return (static_cast<uint64_t>(b) << 32) | (0xFFFFFFFFu - static_cast<uint32_t>(idx));
}

// one K-step of both operands, global -> LDS directly (global_load_lds_dwordx4, no staging registers).
// One wave-instruction fills 8 consecutive rows (1 KB, lane-linear in LDS): lane l writes physical unit
// l & 7 of row r0 + (l >> 3), so it fetches the logical unit (l & 7) ^ ((row >> 1) & 7) — the swizzle is
// applied on the source address. Rows past V / N are clamped to the last row (finite values whose
// columns / rows the epilogue never uses); the host guarantees H % 64 == 0.
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
__device__ __forceinline__ void stage_glds(const FlArgs& a, uint16_t* la, uint16_t* lb, int64_t v0, int64_t t0,
                                           int k0, int w, int lane) {
  const int rsub = lane >> 3, pu = lane & 7;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = (w * 4 + i) * 8, row = r0 + rsub;
    const int u = pu ^ ((row >> 1) & 7);
    const int64_t v = min(v0 + row, a.V - 1), t = min(t0 + row, a.N - 1);
    __builtin_amdgcn_global_load_lds((glb_void*)(a.w + v * a.H + k0 + 8 * u), (lds_void*)(la + r0 * kBK), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((glb_void*)(a.h + t * a.ld_h + k0 + 8 * u), (lds_void*)(lb + r0 * kBK), 16, 0, 0);
  }
}

// MFMAs of one K-step: wave (wv, wt) accumulates C[vb][tb] (32 vocab rows x 32 tokens each)
__device__ __forceinline__ void step_mfma(const uint16_t* la, const uint16_t* lb, int wv, int wt, int lane,
                                          f32x16 (&acc)[2][4]) {
  const int r = lane & 31, hi = lane >> 5;
#pragma unroll
  for (int s = 0; s < kBK / 16; ++s) {
    const int unit = 2 * s + hi;
    bf16x8 af[2], bfr[4];
#pragma unroll
    for (int vb = 0; vb < 2; ++vb)
      af[vb] = as_bf16x8(*reinterpret_cast<const u16x8*>(la + swz(wv * 64 + vb * 32 + r, unit)));
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
      bfr[tb] = as_bf16x8(*reinterpret_cast<const u16x8*>(lb + swz(wt * 128 + tb * 32 + r, unit)));
#pragma unroll
    for (int vb = 0; vb < 2; ++vb)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
        acc[vb][tb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[vb], bfr[tb], acc[vb][tb], 0, 0, 0);
  }
}

// vocabulary row of accumulator register i in vocab block vb (lane half hi)
__device__ __forceinline__ int vrow(int vb, int i, int hi) { return vb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi; }

// workgroup -> (token tile, vocab chunk). Consecutive ids go to different XCDs; the remap gives each XCD a
// contiguous run of ids so the token tiles of a chunk (which share its W tiles) run on one XCD's L2.
__device__ __forceinline__ void wg_coords(const FlArgs& a, int& tt, int& chunk) {
  const int n = a.tok_tiles * a.nchunks, i = blockIdx.x;
  const int q = n / 8, rr = n % 8, xcd = i % 8;
  const int c = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + i / 8;  // bijective remap
  tt = c % a.tok_tiles;
  chunk = c / a.tok_tiles;
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void fused_linear_kernel(FlArgs a) {
  constexpr bool BWD = MODE == MODE_DLOGITS;
  __shared__ __attribute__((aligned(16))) uint16_t lds[kLdsU16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wv = w & 3, wt = w >> 2, hi = lane >> 5;
  int tt, chunk;
  wg_coords(a, tt, chunk);
  const int64_t t0 = static_cast<int64_t>(tt) * kBT;
  const int vt_beg = chunk * a.tiles_per_chunk;
  const int vt_end = min(a.vtiles, vt_beg + a.tiles_per_chunk);
  const int KS = static_cast<int>((a.H + kBK - 1) / kBK);
  const int nsteps = (vt_end - vt_beg) * KS;

  // per-token state of this lane: the 4 token blocks' columns
  int64_t lab[4];
  float m[4], s[4], sz[4];
  uint64_t sel[4] = {0, 0, 0, 0};
  float c_dlp[4], c_den[4], c_lse[4], c_ent[4];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb) {
    const int64_t t = t0 + wt * 128 + tb * 32 + (lane & 31);
    const bool tin = t < a.N;
    lab[tb] = (tin && MODE != MODE_SELECT) ? a.labels[t] : -1;
    m[tb] = -INFINITY;
    s[tb] = 0.f;
    sz[tb] = 0.f;
    if constexpr (BWD) {
      c_dlp[tb] = tin ? a.dlogp[t] : 0.f;
      c_den[tb] = (tin && a.dent) ? a.dent[t] : 0.f;
      c_lse[tb] = tin ? a.lse[t] : 0.f;
      c_ent[tb] = (tin && a.dent) ? a.ent[t] : 0.f;
    }
  }

  f32x16 acc[2][4];
#pragma unroll
  for (int vb = 0; vb < 2; ++vb)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) acc[vb][tb] = f32x16{};

  if (nsteps > 0) stage_glds(a, lds, lds + kTileU16, static_cast<int64_t>(vt_beg) * kBV, t0, 0, w, lane);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    if (step + 1 < nsteps) {  // next K-step into the other buffer (last read before the previous barrier)
      const int ns = step + 1, vt = vt_beg + ns / KS, ks = ns % KS, nb = buf ^ 1;
      stage_glds(a, lds + nb * 2 * kTileU16, lds + nb * 2 * kTileU16 + kTileU16, static_cast<int64_t>(vt) * kBV, t0,
                 ks * kBK, w, lane);
    }
    step_mfma(lds + buf * 2 * kTileU16, lds + buf * 2 * kTileU16 + kTileU16, wv, wt, lane, acc);
    if (step % KS == KS - 1) {
      // ---- epilogue of vocabulary tile vt: rows v0 + wv*64 + vrow(vb, i, hi)
      const int64_t vbase = static_cast<int64_t>(vt_beg + step / KS) * kBV + wv * 64;
      const bool vtail = vbase + 64 > a.V;
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) {
        const int64_t t = t0 + wt * 128 + tb * 32 + (lane & 31);
        if constexpr (MODE == MODE_SELECT) {
          // greedy key = the bf16 logit (the lm_head module output)
#pragma unroll
          for (int vb = 0; vb < 2; ++vb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int64_t v = vbase + vrow(vb, i, hi);
              const uint64_t pk = pack_key(bf16_to_f32(to_bf16_bits(acc[vb][tb][i])), v);
              if ((!vtail || v < a.V) && pk > sel[tb]) sel[tb] = pk;
            }
        } else if constexpr (!BWD) {
          float mx = -INFINITY;
#pragma unroll
          for (int vb = 0; vb < 2; ++vb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const bool ok = !vtail || vbase + vrow(vb, i, hi) < a.V;
              mx = ok ? fmaxf(mx, acc[vb][tb][i] * a.l2e_t) : mx;
            }
          const float mn = fmaxf(m[tb], mx);
          if (mn != -INFINITY) {
            const float alpha = __builtin_amdgcn_exp2f(m[tb] - mn);  // m = -inf -> 0
            float ss = 0.f, szz = 0.f;
#pragma unroll
            for (int vb = 0; vb < 2; ++vb)
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                const bool ok = !vtail || vbase + vrow(vb, i, hi) < a.V;
                const float e = ok ? __builtin_amdgcn_exp2f(fmaf(acc[vb][tb][i], a.l2e_t, -mn)) : 0.f;
                ss += e;
                szz = fmaf(e, acc[vb][tb][i] * a.inv_t, szz);
              }
            s[tb] = fmaf(s[tb], alpha, ss);
            sz[tb] = fmaf(sz[tb], alpha, szz);
            m[tb] = mn;
          }
          // the lane holding z[label] (exactly one in the grid) writes it
          const int64_t d = lab[tb] - vbase;
          if (d >= 0 && d < 64 && t < a.N) {
            const int vb = static_cast<int>(d >> 5), dd = static_cast<int>(d & 31);
            if (((dd >> 2) & 1) == hi) {
              const int ri = (dd & 3) + 4 * (dd >> 3);
              float zv = 0.f;
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                zv = (vb == 0 && i == ri) ? acc[0][tb][i] : zv;
                zv = (vb == 1 && i == ri) ? acc[1][tb][i] : zv;
              }
              a.zlab[t] = zv * a.inv_t;
            }
          }
        } else {
          if (t < a.N) {
            const float dlp = c_dlp[tb], den = c_den[tb], lse = c_lse[tb], hh = c_ent[tb];
#pragma unroll
            for (int vb = 0; vb < 2; ++vb)
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                const int64_t v = vbase + vrow(vb, i, hi);
                if (vtail && v >= a.V) continue;
                const float lp = fmaf(acc[vb][tb][i], a.inv_t, -lse);  // log p
                const float p = __expf(lp);
                float g = -p * fmaf(den, lp + hh, dlp);
                if (v == lab[tb]) g += dlp;
                a.dlt[v * a.ld_dl + t] = to_bf16_bits(g * a.inv_t);
              }
          }
        }
      }
#pragma unroll
      for (int vb = 0; vb < 2; ++vb)
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) acc[vb][tb] = f32x16{};
    }
    __syncthreads();
  }
  if constexpr (MODE == MODE_SELECT) {
    // max over the 8 (vocab wave, lane half) partials of each token, then one atomic per (token, chunk)
    unsigned long long* sb = reinterpret_cast<unsigned long long*>(lds);  // [256 tokens][8]
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) sb[(wt * 128 + tb * 32 + (lane & 31)) * 8 + wv * 2 + hi] = sel[tb];
    __syncthreads();
    if (tid < kBT && t0 + tid < a.N) {
      unsigned long long b = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) b = sb[tid * 8 + k] > b ? sb[tid * 8 + k] : b;
      __hip_atomic_fetch_max(a.best + t0 + tid, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if constexpr (!BWD) {
    // merge the 8 partial states of each token (4 vocab waves x 2 lane halves) in a fixed order
    float* st = reinterpret_cast<float*>(lds);  // [256 tokens][8 slots][3]
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) {
      const int tl = wt * 128 + tb * 32 + (lane & 31), slot = wv * 2 + hi;
      st[(tl * 8 + slot) * 3 + 0] = m[tb];
      st[(tl * 8 + slot) * 3 + 1] = s[tb];
      st[(tl * 8 + slot) * 3 + 2] = sz[tb];
    }
    __syncthreads();
    if (tid < kBT) {
      const int64_t t = t0 + tid;
      if (t < a.N) {
        float mm = -INFINITY;
#pragma unroll
        for (int k = 0; k < 8; ++k) mm = fmaxf(mm, st[(tid * 8 + k) * 3]);
        float ss = 0.f, szz = 0.f;
        if (mm != -INFINITY) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float sc = __builtin_amdgcn_exp2f(st[(tid * 8 + k) * 3] - mm);
            ss = fmaf(st[(tid * 8 + k) * 3 + 1], sc, ss);
            szz = fmaf(st[(tid * 8 + k) * 3 + 2], sc, szz);
          }
        }
        a.part[(static_cast<int64_t>(chunk) * 3 + 0) * a.N + t] = mm;
        a.part[(static_cast<int64_t>(chunk) * 3 + 1) * a.N + t] = ss;
        a.part[(static_cast<int64_t>(chunk) * 3 + 2) * a.N + t] = szz;
      }
    }
  }
}

// fold the chunks of each token in chunk order: lse, entropy, log p(label)
__global__ __launch_bounds__(256) void fused_linear_merge_kernel(const float* part, const float* zlab, int64_t N,
                                                                 int nchunks, float* logp, float* ent, float* lse) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= N) return;
  float mm = -INFINITY;
  for (int c = 0; c < nchunks; ++c) mm = fmaxf(mm, part[(static_cast<int64_t>(c) * 3) * N + t]);
  float ss = 0.f, szz = 0.f;
  for (int c = 0; c < nchunks; ++c) {
    const float mc = part[(static_cast<int64_t>(c) * 3) * N + t];
    if (mc == -INFINITY) continue;
    const float sc = __builtin_amdgcn_exp2f(mc - mm);
    ss = fmaf(part[(static_cast<int64_t>(c) * 3 + 1) * N + t], sc, ss);
    szz = fmaf(part[(static_cast<int64_t>(c) * 3 + 2) * N + t], sc, szz);
  }
  const float l = (mm + __log2f(ss)) * 0.69314718055994531f;  // natural-log LSE
  if (logp) logp[t] = zlab[t] - l;
  if (ent) ent[t] = l - szz / ss;
  if (lse) lse[t] = l;
}

// one thread per token: decode the winning index, reset best[t], finished-row / EOS bookkeeping
// (select_finish_kernel of csrc/vocab.hip)
__global__ __launch_bounds__(256) void fused_select_finish_kernel(unsigned long long* best, int64_t N,
                                                                  const int64_t* dev_step, int64_t pad,
                                                                  const int64_t* eos, int n_eos, int32_t* unfinished,
                                                                  int64_t* out, int64_t ld_out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (r >= N) return;
  const unsigned long long b = best[r];
  best[r] = 0;
  const int64_t choice = static_cast<int64_t>(0xFFFFFFFFu - static_cast<uint32_t>(b));
  const bool alive = unfinished ? unfinished[r] != 0 : true;
  const int64_t tok = alive ? choice : pad;
  out[r * ld_out + (dev_step ? *dev_step : 0)] = tok;
  if (unfinished && alive) {
    for (int k = 0; k < n_eos; ++k)
      if (tok == eos[k]) { unfinished[r] = 0; break; }
  }
}

struct Plan {
  int tok_tiles, vtiles, tiles_per_chunk, nchunks;
};

Plan make_plan(int64_t N, int64_t V) {
  Plan p;
  p.tok_tiles = static_cast<int>((N + kBT - 1) / kBT);
  p.vtiles = static_cast<int>((V + kBV - 1) / kBV);
  // about 4 workgroups per CU over the launch (one resident per CU: 128 KB of LDS)
  const int64_t total = static_cast<int64_t>(p.tok_tiles) * p.vtiles;
  const int64_t target = 4 * static_cast<int64_t>(cu_count());
  p.tiles_per_chunk = static_cast<int>(std::max<int64_t>(1, (total + target - 1) / target));
  p.nchunks = (p.vtiles + p.tiles_per_chunk - 1) / p.tiles_per_chunk;
  return p;
}

}  // namespace
}  // namespace drl

extern "C" {

size_t drl_linear_logprob_workspace_bytes(int64_t N, int64_t H, int64_t V) {
  if (N < 1 || H < 1 || V < 1) return 0;
  const drl::Plan p = drl::make_plan(N, V);
  return (static_cast<size_t>(p.nchunks) * 3 + 1) * static_cast<size_t>(N) * sizeof(float);
}

int drl_linear_logprob_fwd(const void* hidden, int64_t ld_h, const void* weight, const int64_t* labels, int32_t dt,
                           int64_t N, int64_t H, int64_t V, float temperature, float* logp, float* entropy,
                           float* lse, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(hidden && weight && labels && workspace, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "the fused lm_head runs on bf16 operands");
  DRL_CHECK_ARG(N >= 1 && V >= 1 && H >= 64 && H % 64 == 0 && ld_h >= H && ld_h % 8 == 0, "bad shape (H % 64 == 0)");
  DRL_CHECK_ARG(temperature > 0.f, "temperature must be positive");
  DRL_CHECK_ARG(aligned16(hidden) && aligned16(weight), "hidden / weight must be 16-byte aligned");
  DRL_CHECK_ARG(N * 3 < (int64_t(1) << 40) && V < (int64_t(1) << 31), "size out of range");
  const size_t need = drl_linear_logprob_workspace_bytes(N, H, V);
  if (workspace_bytes < need) return fail(DRL_ERR_WORKSPACE, "fused lm_head workspace: need %zu bytes", need);
  const Plan p = make_plan(N, V);
  FlArgs a{};
  a.h = static_cast<const uint16_t*>(hidden);
  a.ld_h = ld_h;
  a.w = static_cast<const uint16_t*>(weight);
  a.labels = labels;
  a.N = N;
  a.H = H;
  a.V = V;
  a.inv_t = 1.f / temperature;
  a.l2e_t = 1.4426950408889634f / temperature;
  a.tok_tiles = p.tok_tiles;
  a.tiles_per_chunk = p.tiles_per_chunk;
  a.nchunks = p.nchunks;
  a.vtiles = p.vtiles;
  a.part = static_cast<float*>(workspace);
  a.zlab = a.part + static_cast<size_t>(p.nchunks) * 3 * N;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fused_linear_kernel<MODE_LOGPROB>, dim3(p.tok_tiles * p.nchunks), dim3(kThreads),
                     0, s, a);
  hipLaunchKernelGGL(fused_linear_merge_kernel, dim3(static_cast<unsigned>((N + 255) / 256)), dim3(256), 0, s, a.part,
                     a.zlab, N, p.nchunks, logp, entropy, lse);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_linear_logprob_dlogits(const void* hidden, int64_t ld_h, const void* weight, const int64_t* labels, int32_t dt,
                               int64_t N, int64_t H, int64_t V, float temperature, const float* dlogp,
                               const float* dentropy, const float* lse, const float* entropy, void* dlogits_t,
                               int64_t ld_dl, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(hidden && weight && labels && dlogp && lse && dlogits_t, "NULL input");
  DRL_CHECK_ARG(!dentropy || entropy, "the entropy gradient needs the forward entropy");
  DRL_CHECK_ARG(dt == DRL_BF16, "the fused lm_head runs on bf16 operands");
  DRL_CHECK_ARG(N >= 1 && V >= 1 && H >= 64 && H % 64 == 0 && ld_h >= H && ld_h % 8 == 0 && ld_dl >= N, "bad shape (H % 64 == 0)");
  DRL_CHECK_ARG(temperature > 0.f, "temperature must be positive");
  DRL_CHECK_ARG(aligned16(hidden) && aligned16(weight), "hidden / weight must be 16-byte aligned");
  const Plan p = make_plan(N, V);
  FlArgs a{};
  a.h = static_cast<const uint16_t*>(hidden);
  a.ld_h = ld_h;
  a.w = static_cast<const uint16_t*>(weight);
  a.labels = labels;
  a.N = N;
  a.H = H;
  a.V = V;
  a.inv_t = 1.f / temperature;
  a.l2e_t = 1.4426950408889634f / temperature;
  a.tok_tiles = p.tok_tiles;
  a.tiles_per_chunk = p.tiles_per_chunk;
  a.nchunks = p.nchunks;
  a.vtiles = p.vtiles;
  a.dlogp = dlogp;
  a.dent = dentropy;
  a.lse = lse;
  a.ent = entropy;
  a.dlt = static_cast<uint16_t*>(dlogits_t);
  a.ld_dl = ld_dl;
  hipLaunchKernelGGL(fused_linear_kernel<MODE_DLOGITS>, dim3(p.tok_tiles * p.nchunks), dim3(kThreads),
                     0, static_cast<hipStream_t>(stream), a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_linear_select_tokens_workspace_bytes(int64_t N) { return N > 0 ? static_cast<size_t>(N) * 8 : 0; }

int drl_linear_select_tokens(const void* hidden, int64_t ld_h, const void* weight, int32_t dt, int64_t N, int64_t H,
                             int64_t V, const drl_sampling_params* p, int32_t* unfinished, int64_t* out_tokens,
                             int64_t ld_out, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(hidden && weight && p && out_tokens, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "the fused lm_head runs on bf16 operands");
  DRL_CHECK_ARG(N >= 1 && V >= 1 && V < (int64_t(1) << 32) && H >= 64 && H % 64 == 0 && ld_h >= H && ld_h % 8 == 0,
                "bad shape (H % 64 == 0)");
  DRL_CHECK_ARG(aligned16(hidden) && aligned16(weight), "hidden / weight must be 16-byte aligned");
  DRL_CHECK_ARG(p->n_eos == 0 || p->eos_ids != nullptr, "n_eos > 0 but eos_ids is NULL");
  if (p->do_sample && p->temperature > 0.f)
    return fail(DRL_ERR_UNSUPPORTED, "sampling draws slice masses then races inside one slice of the logits row: "
                                     "use drl_select_tokens on the lm_head logits");
  if (!workspace || workspace_bytes < drl_linear_select_tokens_workspace_bytes(N) ||
      (reinterpret_cast<uintptr_t>(workspace) & 7u))
    return fail(DRL_ERR_WORKSPACE, "select workspace: need %zu 8-byte aligned bytes, zeroed",
                drl_linear_select_tokens_workspace_bytes(N));
  const Plan pl = make_plan(N, V);
  FlArgs a{};
  a.h = static_cast<const uint16_t*>(hidden);
  a.ld_h = ld_h;
  a.w = static_cast<const uint16_t*>(weight);
  a.N = N;
  a.H = H;
  a.V = V;
  a.inv_t = 1.f;
  a.l2e_t = 1.4426950408889634f;
  a.tok_tiles = pl.tok_tiles;
  a.tiles_per_chunk = pl.tiles_per_chunk;
  a.nchunks = pl.nchunks;
  a.vtiles = pl.vtiles;
  a.dev_step = p->dev_step;
  a.best = static_cast<unsigned long long*>(workspace);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fused_linear_kernel<MODE_SELECT>, dim3(pl.tok_tiles * pl.nchunks), dim3(kThreads), 0, s, a);
  hipLaunchKernelGGL(fused_select_finish_kernel, dim3(static_cast<unsigned>((N + 255) / 256)), dim3(256), 0, s, a.best,
                     N, p->dev_step, p->pad_token_id, p->eos_ids, p->n_eos, unfinished, out_tokens, ld_out);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
