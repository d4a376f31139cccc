// Decode-step projections on fragment-packed operands (the rollout's per-token GEMMs at M = one token
// per sequence, 1..128 rows per rank): replaces the nn.Linear calls of Qwen2Attention / Qwen2MLP that HF
// generate runs once per response token (hf_rollout.py:112-124 -> transformers modeling_qwen2).
//
// Why a layout: at M <= 128 a projection is a weight stream (qkv 2 MB ... gate_up 17 MB per layer) plus an
// activation panel re-read from L2 by every workgroup. Loading MFMA fragments straight from row-major
// operands touches 32 rows x 32 B per wave-instruction and ran at ~1-2.5 TB/s (tools/wsgemm_probe.hip).
// Here both operands are stored in v_mfma_f32_32x32x16_bf16 fragment order — the 64 lanes' 16-B pieces
// of one (32-row block, 16-deep k step) are one contiguous 1 KB — so every load is a fully coalesced 1-KB
// wave read into registers:
//   weights: packed once per rollout from the bf16 compute copy (drl_decode_pack_weight);
//   activations: written packed by their producers (the decode RMSNorm, the decode attention, the SwiGLU
//   epilogue below), element (m, k) at ((k/16 * MBT + m/32) * 64 + ((k/8)&1) * 32 + m%32) * 8 + k%8 with
//   MBT the (padded) number of 32-token blocks (1..16: up to 512 rows).
// Workgroup = 4 waves on one 32-row weight block, one group of MB token blocks and one K slice; every wave
// issues ALL loads of its KSW k-steps before its first MFMA (one memory round trip), the four partial
// tiles meet in LDS in a fixed order. Outputs: fp32 partial sums per K slice (summed, in slice order, by
// the consumer kernel that runs next anyway: decode RoPE, decode RMSNorm), or the SwiGLU activation
// bf16(bf16(silu(g)) * u) written packed for the down projection (gate / up rows interleaved per block by
// the weight packing). Deterministic: fixed summation order everywhere.
#include "common.h"

namespace drl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ uint16_t to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }
__device__ __forceinline__ float bf16r(float f) { return bf16_to_f32(to_bf16_bits(f)); }

// packed activation offset of element (m, k)
__device__ __forceinline__ int64_t pk_off(int64_t m, int64_t k, int64_t MBT) {
  return (((k >> 4) * MBT + (m >> 5)) * 64 + ((k >> 3) & 1) * 32 + (m & 31)) * 8 + (k & 7);
}

// packed fp32 residual (fused-norm step): the fragment of (32-row block, 16-deep k step) as two 1-KB halves, half j
// holding k % 8 in [4j, 4j + 4) of every lane: element (m, k) at ((f * 2 + (k >> 2 & 1)) * 256 + lane * 4 + k % 4,
// f = k/16 * MBT + m/32, lane = ((k/8) & 1) * 32 + m % 32 — each 16-B load of a fragment half is one coalesced 1-KB wave
// read (a lane's 8 consecutive floats side by side would make every wave instruction span 2 KB)
__host__ __device__ __forceinline__ int64_t pkf_off(int64_t m, int64_t k, int64_t MBT) {
  return ((((k >> 4) * MBT + (m >> 5)) * 2 + ((k >> 2) & 1)) * 64 + ((k >> 3) & 1) * 32 + (m & 31)) * 4 + (k & 3);
}

// ------------------------------------------------------------------------------------------- packing
// dst fragment (t, s, lane l): W row rowmap(t, l & 31), k = 16 s + 8 (l >> 5) .. + 7. SwiGLU packing
// (half = I > 0): block t holds gate rows 16t..16t+15 then up rows I+16t..I+16t+15.
// RoPE packing (rope_half = D/2 > 0): block t holds rows head*D + 16q + (0..15) and the rotation partners
// head*D + D/2 + 16q + (0..15), q = t % (D/32), head = t / (D/32), so both halves of a rotated pair meet in one
// workgroup's epilogue.
__global__ __launch_bounds__(256) void pack_weight_kernel(const uint16_t* src, int64_t ld, int64_t N, int64_t K,
                                                          int64_t half, int64_t tiles, uint16_t* dst,
                                                          int64_t rope_half = 0) {
  const int64_t nks = K / 16;
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= tiles * nks * 64) return;
  const int l = static_cast<int>(idx & 63), r = l & 31, h = l >> 5;
  const int64_t s = (idx >> 6) % nks, t = (idx >> 6) / nks;
  int64_t row;
  bool ok;
  if (half > 0) {
    const int64_t c = 16 * t + (r & 15);
    ok = c < half;
    row = r < 16 ? c : half + c;
  } else if (rope_half > 0) {
    const int64_t per = rope_half / 16, head = t / per, q = t % per;
    row = head * 2 * rope_half + 16 * q + (r & 15) + (r < 16 ? 0 : rope_half);
    ok = row < N;
  } else {
    row = 32 * t + r;
    ok = row < N;
  }
  u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  if (ok) v = *reinterpret_cast<const u16x8*>(src + row * ld + 16 * s + 8 * h);
  *reinterpret_cast<u16x8*>(dst + idx * 8) = v;
}

// ------------------------------------------------------------------------------------------- GEMM
struct DgArgs {
  const uint16_t* x;  // packed activations, MBT token blocks
  const uint16_t* w;  // packed weights (tiles, nks)
  int M, N, K, MBT, nks, tiles, half;
  float* part;        // EPI_PARTIAL: (ksplit, M, N) fp32
  uint16_t* out;      // EPI_SWIGLU: packed (MBT blocks, K' = half)
  // EPI_ROPE (qkv_proj of one decode token; weights packed in rotation pairs, whole K per workgroup)
  const uint16_t* bias;
  const int64_t* pos;
  const float* cos_t;
  const float* sin_t;
  uint16_t* q;        // (M, Hkv, G, D)
  uint16_t* kc;       // (M, Hkv, Tk, D)
  uint16_t* vt;       // (M, Hkv, D, ld_vt)
  const int64_t* koff_dev;
  int64_t maxpos, Tk, ld_vt;
  int Hq, Hkv, D;
  // fused-norm decode (round 6): the fp32 residual stream kept fragment-packed (element (m, k) at pk_off(m, k, MBT),
  // fp32), updated in place by the K-split producers (EPI_RESID) and normalised on the fly by the consumers
  float* xr;            // packed fp32 residual stream (MBT blocks, H columns)
  const float* nw;      // NORM consumers: the RMSNorm weight (K)
  float eps;
  unsigned* cnt;        // EPI_RESID over K slices: arrival counters (tiles x mgroups), zero between launches
  int ksplit;
};

constexpr int EPI_PARTIAL = 0, EPI_SWIGLU = 1, EPI_ROPE = 2, EPI_RESID = 3;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// the NW waves' partial tiles (red[wave][token block][register][lane]) summed in wave order: ((r0 + r1) + r2) + ...
template <int NW, int MB>
__device__ __forceinline__ float red_sum(const float (*red)[MB][16][64], int blk, int q, int ln) {
  float v = red[0][blk][q][ln];
#pragma unroll
  for (int w = 1; w < NW; ++w) v += red[w][blk][q][ln];
  return v;
}

// Epilogues of the one-round-trip kernels, from the partial tiles of NW waves in LDS (tile = the 32-row weight block,
// ks = the K slice, mb0 = the first token block). C row i (weight row of the block) <-> register (i & 3) + 4 (i >> 3),
// lane half (i >> 2) & 1; column = token.
// the RoPE epilogue's per-thread operands, loaded with the kernel's first loads instead of behind the reduction: the
// key offset, the two bias values of the thread's column pair (the column is the same in every iteration: 256 threads,
// 16 columns) and, per iteration, the cos / sin of its token's position — issued as soon as the positions land, so
// their round trip runs under the MFMAs and the reduction (inline, the epilogue's dependent pos -> cos / sin loads were
// two memory round trips per iteration after the reduction)
template <int MB>
struct RopePre {
  int64_t koff;
  float b1, b2;
  float cs[2 * MB], sn[2 * MB];
};

template <int NW, int MB, int EPI>
__device__ __forceinline__ void red_epilogue(const DgArgs& a, const float (*red)[MB][16][64], int tile, int ks, int mb0,
                                             int tid, const float4* xres = nullptr,
                                             const RopePre<MB>* pre = nullptr) {
  constexpr int NT = 64 * NW;
  if constexpr (EPI == EPI_PARTIAL) {
    for (int e = tid; e < 1024 * MB; e += NT) {
      const int tl = e >> 5, i = e & 31, blk = tl >> 5, ml = tl & 31;
      const int m = (mb0 + blk) * 32 + ml, n = tile * 32 + i;
      if (m >= a.M || n >= a.N) continue;
      const int q = (i & 3) + 4 * (i >> 3), ln = ml + 32 * ((i >> 2) & 1);
      a.part[(static_cast<int64_t>(ks) * a.M + m) * a.N + n] = red_sum<NW, MB>(red, blk, q, ln);
    }
  } else if constexpr (EPI == EPI_ROPE) {
    // rows 0..15: d = 16 qq + c of head hd, rows 16..31 its partners d + D/2. qkv = bf16(acc + bias), then
    // rope_qkv_fwd_kernel's rotation (q, k heads) and the cache writes at the device key offset koff
    const int half = a.D / 2, per = half / 16, hd = tile / per, qq = tile % per;
    const int64_t koff = pre ? pre->koff : *a.koff_dev;
#pragma unroll
    for (int it = 0; it < 512 * MB / NT; ++it) {
      const int e = tid + NT * it;
      const int tl = e >> 4, c = e & 15, blk = tl >> 5, ml = tl & 31;
      const int m = (mb0 + blk) * 32 + ml;
      if (m >= a.M) continue;
      const int i1 = c, i2 = c + 16;
      const int q1 = (i1 & 3) + 4 * (i1 >> 3), l1 = ml + 32 * ((i1 >> 2) & 1);
      const int q2 = (i2 & 3) + 4 * (i2 >> 3), l2 = ml + 32 * ((i2 >> 2) & 1);
      const int d1 = 16 * qq + c, d2 = d1 + half;
      const int n1 = hd * a.D + d1, n2 = n1 + half;
      const float x1 = bf16r(red_sum<NW, MB>(red, blk, q1, l1) + (pre ? pre->b1 : bf16_to_f32(a.bias[n1])));
      const float x2 = bf16r(red_sum<NW, MB>(red, blk, q2, l2) + (pre ? pre->b2 : bf16_to_f32(a.bias[n2])));
      if (hd < a.Hq + a.Hkv) {
        float cs, sn;
        if (pre) {
          cs = pre->cs[it];
          sn = pre->sn[it];
        } else {
          int64_t p = a.pos[m];
          p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
          cs = a.cos_t[p * half + d1];
          sn = a.sin_t[p * half + d1];
        }
        const float o1 = fmaf(x1, cs, -(x2 * sn)), o2 = fmaf(x2, cs, x1 * sn);
        uint16_t* dst;
        if (hd < a.Hq) {
          const int G = a.Hq / a.Hkv;
          dst = a.q + ((static_cast<int64_t>(m) * a.Hkv + hd / G) * G + hd % G) * a.D;
        } else {
          dst = a.kc + ((static_cast<int64_t>(m) * a.Hkv + (hd - a.Hq)) * a.Tk + koff) * a.D;
        }
        dst[d1] = to_bf16_bits(o1);
        dst[d2] = to_bf16_bits(o2);
      } else {
        uint16_t* dst = a.vt + (static_cast<int64_t>(m) * a.Hkv + (hd - a.Hq - a.Hkv)) * vt_panel(a.ld_vt, a.D, a.Tk);
        dst[vt_index(d1, koff, a.ld_vt, a.D)] = to_bf16_bits(x1);
        dst[vt_index(d2, koff, a.ld_vt, a.D)] = to_bf16_bits(x2);
      }
    }
  } else if constexpr (EPI == EPI_SWIGLU) {
    // SwiGLU: rows 0..15 gate, 16..31 up of output columns 16 * tile + c; thread -> (token, 8 columns)
    for (int e = tid; e < 64 * MB; e += NT) {
      const int tl = e >> 1, hc = e & 1, blk = tl >> 5, ml = tl & 31;
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * hc + j, ig = c, iu = c + 16;
        const int qg = (ig & 3) + 4 * (ig >> 3), lg = ml + 32 * ((ig >> 2) & 1);
        const int qu = (iu & 3) + 4 * (iu >> 3), lu = ml + 32 * ((iu >> 2) & 1);
        const float g = bf16r(red_sum<NW, MB>(red, blk, qg, lg));
        const float u = bf16r(red_sum<NW, MB>(red, blk, qu, lu));
        o[j] = to_bf16_bits(bf16r(silu_fast(g)) * u);
      }
      // packed for the next GEMM (K' = half): k step = tile, 8-column half hc, token (mb0 + blk, ml)
      *reinterpret_cast<u16x8*>(a.out + ((static_cast<int64_t>(tile) * a.MBT + mb0 + blk) * 64 + hc * 32 + ml) * 8) = o;
    }
  } else {
    // EPI_RESID (o_proj / down_proj of the fused-norm decode): the residual add of the decoder layer,
    // x = x + bf16(sum over K slices) (add_rmsnorm_fwd's order: d = ((0 + p_0) + p_1) + ..., then one rounding), on
    // the packed fp32 residual stream in place. Thread -> (token, 4 consecutive output columns: rows 4c .. 4c + 3 of the
    // block = registers 4 (c >> 1) .. + 3 of lane half c & 1). Over K slices every slice publishes its partial tile
    // write-through (sc1 16-B stores, MI355X_MICROARCH.md § visibility, first row of the sc1 table), one lane's
    // agent-scope add counts the arrivals, and the LAST slice to arrive — told by the value its add returned, no
    // waiting, no grid barrier — sums the slices in slice order (sc1 loads) and updates the residual; it also resets
    // the counter for the next launch.
    static_assert(NW == 4 && MB <= 2, "the one-round-trip kernel's 256 threads: MB items per thread");
    __shared__ int s_last;
    const __amdgpu_buffer_rsrc_t rp =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.part, (short)0, a.ksplit * a.M * a.N * 4, 0x00020000);
    float4 v[MB];
    int mm[MB], nn[MB];
#pragma unroll
    for (int it = 0; it < MB; ++it) {
      // token fastest: 32 consecutive threads write one 512-B run of the packed residual, read consecutive LDS words
      const int e = tid + 256 * it, ml = e & 31, c = (e >> 5) & 7, blk = it;
      mm[it] = (mb0 + blk) * 32 + ml;
      nn[it] = tile * 32 + 4 * c;
      const int ln = ml + 32 * (c & 1), q0 = 4 * (c >> 1);
      v[it] = make_float4(red_sum<NW, MB>(red, blk, q0, ln), red_sum<NW, MB>(red, blk, q0 + 1, ln),
                          red_sum<NW, MB>(red, blk, q0 + 2, ln), red_sum<NW, MB>(red, blk, q0 + 3, ln));
      if (a.ksplit > 1 && mm[it] < a.M && nn[it] < a.N)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[it]), rp,
                                               static_cast<uint32_t>(((ks * a.M + mm[it]) * a.N + nn[it]) * 4), 0,
                                               16 /* sc1 */);
    }
    if (a.ksplit > 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
      __syncthreads();
      if (tid == 0) {
        typedef __attribute__((address_space(1))) unsigned gcnt;
        gcnt* c = (gcnt*)(a.cnt + static_cast<int64_t>(tile) * gridDim.z + blockIdx.z);
        const unsigned prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == static_cast<unsigned>(a.ksplit - 1);
        if (s_last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (!s_last) return;
    }
#pragma unroll
    for (int it = 0; it < MB; ++it) {
      const int m = mm[it], n = nn[it];
      if (m >= a.M || n >= a.N) continue;
      float4 d = v[it];
      if (a.ksplit > 1) {
        d = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = 0; k < a.ksplit; ++k) {
          const float4 p = k == ks ? v[it]
                                   : __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                         rp, static_cast<uint32_t>(((k * a.M + m) * a.N + n) * 4), 0, 16 /* sc1 */));
          d.x += p.x; d.y += p.y; d.z += p.z; d.w += p.w;
        }
      }
      float4 x = xres[it];  // loaded at the kernel's start (nobody else writes this tile's residual)
      x.x += bf16r(d.x); x.y += bf16r(d.y); x.z += bf16r(d.z); x.w += bf16r(d.w);
      *reinterpret_cast<float4*>(a.xr + pkf_off(m, n, a.MBT)) = x;
    }
  }
}

template <int MB, int KSW, int EPI>
__global__ __launch_bounds__(256) void decode_gemm_kernel(DgArgs a) {
  __shared__ float red[4][MB][16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = blockIdx.x, ks = blockIdx.y, mb0 = blockIdx.z * MB;
  const int s0 = (ks * 4 + wave) * KSW;
  u16x8 wv[KSW], xv[KSW][MB];
  const uint16_t* wp = a.w + (static_cast<int64_t>(tile) * a.nks + s0) * 512 + lane * 8;
#pragma unroll
  for (int s = 0; s < KSW; ++s) wv[s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp + s * 512));
#pragma unroll
  for (int s = 0; s < KSW; ++s)
#pragma unroll
    for (int i = 0; i < MB; ++i)
      xv[s][i] = *reinterpret_cast<const u16x8*>(a.x + ((static_cast<int64_t>(s0 + s) * a.MBT + mb0 + i) * 64 + lane) * 8);
  float4 xres[MB];
  if constexpr (EPI == EPI_RESID) {  // the residual this thread may update, with the first loads (no later round trip)
#pragma unroll
    for (int it = 0; it < MB; ++it) {
      const int e = tid + 256 * it, m = (mb0 + it) * 32 + (e & 31), n = tile * 32 + 4 * ((e >> 5) & 7);
      xres[it] = m < a.M && n < a.N ? *reinterpret_cast<const float4*>(a.xr + pkf_off(m, n, a.MBT))
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  RopePre<MB> pre;
  int64_t posv[2 * MB];
  if constexpr (EPI == EPI_ROPE) {  // the epilogue's operands with the first loads (RopePre)
    const int per = a.D / 32, c = tid & 15, d1 = 16 * (tile % per) + c, n1 = (tile / per) * a.D + d1;
    pre.koff = *a.koff_dev;
    pre.b1 = bf16_to_f32(a.bias[n1]);
    pre.b2 = bf16_to_f32(a.bias[n1 + a.D / 2]);
#pragma unroll
    for (int it = 0; it < 2 * MB; ++it) {
      const int tl = (tid + 256 * it) >> 4, m = (mb0 + (tl >> 5)) * 32 + (tl & 31);
      posv[it] = a.pos[m < a.M ? m : 0];
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // every load of the wave is in flight before the first MFMA
  if constexpr (EPI == EPI_ROPE) {
    // cos / sin as soon as the positions land (after the operand loads: the MFMAs below wait for those anyway)
    const int half = a.D / 2, per = half / 16, hd = tile / per, d1 = 16 * (tile % per) + (tid & 15);
    if (hd < a.Hq + a.Hkv) {
#pragma unroll
      for (int it = 0; it < 2 * MB; ++it) {
        int64_t p = posv[it];
        p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
        pre.cs[it] = a.cos_t[p * half + d1];
        pre.sn[it] = a.sin_t[p * half + d1];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  f32x16 acc[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) acc[i] = f32x16{};
#pragma unroll
  for (int s = 0; s < KSW; ++s)
#pragma unroll
    for (int i = 0; i < MB; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wv[s]), as_bf16x8(xv[s][i]), acc[i], 0, 0, 0);
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][i][q][lane] = acc[i][q];
  __syncthreads();
  red_epilogue<4, MB, EPI>(a, red, tile, ks, mb0, tid, xres, EPI == EPI_ROPE ? &pre : nullptr);
}

// The decode RMSNorm folded into its consumer GEMM's prologue (round 6; replaces the dec_rmsnorm launch before qkv +
// RoPE and before gate_up + SwiGLU): no norm launch, no grid barrier, nothing published between workgroups. Each
// workgroup reads the packed fp32 residual x of its token blocks over the whole K (which it needs as its operand
// anyway), every wave its K slice of NW: the wave's partial sums of squares per row meet in LDS (wave order, fixed:
// deterministic), rstd = rsqrt(mean + eps) per row, and each fragment is normalised as it is packed for the MFMA:
// y = bf16(w * (x * rstd)) — add_rmsnorm_fwd / HF Qwen2RMSNorm's rounding (fp32 statistics, weight times the fp32
// normalised value, one bf16 rounding for the autocast GEMM input). The norm weight is staged in LDS (its loads issued
// first, so their wait holds no fragment load). The fragment loads are issued before any arithmetic (one memory round
// trip); whole K per workgroup, so the RoPE / SwiGLU epilogues apply.
template <int NW, int MB, int KSW, int EPI>
__global__ __launch_bounds__(64 * NW) void decode_norm_gemm_kernel(DgArgs a) {
  static_assert(EPI == EPI_ROPE || EPI == EPI_SWIGLU, "whole-K epilogues");
  constexpr int NT = 64 * NW, WPT = 1024 / NT;  // norm-weight float4s per thread: K <= 4096
  static_assert(NW * MB >= 4, "the norm weight (<= 4096 floats) is staged in the reduction buffer");
  __shared__ __attribute__((aligned(16))) float red[NW][MB][16][64];
  __shared__ float s_ss[NW][MB][32];
  float* s_w = &red[0][0][0][0];  // the norm weight lives in the reduction buffer until the MFMAs are done
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ml = lane & 31, hh = lane >> 5;
  const int tile = blockIdx.x, mb0 = blockIdx.z * MB;
  const int s0 = wave * KSW;
  float4 wn[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int k = 4 * (tid + j * NT);
    if (k < a.K) wn[j] = *reinterpret_cast<const float4*>(a.nw + k);
  }
  u16x8 wv[KSW];
  float4 xv[KSW][MB][2];
  const uint16_t* wp = a.w + (static_cast<int64_t>(tile) * a.nks + s0) * 512 + lane * 8;
#pragma unroll
  for (int s = 0; s < KSW; ++s) wv[s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp + s * 512));
#pragma unroll
  for (int s = 0; s < KSW; ++s)
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const float* xp = a.xr + (static_cast<int64_t>(s0 + s) * a.MBT + mb0 + i) * 512 + lane * 4;  // pkf_off
      xv[s][i][0] = *reinterpret_cast<const float4*>(xp);
      xv[s][i][1] = *reinterpret_cast<const float4*>(xp + 256);
    }
  __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first use
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int k = 4 * (tid + j * NT);
    if (k < a.K) *reinterpret_cast<float4*>(s_w + k) = wn[j];
  }
  // per-row sum of squares: lane (row ml, k half hh) over its KSW k-steps, the two halves, then the NW waves
  float ss[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    ss[i] = 0.f;
#pragma unroll
    for (int s = 0; s < KSW; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 x = xv[s][i][h];
        ss[i] = fmaf(x.x, x.x, ss[i]);
        ss[i] = fmaf(x.y, x.y, ss[i]);
        ss[i] = fmaf(x.z, x.z, ss[i]);
        ss[i] = fmaf(x.w, x.w, ss[i]);
      }
    ss[i] += __shfl_xor(ss[i], 32, kWave);  // commutative: both halves hold the same sum
    if (hh == 0) s_ss[wave][i][ml] = ss[i];
  }
  __syncthreads();
  float r[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    float t = s_ss[0][i][ml];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += s_ss[w][i][ml];
    r[i] = rsqrtf(t / static_cast<float>(a.K) + a.eps);
  }
  f32x16 acc[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) acc[i] = f32x16{};
#pragma unroll
  for (int s = 0; s < KSW; ++s) {
    const float* wk = s_w + 16 * (s0 + s) + 8 * hh;
    const float4 w0 = *reinterpret_cast<const float4*>(wk), w1 = *reinterpret_cast<const float4*>(wk + 4);
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const float4 x0 = xv[s][i][0], x1 = xv[s][i][1];
      const u16x8 y = u16x8{f32_to_bf16(w0.x * (x0.x * r[i])), f32_to_bf16(w0.y * (x0.y * r[i])),
                            f32_to_bf16(w0.z * (x0.z * r[i])), f32_to_bf16(w0.w * (x0.w * r[i])),
                            f32_to_bf16(w1.x * (x1.x * r[i])), f32_to_bf16(w1.y * (x1.y * r[i])),
                            f32_to_bf16(w1.z * (x1.z * r[i])), f32_to_bf16(w1.w * (x1.w * r[i]))};
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wv[s]), as_bf16x8(y), acc[i], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave's reads of the norm weight are done before the buffer takes the partial tiles
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][i][q][lane] = acc[i][q];
  __syncthreads();
  red_epilogue<NW, MB, EPI>(a, red, tile, 0, mb0, tid);
}

// ------------------------------------------------------------------------------------------- tiled GEMM
// epilogue of the tiled forms, straight from a wave's WB x TB accumulator blocks (rb0 / tb0: its first weight /
// token block, ks: its K slice)
// C row i of a block <-> register (i & 3) + 4 (i >> 3), lane half (i >> 2) & 1; column = token lane & 31
template <int WB, int TB, int EPI>
__device__ __forceinline__ void tiled_epilogue(const DgArgs& a, const f32x16 (&acc)[WB][TB], int rb0, int tb0, int lane,
                                               int ks) {
  const int hh = lane >> 5, ml = lane & 31;
#pragma unroll
  for (int b = 0; b < WB; ++b) {
    const int rb = rb0 + b;
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      const int tb = tb0 + t;
      if (rb >= a.tiles || tb >= a.MBT) continue;
      const int m = tb * 32 + ml;
      const f32x16& c = acc[b][t];
      if constexpr (EPI == EPI_PARTIAL) {
        if (m >= a.M) continue;
        float* dst = a.part + (static_cast<int64_t>(ks) * a.M + m) * a.N;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = rb * 32 + 8 * g + 4 * hh;  // registers 4g .. 4g+3: rows n .. n+3
          if (n + 3 < a.N) {
            *reinterpret_cast<float4*>(dst + n) = make_float4(c[4 * g], c[4 * g + 1], c[4 * g + 2], c[4 * g + 3]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (n + j < a.N) dst[n + j] = c[4 * g + j];
          }
        }
      } else if constexpr (EPI == EPI_SWIGLU) {
        // registers r < 8: gate of output column cc(r) = (r & 3) + 8 (r >> 2) + 4 hh; r + 8: its up row
        uint16_t o[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float g = bf16r(c[r]), u = bf16r(c[r + 8]);
          o[r] = to_bf16_bits(bf16r(silu_fast(g)) * u);
        }
        // half 0 holds columns 0-3 | 8-11, half 1 4-7 | 12-15: swap the middle quads so each half owns 8
        // consecutive columns (half 0: 0-7, half 1: 8-15)
        const uint32_t s_lo = hh ? (o[0] | (uint32_t(o[1]) << 16)) : (o[4] | (uint32_t(o[5]) << 16));
        const uint32_t s_hi = hh ? (o[2] | (uint32_t(o[3]) << 16)) : (o[6] | (uint32_t(o[7]) << 16));
        const uint32_t r_lo = __shfl_xor(s_lo, 32, kWave), r_hi = __shfl_xor(s_hi, 32, kWave);
        u16x8 piece;
        if (hh == 0) {
          piece = u16x8{o[0], o[1], o[2], o[3], static_cast<uint16_t>(r_lo), static_cast<uint16_t>(r_lo >> 16),
                        static_cast<uint16_t>(r_hi), static_cast<uint16_t>(r_hi >> 16)};
        } else {
          piece = u16x8{static_cast<uint16_t>(r_lo), static_cast<uint16_t>(r_lo >> 16), static_cast<uint16_t>(r_hi),
                        static_cast<uint16_t>(r_hi >> 16), o[4], o[5], o[6], o[7]};
        }
        // packed for the next GEMM (K' = half): k step = rb, 8-column half hh, token m
        *reinterpret_cast<u16x8*>(a.out + ((static_cast<int64_t>(rb) * a.MBT + tb) * 64 + hh * 32 + ml) * 8) = piece;
      } else {  // EPI_ROPE: rows 0..15 = d 16 qq + cc of head hd, rows 16..31 its partners d + D/2
        if (m >= a.M) continue;
        const int half = a.D / 2, per_h = half / 16, hd = rb / per_h, qq = rb % per_h;
        const int64_t koff = *a.koff_dev;
        int64_t p = a.pos[m];
        p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
        const int G = a.Hq / a.Hkv;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int cc = (r & 3) + 8 * (r >> 2) + 4 * hh;
          const int d1 = 16 * qq + cc, d2 = d1 + half;
          const int n1 = hd * a.D + d1, n2 = n1 + half;
          const float x1 = bf16r(c[r] + bf16_to_f32(a.bias[n1]));
          const float x2 = bf16r(c[r + 8] + bf16_to_f32(a.bias[n2]));
          if (hd < a.Hq + a.Hkv) {
            const float cs = a.cos_t[p * half + d1], sn = a.sin_t[p * half + d1];
            const float o1 = fmaf(x1, cs, -(x2 * sn)), o2 = fmaf(x2, cs, x1 * sn);
            uint16_t* dst = hd < a.Hq ? a.q + ((static_cast<int64_t>(m) * a.Hkv + hd / G) * G + hd % G) * a.D
                                      : a.kc + ((static_cast<int64_t>(m) * a.Hkv + (hd - a.Hq)) * a.Tk + koff) * a.D;
            dst[d1] = to_bf16_bits(o1);
            dst[d2] = to_bf16_bits(o2);
          } else {
            uint16_t* dst = a.vt + (static_cast<int64_t>(m) * a.Hkv + (hd - a.Hq - a.Hkv)) * vt_panel(a.ld_vt, a.D, a.Tk);
            dst[vt_index(d1, koff, a.ld_vt, a.D)] = to_bf16_bits(x1);
            dst[vt_index(d2, koff, a.ld_vt, a.D)] = to_bf16_bits(x2);
          }
        }
      }
    }
  }
}


// The same packed operands at 97..512 rows, where a projection is an MFMA problem (gate_up at 512 rows:
// 8.9 GFLOP against a 17 MB weight stream), not a weight stream: every wave owns a WB x TB tile of 32 x 32
// output blocks (weight rows x tokens) over the workgroup's whole K slice, so each weight fragment feeds TB
// MFMAs and each activation fragment WB (the one-round-trip kernel above re-reads the activation panel per
// 32-row weight block and reduces 4 K slices through LDS). Fragments are loaded straight into registers
// (1-KB coalesced wave loads) through a DEPTH-deep ring, branch-free (the last loads of a slice repeat its
// last k-step instead of branching), so DEPTH * (WB + TB) loads are always in flight. Workgroup = WW x WT
// waves; the 4 waves' overlapping fragments are served by L1 / L2. Epilogues straight from the
// accumulators: fp32 partials (K slice = gridDim.y), SwiGLU (gate row i and up row i + 16 of a block sit in
// registers r and r + 8 of the same lane; one lane-half exchange forms the packed 16-B pieces), or bias +
// RoPE + KV-cache writes (rotation pairs likewise lane-local).
// ring depth: 8 k-steps in flight for qkv + RoPE's 1-2-fragment wave tiles (one K slice, so its 56-step k chain
// per wave is latency-bound: 15.2 -> 14.3 us at 512 rows, tools/decode_cfg_sweep.py), 4 elsewhere (a deeper ring
// there rules out the K slices those shapes need to fill the chip: o_proj 6.9 -> 10.0 us, down 14.5 -> 26.3)
constexpr int dt_depth(int wb, int tb, int epi) { return epi == EPI_ROPE && wb * tb <= 2 ? 8 : 4; }

template <int WB, int TB, int WW, int WT, int EPI>
__global__ __launch_bounds__(256) void decode_gemm_tiled_kernel(DgArgs a) {
  constexpr int DEPTH = dt_depth(WB, TB, EPI);
  static_assert(WW * WT == 4, "4 waves per workgroup");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ww = wave % WW, wt = wave / WW;
  const int rb0 = (blockIdx.x * WW + ww) * WB;  // first 32-row weight block of this wave
  const int tb0 = (blockIdx.z * WT + wt) * TB;  // first 32-token block
  const int per = a.nks / static_cast<int>(gridDim.y);  // k16 steps of this K slice (a multiple of DEPTH)
  const int s0 = static_cast<int>(blockIdx.y) * per, s1 = s0 + per;
  const uint16_t* wp[WB];
  const uint16_t* xp[TB];
#pragma unroll
  for (int b = 0; b < WB; ++b)  // blocks past the end re-read the last one (never stored)
    wp[b] = a.w + static_cast<int64_t>(min(rb0 + b, a.tiles - 1)) * a.nks * 512 + lane * 8;
  const int64_t xstep = static_cast<int64_t>(a.MBT) * 512;
#pragma unroll
  for (int t = 0; t < TB; ++t) xp[t] = a.x + (static_cast<int64_t>(min(tb0 + t, a.MBT - 1)) * 64 + lane) * 8;
  u16x8 rw[DEPTH][WB], rx[DEPTH][TB];
  auto load = [&](int d, int st) {
#pragma unroll
    for (int b = 0; b < WB; ++b) rw[d][b] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp[b] + st * 512));
#pragma unroll
    for (int t = 0; t < TB; ++t) rx[d][t] = *reinterpret_cast<const u16x8*>(xp[t] + st * xstep);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, s0 + d);
  __builtin_amdgcn_sched_barrier(0);
  f32x16 acc[WB][TB];
#pragma unroll
  for (int b = 0; b < WB; ++b)
#pragma unroll
    for (int t = 0; t < TB; ++t) acc[b][t] = f32x16{};
  for (int st = s0; st < s1; st += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int b = 0; b < WB; ++b)
#pragma unroll
        for (int t = 0; t < TB; ++t)
          acc[b][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(rw[d][b]), as_bf16x8(rx[d][t]), acc[b][t], 0, 0, 0);
      load(d, min(st + d + DEPTH, s1 - 1));
      // keep the refill here: left alone, hipcc sinks every load next to its MFMAs (fewest live registers)
      // and the ring degenerates to one k-step in flight behind a vmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  tiled_epilogue<WB, TB, EPI>(a, acc, rb0, tb0, lane, static_cast<int>(blockIdx.y));
}

// LDS-staged tiled form: the workgroup's fragments (RB = WR * WB weight blocks + TT = WT * TB token blocks per
// k16 step) are copied global -> LDS by LDS-DMA (global_load_lds_dwordx4: one 1-KB fragment per wave
// instruction, lane-linear, so the image needs no swizzle and every ds_read_b128 of a fragment is
// conflict-free) in stages of KST k-steps through NBUF buffers, STAGES_AHEAD stages in flight; each fragment
// leaves L2 once per workgroup instead of once per wave. Order per stage (cdna_hip_programming.md §5,
// "Pipelining across barriers"): counted vmcnt (own copies of this stage landed, the next stages' still in
// flight) -> lgkmcnt(0) + raw s_barrier (everyone's copies landed; everyone's reads of the buffer about to be
// refilled are done) -> refill the oldest buffer -> MFMAs from this stage's buffer. One __shared__ array.
// NBUF: stage buffers, NBUF - 1 stages in flight ahead of the one consumed (round 5: 3 -> up to 6 — at 2 stages ahead
// a workgroup kept 24 KB of copies in flight and each stage waited out most of an L2 / HBM round trip).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WR, int WT, int WB, int TB, int EPI, int KST = 2, int NBUF = 3>
__global__ __launch_bounds__(64 * WR * WT) void decode_gemm_lds_kernel(DgArgs a) {
  constexpr int NW = WR * WT, RB = WR * WB, TT = WT * TB, FR = RB + TT;
  static_assert(NBUF >= 3, "at least one stage ahead besides the one being refilled");
  constexpr int PER_WAVE = KST * FR / NW;  // LDS-DMA instructions per wave and stage
  static_assert(KST * FR % NW == 0, "copies must divide evenly over the waves");
  __shared__ __attribute__((aligned(16))) uint16_t lds[NBUF * KST * FR * 512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WR, wt = wave / WR;
  const int rbw = blockIdx.x * RB, tbw = blockIdx.z * TT;  // workgroup's first weight / token block
  const int per = a.nks / static_cast<int>(gridDim.y);
  const int s0 = static_cast<int>(blockIdx.y) * per;
  const int nst = per / KST;  // stages of this K slice
  const int64_t xstep = static_cast<int64_t>(a.MBT) * 512;
  // this wave's copies: fragment slots idx = wave + NW * c of a stage (slot = j * FR + f)
  const uint16_t* src[PER_WAVE];
  int64_t sstep[PER_WAVE];
  int dsto[PER_WAVE];
#pragma unroll
  for (int c = 0; c < PER_WAVE; ++c) {
    const int idx = wave + NW * c, j = idx / FR, f = idx % FR;
    if (f < RB) {
      src[c] = a.w + (static_cast<int64_t>(min(rbw + f, a.tiles - 1)) * a.nks + j) * 512 + lane * 8;
      sstep[c] = 512;
    } else {
      src[c] = a.x + (static_cast<int64_t>(j) * a.MBT + min(tbw + f - RB, a.MBT - 1)) * 512 + lane * 8;
      sstep[c] = xstep;
    }
    dsto[c] = idx * 512;
  }
  auto issue = [&](int stage) {
    const int st = s0 + min(stage, nst - 1) * KST;  // past the end: repeat the last stage (never read)
    uint16_t* buf = lds + (stage % NBUF) * (KST * FR * 512);
#pragma unroll
    for (int c = 0; c < PER_WAVE; ++c)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src[c] + st * sstep[c]),
                                       (__attribute__((address_space(3))) void*)(buf + dsto[c]), 16, 0, 0);
  };
  f32x16 acc[WB][TB];
#pragma unroll
  for (int b = 0; b < WB; ++b)
#pragma unroll
    for (int t = 0; t < TB; ++t) acc[b][t] = f32x16{};
#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j) issue(j);
  for (int i = 0; i < nst; ++i) {
    // own copies of stage i landed (stages i + 1 .. i + NBUF - 2, PER_WAVE each, may still be in flight)
    wait_vmcnt<(NBUF - 2) * PER_WAVE>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(i + NBUF - 1);  // into the buffer read in iteration i - 1 (every wave is past it)
    const uint16_t* buf = lds + (i % NBUF) * (KST * FR * 512);
#pragma unroll
    for (int j = 0; j < KST; ++j) {
      u16x8 wf[WB], xf[TB];
#pragma unroll
      for (int b = 0; b < WB; ++b)
        wf[b] = *reinterpret_cast<const u16x8*>(buf + (j * FR + wr * WB + b) * 512 + lane * 8);
#pragma unroll
      for (int t = 0; t < TB; ++t)
        xf[t] = *reinterpret_cast<const u16x8*>(buf + (j * FR + RB + wt * TB + t) * 512 + lane * 8);
#pragma unroll
      for (int b = 0; b < WB; ++b)
#pragma unroll
        for (int t = 0; t < TB; ++t)
          acc[b][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wf[b]), as_bf16x8(xf[t]), acc[b][t], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the two repeated stages' copies
  tiled_epilogue<WB, TB, EPI>(a, acc, rbw + wr * WB, tbw + wt * TB, lane, static_cast<int>(blockIdx.y));
}

// ------------------------------------------------------------------------------------------- consumers
// x_out = x_in + bf16(sum_ks part) (fp32 residual stream, bf16 module output: add_rmsnorm_fwd semantics),
// y = bf16(w * (x_out * rsqrt(mean(x_out^2) + eps))) written packed (MBT blocks) or row-major (MBT = 0).
// Two waves per row, each lane owns 8-column chunks tid, tid + 128, ...; every load of the row (x and the NS
// partial slices) is issued before the first add, so the kernel is one dependent memory round trip.
// NS < 0: runtime slice count (loop).
template <int CH, int NS>
__global__ __launch_bounds__(128) void dec_rmsnorm_kernel(const float* x_in, const float* part, int nsplit, float* x_out,
                                                          const float* w, uint16_t* y, int64_t M, int64_t H, int64_t MBT,
                                                          float eps, int64_t XMBT = 0, uint16_t* y2 = nullptr,
                                                          int64_t MBT2 = 0) {
  __shared__ float s_ss[2];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t nch = H / 8;
  float4 xv[CH][2], wv[CH][2];
  constexpr int NSL = NS > 0 ? NS : 1;
  float4 pv[CH][NSL][2];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t ch = tid + 128 * c;
    if (ch < nch) {
      // XMBT > 0: x is the fused-norm decode's packed fp32 residual (8 consecutive columns contiguous)
      const float* xr = XMBT > 0 ? x_in + pkf_off(row, ch * 8, XMBT) : x_in + row * H + ch * 8;
      xv[c][0] = *reinterpret_cast<const float4*>(xr);
      xv[c][1] = *reinterpret_cast<const float4*>(XMBT > 0 ? xr + 256 : xr + 4);
      // the norm weight with the row's first loads: no second memory round trip after the row sum
      wv[c][0] = *reinterpret_cast<const float4*>(w + ch * 8);
      wv[c][1] = *reinterpret_cast<const float4*>(w + ch * 8 + 4);
      if constexpr (NS > 0) {
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          const float* p = part + (static_cast<int64_t>(k) * M + row) * H + ch * 8;
          pv[c][k][0] = *reinterpret_cast<const float4*>(p);
          pv[c][k][1] = *reinterpret_cast<const float4*>(p + 4);
        }
      }
    }
  }
  float v[CH][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t ch = tid + 128 * c;
    if (ch >= nch) continue;
    v[c][0] = xv[c][0].x; v[c][1] = xv[c][0].y; v[c][2] = xv[c][0].z; v[c][3] = xv[c][0].w;
    v[c][4] = xv[c][1].x; v[c][5] = xv[c][1].y; v[c][6] = xv[c][1].z; v[c][7] = xv[c][1].w;
    if (part) {
      float d[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (NS > 0) {
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          d[0] += pv[c][k][0].x; d[1] += pv[c][k][0].y; d[2] += pv[c][k][0].z; d[3] += pv[c][k][0].w;
          d[4] += pv[c][k][1].x; d[5] += pv[c][k][1].y; d[6] += pv[c][k][1].z; d[7] += pv[c][k][1].w;
        }
      } else {
        for (int k = 0; k < nsplit; ++k) {
          const float* p = part + (static_cast<int64_t>(k) * M + row) * H + ch * 8;
          const float4 b0 = *reinterpret_cast<const float4*>(p), b1 = *reinterpret_cast<const float4*>(p + 4);
          d[0] += b0.x; d[1] += b0.y; d[2] += b0.z; d[3] += b0.w;
          d[4] += b1.x; d[5] += b1.y; d[6] += b1.z; d[7] += b1.w;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] += bf16r(d[j]);
    }
    if (x_out) {
      *reinterpret_cast<float4*>(x_out + row * H + ch * 8) = make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
      *reinterpret_cast<float4*>(x_out + row * H + ch * 8 + 4) = make_float4(v[c][4], v[c][5], v[c][6], v[c][7]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) s_ss[tid >> 6] = ss;
  __syncthreads();
  const float r = rsqrtf((s_ss[0] + s_ss[1]) / static_cast<float>(H) + eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t ch = tid + 128 * c;
    if (ch >= nch) continue;
    const float wj[8] = {wv[c][0].x, wv[c][0].y, wv[c][0].z, wv[c][0].w, wv[c][1].x, wv[c][1].y, wv[c][1].z, wv[c][1].w};
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16(wj[j] * (v[c][j] * r));
    if (y) {
      uint16_t* dst = MBT > 0 ? y + pk_off(row, ch * 8, MBT) : y + row * H + ch * 8;
      *reinterpret_cast<u16x8*>(dst) = o;
    }
    // the packed copy the decode lm_head reads (y2, MBT2 blocks), beside a row-major y
    if (y2) *reinterpret_cast<u16x8*>(y2 + pk_off(row, ch * 8, MBT2)) = o;
  }
}

// qkv = bf16(sum_ks part + bias) of one decode token, then rotary embedding (rope_qkv_fwd_kernel's math and
// rounding): q -> (B, Hkv, G, 1, D); k -> cache row koff; v -> V^T cache column koff (and/or row-major v).
struct DecRopeArgs {
  const float* part;
  int nsplit;
  const uint16_t* bias;
  const int64_t* pos;
  const float* cos_t;
  const float* sin_t;
  uint16_t* q;
  uint16_t* k;
  uint16_t* v;
  uint16_t* vt;
  int64_t B, Hq, Hkv, D, Tk, ld_vt, maxpos, koff;
  const int64_t* koff_dev;
};

__global__ __launch_bounds__(256) void dec_rope_kernel(DecRopeArgs a) {
  const int64_t half = a.D / 2, Hall = a.Hq + 2 * a.Hkv, NQ = Hall * a.D;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= a.B * Hall * half) return;
  const int64_t koff = a.koff_dev ? *a.koff_dev : a.koff;
  if (koff < 0 || koff >= a.Tk) return;
  const int64_t j = i % half, h = (i / half) % Hall, b = i / (half * Hall);
  const int64_t c1 = h * a.D + j, c2 = c1 + half;
  float s1 = 0.f, s2 = 0.f;
  for (int k = 0; k < a.nsplit; ++k) {
    s1 += a.part[(k * a.B + b) * NQ + c1];
    s2 += a.part[(k * a.B + b) * NQ + c2];
  }
  const float x1 = bf16r(s1 + bf16_to_f32(a.bias[c1])), x2 = bf16r(s2 + bf16_to_f32(a.bias[c2]));
  if (h < a.Hq + a.Hkv) {
    int64_t p = a.pos[b];
    p = p < 0 ? 0 : (p >= a.maxpos ? a.maxpos - 1 : p);
    const float c = a.cos_t[p * half + j], s = a.sin_t[p * half + j];
    const float o1 = fmaf(x1, c, -(x2 * s)), o2 = fmaf(x2, c, x1 * s);
    uint16_t* dst;
    if (h < a.Hq) {
      const int64_t G = a.Hq / a.Hkv, g = h / G, hi = h % G;
      dst = a.q + ((b * a.Hkv + g) * G + hi) * a.D;
    } else {
      dst = a.k + ((b * a.Hkv + (h - a.Hq)) * a.Tk + koff) * a.D;
    }
    dst[j] = to_bf16_bits(o1);
    dst[j + half] = to_bf16_bits(o2);
  } else {
    const int64_t hv = h - a.Hq - a.Hkv;
    if (a.vt) {
      uint16_t* dst = a.vt + (b * a.Hkv + hv) * vt_panel(a.ld_vt, a.D, a.Tk);
      dst[vt_index(j, koff, a.ld_vt, a.D)] = to_bf16_bits(x1);
      dst[vt_index(j + half, koff, a.ld_vt, a.D)] = to_bf16_bits(x2);
    }
    if (a.v) {
      uint16_t* dst = a.v + ((b * a.Hkv + hv) * a.Tk + koff) * a.D;
      dst[j] = to_bf16_bits(x1);
      dst[j + half] = to_bf16_bits(x2);
    }
  }
}

// ------------------------------------------------------------------------------------------- step prologue
// The per-token bookkeeping of the graphed decode step in one launch (was ~8 torch launches): with t = *t_dev,
// row b's previous token responses[b, t - 1] -> x[b] = float(embed[token]) (the fp32 residual stream input,
// F.embedding), pos[b] = last_pos[b] + t (its rotary position), key_valid[b, t + P - 1] = 1 (the new cache
// slot, index_fill_). The last workgroup to arrive (every other one has read t_dev) publishes *kpos = t + P - 1
// and *t_cur = t for the rest of the step and advances *t_dev to t + 1 for the next replay.
__global__ __launch_bounds__(128) void decode_prologue_kernel(const int64_t* responses, int64_t ld_r, int64_t* t_dev,
                                                              int64_t* t_cur, const int64_t* last_pos, int64_t P,
                                                              const uint16_t* embed, int64_t V, int64_t H, float* x,
                                                              int64_t* pos, int64_t* kpos, uint8_t* valid,
                                                              int64_t ld_valid, unsigned* ticket, int64_t x_mbt) {
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t t = *t_dev;
  int64_t tok = responses[b * ld_r + t - 1];
  tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);
  const uint16_t* e = embed + tok * H;
  for (int64_t c = tid; c < H / 8; c += 128) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(e + 8 * c);
    // x_mbt > 0: the fused-norm decode's packed fp32 residual stream
    float* xr = x_mbt > 0 ? x + pkf_off(b, 8 * c, x_mbt) : x + b * H + 8 * c;
    *reinterpret_cast<float4*>(xr) = make_float4(bf16_to_f32(v[0]), bf16_to_f32(v[1]), bf16_to_f32(v[2]),
                                                 bf16_to_f32(v[3]));
    *reinterpret_cast<float4*>(x_mbt > 0 ? xr + 256 : xr + 4) =
        make_float4(bf16_to_f32(v[4]), bf16_to_f32(v[5]), bf16_to_f32(v[6]), bf16_to_f32(v[7]));
  }
  if (tid == 0) {
    pos[b] = last_pos[b] + t;
    valid[b * ld_valid + t + P - 1] = 1;
  }
  if (last_block_ticket(ticket) && tid == 0) {
    *kpos = t + P - 1;
    *t_cur = t;
    *t_dev = t + 1;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------------------------------- lm_head (<= 64 rows)
// The decode step's lm_head at <= 64 token rows (the N = 8 rank's 64): logits = h W^T, a 272 MB weight stream for
// 17 GFLOP — drl_gemm's 256 x 256 tiles over M = 64 ran it at 3.9 TB/s (594 tiles of 7 k-pairs never fill its
// pipeline). Persistent: one workgroup per CU holds the packed bf16 activation panel (MB token blocks x NKS k16
// steps, 112 KB at 64 rows x 896) in LDS for the whole launch, and owns a contiguous, balanced range of 32-row vocab
// tiles. The packed weight of that range is one contiguous stream; its k16 steps are split evenly over the NWV waves
// (stream-K inside the workgroup), each wave pulling its share through a DEPTH-deep register ring of 1-KB fragment
// loads and running MB MFMAs per step against LDS fragments. A tile a wave finishes from k = 0 is written straight from
// its accumulators (bf16, the drl_gemm epilogue's rounding); a tile split between two waves is summed once, after the
// workgroup barrier, as (first wave's k prefix) + (second wave's suffix) — fixed order, deterministic. No workgroup
// waits on another.
struct LmArgs {
  const uint16_t* h;  // packed bf16 panel (MB token blocks, NKS k16 steps)
  const uint16_t* w;  // packed weight: tiles of 32 vocab rows x NKS k16 steps
  uint16_t* out;      // logits (M, ld) bf16
  int64_t ld;
  int M, V, tiles;
};

template <int MB, int NKS, int NWV, int DEPTH>
__global__ __launch_bounds__(64 * NWV) void decode_lm_head_kernel(LmArgs a) {
  // the split-tile slots (NWV x MB f32x16 per lane) reuse the panel's LDS once the panel is no longer read
  constexpr int PANEL = MB * NKS * 512, SLOTS = NWV * MB * 16 * 64 * 2;
  __shared__ __attribute__((aligned(16))) uint16_t s_x[PANEL > SLOTS ? PANEL : SLOTS];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, g = blockIdx.x;
  const int t0 = static_cast<int>(static_cast<int64_t>(g) * a.tiles / G);
  const int t1 = static_cast<int>(static_cast<int64_t>(g + 1) * a.tiles / G);
  const int n_it = (t1 - t0) * NKS;
  const int i0 = wave * n_it / NWV, i1 = (wave + 1) * n_it / NWV;  // the host keeps i1 - i0 >= NKS
  const uint16_t* wp = a.w + static_cast<int64_t>(t0) * NKS * 512 + lane * 8;
  u16x8 ring[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    ring[d] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp + static_cast<int64_t>(min(i0 + d, i1 - 1)) * 512));
  // the activation panel -> LDS by LDS-DMA (lane-linear 1-KB fragments: the panel's own layout)
  for (int f = wave; f < MB * NKS; f += NWV)
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(a.h + f * 512 + lane * 8),
                                     (__attribute__((address_space(3))) void*)(s_x + f * 512), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x16 acc[MB], head[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) acc[m] = head[m] = f32x16{};
  int ks = i0 % NKS, tile = t0 + i0 / NKS;
  bool in_head = ks != 0, has_head = false;  // this wave's first tile started mid-way: its k = 0 part is the
                                             // previous wave's tail
  const int hh = lane >> 5, ml = lane & 31;
  auto store_tile = [&](int t, const f32x16 (&c)[MB]) {
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int row = 32 * m + ml;
      if (row >= a.M) continue;
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int n = t * 32 + 8 * q4 + 4 * hh;  // registers 4 q4 .. + 3: vocab rows n .. n + 3
        uint16_t* dst = a.out + static_cast<int64_t>(row) * a.ld + n;
        if (n + 3 < a.V) {
          *reinterpret_cast<u16x4*>(dst) = u16x4{to_bf16_bits(c[m][4 * q4]), to_bf16_bits(c[m][4 * q4 + 1]),
                                                 to_bf16_bits(c[m][4 * q4 + 2]), to_bf16_bits(c[m][4 * q4 + 3])};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n + j < a.V) dst[j] = to_bf16_bits(c[m][4 * q4 + j]);
        }
      }
    }
  };
  // the panel fragments of the current k16 step, read one step ahead (the LDS latency under the MFMAs)
  u16x8 xf[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) xf[m] = *reinterpret_cast<const u16x8*>(s_x + (ks * MB + m) * 512 + lane * 8);
  for (int base = i0; base < i1; base += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int i = base + d;
      if (i < i1) {
        const int kn = ks + 1 == NKS ? 0 : ks + 1;
        u16x8 xn[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) xn[m] = *reinterpret_cast<const u16x8*>(s_x + (kn * MB + m) * 512 + lane * 8);
#pragma unroll
        for (int m = 0; m < MB; ++m)
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ring[d]), as_bf16x8(xf[m]), acc[m], 0, 0, 0);
#pragma unroll
        for (int m = 0; m < MB; ++m) xf[m] = xn[m];
        ring[d] = __builtin_nontemporal_load(
            reinterpret_cast<const u16x8*>(wp + static_cast<int64_t>(min(i + DEPTH, i1 - 1)) * 512));
        if (++ks == NKS) {  // a tile's last k16 step
          if (in_head) {
#pragma unroll
            for (int m = 0; m < MB; ++m) head[m] = acc[m];
            in_head = false;
            has_head = true;
          } else {
            store_tile(tile, acc);
          }
#pragma unroll
          for (int m = 0; m < MB; ++m) acc[m] = f32x16{};
          ks = 0;
          ++tile;
        }
      }
      // keep the refill here (decode_gemm_tiled_kernel: otherwise hipcc sinks each load next to its use)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // split tiles: every wave's head partial into LDS (the panel is no longer read), then each tail adds the next
  // wave's head — the tile's k prefix + its suffix
  __syncthreads();
  float* slots = reinterpret_cast<float*>(s_x);
  if (has_head) {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) slots[((wave * MB + m) * 16 + q) * 64 + lane] = head[m][q];
  }
  __syncthreads();
  if (ks != 0) {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] += slots[(((wave + 1) * MB + m) * 16 + q) * 64 + lane];
    store_tile(tile, acc);
  }
}

// ------------------------------------------------------------------------------------------- planning
struct DgPlan {
  int mb, ksw, ksplit, mgroups, tiles, mbt;
};

int g_dg_mb = 0, g_dg_ksw = 0;  // tuning override (drl_decode_gemm_set_plan), 0 = automatic
int g_lm_cfg = -1;              // decode lm_head (waves, ring depth) configuration (drl_decode_lm_head_set_config)

// (token blocks per workgroup, k16 steps per wave) instantiated; registers in flight 4 * ksw * (1 + mb)
struct DgShape { int mb, ksw; };
constexpr DgShape kShapes[] = {{2, 14}, {2, 7}, {2, 4}, {2, 2}, {2, 1}, {1, 19}, {1, 14}, {1, 7}, {1, 4}, {1, 2}, {1, 1}};

bool plan_decode_gemm(int64_t M, int64_t N, int64_t K, int epi, DgPlan& p) {
  if (M < 1 || M > 512 || K % 64 != 0 || N < 1) return false;
  const int blocks = static_cast<int>((M + 31) / 32);
  // one panel layout per M for every producer / consumer: blocks padded to the 2-block workgroup granule
  p.mbt = blocks == 1 ? 1 : (blocks + 1) / 2 * 2;
  p.tiles = static_cast<int>(epi == EPI_SWIGLU ? (N / 2 + 15) / 16 : (N + 31) / 32);
  const int nks = static_cast<int>(K / 16);
  // fewest K slices (partial sums for the consumer) among the shapes that give >= 96 workgroups, then
  // 2-block workgroups (each weight fragment feeds two MFMAs); otherwise the shape with the most workgroups.
  // The SwiGLU / RoPE epilogues need the whole K in one workgroup.
  bool found = false, full = false;
  int64_t best_wgs = 0;
  for (const DgShape& c : kShapes) {
    if (c.mb > p.mbt) continue;
    if (nks % (4 * c.ksw) != 0) continue;
    const int ks = nks / (4 * c.ksw);
    if (epi != EPI_PARTIAL && ks != 1) continue;
    if ((g_dg_mb && c.mb != g_dg_mb) || (g_dg_ksw && c.ksw != g_dg_ksw)) continue;
    const int64_t wgs = static_cast<int64_t>(p.tiles) * (p.mbt / c.mb) * ks;
    const bool ok = wgs >= 96;
    bool take = !found;
    if (found) {
      // among shapes that fill the chip: the fewest K slices, then one-block workgroups (twice the workgroups on the
      // same K slices) — measured faster at 64 / 256 / 512 rows for qkv + RoPE (512 rows: 10.7 -> 9.7 us), o_proj
      // (256 rows: 7.7 -> 5.5) and down_proj (13.4 vs 37.3), profiles/r03_decode_cfg_sweep2.jsonl — except the
      // SwiGLU gate_up, whose 2-block workgroups feed each weight fragment to two MFMAs (64 rows: 8.1 vs 9.0 us)
      const bool more_blocks = epi == EPI_SWIGLU ? c.mb > p.mb : c.mb < p.mb;
      if (ok && !full) take = true;
      else if (ok && full) take = ks < p.ksplit || (ks == p.ksplit && more_blocks);
      else if (!ok && !full) take = wgs > best_wgs;
    }
    if (take) {
      p.mb = c.mb;
      p.ksw = c.ksw;
      p.ksplit = ks;
      p.mgroups = p.mbt / c.mb;
      best_wgs = wgs;
      full = ok;
      found = true;
    }
  }
  return found;
}

// tiled path: (WB, TB, WW, WT, lds) configurations instantiated (lds: the LDS-staged kernel, WW x WT waves)
struct DtShape { int wb, tb, ww, wt, lds; };
// 17-22 (round 5): LDS-staged with deeper rings (NBUF stage buffers, NBUF - 1 stages in flight), larger tiles
// 9-13: larger token panels per workgroup (the activation panel staged once for more weight rows' MFMAs), round 4;
// 14-16: LDS-staged with 4 k-steps per stage (half the barriers, twice the LDS: fewer resident workgroups)
constexpr DtShape kTiled[] = {{2, 2, 4, 2, 1}, {2, 2, 2, 2, 1}, {1, 2, 2, 2, 1}, {2, 1, 2, 2, 1},
                              {2, 2, 2, 2, 0}, {2, 2, 4, 1, 0}, {1, 2, 2, 2, 0}, {1, 2, 4, 1, 0}, {1, 1, 2, 2, 0},
                              {2, 2, 1, 4, 1}, {2, 4, 2, 2, 1}, {1, 4, 2, 2, 1}, {2, 4, 1, 4, 1}, {2, 4, 2, 2, 0},
                              {1, 2, 2, 2, 1}, {2, 1, 2, 2, 1}, {2, 2, 2, 2, 1},
                              {2, 2, 4, 2, 1}, {2, 2, 2, 2, 1}, {1, 2, 2, 2, 1}, {2, 1, 2, 2, 1}, {2, 2, 2, 2, 1},
                              {1, 2, 2, 2, 1}};
constexpr int kNumTiled = static_cast<int>(sizeof(kTiled) / sizeof(kTiled[0]));
int g_dt_force = -1;  // tuning: force configuration index (drl_decode_gemm_force_tiled), -1 = planner
int g_dt_min_rows = 192;  // tuning: smallest M for the tiled path
// 0 = never the tiled path (drl_decode_gemm_set_tiled), 1 = automatic, 2 = automatic with one K slice (tests:
// the partial form in the fused qkv + RoPE launch's summation order)
int g_dt_mode = 1;
int g_dt_max_ks = 4;  // tuning: most K slices of a partial-sum plan (drl_decode_gemm_set_max_splits)

// the tiled plan when the shape is in its range. Configuration by shape class, from the sweep of every
// configuration at 128 / 256 / 512 rows (tools/kernel_bench.py --only decode_gemm, profiles/r02_decode_gemm.jsonl):
//   SwiGLU gate_up from 192 rows: LDS-staged, 64 x 128 workgroup tile (512 rows: 29.1 -> 19.0 us);
//   partials with a long K (down_proj, K 4864) from 384 rows: register ring, 64 x 128 (23.3 -> 14.6 us);
//   partials / qkv + RoPE with a short K from 192 rows: register ring, 64 x 64 (o_proj 7.7 -> 6.7 us,
//   qkv 11.9 -> 8.6 us at 512).
// K slices (partials only, each a multiple of 4 k-steps, <= 4): the fewest that give >= 160 workgroups, else the
// most workgroups. p.mb = 0 marks a tiled plan; p.ksw = index into kTiled.
bool plan_decode_tiled(int64_t M, int64_t N, int64_t K, int epi, DgPlan& p) {
  // gate_up + SwiGLU at 97..191 rows: the LDS-staged kernel with 4 k-steps per stage beats the one-round-trip kernel
  // (128 rows: 11.1 -> 10.0 us; 64 rows: 9.7 against 8.0, so not below; profiles/r04_decode_cfg_sweep_rows64_128.jsonl)
  const bool swiglu_mid = epi == EPI_SWIGLU && M > 96 && M < 192 && g_dt_min_rows >= 192 && g_dt_force < 0;
  if (g_dt_mode == 0 || (M < g_dt_min_rows && !swiglu_mid) || M > 512 || K % 64 != 0 || N < 1) return false;
  // qkv + RoPE (whole K per output block): the one-round-trip kernel's 4 waves on K quarters beat every tiled
  // configuration from 192 rows on (512 rows: 14.2 -> 9.7 us, 256 rows: 14.3 -> 7.3;
  // profiles/r03_decode_cfg_sweep2.jsonl), unless a configuration is forced
  if (epi == EPI_ROPE && g_dt_force < 0) return false;
  int ci;
  if (g_dt_force >= 0) ci = g_dt_force;
  else if (epi == EPI_SWIGLU) ci = swiglu_mid ? 14 : 2;
  // long-K partials (down_proj): 4 k-steps per LDS stage (512 rows: 14.5 -> 13.5 us, 256 rows: 13.2 -> 12.3 against
  // the register-ring and one-round-trip kernels; profiles/r04_decode_cfg_sweep_kst4.jsonl)
  else if (K >= 2048) ci = 15;
  else {
    // short-K partials (o_proj): the one-round-trip kernel below 384 rows (256 rows: 6.75 -> 5.5 us)
    if (epi == EPI_PARTIAL && M < 384 && g_dt_force < 0 && g_dt_min_rows >= 192) return false;
    ci = 8;
  }
  const int blocks = static_cast<int>((M + 31) / 32);
  p.mbt = (blocks + 1) / 2 * 2;
  p.tiles = static_cast<int>(epi == EPI_SWIGLU ? (N / 2 + 15) / 16 : (N + 31) / 32);
  const int nks = static_cast<int>(K / 16);
  const DtShape& c = kTiled[ci];
  const int rows = c.wb * c.ww, toks = c.tb * c.wt;
  const int64_t base = static_cast<int64_t>((p.tiles + rows - 1) / rows) * ((p.mbt + toks - 1) / toks);
  bool found = false;
  int64_t best_wgs = 0;
  for (int ks = 1; ks <= (epi == EPI_PARTIAL && g_dt_mode == 1 ? g_dt_max_ks : 1); ++ks) {
    // register ring: dt_depth k-steps per refill round; LDS stages: 2 k-steps
    if (nks % ks != 0 || (nks / ks) % (c.lds ? 4 : dt_depth(c.wb, c.tb, epi)) != 0) continue;
    const int64_t wgs = base * ks;
    if (found && best_wgs >= 160) break;  // the fewest slices that fill the chip
    if (!found || wgs > best_wgs) {
      p.mb = 0;
      p.ksw = ci;
      p.ksplit = ks;
      p.mgroups = static_cast<int>((p.mbt + toks - 1) / toks);
      best_wgs = wgs;
      found = true;
    }
  }
  return found;
}

template <int EPI>
void launch_dt(const DgArgs& a, const DgPlan& p, hipStream_t s) {
  const DtShape c = kTiled[p.ksw];
  const dim3 grid((p.tiles + c.wb * c.ww - 1) / (c.wb * c.ww), p.ksplit, p.mgroups);
  switch (p.ksw) {
    case 0: hipLaunchKernelGGL((decode_gemm_lds_kernel<4, 2, 2, 2, EPI>), grid, dim3(512), 0, s, a); break;
    case 1: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 2, EPI>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 1, 2, EPI>), grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 1, EPI>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((decode_gemm_tiled_kernel<2, 2, 2, 2, EPI>), grid, dim3(256), 0, s, a); break;
    case 5: hipLaunchKernelGGL((decode_gemm_tiled_kernel<2, 2, 4, 1, EPI>), grid, dim3(256), 0, s, a); break;
    case 6: hipLaunchKernelGGL((decode_gemm_tiled_kernel<1, 2, 2, 2, EPI>), grid, dim3(256), 0, s, a); break;
    case 7: hipLaunchKernelGGL((decode_gemm_tiled_kernel<1, 2, 4, 1, EPI>), grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL((decode_gemm_tiled_kernel<1, 1, 2, 2, EPI>), grid, dim3(256), 0, s, a); break;
    // LDS-staged: (WR, WT, WB, TB) = waves along weight rows / tokens, blocks per wave
    case 9: hipLaunchKernelGGL((decode_gemm_lds_kernel<1, 4, 2, 2, EPI>), grid, dim3(256), 0, s, a); break;
    case 10: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 4, EPI>), grid, dim3(256), 0, s, a); break;
    case 11: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 1, 4, EPI>), grid, dim3(256), 0, s, a); break;
    case 12: hipLaunchKernelGGL((decode_gemm_lds_kernel<1, 4, 2, 4, EPI>), grid, dim3(256), 0, s, a); break;
    case 14: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 1, 2, EPI, 4>), grid, dim3(256), 0, s, a); break;
    case 15: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 1, EPI, 4>), grid, dim3(256), 0, s, a); break;
    case 16: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 2, EPI, 4>), grid, dim3(256), 0, s, a); break;
    case 17: hipLaunchKernelGGL((decode_gemm_lds_kernel<4, 2, 2, 2, EPI, 2, 6>), grid, dim3(512), 0, s, a); break;
    case 18: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 2, EPI, 2, 6>), grid, dim3(256), 0, s, a); break;
    case 19: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 1, 2, EPI, 2, 6>), grid, dim3(256), 0, s, a); break;
    case 20: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 1, EPI, 4, 5>), grid, dim3(256), 0, s, a); break;
    case 21: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 2, 2, EPI, 4, 4>), grid, dim3(256), 0, s, a); break;
    case 22: hipLaunchKernelGGL((decode_gemm_lds_kernel<2, 2, 1, 2, EPI, 4, 4>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((decode_gemm_tiled_kernel<2, 4, 2, 2, EPI>), grid, dim3(256), 0, s, a); break;
  }
}

bool plan_any(int64_t M, int64_t N, int64_t K, int epi, DgPlan& p) {
  return plan_decode_tiled(M, N, K, epi, p) || plan_decode_gemm(M, N, K, epi, p);
}

template <int MB, int EPI>
void launch_dg(const DgArgs& a, const DgPlan& p, hipStream_t s) {
  const dim3 grid(p.tiles, p.ksplit, p.mgroups);
  switch (p.ksw) {
    case 19:
      if constexpr (MB == 1) hipLaunchKernelGGL((decode_gemm_kernel<1, 19, EPI>), grid, dim3(256), 0, s, a);
      break;
    case 14: hipLaunchKernelGGL((decode_gemm_kernel<MB, 14, EPI>), grid, dim3(256), 0, s, a); break;
    case 7: hipLaunchKernelGGL((decode_gemm_kernel<MB, 7, EPI>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((decode_gemm_kernel<MB, 4, EPI>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((decode_gemm_kernel<MB, 2, EPI>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((decode_gemm_kernel<MB, 1, EPI>), grid, dim3(256), 0, s, a); break;
  }
}

// fused-norm consumers: (waves, token blocks per workgroup, k16 steps per wave) instantiated; whole K per workgroup
// (NW x KSW = K / 16). Registers in flight per lane: 4 KSW (weights) + 8 KSW MB (fp32 residual)
struct DnShape { int nw, mb, ksw; };
// (16 waves at K 3584 / 4096 would need more than their 128 registers per lane: those models take the unfused step)
constexpr DnShape kNorm[] = {{4, 1, 14}, {8, 1, 7}, {8, 2, 7}, {4, 2, 7}};
constexpr int kNumNorm = static_cast<int>(sizeof(kNorm) / sizeof(kNorm[0]));
int g_dn_force = -1;     // tuning: force a kNorm configuration (drl_decode_norm_set_plan), -1 = planner
int g_dn_max_rows = 128;  // the fused-norm decode up to this many rows (beyond: the tiled kernels + dec_rmsnorm)
int g_dr_max_ks = 0;     // tuning: most K slices of an EPI_RESID plan (0 = the partial-sum planner's choice)

// the consumer's configuration: the SwiGLU gate_up prefers 2 token blocks per workgroup (each weight fragment feeds
// two MFMAs: the 17 MB weight is read once), qkv + RoPE one (twice the workgroups over a 2 MB weight); among those,
// the fewest waves (longest per-wave chain that fits the registers)
bool plan_norm(int64_t M, int64_t N, int64_t K, int epi, DgPlan& p) {
  if (M < 1 || M > g_dn_max_rows || M > 512 || K % 64 != 0 || K > 4096 || N < 1) return false;
  const int blocks = static_cast<int>((M + 31) / 32);
  p.mbt = blocks == 1 ? 1 : (blocks + 1) / 2 * 2;
  p.tiles = static_cast<int>(epi == EPI_SWIGLU ? (N / 2 + 15) / 16 : (N + 31) / 32);
  const int nks = static_cast<int>(K / 16);
  const int want_mb = epi == EPI_SWIGLU ? 2 : 1;
  int best = -1;
  for (int ci = 0; ci < kNumNorm; ++ci) {
    const DnShape& c = kNorm[ci];
    if (c.nw * c.ksw != nks || c.mb > p.mbt || p.mbt % c.mb != 0) continue;
    if (g_dn_force >= 0 && ci != g_dn_force) continue;
    if (best < 0) { best = ci; continue; }
    const DnShape& b = kNorm[best];
    const bool mb_better = (c.mb == want_mb) != (b.mb == want_mb) ? c.mb == want_mb : false;
    if (mb_better || ((c.mb == want_mb) == (b.mb == want_mb) && c.mb == b.mb && c.nw < b.nw)) best = ci;
  }
  if (best < 0) return false;
  p.mb = kNorm[best].mb;
  p.ksw = best;  // index into kNorm
  p.ksplit = 1;
  p.mgroups = p.mbt / p.mb;
  return true;
}

// the K-split residual producer: the one-round-trip kernel's partial-sum plan (never the tiled kernels)
bool plan_resid(int64_t M, int64_t N, int64_t K, DgPlan& p) {
  if (M > g_dn_max_rows || N % 4 != 0) return false;
  const int max_ks = g_dt_max_ks;
  if (g_dr_max_ks > 0) {  // tuning: at most g_dr_max_ks slices (1 = whole K per workgroup where a shape allows)
    bool found = false;
    for (const DgShape& c : kShapes) {
      const int nks = static_cast<int>(K / 16);
      if (K % 64 != 0 || nks % (4 * c.ksw) != 0) continue;
      const int ks = nks / (4 * c.ksw);
      const int blocks = static_cast<int>((M + 31) / 32), mbt = blocks == 1 ? 1 : (blocks + 1) / 2 * 2;
      if (ks > g_dr_max_ks || c.mb > mbt || c.mb != 1) continue;
      if (!found || ks > p.ksplit) {
        p.mbt = mbt;
        p.tiles = static_cast<int>((N + 31) / 32);
        p.mb = 1;
        p.ksw = c.ksw;
        p.ksplit = ks;
        p.mgroups = mbt;
        found = true;
      }
    }
    return found;
  }
  (void)max_ks;
  return plan_decode_gemm(M, N, K, EPI_PARTIAL, p);
}

template <int EPI>
void launch_dn(const DgArgs& a, const DgPlan& p, hipStream_t s) {
  const DnShape c = kNorm[p.ksw];
  const dim3 grid(p.tiles, 1, p.mgroups);
#define DRL_DN(NW, MB, KSW) \
  hipLaunchKernelGGL((decode_norm_gemm_kernel<NW, MB, KSW, EPI>), grid, dim3(64 * NW), 0, s, a)
  switch (p.ksw) {
    case 0: DRL_DN(4, 1, 14); break;
    case 1: DRL_DN(8, 1, 7); break;
    case 2: DRL_DN(8, 2, 7); break;
    default: DRL_DN(4, 2, 7); break;
  }
#undef DRL_DN
  (void)c;
}

}  // namespace
}  // namespace drl

extern "C" {

void drl_decode_norm_set_plan(int32_t config, int32_t max_rows, int32_t resid_max_splits) {
  drl::g_dn_force = (config >= 0 && config < drl::kNumNorm) ? config : -1;
  drl::g_dn_max_rows = max_rows > 0 ? max_rows : 128;
  drl::g_dr_max_ks = resid_max_splits > 0 ? resid_max_splits : 0;
}

int drl_decode_norm_plan(int64_t M, int64_t N, int64_t K, int32_t epilogue, int32_t* ksplit, int32_t* mbt,
                         int32_t* config) {
  drl::DgPlan p{};
  bool ok;
  if (epilogue == DRL_DECODE_RESID) ok = drl::plan_resid(M, N, K, p);
  else if (epilogue == DRL_DECODE_SWIGLU) ok = drl::plan_norm(M, N, K, drl::EPI_SWIGLU, p);
  else if (epilogue == DRL_DECODE_ROPE) ok = drl::plan_norm(M, N, K, drl::EPI_ROPE, p);
  else return drl::fail(DRL_ERR_INVALID, "decode norm plan: unknown epilogue %d", epilogue);
  if (!ok)
    return drl::fail(DRL_ERR_UNSUPPORTED, "fused-norm decode: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                     (long long)N, (long long)K);
  if (ksplit) *ksplit = p.ksplit;
  if (mbt) *mbt = p.mbt;
  if (config) *config = epilogue == DRL_DECODE_RESID ? p.ksw : p.ksw;
  return DRL_OK;
}

size_t drl_decode_resid_counter_bytes(int64_t M, int64_t N, int64_t K) {
  drl::DgPlan p{};
  if (!drl::plan_resid(M, N, K, p)) return 0;
  return static_cast<size_t>(p.tiles) * p.mgroups * 4;
}

int drl_decode_gemm_resid(const void* x_packed, const void* w_packed, int64_t M, int64_t N, int64_t K, float* x_resid,
                          int64_t x_mbt, float* partials, void* counters, size_t counter_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_packed && w_packed && x_resid, "NULL input");
  DRL_CHECK_ARG(aligned16(x_packed) && aligned16(w_packed) && aligned16(x_resid), "16-byte aligned operands needed");
  DgPlan p{};
  if (!plan_resid(M, N, K, p))
    return fail(DRL_ERR_UNSUPPORTED, "decode residual GEMM: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                (long long)N, (long long)K);
  DRL_CHECK_ARG(x_mbt == p.mbt, "x_mbt %lld != the plan's %d token blocks", (long long)x_mbt, p.mbt);
  DRL_CHECK_ARG(p.ksplit == 1 || (partials && aligned16(partials) && counters &&
                                  counter_bytes >= static_cast<size_t>(p.tiles) * p.mgroups * 4),
                "K slices need the partial slabs (ksplit x M x N fp32) and zeroed counters");
  DgArgs a{};
  a.x = static_cast<const uint16_t*>(x_packed);
  a.w = static_cast<const uint16_t*>(w_packed);
  a.M = static_cast<int>(M);
  a.N = static_cast<int>(N);
  a.K = static_cast<int>(K);
  a.MBT = p.mbt;
  a.nks = static_cast<int>(K / 16);
  a.tiles = p.tiles;
  a.part = partials;
  a.xr = x_resid;
  a.cnt = static_cast<unsigned*>(counters);
  a.ksplit = p.ksplit;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p.mb == 1) launch_dg<1, EPI_RESID>(a, p, s);
  else launch_dg<2, EPI_RESID>(a, p, s);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_gemm_norm(const float* x_resid, const float* norm_weight, float eps, const void* w_packed, int64_t M,
                         int64_t N, int64_t K, void* out_packed, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_resid && norm_weight && w_packed && out_packed, "NULL input");
  DRL_CHECK_ARG(aligned16(x_resid) && aligned16(norm_weight) && aligned16(w_packed) && aligned16(out_packed),
                "16-byte aligned operands needed");
  DRL_CHECK_ARG(N % 32 == 0, "SwiGLU needs N %% 32 == 0");
  DgPlan p{};
  if (!plan_norm(M, N, K, EPI_SWIGLU, p))
    return fail(DRL_ERR_UNSUPPORTED, "decode norm + gate_up: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                (long long)N, (long long)K);
  DgArgs a{};
  a.w = static_cast<const uint16_t*>(w_packed);
  a.M = static_cast<int>(M);
  a.N = static_cast<int>(N);
  a.K = static_cast<int>(K);
  a.MBT = p.mbt;
  a.nks = static_cast<int>(K / 16);
  a.tiles = p.tiles;
  a.half = static_cast<int>(N / 2);
  a.out = static_cast<uint16_t*>(out_packed);
  a.xr = const_cast<float*>(x_resid);
  a.nw = norm_weight;
  a.eps = eps;
  launch_dn<EPI_SWIGLU>(a, p, static_cast<hipStream_t>(stream));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_qkv_rope_norm(const float* x_resid, const float* norm_weight, float eps, const void* w_packed,
                             const void* bias, const int64_t* position_ids, const float* cos_t, const float* sin_t,
                             int64_t maxpos, int64_t M, int64_t K, int64_t Hq, int64_t Hkv, int64_t D, void* q,
                             void* k_cache, void* vt_cache, int64_t Tk, int64_t ld_vt, const int64_t* koff_dev,
                             void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_resid && norm_weight && w_packed && bias && position_ids && cos_t && sin_t && q && k_cache &&
                    vt_cache && koff_dev,
                "NULL input");
  DRL_CHECK_ARG(aligned16(x_resid) && aligned16(norm_weight) && aligned16(w_packed), "16-byte aligned operands needed");
  DRL_CHECK_ARG(Hq >= 1 && Hkv >= 1 && Hq % Hkv == 0 && D % 32 == 0 && (ld_vt >= Tk || ld_vt == DRL_VT_BLOCKED) &&
                    Tk >= 1 && maxpos >= 1,
                "bad shape");
  const int64_t N = (Hq + 2 * Hkv) * D;
  DgPlan p{};
  if (!plan_norm(M, N, K, EPI_ROPE, p))
    return fail(DRL_ERR_UNSUPPORTED, "decode norm + qkv + rope: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                (long long)N, (long long)K);
  DgArgs a{};
  a.w = static_cast<const uint16_t*>(w_packed);
  a.M = static_cast<int>(M);
  a.N = static_cast<int>(N);
  a.K = static_cast<int>(K);
  a.MBT = p.mbt;
  a.nks = static_cast<int>(K / 16);
  a.tiles = p.tiles;
  a.bias = static_cast<const uint16_t*>(bias);
  a.pos = position_ids;
  a.cos_t = cos_t;
  a.sin_t = sin_t;
  a.q = static_cast<uint16_t*>(q);
  a.kc = static_cast<uint16_t*>(k_cache);
  a.vt = static_cast<uint16_t*>(vt_cache);
  a.koff_dev = koff_dev;
  a.maxpos = maxpos;
  a.Tk = Tk;
  a.ld_vt = ld_vt;
  a.Hq = static_cast<int>(Hq);
  a.Hkv = static_cast<int>(Hkv);
  a.D = static_cast<int>(D);
  a.xr = const_cast<float*>(x_resid);
  a.nw = norm_weight;
  a.eps = eps;
  launch_dn<EPI_ROPE>(a, p, static_cast<hipStream_t>(stream));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_final_norm(const float* x_resid, int64_t x_mbt, const float* weight, void* y, int64_t M, int64_t H,
                          int64_t y_mbt, float eps, void* y_packed, int64_t packed_mbt, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_resid && weight && (y || y_packed), "NULL input");
  DRL_CHECK_ARG(!y_packed || (packed_mbt >= 1 && packed_mbt * 32 >= M && aligned16(y_packed)), "packed output");
  DRL_CHECK_ARG(M >= 1 && H >= 8 && H % 8 == 0 && H <= 8 * 128 * 4, "bad shape (H %% 8 == 0, H <= 4096)");
  DRL_CHECK_ARG(x_mbt >= 1 && x_mbt * 32 >= M && (y_mbt == 0 || y_mbt * 32 >= M), "token blocks too few");
  DRL_CHECK_ARG(aligned16(x_resid) && (!y || aligned16(y)) && aligned16(weight), "16-byte aligned buffers needed");
  const int ch = static_cast<int>((H / 8 + 127) / 128);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(M));
  uint16_t* yy = static_cast<uint16_t*>(y);
  uint16_t* y2 = static_cast<uint16_t*>(y_packed);
  if (ch <= 1) hipLaunchKernelGGL((dec_rmsnorm_kernel<1, 0>), grid, dim3(128), 0, s, x_resid, nullptr, 0, nullptr, weight, yy, M, H, y_mbt, eps, x_mbt, y2, packed_mbt);
  else if (ch == 2) hipLaunchKernelGGL((dec_rmsnorm_kernel<2, 0>), grid, dim3(128), 0, s, x_resid, nullptr, 0, nullptr, weight, yy, M, H, y_mbt, eps, x_mbt, y2, packed_mbt);
  else hipLaunchKernelGGL((dec_rmsnorm_kernel<4, 0>), grid, dim3(128), 0, s, x_resid, nullptr, 0, nullptr, weight, yy, M, H, y_mbt, eps, x_mbt, y2, packed_mbt);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

void drl_decode_gemm_force_tiled(int32_t config, int32_t min_rows) {
  drl::g_dt_force = (config >= 0 && config < drl::kNumTiled) ? config : -1;
  drl::g_dt_min_rows = min_rows > 0 ? min_rows : 192;
}

void drl_decode_gemm_set_tiled(int32_t mode) { drl::g_dt_mode = (mode >= 0 && mode <= 2) ? mode : 1; }

void drl_decode_gemm_set_max_splits(int32_t ks) { drl::g_dt_max_ks = (ks >= 1 && ks <= 16) ? ks : 4; }

void drl_decode_gemm_set_plan(int32_t mb, int32_t ksw) {
  drl::g_dg_mb = (mb == 1 || mb == 2) ? mb : 0;
  drl::g_dg_ksw = ksw > 0 ? ksw : 0;
}

int drl_decode_gemm_plan(int64_t M, int64_t N, int64_t K, int32_t epilogue, int32_t* ksplit, int32_t* mbt) {
  drl::DgPlan p{};
  if (!drl::plan_any(M, N, K, epilogue == DRL_DECODE_SWIGLU ? drl::EPI_SWIGLU : drl::EPI_PARTIAL, p))
    return drl::fail(DRL_ERR_UNSUPPORTED, "decode GEMM: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                     (long long)N, (long long)K);
  if (ksplit) *ksplit = p.ksplit;
  if (mbt) *mbt = p.mbt;
  return DRL_OK;
}

size_t drl_decode_pack_weight_elems(int64_t N, int64_t K, int32_t swiglu) {
  if (N < 1 || K < 16 || K % 16) return 0;
  const int64_t tiles = swiglu ? (N / 2 + 15) / 16 : (N + 31) / 32;
  return static_cast<size_t>(tiles * (K / 16) * 512);
}

int drl_decode_pack_weight(const void* w, int64_t ld, int64_t N, int64_t K, int32_t swiglu, void* packed,
                           void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(w && packed, "NULL input");
  DRL_CHECK_ARG(N >= 1 && K >= 16 && K % 16 == 0 && ld >= K && ld % 8 == 0 && aligned16(w) && aligned16(packed),
                "bad shape / alignment");
  DRL_CHECK_ARG(!swiglu || N % 2 == 0, "SwiGLU packing needs W = [gate | up]");
  const int64_t tiles = swiglu ? (N / 2 + 15) / 16 : (N + 31) / 32;
  const int64_t n = tiles * (K / 16) * 64;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(w), ld, N, K,
                     swiglu ? N / 2 : int64_t(0), tiles, static_cast<uint16_t*>(packed));
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_gemm(const void* x_packed, const void* w_packed, int64_t M, int64_t N, int64_t K, int32_t epilogue,
                    float* partials, void* out_packed, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_packed && w_packed, "NULL input");
  DRL_CHECK_ARG(aligned16(x_packed) && aligned16(w_packed), "packed operands must be 16-byte aligned");
  const int epi = epilogue == DRL_DECODE_SWIGLU ? EPI_SWIGLU : EPI_PARTIAL;
  DRL_CHECK_ARG(epilogue == DRL_DECODE_PARTIAL || epilogue == DRL_DECODE_SWIGLU, "unknown epilogue");
  DRL_CHECK_ARG(epi == EPI_PARTIAL ? partials != nullptr : (out_packed != nullptr && aligned16(out_packed)),
                "missing output");
  DRL_CHECK_ARG(epi == EPI_PARTIAL || N % 32 == 0, "SwiGLU needs N % 32 == 0");
  DgPlan p{};
  if (!plan_any(M, N, K, epi, p))
    return fail(DRL_ERR_UNSUPPORTED, "decode GEMM: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                (long long)N, (long long)K);
  DgArgs a{static_cast<const uint16_t*>(x_packed), static_cast<const uint16_t*>(w_packed), static_cast<int>(M),
           static_cast<int>(N), static_cast<int>(K), p.mbt, static_cast<int>(K / 16), p.tiles,
           static_cast<int>(N / 2), partials, static_cast<uint16_t*>(out_packed)};
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p.mb == 0) {
    if (epi == EPI_PARTIAL) launch_dt<EPI_PARTIAL>(a, p, s);
    else launch_dt<EPI_SWIGLU>(a, p, s);
  } else if (p.mb == 1) {
    if (epi == EPI_PARTIAL) launch_dg<1, EPI_PARTIAL>(a, p, s);
    else launch_dg<1, EPI_SWIGLU>(a, p, s);
  } else {
    if (epi == EPI_PARTIAL) launch_dg<2, EPI_PARTIAL>(a, p, s);
    else launch_dg<2, EPI_SWIGLU>(a, p, s);
  }
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_pack_weight_rope(const void* w, int64_t ld, int64_t N, int64_t K, int64_t head_dim, void* packed,
                                void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(w && packed, "NULL input");
  DRL_CHECK_ARG(head_dim % 32 == 0 && head_dim >= 32 && N % head_dim == 0, "rotation-pair packing: head_dim % 32, N % head_dim");
  DRL_CHECK_ARG(K >= 16 && K % 16 == 0 && ld >= K && ld % 8 == 0 && aligned16(w) && aligned16(packed),
                "bad shape / alignment");
  const int64_t tiles = N / 32, n = tiles * (K / 16) * 64;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(w), ld, N, K, int64_t(0), tiles,
                     static_cast<uint16_t*>(packed), head_dim / 2);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_qkv_rope(const void* x_packed, const void* w_packed, const void* bias, const int64_t* position_ids,
                        const float* cos_t, const float* sin_t, int64_t maxpos, int64_t M, int64_t K, int64_t Hq,
                        int64_t Hkv, int64_t D, void* q, void* k_cache, void* vt_cache, int64_t Tk, int64_t ld_vt,
                        const int64_t* koff_dev, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_packed && w_packed && bias && position_ids && cos_t && sin_t && q && k_cache && vt_cache && koff_dev,
                "NULL input");
  DRL_CHECK_ARG(aligned16(x_packed) && aligned16(w_packed), "packed operands must be 16-byte aligned");
  DRL_CHECK_ARG(Hq >= 1 && Hkv >= 1 && Hq % Hkv == 0 && D % 32 == 0 && (ld_vt >= Tk || ld_vt == DRL_VT_BLOCKED) && Tk >= 1 && maxpos >= 1,
                "bad shape");
  const int64_t N = (Hq + 2 * Hkv) * D;
  DgPlan p{};
  if (!plan_any(M, N, K, EPI_ROPE, p))
    return fail(DRL_ERR_UNSUPPORTED, "decode qkv+rope: unsupported shape M=%lld N=%lld K=%lld", (long long)M,
                (long long)N, (long long)K);
  DgArgs a{};
  a.x = static_cast<const uint16_t*>(x_packed);
  a.w = static_cast<const uint16_t*>(w_packed);
  a.M = static_cast<int>(M);
  a.N = static_cast<int>(N);
  a.K = static_cast<int>(K);
  a.MBT = p.mbt;
  a.nks = static_cast<int>(K / 16);
  a.tiles = p.tiles;
  a.bias = static_cast<const uint16_t*>(bias);
  a.pos = position_ids;
  a.cos_t = cos_t;
  a.sin_t = sin_t;
  a.q = static_cast<uint16_t*>(q);
  a.kc = static_cast<uint16_t*>(k_cache);
  a.vt = static_cast<uint16_t*>(vt_cache);
  a.koff_dev = koff_dev;
  a.maxpos = maxpos;
  a.Tk = Tk;
  a.ld_vt = ld_vt;
  a.Hq = static_cast<int>(Hq);
  a.Hkv = static_cast<int>(Hkv);
  a.D = static_cast<int>(D);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p.mb == 0) launch_dt<EPI_ROPE>(a, p, s);
  else if (p.mb == 1) launch_dg<1, EPI_ROPE>(a, p, s);
  else launch_dg<2, EPI_ROPE>(a, p, s);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_rmsnorm(const float* x_in, const float* partials, int32_t nsplit, float* x_out, const float* weight,
                       void* y, int64_t M, int64_t H, int64_t mbt, float eps, void* y_packed, int64_t packed_mbt,
                       void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x_in && weight && y, "NULL input");
  DRL_CHECK_ARG(!y_packed || (packed_mbt >= 1 && packed_mbt * 32 >= M && aligned16(y_packed)), "packed output");
  DRL_CHECK_ARG(M >= 1 && H >= 8 && H % 8 == 0 && H <= 8 * 128 * 4, "bad shape (H %% 8 == 0, H <= 4096)");
  DRL_CHECK_ARG(partials == nullptr || nsplit >= 1, "nsplit < 1");
  DRL_CHECK_ARG(mbt == 0 || mbt * 32 >= M, "mbt too small");
  DRL_CHECK_ARG(aligned16(x_in) && aligned16(y) && aligned16(weight) && (x_out == nullptr || aligned16(x_out)) &&
                    (partials == nullptr || aligned16(partials)),
                "16-byte aligned buffers needed");
  const int ch = static_cast<int>((H / 8 + 127) / 128);
  const int ns = partials ? nsplit : 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(M));
#define DRL_DRN(C, NS) hipLaunchKernelGGL((dec_rmsnorm_kernel<C, NS>), grid, dim3(128), 0, s, x_in, partials, ns, x_out, \
                                          weight, static_cast<uint16_t*>(y), M, H, mbt, eps, int64_t(0),           \
                                          static_cast<uint16_t*>(y_packed), packed_mbt)
#define DRL_DRN_NS(C)                \
  switch (ns) {                      \
    case 0: DRL_DRN(C, 0); break;    \
    case 1: DRL_DRN(C, 1); break;    \
    case 2: DRL_DRN(C, 2); break;    \
    case 4: DRL_DRN(C, 4); break;    \
    case 7: DRL_DRN(C, 7); break;    \
    default: DRL_DRN(C, -1); break;  \
  }
  if (ch <= 1) {
    DRL_DRN_NS(1)
  } else if (ch == 2) {
    DRL_DRN_NS(2)
  } else {
    DRL_DRN(4, -1);
  }
#undef DRL_DRN_NS
#undef DRL_DRN
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_decode_rope(const float* partials, int32_t nsplit, const void* bias, const int64_t* position_ids,
                    const float* cos_t, const float* sin_t, int64_t maxpos, int64_t B, int64_t Hq, int64_t Hkv,
                    int64_t D, void* q, void* k_cache, void* v_cache, void* vt_cache, int64_t Tk, int64_t ld_vt,
                    int64_t koff, const int64_t* koff_dev, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(partials && bias && position_ids && cos_t && sin_t && q && k_cache && (v_cache || vt_cache),
                "NULL input");
  DRL_CHECK_ARG(nsplit >= 1 && B >= 1 && Hq >= 1 && Hkv >= 1 && Hq % Hkv == 0 && D % 2 == 0 && Tk >= 1, "bad shape");
  DRL_CHECK_ARG(vt_cache == nullptr || ld_vt >= Tk || ld_vt == DRL_VT_BLOCKED, "ld_vt < Tk");
  DRL_CHECK_ARG(koff_dev != nullptr || (koff >= 0 && koff < Tk), "key offset out of range");
  DecRopeArgs a{partials, nsplit, static_cast<const uint16_t*>(bias), position_ids, cos_t, sin_t,
                static_cast<uint16_t*>(q), static_cast<uint16_t*>(k_cache), static_cast<uint16_t*>(v_cache),
                static_cast<uint16_t*>(vt_cache), B, Hq, Hkv, D, Tk, ld_vt, maxpos, koff, koff_dev};
  const int64_t n = B * (Hq + 2 * Hkv) * (D / 2);
  hipLaunchKernelGGL(dec_rope_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

void drl_decode_lm_head_set_config(int32_t config) { drl::g_lm_cfg = (config >= 0 && config < 6) ? config : -1; }

int drl_decode_lm_head_plan(int64_t M, int64_t V, int64_t K, int32_t* mbt) {
  using namespace drl;
  const int cus = cu_count();
  const int64_t tiles = (V + 31) / 32;
  // 64 rows at most (the panel in LDS), K = 896 (the instantiated panel width), enough vocab tiles that every wave
  // of every workgroup owns at least one whole tile's k16 steps
  if (M < 1 || M > 64 || K != 896 || V < 32 || cus <= 0 || tiles < 16 * 8)
    return fail(DRL_ERR_UNSUPPORTED, "decode lm_head: unsupported shape M=%lld V=%lld K=%lld", (long long)M,
                (long long)V, (long long)K);
  if (mbt) *mbt = M > 32 ? 2 : 1;
  return DRL_OK;
}

int drl_decode_lm_head(const void* h_packed, int64_t mbt, const void* w_packed, int64_t M, int64_t V, int64_t K,
                       void* logits, int64_t ld, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(h_packed && w_packed && logits, "NULL input");
  int32_t want = 0;
  if (const int rc = drl_decode_lm_head_plan(M, V, K, &want); rc != DRL_OK) return rc;
  DRL_CHECK_ARG(mbt == want, "h_packed must hold %d token blocks", want);
  DRL_CHECK_ARG(aligned16(h_packed) && aligned16(w_packed) && (reinterpret_cast<uintptr_t>(logits) & 7u) == 0 &&
                    ld >= V && ld % 4 == 0,
                "alignment: packed operands 16 B, logits 8 B with ld %% 4 == 0");
  LmArgs a{static_cast<const uint16_t*>(h_packed), static_cast<const uint16_t*>(w_packed),
           static_cast<uint16_t*>(logits), ld, static_cast<int>(M), static_cast<int>(V), static_cast<int>((V + 31) / 32)};
  // (waves, ring depth) instantiated; g_lm_cfg picks one (drl_decode_lm_head_set_config, tuning)
  static constexpr int kCfg[][2] = {{8, 16}, {8, 24}, {8, 32}, {16, 8}, {4, 32}, {16, 12}};
  // measured (profiles/r06_decode_lm_head_64rows.jsonl): 8 waves x 16 loads at 64 rows, 16 waves x 8 at <= 32
  const int ci = g_lm_cfg >= 0 ? g_lm_cfg : (mbt == 1 ? 3 : 0);
  const int NWV = kCfg[ci][0];
  // workgroups: one per CU while each of the NWV waves keeps >= one whole tile of k16 steps
  const int grid = static_cast<int>(std::min<int64_t>(cu_count(), a.tiles / NWV));
  hipStream_t s = static_cast<hipStream_t>(stream);
#define DRL_LM(NW, DP)                                                                                              \
  do {                                                                                                             \
    if (mbt == 1) hipLaunchKernelGGL((decode_lm_head_kernel<1, 56, NW, DP>), dim3(grid), dim3(64 * NW), 0, s, a); \
    else hipLaunchKernelGGL((decode_lm_head_kernel<2, 56, NW, DP>), dim3(grid), dim3(64 * NW), 0, s, a);         \
  } while (0)
  switch (ci) {
    case 1: DRL_LM(8, 24); break;
    case 2: DRL_LM(8, 32); break;
    case 3: DRL_LM(16, 8); break;
    case 4: DRL_LM(4, 32); break;
    case 5: DRL_LM(16, 12); break;
    default: DRL_LM(8, 16); break;
  }
#undef DRL_LM
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

size_t drl_decode_step_prologue_workspace_bytes(void) { return 256; }

int drl_decode_step_prologue(const int64_t* responses, int64_t ld_responses, int64_t* t_dev, int64_t* t_cur,
                             const int64_t* last_pos, int64_t prompt_len, const void* embed, int32_t dt, int64_t V,
                             int64_t H, int64_t B, float* x, int64_t* positions, int64_t* kpos, uint8_t* key_valid,
                             int64_t ld_valid, void* workspace, size_t workspace_bytes, int64_t x_mbt, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(responses && t_dev && t_cur && last_pos && embed && x && positions && kpos && key_valid,
                "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "the decode step prologue reads a bf16 embedding");
  DRL_CHECK_ARG(B >= 1 && H >= 8 && H % 8 == 0 && V >= 1 && prompt_len >= 0, "bad shape (H %% 8 == 0)");
  DRL_CHECK_ARG(aligned16(embed) && aligned16(x), "embedding / x must be 16-byte aligned");
  DRL_CHECK_ARG(x_mbt == 0 || x_mbt * 32 >= B, "x_mbt too small");
  if (!workspace || workspace_bytes < drl_decode_step_prologue_workspace_bytes())
    return fail(DRL_ERR_WORKSPACE, "prologue workspace: need 256 zero-filled bytes");
  hipLaunchKernelGGL(decode_prologue_kernel, dim3(static_cast<unsigned>(B)), dim3(128), 0,
                     static_cast<hipStream_t>(stream), responses, ld_responses, t_dev, t_cur, last_pos, prompt_len,
                     static_cast<const uint16_t*>(embed), V, H, x, positions, kpos, key_valid, ld_valid,
                     static_cast<unsigned*>(workspace), x_mbt);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
