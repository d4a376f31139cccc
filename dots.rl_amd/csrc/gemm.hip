// Transformer GEMMs of the full-sequence passes (prefill, old / ref log-prob, the actor update's forward):
// y = x W^T with x (M, K) and W (N, K) both row-major bf16 (K contiguous: the MFMA-native "TN" form), fp32
// accumulation, bf16 out; replaces the hipBLASLt calls behind nn.Linear in HF Qwen2 (what the reference's
// FSDP actor runs under autocast, dp_actor.py:110 -> modeling_qwen2) with fused epilogues:
//   plain                       y = bf16(x W^T)                              (o_proj, down_proj, lm_head)
//   bias                        y = bf16(x W^T + b)                          (qkv_proj: addmm's single rounding)
//   SwiGLU (W = [gate | up])    a = bf16(bf16(silu(g)) * u), g / u = bf16 of the gate / up sums, optionally
//                               also gu = [g | u] (the backward's saved pre-activation)   (gate_up_proj)
// The SwiGLU form never writes gu when the pass keeps no activations (log-probs, prefill) and never re-reads it.
//
// Workgroup tile BM x BN x BK=64, 8 waves (WM x WN), each a (BM/WM) x (BN/WN) tile of 32 x 32 accumulator blocks
// (v_mfma_f32_32x32x16_bf16). Operand tiles are copied global -> LDS by LDS-DMA (global_load_lds_dwordx4, one
// 1-KB wave instruction = 8 rows x 128 B) through NS = 3 stage buffers with 2 stages in flight: counted vmcnt +
// raw s_barrier per k-tile, the refill of the buffer read one iteration earlier issued right after the barrier
// (cdna_hip_programming.md §5, "Pipelining across barriers"). LDS image per operand: [rows][64 k] with the 16-B
// unit u of row r stored at u ^ ((r >> 1) & 7): the 16 rows of every ds_read_b128 lane group of a 32 x 32 x 16
// fragment read land on 16 distinct 16-B bank slots (conflict-free), and the swizzle is applied on the LDS-DMA
// SOURCE address (the destination of an LDS-DMA is lane-linear). One __shared__ array.
// SwiGLU: the B tile's 32-row blocks alternate gate / up rows of the same 32 output columns, so the gate and up
// sums of an output element sit in the same lane and register of two accumulator blocks.
// Status: this one-barrier-per-k-tile form tops out at ~0.75-0.95 PFLOP/s in its main loop (the "simple
// structure" ceiling of cdna_hip_programming.md §5); gemm_pp_kernel below (256 x 256 ping-pong, two k-tiles per
// iteration in 8 phases) is the automatic choice when K % 128 == 0 and reaches 0.8-1.07 PFLOP/s
// (profiles/r02_gemm_pingpong.jsonl): at or above hipBLASLt on the model's K = 896 projections (qkv + bias,
// o_proj, gate_up + fused SwiGLU 10 % faster than hipBLASLt + the SwiGLU pass), below it on long-K shapes with
// few tiles (down_proj, the dgrad forms) and on the lm_head.
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

constexpr int EPI_NONE = 0, EPI_BIAS = 1, EPI_SWIGLU = 2;

struct GemmArgs {
  const uint16_t* a;  // (M, K), lda
  const uint16_t* b;  // (N, K), ldb   (SwiGLU: gate rows [0, I), up rows [I, 2I))
  uint16_t* c;        // (M, N) or SwiGLU (M, I), ldc
  uint16_t* c2;       // SwiGLU: optional gu (M, 2I), ldc2
  const uint16_t* bias;
  int64_t lda, ldb, ldc, ldc2;
  int M, N, K;        // SwiGLU: N = 2I (weight rows)
  int tm, tn;         // tiles along M and along the weight rows
  int gm;             // ping-pong form: M-tiles per rasterization group
};

// LDS image [rows][BK] with the 16-B unit u of row r at u ^ swz(r): conflict-free ds_read_b128 fragment reads
// (the 16 rows of each lane group hit 16 distinct 16-B bank slots) for 128-B rows (BK 64) and 64-B rows (BK 32)
template <int BK>
__device__ __forceinline__ int swz(int r) { return BK == 64 ? (r >> 1) & 7 : (r >> 2) & 3; }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else static_assert(N < 0, "vmcnt table");
}

// bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"): the workgroups the
// dispatcher places on one XCD get consecutive tile ids (row-major over (tm, tn): they share A panels in L2)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int BM, int BN, int BK, int NS, int WM, int WN, int EPI>
__global__ __launch_bounds__(512) void gemm_nt_kernel(GemmArgs g) {
  constexpr int NW = WM * WN;
  static_assert(NW == 8, "8 waves");
  constexpr int MB = BM / WM / 32, NB = BN / WN / 32;  // 32 x 32 blocks per wave
  constexpr int UPR = BK / 8, RPI = 64 / UPR;          // 16-B units per row, rows per 1-KB LDS-DMA instruction
  constexpr int A_INS = BM / RPI, B_INS = BN / RPI;    // LDS-DMA instructions per stage
  constexpr int PER_WAVE = (A_INS + B_INS) / NW;
  static_assert((A_INS + B_INS) % NW == 0, "stage copies must divide over the waves");
  static_assert(EPI != EPI_SWIGLU || NB % 2 == 0, "SwiGLU pairs gate / up blocks inside a wave");
  constexpr int STAGE = (BM + BN) * BK;  // elements
  __shared__ __attribute__((aligned(16))) uint16_t lds[NS * STAGE];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tmi = t / g.tn, tni = t % g.tn;
  const int m0 = tmi * BM, n0 = tni * BN;
  const int half = g.N / 2;

  // this wave's LDS-DMA copies: instruction q = wave + NW * c covers 8 rows (A rows first, then B rows)
  const uint16_t* src[PER_WAVE];
  int dst[PER_WAVE];
#pragma unroll
  for (int c = 0; c < PER_WAVE; ++c) {
    const int q = wave + NW * c;
    const int rr = lane / UPR, up = lane % UPR;
    if (q < A_INS) {
      const int row = RPI * q + rr;
      const int gm = min(m0 + row, g.M - 1);
      src[c] = g.a + static_cast<int64_t>(gm) * g.lda + 8 * (up ^ swz<BK>(row));
      dst[c] = RPI * q * BK + lane * 8;
    } else {
      const int row = RPI * (q - A_INS) + rr;  // B tile row
      int wrow;
      if constexpr (EPI == EPI_SWIGLU) {
        // tile row blocks alternate gate / up: block bb of the tile -> output columns (n0 / 2) + 32 (bb / 2) + i
        const int bb = row >> 5, i = row & 31;
        const int col = n0 / 2 + 32 * (bb >> 1) + i;
        wrow = (bb & 1) ? half + min(col, half - 1) : min(col, half - 1);
      } else {
        wrow = min(n0 + row, g.N - 1);
      }
      src[c] = g.b + static_cast<int64_t>(wrow) * g.ldb + 8 * (up ^ swz<BK>(row));
      dst[c] = BM * BK + RPI * (q - A_INS) * BK + lane * 8;
    }
  }
  const int nk = g.K / BK;
  auto issue = [&](int kt) {
    const int k0 = min(kt, nk - 1) * BK;  // past the end: repeat the last tile (never read)
    uint16_t* buf = lds + (kt % NS) * STAGE;
#pragma unroll
    for (int c = 0; c < PER_WAVE; ++c)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src[c] + k0),
                                       (__attribute__((address_space(3))) void*)(buf + dst[c]), 16, 0, 0);
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};

  // fragment (32 rows from R0, k16 step s) read offsets of this lane within a tile region
  const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) issue(p);
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt<(NS - 2) * PER_WAVE>();  // own copies of tile kt landed; the NS - 2 later tiles may be in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(kt + NS - 1);  // into the buffer every wave finished reading in iteration kt - 1
#ifdef DRL_GEMM_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
    const uint16_t* As = lds + (kt % NS) * STAGE;
    const uint16_t* Bs = As + BM * BK;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      u16x8 af[MB], bfr[NB];
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int row = (wm * MB + i) * 32 + fr;
        af[i] = *reinterpret_cast<const u16x8*>(As + row * BK + 8 * ((2 * s + fh) ^ swz<BK>(row)));
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int row = (wn * NB + j) * 32 + fr;
        bfr[j] = *reinterpret_cast<const u16x8*>(Bs + row * BK + 8 * ((2 * s + fh) ^ swz<BK>(row)));
      }
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(af[i]), as_bf16x8(bfr[j]), acc[i][j], 0, 0, 0);
    }
#ifdef DRL_GEMM_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef DRL_GEMM_NOSTORE
  if (acc[0][0][0] != 12345.f) return;  // timing probe: main loop only
#endif

  // epilogue: D[i][j] of a block: row i (M) = (r & 3) + 8 (r >> 2) + 4 (lane >> 5), column j (N) = lane & 31
#pragma unroll
  for (int i = 0; i < MB; ++i) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if constexpr (EPI == EPI_SWIGLU) {
        if (j & 1) continue;  // block j = gate, j + 1 = up of the same 32 output columns
        const int col = n0 / 2 + 32 * ((wn * NB + j) >> 1) + fr;
        if (col >= half) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * MB + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (m >= g.M) continue;
          const float gg = bf16r(acc[i][j][r]), uu = bf16r(acc[i][j + 1][r]);
          g.c[static_cast<int64_t>(m) * g.ldc + col] = to_bf16_bits(bf16r(silu_fast(gg)) * uu);
          if (g.c2) {
            g.c2[static_cast<int64_t>(m) * g.ldc2 + col] = to_bf16_bits(gg);
            g.c2[static_cast<int64_t>(m) * g.ldc2 + half + col] = to_bf16_bits(uu);
          }
        }
      } else {
        const int col = n0 + (wn * NB + j) * 32 + fr;
        if (col >= g.N) continue;
        const float bv = EPI == EPI_BIAS ? bf16_to_f32(g.bias[col]) : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * MB + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (m >= g.M) continue;
          g.c[static_cast<int64_t>(m) * g.ldc + col] = to_bf16_bits(acc[i][j][r] + bv);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// 256 x 256 x 64 ping-pong form (cdna_hip_programming.md §5, "The 256² 8-phase template"): the k-loop runs two
// k-tiles per iteration in 8 phases, each { ds_read one operand sub-tile | LDS-DMA one half-tile of a later
// k-tile | barrier | 16 x mfma_f32_16x16x32_bf16 on one C quadrant | barrier }, and the waves of the upper half
// (wr = 1) run one barrier behind the lower half, so while one group multiplies the other reads LDS and issues
// the copies: MFMA and memory work of the CU overlap by construction, not by occupancy.
//   LDS: 2 k-tile buffers x {A0, A1, B0, B1}, each half-tile 128 rows x 64 k (16 KB, the BK-64 swizzle above):
//   128 KB, one workgroup per CU. Wave (wr, wc) owns, in quadrant (qm, qn), tile rows qm*128 + wr*64 + [0, 64)
//   and tile columns qn*128 + wc*32 + [0, 32): every phase of every wave reads the same two half-tiles.
//   Phase order per k-tile: (A0,B0) reads B0 then A0, (A0,B1) reads B1, (A1,B1) reads A1, (A1,B0) reads nothing.
//   Copies: phase p issues half-tile h of k-tile kt (table in the loop); counted vmcnt(6) (3 half-tiles, 2
//   instructions each, in flight) at phases 3 and 7 retires the buffer the next 4 phases read, and a buffer is
//   re-staged only after the phase whose lgkmcnt retired its last reads (WAR) — the template's rules.
// SwiGLU: the B tile's 16-row blocks alternate gate / up rows of the same 16 output columns, so a wave's two
// column blocks in a half are one gate / up pair of the same lanes and registers.
template <int EPI>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs g) {
  constexpr int HT = 128 * 64, BUF = 4 * HT;  // half-tile, k-tile buffer (elements)
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];
  typedef float f32x4 __attribute__((ext_vector_type(4)));

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  // tile order: the 32 workgroups an XCD runs at once get consecutive ids (xcd_remap) and consecutive ids walk
  // groups of g.gm M-tiles column by column, so with g.gm = 4 those 32 tiles are 4 M-tiles x 8 N-tiles: 12
  // operand panels through the XCD's L2 instead of 33 (1 A panel + 32 weight panels) for a row-major walk
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = t / (g.gm * g.tn), first = grp * g.gm, gm = min(g.tm - first, g.gm), r = t % (g.gm * g.tn);
  const int m0 = (first + r % gm) * 256, n0 = (r / gm) * 256;
  const int half = g.N / 2;

  // LDS-DMA sources: half-tile h (0 A0, 1 A1, 2 B0, 3 B1), instruction c covers rows 8 (wave + 8 c) + lane / 8
  const uint16_t* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int hr = 8 * (wave + 8 * c) + (lane >> 3), up = lane & 7;
      // A half qm: tile rows qm * 128 + [0, 128); B half qn: tile columns (hr / 32) * 64 + qn * 32 + hr % 32, so
      // wave wc's columns over both halves are the contiguous wc * 64 + [0, 64) (128-B output row pieces)
      const int row = h < 2 ? (h & 1) * 128 + hr : (hr >> 5) * 64 + (h & 1) * 32 + (hr & 31);
      if (h < 2) {
        src[h][c] = g.a + static_cast<int64_t>(min(m0 + row, g.M - 1)) * g.lda + 8 * (up ^ swz<64>(hr));
      } else {
        int wrow;
        if constexpr (EPI == EPI_SWIGLU) {
          const int bb = row >> 4, col = min(n0 / 2 + 16 * (bb >> 1) + (row & 15), half - 1);
          wrow = (bb & 1) ? half + col : col;
        } else {
          wrow = min(n0 + row, g.N - 1);
        }
        src[h][c] = g.b + static_cast<int64_t>(wrow) * g.ldb + 8 * (up ^ swz<64>(hr));
      }
    }
  const int nk = g.K / 64;  // even (host check)
  auto issue = [&](int h, int kt) {
    const int k0 = min(kt, nk - 1) * 64;  // past the end: repeat the last k-tile into a buffer nobody reads again
    uint16_t* dst = lds + (kt & 1) * BUF + h * HT;
#pragma unroll
    for (int c = 0; c < 2; ++c)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src[h][c] + k0),
                                       (__attribute__((address_space(3))) void*)(dst + (wave + 8 * c) * 512 + lane * 8),
                                       16, 0, 0);
  };
  auto bar = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // nothing moves across the barrier at the IR level either
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{};
  u16x8 af[4][2], bq[2][2][2];  // A sub-tile (4 row blocks x 2 k32); B sub-tiles of both halves (2 col blocks x 2)

  const int fr = lane & 15, fq = lane >> 4;
  auto read_a = [&](const uint16_t* Ah) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + i * 16 + fr;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        af[i][kb] = *reinterpret_cast<const u16x8*>(Ah + row * 64 + 8 * ((4 * kb + fq) ^ swz<64>(row)));
    }
  };
  auto read_b = [&](const uint16_t* Bh, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wc * 32 + j * 16 + fr;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        bq[qn][j][kb] = *reinterpret_cast<const u16x8*>(Bh + row * 64 + 8 * ((4 * kb + fq) ^ swz<64>(row)));
    }
  };

  // prologue: k-tile 0 whole, k-tile 1's B0, A0, B1 (the steady state's phases 5-7 of iteration -1)
  issue(2, 0); issue(0, 0); issue(3, 0); issue(1, 0);
  issue(2, 1); issue(0, 1); issue(3, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();
  if (wr == 1) bar();  // the upper group runs one barrier behind from here on

  for (int kt = 0; kt < nk; kt += 2) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int lp = p & 3, qm = lp >> 1, qn = (lp == 1 || lp == 2) ? 1 : 0;
      const uint16_t* base = lds + (p >> 2) * BUF;
      if (lp == 0) {
        read_b(base + 2 * HT, 0);
        __builtin_amdgcn_sched_barrier(0);
        read_a(base);
      } else if (lp == 1) {
        read_b(base + 3 * HT, 1);
      } else if (lp == 2) {
        read_a(base + HT);
      }
      // copies: p0 A1(kt+1) | p1 B0 p2 A0 p3 B1 p4 A1 (kt+2) | p5 B0 p6 A0 p7 B1 (kt+3); the last pair issues
      // only p0's (nothing past the end: the wait that retires it is then vmcnt(0))
      constexpr int kH[8] = {1, 2, 0, 3, 1, 2, 0, 3};
      const bool last = kt + 2 >= nk;
      if (p == 0 || !last) issue(kH[p], kt + (p == 0 ? 1 : (p <= 4 ? 2 : 3)));
      if (lp == 0) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // the 4 B0 reads (issued first) retired
      if (p == 3) {
        if (last) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
      if (p == 7 && !last) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
            acc[qm][qn][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(af[i][kb]), as_bf16x8(bq[qn][j][kb]),
                                                                        acc[qm][qn][i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wr == 0) bar();  // balance the upper group's extra barrier
#ifdef DRL_GEMM_NOSTORE
  if (acc[0][0][0][0][0] != 12345.f) return;  // timing probe: main loop only
#endif


  // epilogue. Accumulator block (i, j) of quadrant (qm, qn): row = (lane >> 4) * 4 + r, column = lane & 15.
  // Wave rows: qm * 128 + wr * 64 + [0, 64); wave columns: wc * 64 + qn * 32 + j * 16 + [0, 16) (SwiGLU: output
  // columns wc * 32 + qn * 16 + [0, 16), j = 0 gate, 1 up).
  if constexpr (EPI == EPI_SWIGLU) {
    // through LDS as below: per row half, the wave's 64 x 32 block of a (and of g and u when gu is written),
    // row stride 40 elements (80 B: the four 4-row groups of a write on distinct banks), 3 x 5 KB per wave;
    // read back as 64-B row pieces (4 lanes x 16 B)
    constexpr int SLD = 40, REG = 64 * SLD;
    bar();  // copies drained, fragment reads retired: LDS is free
    uint16_t* st = lds + wave * 3 * REG;
    const int ch = lane & 3, col = n0 / 2 + wc * 32 + ch * 8;
    const bool vec = col + 8 <= half && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0 &&
                     (!g.c2 || ((g.ldc2 & 7) == 0 && (half & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c2) & 15) == 0));
#pragma unroll
    for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int o = (i * 16 + fq * 4 + r) * SLD + qn * 16 + fr;
            const float gg = bf16r(acc[qm][qn][i][0][r]), uu = bf16r(acc[qm][qn][i][1][r]);
            st[o] = to_bf16_bits(bf16r(silu_fast(gg)) * uu);
            if (g.c2) {
              st[REG + o] = to_bf16_bits(gg);
              st[2 * REG + o] = to_bf16_bits(uu);
            }
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int lr = it * 16 + (lane >> 2);
        const int m = m0 + qm * 128 + wr * 64 + lr;
        const int o = lr * SLD + ch * 8;
        const u16x8 va = *reinterpret_cast<const u16x8*>(st + o);
        u16x8 vg, vu;
        if (g.c2) {
          vg = *reinterpret_cast<const u16x8*>(st + REG + o);
          vu = *reinterpret_cast<const u16x8*>(st + 2 * REG + o);
        }
        if (m >= g.M || col >= half) continue;
        uint16_t* pa = g.c + static_cast<int64_t>(m) * g.ldc + col;
        uint16_t* pg = g.c2 ? g.c2 + static_cast<int64_t>(m) * g.ldc2 + col : nullptr;
        if (vec) {
          *reinterpret_cast<u16x8*>(pa) = va;
          if (pg) {
            *reinterpret_cast<u16x8*>(pg) = vg;
            *reinterpret_cast<u16x8*>(pg + half) = vu;
          }
        } else {
          for (int e = 0; e < 8 && col + e < half; ++e) {
            pa[e] = va[e];
            if (pg) {
              pg[e] = vg[e];
              pg[half + e] = vu[e];
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  } else {
    // through LDS: each wave stages its 64 x 64 bf16 block of one row half (qm) at a time (row stride 72
    // elements: the four 4-row groups of a write land on distinct banks; 8 waves x 9 KB), then stores 128-B row
    // pieces as 16-B lanes
    constexpr int SLD = 72;
    bar();  // every wave's copies drained (vmcnt(0) above) and every fragment read retired: LDS is free
    uint16_t* st = lds + wave * 64 * SLD;
    const int ch = lane & 7, col = n0 + wc * 64 + ch * 8;
    const bool vec = col + 8 <= g.N && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0;
#pragma unroll
    for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int lc = qn * 32 + j * 16 + fr;
          const float bv = EPI == EPI_BIAS ? bf16_to_f32(g.bias[min(n0 + wc * 64 + lc, g.N - 1)]) : 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              st[(i * 16 + fq * 4 + r) * SLD + lc] = to_bf16_bits(acc[qm][qn][i][j][r] + bv);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back only its own region
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int lr = it * 8 + (lane >> 3);
        const int m = m0 + qm * 128 + wr * 64 + lr;
        const u16x8 v = *reinterpret_cast<const u16x8*>(st + lr * SLD + ch * 8);
        if (m >= g.M || col >= g.N) continue;
        uint16_t* dstp = g.c + static_cast<int64_t>(m) * g.ldc + col;
        if (vec) {
          *reinterpret_cast<u16x8*>(dstp) = v;
        } else {
          for (int e = 0; e < 8 && col + e < g.N; ++e) dstp[e] = v[e];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next half's writes
    }
  }
}

int g_gemm_group = 0;  // tuning: M-tiles per rasterization group of the ping-pong form, 0 = automatic (4)

int launch_pp(GemmArgs& g, int epi, hipStream_t s) {
  g.tm = (g.M + 255) / 256;
  g.tn = (g.N + 255) / 256;
  g.gm = g_gemm_group > 0 ? g_gemm_group : 4;
  const dim3 grid(static_cast<unsigned>(g.tm * g.tn));
  if (epi == EPI_NONE) hipLaunchKernelGGL(gemm_pp_kernel<EPI_NONE>, grid, dim3(512), 0, s, g);
  else if (epi == EPI_BIAS) hipLaunchKernelGGL(gemm_pp_kernel<EPI_BIAS>, grid, dim3(512), 0, s, g);
  else hipLaunchKernelGGL(gemm_pp_kernel<EPI_SWIGLU>, grid, dim3(512), 0, s, g);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

template <int BM, int BN, int BK, int NS, int WM, int WN>
int launch(GemmArgs& g, int epi, hipStream_t s) {
  g.tm = (g.M + BM - 1) / BM;
  g.tn = (g.N + BN - 1) / BN;  // B tiles over the weight rows (SwiGLU: BN / 2 gate + BN / 2 up rows each)
  const dim3 grid(static_cast<unsigned>(g.tm * g.tn));
  if (epi == EPI_NONE) hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, BK, NS, WM, WN, EPI_NONE>), grid, dim3(512), 0, s, g);
  else if (epi == EPI_BIAS) hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, BK, NS, WM, WN, EPI_BIAS>), grid, dim3(512), 0, s, g);
  else hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, BK, NS, WM, WN, EPI_SWIGLU>), grid, dim3(512), 0, s, g);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int g_gemm_tile = 0;  // tuning: 0 = automatic, 1..9 = the configurations of drl_gemm_bf16_nt

}  // namespace
}  // namespace drl

extern "C" {

void drl_gemm_set_group(int32_t group_m) { drl::g_gemm_group = (group_m >= 1 && group_m <= 64) ? group_m : 0; }

void drl_gemm_set_tile(int32_t tile) { drl::g_gemm_tile = (tile >= 0 && tile <= 9) ? tile : 0; }

int drl_gemm_bf16_nt(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int64_t M,
                     int64_t N, int64_t K, const void* bias, int32_t epilogue, void* c2, int64_t ldc2, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(a && b && c, "NULL input");
  DRL_CHECK_ARG(M >= 1 && N >= 1 && K >= 64 && K % 64 == 0, "bad shape M=%lld N=%lld K=%lld (K %% 64 == 0)",
                (long long)M, (long long)N, (long long)K);
  DRL_CHECK_ARG(M < (1ll << 31) && N < (1ll << 31), "shape too large");
  DRL_CHECK_ARG(epilogue >= DRL_GEMM_PLAIN && epilogue <= DRL_GEMM_SWIGLU, "unknown epilogue %d", epilogue);
  DRL_CHECK_ARG(epilogue != DRL_GEMM_BIAS || bias != nullptr, "bias epilogue without bias");
  DRL_CHECK_ARG(epilogue != DRL_GEMM_SWIGLU || (N % 64 == 0), "SwiGLU: N = 2I with I %% 32 == 0");
  DRL_CHECK_ARG(aligned16(a) && aligned16(b) && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K,
                "A / B: 16-byte aligned rows with ld %% 8 == 0");
  const int64_t ncols = epilogue == DRL_GEMM_SWIGLU ? N / 2 : N;
  DRL_CHECK_ARG(ldc >= ncols && (c2 == nullptr || ldc2 >= N), "ldc");
  GemmArgs g{};
  g.a = static_cast<const uint16_t*>(a);
  g.b = static_cast<const uint16_t*>(b);
  g.c = static_cast<uint16_t*>(c);
  g.c2 = static_cast<uint16_t*>(c2);
  g.bias = static_cast<const uint16_t*>(bias);
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldc2 = ldc2;
  g.M = static_cast<int>(M); g.N = static_cast<int>(N); g.K = static_cast<int>(K);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int epi = epilogue == DRL_GEMM_PLAIN ? EPI_NONE : (epilogue == DRL_GEMM_BIAS ? EPI_BIAS : EPI_SWIGLU);
  int tile = g_gemm_tile;
  if (tile == 0) {
    // the ping-pong form wherever k-tiles pair up and the 256 x 256 grid is not tiny; else 256 x 128 unless that
    // leaves most CUs idle (narrow N at few rows): 128 x 128
    const int64_t wgs = ((M + 255) / 256) * ((N + 127) / 128);
    const int64_t wgs_pp = ((M + 255) / 256) * ((N + 255) / 256);
    tile = (K % 128 == 0 && wgs_pp >= 64) ? 9 : (wgs >= 2 * cu_count() ? 1 : 2);
  }
  switch (tile) {  // (BM, BN, BK, stages): LDS 147 / 98 / 74 / 49 / 64 KB -> 1 / 1 / 2 / 3 / 2 workgroups per CU
    case 1: return launch<256, 128, 64, 3, 4, 2>(g, epi, s);
    case 2: return launch<128, 128, 64, 3, 4, 2>(g, epi, s);
    case 3: return launch<256, 128, 32, 3, 4, 2>(g, epi, s);
    case 4: return launch<128, 128, 32, 3, 4, 2>(g, epi, s);
    // 256 x 256, 2 x 4 waves of 128 x 64 (6 fragment reads per 8 MFMAs: half the LDS traffic per FLOP of the
    // 64 x 64 wave tiles above), 128 / 128 / 96 KB of LDS
    case 6: return launch<256, 256, 64, 2, 2, 4>(g, epi, s);
    case 7: return launch<256, 256, 32, 4, 2, 4>(g, epi, s);
    case 8: return launch<256, 256, 32, 3, 2, 4>(g, epi, s);
    case 9:  // ping-pong 256 x 256 (two k-tiles per iteration)
      if (g.K % 128 == 0) return launch_pp(g, epi, s);
      return launch<256, 256, 64, 2, 2, 4>(g, epi, s);
    default: return launch<128, 128, 64, 2, 4, 2>(g, epi, s);
  }
}

}  // extern "C"
