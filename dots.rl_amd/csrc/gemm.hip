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
// Status (profiles/r02_gemm_nt_vs_hipblaslt.jsonl): correct (tests/test_gemm_gpu.py) but 1.2-1.7x slower than
// hipBLASLt on the log-prob / update shapes — this one-barrier-per-k-tile structure tops out at ~0.75-0.95
// PFLOP/s in its main loop (the "simple structure" ceiling of cdna_hip_programming.md §5), so the model keeps
// hipBLASLt for the full-sequence GEMMs; the phase-interleaved 256 x 256 schedule is the next step.
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
          g.c[static_cast<int64_t>(m) * g.ldc + col] = to_bf16_bits(bf16r(gg / (1.f + expf(-gg))) * uu);
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

int g_gemm_tile = 0;  // tuning: 0 = automatic, 1..8 = the configurations of drl_gemm_bf16_nt

}  // namespace
}  // namespace drl

extern "C" {

void drl_gemm_set_tile(int32_t tile) { drl::g_gemm_tile = (tile >= 0 && tile <= 8) ? tile : 0; }

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
    // 256 x 128 unless that leaves most CUs idle (narrow N at few rows): 128 x 128
    const int64_t wgs = ((M + 255) / 256) * ((N + 127) / 128);
    tile = wgs >= 2 * cu_count() ? 1 : 2;
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
    default: return launch<128, 128, 64, 2, 4, 2>(g, epi, s);
  }
}

}  // extern "C"
