// Every transformer GEMM of the actor's full-sequence passes on one kernel family: forward (y = x W^T), dgrad
// (dx = dy W, the weight read in its stored (out, in) layout — no transposed copy) and wgrad (dW += dy^T x, fp32
// accumulation in place), for the hipBLASLt calls behind nn.Linear's forward and autograd in HF Qwen2 / Llama under
// the reference's autocast (dp_actor.py:110, fsdp_workers.py FSDP + HF path).
//
//   C(m, n) = sum_k A(m, k) B(n, k)     A(m, k) = a[m * lda + k] (layout "K": row-major (M, K))
//                                                 a[k * lda + m] (layout "T": row-major (K, M))
//                                       B(n, k) likewise over (N, K) / (K, N)
//   forward  A = x (K),  B = W (K)                    bf16 out, + bias / SwiGLU epilogues
//   dgrad    A = dy (K), B = W (T: W is (out, in) = (K, N))   bf16 out
//   wgrad    A = dy (T), B = x (T)                    fp32 out, C (+)= acc
//
// Main loop: a 256 x 256 x (2 x 64) ping-pong (round 2's forward-only kernel, since folded in here; 8 phases per k-tile pair, upper wave group one
// barrier behind, counted vmcnt, 2 LDS buffers of 4 half-tiles), with every operand half-tile copied global -> LDS
// by buffer_load ... lds (one 1-KB wave instruction per 16-B lane): reads outside the operand's byte range return
// zeros, so row / column / k tails need no clamping (a k tail is zero in a T operand; K operands need K % 128 == 0).
// LDS images per half-tile (16 KB): layout K = [128 rows][64 k] (128-B rows, 16-B unit u of row r at u ^ ((r>>1)&7):
// conflict-free ds_read_b128 fragment reads); layout T = [64 k][128 m|n] (256-B rows, 16-B chunk c of row r at
// c ^ 2((r & 3) | ((r >> 1) & 4))), read as the MFMA operand with ds_read_b64_tr_b16 (4 k-rows x 16 columns per
// 16-lane group; the XOR puts the 8 rows a 32-lane half reads on 8 distinct 32-B bank windows: conflict-free).
//
// Work decomposition: stream-K over (tile, k-pair) iterations (cdna_hip_programming.md §5 "Decomposition first"),
// grid = at most one workgroup per CU. The first `dp_tiles` tiles are dealt whole (tile wg, wg + G, ...); the rest
// form one iteration space split into G contiguous, balanced ranges. A range's first segment that starts inside a
// tile (a "tail") stores its fp32 partial tile to the workgroup's slab write-through (sc1) and publishes a flag;
// the workgroup that holds the tile's k = 0 segment (its "head", always the LAST segment of that workgroup's range,
// so the tails it waits for were computed first) adds its own accumulator and the tails' slabs in k order — a fixed
// order, so results are bit-reproducible — and runs the epilogue. The flag is reset by its consumer: every launch
// starts and ends with the flag words zero (graph-replay safe).
//
// Co-residency (one 128-KB-LDS workgroup per CU; spinning workgroups need their partners resident):
//   stream-K (mode 1) and all-split-K (mode 3): grid <= CU count, so every workgroup is resident at once; a stream-K
//     head only waits for workgroups with a larger index, which the dispatcher started no later than itself;
//   whole tiles (mode 2) nobody waits — EXCEPT the tail split-K form: whole tiles [0, sk_base) are followed by
//     r * St split slices (r = tiles % CUs, r * St <= CU count) whose S slices spin on each other's arrival count.
//     The grid then exceeds the CU count. It is deadlock-free because (a) the dispatcher deals workgroups in index
//     order, so the slices (the highest indices) are dealt only after every whole tile has been placed, and a CU that
//     frees up takes the next slice; (b) r * St <= CUs, so once the whole tiles drain, all slices of a tile fit at
//     once; (c) no OTHER spinning launch runs concurrently on the chip — two spinning grids on two streams could each
//     hold CUs the other's slices wait for. qwen2.dgrad_wgrad enforces (c) for the concurrent dgrad / wgrad pair (at
//     most one of the two may take a spinning plan, drl_gemm_plan) and nothing else launches drl_gemm concurrently.
// A spin that exceeds 2^28 polls records 1 in the timeout word (flags + CU count, inside the workspace for every grid)
// and finishes with a wrong tile rather than hanging; tests read the word back (tests/test_gemm_sk_gpu.py).
#include "common.h"

#include <type_traits>

namespace drl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ uint16_t to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }
__device__ __forceinline__ float bf16r(float f) { return bf16_to_f32(to_bf16_bits(f)); }
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// two f32 -> packed bf16 pair (one v_cvt_pk_bf16_f32; the rounding of to_bf16_bits)
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

constexpr int EPI_NONE = 0, EPI_BIAS = 1, EPI_SWIGLU = 2, EPI_F32 = 3, EPI_SWIGLU_BWD = 4;
constexpr int HT = 128 * 64, BUF = 4 * HT;  // half-tile, k-tile buffer (elements)
constexpr int SLAB = 256 * 256;              // fp32 elements of one partial tile

struct SkArgs {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* c;         // bf16 out (M, N) or SwiGLU (M, N / 2)
  uint16_t* c2;        // SwiGLU: optional gu (M, N) written; SwiGLU backward: gu (M, 2N) read
  float* c32;          // EPI_F32 out (M, N)
  const uint16_t* bias;
  float* ws;           // stream-K slabs, gridDim.x x SLAB
  unsigned* flags;     // publish flags / split-K arrival counts (zero between launches)
  unsigned* tmo;       // the residency-timeout word: flags + CU count, a fixed index inside the workspace whatever the
                       // grid (tail split-K grids exceed the CU count), zero unless a spin-wait timed out
  int64_t lda, ldb, ldc, ldc2;
  uint32_t a_bytes, b_bytes;
  int64_t a_total;     // > 0: a layout-K A operand beyond one buffer range, its descriptor rebased per tile (a + m0 rows)
                       // (layout T: the operand's total bytes, with a_kblk)
  int a_kblk;          // > 0: a layout-T A operand beyond one buffer range (K along its rows): every tile walks its k
                       // loop in blocks of a_kblk rows (a multiple of 128), the A descriptor rebased at each block
  int M, N, K;
  int tm, tn, gm;      // tiles along M and N; M-tiles per rasterization group
  int P;               // k-tile pairs per tile
  int nkt;             // k-tiles holding data (ceil(K / 64)); a pair's second tile past it reads as zeros
  int dp_tiles;        // tiles dealt whole before the stream-K region
  int n_tiles;
  int beta;            // EPI_F32: 1 = C += acc
  int splits;          // > 1: uniform split-K, workgroup sk_base + j = split (j % splits) of tile sk_tile0 + j / splits
  int sk_base;         // split-K after whole tiles: workgroups [0, sk_base) take whole tiles 0 .. sk_base - 1 first
  int sk_tile0;        // first split tile (= sk_base; 0 for an all split-K grid)
  int sk_order;        // all-split-K grids: 1 = slice-major workgroup order (drl_gemm_set_debug bit 8; measured mixed:
                       // qkv wgrad 276 -> 264 us, o 200 -> 217, down 719 -> 726, profiles/r06_gemm_modes.jsonl)
  int dbg;             // measurement only (drl_gemm_set_debug): 1 = whole tiles skip their epilogue, 2 = the plain
                       // bf16 epilogue stages but does not store
};

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__device__ __forceinline__ int swz_k(int r) { return (r >> 1) & 7; }                 // layout K, 16-B units
__device__ __forceinline__ int swz_t(int r) { return 2 * ((r & 3) | ((r >> 1) & 4)); }  // layout T, 16-B chunks

typedef __attribute__((address_space(3))) void lds_void;

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3 of a 4 x 16 block; lane i
// of the group receives column i of the 4 rows (cdna_hip_programming.md §5.5 T10). Inline asm: hipcc's own form
// makes the compiler drain every LDS-DMA in flight (vmcnt(0)) before each read, which serialises the pipeline; the
// asm read is waited for by the schedule's own lgkmcnt, with sched_barrier(0) after it (§5.4 rule 18) and the
// 64-bit halves joined only behind that barrier.
__device__ __forceinline__ uint64_t ds_read_tr(uint32_t addr, const int off) {  // off: constant after unrolling
  uint64_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(off));
  return r;
}
__device__ __forceinline__ u16x8 join(uint64_t lo, uint64_t hi) {
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(u16x8, u64x2{lo, hi});
}

// LDS map (elements): operand region (A: 0, B: 32768) + k-tile buffer * 16384 + half * 8192, so every read of one
// operand sits within 64 KB of one base address (the DS offset field is 16 bits)
__device__ __forceinline__ constexpr int lds_half(int h, int buf) { return (h >> 1) * 32768 + buf * 16384 + (h & 1) * 8192; }

template <int EPI, int AT, int BT>
__global__ __launch_bounds__(512) void gemm_sk_kernel(SkArgs g) {
  static_assert(EPI != EPI_SWIGLU || BT == 0, "SwiGLU pairs gate / up weight rows (layout K)");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  // tail mode (whole tiles, then the last partial round's tiles split over the CUs): the whole-tile workgroups are
  // XCD-remapped among themselves; the split slices keep their launch order, so they are dispatched after every whole
  // tile and a tile's slices run side by side
  const bool tail_mode = g.splits > 1 && g.sk_base > 0;
  const int wg = (tail_mode && static_cast<int>(blockIdx.x) >= g.sk_base)
                     ? static_cast<int>(blockIdx.x)
                     : xcd_remap(blockIdx.x, tail_mode ? g.sk_base : G);
  const int half = g.N / 2;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)g.a, (short)0, (int)g.a_bytes, 0x00020000);
  uint32_t a_end = g.a_bytes;  // ra's byte range (the out-of-range soffset of a phantom k-tile)
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)g.b, (short)0, (int)g.b_bytes, 0x00020000);

  // per-lane byte offsets of this wave's two copy instructions of each half-tile h (0 A0, 1 A1, 2 B0, 3 B1) for the
  // current tile, and the byte advance of one k-tile per operand
  uint32_t voff[4][2];
  int a_kt0 = 0;  // the first k-tile of ra's range (layout-T K blocks: ra rebased per block)
  const uint32_t kstep_a = AT ? static_cast<uint32_t>(64 * g.lda * 2) : 128u;
  const uint32_t kstep_b = BT ? static_cast<uint32_t>(64 * g.ldb * 2) : 128u;

  // hn (a half-width tile: at most 128 valid columns, the last tile column of N % 256 in (0, 128]): B half 2 holds the
  // tile's 128 columns contiguously (wave wc reads columns wc * 32 ..), half 3 is never read (its copies go out of
  // range: zeros, no memory traffic)
  auto setup_tile = [&](int m0, int n0, bool hn = false) {
    int am0 = m0;  // A rows are addressed from the descriptor's base row
    if constexpr (!AT) {
      if (g.a_total > 0) {  // the tile's rows onward as their own buffer range (every offset below stays 32-bit)
        const int64_t off = static_cast<int64_t>(m0) * g.lda * 2;
        const int64_t rem = g.a_total - off;
        a_end = static_cast<uint32_t>(rem < 0x7fffffff ? rem : 0x7fffffff);
        ra = __builtin_amdgcn_make_buffer_rsrc((void*)(reinterpret_cast<const char*>(g.a) + off), (short)0, (int)a_end,
                                               0x00020000);
        am0 = 0;
      }
    }
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int q = wave + 8 * c;
        const bool is_a = h < 2;
        const bool tr = is_a ? AT : BT;
        if (!tr) {
          const int hr = 8 * q + (lane >> 3), up = lane & 7;
          int grow;
          if (is_a) {
            grow = am0 + (h & 1) * 128 + hr;
          } else if constexpr (EPI == EPI_SWIGLU) {
            // tile row blocks of 16 alternate gate / up rows of the same 16 output columns
            const int row = (hr >> 5) * 64 + (h & 1) * 32 + (hr & 31);
            const int bb = row >> 4, col = min(n0 / 2 + 16 * (bb >> 1) + (row & 15), half - 1);
            grow = (bb & 1) ? half + col : col;
          } else {
            grow = hn ? n0 + hr : n0 + (hr >> 5) * 64 + (h & 1) * 32 + (hr & 31);
          }
          const int64_t ld = is_a ? g.lda : g.ldb;
          voff[h][c] = static_cast<uint32_t>((static_cast<int64_t>(grow) * ld + 8 * (up ^ swz_k(hr))) * 2);
        } else {
          const int row = 4 * q + (lane >> 4), ch = (lane & 15) ^ swz_t(row);
          const int col = is_a ? m0 + (h & 1) * 128 + 8 * ch
                               : (hn ? n0 + 8 * ch : n0 + (ch >> 2) * 64 + (h & 1) * 32 + (ch & 3) * 8);
          const int64_t ld = is_a ? g.lda : g.ldb;
          voff[h][c] = static_cast<uint32_t>((static_cast<int64_t>(row) * ld + col) * 2);
        }
      }
  };
  // buf = kt & 1, passed as a constant of the unrolled schedule (segments start at even k-tiles)
  auto issue = [&](int h, int buf, int kt, int kt_end, bool hn = false) {
    // past the segment's end: repeat its last k-tile into a buffer nobody reads again (keeps vmcnt counts static)
    const int k = min(kt, kt_end - 1);
    uint16_t* dst = lds + lds_half(h, buf);
    const bool is_a = h < 2;
    // k-tile past the data (K % 128 == 64), or B half 3 of a half-width tile: an soffset of the whole byte range puts
    // every lane out of range (zeros)
    const uint32_t soff = (k >= g.nkt || (hn && h == 3))
                              ? (is_a ? a_end : g.b_bytes)
                              : static_cast<uint32_t>(is_a ? k - a_kt0 : k) * (is_a ? kstep_a : kstep_b);
#pragma unroll
    for (int c = 0; c < 2; ++c)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(is_a ? ra : rb, (lds_void*)(dst + (wave + 8 * c) * 512 + lane * 8), 16,
                                               voff[h][c], soff, 0, 0);
  };
  auto bar = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4 acc[2][2][4][2];
  u16x8 af[4][2], bq[2][2][2];  // layout-K fragments
  uint64_t at[4][2][2], bt[2][2][2][2];  // layout-T fragment halves (i|j, kb, h2), joined at the MFMA

  // fragment reads. Layout K: one ds_read_b128 (rows fr, k 8 fq .. 8 fq + 7 of a 32-deep k block). Layout T: two
  // transposed reads (k rows 8 fq + 4 h2 + [0, 4)), lane 4q+p addressing row q, columns 4p .. 4p + 3.
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const int tsw = 2 * (tq | 4 * (fq & 1));  // swz_t of every row this lane addresses
  const uint32_t lds32 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) uint16_t*)lds));
  auto tr_addr = [&](int region, int col0) {  // byte address of (row 8 fq + tq, 16-column block col0) of a T image
    const int chunk = (col0 >> 3) + (tp >> 1);
    return lds32 + 2 * (region + (8 * fq + tq) * 128 + 8 * (chunk ^ tsw) + 4 * (tp & 1));
  };
  uint32_t ta[4], tb[2];
  if constexpr (AT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ta[i] = tr_addr(0, wr * 64 + i * 16);
  }
  if constexpr (BT) {
#pragma unroll
    for (int j = 0; j < 2; ++j) tb[j] = tr_addr(32768, wc * 32 + j * 16);
  }
  // half-tile h of k-tile buffer `buf` (compile-time after unrolling)
  auto read_a = [&](int buf, int h) {
    const uint16_t* Ah = lds + lds_half(h, buf);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (!AT) {
        const int row = wr * 64 + i * 16 + fr;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          af[i][kb] = *reinterpret_cast<const u16x8*>(Ah + row * 64 + 8 * ((4 * kb + fq) ^ swz_k(row)));
      } else {
#define DRL_TRA(KB, H2) at[i][KB][H2] = ds_read_tr(ta[i], 2 * (lds_half(h, buf) + KB * 32 * 128 + H2 * 4 * 128))
        DRL_TRA(0, 0); DRL_TRA(0, 1); DRL_TRA(1, 0); DRL_TRA(1, 1);
#undef DRL_TRA
      }
    }
  };
  auto read_b = [&](int buf, int h, int qn) {
    const uint16_t* Bh = lds + lds_half(h, buf);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (!BT) {
        const int row = wc * 32 + j * 16 + fr;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          bq[qn][j][kb] = *reinterpret_cast<const u16x8*>(Bh + row * 64 + 8 * ((4 * kb + fq) ^ swz_k(row)));
      } else {
#define DRL_TRB(KB, H2) \
  bt[qn][j][KB][H2] = ds_read_tr(tb[j], 2 * (lds_half(h, buf) - 32768 + KB * 32 * 128 + H2 * 4 * 128))
        DRL_TRB(0, 0); DRL_TRB(0, 1); DRL_TRB(1, 0); DRL_TRB(1, 1);
#undef DRL_TRB
      }
    }
  };
  constexpr int NB_READS = BT ? 8 : 4;   // LDS instructions of one B sub-tile read
  constexpr int NA_READS = AT ? 16 : 8;  // of one A sub-tile read

  // one segment: k-tile pairs [p0, p1) of the current tile accumulated into acc (zeroed first unless keep)
  // hn (uniform): a half-width tile — the quadrants qn = 1 hold no columns, so their MFMAs are skipped by a scalar
  // branch (those phases keep their copies and barriers: the schedule's vmcnt counts and the wave groups'
  // pairing stay as they are; one instance of the loop — a second, compile-time instance spilled 120-340 registers)
  auto run = [&](int p0, int p1, bool keep, bool hn) __attribute__((always_inline)) {
    if (!keep) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{};
    }
    const int k0 = 2 * p0, k1 = 2 * p1;  // k-tiles [k0, k1)
    issue(2, 0, k0, k1, hn); issue(0, 0, k0, k1, hn); issue(3, 0, k0, k1, hn); issue(1, 0, k0, k1, hn);
    issue(2, 1, k0 + 1, k1, hn); issue(0, 1, k0 + 1, k1, hn); issue(3, 1, k0 + 1, k1, hn);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    bar();
    if (wr == 1) bar();  // the upper group runs one barrier behind
    for (int kt = k0; kt < k1; kt += 2) {
      const bool last = kt + 2 >= k1;
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int lp = p & 3, qm = lp >> 1, qn = (lp == 1 || lp == 2) ? 1 : 0;
        const int buf = p >> 2;
        if (lp == 0) {
          read_b(buf, 2, 0);
          __builtin_amdgcn_sched_barrier(0);
          read_a(buf, 0);
        } else if (lp == 1) {
          read_b(buf, 3, 1);  // also for a half-width tile (unread there): a conditional read kept bq[1] live across
                              // the loop (16 registers spilled)
        } else if (lp == 2) {
          read_a(buf, 1);
        }
        constexpr int kH[8] = {1, 2, 0, 3, 1, 2, 0, 3};
        constexpr int kD[8] = {1, 2, 2, 2, 2, 3, 3, 3};
        if (p == 0 || !last) issue(kH[p], kD[p] & 1, kt + kD[p], k1, hn);
        if (lp == 0) {  // the B0 reads (issued first) retired before the barrier (WAR of the next copies)
          if constexpr (NA_READS >= 15) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
          else if constexpr (NA_READS == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        }
        if (p == 3) {
          if (last) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        }
        if (p == 7 && !last) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        bar();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // nothing that uses an asm read's result moves above its wait
        __builtin_amdgcn_s_setprio(1);
        if (!(hn && qn == 1))
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
              const u16x8 fa = AT ? join(at[i][kb][0], at[i][kb][1]) : af[i][kb];
              const u16x8 fb = BT ? join(bt[qn][j][kb][0], bt[qn][j][kb][1]) : bq[qn][j][kb];
              // operands swapped: the 16 x 16 block is accumulated transposed, so lane (fq, fr) holds output row
              // fr, columns 4 fq .. 4 fq + 3 — the epilogue stores straight from registers
              acc[qm][qn][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(fb), as_bf16x8(fa),
                                                                          acc[qm][qn][i][j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
        bar();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wr == 0) bar();  // balance the upper group's extra barrier
  };
  (void)NB_READS;
  // k-pairs [p0, p1) of the current tile; a layout-T A operand past one buffer range is walked in blocks of a_kblk
  // rows, the descriptor rebased at each (one launch, the fp32 output read and written once — the round-5 host loop
  // launched one GEMM per block, each a read-modify-write of the whole output)
  auto run_k = [&](int p0, int p1, bool hn) __attribute__((always_inline)) {
    const bool blk = AT && g.a_kblk > 0;
    const int bp = blk ? g.a_kblk / 128 : max(p1, 1);  // k-pairs per block (one block without K blocking)
    bool keep = false;
    for (int q0 = blk ? (p0 / bp) * bp : p0; q0 < p1; q0 += bp) {
      const int lo = max(p0, q0), hi = min(p1, q0 + bp);
      if constexpr (AT) {
        if (blk) {
          const int64_t off = static_cast<int64_t>(q0) * 128 * g.lda * 2;
          const int64_t rem = g.a_total - off;
          a_end = static_cast<uint32_t>(rem < 0x7fffffff ? rem : 0x7fffffff);
          ra = __builtin_amdgcn_make_buffer_rsrc((void*)(reinterpret_cast<const char*>(g.a) + off), (short)0,
                                                 (int)a_end, 0x00020000);
          a_kt0 = 2 * q0;
        }
      }
      run(lo, hi, keep, hn);
      keep = true;
    }
  };

  // ------------------------------------------------------------------------------------------ epilogues
  // accumulator block (i, j) of quadrant (qm, qn), transposed (the MFMA's operands are swapped): lane (fq, fr) holds
  // tile row qm * 128 + wr * 64 + i * 16 + fr, tile columns wc * 64 + qn * 32 + j * 16 + 4 fq + (0..3) (SwiGLU: output
  // columns wc * 32 + qn * 16 + 4 fq + (0..3), j = 0 gate, 1 up). Staged through LDS as one 8-B (bf16) / 16-B (fp32)
  // write per block and lane — a quarter of the 2-byte writes the untransposed layout needs (that staging cost
  // 3.7 us per 256 x 256 tile, profiles/r03_gemm_fixed_cost.jsonl) — then read back as 16-B row pieces for coalesced
  // 128-B row stores (storing the 8-B pieces straight from the registers, 16 rows x 32 B per wave instruction,
  // measured 3x slower).
  // HALF: a half-width tile (setup_tile's hn): accumulator block (i, j) of quadrant (qm, 0) holds tile columns
  // wc * 32 + j * 16 + 4 fq + (0..3); the quadrants qn = 1 hold nothing
  auto epilogue = [&](int m0, int n0, auto half_tag) {
    constexpr bool HALF = decltype(half_tag)::value;
    bar();  // every fragment read retired and every copy drained: LDS is free for staging
    if (g.dbg & 4) {  // measurement: the epilogue's two barriers only
      bar();
      return;
    }
    if constexpr (EPI == EPI_F32) {
      // per quadrant: the wave's 64 x 32 fp32 block (row stride 36 floats), read back as 16-B row pieces (8 lanes per
      // 128-B row) for a coalesced read-modify-write of the fp32 output
      constexpr int SLD = 36;
      float* st = reinterpret_cast<float*>(lds) + wave * 64 * SLD;
      const int ch = lane & 7;
      const bool vec = (g.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(g.c32) & 15) == 0;
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int qn = 0; qn < 2; ++qn) {
          if (HALF && qn == 1) continue;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              *reinterpret_cast<f32x4*>(st + (i * 16 + fr) * SLD + j * 16 + 4 * fq) = acc[qm][qn][i][j];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const int col = HALF ? n0 + wc * 32 + 4 * ch : n0 + wc * 64 + qn * 32 + 4 * ch;
#pragma unroll
          for (int it = 0; it < 8; ++it) {
            const int lr = it * 8 + (lane >> 3);
            const int m = m0 + qm * 128 + wr * 64 + lr;
            const f32x4 v = *reinterpret_cast<const f32x4*>(st + lr * SLD + 4 * ch);
            if (m >= g.M || col >= g.N) continue;
            float* p = g.c32 + static_cast<int64_t>(m) * g.ldc + col;
            if (vec && col + 4 <= g.N) {
              *reinterpret_cast<f32x4*>(p) = g.beta ? *reinterpret_cast<const f32x4*>(p) + v : v;
            } else {
              for (int e = 0; e < 4 && col + e < g.N; ++e) p[e] = g.beta ? p[e] + v[e] : v[e];
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next quadrant's writes
        }
    } else if constexpr (EPI == EPI_SWIGLU) {
      constexpr int SLD = 40, REG = 64 * SLD;
      uint16_t* st = lds + wave * 3 * REG;
      const int ch = lane & 3, col = n0 / 2 + wc * 32 + ch * 8;
      const bool vec = col + 8 <= half && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0 &&
                       (!g.c2 || ((g.ldc2 & 7) == 0 && (half & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c2) & 15) == 0));
      const bool interior = m0 + 256 <= g.M && n0 / 2 + 128 <= half && (g.ldc & 7) == 0 &&
                            (reinterpret_cast<uintptr_t>(g.c) & 15) == 0 &&
                            (!g.c2 || ((g.ldc2 & 7) == 0 && (half & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c2) & 15) == 0));
#pragma unroll
      for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int o = (i * 16 + fr) * SLD + qn * 16 + 4 * fq;
            u16x4 a4, g4, u4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gg = bf16r(acc[qm][qn][i][0][r]), uu = bf16r(acc[qm][qn][i][1][r]);
              a4[r] = to_bf16_bits(bf16r(silu_fast(gg)) * uu);
              g4[r] = to_bf16_bits(gg);
              u4[r] = to_bf16_bits(uu);
            }
            *reinterpret_cast<u16x4*>(st + o) = a4;
            if (g.c2) {
              *reinterpret_cast<u16x4*>(st + REG + o) = g4;
              *reinterpret_cast<u16x4*>(st + 2 * REG + o) = u4;
            }
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (interior) {  // whole tile inside (uniform): one row base per output, rows 16 apart, no per-row tests
          const int64_t m = m0 + qm * 128 + wr * 64 + (lane >> 2);
          uint16_t* pa = g.c + m * g.ldc + col;
          uint16_t* pg = g.c2 ? g.c2 + m * g.ldc2 + col : nullptr;
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int o = (it * 16 + (lane >> 2)) * SLD + ch * 8;
            *reinterpret_cast<u16x8*>(pa + it * 16 * g.ldc) = *reinterpret_cast<const u16x8*>(st + o);
            if (pg) {
              *reinterpret_cast<u16x8*>(pg + it * 16 * g.ldc2) = *reinterpret_cast<const u16x8*>(st + REG + o);
              *reinterpret_cast<u16x8*>(pg + it * 16 * g.ldc2 + half) = *reinterpret_cast<const u16x8*>(st + 2 * REG + o);
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          continue;
        }
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
      constexpr int SLD = 72;
      uint16_t* st = lds + wave * 64 * SLD;
      const int ch = lane & 7, col = n0 + wc * 64 + ch * 8;
      const bool vec = col + 8 <= g.N && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0 &&
                       (EPI != EPI_SWIGLU_BWD || ((g.ldc2 & 7) == 0 && (g.N & 7) == 0 &&
                                                  (reinterpret_cast<uintptr_t>(g.c2) & 15) == 0));
      const bool interior = m0 + 256 <= g.M && n0 + 256 <= g.N && (g.ldc & 7) == 0 &&
                            (reinterpret_cast<uintptr_t>(g.c) & 15) == 0;
      if constexpr (EPI == EPI_SWIGLU_BWD) {
        // the down_proj dgrad fused with the SwiGLU backward. Per quadrant: stage bf16(d a) through LDS, then read
        // the saved gate / up of the same columns and write dgu. Lambdas called with constants (not loops): the
        // accumulator indices stay static (a loop here left them in scratch).
        auto stage = [&](const int qm) __attribute__((always_inline)) {
#pragma unroll
            for (int qn = 0; qn < 2; ++qn)
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const int lc = qn * 32 + j * 16 + 4 * fq;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const f32x4 v = acc[qm][qn][i][j];
                  uint2 w;
                  w.x = pk_bf16(v[0], v[1]);
                  w.y = pk_bf16(v[2], v[3]);
                  *reinterpret_cast<uint2*>(st + (i * 16 + fr) * SLD + lc) = w;
                }
              }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        };
        // whole tile inside (uniform): the 8 row pieces' gate / up loads go out in two batches of 4 (8 x 16 B in
        // flight per lane, one row base per operand) instead of 2 loads behind each row's bounds test
        auto fast = [&](const int qm) __attribute__((always_inline)) {
            const int64_t m = m0 + qm * 128 + wr * 64 + (lane >> 3);
            const uint16_t* gp = g.c2 + m * g.ldc2 + col;
            uint16_t* dp = g.c + m * g.ldc + col;
            const int64_t sg = 8 * g.ldc2, sd = 8 * g.ldc;
            auto one = [&](int it, u32x4 gw, u32x4 uw) __attribute__((always_inline)) {
              const u16x8 v = *reinterpret_cast<const u16x8*>(st + (it * 8 + (lane >> 3)) * SLD + ch * 8);
              const u16x8 gv = __builtin_bit_cast(u16x8, gw), uv = __builtin_bit_cast(u16x8, uw);
              u16x8 dg, du;
#pragma unroll
              for (int e = 0; e < 8; ++e) {  // swiglu_bwd's math and roundings (as the row path below)
                const float d = bf16_to_f32(v[e]), gg = bf16_to_f32(gv[e]), uu = bf16_to_f32(uv[e]);
                const float sig = sigmoid_fast(gg);
                dg[e] = to_bf16_bits(bf16r(d * uu) * (sig * (1.f + gg * (1.f - sig))));
                du[e] = to_bf16_bits(d * bf16r(gg * sig));
              }
              *reinterpret_cast<u16x8*>(dp + it * sd) = dg;
              *reinterpret_cast<u16x8*>(dp + it * sd + g.N) = du;
            };
#pragma unroll
            for (int hb = 0; hb < 2; ++hb) {
              const u32x4 g0 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 0) * sg);
              const u32x4 u0 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 0) * sg + g.N);
              const u32x4 g1 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 1) * sg);
              const u32x4 u1 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 1) * sg + g.N);
              const u32x4 g2 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 2) * sg);
              const u32x4 u2 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 2) * sg + g.N);
              const u32x4 g3 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 3) * sg);
              const u32x4 u3 = *reinterpret_cast<const u32x4*>(gp + (4 * hb + 3) * sg + g.N);
              one(4 * hb + 0, g0, u0);
              one(4 * hb + 1, g1, u1);
              one(4 * hb + 2, g2, u2);
              one(4 * hb + 3, g3, u3);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        };
        // any tile: row by row with bounds tests
        auto rows = [&](const int qm) __attribute__((always_inline)) {
#pragma unroll
          for (int it = 0; it < 8; ++it) {
            const int lr = it * 8 + (lane >> 3);
            const int m = m0 + qm * 128 + wr * 64 + lr;
            const u16x8 v = *reinterpret_cast<const u16x8*>(st + lr * SLD + ch * 8);
            if (m >= g.M || col >= g.N) continue;
            uint16_t* dstp = g.c + static_cast<int64_t>(m) * g.ldc + col;
            // v = bf16(d a) of columns col..col+7; gate / up of the same columns from the saved gu row -> dgu
            // (swiglu_bwd's math and roundings: dg = bf16(d*u) * sig (1 + g (1 - sig)), du = d * bf16(g sig))
            const uint16_t* gp = g.c2 + static_cast<int64_t>(m) * g.ldc2 + col;
            u16x8 gq, uq;
            if (vec) {
              gq = *reinterpret_cast<const u16x8*>(gp);
              uq = *reinterpret_cast<const u16x8*>(gp + g.N);
            } else {
              for (int e = 0; e < 8; ++e) {
                gq[e] = col + e < g.N ? gp[e] : 0;
                uq[e] = col + e < g.N ? gp[g.N + e] : 0;
              }
            }
            u16x8 dg, du;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = bf16_to_f32(v[e]), gg = bf16_to_f32(gq[e]), uu = bf16_to_f32(uq[e]);
              const float sig = sigmoid_fast(gg);
              dg[e] = to_bf16_bits(bf16r(d * uu) * (sig * (1.f + gg * (1.f - sig))));
              du[e] = to_bf16_bits(d * bf16r(gg * sig));
            }
            if (vec) {
              *reinterpret_cast<u16x8*>(dstp) = dg;
              *reinterpret_cast<u16x8*>(dstp + g.N) = du;
            } else {
              for (int e = 0; e < 8 && col + e < g.N; ++e) {
                dstp[e] = dg[e];
                dstp[g.N + e] = du[e];
              }
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        };
        const bool whole = interior && vec;
        stage(0);
        if (whole) fast(0);
        else rows(0);
        stage(1);
        if (whole) fast(1);
        else rows(1);
      } else if constexpr (HALF) {
        // half-width tile: per quadrant the wave's 64 x 32 block, stored as 4 16-B pieces per 64-B row
        const int c4 = lane & 3, colh = n0 + wc * 32 + c4 * 8;
        const bool vech = colh + 8 <= g.N && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int lc = j * 16 + 4 * fq;
            float bb[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (EPI == EPI_BIAS) {
#pragma unroll
              for (int e = 0; e < 4; ++e) bb[e] = bf16_to_f32(g.bias[min(n0 + wc * 32 + lc + e, g.N - 1)]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const f32x4 v = acc[qm][0][i][j];
              uint2 w;
              if constexpr (EPI == EPI_BIAS) {
                w.x = pk_bf16(v[0] + bb[0], v[1] + bb[1]);
                w.y = pk_bf16(v[2] + bb[2], v[3] + bb[3]);
              } else {
                w.x = pk_bf16(v[0], v[1]);
                w.y = pk_bf16(v[2], v[3]);
              }
              *reinterpret_cast<uint2*>(st + (i * 16 + fr) * SLD + lc) = w;
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int lr = it * 16 + (lane >> 2);
            const int m = m0 + qm * 128 + wr * 64 + lr;
            const u16x8 v = *reinterpret_cast<const u16x8*>(st + lr * SLD + c4 * 8);
            if (m >= g.M || colh >= g.N) continue;
            uint16_t* dstp = g.c + static_cast<int64_t>(m) * g.ldc + colh;
            if (vech) {
              *reinterpret_cast<u16x8*>(dstp) = v;
            } else {
              for (int e = 0; e < 8 && colh + e < g.N; ++e) dstp[e] = v[e];
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      } else {
#pragma unroll
      for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int lc = qn * 32 + j * 16 + 4 * fq;
            float bb[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (EPI == EPI_BIAS) {
#pragma unroll
              for (int e = 0; e < 4; ++e) bb[e] = bf16_to_f32(g.bias[min(n0 + wc * 64 + lc + e, g.N - 1)]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const f32x4 v = acc[qm][qn][i][j];
              // two v_cvt_pk_bf16_f32 per block (no bias: no +0.0 adds, which the compiler must keep for -0.0)
              uint2 w;
              if constexpr (EPI == EPI_BIAS) {
                w.x = pk_bf16(v[0] + bb[0], v[1] + bb[1]);
                w.y = pk_bf16(v[2] + bb[2], v[3] + bb[3]);
              } else {
                w.x = pk_bf16(v[0], v[1]);
                w.y = pk_bf16(v[2], v[3]);
              }
              *reinterpret_cast<uint2*>(st + (i * 16 + fr) * SLD + lc) = w;
            }
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (EPI != EPI_SWIGLU_BWD && interior && !(g.dbg & 2)) {
          // whole tile inside C (uniform): one row base, rows 8 apart, no per-row tests
          uint16_t* dst = g.c + static_cast<int64_t>(m0 + qm * 128 + wr * 64 + (lane >> 3)) * g.ldc + col;
          const int64_t step = 8 * g.ldc;
#pragma unroll
          for (int it = 0; it < 8; ++it)
            *reinterpret_cast<u16x8*>(dst + it * step) =
                *reinterpret_cast<const u16x8*>(st + (it * 8 + (lane >> 3)) * SLD + ch * 8);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          continue;
        }
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int lr = it * 8 + (lane >> 3);
          const int m = m0 + qm * 128 + wr * 64 + lr;
          const u16x8 v = *reinterpret_cast<const u16x8*>(st + lr * SLD + ch * 8);
          if (m >= g.M || col >= g.N) continue;
          uint16_t* dstp = g.c + static_cast<int64_t>(m) * g.ldc + col;
          if (g.dbg & 2) {  // measurement: staging without the output stores
            if (v[0] == 0x7fffu && v[1] == 0x1234u) dstp[0] = 0;
          } else if (vec) {
            *reinterpret_cast<u16x8*>(dstp) = v;
          } else {
            for (int e = 0; e < 8 && col + e < g.N; ++e) dstp[e] = v[e];
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      }
    }
    bar();  // staging reads done before the next segment's copies land in LDS
  };

  auto tile_origin = [&](int t, int& m0, int& n0) {
    const int grp = t / (g.gm * g.tn), first = grp * g.gm, gm = min(g.tm - first, g.gm), r = t % (g.gm * g.tn);
    m0 = (first + r % gm) * 256;
    n0 = (r / gm) * 256;
  };

  typedef __attribute__((address_space(1))) unsigned gflag;
  // ------------------------------------------------------------------------------------------ uniform split-K
  // Few tiles, long K (the weight gradients of the small projections, down_proj, the N = H dgrads, the lm_head
  // dgrad): the S workgroups of a tile each accumulate a k-pair range, publish it (sc1 slab + arrival count), wait for
  // all S arrivals, then each reduces 1/S of the tile's registers over the S slabs in split order (a fixed order:
  // bit-reproducible) and writes that share through the epilogue — the combine runs on all S workgroups at once.
  if (g.splits > 1 && wg >= g.sk_base) {
    // slice order: tile-major (a tile's S slices on consecutive workgroups) or, with sk_order (all-split-K grids
    // only), slice-major — the same k-range of every tile on consecutive workgroups, which the XCD remap places on
    // one XCD at once, so tiles of one row / column read the same k window of A / B through the shared L2. The slab of
    // (tile ti, slice s) sits at index s * nt + ti, the combine reads them in split order either way (same bits).
    const int S = g.splits, rel = wg - g.sk_base, nt = (G - g.sk_base) / S;
    const bool smaj = g.sk_order && g.sk_base == 0;
    const int ti = smaj ? rel % nt : rel / S, t = g.sk_tile0 + ti, sp = smaj ? rel / nt : rel - ti * S;
    const int slab_tile = smaj ? ti : ti * S, slab_step = smaj ? nt : 1;  // slab of (ti, s) = slab_tile + s * step
    int m0, n0;
    {
      const int grp = t / (g.gm * g.tn), first = grp * g.gm, gmm = min(g.tm - first, g.gm), r = t % (g.gm * g.tn);
      m0 = (first + r % gmm) * 256;
      n0 = (r / gmm) * 256;
    }
    setup_tile(m0, n0);
    run_k(sp * g.P / S, (sp + 1) * g.P / S, false);
    const __amdgpu_buffer_rsrc_t rws =
        __builtin_amdgcn_make_buffer_rsrc((void*)g.ws, (short)0, (G - g.sk_base) * SLAB * 4, 0x00020000);
    const uint32_t vo = static_cast<uint32_t>(slab_tile + sp * slab_step) * SLAB * 4 + threadIdx.x * 16;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][b][i][j]), rws, vo,
                                                   (((a * 2 + b) * 4 + i) * 2 + j) * 8192, 16 /* sc1 */);
    // arrival: every storing wave drains its sc1 stores, the barrier, ONE lane's agent-scope add; then ONE lane polls
    // the count (sc1 loads) until all S slices arrived (MI355X_MICROARCH.md § visibility, first row of the sc1 table)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    gflag* cnt = (gflag*)(g.flags + ti);
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < static_cast<unsigned>(S)) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 28)) {  // residency violated: record it and finish (wrong tile) instead of hanging
          __hip_atomic_store((gflag*)g.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the barrier
    // this slice's share of the tile: register groups [32 sp / S, 32 (sp + 1) / S)
    const int r0 = 32 * sp / S, r1 = 32 * (sp + 1) / S;
    const uint32_t vt = static_cast<uint32_t>(slab_tile) * SLAB * 4 + threadIdx.x * 16;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int reg = ((a * 2 + b) * 4 + i) * 2 + j;
            if (reg < r0 || reg >= r1) continue;
            f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rws, vt, reg * 8192, 16));
            for (int s2 = 1; s2 < S; ++s2)
              v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rws, vt + s2 * slab_step * SLAB * 4,
                                                                                   reg * 8192, 16));
            // transposed block (see the epilogue): row fr, columns 4 fq + r
            const int m = m0 + a * 128 + wr * 64 + i * 16 + fr;
            if (m >= g.M) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int col = n0 + wc * 64 + b * 32 + j * 16 + 4 * fq + r;
              if (col >= g.N) continue;
              if constexpr (EPI == EPI_F32) {
                float* p = g.c32 + static_cast<int64_t>(m) * g.ldc + col;
                *p = g.beta ? *p + v[r] : v[r];
              } else if constexpr (EPI != EPI_SWIGLU && EPI != EPI_SWIGLU_BWD) {
                const float bv = EPI == EPI_BIAS ? bf16_to_f32(g.bias[col]) : 0.f;
                g.c[static_cast<int64_t>(m) * g.ldc + col] = to_bf16_bits(v[r] + bv);
              }
            }
          }
    // departure: the last of the S slices to finish reading resets the count (every launch ends with it at zero)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == static_cast<unsigned>(2 * S - 1)) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  // ------------------------------------------------------------------------------------------ whole tiles
  // a half-width tile (the last tile column of N % 256 in (0, 128]: the N = 896 / 1152 outputs): half the MFMAs
  // (plain / fp32 epilogues; drl_gemm_set_debug bit 32 turns it off). Layout-T B only (the input and weight
  // gradients): in the layout-K B kernels (the forwards) the extra path cost registers (11 -> 38 spilled) and their
  // whole launch 2-8 % (profiles/r06_gemm_half_tile_ab.txt), more than the skipped MFMAs give back
  constexpr bool kHalfOk = (EPI == EPI_NONE || EPI == EPI_BIAS || EPI == EPI_F32) && BT == 1;
  for (int t = wg; t < g.dp_tiles; t += G) {
    int m0, n0;
    tile_origin(t, m0, n0);
    const bool hn = kHalfOk && n0 + 128 >= g.N && !(g.dbg & 32);
    setup_tile(m0, n0, hn);
    run_k(0, g.P, hn);
    if (g.dbg & 1) continue;
    if constexpr (kHalfOk) {
      if (hn) {
        epilogue(m0, n0, std::true_type{});
        continue;
      }
    }
    epilogue(m0, n0, std::false_type{});
  }
  if (tail_mode) return;

  // ------------------------------------------------------------------------------------------ stream-K region
  // 32-bit iteration arithmetic (the host keeps the iteration space below 2^23)
  const int I = (g.n_tiles - g.dp_tiles) * g.P;
  if (I == 0) return;
  auto range_begin = [&](int w) { return static_cast<int>((static_cast<unsigned>(w) * static_cast<unsigned>(I)) /
                                                          static_cast<unsigned>(G)); };
  int it = range_begin(wg);
  const int end = range_begin(wg + 1);
  const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc((void*)g.ws, (short)0, G * SLAB * 4, 0x00020000);
  while (it < end) {
    const int ts = it / g.P;
    const int kb = it - ts * g.P;
    const int ke = min(g.P, end - ts * g.P);
    const int t = g.dp_tiles + ts;
    int m0, n0;
    tile_origin(t, m0, n0);
    setup_tile(m0, n0);
    run(kb, ke, false, false);
    if (kb != 0) {
      // tail: publish the partial tile (register order: coalesced 16-B lanes)
      // buffer stores: per-lane voffset + a constant soffset per register (no 64-bit address per register for the
      // compiler to hoist out of the loop and spill)
      const uint32_t vo = static_cast<uint32_t>(wg) * SLAB * 4 + threadIdx.x * 16;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][b][i][j]), rws, vo,
                                                     (((a * 2 + b) * 4 + i) * 2 + j) * 8192, 16 /* sc1 */);
      // publish (MI355X_MICROARCH.md § visibility, first row of the sc1 table; cdna_hip_programming.md §6 G16 R1):
      // write-through (sc1) 16-B payload stores drained by EVERY storing wave, the workgroup barrier, then ONE lane's
      // agent-scope flag store — no release fence (a buffer_wbl2 would write back the whole XCD L2 mid-GEMM)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_store((__attribute__((address_space(1))) unsigned*)(g.flags + wg), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (ke < g.P) {
        // head of a split tile: add the tails of the workgroups that follow, in k order
        const int tile_end = (ts + 1) * g.P;
        for (int w2 = wg + 1; w2 < G && range_begin(w2) < tile_end; ++w2) {
          // consume: ONE lane polls the flag (relaxed agent = sc1 load), the workgroup barrier, then every load of
          // the slab is an sc1 buffer load (no acquire: it would invalidate the XCD's L2 under the running GEMM)
          if (threadIdx.x == 0) {
            unsigned spins = 0;
            while (__hip_atomic_load((gflag*)(g.flags + w2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
              __builtin_amdgcn_s_sleep(1);
              if (++spins > (1u << 28)) {  // residency violated: record it and finish (wrong tile) instead of hanging
                __hip_atomic_store((gflag*)g.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
              }
            }
            __hip_atomic_store((gflag*)(g.flags + w2), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          __syncthreads();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the barrier
          const uint32_t vo = static_cast<uint32_t>(w2) * SLAB * 4 + threadIdx.x * 16;
          // 2 loads in flight at a time: the 128 accumulator registers leave no room for more
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int reg = ((a * 2 + b) * 4 + i) * 2;
                const u32x4 s0 = __builtin_amdgcn_raw_buffer_load_b128(rws, vo, reg * 8192, 16 /* sc1 */);
                const u32x4 s1 = __builtin_amdgcn_raw_buffer_load_b128(rws, vo, (reg + 1) * 8192, 16 /* sc1 */);
                acc[a][b][i][0] += __builtin_bit_cast(f32x4, s0);
                acc[a][b][i][1] += __builtin_bit_cast(f32x4, s1);
                __builtin_amdgcn_sched_barrier(0);
              }
        }
      }
      epilogue(m0, n0, std::false_type{});
    }
    it = ts * g.P + ke;
    bar();  // LDS free (the tail path stages nothing, but the next segment's copies must not pass slower waves)
  }
}

inline bool epi_is_swiglu(int epilogue) { return epilogue == DRL_GEMM_SWIGLU; }
// epilogues that need whole tiles (no uniform split-K: its combine stores element by element)
inline bool epi_whole_tiles(int epilogue) { return epilogue == DRL_GEMM_SWIGLU || epilogue == DRL_GEMM_SWIGLU_BWD; }

struct SkTuning {
  int grid = 0;      // 0 = CU count
  int group = 4;     // M-tiles per rasterization group
  int mode = 0;      // 0 automatic (whole tiles, or uniform split-K for few long-K tiles), 1 stream-K (whole-tile
                     // rounds + a stream-K tail), 2 whole tiles only, 3 uniform split-K
  int param = 0;     // mode 1: minimum k-pairs per workgroup; mode 3: splits per tile (0 automatic)
  bool group_set = false;  // group given through drl_gemm_set_sk_tuning (else chosen per shape)
};
SkTuning g_sk;
int g_sk_dbg = 0;
int g_sk_kloop = 0;  // 1: layout-T operands past 2 GB as the round-5 host loop of K-block launches (A/B measurement)

template <int AT, int BT>
int launch_sk_layout(SkArgs& g, int epi, int grid, hipStream_t s) {
  const dim3 gr(static_cast<unsigned>(grid));
  switch (epi) {
    case EPI_NONE: hipLaunchKernelGGL((gemm_sk_kernel<EPI_NONE, AT, BT>), gr, dim3(512), 0, s, g); break;
    case EPI_F32: hipLaunchKernelGGL((gemm_sk_kernel<EPI_F32, AT, BT>), gr, dim3(512), 0, s, g); break;
    case EPI_BIAS:
      if constexpr (AT == 0 && BT == 0) hipLaunchKernelGGL((gemm_sk_kernel<EPI_BIAS, 0, 0>), gr, dim3(512), 0, s, g);
      break;
    case EPI_SWIGLU:
      if constexpr (AT == 0 && BT == 0) hipLaunchKernelGGL((gemm_sk_kernel<EPI_SWIGLU, 0, 0>), gr, dim3(512), 0, s, g);
      break;
    case EPI_SWIGLU_BWD:
      if constexpr (AT == 0 && BT == 1) hipLaunchKernelGGL((gemm_sk_kernel<EPI_SWIGLU_BWD, 0, 1>), gr, dim3(512), 0, s, g);
      break;
  }
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // namespace
}  // namespace drl

namespace drl {
namespace {
// The decomposition of one launch from its tile grid (g.tm, g.tn, g.P, g.n_tiles set) and the CU count: sets
// g.splits / g.dp_tiles / g.sk_base / g.sk_tile0, the grid and the mode (1 stream-K, 2 whole tiles, 3 uniform
// split-K). Host-only arithmetic (drl_gemm_plan reports it without a device).
int plan_decomposition(SkArgs& g, int epilogue, int cus, int& grid, int& mode) {
  // decomposition (grid never above the CU count: co-residency). Automatic: uniform split-K when the tiles fill at
  // most half the CUs and K is long enough to split (S = the most splits that fit the CUs, >= 2 k-pairs each, <= 16;
  // the SwiGLU epilogue pairs whole tiles, never split), else whole tiles in rounds.
  const int cap = g_sk.grid > 0 ? std::min(g_sk.grid, cus) : cus;
  grid = cap;
  mode = g_sk.mode;
  int S = 1;
  if (mode == 0 && g.n_tiles * 2 <= cap && g.P >= 256 && !epi_is_swiglu(epilogue)) {
    if (g.n_tiles * 12 <= cap && !epi_whole_tiles(epilogue)) {
      // very long K over at most a twelfth of the CUs in tiles (the small projections' weight gradients over the
      // update pass's tokens: o 16, qkv 20 tiles x 642 k-pairs): uniform split-K over every CU, up to 16 slices —
      // 246 -> 198 us (o, 12 slices) and 340 -> 264 us (qkv, 8 slices) against stream-K, whose tile heads add the
      // other workgroups' slabs one after another (profiles/r05_gemm_wgrad_splitk.jsonl)
      S = std::min(16, cap / g.n_tiles);
      mode = 3;
    } else if (g.n_tiles * 3 <= cap && (g.P < 1024 || g.n_tiles * 4 > cap) && !epi_whole_tiles(epilogue)) {
      // 3 slices per tile where they fit the CUs (down_proj's weight gradient: 76 tiles x 642 / 1284 k-pairs at 82144 /
      // 164288 tokens): 890 -> 698 and 1758 -> 1386 us against stream-K (profiles/r05_gemm_pair_probe.jsonl,
      // profiles/r05_gemm_sk_sweep_pass_rows.jsonl; 2 slices lose: 941 us); 22-63 tiles over >= 1024 k-pairs stay on
      // stream-K
      S = cap / g.n_tiles;
      mode = 3;
    } else {
      mode = 1;  // very long K over few tiles (the lm_head dgrad: 32 tiles x 1187 k-pairs): stream-K measured best
    }
  } else if (mode == 0 && epi_is_swiglu(epilogue) && g.n_tiles >= 8 * cap && g_sk.grid == 0) {
    // the gate_up + SwiGLU forward over a pass's tokens (38 tile columns x 321 / 642 tile rows: 47 / 95 rounds):
    // persistent whole-tile rounds + a stream-K tail (each split tile's head combines its k-order partials, then the
    // epilogue runs on the whole tile) against one workgroup per tile: 1282 -> 1232 us at 82144 rows, 2533 -> 2465
    // at 164288 (profiles/r05_gemm_sk_sweep_pass_rows.jsonl)
    mode = 1;
  } else if (mode == 0 || mode == 3) {
    // at most 8 splits of >= 6 k-pairs each (profiles/r03_gemm_sk_sweep.jsonl: more or shorter splits lose to the
    // slab traffic and the per-split pipeline fill)
    S = mode == 3 && g_sk.param > 0 ? g_sk.param : std::min({cap / std::max(1, g.n_tiles), 8, g.P / 6});
    S = std::max(1, std::min({S, g.P, 32, cap / std::max(1, g.n_tiles)}));
    if (epi_whole_tiles(epilogue) || g.n_tiles * 2 > cap) S = 1;
    mode = S > 1 ? 3 : 2;
  }
  g.splits = 1;
  if (mode == 3 && epi_whole_tiles(epilogue)) mode = 2;  // a forced split-K tuning: whole tiles instead
  if (mode == 3) {
    g.splits = S;
    g.dp_tiles = 0;
    g.sk_base = g.sk_tile0 = 0;
    grid = g.n_tiles * S;
  } else if (mode == 2) {
    // whole tiles, one workgroup per tile (no whole tile waits on another; the tail split-K slices below do, under the
    // co-residency rules of the file header): the hardware
    // deals tiles to CUs as they free up, so a kernel on a second stream (the weight gradient beside its input
    // gradient) fills the CUs a short grid leaves idle instead of waiting behind a persistent grid's static rounds
    g.dp_tiles = g.n_tiles;
    grid = g_sk.grid > 0 ? std::min(cap, g.n_tiles) : g.n_tiles;
    // a last round of at most a quarter of the CUs (the N = 896 outputs at the passes' token counts: 1284 = 5 x 256
    // + 4 tiles, 2568 = 10 x 256 + 8) would hold the whole launch for one more tile time while the other CUs idle:
    // over a long K (>= 16 k-pairs) those r tiles split K over S = cap / r slices instead (uniform split-K, <= 16
    // slices): down_proj's forward at the update pass's 82144 rows 628 -> 611 us; at K = 896 (7 k-pairs) the slices'
    // pipeline fill and combine cost more than the round they save (o_proj dgrad 151 -> 157 us), so not there
    // (profiles/r05_gemm_tail_splitk.jsonl); up to a third of the CUs since the lm_head weight gradient's K blocks
    // (2376 tiles, r = 72, 52 k-pairs): 17.73 -> 17.33 ms per call (profiles/r05_gemm_tail3_lm_head_wgrad.jsonl)
    const int r = g.n_tiles % cap;
    if (g_sk.mode == 0 && g_sk.grid == 0 && !epi_whole_tiles(epilogue) && g.n_tiles > cap && r > 0 && 3 * r <= cap &&
        g.P >= 16) {
      const int St = std::min({16, cap / r, g.P / 2});
      if (St >= 2) {
        g.splits = St;
        g.dp_tiles = g.sk_base = g.sk_tile0 = g.n_tiles - r;
        grid = g.n_tiles - r + r * St;
      }
    }
  } else {
    const int full = g.n_tiles / grid;
    const int dp = (g.n_tiles % grid == 0) ? g.n_tiles : std::max(0, full - 1) * grid;
    g.dp_tiles = dp;
    const int64_t I = static_cast<int64_t>(g.n_tiles - dp) * g.P;
    const int min_iters = g_sk.param > 0 ? g_sk.param : 2;
    DRL_CHECK_ARG(I < (1 << 23), "stream-K iteration space too large");
    if (dp == 0 && I > 0) grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(grid, I / min_iters)));
  }
  return DRL_OK;
}

}  // namespace
}  // namespace drl

extern "C" {

int64_t drl_gemm_workspace_bytes(void) {
  const int cus = drl::cu_count();
  if (cus <= 0) return -1;
  return static_cast<int64_t>(cus) * drl::SLAB * 4 + static_cast<int64_t>(cus + 1) * 4 + 256;
}

void drl_gemm_set_debug(int32_t flags) {
  drl::g_sk_dbg = flags;
  drl::g_sk_kloop = (flags & 16) ? 1 : 0;
}

int drl_gemm_plan(int64_t M, int64_t N, int64_t K, int32_t epilogue, int32_t cus, int32_t* info) {
  using namespace drl;
  DRL_CHECK_ARG(info != nullptr && M >= 1 && N >= 1 && K >= 1 && cus >= 1, "bad plan query");
  DRL_CHECK_ARG(epilogue >= DRL_GEMM_PLAIN && epilogue <= DRL_GEMM_SWIGLU_BWD, "unknown epilogue %d", epilogue);
  SkArgs g{};
  g.tm = static_cast<int>((M + 255) / 256);
  g.tn = static_cast<int>((N + 255) / 256);
  g.P = static_cast<int>((K + 127) / 128);
  g.n_tiles = g.tm * g.tn;
  int grid = 0, mode = 0;
  if (const int rc = plan_decomposition(g, epilogue, cus, grid, mode); rc != DRL_OK) return rc;
  info[0] = mode;
  info[1] = g.splits;
  info[2] = grid;
  info[3] = g.dp_tiles;
  info[4] = g.sk_base;
  return DRL_OK;
}

void drl_gemm_set_sk_tuning(int32_t grid, int32_t group, int32_t mode, int32_t param) {
  drl::g_sk.grid = grid > 0 ? grid : 0;
  drl::g_sk.group = (group >= 1 && group <= 64) ? group : 4;
  drl::g_sk.group_set = group >= 1 && group <= 64;
  drl::g_sk.mode = (mode >= 0 && mode <= 3) ? mode : 0;
  drl::g_sk.param = param > 0 ? param : 0;
}

int drl_gemm(const void* a, int64_t lda, int32_t a_layout, const void* b, int64_t ldb, int32_t b_layout, void* c,
             int64_t ldc, int32_t c_dtype, int32_t beta, int64_t M, int64_t N, int64_t K, const void* bias,
             int32_t epilogue, void* c2, int64_t ldc2, void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace drl;
  // a layout-K A operand beyond one buffer range (the lm_head input gradient's d_logits, 65536 x 151936 bf16 = 19.9 GB;
  // the prefill's 262144 x 4864 down_proj input) runs as ONE launch whose A descriptor is rebased per tile (base row m0,
  // 32-bit offsets within the tile's rows onward) — round 4 launched row blocks of 26 tile rows each, 104 tiles over
  // 256 CUs per launch; the same tiles, the same result
  const bool a_rebase = a_layout == DRL_LAYOUT_K && a && lda > 0 && M * lda * 2 + 320ll * lda * 2 >= (1ll << 31);
  // a layout-T operand beyond one buffer range has K along its rows (the weight gradient over a long token batch, e.g.
  // the lm_head's d_logits^T at 8192 rows x 151936): K blocks of whole 128-deep k-pairs accumulated into the fp32
  // output (the first block with the caller's beta, the rest with beta = 1)
  const auto t_bytes = [&](int32_t layout, int64_t ld) { return layout == DRL_LAYOUT_T ? K * ld * 2 + 320ll * ld * 2 : 0; };
  // a layout-T A past one buffer range with B within one: ONE launch whose tiles walk K in blocks (a_kblk), when the
  // decomposition is whole tiles (+ a split-K tail) — the lm_head weight gradient's d_logits^T
  bool a_kblocks = false;
  if (a && b && lda > 0 && ldb > 0 && a_layout == DRL_LAYOUT_T && t_bytes(a_layout, lda) >= (1ll << 31) &&
      t_bytes(b_layout, ldb) < (1ll << 31) && c_dtype == DRL_F32 && epilogue == DRL_GEMM_PLAIN && !g_sk_kloop) {
    SkArgs q{};
    q.tm = static_cast<int>((M + 255) / 256);
    q.tn = static_cast<int>((N + 255) / 256);
    q.P = static_cast<int>((K + 127) / 128);
    q.n_tiles = q.tm * q.tn;
    int grid_q = 0, mode_q = 0;
    a_kblocks = plan_decomposition(q, epilogue, cu_count(), grid_q, mode_q) == DRL_OK && mode_q == 2 &&
                lda * 2 * 128 < (1ll << 31) && M * 2 + 640 < (1ll << 31);
  }
  if (!a_kblocks && a && b && lda > 0 && ldb > 0 &&
      (t_bytes(a_layout, lda) >= (1ll << 31) || t_bytes(b_layout, ldb) >= (1ll << 31))) {
    DRL_CHECK_ARG(c_dtype == DRL_F32 && epilogue == DRL_GEMM_PLAIN,
                  "a layout-T operand over 2 GB needs the fp32 accumulating output (K split)");
    const int64_t ld = std::max(a_layout == DRL_LAYOUT_T ? lda : 0, b_layout == DRL_LAYOUT_T ? ldb : 0);
    const int64_t kb = std::max<int64_t>(128, ((1ll << 31) / (ld * 2) - 320) / 128 * 128);
    for (int64_t k0 = 0; k0 < K; k0 += kb) {
      const int64_t kk = std::min(kb, K - k0);
      const char* ak = static_cast<const char*>(a) + (a_layout == DRL_LAYOUT_T ? k0 * lda : k0) * 2;
      const char* bk = static_cast<const char*>(b) + (b_layout == DRL_LAYOUT_T ? k0 * ldb : k0) * 2;
      const int rc = drl_gemm(ak, lda, a_layout, bk, ldb, b_layout, c, ldc, c_dtype, k0 == 0 ? beta : 1, M, N, kk,
                              bias, epilogue, c2, ldc2, workspace, workspace_bytes, stream);
      if (rc != DRL_OK) return rc;
    }
    return DRL_OK;
  }
  DRL_CHECK_ARG(a && b && c, "NULL operand");
  DRL_CHECK_ARG(a_layout == DRL_LAYOUT_K || a_layout == DRL_LAYOUT_T, "a_layout");
  DRL_CHECK_ARG(b_layout == DRL_LAYOUT_K || b_layout == DRL_LAYOUT_T, "b_layout");
  DRL_CHECK_ARG(M >= 1 && N >= 1 && K >= 1 && M < (1ll << 30) && N < (1ll << 30) && K < (1ll << 30),
                "bad shape M=%lld N=%lld K=%lld", (long long)M, (long long)N, (long long)K);
  DRL_CHECK_ARG(epilogue >= DRL_GEMM_PLAIN && epilogue <= DRL_GEMM_SWIGLU_BWD, "unknown epilogue %d", epilogue);
  DRL_CHECK_ARG(c_dtype == DRL_BF16 || (c_dtype == DRL_F32 && epilogue == DRL_GEMM_PLAIN),
                "fp32 output takes the plain epilogue");
  DRL_CHECK_ARG(epilogue == DRL_GEMM_PLAIN || epilogue == DRL_GEMM_SWIGLU_BWD ||
                (a_layout == DRL_LAYOUT_K && b_layout == DRL_LAYOUT_K),
                "bias / SwiGLU epilogues need layout-K operands (the forward)");
  DRL_CHECK_ARG(epilogue != DRL_GEMM_SWIGLU_BWD ||
                (a_layout == DRL_LAYOUT_K && b_layout == DRL_LAYOUT_T && c2 != nullptr && ldc2 >= 2 * N && ldc >= 2 * N),
                "SwiGLU backward: the down_proj dgrad (A layout K, B layout T) with c2 = gu (M, 2N), c = dgu (M, 2N)");
  DRL_CHECK_ARG(epilogue != DRL_GEMM_BIAS || bias != nullptr, "bias epilogue without bias");
  DRL_CHECK_ARG(epilogue != DRL_GEMM_SWIGLU || N % 64 == 0, "SwiGLU: N = 2I with I %% 32 == 0");
  // a layout-K operand has K contiguous: a partial k-tile would read the next row, so whole 64-deep k-tiles (a
  // missing second tile of the last pair reads as zeros)
  DRL_CHECK_ARG((a_layout == DRL_LAYOUT_T && b_layout == DRL_LAYOUT_T) || K % 64 == 0,
                "K %% 64 == 0 unless both operands are layout T (K=%lld)", (long long)K);
  const int64_t a_rows = a_layout == DRL_LAYOUT_K ? M : K, a_cols = a_layout == DRL_LAYOUT_K ? K : M;
  const int64_t b_rows = b_layout == DRL_LAYOUT_K ? N : K, b_cols = b_layout == DRL_LAYOUT_K ? K : N;
  DRL_CHECK_ARG(lda >= a_cols && ldb >= b_cols && lda % 8 == 0 && ldb % 8 == 0 && aligned16(a) && aligned16(b),
                "A / B: 16-byte aligned rows with ld %% 8 == 0 and ld >= the contiguous extent");
  // 32-bit buffer offsets: the byte range plus one tile of overhang must stay below 2^32
  const int64_t a_bytes = a_rows * lda * 2, b_bytes = b_rows * ldb * 2;
  // (below 2 GB: voffset + a whole-range soffset must not wrap around 2^32)
  DRL_CHECK_ARG((a_rebase || a_kblocks ? 576ll * lda * 2 : a_bytes + 320ll * lda * 2) < (1ll << 31) &&
                    b_bytes + 320ll * ldb * 2 < (1ll << 31),
                "operand larger than the 2 GB buffer range");
  const int64_t ncols = epilogue == DRL_GEMM_SWIGLU ? N / 2 : N;
  DRL_CHECK_ARG(ldc >= ncols && (c2 == nullptr || ldc2 >= N), "ldc");
  const int64_t need = drl_gemm_workspace_bytes();
  DRL_CHECK_ARG(workspace != nullptr && workspace_bytes >= need && aligned16(workspace),
                "workspace: drl_gemm_workspace_bytes() = %lld bytes, flag words zeroed once", (long long)need);

  SkArgs g{};
  g.a = static_cast<const uint16_t*>(a);
  g.b = static_cast<const uint16_t*>(b);
  if (c_dtype == DRL_F32) g.c32 = static_cast<float*>(c);
  else g.c = static_cast<uint16_t*>(c);
  g.c2 = static_cast<uint16_t*>(c2);
  g.bias = static_cast<const uint16_t*>(bias);
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldc2 = ldc2;
  g.a_bytes = static_cast<uint32_t>(a_rebase || a_kblocks ? 0 : a_bytes);
  g.a_total = a_rebase || a_kblocks ? a_bytes : 0;
  // K-block rows: the most whole k-pairs whose rows (plus a tile of overhang) stay inside one 2 GB range
  g.a_kblk = a_kblocks ? static_cast<int>(std::max<int64_t>(128, ((1ll << 31) / (lda * 2) - 320) / 128 * 128)) : 0;
  g.b_bytes = static_cast<uint32_t>(b_bytes);
  g.M = static_cast<int>(M); g.N = static_cast<int>(N); g.K = static_cast<int>(K);
  g.beta = beta ? 1 : 0;
  g.dbg = g_sk_dbg;
  g.sk_order = (g_sk_dbg & 8) ? 1 : 0;
  g.tm = static_cast<int>((M + 255) / 256);
  g.tn = static_cast<int>((N + 255) / 256);
  g.P = static_cast<int>((K + 127) / 128);
  // rasterization group (M-tiles per group), unless tuned: narrow outputs (4 / 5 tile columns) over short K take 16 / 8
  // (the A panel shared by more workgroups of an XCD), over long K 1; few M-tiles x many tile columns (down_proj's
  // weight gradient) 2; the lm_head forward's 594 tile columns 8 (profiles/r04_gemm_groups_82144.jsonl: 2-5 % each)
  g.gm = g_sk.group;
  if (!g_sk.group_set) {
    if (g.tn <= 5) g.gm = g.P > 16 ? 1 : (g.tn == 5 ? 8 : 16);
    else if (g.tm <= 5) g.gm = 2;
    else if (g.tn >= 256) g.gm = 8;
  }
  g.nkt = static_cast<int>((K + 63) / 64);
  g.n_tiles = g.tm * g.tn;
  const int cus = cu_count();
  g.ws = static_cast<float*>(workspace);
  g.flags = reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + static_cast<int64_t>(cus) * SLAB * 4);
  g.tmo = g.flags + cus;

  int grid = 0, mode = 0;
  if (const int rc = plan_decomposition(g, epilogue, cus, grid, mode); rc != DRL_OK) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int epi = epilogue == DRL_GEMM_PLAIN ? (c_dtype == DRL_F32 ? EPI_F32 : EPI_NONE)
                  : epilogue == DRL_GEMM_BIAS ? EPI_BIAS : epilogue == DRL_GEMM_SWIGLU ? EPI_SWIGLU : EPI_SWIGLU_BWD;
  if (a_layout == DRL_LAYOUT_K && b_layout == DRL_LAYOUT_K) return launch_sk_layout<0, 0>(g, epi, grid, s);
  if (a_layout == DRL_LAYOUT_K) return launch_sk_layout<0, 1>(g, epi, grid, s);
  if (b_layout == DRL_LAYOUT_K) return launch_sk_layout<1, 0>(g, epi, grid, s);
  return launch_sk_layout<1, 1>(g, epi, grid, s);
}

}  // extern "C"
