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

// backward workgroup plans (profiles/r05_flash_bwd_ab.txt, update-pass shape B 256, T 768, head_dim 64):
// dQ on 4-wave workgroups over head sets (2 per CU, each one's staging / epilogue beside the other's key loop) and
// dK / dV on 2 key tiles per workgroup — with the tile copies' scalar addressing, 1362 -> 1235 us per backward
#ifndef DQ_WAVES
#define DQ_WAVES 4
#endif
#ifndef DKDV_KT64
#define DKDV_KT64 2
#endif
#ifndef DKDV_WAVES64
#define DKDV_WAVES64 8
#endif

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
  // optional (B,): query tiles wholly below q_start[b] are skipped (their out / lse rows are left unwritten) — the
  // shared-prompt copies of prefix sharing, whose outputs nothing reads
  const int32_t* q_start;
  // optional (B * Tq,): out row of query (b, t) in a packed (rows, Hkv * G * D) out, < 0: not written
  const int64_t* out_row;
};

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }

// lane i and lane i ^ 32 combined on both (one v_permlane32_swap, no LDS round trip): swapping the upper half
// of one copy of x with the lower half of another leaves, on every lane, the lower half's value in the first
// and the upper half's in the second, so both lanes of a pair see the same operands in the same order. Inline
// asm: the builtin's two results are folded into one by this compiler (measured: the max vanished), and the
// s_nops cover the VALU -> permlane -> VALU wait states.
__device__ __forceinline__ float pair_max(float x) {
  float lo = x, hi = x;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1\n\tv_max_f32 %0, %0, %1" : "+v"(lo), "+v"(hi));
  return lo;
}
__device__ __forceinline__ float pair_sum(float x) {
  float lo = x, hi = x;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1\n\tv_add_f32 %0, %0, %1" : "+v"(lo), "+v"(hi));
  return lo;
}

// XCD-aware tile order (cdna_hip_programming.md §5.5 T1): workgroups are dealt round-robin to the 8 XCDs,
// each with its own L2. Remap the linear workgroup id so that all tiles of one (sequence, KV head) land on
// the same XCD (its K / V stay in that L2) and, within an XCD, run in tile order. Returns (tile, bh).
// Placement only changes speed, never results.
__device__ __forceinline__ void xcd_tile_order(int ntiles, int nbh, int& tile, int64_t& bh) {
  const int64_t n = static_cast<int64_t>(ntiles) * nbh;
  const int64_t i = static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x;
  int64_t c = i;
  if (n % 8 == 0) c = (i % 8) * (n / 8) + i / 8;
  bh = c / ntiles;
  tile = static_cast<int>(c % ntiles);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
// ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10): per 16-lane group, lane 4q+p addresses row q,
// columns 4p..4p+3 of a 4 x 16 block; lane i receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ u16x4 lds_tr16(const uint16_t* p) {
  const s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(u16x4, r);
}

// Swizzled [32 positions][64] bf16 image (128-B rows, no padding): the 16-B unit u of row r is stored at
// unit u ^ f(r). f is a bijection on r & 7 (conflict-free 16-B row writes: 8 consecutive rows cover all 8
// units) that also flips bit 2 between rows r and r + 2 (the 4 rows of a transposing read never share banks).
__device__ __forceinline__ int xsw(int r) { return (r & 7) ^ ((r & 2) << 1); }
// 128-B rows (head_dim 64): the unit mask also keeps the wave's 16-B row reads (ds_read_b128, lane groups {0-3, 12-15,
// 20-27} / {4-11, 16-19, 28-31} of each half) conflict-free — the 8 even and the 8 odd rows of each lane group take 8
// distinct masks (xsw gave each mask to two of them: 2-way conflicts on every Q / dO fragment read of the dK / dV
// kernel) — while rows r and r + 2 (r % 4 == 0) still differ in bit 2 for the transposing reads
template <int XR>
__device__ __forceinline__ int xswz(int r) { return XR == 64 ? (((r >> 3) & 3) | ((r << 1) & 4)) : xsw(r); }
// XR = row length in elements (the head dim: 64 -> 128-B rows, 128 -> 256-B rows; the swizzle permutes the
// 16-B units within each aligned group of 8)
template <int XR = 64>
__device__ __forceinline__ int ximg_off(int r, int col) {  // element offset of (row r, column col)
  return r * XR + 8 * ((col >> 3) ^ xswz<XR>(r)) + (col & 7);
}

// A operand "X^T" (rows = head dim, k = positions in the accumulator order) of a 32-position x 64 tile X in
// the swizzled image above: k-step s, head-dim tile mt. Two transposing reads: element j of lane half h is
// position 16s + 8(j>>2) + 4h + (j&3), head-dim 32mt + (lane & 31).
template <int XR = 64>
__device__ __forceinline__ u16x8 lds_xt_operand(const uint16_t* x, int mt, int s, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, h = lane >> 5;
  const int col = 32 * mt + (lane & 16) + 4 * p;
  const u16x4 lo = lds_tr16(x + ximg_off<XR>(16 * s + 4 * h + q, col));
  const u16x4 hi = lds_tr16(x + ximg_off<XR>(16 * s + 8 + 4 * h + q, col));
  return u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// round-to-nearest-even f32 -> bf16 (one v_cvt_pk_bf16_f32; NaN stays NaN)
__device__ __forceinline__ uint16_t to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// two f32 -> packed bf16 pair (one v_cvt_pk_bf16_f32; the same rounding as to_bf16_bits)
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}

// K / V tiles of one 32-key block staged in LDS and shared by the G waves of the workgroup.
// K: [32 keys][D] rows of D*2 + 16 bytes (16-B aligned, conflict-free ds_read_b128 of a key row slice);
// V^T: [D][32 keys] rows of 80 bytes, keys permuted within each 16-key group as 0-3, 8-11, 4-7, 12-15 so that
// the 8 keys one lane half needs for a k-step of O^T += V^T P^T (16s + 4h + {0..3, 8..11}) are one
// conflict-free ds_read_b128 (80-B rows: 16 consecutive rows cover all 64 banks).
template <int D>
struct KVTile {
  static constexpr int KROW = D + 8;   // u16 per K row
  static constexpr int VROW = 40;      // u16 per V^T row
  static constexpr int KSZ = 32 * KROW, VSZ = D * VROW;
  static constexpr int NCH = (32 * D + D * 32) * 2 / 16;  // 16-B chunks per block
  static constexpr int CPT = NCH / 512;                   // chunks per thread (512-thread workgroups)
};

// global -> registers: chunk c < 32*D/8 is K row c / (D/8), 16-B column c % (D/8); the rest V^T row
// d = c' / 4, 16-B column c' % 4 (keys 8*col .. 8*col+7). Keys >= Tk load as zero.
// the same for a block wholly below Tk (the caller's test is on k0 alone, so it is uniform over the
// workgroup): no per-key bounds tests in the steady-state key loop
// dQ's K^T chunk cc of a staged key block -> (row d, 16-B column col of the block's 4): 8 rows x 4 columns per 32
// chunks, the row fastest. The staging store of a chunk is two 8-B writes to the permuted places of its 80-B row (20
// dwords): with d fastest, the 16 lanes of each ds_write_b64 lane group write 8 rows x 2 columns = 32 distinct banks,
// where d = cc / 4 put rows r .. r + 3 in a group (rows r and r + 2 share 4 banks: 2-way conflicts, 1.2M conflict
// cycles per dispatch). Same LDS image. The forward's V^T staging keeps d = cc / 4: there the remap (row-fastest, or
// rows {r, r + 1, r + 4, r + 5} with 4 columns each) removed its conflicts too but measured 1-2 % slower
// (profiles/r06_flash_staging_conflicts.txt)
__device__ __forceinline__ int tr_row(int cc) { return 8 * (cc >> 5) + (cc & 7); }
__device__ __forceinline__ int tr_col(int cc) { return (cc >> 3) & 3; }

template <int D>
__device__ __forceinline__ void kv_issue_full(const uint16_t* kbase, const uint16_t* vtbase, int64_t ld_vt,
                                              int64_t k0, int tid, u16x8 (&r)[KVTile<D>::CPT]) {
  constexpr int KCH = 32 * D / 8;
#pragma unroll
  for (int i = 0; i < KVTile<D>::CPT; ++i) {
    const int c = tid + 512 * i;
    if (c < KCH) {
      const int row = c / (D / 8), col = c % (D / 8);
      r[i] = *reinterpret_cast<const u16x8*>(kbase + (k0 + row) * D + col * 8);
    } else {
      const int cc = c - KCH, d = cc / 4, col = cc % 4;
      r[i] = *reinterpret_cast<const u16x8*>(vtbase + vt_index(d, k0 + col * 8, ld_vt, D));
    }
  }
}

template <int D>
__device__ __forceinline__ void kv_issue(const uint16_t* kbase, const uint16_t* vtbase, int64_t ld_vt, int64_t k0,
                                         int64_t Tk, int tid, u16x8 (&r)[KVTile<D>::CPT]) {
  constexpr int KCH = 32 * D / 8;
#pragma unroll
  for (int i = 0; i < KVTile<D>::CPT; ++i) {
    const int c = tid + 512 * i;
    if (c < KCH) {
      const int row = c / (D / 8), col = c % (D / 8);
      const int64_t key = k0 + row;
      r[i] = key < Tk ? *reinterpret_cast<const u16x8*>(kbase + key * D + col * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    } else {
      const int cc = c - KCH, d = cc / 4, col = cc % 4;
      const int64_t kk = k0 + col * 8;
      const uint16_t* src = vtbase + vt_index(d, kk, ld_vt, D);  // 8 keys inside one 32-key block
      if (kk + 7 < Tk) {
        r[i] = *reinterpret_cast<const u16x8*>(src);
      } else {
        u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (kk + j < Tk) v[j] = src[j];
        r[i] = v;
      }
    }
  }
}

template <int D>
__device__ __forceinline__ void kv_store(uint16_t* kl, uint16_t* vl, int tid, const u16x8 (&r)[KVTile<D>::CPT]) {
  constexpr int KCH = 32 * D / 8;
#pragma unroll
  for (int i = 0; i < KVTile<D>::CPT; ++i) {
    const int c = tid + 512 * i;
    if (c < KCH) {
      const int row = c / (D / 8), col = c % (D / 8);
      *reinterpret_cast<u16x8*>(kl + row * KVTile<D>::KROW + col * 8) = r[i];
    } else {
      const int cc = c - KCH, d = cc / 4, col = cc % 4;
      // keys 8col .. 8col+3 and 8col+4 .. 8col+7 to their permuted places (KVTile): two 8-B stores
      uint16_t* dst = vl + d * KVTile<D>::VROW + (col >> 1) * 16 + (col & 1) * 4;
      *reinterpret_cast<u16x4*>(dst) = u16x4{r[i][0], r[i][1], r[i][2], r[i][3]};
      *reinterpret_cast<u16x4*>(dst + 8) = u16x4{r[i][4], r[i][5], r[i][6], r[i][7]};
    }
  }
}

// key-valid bytes of the 32-key block at k0, staged with the block's K / V: thread tid < 8 holds the word of
// keys k0 + 4 tid .. k0 + 4 tid + 3 (0 past T). Read from LDS by the compute, so the key loop never waits
// on a global load of its own.
__device__ __forceinline__ uint32_t valid_issue(const uint8_t* vrow, int64_t k0, int64_t T, int tid) {
  if (tid >= 8) return 0u;
  const int64_t kb = k0 + 4 * tid;
  if (kb + 3 < T) return *reinterpret_cast<const uint32_t*>(vrow + kb);
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) v |= (kb + j < T ? static_cast<uint32_t>(vrow[kb + j]) : 0u) << (8 * j);
  return v;
}

template <int D>
__global__ __launch_bounds__(512, D == 64 ? 4 : 1) void flash_fwd_kernel(FlashArgs a) {
  constexpr int KS = D / 16;  // k-steps of S^T = K Q^T over the head dim
  constexpr int MT = D / 32;  // 32-row tiles of O^T over the head dim
  using TL = KVTile<D>;
  // two 32-key blocks per LDS buffer and per barrier: the two S^T chains of an iteration are independent, so
  // one block's softmax overlaps the other's MFMAs, and the per-block barrier / staging round trip is halved
  __shared__ __attribute__((aligned(16))) uint16_t lds_k[2][2][TL::KSZ];
  __shared__ __attribute__((aligned(16))) uint16_t lds_v[2][2][TL::VSZ];
  __shared__ uint32_t lds_vw[2][2][8];
  const int tid = threadIdx.x;
  const int lane = tid & 63, g = tid >> 6;
  const bool computes = g < a.G;  // waves >= G only help staging
  const int qi = lane & 31, h = lane >> 5;
  const int64_t ntiles = (a.Tq + 31) / 32;
  int tile;
  int64_t bh;
  xcd_tile_order(static_cast<int>(ntiles), static_cast<int>(gridDim.y), tile, bh);
  const int64_t b = bh / a.Hkv;
  const int64_t t0 = (ntiles - 1 - tile) * 32;  // longest causal rows first
  if (a.q_start && t0 + 32 <= a.q_start[b]) return;  // uniform: a skipped tile
  const int64_t tq = t0 + qi;
  const bool qvalid = computes && tq < a.Tq;

  bf16x8 qf[KS];
  {
    const int gg = computes ? g : 0;
    const uint16_t* qrow = a.q + ((bh * a.G + gg) * a.Tq + (qvalid ? tq : 0)) * D + 8 * h;
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
  const uint16_t* vtbase = a.vt + bh * vt_panel(a.ld_vt, D, a.ld_k);
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  const int64_t kmax = min(a.Tk, t0 + 31 + a.qoff + 1);  // causal limit of the tile's last query
  const int64_t nb = (kmax + 31) / 32;
  const int qpos = static_cast<int>(tq + a.qoff);  // positions fit in 32 bits (host check)
  const int qlo = static_cast<int>(t0 + a.qoff);     // smallest query position of the tile

  // one 32-key block: S^T, online softmax, O^T += V^T P^T (LDS buffer cur holds the block at k0)
  auto block = [&](int cur, int sl, int64_t k0) {
    // ---- S^T (32 keys x 32 queries): A = K rows from LDS (lane & 31 = key), B = Q fragments
    f32x16 st = f32x16{};
    const uint16_t* krow = lds_k[cur][sl] + qi * TL::KROW + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(krow + 16 * s);
      st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kv), qf[s], st, 0, 0, 0);
    }
    // ---- mask + scale; register r holds key k0 + (r & 3) + 8 * (r >> 2) + 4h of query tq
    const int kbase0 = static_cast<int>(k0) + 4 * h;
    uint32_t vw[4];
    bool allv = true;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      vw[c] = lds_vw[cur][sl][h + 2 * c];  // keys kbase0 + 8c .. + 3
      allv &= vw[c] == 0x01010101u;
    }
    // blocks strictly below the diagonal with every key valid need no mask (wave-uniform test)
    const bool full = __all(allv) && static_cast<int>(k0) + 31 <= qlo;
    // raw-score max (the scale is positive: max(s * scale) = scale * max(s)); masked scores -> -inf
    float mxr = -INFINITY;
    if (!full) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * c + j;
          const bool ok = ((vw[c] >> (8 * j)) & 0xffu) != 0u && kbase0 + 8 * c + j <= qpos;
          st[r] = ok ? st[r] : -INFINITY;
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) mxr = fmaxf(mxr, st[r]);
    mxr = pair_max(mxr);
    const float mx = mxr * a.scale_log2;
    // deferred rescale: the reference max moves only when the block's max exceeds it by more than 8 (log2
    // units), so p <= 2^8 and most blocks skip the O^T rescale; the final O / l and LSE are exact either way
    const float mn = mx > m + 8.f ? mx : m;
    const float mref = mn == -INFINITY ? 0.f : mn;  // keeps exp2(-inf - mref) = 0, never NaN
    const float alpha = __builtin_amdgcn_exp2f(m - mref);
    m = mn;
    float ps0 = 0.f, ps1 = 0.f;
    uint32_t pw[8];  // P in bf16, element pairs (2k, 2k + 1)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float p0 = __builtin_amdgcn_exp2f(fmaf(st[2 * k], a.scale_log2, -mref));
      const float p1 = __builtin_amdgcn_exp2f(fmaf(st[2 * k + 1], a.scale_log2, -mref));
      ps0 += p0;
      ps1 += p1;
      pw[k] = pk_bf16(p0, p1);
    }
    lsum = lsum * alpha + (ps0 + ps1);
    if (!__all(alpha == 1.f)) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) o[mt] *= alpha;
    }
    u16x8 pb[2];
    pb[0] = __builtin_bit_cast(u16x8, u32x4{pw[0], pw[1], pw[2], pw[3]});
    pb[1] = __builtin_bit_cast(u16x8, u32x4{pw[4], pw[5], pw[6], pw[7]});
    // ---- O^T += V^T P^T; k-step s: element j of lane half h is key k0 + 16s + 8(j>>2) + 4h + (j&3)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const uint16_t* vtl = lds_v[cur][sl] + (32 * mt + qi) * TL::VROW + 8 * h;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const u16x8 vv = *reinterpret_cast<const u16x8*>(vtl + 16 * s);
        o[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(vv), as_bf16x8(pb[s]), o[mt], 0, 0, 0);
      }
    }
  };
  // K/V staging: blocks ib + 2, ib + 3 are issued into registers at the start of the iteration over blocks
  // ib, ib + 1 (in flight under the compute) and written to the other LDS buffer at its end; the key-valid
  // words travel with them
  u16x8 stage[2][TL::CPT];
  uint32_t vst[2] = {0u, 0u};
  // the first two blocks: both issued before either is stored (one memory round trip, not two)
#pragma unroll
  for (int sl = 0; sl < 2; ++sl)
    if (sl < nb) {
      kv_issue<D>(kbase, vtbase, a.ld_vt, sl * 32, a.Tk, tid, stage[sl]);
      vst[sl] = valid_issue(vrow, sl * 32, a.Tk, tid);
    }
#pragma unroll
  for (int sl = 0; sl < 2; ++sl)
    if (sl < nb) {
      kv_store<D>(lds_k[0][sl], lds_v[0][sl], tid, stage[sl]);
      if (tid < 8) lds_vw[0][sl][tid] = vst[sl];
    }
  __syncthreads();
  for (int64_t ib = 0; ib < nb; ib += 2) {
    const int cur = static_cast<int>((ib >> 1) & 1);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
      if (ib + 2 + sl < nb) {
        const int64_t k0 = (ib + 2 + sl) * 32;
        if (k0 + 32 <= a.Tk) {
          kv_issue_full<D>(kbase, vtbase, a.ld_vt, k0, tid, stage[sl]);
          if (tid < 8) vst[sl] = *reinterpret_cast<const uint32_t*>(vrow + k0 + 4 * tid);
        } else {
          kv_issue<D>(kbase, vtbase, a.ld_vt, k0, a.Tk, tid, stage[sl]);
          vst[sl] = valid_issue(vrow, k0, a.Tk, tid);
        }
      }
    if (computes) {
      block(cur, 0, ib * 32);
      if (ib + 1 < nb) block(cur, 1, (ib + 1) * 32);
    }
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
      if (ib + 2 + sl < nb) {
        kv_store<D>(lds_k[cur ^ 1][sl], lds_v[cur ^ 1][sl], tid, stage[sl]);
        if (tid < 8) lds_vw[cur ^ 1][sl][tid] = vst[sl];
      }
    __syncthreads();
  }
  // ---- finalize: O^T register r of tile mt = head-dim row 32mt + (r & 3) + 8(r >> 2) + 4h of query tq
  const float lt = pair_sum(lsum);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (!qvalid) return;
  if (a.lse != nullptr && h == 0)
    a.lse[(bh * a.G + g) * a.Tq + tq] = lt > 0.f ? (m + __builtin_amdgcn_logf(lt)) * 0.6931471805599453f : -INFINITY;
  const int64_t orw = a.out_row ? a.out_row[b * a.Tq + tq] : (b * a.Tq + tq);
  if (orw < 0) return;
  uint16_t* orow = a.out + ((orw * a.Hkv + (bh % a.Hkv)) * a.G + g) * D;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u16x4 w = u16x4{to_bf16_bits(o[mt][4 * c] * inv), to_bf16_bits(o[mt][4 * c + 1] * inv),
                            to_bf16_bits(o[mt][4 * c + 2] * inv), to_bf16_bits(o[mt][4 * c + 3] * inv)};
      *reinterpret_cast<u16x4*>(orow + 32 * mt + 8 * c + 4 * h) = w;
    }
  }
}

// ------------------------------------------------------------------------------------------ backward
// FA2-style backward in two launches, recomputing P from the forward's LSE (nothing of size T x T is
// stored): (1) dq_kernel, query-tile centric in the forward's S^T orientation (lane = query): dP^T =
// V dO^T, dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T (K, V and the head-dim-major K^T copy staged in
// LDS, shared by the G query heads of the workgroup); it also writes delta = rowsum(dO * O).
// (2) dkdv_kernel, key-tile centric in the S orientation (lane = key): S = Q K^T, dP = dO V^T, then
// dV^T += dO^T P and dK^T += Q^T dS take P / dS straight from the accumulators, and their transposed A
// operands come from each wave's LDS image of the Q / dO tile through ds_read_b64_tr_b16 (no transposed
// copies in HBM). The G query heads of a KV group are the G waves of the workgroup; their dK / dV
// partials are summed in LDS in a fixed order (deterministic). Reference: autograd of the eager attention
// under dp_actor.py:90-280.
struct FlashBwdArgs {
  const uint16_t* q;      // (B, Hkv, G, T, D)
  const uint16_t* k;      // (B, Hkv, T, D)
  const uint16_t* kt;     // (B, Hkv, D, ld_t)
  const uint16_t* v;      // (B, Hkv, T, D)
  const uint16_t* o;      // (B, T, Hkv, G, D)
  const uint16_t* dout;   // (B, T, Hkv, G, D)
  const float* lse;       // (B, Hkv, G, T)
  const uint8_t* valid;
  int64_t ld_valid;
  float* delta;  // (B, Hkv, G, T)
  uint16_t* dq;  // (B, Hkv, G, T, D)
  uint16_t* dk;  // (B, Hkv, T, D)
  uint16_t* dv;  // (B, Hkv, T, D)
  int64_t Hkv, G, T, ld_t;
  float scale, scale_log2;
  // optional (B,): query tiles wholly below q_start[b] carry no gradient (dO = 0 there): dq is written as zeros,
  // and the dK / dV key loops start at the first kept tile
  const int32_t* q_start;
  // optional (B * T,): o is packed (rows, Hkv * G * D) and query (b, t) reads row o_row[b * T + t]; a negative entry
  // (a row whose dO is zero: pads, shared copies) reads row 0 — delta = rowsum(dO * O) = 0 either way
  const int64_t* o_row;
};

__device__ __forceinline__ float bf2f(uint16_t x) { return bf16_to_f32(x); }

// a wave-uniform 64-bit value into SGPRs (readfirstlane of both halves)
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}


// dq_kernel's per-key-block tiles in LDS, shared by the G waves (query heads) of the workgroup:
// K and V row-major [32 keys][D] (rows padded to D + 8 elements) and K^T [D][32 keys] (rows of 40, keys
// permuted within each 16-key group as in KVTile's V^T: one ds_read_b128 per k-step of dQ^T += K^T dS^T).
template <int D, int NT = 512>
struct DqTile {
  static constexpr int ROW = D + 8, TROW = 40;
  static constexpr int RSZ = 32 * ROW, TSZ = D * TROW;
  static constexpr int RCH = 32 * D / 8;        // 16-B chunks of one row-major tile
  static constexpr int NCH = 2 * RCH + D * 4;   // K, V, K^T
  static constexpr int CPT = (NCH + NT - 1) / NT;  // chunks per thread (NT-thread workgroups)
};

template <int D, int NT>
__device__ __forceinline__ void dq_issue(const uint16_t* kb, const uint16_t* vb, const uint16_t* ktb, int64_t ld_t,
                                         int k0, int T, int tid, u16x8 (&r)[DqTile<D, NT>::CPT]) {
  using TL = DqTile<D, NT>;
#pragma unroll
  for (int i = 0; i < TL::CPT; ++i) {
    const int c = tid + NT * i;
    u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (c < 2 * TL::RCH) {
      const int cc = c % TL::RCH, row = cc / (D / 8), col = cc % (D / 8);
      const int key = k0 + row;
      if (key < T) v = *reinterpret_cast<const u16x8*>((c < TL::RCH ? kb : vb) + static_cast<int64_t>(key) * D + col * 8);
    } else if (c < TL::NCH) {
      const int cc = c - 2 * TL::RCH, d = tr_row(cc), col = tr_col(cc);
      const int kk = k0 + col * 8;
      const uint16_t* src = ktb + static_cast<int64_t>(d) * ld_t + kk;
      if (kk + 7 < T) {
        v = *reinterpret_cast<const u16x8*>(src);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (kk + j < T) v[j] = src[j];
      }
    }
    r[i] = v;
  }
}

// dq_issue for a block wholly below T (uniform test on k0 by the caller): no per-key bounds tests, and branch-free —
// every thread issues every one of its loads (a chunk index past the tile re-reads a row-major chunk that dq_store
// discards), the source chosen by an address select. A load under a per-thread branch into a register initialised
// to zero made hipcc wait for ALL loads in flight (vmcnt(0)) before each of them, serialising the two-ahead prefetch
// into one memory round trip per chunk.
template <int D, int NT>
__device__ __forceinline__ void dq_issue_full(const uint16_t* kb, const uint16_t* vb, const uint16_t* ktb,
                                              int64_t ld_t, int k0, int tid, u16x8 (&r)[DqTile<D, NT>::CPT]) {
  using TL = DqTile<D, NT>;
#pragma unroll
  for (int i = 0; i < TL::CPT; ++i) {
    const int c0 = tid + NT * i, c = c0 < TL::NCH ? c0 : c0 % (2 * TL::RCH);
    const int cc = c % TL::RCH, row = cc / (D / 8), col = cc % (D / 8);
    const uint16_t* rm = (c < TL::RCH ? kb : vb) + static_cast<int64_t>(k0 + row) * D + col * 8;
    const int ct = c - 2 * TL::RCH, d = tr_row(ct), colt = tr_col(ct);
    const uint16_t* tm = ktb + static_cast<int64_t>(d) * ld_t + k0 + colt * 8;
    r[i] = *reinterpret_cast<const u16x8*>(c < 2 * TL::RCH ? rm : tm);
  }
}

template <int D, int NT>
__device__ __forceinline__ void dq_store(uint16_t* kl, uint16_t* vl, uint16_t* ktl, int tid,
                                         const u16x8 (&r)[DqTile<D, NT>::CPT]) {
  using TL = DqTile<D, NT>;
#pragma unroll
  for (int i = 0; i < TL::CPT; ++i) {
    const int c = tid + NT * i;
    if (c < 2 * TL::RCH) {
      const int cc = c % TL::RCH, row = cc / (D / 8), col = cc % (D / 8);
      *reinterpret_cast<u16x8*>((c < TL::RCH ? kl : vl) + row * TL::ROW + col * 8) = r[i];
    } else if (c < TL::NCH) {
      const int cc = c - 2 * TL::RCH, d = tr_row(cc), col = tr_col(cc);
      uint16_t* dst = ktl + d * TL::TROW + (col >> 1) * 16 + (col & 1) * 4;  // permuted (DqTile)
      *reinterpret_cast<u16x4*>(dst) = u16x4{r[i][0], r[i][1], r[i][2], r[i][3]};
      *reinterpret_cast<u16x4*>(dst + 8) = u16x4{r[i][4], r[i][5], r[i][6], r[i][7]};
    }
  }
}

// NW waves per workgroup over query heads hs * NW .. hs * NW + NW - 1 of the KV head (gridDim.y = B * Hkv * HS, HS =
// ceil(G / NW) head sets); waves past G only stage K / V / K^T
template <int D, int NW = 8>
__global__ __launch_bounds__(64 * NW) void flash_dq_kernel(FlashBwdArgs a) {
  constexpr int KS = D / 16, MT = D / 32, NT = 64 * NW;
  using TL = DqTile<D, NT>;
  __shared__ __attribute__((aligned(16))) uint16_t lds_k[2][TL::RSZ];
  __shared__ __attribute__((aligned(16))) uint16_t lds_v[2][TL::RSZ];
  __shared__ __attribute__((aligned(16))) uint16_t lds_kt[2][TL::TSZ];
  __shared__ uint32_t lds_vw[2][8];
  const int tid = threadIdx.x;
  const int HS = static_cast<int>((a.G + NW - 1) / NW);
  const int lane = tid & 63;
  const int qi = lane & 31, h = lane >> 5;
  const int T = static_cast<int>(a.T);
  const int ntiles = (T + 31) / 32;
  int tile;
  int64_t bhs;
  xcd_tile_order(ntiles, static_cast<int>(gridDim.y), tile, bhs);
  const int64_t bh = bhs / HS;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6) + NW * static_cast<int>(bhs % HS);  // scalar: uniform branches
  const bool computes = g < a.G;
  const int64_t b = bh / a.Hkv, hkv = bh % a.Hkv;
  const int t0 = (ntiles - 1 - tile) * 32;  // longest causal rows first
  const int tq = t0 + qi;
  const bool qvalid = computes && tq < T;
  const int64_t head = bh * a.G + (computes ? g : 0);
  if (a.q_start && t0 + 32 <= a.q_start[b]) {  // uniform: a skipped tile's dq rows are zero
    if (qvalid) {
#pragma unroll
      for (int s = 0; s < KS; ++s)
        *reinterpret_cast<u16x8*>(a.dq + (head * T + tq) * D + 16 * s + 8 * h) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    return;
  }
  bf16x8 qf[KS], dof[KS];
  float dl = 0.f;
  {
    const uint16_t* qrow = a.q + (head * T + (qvalid ? tq : 0)) * D + 8 * h;
    const int64_t orow_off = (((b * T + (qvalid ? tq : 0)) * a.Hkv + hkv) * a.G + (computes ? g : 0)) * D + 8 * h;
    const int64_t oq = a.o_row ? max(a.o_row[b * T + (qvalid ? tq : 0)], int64_t(0)) : b * T + (qvalid ? tq : 0);
    const int64_t oo_off = ((oq * a.Hkv + hkv) * a.G + (computes ? g : 0)) * D + 8 * h;  // O (packed or padded)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 qv = *reinterpret_cast<const u16x8*>(qrow + 16 * s);
      u16x8 dv = *reinterpret_cast<const u16x8*>(a.dout + orow_off + 16 * s);
      const u16x8 ov = *reinterpret_cast<const u16x8*>(a.o + oo_off + 16 * s);
      if (!qvalid) qv = dv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 8; ++j) dl = fmaf(bf2f(dv[j]), bf2f(ov[j]), dl);
      qf[s] = as_bf16x8(qv);
      dof[s] = as_bf16x8(dv);
    }
  }
  dl = pair_sum(dl);  // delta = rowsum(dO * O) of query tq
  if (qvalid && h == 0) a.delta[head * T + tq] = dl;
  const float lse2 = qvalid ? a.lse[head * T + tq] * 1.4426950408889634f : -INFINITY;
  const float lref = lse2 == -INFINITY ? INFINITY : lse2;  // exp2(x - inf) = 0 for rows with no allowed key
  f32x16 dqt[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) dqt[mt] = f32x16{};
  const uint16_t* kbase = a.k + bh * a.T * D;
  const uint16_t* vbase = a.v + bh * a.T * D;
  const uint16_t* ktbase = a.kt + bh * D * a.ld_t;
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  const int nb = (min(T, t0 + 32) + 31) / 32;
  // key blocks staged global -> registers -> LDS two blocks ahead: block j's loads go out two iterations before
  // its LDS store (register sets alternate by block parity), so each iteration's compute covers two iterations of
  // load latency instead of one (the per-block compute is a few hundred cycles, an L2 / HBM round trip more)
  u16x8 stage[2][TL::CPT];
  uint32_t vst[2] = {0u, 0u};
  auto issue_blk = [&](int j, int set) {
    const int kk = j * 32;
    if (kk + 32 <= T) {
      dq_issue_full<D, NT>(kbase, vbase, ktbase, a.ld_t, kk, tid, stage[set]);
      vst[set] = *reinterpret_cast<const uint32_t*>(vrow + kk + 4 * (tid & 7));  // every thread: no branch
    } else {
      dq_issue<D, NT>(kbase, vbase, ktbase, a.ld_t, kk, T, tid, stage[set]);
      vst[set] = valid_issue(vrow, kk, T, tid);
    }
  };
  issue_blk(0, 0);
  if (nb > 1) issue_blk(1, 1);
  dq_store<D, NT>(lds_k[0], lds_v[0], lds_kt[0], tid, stage[0]);
  if (tid < 8) lds_vw[0][tid] = vst[0];
  __syncthreads();
  // one key block; cur (the LDS buffer and register set parity) is a literal at both call sites, so each parity is
  // straight-line code with its own register set (a runtime parity branch let hipcc reuse one set's registers as
  // temporaries in the other path, behind a vmcnt(0) that drained the two-ahead prefetch)
  auto step = [&](const int ib, const int cur) __attribute__((always_inline)) {
    const int k0 = ib * 32;
    // block ib + 2 into the register set block ib left (stored to LDS in the previous iteration)
    if (ib + 2 < nb) {
      if (cur == 0) issue_blk(ib + 2, 0);
      else issue_blk(ib + 2, 1);
    }
    if (computes) {
      f32x16 st = f32x16{}, dpt = f32x16{};
      const uint16_t* kr = lds_k[cur] + qi * TL::ROW + 8 * h;
      const uint16_t* vr = lds_v[cur] + qi * TL::ROW + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const u16x8 kv = *reinterpret_cast<const u16x8*>(kr + 16 * s);
        const u16x8 vv = *reinterpret_cast<const u16x8*>(vr + 16 * s);
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kv), qf[s], st, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(vv), dof[s], dpt, 0, 0, 0);
      }
      const int kbase0 = k0 + 4 * h;
      uint32_t vw[4];
      bool allv = true;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        vw[c] = lds_vw[cur][h + 2 * c];  // keys kbase0 + 8c .. + 3
        allv &= vw[c] == 0x01010101u;
      }
      const bool full = __all(allv) && k0 + 31 <= t0;
      u16x8 dsb[2];
      if (full) {  // uniform: the unmasked form (a full block's rows all have an allowed key: lref finite)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[r], a.scale_log2, -lref));
          dsb[r >> 3][r & 7] = to_bf16_bits(p * (dpt[r] - dl));
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * c + j;
            const bool ok = ((vw[c] >> (8 * j)) & 0xffu) != 0u && kbase0 + 8 * c + j <= tq;
            const float p = ok ? __builtin_amdgcn_exp2f(fmaf(st[r], a.scale_log2, -lref)) : 0.f;
            dsb[r >> 3][r & 7] = to_bf16_bits(p * (dpt[r] - dl));
          }
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint16_t* ktl = lds_kt[cur] + (32 * mt + qi) * TL::TROW + 8 * h;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const u16x8 kv = *reinterpret_cast<const u16x8*>(ktl + 16 * s);
          dqt[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kv), as_bf16x8(dsb[s]), dqt[mt], 0, 0, 0);
        }
      }
    }
    if (ib + 1 < nb) {  // block ib + 1 (register set cur ^ 1) into the other LDS buffer
      if (cur == 0) {
        dq_store<D, NT>(lds_k[1], lds_v[1], lds_kt[1], tid, stage[1]);
        if (tid < 8) lds_vw[1][tid] = vst[1];
      } else {
        dq_store<D, NT>(lds_k[0], lds_v[0], lds_kt[0], tid, stage[0]);
        if (tid < 8) lds_vw[0][tid] = vst[0];
      }
    }
    __syncthreads();
  };
  for (int ib = 0; ib < nb; ib += 2) {
    step(ib, 0);
    if (ib + 1 < nb) step(ib + 1, 1);
  }
  if (!qvalid) return;
  uint16_t* dqrow = a.dq + (head * T + tq) * D;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u16x4 w = u16x4{to_bf16_bits(dqt[mt][4 * c] * a.scale), to_bf16_bits(dqt[mt][4 * c + 1] * a.scale),
                            to_bf16_bits(dqt[mt][4 * c + 2] * a.scale), to_bf16_bits(dqt[mt][4 * c + 3] * a.scale)};
      *reinterpret_cast<u16x4*>(dqrow + 32 * mt + 8 * c + 4 * h) = w;
    }
  }
}

// dQ over TWO adjacent 32-row query tiles per workgroup (round 6): each key block staged into LDS (K, V, K^T) feeds both
// tiles' products, so the global -> LDS staging and the block barrier are paid once per two tiles' MFMAs; the lower
// tile skips the upper tile's last (diagonal) block. Per (query row, head) every product, mask and rounding is the
// one-tile kernel's in its order: bit-identical to flash_dq_kernel (tests/test_layers_gpu.py). KV2 = 1: the K / V
// fragments of a block are read from LDS once and kept in registers for both tiles.
template <int D, int NW = 4, int KV2 = 1>
__global__ __launch_bounds__(64 * NW) void flash_dq2_kernel(FlashBwdArgs a) {
  constexpr int KS = D / 16, MT = D / 32, NT = 64 * NW;
  using TL = DqTile<D, NT>;
  __shared__ __attribute__((aligned(16))) uint16_t lds_k[2][TL::RSZ];
  __shared__ __attribute__((aligned(16))) uint16_t lds_v[2][TL::RSZ];
  __shared__ __attribute__((aligned(16))) uint16_t lds_kt[2][TL::TSZ];
  __shared__ uint32_t lds_vw[2][8];
  const int tid = threadIdx.x;
  const int HS = static_cast<int>((a.G + NW - 1) / NW);
  const int lane = tid & 63;
  const int qi = lane & 31, h = lane >> 5;
  const int T = static_cast<int>(a.T);
  const int ntiles = (T + 31) / 32, npairs = (ntiles + 1) / 2;
  int pair;
  int64_t bhs;
  xcd_tile_order(npairs, static_cast<int>(gridDim.y), pair, bhs);
  const int64_t bh = bhs / HS;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6) + NW * static_cast<int>(bhs % HS);  // scalar: uniform branches
  const bool computes = g < a.G;
  const int64_t b = bh / a.Hkv, hkv = bh % a.Hkv;
  const int64_t head = bh * a.G + (computes ? g : 0);
  // tile 1: the pair's upper tile (longest causal rows first), tile 0 the one below it (absent for an odd first pair)
  const int thi = ntiles - 1 - 2 * pair;
  int t0[2] = {(thi - 1) * 32, thi * 32};
  bool act[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const bool present = u == 1 || thi >= 1;
    const bool skipped = present && a.q_start && t0[u] + 32 <= a.q_start[b];  // uniform: dq rows zero
    if (skipped && computes && t0[u] + qi < T) {
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2)
        *reinterpret_cast<u16x8*>(a.dq + (head * T + t0[u] + qi) * D + 16 * s2 + 8 * h) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    act[u] = present && !skipped;
  }
  if (!act[1]) return;  // the upper tile skipped: so is the lower (workgroup-uniform)
  bf16x8 qf[2][KS], dof[2][KS];
  float dl[2], lref[2];
  int tq[2];
  bool qvalid[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    tq[u] = t0[u] + qi;
    qvalid[u] = computes && act[u] && tq[u] < T;
    float d = 0.f;
    const int tr = qvalid[u] ? tq[u] : 0;
    const uint16_t* qrow = a.q + (head * T + tr) * D + 8 * h;
    const int64_t orow_off = (((b * T + tr) * a.Hkv + hkv) * a.G + (computes ? g : 0)) * D + 8 * h;
    const int64_t oq = a.o_row ? max(a.o_row[b * T + tr], int64_t(0)) : b * T + tr;
    const int64_t oo_off = ((oq * a.Hkv + hkv) * a.G + (computes ? g : 0)) * D + 8 * h;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      u16x8 qv = *reinterpret_cast<const u16x8*>(qrow + 16 * s2);
      u16x8 dv = *reinterpret_cast<const u16x8*>(a.dout + orow_off + 16 * s2);
      const u16x8 ov = *reinterpret_cast<const u16x8*>(a.o + oo_off + 16 * s2);
      if (!qvalid[u]) qv = dv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 8; ++j) d = fmaf(bf2f(dv[j]), bf2f(ov[j]), d);
      qf[u][s2] = as_bf16x8(qv);
      dof[u][s2] = as_bf16x8(dv);
    }
    d = pair_sum(d);  // delta = rowsum(dO * O) of query tq
    dl[u] = d;
    if (qvalid[u] && h == 0) a.delta[head * T + tq[u]] = d;
    const float lse2 = qvalid[u] ? a.lse[head * T + tq[u]] * 1.4426950408889634f : -INFINITY;
    lref[u] = lse2 == -INFINITY ? INFINITY : lse2;
  }
  f32x16 dqt[2][MT];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) dqt[u][mt] = f32x16{};
  const uint16_t* kbase = a.k + bh * a.T * D;
  const uint16_t* vbase = a.v + bh * a.T * D;
  const uint16_t* ktbase = a.kt + bh * D * a.ld_t;
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  const int nb = (min(T, t0[1] + 32) + 31) / 32;                   // blocks of the upper tile
  const int nb_lo = act[0] ? (min(T, t0[0] + 32) + 31) / 32 : 0;  // of the lower tile
  u16x8 stage[2][TL::CPT];
  uint32_t vst[2] = {0u, 0u};
  auto issue_blk = [&](int j, int set) {
    const int kk = j * 32;
    if (kk + 32 <= T) {
      dq_issue_full<D, NT>(kbase, vbase, ktbase, a.ld_t, kk, tid, stage[set]);
      vst[set] = *reinterpret_cast<const uint32_t*>(vrow + kk + 4 * (tid & 7));
    } else {
      dq_issue<D, NT>(kbase, vbase, ktbase, a.ld_t, kk, T, tid, stage[set]);
      vst[set] = valid_issue(vrow, kk, T, tid);
    }
  };
  issue_blk(0, 0);
  if (nb > 1) issue_blk(1, 1);
  dq_store<D, NT>(lds_k[0], lds_v[0], lds_kt[0], tid, stage[0]);
  if (tid < 8) lds_vw[0][tid] = vst[0];
  __syncthreads();
  auto step = [&](const int ib, const int cur) __attribute__((always_inline)) {
    const int k0 = ib * 32;
    if (ib + 2 < nb) {
      if (cur == 0) issue_blk(ib + 2, 0);
      else issue_blk(ib + 2, 1);
    }
    if (computes) {
      const uint16_t* kr = lds_k[cur] + qi * TL::ROW + 8 * h;
      const uint16_t* vr = lds_v[cur] + qi * TL::ROW + 8 * h;
      u16x8 kv[KV2 ? KS : 1], vv[KV2 ? KS : 1];
      if constexpr (KV2) {
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          kv[s2] = *reinterpret_cast<const u16x8*>(kr + 16 * s2);
          vv[s2] = *reinterpret_cast<const u16x8*>(vr + 16 * s2);
        }
      }
      const int kbase0 = k0 + 4 * h;
      uint32_t vw[4];
      bool allv = true;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        vw[c] = lds_vw[cur][h + 2 * c];
        allv &= vw[c] == 0x01010101u;
      }
      allv = __all(allv);
      u16x8 dsb[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 0 && ib >= nb_lo) continue;  // uniform: the lower tile's blocks end one earlier
        f32x16 st = f32x16{}, dpt = f32x16{};
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          const u16x8 k_ = KV2 ? kv[KV2 ? s2 : 0] : *reinterpret_cast<const u16x8*>(kr + 16 * s2);
          const u16x8 v_ = KV2 ? vv[KV2 ? s2 : 0] : *reinterpret_cast<const u16x8*>(vr + 16 * s2);
          st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(k_), qf[u][s2], st, 0, 0, 0);
          dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(v_), dof[u][s2], dpt, 0, 0, 0);
        }
        const bool full = allv && k0 + 31 <= t0[u];
        if (full) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(st[r], a.scale_log2, -lref[u]));
            dsb[u][r >> 3][r & 7] = to_bf16_bits(p * (dpt[r] - dl[u]));
          }
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * c + j;
              const bool ok = ((vw[c] >> (8 * j)) & 0xffu) != 0u && kbase0 + 8 * c + j <= tq[u];
              const float p = ok ? __builtin_amdgcn_exp2f(fmaf(st[r], a.scale_log2, -lref[u])) : 0.f;
              dsb[u][r >> 3][r & 7] = to_bf16_bits(p * (dpt[r] - dl[u]));
            }
          }
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint16_t* ktl = lds_kt[cur] + (32 * mt + qi) * TL::TROW + 8 * h;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const u16x8 kt_ = *reinterpret_cast<const u16x8*>(ktl + 16 * s2);
          dqt[1][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kt_), as_bf16x8(dsb[1][s2]), dqt[1][mt], 0, 0, 0);
          if (ib < nb_lo)
            dqt[0][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kt_), as_bf16x8(dsb[0][s2]), dqt[0][mt], 0, 0,
                                                                 0);
        }
      }
    }
    if (ib + 1 < nb) {
      if (cur == 0) {
        dq_store<D, NT>(lds_k[1], lds_v[1], lds_kt[1], tid, stage[1]);
        if (tid < 8) lds_vw[1][tid] = vst[1];
      } else {
        dq_store<D, NT>(lds_k[0], lds_v[0], lds_kt[0], tid, stage[0]);
        if (tid < 8) lds_vw[0][tid] = vst[0];
      }
    }
    __syncthreads();
  };
  for (int ib = 0; ib < nb; ib += 2) {
    step(ib, 0);
    if (ib + 1 < nb) step(ib + 1, 1);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!qvalid[u]) continue;
    uint16_t* dqrow = a.dq + (head * T + tq[u]) * D;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const u16x4 w = u16x4{to_bf16_bits(dqt[u][mt][4 * c] * a.scale), to_bf16_bits(dqt[u][mt][4 * c + 1] * a.scale),
                              to_bf16_bits(dqt[u][mt][4 * c + 2] * a.scale), to_bf16_bits(dqt[u][mt][4 * c + 3] * a.scale)};
        *reinterpret_cast<u16x4*>(dqrow + 32 * mt + 8 * c + 4 * h) = w;
      }
    }
  }
}

// NW waves per workgroup; wave w handles query heads w, w + NW, ... of the KV head (its dK / dV partials
// accumulate over them in registers). head_dim 64: NW = 8 (one head per wave, G <= 8); head_dim 128: NW = 4,
// one wave per SIMD, so the 128 accumulator registers of dK^T / dV^T and the Q / dO rows fit without spilling.
// KT key tiles per workgroup (head_dim 64: 2): each Q / dO tile a wave stages feeds the KT tiles' products, so the
// L2 -> LDS traffic per MFMA halves (one 32-key tile per staged tile re-reads every query tile after it per key tile:
// the per-CU ingest, not the matrix pipe, bounded the one-tile form). Each key tile's terms are the one-tile
// kernel's, accumulated in the same (head, query tile) order: bit-identical to KT = 1.
template <int D, int NW, int KT = 1>
__global__ __launch_bounds__(64 * NW) void flash_dkdv_kernel(FlashBwdArgs a) {
  constexpr int KS = D / 16, MT = D / 32, KROW = D + 8;
  // per wave, two buffers of the swizzled image (ximg_off) of a query tile's Q and dO rows, filled two tiles ahead
  // by LDS-DMA (global_load_lds of whole 16-B units, the swizzle applied on the source address: a wave instruction
  // writes 1 KB lane-linearly); after the key loop the same LDS holds every wave's dK / dV partial for the
  // cross-wave reduction
  constexpr int XROW = D;
  constexpr int UPR = D / 8, RPI = 64 / UPR;  // 16-B units per row, rows per wave instruction
  constexpr int NDMA = 2 * (32 / RPI) + 2;    // LDS-DMA instructions per query tile: Q, dO rows + LSE, delta
  constexpr int PW = 2 * MT * 16 * 64;        // floats of one wave's dK^T + dV^T partial
  constexpr int XW_ELEMS = NW * 4 * 32 * XROW > NW * PW * 2 ? NW * 4 * 32 * XROW : NW * PW * 2;
  static_assert(D == 64 || D == 128, "head_dim 64 or 128");
  __shared__ __attribute__((aligned(16))) uint16_t kv_lds[2][KT * 32 * KROW];  // the key tiles' K and V rows
  __shared__ __attribute__((aligned(16))) uint16_t xw_raw[XW_ELEMS];     // [wave][buffer][Q / dO][position][d]
  auto xw = reinterpret_cast<uint16_t (*)[2][2][32 * XROW]>(xw_raw);
  // per wave, two slots of [LSE of the tile's 32 queries | their delta], one per image buffer
  __shared__ __attribute__((aligned(16))) float lsd[NW][2][64];
  const int tid = threadIdx.x;
  // the wave index as a scalar (readfirstlane): the heads, tile copies' base addresses and LDS slots derived from it
  // stay in SGPRs instead of holding 64-bit per-lane copies in VGPRs through the loop
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int T = static_cast<int>(a.T);
  const int ntiles = (T + 31) / 32;
  int tile;
  int64_t bh;
  xcd_tile_order((ntiles + KT - 1) / KT, static_cast<int>(gridDim.y), tile, bh);
  const int64_t b = bh / a.Hkv, hkv = bh % a.Hkv;
  const int k0 = tile * 32 * KT;  // key tile 0 has the most query tiles: dispatched first
  // first query tile of the loop: the causal start k0, or past the skipped tiles (q_start)
  const int ts = a.q_start ? max(k0, a.q_start[b] & ~31) : k0;
  int keyj[KT];
  bool kval[KT];
#pragma unroll
  for (int j = 0; j < KT; ++j) {
    keyj[j] = k0 + 32 * j + li;
    kval[j] = keyj[j] < T && a.valid[b * a.ld_valid + keyj[j]] != 0;
  }
  // NW = 8 >= G: the block has exactly G waves, one head each (a one-trip loop the compiler folds)
  const int g_end = NW >= 8 ? wv + 1 : static_cast<int>(a.G);
  // query tile tt of head g into image buffer `buf`: rows tt .. tt + 31 of Q and dO (rows past T read row T - 1:
  // finite values whose probabilities the LSE mask zeroes) and the rows' LSE (lanes 0-31) / delta (lanes 32-63)
  // The copies are inline asm: hipcc's own global_load_lds makes it wait for every LDS-DMA in flight (vmcnt(0))
  // before the next read of ANY of this kernel's LDS, which would drain the prefetch at each iteration's first
  // read; the asm copies are invisible to it, and the loop counts them itself (vmcnt(NDMA) / vmcnt(0)). m0 is not
  // declared clobbered (a reserved register: hipcc sets it itself before each of its own uses).
  const uint32_t lds_x = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) uint16_t*)xw_raw));
  const uint32_t lds_l = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) float*)&lsd[0][0][0]));
  // Q / dO rows address as a wave-uniform base (SGPR pair: the head's Q panel, the (b, kv head, g) column of dO) plus a
  // 32-bit per-lane byte offset (the saddr form), so a copy costs a few 32-bit ops instead of 64-bit index math
  const uint32_t drow = static_cast<uint32_t>(a.Hkv * a.G * D * 2);  // bytes per dO row (all heads of a position)
  auto tile_issue = [&](int g, int tt, int buf) {
    const int64_t head = bh * a.G + g;
    const uint64_t qb = uniform64(reinterpret_cast<uint64_t>(a.q + head * a.T * D));
    const uint64_t db = uniform64(reinterpret_cast<uint64_t>(a.dout + ((b * T * a.Hkv + hkv) * a.G + g) * D));
    const uint32_t xb = lds_x + 2 * static_cast<uint32_t>(((wv * 2 + buf) * 2) * 32 * XROW);
#pragma unroll
    for (int i = 0; i < 32 / RPI; ++i) {
      const int r = i * RPI + lane / UPR, u = (lane % UPR) ^ xswz<XROW>(r);
      const uint32_t tr = static_cast<uint32_t>(min(tt + r, T - 1));
      const uint32_t oq = tr * (D * 2) + 16 * u, od = tr * drow + 16 * u;
      const uint32_t dq_ = __builtin_amdgcn_readfirstlane(xb + 2 * i * RPI * XROW);
      const uint32_t dd_ = __builtin_amdgcn_readfirstlane(xb + 2 * (32 * XROW + i * RPI * XROW));
      asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(oq), "s"(qb), "s"(dq_) : "memory");
      asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(od), "s"(db), "s"(dd_) : "memory");
    }
    // LSE (lanes 0-31) and delta (lanes 32-63) of the tile's rows: one copy per lane half from its own SGPR base (both
    // execute, each under its half's exec mask, and land lane-linearly in the same 64-float slot)
    const uint32_t ol = static_cast<uint32_t>(min(tt + li, T - 1)) * 4u;
    const uint64_t lb = uniform64(reinterpret_cast<uint64_t>(a.lse + head * a.T));
    const uint64_t tb = uniform64(reinterpret_cast<uint64_t>(a.delta + head * a.T));
    const uint32_t dl_ = __builtin_amdgcn_readfirstlane(lds_l + 4 * static_cast<uint32_t>((wv * 2 + buf) * 64));
    if (h == 0) asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" :: "v"(ol), "s"(lb), "s"(dl_) : "memory");
    else asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" :: "v"(ol), "s"(tb), "s"(dl_) : "memory");
  };
  // the first head's first two query tiles are issued before the K / V staging, so the workgroup's opening memory
  // round trips overlap (the staging barrier waits for all of them)
  if (wv < g_end && ts < T) {
    tile_issue(wv, ts, 0);
    if (ts + 32 < T) tile_issue(wv, ts + 32, 1);
  }
  // stage the key tiles' K and V rows once; every wave (query head) reads them from LDS
  for (int c = tid; c < 2 * KT * 32 * (D / 8); c += blockDim.x) {
    const int which = c / (KT * 32 * (D / 8)), cc = c % (KT * 32 * (D / 8)), row = cc / (D / 8), col = cc % (D / 8);
    const int kk = k0 + row;
    u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (kk < T) v = *reinterpret_cast<const u16x8*>((which ? a.v : a.k) + (bh * a.T + kk) * D + col * 8);
    *reinterpret_cast<u16x8*>(&kv_lds[which][row * KROW + col * 8]) = v;
  }
  __syncthreads();
  f32x16 dkt[KT][MT], dvt[KT][MT];
#pragma unroll
  for (int j = 0; j < KT; ++j)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) dkt[j][mt] = dvt[j][mt] = f32x16{};
  for (int g = wv; g < g_end; g += NW) {
  if (g != wv && ts < T) {  // a later head of this wave (NW < G): its first two tiles now
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous head's reads of both buffers are done
    tile_issue(g, ts, 0);
    if (ts + 32 < T) tile_issue(g, ts + 32, 1);
  }
  for (int t0 = ts; t0 < T; t0 += 32) {
    const int buf = ((t0 - ts) >> 5) & 1;
    const uint16_t* xq = xw[wv][buf][0];
    const uint16_t* xd = xw[wv][buf][1];
    // this tile's LDS-DMA landed; the next tile's (issued one iteration earlier) stays in flight
    if (t0 + 32 < T) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool rows_in = t0 + 32 <= T;  // uniform
#pragma unroll
    for (int kh = 0; kh < KT; ++kh) {
    const int kj = k0 + 32 * kh, key = keyj[kh];
    if (KT > 1 && t0 + 31 < kj) continue;  // uniform: every key of this tile is after every query row
    // this query tile's Q / dO fragments and LSE / delta, read from the wave's LDS slots per key tile (re-reading them
    // is cheaper than holding them live across the KT tiles' products)
    u16x8 qa[KS], da[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qa[s] = *reinterpret_cast<const u16x8*>(xq + ximg_off<XROW>(li, 16 * s + 8 * h));
      da[s] = *reinterpret_cast<const u16x8*>(xd + ximg_off<XROW>(li, 16 * s + 8 * h));
    }
    float4 l4[4], d4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int qb = t0 + 8 * c + 4 * h;
      l4[c] = *reinterpret_cast<const float4*>(&lsd[wv][buf][8 * c + 4 * h]);
      d4[c] = *reinterpret_cast<const float4*>(&lsd[wv][buf][32 + 8 * c + 4 * h]);
      if (!rows_in) {
        l4[c] = make_float4(qb < T ? l4[c].x : -INFINITY, qb + 1 < T ? l4[c].y : -INFINITY,
                            qb + 2 < T ? l4[c].z : -INFINITY, qb + 3 < T ? l4[c].w : -INFINITY);
        d4[c] = make_float4(qb < T ? d4[c].x : 0.f, qb + 1 < T ? d4[c].y : 0.f, qb + 2 < T ? d4[c].z : 0.f,
                            qb + 3 < T ? d4[c].w : 0.f);
      }
    }
    const uint16_t* kl = kv_lds[0] + (32 * kh + li) * KROW + 8 * h;
    const uint16_t* vl = kv_lds[1] + (32 * kh + li) * KROW + 8 * h;
    // S = Q K^T and dP = dO V^T: A = rows of query t0 + li; C row r -> query t0 + (r&3) + 8(r>>2) + 4h
    f32x16 sc = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(kl + 16 * s);
      const u16x8 vv = *reinterpret_cast<const u16x8*>(vl + 16 * s);
      sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(qa[s]), as_bf16x8(kv), sc, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(da[s]), as_bf16x8(vv), dp, 0, 0, 0);
    }
    u16x8 pb[2], dsb[2];
    // block entirely at or below the diagonal, all keys valid, all queries in range: no mask, and every query
    // row has an allowed key (finite LSE)
    const bool full = __all(kval[kh]) && t0 >= kj + 31 && rows_in;
    if (full) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float nl[4] = {-l4[c].x * 1.4426950408889634f, -l4[c].y * 1.4426950408889634f,
                             -l4[c].z * 1.4426950408889634f, -l4[c].w * 1.4426950408889634f};
        const float dv4[4] = {d4[c].x, d4[c].y, d4[c].z, d4[c].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * c + j;
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[r], a.scale_log2, nl[j]));
          pb[r >> 3][r & 7] = to_bf16_bits(p);
          dsb[r >> 3][r & 7] = to_bf16_bits(p * (dp[r] - dv4[j]));
        }
      }
    } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int qb = t0 + 8 * c + 4 * h;
      const float lv[4] = {l4[c].x, l4[c].y, l4[c].z, l4[c].w}, dv4[4] = {d4[c].x, d4[c].y, d4[c].z, d4[c].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * c + j;
        const float l2 = lv[j] == -INFINITY ? INFINITY : lv[j] * 1.4426950408889634f;  // no allowed key: p = 0
        const bool ok = kval[kh] && key <= qb + j;
        const float p = ok ? __builtin_amdgcn_exp2f(fmaf(sc[r], a.scale_log2, -l2)) : 0.f;
        pb[r >> 3][r & 7] = to_bf16_bits(p);
        dsb[r >> 3][r & 7] = to_bf16_bits(p * (dp[r] - dv4[j]));
      }
    }
    }
    // dV^T += dO^T P and dK^T += Q^T dS: A operands read transposed from the wave's Q / dO image
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const u16x8 dov = lds_xt_operand<XROW>(xd, mt, s, lane);
        const u16x8 qtv = lds_xt_operand<XROW>(xq, mt, s, lane);
        dvt[kh][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(dov), as_bf16x8(pb[s]), dvt[kh][mt], 0, 0, 0);
        dkt[kh][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(qtv), as_bf16x8(dsb[s]), dkt[kh][mt], 0, 0, 0);
      }
    }
    }  // key tiles
    // refill this buffer with the tile two ahead once this wave's reads of it (and of its LSE slot) are done
    if (t0 + 64 < T) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      tile_issue(g, t0 + 64, buf);
    }
  }
  }  // query heads of this wave
  // every wave's partial into its own LDS slot (the buffer overlays the Q / dO images, so every wave must be past its
  // key loop first), ONE barrier, then all threads sum 4-element groups over the waves in wave order — the additions
  // (0 + p0) + p1 + ... of a wave-by-wave reduction, so the result is unchanged — and store them; key tile by key tile
  const int nw = a.G < NW ? static_cast<int>(a.G) : NW;
  float* part = reinterpret_cast<float*>(xw_raw);  // [wave][dk / dv][tile][register][lane]
#pragma unroll
  for (int j = 0; j < KT; ++j) {
    __syncthreads();
    if (wv < nw) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          part[wv * PW + (mt * 16 + r) * 64 + lane] = dkt[j][mt][r];
          part[wv * PW + ((MT + mt) * 16 + r) * 64 + lane] = dvt[j][mt][r];
        }
    }
    __syncthreads();
    for (int gi = tid; gi < 2 * MT * 4 * 64; gi += blockDim.x) {
      const int ln = gi & 63, c = (gi >> 6) & 3, mt = (gi >> 8) % MT, which = (gi >> 8) / MT;
      const int kk = k0 + 32 * j + (ln & 31);
      if (kk >= T) continue;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int w = 0; w < nw; ++w) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += part[w * PW + ((which * MT + mt) * 16 + 4 * c + e) * 64 + ln];
      }
      u16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = to_bf16_bits(which ? acc[e] : acc[e] * a.scale);
      *reinterpret_cast<u16x4*>((which ? a.dv : a.dk) + (bh * a.T + kk) * D + 32 * mt + 8 * c + 4 * (ln >> 5)) = o;
    }
  }
}

// ------------------------------------------------------------------------------------------ decode
// One new token per sequence against the KV cache, on MFMA: the G query heads of a KV head are the
// "queries" of the forward kernel's S^T = K Q^T tile (columns >= G are zero padding), so the online
// softmax stays lane-local and P^T feeds O^T += V^T P^T from the accumulators. Workgroup = (sequence,
// KV head), NW waves splitting the cached keys into interleaved 32-key blocks (each wave's next block
// is loaded while it computes the current one); the NW partial softmax states are merged in LDS.
// The cache holds K row-major (B, Hkv, ld_k, D) and V head-dim-major (B, Hkv, D, ld_vt), the layout
// drl_rope_qkv_fwd writes with koff / koff_dev. HBM-bound: 4 * D bytes per cached key.
struct DecodeArgs {
  const uint16_t* q;   // (B, Hkv, G, D)
  const uint16_t* k;   // (B, Hkv, ld_k, D)
  const uint16_t* vt;  // (B, Hkv, D, ld_vt)
  const uint8_t* valid;
  int64_t ld_valid;
  const int64_t* qpos_ptr;
  int64_t qpos;
  int64_t Hkv, G, ld_k, ld_vt, L;
  float scale_log2;
  uint16_t* out;  // (B, Hkv, G, D), or fragment-packed (out_mbt 32-row blocks) for the decode o_proj GEMM
  int64_t out_mbt;
  float* slabs;        // split-K: (B*Hkv, splits, 64 + 32*D) fp32 partial states (m, l, unnormalised o)
  unsigned* tickets;   // split-K: (B*Hkv) arrival counters, zero between launches
  // prompt groups: sequences b = p * group + r (r < group) share one prompt, whose keys [0, shared) are read from
  // cache row p (the rollout prefills each distinct prompt once); group 1 / shared 0: every row reads its own
  int64_t group, shared;
  int64_t rpt;  // decode_group_kernel: rows per column tile (0: 32 / G, every column of the MFMA tile in use)
  int64_t xmap;  // workgroup -> XCD placement: 0 = units dealt round-robin over the XCDs, 1 = a contiguous eighth of the
                 // units (and so of the cache rows and their pages) per XCD
};

// workgroup bid's index in an XCD-major order (xmap 1): the dispatcher deals consecutive workgroups to the 8 XCDs in turn
// (MI355X_MICROARCH.md, workgroup dispatch), so XCD x runs bid = x, x + 8, ...; renumbered, XCD x takes indices
// [x * total / 8, (x + 1) * total / 8)
__device__ __forceinline__ unsigned dec_xcd_major(unsigned bid, unsigned total) {
  return (bid & 7u) * (total >> 3) + (bid >> 3);
}

// (sequence, KV head) of workgroup `bid` under prompt groups: the group's rows of one (prompt, head) run as
// workgroups bid, bid + 8, ..., i.e. on one XCD under the observed round-robin dealing (MI355X_MICROARCH.md,
// workgroup dispatch), next to each other in time, so the shared prompt keys one of them fetches are L2 hits for
// the others (speed only: any placement gives the same result). 32-bit arithmetic: a 64-bit division is a software
// routine of ~100 instructions, and this mapping runs before the first load of every workgroup
__device__ __forceinline__ int64_t dec_grouped_bh(unsigned bid, unsigned group, unsigned Hkv, unsigned total,
                                                  int64_t xmap = 0) {
  const unsigned units = total / group;
  unsigned u, r;
  if (xmap && total % 8u == 0) {
    const unsigned idx = dec_xcd_major(bid, total);
    u = idx / group;
    r = idx % group;
  } else if (units % 8u == 0) {
    const unsigned slot = bid >> 3;
    r = slot % group;
    u = (slot / group) * 8u + (bid & 7u);
  } else {
    u = bid / group;
    r = bid % group;
  }
  const unsigned p = u / Hkv, hd = u - p * Hkv;
  return (static_cast<int64_t>(p) * group + r) * Hkv + hd;
}

// one 32-key block of the cache for lane (qi, h): K rows (A operand of S^T = K Q^T), V^T columns
// (A operand of O^T = V^T P^T) and the key-valid bytes of the keys this lane's scores cover
template <int D>
struct DecBlock {
  u16x8 kf[D / 16];
  u16x8 vf[D / 32][2];
  uint32_t vb[4];
};

// Coalesced block loader: a 32-key block is 4 KB of contiguous K rows and D rows x 64 B of V^T. A wave
// fetches it with whole 1-KB instructions (16 B per lane, K: 8 lanes per 128-B row; V^T: 4 lanes per 64-B
// row segment) instead of fragment-shaped loads that touch 32 rows x 16-32 B per instruction, then
// re-shapes it through its own LDS slot (no cross-wave sync: the wave writes and reads its slot in order).
template <int D>
struct DecRaw {
  u16x8 k[D / 16];
  u16x8 v[D / 16];
  uint32_t vb[4];
  int k0;  // first key of the block
};

// Every load is a whole 16 B at an in-bounds address (rows clamped to kend - 1, V^T columns to the row). The
// positions >= kend of a tail block are zeroed by dec_fix_tail when the block is consumed, not here: a select on
// the loaded registers right after the load made the wave wait for it (and every load before it) at issue time,
// which cost the prefetch of every tail block (most decode steps end in a partial block).
// The loads are buffer loads through descriptors of the wave-uniform K panel / V^T panel / key-valid row (their bases
// readfirstlane'd, so no waterfall loop: cdna_hip_programming.md T8 / T20) with 32-bit per-lane byte offsets: the
// 64-bit per-lane index math of flat loads was most of the loop's VALU (52 VALU per MFMA, profiles/r05_pmc_decattn_sq.json).
// The descriptors' byte ranges are the row's K panel (kcap keys), V^T panel and key-valid row: a key past the panel,
// a V^T column past the plain panel's row or a key-valid word past the row reads as zero (buffer range check), so no
// per-lane clamp is needed — the keys past kend within the panel are garbage until dec_fix_tail zeroes them (K rows,
// V^T columns) and masks their key-valid bytes when the block is consumed
template <int D>
__device__ __forceinline__ void dec_load_raw(const uint16_t* kb, const uint16_t* vtb, const uint8_t* vrow,
                                             int64_t ld_vt, int64_t ld_valid, int k0, int kcap, int lane, int h,
                                             DecRaw<D>& r) {
  constexpr int UPR = D / 8;  // 16-B units per K row
  r.k0 = k0;
  const bool blocked = ld_vt == DRL_VT_BLOCKED;
  const auto rk = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(uniform64(reinterpret_cast<uint64_t>(kb))),
                                                    0, kcap * D * 2, 0x00020000);
  const auto rv = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(uniform64(reinterpret_cast<uint64_t>(vtb))),
                                                    0, static_cast<int>(vt_panel(ld_vt, D, kcap)) * 2, 0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(uniform64(reinterpret_cast<uint64_t>(vrow))),
                                                    0, static_cast<int>(ld_valid), 0x00020000);
  // the key-valid words first: the oldest loads of an item, so the consumer waits for them without draining the
  // next item's loads behind them
#pragma unroll
  for (int c = 0; c < 4; ++c) r.vb[c] = __builtin_amdgcn_raw_buffer_load_b32(rb, k0 + 8 * c + 4 * h, 0, 0);
  const int ldv = static_cast<int>(blocked ? 0 : ld_vt);
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    const int c = lane + 64 * i;
    const int key = k0 + c / UPR;
    r.k[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, (key * D + 8 * (c % UPR)) * 2, 0, 0));
    const int d = c >> 2, kk = k0 + 8 * (c & 3);
    // blocked (key >> 5) * 32 * D + d * 32 + (key & 31) with key = kk, k0 % 32 == 0; else d * ld_vt + key
    const int vo = blocked ? k0 * D + d * 32 + 8 * (c & 3) : d * ldv + min(kk, ldv - 8);
    r.v[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rv, vo * 2, 0, 0));
  }
}

// the tail block's positions >= kend: K rows and V^T columns zeroed, key-valid bytes cleared (a no-op elsewhere)
template <int D>
__device__ __forceinline__ void dec_fix_tail(DecRaw<D>& r, int kend, int64_t ld_valid, int lane, int h) {
  constexpr int UPR = D / 8;
  const int k0 = r.k0;
  if (k0 + 32 <= kend) return;
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    const int c = lane + 64 * i;
    if (k0 + c / UPR >= kend) r.k[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    const int kk = k0 + 8 * (c & 3);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (kk + j >= kend) r.v[i][j] = 0;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int kk = k0 + 8 * c + 4 * h;
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) keep |= (kk + j < kend ? 0xffu : 0u) << (8 * j);
    r.vb[c] = kk + 3 < ld_valid ? (r.vb[c] & keep) : 0u;
  }
}

// raw block -> the wave's LDS slot -> MFMA fragments (the same DecBlock the fragment-shaped loader fills).
// K slot [32][D]: 16-B unit u of row r at u ^ (r & 7); V^T slot [D][32 keys]: 8-B slot t of row d at
// t ^ ((d >> 2) & 7) (conflict-free ds_read_b64 over 32 consecutive rows).
template <int D>
__device__ __forceinline__ void dec_reshape(const DecRaw<D>& r, uint16_t* ks, uint16_t* vs, int lane, int qi, int h,
                                            DecBlock<D>& blk) {
  constexpr int UPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    const int c = lane + 64 * i, row = c / UPR, u = c % UPR;
    *reinterpret_cast<u16x8*>(ks + row * D + 8 * (u ^ (row & 7))) = r.k[i];
    const int d = c >> 2, t0 = 2 * (c & 3), sw = (d >> 2) & 7;
    *reinterpret_cast<u16x4*>(vs + d * 32 + 4 * (t0 ^ sw)) = u16x4{r.v[i][0], r.v[i][1], r.v[i][2], r.v[i][3]};
    *reinterpret_cast<u16x4*>(vs + d * 32 + 4 * ((t0 + 1) ^ sw)) = u16x4{r.v[i][4], r.v[i][5], r.v[i][6], r.v[i][7]};
  }
#pragma unroll
  for (int s = 0; s < D / 16; ++s)
    blk.kf[s] = *reinterpret_cast<const u16x8*>(ks + qi * D + 8 * ((2 * s + h) ^ (qi & 7)));
#pragma unroll
  for (int mt = 0; mt < D / 32; ++mt) {
    const int d = 32 * mt + qi, sw = (d >> 2) & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u16x4 lo = *reinterpret_cast<const u16x4*>(vs + d * 32 + 4 * ((4 * s + h) ^ sw));
      const u16x4 hi = *reinterpret_cast<const u16x4*>(vs + d * 32 + 4 * ((4 * s + 2 + h) ^ sw));
      blk.vf[mt][s] = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) blk.vb[c] = r.vb[c];
}

// online-softmax step over one loaded block (scores, running max / sum, O^T accumulation)
template <int D>
__device__ __forceinline__ void dec_block(const DecBlock<D>& blk, const bf16x8 (&qf)[D / 16], float scale_log2,
                                          float& m, float& lsum, f32x16 (&o)[D / 32]) {
  constexpr int KS = D / 16, MT = D / 32;
  f32x16 st = f32x16{};
#pragma unroll
  for (int s = 0; s < KS; ++s) st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(blk.kf[s]), qf[s], st, 0, 0, 0);
  float x[16], mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * c + j;
      x[r] = ((blk.vb[c] >> (8 * j)) & 0xffu) != 0u ? st[r] * scale_log2 : -INFINITY;
      mx = fmaxf(mx, x[r]);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
  const float mn = fmaxf(m, mx);
  const float mref = mn == -INFINITY ? 0.f : mn;
  const float alpha = __builtin_amdgcn_exp2f(m - mref);
  m = mn;
  float ps = 0.f;
  u16x8 pb[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = __builtin_amdgcn_exp2f(x[r] - mref);
    ps += p;
    pb[r >> 3][r & 7] = to_bf16_bits(p);
  }
  lsum = lsum * alpha + ps;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    o[mt] *= alpha;
#pragma unroll
    for (int s = 0; s < 2; ++s)
      o[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(blk.vf[mt][s]), as_bf16x8(pb[s]), o[mt], 0, 0, 0);
  }
}

// raw block -> the wave's LDS slot only (fragments are read just in time by dec_block_lds)
template <int D>
__device__ __forceinline__ void dec_stage(const DecRaw<D>& r, uint16_t* ks, uint16_t* vs, int lane) {
  constexpr int UPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    const int c = lane + 64 * i, row = c / UPR, u = c % UPR;
    *reinterpret_cast<u16x8*>(ks + row * D + 8 * (u ^ (row & 7))) = r.k[i];
    const int d = c >> 2, t0 = 2 * (c & 3), sw = (d >> 2) & 7;
    *reinterpret_cast<u16x4*>(vs + d * 32 + 4 * (t0 ^ sw)) = u16x4{r.v[i][0], r.v[i][1], r.v[i][2], r.v[i][3]};
    *reinterpret_cast<u16x4*>(vs + d * 32 + 4 * ((t0 + 1) ^ sw)) = u16x4{r.v[i][4], r.v[i][5], r.v[i][6], r.v[i][7]};
  }
}

// dec_block with the K / V^T fragments read from the wave's LDS slot as each MFMA needs them (register-lean:
// lets several waves share a SIMD, so the staging of one block overlaps the math of another)
template <int D>
__device__ __forceinline__ void dec_block_lds(const uint16_t* ks, const uint16_t* vs, const uint32_t (&vb)[4],
                                              const bf16x8 (&qf)[D / 16], float scale_log2, int qi, int h, float& m,
                                              float& lsum, f32x16 (&o)[D / 32]) {
  constexpr int KS = D / 16, MT = D / 32;
  f32x16 st = f32x16{};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const u16x8 kf = *reinterpret_cast<const u16x8*>(ks + qi * D + 8 * ((2 * s + h) ^ (qi & 7)));
    st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kf), qf[s], st, 0, 0, 0);
  }
  float mx = -INFINITY;
  // every key of the block valid for every lane (the common case: a full block past the left padding): the unmasked
  // form, the same products (uniform branch)
  if (__all((vb[0] & vb[1] & vb[2] & vb[3]) == 0x01010101u)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      st[r] = st[r] * scale_log2;
      mx = fmaxf(mx, st[r]);
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * c + j;
        st[r] = ((vb[c] >> (8 * j)) & 0xffu) != 0u ? st[r] * scale_log2 : -INFINITY;
        mx = fmaxf(mx, st[r]);
      }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
  const float mn = fmaxf(m, mx);
  const float mref = mn == -INFINITY ? 0.f : mn;
  const float alpha = __builtin_amdgcn_exp2f(m - mref);
  m = mn;
  float ps = 0.f;
  u16x8 pb[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = __builtin_amdgcn_exp2f(st[r] - mref);
    ps += p;
    pb[r >> 3][r & 7] = to_bf16_bits(p);
  }
  lsum = lsum * alpha + ps;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    o[mt] *= alpha;
    const int d = 32 * mt + qi, sw = (d >> 2) & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u16x4 lo = *reinterpret_cast<const u16x4*>(vs + d * 32 + 4 * ((4 * s + h) ^ sw));
      const u16x4 hi = *reinterpret_cast<const u16x4*>(vs + d * 32 + 4 * ((4 * s + 2 + h) ^ sw));
      const u16x8 vf = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(vf), as_bf16x8(pb[s]), o[mt], 0, 0, 0);
    }
  }
}

// output element (sequence b, column k of (Hq * D)): row-major or fragment-packed (csrc/decode_gemm.hip layout)
__device__ __forceinline__ uint16_t* dec_out_ptr(const DecodeArgs& a, int64_t b, int64_t k, int64_t row_off) {
  if (a.out_mbt == 0) return a.out + row_off;  // row-major: row_off is the (b, k) offset
  return a.out + ((((k >> 4) * a.out_mbt + (b >> 5)) * 64 + ((k >> 3) & 1) * 32 + (b & 31)) * 8 + (k & 7));
}

template <int D, int NW, bool LEAN = false, bool SPLIT = false, int NB = 2, int LNB = 1>
__global__ __launch_bounds__(64 * NW) void decode_mfma_kernel(DecodeArgs a) {
  constexpr int KS = D / 16, MT = D / 32;
  __shared__ float s_m[NW][32], s_l[NW][32];
  // per wave: its K / V^T staging slot during the key loop, then its partial O^T (same 64*D*2... bytes)
  __shared__ __attribute__((aligned(16))) float s_o[NW][MT][16][64];
  __shared__ __attribute__((aligned(16))) uint32_t s_vb[LEAN && LNB > 1 ? NW : 1][4 * 64];  // deep lean ring only
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar wave index
  const int qi = lane & 31, h = lane >> 5;
  const unsigned hkv32 = static_cast<unsigned>(a.Hkv), grp32 = static_cast<unsigned>(a.group);
  const int64_t bh = a.group > 1 ? dec_grouped_bh(blockIdx.x, grp32, hkv32, gridDim.x, a.xmap)
                                 : (a.xmap && gridDim.x % 8 == 0 ? dec_xcd_major(blockIdx.x, gridDim.x) : blockIdx.x);
  const unsigned b32 = static_cast<unsigned>(bh) / hkv32;  // 32-bit: see dec_grouped_bh
  const int64_t b = b32;
  const uint16_t* kb = a.k + bh * a.ld_k * D;
  const uint16_t* vtb = a.vt + bh * vt_panel(a.ld_vt, D, a.ld_k);
  const uint8_t* vrow = a.valid + b * a.ld_valid;
  // the shared prompt keys [0, a.shared) of this row: cache row b / group (same KV head)
  const int64_t bs = b32 / grp32, bhs = bs * a.Hkv + (bh - b * a.Hkv);
  const uint16_t* kbs = a.k + bhs * a.ld_k * D;
  const uint16_t* vtbs = a.vt + bhs * vt_panel(a.ld_vt, D, a.ld_k);
  // key validity always from the row's own bytes: every row holds its prompt's mask (KVCache.share_prompts), while
  // a source row p < B / group is itself a sample of prompt p / group and carries THAT prompt's mask
  auto load_to = [&](int k0, int kcap, DecRaw<D>& r) {  // a.shared is a multiple of 32: wholly shared or wholly own
    if (k0 < a.shared) dec_load_raw<D>(kbs, vtbs, vrow, a.ld_vt, a.ld_valid, k0, kcap, lane, h, r);
    else dec_load_raw<D>(kb, vtb, vrow, a.ld_vt, a.ld_valid, k0, kcap, lane, h, r);
  };
  constexpr int NR = LEAN ? LNB : NB;
  DecRaw<D> R[NR];
  // without key splits a wave's first block is block w whatever the query position: it is issued before the position
  // (a device scalar) is known, its keys clamped to the cache capacity instead of kend (in bounds either way; the keys
  // >= kend of a tail block are zeroed by dec_fix_tail when it is consumed, and a wave without blocks never reads it),
  // so the position's load runs beside the first key loads instead of ahead of them. Same values: bit-identical.
  const bool spec = gridDim.y == 1 && 32 * w + 32 <= a.ld_k;
  if (spec) load_to(32 * w, static_cast<int>(a.ld_k), R[0]);
  const int qpos = static_cast<int>(a.qpos_ptr ? *a.qpos_ptr : a.qpos);
  const int kend = static_cast<int>(min(a.L, static_cast<int64_t>(qpos) + 1));
  auto load = [&](int k0, DecRaw<D>& r) { load_to(k0, static_cast<int>(a.ld_k), r); };
  // split-K over gridDim.y workgroups: split y takes 32-key blocks [y*n/S, (y+1)*n/S) of the n live blocks;
  // each wave takes blocks ib0, ib0 + NW, ... and has its first NB (LEAN: 1) in flight together with q
  const int nall = (kend + 31) / 32, S = gridDim.y, y = blockIdx.y;
  const int bbeg = y * nall / S, nblk = (y + 1) * nall / S;
  const int ib0 = bbeg + w;
  uint16_t* kslot = reinterpret_cast<uint16_t*>(&s_o[w][0][0][0]);  // 32 * D bf16
  uint16_t* vslot = kslot + 32 * D;                                 // D * 32 bf16
  const int nit = ib0 < nblk ? (nblk - ib0 + NW - 1) / NW : 0;        // this wave's blocks
  if constexpr (LEAN && LNB > 1) {  // every load unconditional: block indices clamped to the wave's last block
    if (nit > 0) {
#pragma unroll
      for (int j = 0; j < LNB; ++j)
        if (!(spec && j == 0)) load(32 * (ib0 + min(j, nit - 1) * NW), R[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < NR; ++j)
      if (ib0 + j * NW < nblk && !(spec && j == 0)) load(32 * (ib0 + j * NW), R[j]);
  }
  bf16x8 qf[KS];
  {
    const bool qv = qi < a.G;
    const uint16_t* qrow = a.q + (bh * a.G + (qv ? qi : 0)) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 v = *reinterpret_cast<const u16x8*>(qrow + 16 * s);
      if (!qv) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[s] = as_bf16x8(v);
    }
  }
  f32x16 o[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) o[mt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;
  if constexpr (LEAN && LNB > 1) {
    // LNB blocks in flight per wave (decode_group_kernel's ring): stage block j, refill its registers with block
    // j + LNB (clamped to the wave's last block: an unconditional refill, so hipcc counts the loads behind each register
    // set instead of waiting for all of them), then the softmax step from LDS. A block past the wave's end is staged
    // and consumed with no valid key (an exact no-op: alpha = 1, p = 0); the key-valid words go through the wave's LDS
    // slot (carried in registers past the refill they made hipcc drain every load). Same blocks, same order: bit-identical
    // to the one-in-flight loop.
    u32x4* vbslot = reinterpret_cast<u32x4*>(&s_vb[w][0]);
    for (int j = 0; j < nit; j += LNB) {
#pragma unroll
      for (int i = 0; i < LNB; ++i) {
        const int jj = j + i;
        dec_fix_tail<D>(R[i], kend, a.ld_valid, lane, h);
        dec_stage<D>(R[i], kslot, vslot, lane);
        vbslot[lane] = jj < nit ? u32x4{R[i].vb[0], R[i].vb[1], R[i].vb[2], R[i].vb[3]} : u32x4{0u, 0u, 0u, 0u};
        load(32 * (ib0 + min(jj + LNB, nit - 1) * NW), R[i]);
        const u32x4 v4 = vbslot[lane];
        const uint32_t vb[4] = {v4[0], v4[1], v4[2], v4[3]};
        dec_block_lds<D>(kslot, vslot, vb, qf, a.scale_log2, qi, h, m, lsum, o);
      }
    }
  } else if constexpr (LEAN) {
    // one block in flight per wave: stage it to the slot, issue the next, compute from LDS
    for (int ib = ib0; ib < nblk; ib += NW) {
      dec_fix_tail<D>(R[0], kend, a.ld_valid, lane, h);
      dec_stage<D>(R[0], kslot, vslot, lane);
      const uint32_t vb[4] = {R[0].vb[0], R[0].vb[1], R[0].vb[2], R[0].vb[3]};
      if (ib + NW < nblk) load(32 * (ib + NW), R[0]);
      dec_block_lds<D>(kslot, vslot, vb, qf, a.scale_log2, qi, h, m, lsum, o);
    }
  } else
  // ring of NB raw blocks: block ib + j * NW is reshaped out of R[j], whose next load is issued right after
  for (int ib = ib0; ib < nblk; ib += NB * NW) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int ibj = ib + j * NW;
      if (ibj < nblk) {
        DecBlock<D> blk;
        dec_fix_tail<D>(R[j], kend, a.ld_valid, lane, h);
        dec_reshape<D>(R[j], kslot, vslot, lane, qi, h, blk);
        if (ibj + NB * NW < nblk) load(32 * (ibj + NB * NW), R[j]);
        dec_block<D>(blk, qf, a.scale_log2, m, lsum, o);
      }
    }
  }
  // merge the 4 waves' states per query column (head) in a fixed order
  const float lt = lsum + __shfl_xor(lsum, 32, kWave);
  if (h == 0) { s_m[w][qi] = m; s_l[w][qi] = lt; }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) s_o[w][mt][r][lane] = o[mt][r];
  __syncthreads();
  if (SPLIT && S > 1) {
    // this split's state -> write-through slab; the last of the S splits merges them in split order
    float* slab = a.slabs + (bh * S + y) * (64 + 32 * D);
    if (w == 0) {
      if (h == 0) {
        float mm = -INFINITY;
#pragma unroll
        for (int v = 0; v < NW; ++v) mm = fmaxf(mm, s_m[v][qi]);
        const float mref = mm == -INFINITY ? 0.f : mm;
        float ll = 0.f;
#pragma unroll
        for (int v = 0; v < NW; ++v) ll += s_l[v][qi] * __builtin_amdgcn_exp2f(s_m[v][qi] - mref);
        store_f32_sc1(slab + qi, mm);
        store_f32_sc1(slab + 32 + qi, ll);
      }
      float mm = -INFINITY;
#pragma unroll
      for (int v = 0; v < NW; ++v) mm = fmaxf(mm, s_m[v][qi]);
      const float mref = mm == -INFINITY ? 0.f : mm;
      float sc[NW];
#pragma unroll
      for (int v = 0; v < NW; ++v) sc[v] = __builtin_amdgcn_exp2f(s_m[v][qi] - mref);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float acc = 0.f;
#pragma unroll
          for (int v = 0; v < NW; ++v) acc = fmaf(s_o[v][mt][r][lane], sc[v], acc);
          store_f32_sc1(slab + 64 + (mt * 16 + r) * 64 + lane, acc);  // (row r of tile mt, lane) as held
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int s_last;
    if (tid == 0) {
      const unsigned t = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)(a.tickets + bh), 1u,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = t == static_cast<unsigned>(S - 1);
    }
    __syncthreads();
    if (!s_last || w != 0) return;
    const float* base = a.slabs + bh * S * (64 + 32 * D);
    float mm = -INFINITY;
    for (int v = 0; v < S; ++v) mm = fmaxf(mm, load_f32_sc1(base + v * (64 + 32 * D) + qi));
    const float mref = mm == -INFINITY ? 0.f : mm;
    float ll = 0.f;
    for (int v = 0; v < S; ++v) {
      const float* sl = base + v * (64 + 32 * D);
      ll += load_f32_sc1(sl + 32 + qi) * __builtin_amdgcn_exp2f(load_f32_sc1(sl + qi) - mref);
    }
    const float inv = ll > 0.f ? 1.f / ll : 0.f;
    float acc[MT][16];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
    for (int v = 0; v < S; ++v) {
      const float* sl = base + v * (64 + 32 * D);
      const float sc = __builtin_amdgcn_exp2f(load_f32_sc1(sl + qi) - mref);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mt][r] = fmaf(load_f32_sc1(sl + 64 + (mt * 16 + r) * 64 + lane), sc, acc[mt][r]);
    }
    if (tid == 0) __hip_atomic_store((__attribute__((address_space(1))) unsigned*)(a.tickets + bh), 0u,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (qi >= a.G) return;
    const int64_t kq = ((bh % a.Hkv) * a.G + qi) * D;  // column of (b, query head) in (Hq * D)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        u16x4 wv;
#pragma unroll
        for (int j = 0; j < 4; ++j) wv[j] = to_bf16_bits(acc[mt][4 * c + j] * inv);
        const int64_t k = kq + 32 * mt + 8 * c + 4 * h;
        *reinterpret_cast<u16x4*>(dec_out_ptr(a, b, k, (bh * a.G + qi) * D + 32 * mt + 8 * c + 4 * h)) = wv;
      }
    return;
  }
  // every wave merges its share of the (tile, 4-row group) outputs: NW partial states per element, summed in
  // wave order (the same fixed order whichever wave does it)
  if (qi >= a.G) return;
  float mm = -INFINITY;
#pragma unroll
  for (int v = 0; v < NW; ++v) mm = fmaxf(mm, s_m[v][qi]);
  const float mref = mm == -INFINITY ? 0.f : mm;
  float sc[NW], ll = 0.f;
#pragma unroll
  for (int v = 0; v < NW; ++v) {
    sc[v] = __builtin_amdgcn_exp2f(s_m[v][qi] - mref);
    ll += s_l[v][qi] * sc[v];
  }
  const float inv = ll > 0.f ? 1.f / ll : 0.f;
  const int64_t kq = ((bh % a.Hkv) * a.G + qi) * D;  // column of (b, query head) in (Hq * D)
  for (int g = w; g < 4 * MT; g += NW) {
    const int mt = g >> 2, c = g & 3;
    u16x4 wv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) acc = fmaf(s_o[v][mt][4 * c + j][lane], sc[v], acc);
      wv[j] = to_bf16_bits(acc * inv);
    }
    const int64_t k = kq + 32 * mt + 8 * c + 4 * h;
    *reinterpret_cast<u16x4*>(dec_out_ptr(a, b, k, (bh * a.G + qi) * D + 32 * mt + 8 * c + 4 * h)) = wv;
  }
}

// Prompt groups on one workgroup: the rows p * group + r of one prompt read the same shared key blocks, so a
// workgroup takes the query columns of 32 / G of them at once (G query heads each: 4 rows x 7 heads for Qwen2.5)
// and each shared block is loaded ONCE for those rows (the per-row kernel loads it once per row, from L2 after the
// first). Workgroup = (prompt p, KV head, column tile of 32 / G rows); its NW waves take the key blocks of residue
// class w mod NW exactly as decode_mfma_kernel<D, NW> does per row: first the shared blocks (all columns), then
// each row's own blocks of that class (only that row's columns take part: every other lane sees its keys as
// invalid, and an all-invalid block is an exact no-op on the running state: alpha = 1, p = 0). Every column
// therefore runs the per-row kernel's arithmetic in the per-row kernel's order — MFMA columns are independent,
// the softmax is lane-local per column — and the result is bit-identical to decode_mfma_kernel<D, NW> on a cache
// where every row holds its own copy of the prompt keys. Contract: the rows of a group have identical key-valid
// bytes below `shared` (the rollout's KVCache.share_prompts copies them); the shared blocks' validity is read from
// the group's first row. One block in flight per wave (the register-lean loop).
template <int D, int NW, int NB = 2>
__global__ __launch_bounds__(64 * NW) void decode_group_kernel(DecodeArgs a) {
  constexpr int KS = D / 16, MT = D / 32;
  __shared__ float s_m[NW][32], s_l[NW][32];
  __shared__ __attribute__((aligned(16))) uint32_t s_vb[NW][4 * 64];  // per wave: the staged item's key-valid words
  __shared__ __attribute__((aligned(16))) float s_o[NW][MT][16][64];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar wave index
  const int qi = lane & 31, h = lane >> 5;
  const int G = static_cast<int>(a.G), group = static_cast<int>(a.group);
  const int rpt = a.rpt > 0 ? static_cast<int>(a.rpt) : 32 / G, ntile = (group + rpt - 1) / rpt;
  const unsigned units = gridDim.x / static_cast<unsigned>(ntile), nt32 = static_cast<unsigned>(ntile);
  unsigned unit, ct;  // 32-bit mapping (dec_grouped_bh)
  if (a.xmap && gridDim.x % 8 == 0) {
    const unsigned idx = dec_xcd_major(blockIdx.x, gridDim.x);
    unit = idx / nt32;
    ct = idx % nt32;
  } else if (units % 8 == 0) {  // the column tiles of one (prompt, head) on one XCD, back to back
    const unsigned slot = blockIdx.x >> 3;
    ct = slot % nt32;
    unit = (slot / nt32) * 8 + (blockIdx.x & 7);
  } else {
    unit = blockIdx.x / nt32;
    ct = blockIdx.x % nt32;
  }
  const unsigned p32 = unit / static_cast<unsigned>(a.Hkv);
  const int64_t p = p32, hd = unit - p32 * static_cast<unsigned>(a.Hkv);
  const int nr = min(rpt, group - static_cast<int>(ct) * rpt);  // rows of this tile
  const int rl = qi / G, g = qi - rl * G;                         // this lane's column: local row, query head
  const bool col_ok = rl < nr;
  const int64_t b0 = p * group + ct * rpt;                        // first row of the tile
  const int64_t bcol = b0 + (col_ok ? rl : 0);
  const int64_t panel = vt_panel(a.ld_vt, D, a.ld_k);
  const uint16_t* kbs = a.k + (p * a.Hkv + hd) * a.ld_k * D;     // shared keys: cache row p
  const uint16_t* vtbs = a.vt + (p * a.Hkv + hd) * panel;
  const uint8_t* vrows = a.valid + p * group * a.ld_valid;        // the group's first row's mask
  DecRaw<D> R[NB];  // NB items in flight per wave (static indexing: every use below is unrolled)
  // the wave's first NB shared blocks (w, w + NW, ...) issued before the query position is known, keys clamped to the
  // cache capacity (decode_mfma_kernel's speculative first block); kept when the item list starts with them (every
  // decode step: the position is past the prompt), reloaded otherwise
  const int nsh_all = static_cast<int>(a.shared / 32);
  bool spec[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    spec[j] = nsh_all > w + j * NW;
    if (spec[j])
      dec_load_raw<D>(kbs, vtbs, vrows, a.ld_vt, a.ld_valid, 32 * (w + j * NW), static_cast<int>(a.ld_k), lane, h, R[j]);
  }
  const int qpos = static_cast<int>(a.qpos_ptr ? *a.qpos_ptr : a.qpos);
  const int kend = static_cast<int>(min(a.L, static_cast<int64_t>(qpos) + 1));
  const int nall = (kend + 31) / 32, nsh = min(nsh_all, nall);
  const int n_sh = nsh > w ? (nsh - w + NW - 1) / NW : 0;         // shared blocks of class w
  const int own0 = nsh + ((w - nsh) % NW + NW) % NW;              // first own block of class w
  const int n_own = nall > own0 ? (nall - own0 + NW - 1) / NW : 0;
  const int items = n_sh + nr * n_own;
  // item j -> block index, source row (-1: shared) ; loads through the per-row kernel's raw loader
  auto load = [&](int j, DecRaw<D>& r) {
    if (j < n_sh) {
      dec_load_raw<D>(kbs, vtbs, vrows, a.ld_vt, a.ld_valid, 32 * (w + j * NW), static_cast<int>(a.ld_k), lane, h, r);
    } else {
      const int jj = j - n_sh, rr = jj / n_own, ib = own0 + (jj - rr * n_own) * NW;
      const int64_t bh = (b0 + rr) * a.Hkv + hd;
      dec_load_raw<D>(a.k + bh * a.ld_k * D, a.vt + bh * panel, a.valid + (b0 + rr) * a.ld_valid, a.ld_vt,
                      a.ld_valid, 32 * ib, static_cast<int>(a.ld_k), lane, h, r);
    }
  };
  uint16_t* kslot = reinterpret_cast<uint16_t*>(&s_o[w][0][0][0]);
  uint16_t* vslot = kslot + 32 * D;
  // every load below is unconditional (item indices clamped to the last item; a phantom item past the end is staged
  // and consumed as an all-invalid block): with a conditional refill hipcc cannot count the loads behind a register
  // set and waits for every load in flight (vmcnt(0)) at each stage, one item in flight instead of NB
  if (items > 0) {
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (!(spec[j] && nsh == nsh_all)) load(min(j, items - 1), R[j]);  // item j is shared block w + j NW: issued
  }
  bf16x8 qf[KS];
  {
    const uint16_t* qrow = a.q + ((bcol * a.Hkv + hd) * a.G + g) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 v = *reinterpret_cast<const u16x8*>(qrow + 16 * s);
      if (!col_ok) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[s] = as_bf16x8(v);
    }
  }
  f32x16 o[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) o[mt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;
  // stage item j to the wave's slot, refill its registers with item j + 2, then the online-softmax step from LDS
  // the key-valid words go through the wave's LDS slot with K / V^T: carried in registers past the refill of R they
  // made hipcc wait for every load in flight (vmcnt(0)) at each step, one item in flight instead of two
  u32x4* vbslot = reinterpret_cast<u32x4*>(&s_vb[w][0]);
  auto step = [&](int j, DecRaw<D>& R) {
    dec_fix_tail<D>(R, kend, a.ld_valid, lane, h);
    dec_stage<D>(R, kslot, vslot, lane);
    // an own block takes part only in its row's columns; a phantom item (j >= items) in none
    const bool act = j < items && (j < n_sh || (j - n_sh) / n_own == rl);
    vbslot[lane] = act ? u32x4{R.vb[0], R.vb[1], R.vb[2], R.vb[3]} : u32x4{0u, 0u, 0u, 0u};
    load(min(j + NB, items - 1), R);  // unconditional refill (past the end: the last item again)
    const u32x4 v4 = vbslot[lane];
    const uint32_t vb[4] = {v4[0], v4[1], v4[2], v4[3]};
    dec_block_lds<D>(kslot, vslot, vb, qf, a.scale_log2, qi, h, m, lsum, o);
  };
  for (int j = 0; j < items; j += NB) {
    // items past the end are phantoms: an exact no-op on m / lsum / o (alpha = 1, p = 0)
#pragma unroll
    for (int i = 0; i < NB; ++i) step(j + i, R[i]);
  }
  // merge the NW waves' states per column in wave order (decode_mfma_kernel's non-split merge)
  const float lt = lsum + __shfl_xor(lsum, 32, kWave);
  if (h == 0) { s_m[w][qi] = m; s_l[w][qi] = lt; }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) s_o[w][mt][r][lane] = o[mt][r];
  __syncthreads();
  if (!col_ok) return;
  float mm = -INFINITY;
#pragma unroll
  for (int v = 0; v < NW; ++v) mm = fmaxf(mm, s_m[v][qi]);
  const float mref = mm == -INFINITY ? 0.f : mm;
  float sc[NW], ll = 0.f;
#pragma unroll
  for (int v = 0; v < NW; ++v) {
    sc[v] = __builtin_amdgcn_exp2f(s_m[v][qi] - mref);
    ll += s_l[v][qi] * sc[v];
  }
  const float inv = ll > 0.f ? 1.f / ll : 0.f;
  const int64_t bh = bcol * a.Hkv + hd;
  const int64_t kq = (hd * a.G + g) * D;  // column of (b, query head) in (Hq * D)
  for (int gg = w; gg < 4 * MT; gg += NW) {
    const int mt = gg >> 2, c = gg & 3;
    u16x4 wv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) acc = fmaf(s_o[v][mt][4 * c + j][lane], sc[v], acc);
      wv[j] = to_bf16_bits(acc * inv);
    }
    const int64_t k = kq + 32 * mt + 8 * c + 4 * h;
    *reinterpret_cast<u16x4*>(dec_out_ptr(a, bcol, k, (bh * a.G + g) * D + 32 * mt + 8 * c + 4 * h)) = wv;
  }
}

// decode_group_kernel with the rows' own blocks balanced over the waves. There, wave w takes every own block of class
// w (block index = w mod NW) for all the tile's rows: at 512 rows x 2 KV heads (4 rows per tile, 16 shared + 1..8 own
// blocks, 8 waves) the waves holding an own class run 2 shared + 4 own items while the rest run 2, so the critical
// path is 6 items at every cache length. Here a column's state per class is still built in the per-row kernel's order —
// the class's shared blocks, then its own blocks — but the own part runs as units (class c, row r), dealt round-robin
// over the waves after the shared phase: each wave leaves its class state in LDS after its shared items (one barrier),
// a unit loads its class's state, runs row r's own blocks of that class (only row r's columns take part: every other
// column sees all-invalid blocks, an exact no-op) and writes back row r's columns of the state. Units of one class touch
// disjoint columns, so they may run on any waves in any order: the result is bit-identical to decode_group_kernel (and
// the per-row kernel) at the same wave count, with 2 + ceil(4 * own / 8) items on the critical path instead of 6.
template <int D, int NW, int NB = 2>
__global__ __launch_bounds__(64 * NW) void decode_group_bal_kernel(DecodeArgs a) {
  constexpr int KS = D / 16, MT = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t s_stage[NW][64 * D];  // per wave: K [32][D], V^T [D][32]
  __shared__ __attribute__((aligned(16))) float s_so[NW][MT][16][64];   // class states: O^T accumulators
  __shared__ float s_sm[NW][64], s_sl[NW][64];                          // class states: running max / sum per lane
  __shared__ __attribute__((aligned(16))) uint32_t s_vb[NW][4 * 64];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qi = lane & 31, h = lane >> 5;
  const int G = static_cast<int>(a.G), group = static_cast<int>(a.group);
  const int rpt = a.rpt > 0 ? static_cast<int>(a.rpt) : 32 / G, ntile = (group + rpt - 1) / rpt;
  const unsigned units = gridDim.x / static_cast<unsigned>(ntile), nt32 = static_cast<unsigned>(ntile);
  unsigned unit, ct;  // 32-bit mapping (dec_grouped_bh)
  if (a.xmap && gridDim.x % 8 == 0) {
    const unsigned idx = dec_xcd_major(blockIdx.x, gridDim.x);
    unit = idx / nt32;
    ct = idx % nt32;
  } else if (units % 8 == 0) {
    const unsigned slot = blockIdx.x >> 3;
    ct = slot % nt32;
    unit = (slot / nt32) * 8 + (blockIdx.x & 7);
  } else {
    unit = blockIdx.x / nt32;
    ct = blockIdx.x % nt32;
  }
  const unsigned p32 = unit / static_cast<unsigned>(a.Hkv);
  const int64_t p = p32, hd = unit - p32 * static_cast<unsigned>(a.Hkv);
  const int nr = min(rpt, group - static_cast<int>(ct) * rpt);
  const int rl = qi / G, g = qi - rl * G;
  const bool col_ok = rl < nr;
  const int64_t b0 = p * group + ct * rpt;
  const int64_t bcol = b0 + (col_ok ? rl : 0);
  const int qpos = static_cast<int>(a.qpos_ptr ? *a.qpos_ptr : a.qpos);
  const int kend = static_cast<int>(min(a.L, static_cast<int64_t>(qpos) + 1));
  const int64_t panel = vt_panel(a.ld_vt, D, a.ld_k);
  const uint16_t* kbs = a.k + (p * a.Hkv + hd) * a.ld_k * D;
  const uint16_t* vtbs = a.vt + (p * a.Hkv + hd) * panel;
  const uint8_t* vrows = a.valid + p * group * a.ld_valid;
  const int nall = (kend + 31) / 32, nsh = min(static_cast<int>(a.shared / 32), nall);
  const int n_sh = nsh > w ? (nsh - w + NW - 1) / NW : 0;  // shared blocks of class w
  const int nown = nall - nsh;                              // own blocks of every row
  const int nunits = min(nown, NW) * nr;                    // unit u: class index u / nr (class (nsh + u / nr) % NW)
  // own blocks of the class with index j: nsh + j, nsh + j + NW, ...
  auto unit_items = [&](int u) { return (nown - u / nr + NW - 1) / NW; };
  int n_oi = 0;
  for (int u = w; u < nunits; u += NW) n_oi += unit_items(u);
  const int items = n_sh + n_oi;
  // own item jj of this wave -> its unit and its place in the unit (scalar walk over the wave's few units)
  auto locate = [&](int jj, int& u) {
    u = w;
    for (;;) {
      const int n = unit_items(u);
      if (jj < n) break;
      jj -= n;
      u += NW;
    }
    return jj;
  };
  auto load = [&](int j, DecRaw<D>& r) {
    if (j < n_sh) {
      dec_load_raw<D>(kbs, vtbs, vrows, a.ld_vt, a.ld_valid, 32 * (w + j * NW), static_cast<int>(a.ld_k), lane, h, r);
    } else {
      int u;
      const int i = locate(j - n_sh, u);
      const int jc = u / nr, rr = u - jc * nr;
      const int64_t bh = (b0 + rr) * a.Hkv + hd;
      dec_load_raw<D>(a.k + bh * a.ld_k * D, a.vt + bh * panel, a.valid + (b0 + rr) * a.ld_valid, a.ld_vt,
                      a.ld_valid, 32 * (nsh + jc + NW * i), static_cast<int>(a.ld_k), lane, h, r);
    }
  };
  DecRaw<D> R[NB];
  uint16_t* kslot = &s_stage[w][0];
  uint16_t* vslot = kslot + 32 * D;
  if (items > 0) {
#pragma unroll
    for (int j = 0; j < NB; ++j) load(min(j, items - 1), R[j]);
  }
  bf16x8 qf[KS];
  {
    const uint16_t* qrow = a.q + ((bcol * a.Hkv + hd) * a.G + g) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 v = *reinterpret_cast<const u16x8*>(qrow + 16 * s);
      if (!col_ok) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[s] = as_bf16x8(v);
    }
  }
  f32x16 o[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) o[mt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;
  auto save = [&](int cls) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) s_so[cls][mt][r][lane] = o[mt][r];
    s_sm[cls][lane] = m;
    s_sl[cls][lane] = lsum;
  };
  auto restore = [&](int cls) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[mt][r] = s_so[cls][mt][r][lane];
    m = s_sm[cls][lane];
    lsum = s_sl[cls][lane];
  };
  // every wave: its class state after its shared items -> LDS, then one barrier (raw s_barrier: a __syncthreads fence
  // would drain the loads in flight)
  bool crossed = false;
  auto cross = [&] {
    save(w);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    crossed = true;
  };
  int cur_u = -1;
  u32x4* vbslot = reinterpret_cast<u32x4*>(&s_vb[w][0]);
  auto step = [&](int j, DecRaw<D>& R) {
    int row = -1, cls = 0;
    bool last = false;
    if (j >= n_sh && j < items) {
      if (!crossed) cross();
      int u;
      const int i = locate(j - n_sh, u);
      const int jc = u / nr;
      row = u - jc * nr;
      cls = (nsh + jc) % NW;
      if (u != cur_u) {  // the unit's first item: its class state (the previous unit was written back)
        restore(cls);
        cur_u = u;
      }
      last = i == unit_items(u) - 1;
    }
    dec_fix_tail<D>(R, kend, a.ld_valid, lane, h);
    dec_stage<D>(R, kslot, vslot, lane);
    const bool act = j < items && (row < 0 || row == rl);
    vbslot[lane] = act ? u32x4{R.vb[0], R.vb[1], R.vb[2], R.vb[3]} : u32x4{0u, 0u, 0u, 0u};
    load(min(j + NB, items - 1), R);
    const u32x4 v4 = vbslot[lane];
    const uint32_t vb[4] = {v4[0], v4[1], v4[2], v4[3]};
    dec_block_lds<D>(kslot, vslot, vb, qf, a.scale_log2, qi, h, m, lsum, o);
    if (last && rl == row) save(cls);  // row `row`'s columns of the class state
  };
  for (int j = 0; j < items; j += NB) {
#pragma unroll
    for (int i = 0; i < NB; ++i) step(j + i, R[i]);
  }
  if (!crossed) cross();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (!col_ok) return;
  // merge the NW class states per column in class order (decode_group_kernel's merge)
  float mm = -INFINITY;
#pragma unroll
  for (int v = 0; v < NW; ++v) mm = fmaxf(mm, s_sm[v][qi]);
  const float mref = mm == -INFINITY ? 0.f : mm;
  float sc[NW], ll = 0.f;
#pragma unroll
  for (int v = 0; v < NW; ++v) {
    sc[v] = __builtin_amdgcn_exp2f(s_sm[v][qi] - mref);
    ll += (s_sl[v][qi] + s_sl[v][qi + 32]) * sc[v];
  }
  const float inv = ll > 0.f ? 1.f / ll : 0.f;
  const int64_t bh = bcol * a.Hkv + hd;
  const int64_t kq = (hd * a.G + g) * D;
  for (int gg = w; gg < 4 * MT; gg += NW) {
    const int mt = gg >> 2, c = gg & 3;
    u16x4 wv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) acc = fmaf(s_so[v][mt][4 * c + j][lane], sc[v], acc);
      wv[j] = to_bf16_bits(acc * inv);
    }
    const int64_t k = kq + 32 * mt + 8 * c + 4 * h;
    *reinterpret_cast<u16x4*>(dec_out_ptr(a, bcol, k, (bh * a.G + g) * D + 32 * mt + 8 * c + 4 * h)) = wv;
  }
}

}  // namespace

int g_dec_nw = 0, g_dec_splits = 0;  // tuning override (drl_decode_attention_set_plan), 0 = automatic
int g_dq_variant = 0;  // drl_flash_attn_bwd_set_variant: 0 = one query tile per dQ workgroup, 1 = two tiles (K / V in
                       // registers), 2 = two tiles re-reading K / V from LDS. The two-tile kernel measured slower
                       // (update shape: 1227 -> 1474 us per backward, profiles/r06_flash_dq_two_tiles_rejected.jsonl):
                       // 333 registers per lane, one wave per SIMD, where the one-tile kernel runs two workgroups per CU
// drl_decode_group_set_plan: rows per column tile (0 = 32 / G). Items in flight per wave: 2 (3 or 4 spill at 8 waves
// and measured 1.5-3x slower; fewer rows per tile re-read the shared blocks per tile and measured slower too:
// profiles/r06_decode_group_sweep.jsonl)
int g_grp_rpt = 0;
int g_dec_xmap = 0;  // drl_decode_group_set_plan: workgroup -> XCD placement of the decode attention (DecodeArgs::xmap)
int g_grp_bal = -1;               // drl_decode_group_set_plan: own blocks balanced over the waves (-1 = automatic)
int g_dec_lean_depth = 0;  // blocks in flight of the automatic register-lean plan (0 = the planner's choice)
int g_dec_variant = 0;  // drl_decode_attention_set_variant: 1 = one block in flight (LDS fragments), 2..4 = ring depth

// key splits for decode attention. Measured (tools/kernel_bench.py --only decode_sweep, B 64..512,
// L 513..768): a split never beat one workgroup per (sequence, KV head) with 8 waves — the slab hand-off
// costs more than the extra CUs give back at these cache lengths — so splits are only used when a long
// cache leaves the grid short of the chip (more than 64 key blocks per wave group of 8).
int decode_splits(int64_t B, int64_t Hkv, int64_t L) {
  if (g_dec_splits) return g_dec_splits;
  const int64_t wgs = B * Hkv, cus = cu_count();
  int s = 1;
  while (s < 8 && wgs * s * 2 <= cus && L / (32 * 8 * 2 * s) >= 8) s *= 2;
  return s;
}

}  // namespace drl

extern "C" {

int drl_flash_attn_fwd(const void* q, const void* k, const void* vt, int32_t dt, const uint8_t* key_valid,
                       int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t Tq, int64_t Tk,
                       int64_t ld_k, int64_t ld_vt, int64_t qoff, const int32_t* q_start, float scale, void* out,
                       float* lse, void* stream) {
  return drl_flash_attn_fwd_rows(q, k, vt, dt, key_valid, ld_valid, B, Hkv, G, D, Tq, Tk, ld_k, ld_vt, qoff, q_start,
                                 scale, out, nullptr, lse, stream);
}

int drl_flash_attn_fwd_rows(const void* q, const void* k, const void* vt, int32_t dt, const uint8_t* key_valid,
                            int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t Tq, int64_t Tk,
                            int64_t ld_k, int64_t ld_vt, int64_t qoff, const int32_t* q_start, float scale, void* out,
                            const int64_t* out_row, float* lse, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(q && k && vt && key_valid && out, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "flash attention runs on bf16 operands");
  DRL_CHECK_ARG(D == 64 || D == 128, "head_dim must be 64 or 128");
  DRL_CHECK_ARG(B >= 1 && Hkv >= 1 && G >= 1 && G <= 8 && Tq >= 1 && Tk >= 1 && qoff >= 0, "bad shape");
  DRL_CHECK_ARG(ld_vt == DRL_VT_BLOCKED || (ld_vt >= Tk && ld_vt % 8 == 0),
                "ld_vt must be >= Tk and a multiple of 8 (or DRL_VT_BLOCKED)");
  DRL_CHECK_ARG(ld_k >= Tk, "ld_k < Tk");
  DRL_CHECK_ARG(Tk + qoff < (int64_t(1) << 30), "positions must fit in 32 bits");
  DRL_CHECK_ARG(ld_valid >= Tk && ld_valid % 4 == 0 && (reinterpret_cast<uintptr_t>(key_valid) & 3u) == 0,
                "key_valid rows must be 4-byte aligned");
  DRL_CHECK_ARG(aligned16(q) && aligned16(k) && aligned16(vt) && (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                "misaligned operand");
  FlashArgs a{static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k), static_cast<const uint16_t*>(vt),
              key_valid, ld_valid, static_cast<uint16_t*>(out), lse, Hkv, G, Tq, Tk, ld_k, ld_vt, qoff,
              scale * 1.4426950408889634f, q_start, out_row};
  const dim3 grid(static_cast<unsigned>((Tq + 31) / 32), static_cast<unsigned>(B * Hkv));
  const dim3 block(512);  // waves >= G stage K/V only
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (D == 64) hipLaunchKernelGGL(flash_fwd_kernel<64>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(flash_fwd_kernel<128>, grid, block, 0, s, a);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

int drl_flash_attn_bwd(const void* q, const void* k, const void* kt, const void* v, const void* o, const void* dout,
                       const float* lse, int32_t dt, const uint8_t* key_valid, int64_t ld_valid, int64_t B,
                       int64_t Hkv, int64_t G, int64_t D, int64_t T, int64_t ld_t, const int32_t* q_start, float scale,
                       float* delta, void* dq, void* dk, void* dv, void* stream) {
  return drl_flash_attn_bwd_rows(q, k, kt, v, o, nullptr, dout, lse, dt, key_valid, ld_valid, B, Hkv, G, D, T, ld_t,
                                 q_start, scale, delta, dq, dk, dv, stream);
}

int drl_flash_attn_bwd_rows(const void* q, const void* k, const void* kt, const void* v, const void* o,
                            const int64_t* o_row, const void* dout, const float* lse, int32_t dt,
                            const uint8_t* key_valid, int64_t ld_valid, int64_t B, int64_t Hkv, int64_t G, int64_t D,
                            int64_t T, int64_t ld_t, const int32_t* q_start, float scale, float* delta, void* dq,
                            void* dk, void* dv, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(q && k && kt && v && o && dout && lse && key_valid && delta && dq && dk && dv,
                "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "flash attention runs on bf16 operands");
  DRL_CHECK_ARG(D == 64 || D == 128, "the fused backward supports head_dim 64 and 128");
  DRL_CHECK_ARG(B >= 1 && Hkv >= 1 && G >= 1 && G <= 8 && T >= 1, "bad shape");
  DRL_CHECK_ARG(T % 8 == 0 && ld_t >= T && ld_t % 8 == 0, "T and ld_t must be multiples of 8");
  DRL_CHECK_ARG(ld_valid >= T, "ld_valid < T");
  FlashBwdArgs a{static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k), static_cast<const uint16_t*>(kt),
                 static_cast<const uint16_t*>(v), static_cast<const uint16_t*>(o), static_cast<const uint16_t*>(dout),
                 lse, key_valid, ld_valid, delta, static_cast<uint16_t*>(dq), static_cast<uint16_t*>(dk),
                 static_cast<uint16_t*>(dv), Hkv, G, T, ld_t, scale, scale * 1.4426950408889634f, q_start, o_row};
  const dim3 grid(static_cast<unsigned>((T + 31) / 32), static_cast<unsigned>(B * Hkv));
  constexpr int kDqWaves = DQ_WAVES, kDkdvWaves64 = DKDV_WAVES64, kKT64 = DKDV_KT64;
  const dim3 grid_kv64(static_cast<unsigned>((T + 32 * kKT64 - 1) / (32 * kKT64)), static_cast<unsigned>(B * Hkv));
  const dim3 grid_dq(static_cast<unsigned>((T + 31) / 32),
                     static_cast<unsigned>(B * Hkv * ((G + kDqWaves - 1) / kDqWaves)));
  const dim3 block_dq(64 * kDqWaves);  // waves >= G only stage K / V / K^T
  const dim3 block_kv(static_cast<unsigned>(64 * std::min<int64_t>(G, D == 64 ? kDkdvWaves64 : 4)));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // dQ over one query tile per workgroup; the two-tile form (flash_dq2_kernel) on request (A/B); head_dim 64
  const dim3 grid_dq2(static_cast<unsigned>(((T + 31) / 32 + 1) / 2),
                      static_cast<unsigned>(B * Hkv * ((G + kDqWaves - 1) / kDqWaves)));
  if (D == 64) {
    if (g_dq_variant == 1) hipLaunchKernelGGL((flash_dq2_kernel<64, kDqWaves, 1>), grid_dq2, block_dq, 0, s, a);
    else if (g_dq_variant == 2) hipLaunchKernelGGL((flash_dq2_kernel<64, kDqWaves, 0>), grid_dq2, block_dq, 0, s, a);
    else hipLaunchKernelGGL((flash_dq_kernel<64, kDqWaves>), grid_dq, block_dq, 0, s, a);
    hipLaunchKernelGGL((flash_dkdv_kernel<64, kDkdvWaves64, kKT64>), grid_kv64, block_kv, 0, s, a);
  } else {
    hipLaunchKernelGGL((flash_dq_kernel<128, kDqWaves>), grid_dq, block_dq, 0, s, a);
    hipLaunchKernelGGL((flash_dkdv_kernel<128, 4>), grid, block_kv, 0, s, a);
  }
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

void drl_flash_attn_bwd_set_variant(int32_t variant) { drl::g_dq_variant = (variant >= 0 && variant <= 2) ? variant : 0; }

void drl_decode_attention_set_variant(int32_t variant) {
  drl::g_dec_variant = (variant >= 1 && variant <= 5) ? variant : 0;
}

void drl_decode_group_set_plan(int32_t rows_per_tile, int32_t xcd_map, int32_t balanced) {
  drl::g_grp_rpt = rows_per_tile >= 1 && rows_per_tile <= 32 ? rows_per_tile : 0;
  drl::g_dec_xmap = xcd_map == 1 ? 1 : 0;
  drl::g_grp_bal = balanced == 0 || balanced == 1 ? balanced : -1;
}

void drl_decode_attention_set_plan(int32_t waves, int32_t splits) {
  drl::g_dec_nw = (waves == 2 || waves == 4 || waves == 8 || waves == 16) ? waves : 0;
  drl::g_dec_splits = (splits >= 1 && splits <= 16) ? splits : 0;
}

size_t drl_decode_attention_vt_workspace_bytes(int64_t B, int64_t Hkv, int64_t D, int64_t L) {
  const int splits = drl::decode_splits(B, Hkv, L);
  if (splits == 1) return 0;
  return drl::round_up(static_cast<size_t>(B * Hkv) * sizeof(unsigned), 256) +
         static_cast<size_t>(B * Hkv) * splits * (64 + 32 * D) * sizeof(float);
}

int drl_decode_attention_vt(const void* q, const void* k_cache, const void* vt_cache, int32_t dt,
                            const uint8_t* key_valid, int64_t ld_valid, const int64_t* qpos_ptr, int64_t qpos,
                            int64_t B, int64_t Hkv, int64_t G, int64_t D, int64_t ld_k, int64_t ld_vt, int64_t L,
                            int64_t group, int64_t shared_keys, float scale, void* out, int64_t out_mbt,
                            void* workspace, size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(q && k_cache && vt_cache && key_valid && out, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "MFMA decode attention runs on bf16");
  DRL_CHECK_ARG(out_mbt == 0 || out_mbt * 32 >= B, "out_mbt too small for B rows");
  DRL_CHECK_ARG(D == 64 || D == 128, "head_dim must be 64 or 128");
  DRL_CHECK_ARG(B >= 1 && Hkv >= 1 && G >= 1 && G <= 32 && L >= 1 && L <= ld_k &&
                    (ld_vt == DRL_VT_BLOCKED || L <= ld_vt), "bad shape");
  DRL_CHECK_ARG(ld_vt % 8 == 0 && ld_valid % 4 == 0 && (reinterpret_cast<uintptr_t>(key_valid) & 3u) == 0 &&
                    ld_k < (int64_t(1) << 30),
                "ld_vt must be a multiple of 8 and key_valid rows 4-byte aligned");
  DRL_CHECK_ARG(aligned16(q) && aligned16(k_cache) && aligned16(vt_cache) && (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                "misaligned operand (q, caches 16-byte aligned)");
  DRL_CHECK_ARG(ld_k * D * 2 < (int64_t(1) << 31) && vt_panel(ld_vt, D, ld_k) * 2 < (int64_t(1) << 31) &&
                    ld_valid < (int64_t(1) << 31),
                "one sequence's K / V^T panel and key-valid row must be below 2 GB (31-bit buffer offsets)");
  DRL_CHECK_ARG(group >= 1 && B % group == 0 && shared_keys >= 0 && shared_keys % 32 == 0 && shared_keys <= L &&
                    (group > 1 || shared_keys == 0),
                "prompt groups: group must divide B, shared_keys a multiple of 32 within L (0 without groups)");
  DecodeArgs a{static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k_cache),
               static_cast<const uint16_t*>(vt_cache), key_valid, ld_valid, qpos_ptr, qpos, Hkv, G, ld_k, ld_vt, L,
               scale * 1.4426950408889634f, static_cast<uint16_t*>(out), out_mbt, nullptr, nullptr, group,
               shared_keys, 0, g_dec_xmap};
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rpt0 = static_cast<int>(32 / G), ntile0 = static_cast<int>((group + rpt0 - 1) / rpt0);
  if (group > 1 && shared_keys > 0 && B / group * Hkv * ntile0 * 2 >= cu_count()) {
    // prompt groups: one workgroup per (prompt, KV head, column tile of 32 / G rows), each shared block loaded once
    // per tile (decode_group_kernel); bit-identical to the per-row kernel at the same wave count without splits.
    // 8 waves (D = 64; 4 at D = 128) so a workgroup's key blocks are spread over as many in-flight loads as the
    // per-row 8-wave plan (profiles/r04_decode_group.jsonl: 512 rows, 640 keys: 14.9 us against 25.1 for the
    // per-row kernel reading the prompt rows). Below half a workgroup per CU (64 rows: 32 workgroups) the per-row
    // kernel's one workgroup per (row, KV head) keeps more of the chip busy: 0.304 vs 0.331 s per 64-row rollout
    const int nwg = g_dec_nw ? g_dec_nw : (D == 64 ? 8 : 4);
    DRL_CHECK_ARG(D == 64 ? (nwg == 2 || nwg == 4 || nwg == 8 || nwg == 16) : (nwg == 2 || nwg == 4),
                  "prompt-group decode attention: %d waves at head_dim %lld", nwg, (long long)D);
    const int rpt = g_grp_rpt ? std::min(g_grp_rpt, rpt0) : rpt0, ntile = static_cast<int>((group + rpt - 1) / rpt);
    a.rpt = rpt;
    const dim3 g_(static_cast<unsigned>(B / group * Hkv * ntile)), b_(64 * nwg);
    // balanced own blocks: bit-identical but measured slower at every cache length of the bench (512 rows, L 520..767:
    // 13.3 / 14.2 / 15.3 / 20.4 / 22.1 against 13.1 / 13.6 / 12.9 / 18.0 / 20.1 us, profiles/r06_decode_group_sweep.jsonl):
    // the items on a wave's path are not what bounds the call; on request only
    const bool bal = g_grp_bal == 1;
    if (bal && D == 64 && (nwg == 4 || nwg == 8)) {
      if (nwg == 4) hipLaunchKernelGGL((decode_group_bal_kernel<64, 4>), g_, b_, 0, s, a);
      else hipLaunchKernelGGL((decode_group_bal_kernel<64, 8>), g_, b_, 0, s, a);
    } else if (bal && D == 128 && nwg == 4) {
      hipLaunchKernelGGL((decode_group_bal_kernel<128, 4>), g_, b_, 0, s, a);
    } else if (D == 64) {
      if (nwg == 2) hipLaunchKernelGGL((decode_group_kernel<64, 2>), g_, b_, 0, s, a);
      else if (nwg == 4) hipLaunchKernelGGL((decode_group_kernel<64, 4>), g_, b_, 0, s, a);
      else if (nwg == 8) hipLaunchKernelGGL((decode_group_kernel<64, 8>), g_, b_, 0, s, a);
      else hipLaunchKernelGGL((decode_group_kernel<64, 16>), g_, b_, 0, s, a);
    } else {
      if (nwg == 2) hipLaunchKernelGGL((decode_group_kernel<128, 2>), g_, b_, 0, s, a);
      else hipLaunchKernelGGL((decode_group_kernel<128, 4>), g_, b_, 0, s, a);
    }
    DRL_LAUNCH_CHECK();
    return DRL_OK;
  }
  const int64_t wgs = B * Hkv, cus = cu_count();
  const int splits = decode_splits(B, Hkv, L);
  // waves per workgroup and key-loop variant (tools/kernel_bench.py --only decode_sweep): 8 waves with two
  // blocks in flight while the grid fits the chip (B=64: 8.7 us at L=768, latency-bound); beyond it the
  // register-lean loop (2 waves per SIMD) with 4 waves up to 2 workgroups per CU, else 2 (B=512, L=768:
  // 201 MB in 34.7 us = 5.8 TB/s, 0.92 of the measured 6.3 TB/s copy rate)
  // round 2, caches cold as in the rollout (24 layers' caches >> the 256 MB MALL; tools/kernel_bench.py --only
  // decode_cold, L=640): the register-lean loop at every grid, 8 waves up to one workgroup per CU (B=64:
  // 11.5 -> 9.7 us, B=128: 15.0 -> 12.0); 4 waves measured 35.8 vs 37.3 us at B=512 in isolation but 41.9 vs
  // 39.3 in the rollout (rocprof), so 2 waves beyond two workgroups per CU
  const int nw = g_dec_nw ? g_dec_nw : (wgs <= cus ? 8 : (wgs <= 2 * cus ? 4 : 2));
  const bool lean = g_dec_nw ? (g_dec_variant == 1 || g_dec_variant >= 5) : true;
  // blocks in flight per wave (small grids): all of a wave's blocks at the cache capacity, up to 4
  const int64_t per_wave = ((L + 31) / 32 + nw - 1) / nw;
  const int nb = g_dec_nw ? (g_dec_variant > 2 ? g_dec_variant : 2) : (per_wave >= 4 ? 4 : per_wave >= 3 ? 3 : 2);
  // blocks in flight per wave of the register-lean loop: 1. Two (variant 5 of a forced plan; 3 spill at 8 waves' 256
  // registers) measured slower at the N = 8 rank's 64 rows: 7.1 -> 8.8 / 7.3 -> 8.4 / 8.6 -> 10.9 us per call at L = 520 /
  // 640 / 767, 206 -> 254 us per token in situ (profiles/r06_decode_attn_lean2_rejected.jsonl, profiles/r06_decode_step_64rows_lean2_rejected.txt): the phantom step that
  // pads a wave's 2-3 blocks to the ring and the key-valid hand-off through LDS cost more than the overlap gives
  const int ldepth = g_dec_nw ? (g_dec_variant == 5 ? 2 : 1) : (g_dec_lean_depth ? g_dec_lean_depth : 1);
  if (splits > 1) {
    const size_t need = drl_decode_attention_vt_workspace_bytes(B, Hkv, D, L);
    if (!workspace || workspace_bytes < need || (reinterpret_cast<uintptr_t>(workspace) & 255u))
      return fail(DRL_ERR_WORKSPACE, "decode attention workspace: need %zu bytes, 256-byte aligned, zeroed", need);
    a.tickets = static_cast<unsigned*>(workspace);
    a.slabs = reinterpret_cast<float*>(static_cast<char*>(workspace) + round_up(static_cast<size_t>(wgs) * sizeof(unsigned), 256));
  }
#define DRL_DEC(DD, NN)                                                                                          \
  do {                                                                                                           \
    const dim3 g_(B * Hkv, splits), b_(64 * NN);                                                                  \
    if (splits > 1) hipLaunchKernelGGL((decode_mfma_kernel<DD, NN, false, true>), g_, b_, 0, s, a);              \
    else if (lean && ldepth >= 2 && DD == 64 && NN == 8)                                                         \
      hipLaunchKernelGGL((decode_mfma_kernel<DD, NN, true, false, 2, 2>), g_, b_, 0, s, a);                      \
    else if (lean) hipLaunchKernelGGL((decode_mfma_kernel<DD, NN, true, false>), g_, b_, 0, s, a);              \
    else {                                                                                                       \
      bool done_ = false;                                                                                        \
      if constexpr (DD == 64 && (NN == 4 || NN == 8)) {                                                          \
        done_ = nb >= 3;                                                                                         \
        if (nb == 3) hipLaunchKernelGGL((decode_mfma_kernel<DD, NN, false, false, 3>), g_, b_, 0, s, a);         \
        else if (nb >= 4) hipLaunchKernelGGL((decode_mfma_kernel<DD, NN, false, false, 4>), g_, b_, 0, s, a);    \
      }                                                                                                          \
      if (!done_) hipLaunchKernelGGL((decode_mfma_kernel<DD, NN, false, false>), g_, b_, 0, s, a);               \
    }                                                                                                            \
  } while (0)
  if (D == 64) {
    if (nw == 2) DRL_DEC(64, 2);
    else if (nw == 4) DRL_DEC(64, 4);
    else if (nw == 8) DRL_DEC(64, 8);
    else DRL_DEC(64, 16);
  } else {
    if (nw == 2) DRL_DEC(128, 2);
    else DRL_DEC(128, 4);  // D=128 at 8+ waves would spill
  }
#undef DRL_DEC
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
