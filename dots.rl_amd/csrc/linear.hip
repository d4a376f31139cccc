// Weight-streaming linear layer for the decode step (few token rows): y (M, N) = x (M, K) · W^T (+ bias),
// W (N, K) row-major (the nn.Linear layout), bf16 operands, fp32 accumulation on v_mfma_f32_32x32x16_bf16.
//
// Decoding one token per sequence turns every projection of the layer into a GEMM with M = the rank's
// rollout rows (64 per GPU at DP=8) where library GEMMs sit on a ~10 µs latency floor (one workgroup per
// output tile walking K serially). Here the K loop is spread instead: a workgroup owns 32 rows of W and a
// block of token rows, its 16 waves split K so each wave issues all loads of its slice at once (one HBM
// round trip; W is streamed nontemporal, x is L2-resident), and long K (down_proj, K = 4864) is further
// split over workgroups. Partials meet in a fixed order — waves through LDS, K-split workgroups through
// write-through slabs taken by the last arriver of a ticket — so the result is bitwise reproducible.
// The epilogue fuses the bias (qkv_proj) or SwiGLU (gate_up_proj: the workgroup's 32 rows are 16 gate rows
// and the matching 16 up rows, so the (M, 2I) gate|up activation is never written).
// Roofline: HBM-bound on the weight stream, algorithmic bytes = 2·N·K + 2·M·K + 2·M·N_out per call.
//
// MFMA operand mapping (A = W tile, B = x^T): lane l feeds A row l&31 and B column l&31 with k = 8(l>>5)+j;
// C column (token row) = l&31, C row (W row) = (r&3) + 8(r>>2) + 4(l>>5) for accumulator register r.
#include "common.h"

namespace drl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ uint16_t to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }
__device__ __forceinline__ float bf16r(float f) { return bf16_to_f32(to_bf16_bits(f)); }

struct LinearArgs {
  const uint16_t* x;
  int64_t ld_x;
  const uint16_t* w;
  const uint16_t* bias;
  uint16_t* out;
  int64_t ld_out;
  int M, N, K;
  int half;       // SwiGLU: I (W rows = [gate (I) | up (I)])
  int tiles;      // workgroup tiles along N
  int ksplit;     // workgroups along K (gridDim.y)
  float* slabs;   // ksplit x tiles x mblocks x (32*MB*32) fp32 partials (ksplit > 1)
  unsigned* tickets;  // tiles x mblocks arrival counters, zero between launches
};

// C row i (0..31) of the 32x32 tile <-> (accumulator register, lane half)
__device__ __forceinline__ int reg_of_row(int i) { return (i & 3) + 4 * (i >> 3); }
__device__ __forceinline__ int half_of_row(int i) { return (i >> 2) & 1; }

template <int EPI>
__device__ __forceinline__ void store_out(const LinearArgs& a, int tile, int m, int i, float v, float v_up) {
  if (m >= a.M) return;
  if constexpr (EPI == DRL_LINEAR_SWIGLU) {
    const int n = tile * 16 + i;
    if (n >= a.half) return;
    const float g = bf16r(v), u = bf16r(v_up);
    a.out[static_cast<int64_t>(m) * a.ld_out + n] = to_bf16_bits(bf16r(silu_fast(g)) * u);
  } else {
    const int n = tile * 32 + i;
    if (n >= a.N) return;
    if constexpr (EPI == DRL_LINEAR_BIAS) v += bf16_to_f32(a.bias[n]);
    a.out[static_cast<int64_t>(m) * a.ld_out + n] = to_bf16_bits(v);
  }
}

// KW waves split this workgroup's K range; each wave loads up to S k-steps (16 deep) per round trip.
template <int MB, int KW, int EPI>
__global__ __launch_bounds__(64 * KW) void linear_decode_kernel(LinearArgs a) {
  constexpr int NT = 64 * KW;
  constexpr int S = MB == 1 ? 8 : (MB == 2 ? 4 : 2);  // register budget: S * (1 + MB) * 4 VGPRs in flight
  __shared__ float red[KW][16][65];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x, ks = blockIdx.y, mblk = blockIdx.z;
  const int m_base = mblk * 32 * MB;

  int wrow;
  if constexpr (EPI == DRL_LINEAR_SWIGLU) wrow = r < 16 ? tile * 16 + r : a.half + tile * 16 + (r - 16);
  else wrow = tile * 32 + r;
  const bool wok = wrow < a.N;
  const uint16_t* wp = a.w + static_cast<int64_t>(wok ? wrow : 0) * a.K + 8 * h;
  const uint16_t* xp[MB];
  bool xok[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m_base + 32 * mb + r;
    xok[mb] = m < a.M;
    xp[mb] = a.x + static_cast<int64_t>(xok[mb] ? m : 0) * a.ld_x + 8 * h;
  }
  const int nsteps = a.K >> 4;
  const int g0 = ks * nsteps / a.ksplit, g1 = (ks + 1) * nsteps / a.ksplit;
  const int s0 = g0 + wave * (g1 - g0) / KW, s1 = g0 + (wave + 1) * (g1 - g0) / KW;

  f32x16 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = f32x16{};
  const u16x8 zero{};
  for (int s = s0; s < s1; s += S) {
    u16x8 wv[S], xv[S][MB];
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const bool in = s + u < s1;
      wv[u] = (in && wok) ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp + 16 * (s + u))) : zero;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        xv[u][mb] = (in && xok[mb]) ? *reinterpret_cast<const u16x8*>(xp[mb] + 16 * (s + u)) : zero;
    }
#pragma unroll
    for (int u = 0; u < S; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wv[u]), as_bf16x8(xv[u][mb]), acc[mb], 0, 0, 0);
      }
    }
  }

  const bool split = a.ksplit > 1;
  const int mblocks = gridDim.z;
  float* slab = split ? a.slabs + ((static_cast<int64_t>(ks) * a.tiles + tile) * mblocks + mblk) * (1024 * MB) : nullptr;
  // wave partials meet in LDS (fixed order), one 32-token block at a time; element e = token (e>>5), row (e&31)
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][q][lane] = acc[mb][q];
    __syncthreads();
    if (split) {
      for (int e = tid; e < 1024; e += NT) {
        const int ml = e >> 5, i = e & 31;
        const int q = reg_of_row(i), ln = ml + 32 * half_of_row(i);
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < KW; ++w) v += red[w][q][ln];
        store_f32_sc1(slab + mb * 1024 + e, v);
      }
    } else if constexpr (EPI == DRL_LINEAR_SWIGLU) {
      for (int e = tid; e < 512; e += NT) {
        const int ml = e >> 4, i = e & 15;
        const int q = reg_of_row(i), ln = ml + 32 * half_of_row(i);
        float g = 0.f, u = 0.f;
#pragma unroll
        for (int w = 0; w < KW; ++w) {
          g += red[w][q][ln];
          u += red[w][q + 8][ln];
        }
        store_out<EPI>(a, tile, m_base + 32 * mb + ml, i, g, u);
      }
    } else {
      for (int e = tid; e < 1024; e += NT) {
        const int ml = e >> 5, i = e & 31;
        const int q = reg_of_row(i), ln = ml + 32 * half_of_row(i);
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < KW; ++w) v += red[w][q][ln];
        store_out<EPI>(a, tile, m_base + 32 * mb + ml, i, v, 0.f);
      }
    }
    __syncthreads();
  }
  if (!split) return;

  // K-split: the last of the ksplit workgroups of this (tile, token block) sums the slabs in ks order
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ticket = a.tickets + tile * mblocks + mblk;
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add((gu32_t*)(ticket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == static_cast<unsigned>(a.ksplit - 1);
  }
  __syncthreads();
  if (!s_last) return;
  const int64_t kstride = static_cast<int64_t>(a.tiles) * mblocks * (1024 * MB);
  const float* base = a.slabs + (static_cast<int64_t>(tile) * mblocks + mblk) * (1024 * MB);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    if constexpr (EPI == DRL_LINEAR_SWIGLU) {
      for (int e = tid; e < 512; e += NT) {
        const int ml = e >> 4, i = e & 15;
        float g = 0.f, u = 0.f;
        for (int k = 0; k < a.ksplit; ++k) {
          g += load_f32_sc1(base + k * kstride + mb * 1024 + ml * 32 + i);
          u += load_f32_sc1(base + k * kstride + mb * 1024 + ml * 32 + i + 16);
        }
        store_out<EPI>(a, tile, m_base + 32 * mb + ml, i, g, u);
      }
    } else {
      for (int e = tid; e < 1024; e += NT) {
        float v = 0.f;
        for (int k = 0; k < a.ksplit; ++k) v += load_f32_sc1(base + k * kstride + mb * 1024 + e);
        store_out<EPI>(a, tile, m_base + 32 * mb + (e >> 5), e & 31, v, 0.f);
      }
    }
  }
  if (tid == 0) __hip_atomic_store((gu32_t*)(ticket), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct LinearPlan {
  int mb, kw, mblocks, tiles, ksplit;
};

int g_plan_kw = 0, g_plan_ks = 0;  // tuning override (drl_linear_decode_set_plan), 0 = automatic

LinearPlan plan_linear(int64_t M, int64_t N, int64_t K, int epilogue) {
  LinearPlan p{};
  p.mb = M <= 32 ? 1 : (M <= 64 ? 2 : 4);
  p.mblocks = static_cast<int>((M + 32 * p.mb - 1) / (32 * p.mb));
  p.tiles = static_cast<int>(epilogue == DRL_LINEAR_SWIGLU ? (N / 2 + 15) / 16 : (N + 31) / 32);
  const int64_t nsteps = K / 16;
  const int64_t wgs = static_cast<int64_t>(p.tiles) * p.mblocks;
  // 4 waves per workgroup; split K over workgroups until the grid covers the chip or a wave would get
  // fewer than 2 k-steps
  p.kw = 4;
  int ks = 1;
  while (wgs * ks * 2 <= cu_count() && nsteps / (2 * ks * p.kw) >= 2 && ks < 16) ks *= 2;
  p.ksplit = ks;
  if (g_plan_kw) p.kw = g_plan_kw;
  if (g_plan_ks) p.ksplit = static_cast<int>(g_plan_ks < nsteps ? g_plan_ks : nsteps);
  return p;
}

template <int EPI, int KW>
void launch_linear_kw(const LinearArgs& a, const LinearPlan& p, hipStream_t s) {
  const dim3 grid(p.tiles, p.ksplit, p.mblocks);
  if (p.mb == 1) hipLaunchKernelGGL((linear_decode_kernel<1, KW, EPI>), grid, dim3(64 * KW), 0, s, a);
  else if (p.mb == 2) hipLaunchKernelGGL((linear_decode_kernel<2, KW, EPI>), grid, dim3(64 * KW), 0, s, a);
  else hipLaunchKernelGGL((linear_decode_kernel<4, KW, EPI>), grid, dim3(64 * KW), 0, s, a);
}

template <int EPI>
void launch_linear(const LinearArgs& a, const LinearPlan& p, hipStream_t s) {
  if (p.kw == 16) launch_linear_kw<EPI, 16>(a, p, s);
  else if (p.kw == 8) launch_linear_kw<EPI, 8>(a, p, s);
  else launch_linear_kw<EPI, 4>(a, p, s);
}

}  // namespace
}  // namespace drl

extern "C" {

void drl_linear_decode_set_plan(int32_t waves, int32_t ksplit) {
  drl::g_plan_kw = (waves == 4 || waves == 8 || waves == 16) ? waves : 0;
  drl::g_plan_ks = ksplit > 0 ? ksplit : 0;
}

size_t drl_linear_decode_workspace_bytes(int64_t M, int64_t N, int64_t K, int32_t epilogue) {
  using namespace drl;
  if (M < 1 || N < 1 || K < 16) return 0;
  const LinearPlan p = plan_linear(M, N, K, epilogue);
  if (p.ksplit == 1) return 0;
  const size_t tickets = round_up(static_cast<size_t>(p.tiles) * p.mblocks * sizeof(unsigned), 256);
  return tickets + static_cast<size_t>(p.ksplit) * p.tiles * p.mblocks * 1024 * p.mb * sizeof(float);
}

int drl_linear_decode(const void* x, int64_t ld_x, const void* w, const void* bias, int32_t dt, int64_t M,
                      int64_t N, int64_t K, int32_t epilogue, void* out, int64_t ld_out, void* workspace,
                      size_t workspace_bytes, void* stream) {
  using namespace drl;
  DRL_CHECK_ARG(x && w && out, "NULL input");
  DRL_CHECK_ARG(dt == DRL_BF16, "the decode linear runs on bf16 operands");
  DRL_CHECK_ARG(M >= 1 && M <= 128, "the decode linear takes 1..128 token rows (M=%lld)", (long long)M);
  DRL_CHECK_ARG(N >= 1 && K >= 16 && N < (1 << 30) && K < (1 << 24), "bad shape");
  DRL_CHECK_ARG(K % 16 == 0, "K must be a multiple of 16");
  DRL_CHECK_ARG(ld_x >= K && ld_x % 8 == 0 && aligned16(x) && aligned16(w), "x rows / W must be 16-byte aligned");
  DRL_CHECK_ARG(epilogue == DRL_LINEAR_NONE || epilogue == DRL_LINEAR_BIAS || epilogue == DRL_LINEAR_SWIGLU,
                "unknown epilogue");
  DRL_CHECK_ARG(epilogue != DRL_LINEAR_BIAS || bias, "BIAS epilogue needs a bias");
  DRL_CHECK_ARG(epilogue != DRL_LINEAR_SWIGLU || N % 2 == 0, "SWIGLU needs W = [gate | up] (even N)");
  const int64_t n_out = epilogue == DRL_LINEAR_SWIGLU ? N / 2 : N;
  DRL_CHECK_ARG(ld_out >= n_out, "ld_out < output width");
  const LinearPlan p = plan_linear(M, N, K, epilogue);
  const size_t need = drl_linear_decode_workspace_bytes(M, N, K, epilogue);
  if (need && (!workspace || workspace_bytes < need || (reinterpret_cast<uintptr_t>(workspace) & 255u)))
    return fail(DRL_ERR_WORKSPACE, "linear workspace: need %zu bytes, 256-byte aligned, tickets zeroed", need);
  LinearArgs a{static_cast<const uint16_t*>(x), ld_x, static_cast<const uint16_t*>(w),
               static_cast<const uint16_t*>(bias), static_cast<uint16_t*>(out), ld_out, static_cast<int>(M),
               static_cast<int>(N), static_cast<int>(K), static_cast<int>(N / 2), p.tiles, p.ksplit, nullptr, nullptr};
  if (need) {
    a.tickets = static_cast<unsigned*>(workspace);
    a.slabs = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                       round_up(static_cast<size_t>(p.tiles) * p.mblocks * sizeof(unsigned), 256));
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (epilogue == DRL_LINEAR_NONE) launch_linear<DRL_LINEAR_NONE>(a, p, s);
  else if (epilogue == DRL_LINEAR_BIAS) launch_linear<DRL_LINEAR_BIAS>(a, p, s);
  else launch_linear<DRL_LINEAR_SWIGLU>(a, p, s);
  DRL_LAUNCH_CHECK();
  return DRL_OK;
}

}  // extern "C"
