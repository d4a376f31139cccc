// Decode-step GEMM probe: y (M, N) = x (M, K) W^T at M = 64 token rows, W (N, K) bf16 streamed once.
// Where does a small-M GEMM launch spend its ~10 us? Variants of one workgroup shape (32 W rows per
// workgroup, 4 waves splitting K, everything issued in one round trip), timed over back-to-back launches
// that rotate through > 512 MB of weight copies (every call streams its W from HBM):
//   mode 0: W only (fragment-shaped loads, x = constant), MFMA, LDS reduce, bf16 store   -> the W floor
//   mode 1: W + x both fragment-shaped direct loads
//   mode 2: W fragment loads + x staged to LDS by global_load_lds in full 128-B lines
//   mode 3: W only, nothing computed or reduced: loads + one store per wave              -> launch + HBM floor
//   mode 4: empty workgroups (launch floor at this grid)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/wsgemm_probe tools/wsgemm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#ifndef SCHED_PIN
#define SCHED_PIN 1
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }

// KS = k16-steps per wave (K / 16 / 4 waves / ksplit); MB = 32-token blocks
template <int MODE, int KS, int MB>
__global__ __launch_bounds__(256) void probe(const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
                                             unsigned short* __restrict__ y, int N, int K, int M) {
  __shared__ __attribute__((aligned(16))) unsigned short xs[(MODE == 2) ? MB * 32 * KS * 16 * 4 : 8];
  __shared__ float red[4][16][65 * MB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x;
  if constexpr (MODE == 4) {
    if (tid == 0 && tile == 0) y[0] = 0;
    return;
  }
  const int kw0 = wave * KS * 16;  // this wave's first k
  const unsigned short* wp = w + (long)(tile * 32 + r) * K + kw0 + 8 * h;
  u16x8 wv[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) wv[s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp + 16 * s));
#if SCHED_PIN
  __builtin_amdgcn_sched_barrier(0);  // keep every W load issued before the first use (one round trip)
#endif
  if constexpr (MODE == 3 || MODE == 7 || MODE == 8) {
    u16x8 acc = wv[0];
#pragma unroll
    for (int s = 1; s < KS; ++s) acc ^= wv[s];
    if constexpr (MODE == 3) {
      if (lane == 0) y[tile * 4 + wave] = acc[0] ^ acc[7];
    } else if constexpr (MODE == 7) {  // one 16-B store per lane: 1 KB contiguous per wave
      *reinterpret_cast<u16x8*>(y + (long)(tile * 4 + wave) * 512 + lane * 8) = acc;
    } else {  // mode 0's output pattern (8 scattered 2-B stores per thread) without MFMA / LDS
      for (int e = tid; e < 1024 * MB; e += 256) {
        const int tok = e >> 5, i = e & 31;
        y[(long)tok * N + tile * 32 + i] = acc[e & 7];
      }
    }
    return;
  }
  u16x8 xv[KS][MB];
  const u16x8 one = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
  if constexpr (MODE == 1) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        xv[s][mb] = *reinterpret_cast<const u16x8*>(x + (long)(mb * 32 + r) * K + kw0 + 8 * h + 16 * s);
#if SCHED_PIN
    __builtin_amdgcn_sched_barrier(0);
#endif
  } else if constexpr (MODE == 2) {
    // the workgroup's x slice: M rows x (4 * KS * 16) columns of k starting at 0; rows of KS*16*4 elements.
    // glds: 1 KB per wave-instruction = 64 lanes x 16 B along a row (lane-linear); row length 4*KS*16*2 B
    constexpr int ROW = 4 * KS * 16;         // elements per LDS row
    constexpr int UNITS = ROW / 8;           // 16-B units per row
    constexpr int TOTAL = MB * 32 * UNITS;   // units in the slice
#pragma unroll
    for (int i = 0; i < (TOTAL + 255) / 256; ++i) {
      const int u0 = (i * 256) + wave * 64;  // first unit of this wave-instruction
      if (u0 < TOTAL) {
        const int u = u0 + lane, row = u / UNITS, cu = u % UNITS;
        __builtin_amdgcn_global_load_lds((glb_void*)(x + (long)row * K + (cu ^ (row & 7)) * 8), (lds_void*)(xs + u0 * 8), 16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        xv[s][mb] = *reinterpret_cast<const u16x8*>(xs + (mb * 32 + r) * ROW + 8 * ((((kw0 + 8 * h + 16 * s) >> 3)) ^ (r & 7)));
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) xv[s][mb] = one;
  }
  f32x16 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = f32x16{};
  if constexpr (MODE == 6) {  // VALU instead of MFMA (same loads, reduce and store)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[mb][q] += __uint_as_float(static_cast<unsigned>(wv[s][q]) << 16);
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wv[s]), as_bf16x8(xv[s][mb]), acc[mb], 0, 0, 0);
  }
  if constexpr (MODE == 5) {  // no LDS reduce: every wave stores its fp32 partial tile
    float* yf = reinterpret_cast<float*>(y) + (long)(tile * 4 + wave) * 1024 * MB;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int q = 0; q < 16; ++q) yf[(mb * 16 + q) * 64 + lane] = acc[mb][q];
    return;
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][q][mb * 65 + lane] = acc[mb][q];
  __syncthreads();
  if constexpr (MODE == 9) {  // MFMA + LDS reduce, no output stores (one per workgroup)
    if (tid == 0) y[tile] = __builtin_bit_cast(unsigned short, static_cast<__bf16>(red[1][2][3] + red[2][3][4]));
    return;
  }
  // 32 rows x 32*MB tokens; thread -> (token, row pair)
  for (int e = tid; e < 1024 * MB; e += 256) {
    const int tok = e >> 5, i = e & 31, mb = tok >> 5, ml = tok & 31;
    const int q = (i & 3) + 4 * (i >> 3), ln = ml + 32 * ((i >> 2) & 1);
    float v = red[0][q][mb * 65 + ln] + red[1][q][mb * 65 + ln] + red[2][q][mb * 65 + ln] + red[3][q][mb * 65 + ln];
    y[(long)tok * N + tile * 32 + i] = __builtin_bit_cast(unsigned short, static_cast<__bf16>(v));
  }
}

// modes 10 / 11: the workgroup's 32 W rows staged to LDS in full lines by global_load_lds (1 KB contiguous per
// wave-instruction), fragments read from LDS; x constant (10) or fragment loads from L2 (11)
template <int MODE, int KS, int MB>
__global__ __launch_bounds__(256) void probe_lds(const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
                                                 unsigned short* __restrict__ y, int N, int K, int M) {
  constexpr int ROW = 4 * KS * 16, UNITS = ROW / 8, TOTAL = 32 * UNITS;
  __shared__ __attribute__((aligned(16))) unsigned short ws_[32 * ROW];
  __shared__ float red[4][16][65 * MB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x;
  const unsigned short* wt = w + (long)tile * 32 * K;
#pragma unroll
  for (int i = 0; i < (TOTAL + 255) / 256; ++i) {
    const int u0 = i * 256 + wave * 64;
    if (u0 < TOTAL) {
      const int u = u0 + lane, row = u / UNITS, cu = u % UNITS;
      __builtin_amdgcn_global_load_lds((glb_void*)(wt + (long)row * K + (cu ^ (row & 7)) * 8), (lds_void*)(ws_ + u0 * 8), 16, 0, 2);
    }
  }
  const int kw0 = wave * KS * 16;
  u16x8 xv[KS][MB];
  const u16x8 one = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
      xv[s][mb] = MODE == 11 ? *reinterpret_cast<const u16x8*>(x + (long)(mb * 32 + r) * K + kw0 + 8 * h + 16 * s) : one;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x16 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = f32x16{};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const u16x8 wv = *reinterpret_cast<const u16x8*>(ws_ + r * ROW + 8 * (((kw0 + 8 * h + 16 * s) >> 3) ^ (r & 7)));
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
      acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wv), as_bf16x8(xv[s][mb]), acc[mb], 0, 0, 0);
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][q][mb * 65 + lane] = acc[mb][q];
  __syncthreads();
  for (int e = tid; e < 1024 * MB; e += 256) {
    const int tok = e >> 5, i = e & 31, mb = tok >> 5, ml = tok & 31;
    const int q = (i & 3) + 4 * (i >> 3), ln = ml + 32 * ((i >> 2) & 1);
    float v = red[0][q][mb * 65 + ln] + red[1][q][mb * 65 + ln] + red[2][q][mb * 65 + ln] + red[3][q][mb * 65 + ln];
    y[(long)tok * N + tile * 32 + i] = __builtin_bit_cast(unsigned short, static_cast<__bf16>(v));
  }
}

// mode 12: both operands pre-packed in MFMA fragment order (W once per rollout, x by its producer): the
// fragment of (32-row block, k16-step s) is 64 lanes x 16 B contiguous, so every load instruction is one
// fully coalesced 1-KB read straight into registers; mode 13: same with x constant (W path alone)
template <int MODE, int KS, int MB>
__global__ __launch_bounds__(256) void probe_packed(const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
                                                    unsigned short* __restrict__ y, int N, int K, int M) {
  __shared__ float red[4][16][65 * MB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = blockIdx.x;
  const int nks = K / 16;
  const int s0 = wave * KS;
  // W packed: ((tile * nks + s) * 64 + lane) * 8 ; x packed: ((s * MB + mb) * 64 + lane) * 8
  u16x8 wv[KS], xv[KS][MB];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    wv[s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(w + ((long)(tile * nks + s0 + s) * 64 + lane) * 8));
  const u16x8 one = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
      xv[s][mb] = MODE == 12 ? *reinterpret_cast<const u16x8*>(x + ((long)((s0 + s) * MB + mb) * 64 + lane) * 8) : one;
  __builtin_amdgcn_sched_barrier(0);
  f32x16 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = f32x16{};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
      acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wv[s]), as_bf16x8(xv[s][mb]), acc[mb], 0, 0, 0);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][q][mb * 65 + lane] = acc[mb][q];
  __syncthreads();
  for (int e = tid; e < 1024 * MB; e += 256) {
    const int tok = e >> 5, i = e & 31, mb = tok >> 5, ml = tok & 31;
    const int q = (i & 3) + 4 * (i >> 3), ln = ml + 32 * ((i >> 2) & 1);
    float v = red[0][q][mb * 65 + ln] + red[1][q][mb * 65 + ln] + red[2][q][mb * 65 + ln] + red[3][q][mb * 65 + ln];
    y[(long)tok * N + tile * 32 + i] = __builtin_bit_cast(unsigned short, static_cast<__bf16>(v));
  }
}

template <int MODE, int KS, int MB>
int run(const char* name, int N, int K, int M, unsigned short* x, std::vector<unsigned short*>& ws, unsigned short* y) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int ncopy = ws.size();
  auto launch = [&](unsigned short* wp) {
    if constexpr (MODE >= 12) hipLaunchKernelGGL((probe_packed<MODE, KS, MB>), dim3(N / 32), dim3(256), 0, 0, x, wp, y, N, K, M);
    else if constexpr (MODE >= 10) hipLaunchKernelGGL((probe_lds<MODE, KS, MB>), dim3(N / 32), dim3(256), 0, 0, x, wp, y, N, K, M);
    else hipLaunchKernelGGL((probe<MODE, KS, MB>), dim3(N / 32), dim3(256), 0, 0, x, wp, y, N, K, M);
  };
  for (int i = 0; i < 20; ++i) launch(ws[i % ncopy]);
  CK(hipDeviceSynchronize());
  const int iters = 400;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) launch(ws[i % ncopy]);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / iters;
  printf("{\"probe\": \"%s\", \"pin\": %d, \"mode\": %d, \"N\": %d, \"K\": %d, \"M\": %d, \"wgs\": %d, \"us\": %.2f, \"w_GBps\": %.0f}\n",
         name, SCHED_PIN, MODE, N, K, M, N / 32, us, 2.0 * N * K / us / 1e3);
  return 0;
}

int main() {
  const int M = 64;
  unsigned short* x;
  unsigned short* y;
  CK(hipMalloc(&x, 128 * 8192 * 2));
  CK(hipMalloc(&y, 128 * 16384 * 16));
  CK(hipMemset(x, 0, 128 * 8192 * 2));
  struct Shape { const char* name; int N, K; };
  // qkv_proj (1152 x 896), gate_up_proj (9728 x 896) at full K per workgroup (KS = 896/64 = 14)
  for (Shape sh : {Shape{"qkv", 1152, 896}, Shape{"gate_up", 9728, 896}}) {
    std::vector<unsigned short*> ws;
    const size_t bytes = size_t(sh.N) * sh.K * 2;
    const int ncopy = int(600e6 / bytes) + 2;
    for (int i = 0; i < ncopy; ++i) {
      unsigned short* p;
      CK(hipMalloc(&p, bytes));
      CK(hipMemset(p, 0, bytes));
      ws.push_back(p);
    }
    if (run<4, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<0, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<1, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<9, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<10, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<11, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<12, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<13, 14, 2>(sh.name, sh.N, sh.K, M, x, ws, y)) return 1;
    if (run<12, 14, 1>(sh.name, sh.N, sh.K, 32, x, ws, y)) return 1;
    if (run<12, 14, 4>(sh.name, sh.N, sh.K, 128, x, ws, y)) return 1;
    for (auto p : ws) CK(hipFree(p));
  }
  return 0;
}
