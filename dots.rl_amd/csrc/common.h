// Shared device/host helpers for the gfx950 kernels behind include/dotsrl_amd.h.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>

#include "dotsrl_amd.h"

namespace drl {

// ---------------------------------------------------------------- host: errors
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define DRL_CHECK_ARG(cond, ...)                     \
  do {                                               \
    if (!(cond)) return ::drl::fail(DRL_ERR_INVALID, __VA_ARGS__); \
  } while (0)

#define DRL_HIP(call)                                                                               \
  do {                                                                                              \
    hipError_t e_ = (call);                                                                         \
    if (e_ != hipSuccess)                                                                           \
      return ::drl::fail(DRL_ERR_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                                 \
  } while (0)

#define DRL_LAUNCH_CHECK() DRL_HIP(hipGetLastError())

int cu_count();  // cached per device

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// V^T (head-dim-major V) of one (sequence, KV head): rows of ld_vt keys, or with ld_vt == DRL_VT_BLOCKED the
// key-blocked cache layout [ceil(cap / 32)][D][32] (one 32-key block's V^T is 32 * D contiguous elements, so
// a decode / prefill block fetch is one contiguous 4-KB (D = 64) run instead of D row pieces). cap = the K
// capacity (ld_k / Tk) the panel is sized for.
__host__ __device__ __forceinline__ int64_t vt_index(int64_t d, int64_t key, int64_t ld_vt, int64_t D) {
  return ld_vt == DRL_VT_BLOCKED ? (key >> 5) * (32 * D) + d * 32 + (key & 31) : d * ld_vt + key;
}
__host__ __device__ __forceinline__ int64_t vt_panel(int64_t ld_vt, int64_t D, int64_t cap) {
  return ld_vt == DRL_VT_BLOCKED ? (cap + 31) / 32 * 32 * D : D * ld_vt;
}

// ---------------------------------------------------------------- device: wave/block reductions
constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// bf16 <-> f32 (bit-level; bf16 stored as uint16_t)
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }
// logistic sigmoid and SiLU (F.silu: x * sigmoid(x)) on the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32, ~1 ulp
// each): one form for every SwiGLU in the library (GEMM / decode epilogues, the elementwise kernels) so the paths
// agree with each other bit for bit; against expf + IEEE division it differs by a few fp32 ulp, below the bf16
// rounding every caller applies next. exp2(+inf) -> rcp(inf) = 0: silu(-large) = -0, silu(+large) = x, NaN stays NaN.
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float silu_fast(float x) { return x * sigmoid_fast(x); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // round-to-nearest-even, NaN stays NaN: gfx950's v_cvt_pk_bf16_f32 (one instruction; the integer form — a NaN
  // test, a carry add and a shift — was most of the VALU of the bf16-writing streams: K2's backward, the norms)
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

// Sampling as a race of exponential clocks (the Gumbel-max form of the categorical draw): token i wins iff
// z_i - log(E_i) is the row maximum, E_i = -log(1 - v_i) ~ Exp(1) with v_i = ((bits >> 8) + 0.5) / 2^24 a
// 24-bit Philox uniform in (0, 1). Hardware log2 (v_log_f32) instead of libm: E from a 4-term series below
// v = 2^-6 (relative error < 3e-8, where E is small and the key large) and from log2(1 - v) above (1 - v is
// rounded to 2^-25, i.e. < 2e-6 relative in E at v = 2^-6); log(E) = ln2 * log2(E). Keys stay within 2e-6
// of the libm / numpy float32 form the oracle uses (oracle.race_keys).
__device__ __forceinline__ float race_key(float z, uint32_t bits) {
  const float v = (static_cast<float>(bits >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float e = v < 0.015625f ? v * (1.f + v * (0.5f + v * (0.33333334f + v * 0.25f)))
                                : -0.6931471805599453f * __builtin_amdgcn_logf(1.f - v);
  return z - 0.6931471805599453f * __builtin_amdgcn_logf(e);
}

// Mask element -> 0/1 float, for the mask dtypes the boundary accepts.
template <int DT>
__device__ __forceinline__ float mask_at(const void* m, int64_t i) {
  if constexpr (DT == DRL_I64) return static_cast<float>(static_cast<const int64_t*>(m)[i]);
  else if constexpr (DT == DRL_I32) return static_cast<float>(static_cast<const int32_t*>(m)[i]);
  else if constexpr (DT == DRL_U8) return static_cast<float>(static_cast<const uint8_t*>(m)[i]);
  else return static_cast<const float*>(m)[i];
}

// Grid barrier for persistent launches whose every workgroup is co-resident (grid <= CUs x occupancy).
// Counter form with agent-scope release before arrive and acquire after (MI355X_MICROARCH.md,
// "barrier-counter"); `counter` is zeroed on the stream before the launch. A bounded spin sets
// *timeout instead of hanging the GPU if residency was ever violated.
__device__ __forceinline__ void grid_barrier(unsigned* counter, unsigned expected, unsigned* timeout) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < expected) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 26)) {
        __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// "Last workgroup to arrive" ticket over write-through partials (cdna_hip_programming.md §6 G16, R1):
// every workgroup stores its partials with store_sc1 (write-through, so no release fence and no L2
// write-back per workgroup, which cost K1 ~30 us at 2^26 tokens), drains them (s_waitcnt vmcnt(0) in
// every storing wave, then the barrier) and takes a relaxed agent-scope ticket; the one that draws
// gridDim-1 reads ALL partials with load_sc1 (bypassing its possibly stale L1, no acquire) and reduces
// them in a fixed order (bitwise-reproducible result). Returns true in every thread of that workgroup.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;  // global (not flat) accesses; C casts below
__device__ __forceinline__ void store_sc1(double* p, double v) {
  __hip_atomic_store((gu64_t*)(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
typedef __attribute__((address_space(1))) unsigned gu32_t;
__device__ __forceinline__ void store_f32_sc1(float* p, float v) {
  __hip_atomic_store((gu32_t*)(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float load_f32_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load((const gu32_t*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ double load_sc1(const double* p) {
  return __longlong_as_double(static_cast<long long>(
      __hip_atomic_load((const gu64_t*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
__device__ __forceinline__ bool last_block_ticket(unsigned* ticket) {
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)(ticket),
                                              1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (t == gridDim.x - 1);
  }
  __syncthreads();
  return is_last != 0;
}

}  // namespace drl
