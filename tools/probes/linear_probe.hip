// Where does a decode-linear workgroup spend its time? Variants of the weight-streaming GEMM inner loop
// (16 waves split K, 32 W rows per workgroup, 64 token rows) timed over back-to-back launches:
//   mode 0: W nontemporal + x loads + MFMA (as csrc/linear.hip)   mode 1: W plain loads
//   mode 2: W only (x operand = constant)                         mode 3: x only (W operand = constant)
//   mode 4: the same W bytes as fully coalesced 1-KB wave loads (access-pattern cost)
//   mode 5/6: k-permuted operands (64 contiguous bytes per lane over 4 k-steps), plain loads, with/without
//             K-slice stagger across workgroups;  mode 7: prepacked W (MFMA order) + k-permuted x + stagger
// Build: hipcc --offload-arch=gfx950 -O3 -o build/linear_probe tools/linear_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const unsigned short* x, const unsigned short* w, float* out, int N, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x;
  const int nsteps = K >> 4;
  const int sw = (MODE == 5 || MODE == 7) ? (wave + tile) & 15 : wave;  // stagger K slices across workgroups
  const int s0 = sw * nsteps / 16, s1 = (sw + 1) * nsteps / 16;
  const unsigned short* wp = w + (long)(tile * 32 + r) * K + 8 * h;
  const unsigned short* xp0 = x + (long)r * K + 8 * h;
  const unsigned short* xp1 = x + (long)(32 + r) * K + 8 * h;
  f32x16 a0{}, a1{};
  u16x8 wv[4], x0[4], x1[4];
  const u16x8 one = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int s = s0 + u;
    const bool in = s < s1;
    // modes 5/6: k-permuted operands: lane half h, sub-step u <-> k = 64*(s0/4 group) + 32h + 8u (+j), so each
    // lane reads 64 contiguous bytes of its row over the 4 sub-steps (whole 128-B lines per row pair)
    const long kp = 16L * s0 + 32 * h + 8 * u - 8 * h;  // (wp/xp already include 8h)
    if (MODE == 5 || MODE == 6) {
      wv[u] = in ? *reinterpret_cast<const u16x8*>(wp + kp) : one;
      x0[u] = in ? *reinterpret_cast<const u16x8*>(xp0 + kp) : one;
      x1[u] = in ? *reinterpret_cast<const u16x8*>(xp1 + kp) : one;
      continue;
    }
    if (MODE == 7) {  // prepacked W: 1 KB contiguous per wave instruction (MFMA operand order)
      wv[u] = in ? *reinterpret_cast<const u16x8*>(w + ((long)tile * nsteps + s) * 512 + lane * 8) : one;
      x0[u] = in ? *reinterpret_cast<const u16x8*>(xp0 + kp) : one;
      x1[u] = in ? *reinterpret_cast<const u16x8*>(xp1 + kp) : one;
      continue;
    }
    if (MODE == 3) wv[u] = one;
    else if (MODE == 1) wv[u] = in ? *reinterpret_cast<const u16x8*>(wp + 16 * s) : one;
    else if (MODE == 4) {  // same bytes per wave, fully coalesced 1-KB wave loads over the tile's rows
      const long off = ((long)(wave * 4 + u) * 512 + lane * 8) % (32L * K);
      wv[u] = in ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(w + (long)tile * 32 * K + off)) : one;
    }
    else wv[u] = in ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wp + 16 * s)) : one;
    if (MODE == 2) { x0[u] = one; x1[u] = one; }
    else {
      x0[u] = in ? *reinterpret_cast<const u16x8*>(xp0 + 16 * s) : one;
      x1[u] = in ? *reinterpret_cast<const u16x8*>(xp1 + 16 * s) : one;
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wv[u]), __builtin_bit_cast(bf16x8, x0[u]), a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wv[u]), __builtin_bit_cast(bf16x8, x1[u]), a1, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += a0[q] + a1[q];
  if (s == 12345.f) out[blockIdx.x * 1024 + threadIdx.x] = s;
}

__global__ void empty_kernel() {}

template <int MODE>
int run(const char* name, const unsigned short* x, const unsigned short* const* ws, int ncopy, float* out, int N, int K) {
  const int tiles = N / 32;
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(tiles), dim3(1024), 0, 0, x, ws[i % ncopy], out, N, K);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int reps = 200;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(tiles), dim3(1024), 0, 0, x, ws[i % ncopy], out, N, K);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"probe\": \"%s\", \"N\": %d, \"K\": %d, \"us\": %.2f}\n", name, N, K, ms / reps * 1e3);
  return 0;
}

int main() {
  const int K = 896;
  float* out;
  unsigned short* x;
  CK(hipMalloc(&out, 1 << 26));
  CK(hipMalloc(&x, 64 * K * 2));
  CK(hipMemset(x, 0, 64 * K * 2));
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0);
    CK(hipEventRecord(a));
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"probe\": \"empty_kernel\", \"us\": %.2f}\n", ms / 200 * 1e3);
  }
  for (int N : {1152, 9728, 151936}) {
    const size_t wbytes = (size_t)N * K * 2;
    const int ncopy = (int)(600e6 / wbytes) + 1;
    std::vector<unsigned short*> hw(ncopy);
    for (auto& p : hw) { CK(hipMalloc(&p, wbytes)); CK(hipMemset(p, 0, wbytes)); }
    run<0>("nt_w+x", x, hw.data(), ncopy, out, N, K);
    run<1>("plain_w+x", x, hw.data(), ncopy, out, N, K);
    run<2>("w_only", x, hw.data(), ncopy, out, N, K);
    run<3>("x_only", x, hw.data(), ncopy, out, N, K);
    run<4>("w_coalesced+x", x, hw.data(), ncopy, out, N, K);
    run<0>("nt_w+x_hot", x, hw.data(), 1, out, N, K);
    run<5>("kperm_plain_stagger", x, hw.data(), ncopy, out, N, K);
    run<6>("kperm_plain", x, hw.data(), ncopy, out, N, K);
    run<7>("prepacked_w_kperm_x_stagger", x, hw.data(), ncopy, out, N, K);
    for (auto p : hw) CK(hipFree(p));
  }
  return 0;
}
