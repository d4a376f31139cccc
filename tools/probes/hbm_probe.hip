// HBM streaming ceilings for K1's access shape (5 fp32 streams read, 2 written, + an int64 mask pass):
// what a kernel with no math reaches on this MI355X, to judge K1's fraction against an achievable rate.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/hbm_probe tools/hbm_probe.hip ; run: build/hbm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NR, int NW, bool NT, int U>
__global__ __launch_bounds__(256) void stream_kernel(const f4* const* __restrict__ in, f4* const* __restrict__ out,
                                                     long n4, int per) {
  const long begin = (long)blockIdx.x * per * 256 * U;
  for (long base = begin; base < begin + (long)per * 256 * U && base < n4; base += 256L * U) {
    f4 v[U][NR];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const long i = base + u * 256 + threadIdx.x;
        if (i < n4) {
          if constexpr (NT) v[u][r] = __builtin_nontemporal_load(in[r] + i);
          else v[u][r] = in[r][i];
        }
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * 256 + threadIdx.x;
      if (i >= n4) continue;
      f4 s = v[u][0];
#pragma unroll
      for (int r = 1; r < NR; ++r) s += v[u][r];
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        if constexpr (NT) __builtin_nontemporal_store(s, out[w] + i);
        else out[w][i] = s;
      }
    }
  }
}

template <int NR, int NW, bool NT, int U>
int run(const char* name, f4** d_in, f4** d_out, long n4, int wg_per_cu, int cus) {
  const long iters_total = (n4 + 256L * U - 1) / (256L * U);
  const int grid = wg_per_cu * cus;
  const int per = (int)((iters_total + grid - 1) / grid);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((stream_kernel<NR, NW, NT, U>), dim3(grid), dim3(256), 0, 0, d_in, d_out, n4, per);
  CK(hipEventRecord(a));
  const int reps = 20;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((stream_kernel<NR, NW, NT, U>), dim3(grid), dim3(256), 0, 0, d_in, d_out, n4, per);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)n4 * 16 * (NR + NW);
  printf("{\"probe\": \"%s\", \"wg_per_cu\": %d, \"unroll\": %d, \"nt\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name, wg_per_cu, U,
         (int)NT, ms / reps * 1e3, bytes / (ms / reps * 1e-3) / 1e12);
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const long N = 1L << 26;  // tokens
  const long n4 = N / 4;
  std::vector<f4*> h_in(5), h_out(2);
  for (auto& p : h_in) { CK(hipMalloc(&p, N * 4)); CK(hipMemset(p, 0, N * 4)); }
  for (auto& p : h_out) CK(hipMalloc(&p, N * 4));
  f4** d_in; f4** d_out;
  CK(hipMalloc(&d_in, 5 * sizeof(f4*)));
  CK(hipMalloc(&d_out, 2 * sizeof(f4*)));
  CK(hipMemcpy(d_in, h_in.data(), 5 * sizeof(f4*), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_out, h_out.data(), 2 * sizeof(f4*), hipMemcpyHostToDevice));
  for (int wpc : {2, 4, 8}) {
    run<1, 1, false, 1>("copy_1r1w", d_in, d_out, n4, wpc, cus);
    run<5, 2, false, 1>("k1_5r2w", d_in, d_out, n4, wpc, cus);
    run<5, 2, false, 2>("k1_5r2w", d_in, d_out, n4, wpc, cus);
    run<5, 2, true, 1>("k1_5r2w", d_in, d_out, n4, wpc, cus);
    run<5, 2, true, 2>("k1_5r2w", d_in, d_out, n4, wpc, cus);
    run<2, 0, false, 2>("read_int64_mask", d_in, d_out, n4, wpc, cus);
    run<5, 0, false, 2>("read_5r", d_in, d_out, n4, wpc, cus);
  }
  return 0;
}
