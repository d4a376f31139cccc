// K1 access-shape streaming probe: 5 fp32 streams + one int64 stream read (28 B / token), 2 fp32 streams
// written (8 B / token), no math, at 2^26 tokens (2.4 GB per pass, far past the 256 MiB Infinity Cache).
// Variants: chunk-to-workgroup assignment (contiguous runs per workgroup vs grid-stride windows), chunks in
// flight per lane, nontemporal loads / stores, workgroups per CU, workgroup size.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/k1_stream_probe tools/probes/k1_stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

struct P {
  const f4* in[5];
  const f4* mask;  // 2 f4 per 4 tokens
  f4* out[2];
  long n4;         // groups of 4 tokens
};

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// STRIDE: chunk c of iteration i = i * grid + blockIdx.x (all workgroups sweep one window together)
// else contiguous runs of chunks per workgroup
__global__ void fill_rand(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (float)(x & 0xffffff) * (1.0f / 16777216.0f) - 0.5f;
  }
}

template <int TPB, int U, bool STRIDE, bool NTL, bool NTS, bool MATH = false>
__global__ __launch_bounds__(TPB) void k1_shape(P p) {
  const long nch = (p.n4 + TPB - 1) / TPB;
  const long per = (nch + gridDim.x - 1) / gridDim.x;
  const long step = STRIDE ? (long)gridDim.x : 1;
  const long c0 = STRIDE ? blockIdx.x : blockIdx.x * per;
  const long cend = STRIDE ? nch : min(nch, c0 + per);
  for (long c = c0; c < cend; c += step * U) {
    f4 v[U][7];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = (c + u * step) * TPB + threadIdx.x;
      if (c + u * step < cend && i < p.n4) {
#pragma unroll
        for (int r = 0; r < 5; ++r) v[u][r] = ld<NTL>(p.in[r] + i);
        v[u][5] = ld<NTL>(p.mask + 2 * i);
        v[u][6] = ld<NTL>(p.mask + 2 * i + 1);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = (c + u * step) * TPB + threadIdx.x;
      if (c + u * step < cend && i < p.n4) {
        f4 s = v[u][0] + v[u][1] + v[u][2] + v[u][3] + v[u][4] + v[u][5] + v[u][6];
        if constexpr (MATH) {  // about K1's per-token VALU work: two exps, clamps, selects
          s.x = expf(fminf(s.x, 20.f)) * v[u][2].x + expf(v[u][4].x - v[u][1].x);
          s.y = expf(fminf(s.y, 20.f)) * v[u][2].y + expf(v[u][4].y - v[u][1].y);
          s.z = expf(fminf(s.z, 20.f)) * v[u][2].z + expf(v[u][4].z - v[u][1].z);
          s.w = expf(fminf(s.w, 20.f)) * v[u][2].w + expf(v[u][4].w - v[u][1].w);
        }
        st<NTS>(p.out[0] + i, s);
        st<NTS>(p.out[1] + i, s * 2.f);
      }
    }
  }
}

template <int TPB, int U, bool STRIDE, bool NTL, bool NTS, bool MATH = false>
int run(P p, int wpc, int cus) {
  const int grid = wpc * cus;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k1_shape<TPB, U, STRIDE, NTL, NTS, MATH>), dim3(grid), dim3(TPB), 0, 0, p);
  const int reps = 10;
  float best = 1e30f, tot = 0.f;
  for (int w = 0; w < reps; ++w) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k1_shape<TPB, U, STRIDE, NTL, NTS, MATH>), dim3(grid), dim3(TPB), 0, 0, p);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
    tot += ms;
  }
  const double bytes = (double)p.n4 * 4 * 36;
  printf("{\"math\": %d, \"tpb\": %d, \"U\": %d, \"stride\": %d, \"nt_load\": %d, \"nt_store\": %d, \"wg_per_cu\": %d, "
         "\"mean_us\": %.1f, \"TBps_mean\": %.3f, \"TBps_best\": %.3f}\n",
         (int)MATH, TPB, U, (int)STRIDE, (int)NTL, (int)NTS, wpc, tot / reps * 1e3, bytes / (tot / reps * 1e-3) / 1e12,
         bytes / (best * 1e-3) / 1e12);
  fflush(stdout);
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const long N = 1L << 26;
  P p{};
  p.n4 = N / 4;
  for (int r = 0; r < 5; ++r) { f4* q; CK(hipMalloc(&q, N * 4)); CK(hipMemset(q, 0, N * 4)); p.in[r] = q; }
  { f4* q; CK(hipMalloc(&q, N * 8)); CK(hipMemset(q, 0, N * 8)); p.mask = q; }
  for (int w = 0; w < 2; ++w) CK(hipMalloc(&p.out[w], N * 4));
  run<256, 2, true, true, true>(p, 2, cus);
  run<256, 2, true, true, true, true>(p, 2, cus);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (float*)p.in[r], N, 17u + r);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (float*)p.mask, 2 * N, 99u);
  CK(hipDeviceSynchronize());
  printf("random data\n");
  run<256, 2, true, true, true>(p, 2, cus);
  run<256, 2, true, true, true, true>(p, 2, cus);
  run<256, 1, true, true, true, true>(p, 2, cus);
  run<256, 4, true, true, true, true>(p, 2, cus);
  run<256, 2, true, true, true, true>(p, 4, cus);
  run<512, 2, true, true, true, true>(p, 1, cus);
  run<1024, 1, true, true, true, true>(p, 1, cus);
  return 0;
}
