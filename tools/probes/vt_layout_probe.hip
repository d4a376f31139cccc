// Decode-attention stream shape probe: per (sequence, KV head) workgroup, 2 waves read 32-key blocks of K (4 KB
// contiguous) and V^T either as 64 rows x 64 B at the cache's row stride (today's layout) or as one contiguous 4-KB
// tile (key-blocked layout). Cold: 4 cache copies (> the 256 MB MALL) read in turn. Prints GB/s per layout.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

template <bool BLOCKED>
__global__ __launch_bounds__(128) void stream(const unsigned short* k, const unsigned short* vt, int L, int ld,
                                              float* out) {
  const int bh = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned short* kb = k + (size_t)bh * ld * 64;
  const unsigned short* vb = vt + (size_t)bh * 64 * ld;
  float acc = 0.f;
  const int nblk = (L + 31) / 32;
  for (int ib = w; ib < nblk; ib += 2) {
    const int k0 = ib * 32;
    u16x8 r[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      r[i] = *reinterpret_cast<const u16x8*>(kb + (size_t)(k0 + c / 8) * 64 + 8 * (c % 8));
      if (BLOCKED) r[4 + i] = *reinterpret_cast<const u16x8*>(vb + (size_t)ib * 64 * 32 + c * 8);
      else r[4 + i] = *reinterpret_cast<const u16x8*>(vb + (size_t)(c >> 2) * ld + k0 + 8 * (c & 3));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += (float)(r[i][0] ^ r[i][7]);
  }
  if (acc == 12345.f) out[bh] = acc;
}

int main() {
  const int B = 512, Hkv = 2, L = 640, ld = 768, copies = 4;
  const size_t per = (size_t)B * Hkv * ld * 64;  // elements per K (or V^T) copy
  std::vector<unsigned short*> K(copies), V(copies);
  for (int c = 0; c < copies; ++c) {
    hipMalloc(&K[c], per * 2); hipMalloc(&V[c], per * 2);
    hipMemset(K[c], 1, per * 2); hipMemset(V[c], 1, per * 2);
  }
  float* out; hipMalloc(&out, B * Hkv * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = (double)B * Hkv * L * 64 * 2 * 2;
  for (int rep = 0; rep < 2; ++rep)
    for (int blocked = 0; blocked < 2; ++blocked) {
      const int iters = 40;
      hipEventRecord(e0);
      for (int it = 0; it < iters; ++it) {
        const int c = it % copies;
        if (blocked) hipLaunchKernelGGL(stream<true>, dim3(B * Hkv), dim3(128), 0, 0, K[c], V[c], L, ld, out);
        else hipLaunchKernelGGL(stream<false>, dim3(B * Hkv), dim3(128), 0, 0, K[c], V[c], L, ld, out);
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / iters;
      printf("{\"layout\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}\n", blocked ? "key_blocked" : "row_strided", us,
             bytes / (us * 1e-6) / 1e9);
    }
  return 0;
}
