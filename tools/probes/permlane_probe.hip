// v_permlane32_swap semantics probe: prints both results of __builtin_amdgcn_permlane32_swap(u, u) and (a, b) for
// a few lanes (u = lane, a = lane, b = 100 + lane)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(l, l, true, false);
  const auto s = __builtin_amdgcn_permlane32_swap(l, 100u + l, true, false);
  out[4 * l] = r[0]; out[4 * l + 1] = r[1]; out[4 * l + 2] = s[0]; out[4 * l + 3] = s[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 64 * 16);
  k<<<1, 64>>>(d);
  unsigned h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %d: swap(u,u) = %u %u   swap(l, 100+l) = %u %u\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
  return 0;
}
