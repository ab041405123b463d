// Probe of v_permlane16_swap_b32 semantics on gfx950: prints, for lanes 0,16,32,48, the two
// results of permlane16_swap(a = 100 + lane, b = 200 + lane).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(100u + l, 200u + l, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 128 * sizeof(unsigned));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 8) printf("lane %2d: r0=%u r1=%u\n", l, h[l], h[64 + l]);
  return 0;
}
