// SwiGLU activation for the Llama MLP: out = silu(gate) * up, reading the fused
// gate_up GEMM output [T, 2F] (gate | up) and writing [T, F]. Memory bound:
// 16-byte vectors, 2D grid (row, column-chunk) so prefill rows and decode
// batches both fill the chip.
#include "common.h"

namespace pa {

__global__ __launch_bounds__(256) void silu_mul_kernel(bf16* __restrict__ out,
                                                       const bf16* __restrict__ in, int F) {
  const int row = blockIdx.y;
  const int v = blockIdx.x * 256 + threadIdx.x;  // vector index within the row
  if (v * 8 >= F) return;
  const bf16* g = in + (size_t)row * 2 * F;
  bf16x8 a = *reinterpret_cast<const bf16x8*>(g + v * 8);
  bf16x8 b = *reinterpret_cast<const bf16x8*>(g + F + v * 8);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = bf2f(a[j]);
    const float s = x / (1.f + __expf(-x));
    o[j] = f2bf(bf2f(f2bf(s)) * bf2f(b[j]));
  }
  *reinterpret_cast<bf16x8*>(out + (size_t)row * F + v * 8) = o;
}

}  // namespace pa

extern "C" int pa_silu_mul(void* out, const void* in, int T, int F, hipStream_t st) {
  if (T <= 0) return 0;
  if (F % 8 != 0) return -1;
  dim3 g((F / 8 + 255) / 256, T);
  hipLaunchKernelGGL(pa::silu_mul_kernel, g, dim3(256), 0, st, (pa::bf16*)out,
                     (const pa::bf16*)in, F);
  return (int)hipGetLastError();
}
