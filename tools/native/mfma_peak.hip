// MFMA speed of light on this chip under sustained load: every wave of a full grid
// issues back-to-back v_mfma_f32_32x32x16_bf16 on register operands (4 independent
// accumulators), no memory traffic. Reports TFLOP/s; compare with the GEMMs' rates.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * (threadIdx.x - i));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keeps the work alive
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 24);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 4096;
  for (int wpc : {1, 2, 4, 8}) {  // workgroups (of 4 waves) per CU
    const int grid = cus * wpc;
    hipLaunchKernelGGL(mfma_loop, dim3(grid), dim3(256), 0, 0, out, 64);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(mfma_loop, dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 5.0 * grid * 4 /*waves*/ * (double)iters * 4 /*mfma*/ * 32 * 32 * 16 * 2;
    std::printf("{\"cus\": %d, \"wg_per_cu\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", cus, wpc, ms, flops / ms / 1e9);
  }
  hipFree(out);
  return 0;
}
