// Weight prefetch into the Infinity Cache (MALL) on a side stream (decode steps).
//
// The decode projections are latency-bound rather than bandwidth-bound: cold, the
// 34 MB O projection streams at 2.6 TB/s and the 50 MB QKV at 3.4 TB/s, but at 3.9 and
// 4.2 TB/s when their weights already sit in the 256 MB memory-side cache
// (profiles/r2_mall_warm.jsonl). The model therefore forks a side stream inside the
// decode hipGraph that reads the NEXT projection's weights while the current kernel
// (attention, which leaves most CUs and HBM idle at small batch, or the down
// projection) runs; the consumer then hits MALL. This kernel only has to generate
// the line fills: one 16-byte load per 64-byte line, a few workgroups, results folded
// into a value that is stored only if it equals an impossible pattern (keeps the loads
// alive; vector store, never taken in practice).
#include "common.h"

namespace pa {

__global__ __launch_bounds__(256) void prefetch_kernel(const u32x4* __restrict__ p, long long lines,
                                                       u32x4* __restrict__ sink) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  // 4 loads in flight per thread per iteration
  for (; i + 3 * stride < lines; i += 4 * stride) {
    const u32x4 a = p[4 * i];
    const u32x4 b = p[4 * (i + stride)];
    const u32x4 c = p[4 * (i + 2 * stride)];
    const u32x4 d = p[4 * (i + 3 * stride)];
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < lines; i += stride) acc ^= p[4 * i];
  if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == 0xF39CC060u && acc.w == 0x5CEDC834u)
    sink[threadIdx.x] = acc;
}

}  // namespace pa

extern "C" int pa_prefetch(const void* p, long long bytes, void* sink, int wgs, hipStream_t st) {
  if (p == nullptr || sink == nullptr || bytes < 64 || (reinterpret_cast<uintptr_t>(p) & 15) || wgs < 1)
    return -1;
  const long long lines = bytes / 64;  // whole 64-B lines only: never reads past the buffer
  hipLaunchKernelGGL(pa::prefetch_kernel, dim3(wgs), dim3(256), 0, st, reinterpret_cast<const pa::u32x4*>(p),
                     lines, reinterpret_cast<pa::u32x4*>(sink));
  return (int)hipGetLastError();
}
