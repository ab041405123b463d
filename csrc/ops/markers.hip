// Timeline markers for profiles: an empty kernel launched at the start and at the end of a
// benchmark's timed region, so that a rocprofv3 --kernel-trace database can be cut to exactly
// that region in the GPU's own clock (tools/prof_summary.py --between-markers). It reads and
// writes nothing.
#include "common.h"

namespace pa {
template <int ID>
__global__ void timeline_marker_kernel() {}
}  // namespace pa

extern "C" int pa_timeline_marker(int id, hipStream_t st) {
  if (id == 0) hipLaunchKernelGGL(pa::timeline_marker_kernel<0>, dim3(1), dim3(64), 0, st);
  else hipLaunchKernelGGL(pa::timeline_marker_kernel<1>, dim3(1), dim3(64), 0, st);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Diagnostics: what a kernel boundary costs after a kernel that WRITES (tools/launch_gap.py).
// Fills n16 16-byte chunks of dst with one of four store forms: 0 plain, 1 non-temporal,
// 2 write-through (buffer store, sc1), 3 plain + a read of one line (so the kernel is not
// write-only). The data is never read back; only the chain's wall time matters.
namespace pa {
__global__ __launch_bounds__(256) void store_test_kernel(u32x4* dst, long long n16, int mode) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const u32x4 v = {(uint32_t)threadIdx.x, (uint32_t)blockIdx.x, 0u, 1u};
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    if (mode == 1) __builtin_nontemporal_store(v, dst + i);
    else if (mode == 2 && i < (1ll << 27)) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(i * 16), 0, 16);
    else dst[i] = v;
  }
}
}  // namespace pa

extern "C" int pa_store_test(void* dst, long long n16, int mode, int grid, hipStream_t st) {
  if (n16 <= 0 || grid <= 0) return 0;
  hipLaunchKernelGGL(pa::store_test_kernel, dim3(grid), dim3(256), 0, st, (pa::u32x4*)dst, n16, mode);
  return (int)hipGetLastError();
}
