// Shared device helpers for the pilottai_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in csrc/ops:
//   * wave64 everywhere (block sizes are multiples of 64, lane = threadIdx.x & 63),
//   * bf16 tensors are moved as 16-byte vectors (8 x bf16) whenever the row
//     length allows it (guide Guideline 13: scalar bf16 loads cost ~2x),
//   * accumulation is fp32; conversion back to bf16 uses the hardware
//     v_cvt_pk_bf16_f32 path (plain __bf16 casts, NaN-preserving),
//   * launchers are plain C functions that take raw device pointers and a
//     hipStream_t so they can be captured into hipGraphs (no syncs, no mallocs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pa {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of NWAVES waves; `red` must hold NWAVES floats.
template <int NWAVES>
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) t += red[i];
  __syncthreads();
  return t;
}

// In-launch split-K / partition hand-off (cdna_hip_programming.md §6 Guideline 16 and §5
// "In-launch split-K reduction"). Protocol, in this order:
//   producer  every wave stores its partial write-through (sc1 buffer stores), then
//             runs asm `s_waitcnt vmcnt(0)` (EVERY storing wave drains: Pitfall 14),
//             then calls handoff_last();
//   release   (acquire >= 2, the default) one lane runs an agent-scope release
//             (buffer_wbl2 sc1) and drains it, behind the workgroup barrier;
//   ticket    one lane takes a relaxed agent-scope ticket after a workgroup barrier;
//   consumer  the workgroup that drew ticket n-1 resets the counter for the next launch and
//             runs ONE agent-scope acquire (`buffer_inv sc1`, completion awaited by an asm
//             vmcnt(0)) before the barrier that releases its readers.
// The acquire makes the hand-off placement-independent for ANY number of workgroups per CU
// (the sc1-loads-only form is validated only at one workgroup per CU: MI355X_MICROARCH.md
// "Valid forms", condition (4)); the readers may then use plain or sc1 loads.
// `acquire` = 0 keeps the old sc1-only consumer and 1 the acquire without the release
// (diagnostics: tools/splitk_check.py, tools/handoff_cost.py).
// Every thread of the workgroup must call it; it returns true in all of them for the last
// arriver. `lflag` is an int in the kernel's single LDS array.
typedef __attribute__((address_space(1))) int handoff_gi32;
__device__ __forceinline__ bool handoff_last(int* counter, int n, int* lflag, int acquire) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (acquire >= 2) {  // agent-scope release (L2 write-back) on top of the sc1 stores
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int tk = __hip_atomic_fetch_add((handoff_gi32*)counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == n - 1;
    if (last) {
      __hip_atomic_store((handoff_gi32*)counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (acquire) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    *lflag = last;
  }
  __syncthreads();
  return *lflag != 0;
}

// host-side hand-off modes passed to the kernels with an in-launch hand-off: the GEMM
// split-K slabs (decode / wide / mid / prefill) and the attention partition merge
extern int g_handoff_acquire;
extern int g_handoff_attn;

// Cheap stateless 32-bit hash (splitmix-style finaliser) used as a counter-based
// RNG for sampling: u = hash(seed, row, col) -> uniform in (0, 1).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU;
  x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint32_t row, uint32_t col) {
  uint32_t h = mix32((uint32_t)seed ^ mix32(row * 0x9E3779B9U + (uint32_t)(seed >> 32)));
  h = mix32(h ^ (col * 0x85EBCA6BU + 0x27d4eb2fU));
  // 24 random bits -> (0,1), never exactly 0 or 1
  return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

}  // namespace pa
