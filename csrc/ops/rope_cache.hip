// Rotary embedding fused with the paged KV-cache write.
//
// Input is the fused QKV GEMM output [T, (H + 2*KV) * 128]. For every token:
//   q  -> rotate-half RoPE -> q_out[T, H, 128]
//   k  -> rotate-half RoPE -> k_cache[block][kv][128/8][slot][8]  (fragment-major keys)
//   v  ->                     v_cache[block][kv][128][slot]      (transposed values)
// Both page layouts are chosen for the attention kernel's MFMA operand loads
// (attention.hip): a K A-fragment (8 dims of 16 keys) and a V^T A-fragment
// (8 keys of 16 dims) are each ONE contiguous 256-B run of a page, so every
// fragment load instruction reads whole 128-B lines.
// cos/sin come from a host-precomputed fp32 table [max_pos, 128] (cos | sin),
// so no transcendental work runs on the GPU (guide App. B, element-wise/RoPE).
#include "common.h"

namespace pa {

constexpr int HD = 128;

template <int BLK>
__global__ __launch_bounds__(256) void rope_cache_kernel(
    bf16* __restrict__ q_out, bf16* __restrict__ k_cache, bf16* __restrict__ v_cache,
    const bf16* __restrict__ qkv, const int* __restrict__ positions,
    const int* __restrict__ slot_mapping, const float* __restrict__ cos_sin, int H, int KV,
    int ld, int apply_rope) {
  const int t = blockIdx.x;
  const bf16* row = qkv + (size_t)t * ld;
  const int pos = positions[t];
  const float* cs = cos_sin + (size_t)pos * HD;
  const int slot = slot_mapping[t];
  const int nq = H * 16;          // 16 threads per head, 4 rotary pairs each
  const int nk = KV * 16;
  const int nunits = nq + nk + KV * 16;
  for (int u = threadIdx.x; u < nunits; u += 256) {
    if (u < nq + nk) {
      const bool is_q = u < nq;
      const int hh = is_q ? (u >> 4) : ((u - nq) >> 4);
      const int i = ((is_q ? u : (u - nq)) & 15) * 4;  // first rotary index of this unit
      const bf16* src = row + (is_q ? hh * HD : (H + hh) * HD);
      bf16x4 x1 = *reinterpret_cast<const bf16x4*>(src + i);
      bf16x4 x2 = *reinterpret_cast<const bf16x4*>(src + i + 64);
      bf16x4 o1, o2;
      if (apply_rope) {
        f32x4 c = *reinterpret_cast<const f32x4*>(cs + i);
        f32x4 s = *reinterpret_cast<const f32x4*>(cs + 64 + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = bf2f(x1[j]), b = bf2f(x2[j]);
          o1[j] = f2bf(a * c[j] - b * s[j]);
          o2[j] = f2bf(b * c[j] + a * s[j]);
        }
      } else {
        o1 = x1;
        o2 = x2;
      }
      if (is_q) {
        bf16* dst = q_out + ((size_t)t * H + hh) * HD;
        *reinterpret_cast<bf16x4*>(dst + i) = o1;
        *reinterpret_cast<bf16x4*>(dst + i + 64) = o2;
      } else if (slot >= 0) {
        const int blk = slot / BLK, off = slot % BLK;
        bf16* page = k_cache + ((size_t)blk * KV + hh) * HD * BLK;  // [16 chunks][BLK][8]
        *reinterpret_cast<bf16x4*>(page + ((size_t)(i >> 3) * BLK + off) * 8 + (i & 7)) = o1;
        *reinterpret_cast<bf16x4*>(page + ((size_t)((i + 64) >> 3) * BLK + off) * 8 + (i & 7)) = o2;
      }
    } else if (slot >= 0) {
      const int uu = u - nq - nk;
      const int hh = uu >> 4, d0 = (uu & 15) * 8;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(row + (H + KV + hh) * HD + d0);
      const int blk = slot / BLK, off = slot % BLK;
      bf16* dst = v_cache + ((size_t)blk * KV + hh) * HD * BLK + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[(size_t)(d0 + j) * BLK] = v[j];
    }
  }
}

}  // namespace pa

extern "C" int pa_rope_cache(void* q_out, void* k_cache, void* v_cache, const void* qkv,
                             const int* positions, const int* slot_mapping, const float* cos_sin,
                             int T, int H, int KV, int ld, int block_size, int apply_rope,
                             hipStream_t st) {
  if (T <= 0) return 0;
  if (block_size != 16) return -1;
  hipLaunchKernelGGL(pa::rope_cache_kernel<16>, dim3(T), dim3(256), 0, st, (pa::bf16*)q_out,
                     (pa::bf16*)k_cache, (pa::bf16*)v_cache, (const pa::bf16*)qkv, positions,
                     slot_mapping, cos_sin, H, KV, ld, apply_rope);
  return (int)hipGetLastError();
}
