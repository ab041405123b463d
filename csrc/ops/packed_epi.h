// Register epilogues shared by the packed-weight projection kernels (gemm_mid.hip,
// gemm_prefill.hip). Both run the MFMA as C^T = W · x^T, so after the k-loop each lane
// holds 4 CONSECUTIVE output columns [cq, cq + 4) of one token row m for every 16-column
// tile it owns; the epilogues below turn that quad into bf16 outputs:
//
//   EP_PLAIN     y = acc
//   EP_SILU      y = silu(gate) * up over the interleaved (gate t, up t) packed tiles
//   EP_RESID     y = resid + acc, returning sum(y^2) of the written bf16 values (the next
//                RMSNorm's row statistics, accumulated by the caller)
//   EP_ROPEPERM  y = acc in the natural QKV column order (rope-permuted packed tiles)
//   EP_ROPEKV    RoPE on the (i, i + 64) tile pairs of the rope-packed QKV, q -> q_out,
//                k / v -> the layer's paged cache at slots[m] (replaces rope_cache.hip)
//
// AT is any argument struct with the fields used here (y, ldy, resid, ldr, q_out,
// k_cache, v_cache, positions, slots, cos_sin, H, KV).
#pragma once
#include "common.h"

namespace pa {
namespace pk {

enum { EP_PLAIN = 0, EP_SILU = 1, EP_RESID = 2, EP_ROPEPERM = 3, EP_ROPEKV = 4 };

template <int EPI>
constexpr bool pair_epi() { return EPI == EP_SILU || EPI == EP_ROPEKV; }

// packed rope-QKV tile -> first column of its original tile
__device__ __forceinline__ int ropeperm_tile(int tile) {
  const int p = tile & 7;  // packed position inside a head -> original tile (0,4,1,5,2,6,3,7)
  return (tile & ~7) + ((p & 1) ? 4 + (p >> 1) : (p >> 1));
}

// Epilogue for one token row m and 4 consecutive columns [cq, cq + 4) of packed tile
// `tile` (and, for the pair epilogues, the same 4 columns of tile + 1 in v2).
template <int EPI, class AT>
__device__ __forceinline__ float store_quad(const AT& A, int m, int tile, int cq, f32x4 v, f32x4 v2) {
  if constexpr (EPI == EP_SILU) {
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (bf16)(v[r] / (1.f + __expf(-v[r])) * v2[r]);
    *reinterpret_cast<bf16x4*>(A.y + (size_t)m * A.ldy + (tile >> 1) * 16 + cq) = o;
    return 0.f;
  } else if constexpr (EPI == EP_ROPEKV) {
    // tile even: original tile i (dims 16i + cq ..), tile + 1: original tile i + 4 (dims + 64)
    const int hh = tile >> 3;
    const int d = 16 * ((tile & 7) >> 1) + cq;
    f32x4 o1 = v, o2 = v2;
    if (hh < A.H + A.KV) {
      const float* cs = A.cos_sin + (size_t)A.positions[m] * 128;
      const f32x4 c = *reinterpret_cast<const f32x4*>(cs + d);
      const f32x4 s = *reinterpret_cast<const f32x4*>(cs + 64 + d);
      o1 = v * c - v2 * s;
      o2 = v2 * c + v * s;
    }
    bf16x4 b1, b2;
#pragma unroll
    for (int r = 0; r < 4; ++r) { b1[r] = (bf16)o1[r]; b2[r] = (bf16)o2[r]; }
    if (hh < A.H) {
      bf16* dst = A.q_out + ((size_t)m * A.H + hh) * 128;
      *reinterpret_cast<bf16x4*>(dst + d) = b1;
      *reinterpret_cast<bf16x4*>(dst + d + 64) = b2;
    } else {
      const int slot = A.slots[m];
      if (slot >= 0) {
        const int blk = slot >> 4, off = slot & 15;
        if (hh < A.H + A.KV) {
          bf16* page = A.k_cache + ((size_t)blk * A.KV + (hh - A.H)) * 128 * 16;
          *reinterpret_cast<bf16x4*>(page + ((size_t)(d >> 3) * 16 + off) * 8 + (d & 7)) = b1;
          *reinterpret_cast<bf16x4*>(page + ((size_t)((d + 64) >> 3) * 16 + off) * 8 + (d & 7)) = b2;
        } else {
          bf16* page = A.v_cache + ((size_t)blk * A.KV + (hh - A.H - A.KV)) * 128 * 16 + off;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            page[(size_t)(d + r) * 16] = b1[r];
            page[(size_t)(d + 64 + r) * 16] = b2[r];
          }
        }
      }
    }
    return 0.f;
  } else {
    const int col = (EPI == EP_ROPEPERM ? ropeperm_tile(tile) * 16 : tile * 16) + cq;
    if constexpr (EPI == EP_RESID) {
      const bf16x4 rv = *reinterpret_cast<const bf16x4*>(A.resid + (size_t)m * A.ldr + col);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
    }
    bf16x4 o;
    float sq = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = (bf16)v[r];
      const float f = (float)o[r];
      sq = fmaf(f, f, sq);
    }
    *reinterpret_cast<bf16x4*>(A.y + (size_t)m * A.ldy + col) = o;
    return sq;
  }
}

// Non-pair epilogues on two adjacent tiles at once, stored 16 B per lane: lanes g and g ^ 1
// (lane groups of 16) trade halves (lane ^ 16 exchange), so lane (g, c) ends with 8
// consecutive columns of ONE tile — tile `tile` for even g, tile + 1 for odd g — starting
// at column 8 (g >> 1). One dwordx4 store per lane instead of two dwordx2 (the guide's T21:
// a store-issue-bound epilogue tail halves). a = tile's quad, b = tile + 1's quad (columns
// 4 g .. 4 g + 3 of each). Returns sum(y^2) of the written bf16 values (EP_RESID).
template <int EPI, class AT>
__device__ __forceinline__ float store_pair_wide(const AT& A, int m, int tile, int g, f32x4 a, f32x4 b) {
  static_assert(!pair_epi<EPI>(), "pair epilogues keep store_quad");
  const bool odd = g & 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // even g keeps a and receives the partner's a; odd g the reverse
    const float got = __shfl_xor(odd ? a[r] : b[r], 16, 64);
    if (odd) a[r] = got; else b[r] = got;
  }
  const int t = tile + (g & 1);
  const int col = (EPI == EP_ROPEPERM ? ropeperm_tile(t) * 16 : t * 16) + 8 * (g >> 1);
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  if constexpr (EPI == EP_RESID) {
    const bf16x8 rv = *reinterpret_cast<const bf16x8*>(A.resid + (size_t)m * A.ldr + col);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += (float)rv[r];
  }
  bf16x8 o;
  float sq = 0.f;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    o[r] = (bf16)v[r];
    const float f = (float)o[r];
    sq = fmaf(f, f, sq);
  }
  *reinterpret_cast<bf16x8*>(A.y + (size_t)m * A.ldy + col) = o;
  return sq;
}

}  // namespace pk
}  // namespace pa
