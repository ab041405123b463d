// Four-wave 256 x 256 MFMA GEMM for the large-M projections (one wave per SIMD; included by
// gemm_prefill.hip, which owns the argument struct, the planner and the launcher).
//
//     y[M, N] = epi( rownorm(x)[M, K] · W[N, K]^T )      bf16 in/out, fp32 accumulate
//
// Why a second 256 x 256 kernel: the ping-pong kernel (gemm_pingpong.h) runs its loop within
// 5-9 % of the MFMA cycle floor, but the chip holds a lower clock under it than under
// hipBLASLt's 4096^3 kernel (1.90 vs 1.98 GHz from GRBM_GUI_ACTIVE, profiles/r5_gemm_clock.md):
// its 8 waves of 128 x 64 outputs read 24 fragments per 64 MFMAs from LDS, hipBLASLt's 4 waves
// of 128 x 128 read 16 (SQ_INSTS_LDS 3.28 M vs 2.12 M per 4096^3 launch). Fewer LDS bytes per
// MFMA is the energy lever the guide ranks for a power-limited loop (§5.4 rule 28).
//
// Structure:
//   * 256 threads = 4 waves, one per SIMD; wave (wn, wm) = (wid & 1, wid >> 1) owns W rows
//     [128 wn, +128) x tokens [128 wm, +128): acc[8 n-frags][8 m-frags] of
//     v_mfma_f32_16x16x32_bf16 (256 accumulators, AGPRs), run as C^T = W · x^T so the
//     packed_epi.h register epilogues apply unchanged (lane = 4 columns of one token);
//   * the k loop advances 32 k per STEP; a step's operands are one 32-KiB LDS stage:
//       W: the 16 packed 1-KiB chunks (n16 tile, 32 k) of the tile's 256 rows, lane-linear;
//          staged by buffer_load ... lds (per-lane 32-bit voffset, step advance in soffset);
//       x: 16 fragment images of 16 tokens x 32 k, staged FRAGMENT-MAJOR by the LDS-DMA
//          itself (lane l of the wave instruction loads token 16 f + (l & 15), k 8 (l >> 4)),
//          so every ds_read_b128 is lane-linear and conflict-free without a swizzle;
//   * four stages (128 KiB) rotate: step s + 3 is issued while step s computes; the x
//     fragments are read one step ahead into the other of two register sets, the W
//     fragments two 8-MFMA chunks ahead through a 4-entry ring:
//         iteration s:  LDS-DMA step s + 3 -> stage (s + 3) % 4     (8 per wave)
//                       ds_read x of step s + 1, W of step s / s + 1 (16 per wave)
//                       64 MFMAs
//                       lgkmcnt(0), vmcnt(8) [step s + 2 landed], ONE s_barrier
//     A stage is overwritten two barriers after its last read; a step's data is read one
//     barrier after the counted wait that retired it (guide: "read a staged buffer one phase
//     after the wait that retires it");
//   * the loads are hand-placed between 8-MFMA chunks and fenced with sched_barrier (one
//     wave per SIMD has no partner wave to fill its issue gaps).
// Work items, the split-K tail and the epilogues are those of the ping-pong kernel.
#pragma once
#include "common.h"
#include "packed_epi.h"

namespace pa {
namespace pf {

constexpr int W4_STAGE = 32768;  // bytes per 32-k step: W 16 KiB | x 16 KiB
constexpr int W4_SMEM = 4 * W4_STAGE;

template <int EPI, bool NORM>
__device__ __forceinline__ void w4_tile(const Args& A, const int bid, const int nblocks, char* smem) {
  constexpr int SLABF = 256 * 256;  // floats per split slab
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wid & 1, wm = wid >> 1;
  const int g = lane >> 4, c = lane & 15;

  const int KT = A.K >> 6;
  int tile, kt0, kt1, slice = -1;
  if (bid < A.full) {
    const int q8 = A.full >> 3, r8 = A.full & 7, xcd = bid & 7;
    tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    kt0 = 0;
    kt1 = KT;
  } else {
    const int nb = nblocks - A.full, w0 = bid - A.full;
    const int q8 = nb >> 3, r8 = nb & 7, xcd = w0 & 7;
    const int w2 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (w0 >> 3);
    tile = A.full + w2 / A.S;
    slice = w2 % A.S;
    kt0 = slice * A.per;
    kt1 = min(KT, kt0 + A.per);
  }
  const int mt = tile % A.MT, nt = tile / A.MT;
  const int row0 = mt * 256;
  const int n = 2 * (kt1 - kt0);  // 32-k steps, >= 4 (launcher: >= 2 k-tiles per item)
  const int ks0 = 2 * kt0;

  if (A.ss_zero && bid == 0)
    for (int i = threadIdx.x; i < A.M; i += 256) A.ss_zero[i] = 0.f;

  // ---- LDS-DMA sources: wave w stages W chunks 4 w .. 4 w + 3 and x fragments 4 w .. 4 w + 3,
  // as buffer_load ... lds with a per-lane 32-bit voffset and the step's advance in the
  // SGPR soffset (no per-issue 64-bit address arithmetic in VGPRs).
  const int KS = A.K >> 5;
  uint32_t wo[4], xo[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = 4 * wid + q;
    wo[q] = (uint32_t)(f * KS) * 1024u + lane * 16;
    const int row = min(row0 + 16 * f + c, A.M - 1);
    xo[q] = (uint32_t)row * (uint32_t)(A.ldx * 2) + 16 * g;
  }
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A.wp + (size_t)nt * 16 * KS * 512), 0, 16 * KS * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A.x, 0, (int)min(((long long)(A.M - 1) * A.ldx + A.K) * 2, 0x7fffffffll), 0x00020000);
  auto stage = [&](int s) -> char* { return smem + (s & 3) * W4_STAGE; };
  // LDS-DMA piece q (0-7) of step s: W chunk 4 wid + (q >> 1) (q even) or x fragment
  // 4 wid + (q >> 1) (q odd)
  auto issue1 = [&](int s, int q) {
    char* st = stage(s) + (4 * wid + (q >> 1)) * 1024;
    if (q & 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_t*)(st + 16384), 16, xo[q >> 1], (ks0 + s) * 64, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_t*)st, 16, wo[q >> 1], (ks0 + s) * 1024, 0, 0);
  };
  // fragment reads of step s: W n-frag 8 wn + k, x m-frag 8 wm + k
  auto read_w = [&](int s, int k, bf16x8& wf) {
    wf = *reinterpret_cast<const bf16x8*>(stage(s) + lane * 16 + (8 * wn + k) * 1024);
  };
  auto read_x = [&](int s, int k, bf16x8& xf) {
    xf = *reinterpret_cast<const bf16x8*>(stage(s) + lane * 16 + 16384 + (8 * wm + k) * 1024);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // registers: the x fragments of a step are held whole (two sets: this step's and the next
  // one's); the W fragments go through a ring of 4, each read two chunks before its use
  bf16x8 xa[8], xb2[8], wr[4];

  // One step, hand-placed: 8 chunks of 8 MFMAs (W n-frag k x the 8 x m-frags). Ahead of
  // chunk k: LDS-DMA piece k of step s + 3, x fragment k of step s + 1, and W fragment k + 2
  // of this step (k <= 5) or k - 6 of step s + 1; sched_barrier fences keep hipcc from
  // regrouping them. ST: 0 steady (issue s + 3, wait for s + 2), 1: s + 3 == n (wait for the
  // last issued step), 2: s + 2 == n (reads only), 3: the last step (MFMAs only).
  auto step = [&](int s, auto st, const bf16x8(&xc)[8], bf16x8(&xn)[8]) {
    constexpr int S = decltype(st)::value;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (S == 0) issue1(s + 3, k);
      if constexpr (S < 3) read_x(s + 1, k, xn[k]);
      if (k < 6) read_w(s, k + 2, wr[(k + 2) & 3]);
      else if constexpr (S < 3) read_w(s + 1, k - 6, wr[(k + 2) & 3]);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[k][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[k & 3], xc[j], acc[k][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (S < 3) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this step's reads of stage s + 1 done
      if constexpr (S == 0) wait_vm<8>();
      else if constexpr (S == 1) wait_vm<0>();
      raw_barrier();
    }
  };

#pragma unroll
  for (int q = 0; q < 8; ++q) issue1(0, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) issue1(1, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) issue1(2, q);
  wait_vm<8>();  // steps 0 and 1 landed
  raw_barrier();
#pragma unroll
  for (int k = 0; k < 8; ++k) read_x(0, k, xa[k]);
  read_w(0, 0, wr[0]);
  read_w(0, 1, wr[1]);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  int s = 0;
  for (; s + 4 < n; s += 2) {
    step(s, ic<0>{}, xa, xb2);
    step(s + 1, ic<0>{}, xb2, xa);
  }
  step(s, ic<0>{}, xa, xb2);
  step(s + 1, ic<1>{}, xb2, xa);
  step(s + 2, ic<2>{}, xa, xb2);
  step(s + 3, ic<3>{}, xb2, xa);

  // ---- split tiles: publish, the last arriver sums the other slices into its registers
  if (slice >= 0) {
    float* base = A.ws + (size_t)(tile - A.full) * A.S * SLABF;
    {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(base + (size_t)slice * SLABF, 0, SLABF * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                 (((wid * 8 + i) * 8 + j) * 64 + lane) * 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(A.counters + (tile - A.full), A.S, reinterpret_cast<int*>(smem), A.acq)) return;
    for (int p = 0; p < A.S; ++p) {
      if (p == slice) continue;
      const __amdgpu_buffer_rsrc_t rp =
          __builtin_amdgcn_make_buffer_rsrc(base + (size_t)p * SLABF, 0, SLABF * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f32x4 tt[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          tt[j] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, (((wid * 8 + i) * 8 + j) * 64 + lane) * 16, 0, 16));
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] += tt[j];
      }
    }
  }

  // ---- register epilogue: acc[i][j] holds token row0 + 128 wm + 16 j + c, columns
  // 4 g .. 4 g + 3 of 16-column tile nt * 16 + 8 wn + i
  const float inv_k = 1.f / (float)A.K;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = row0 + wm * 128 + 16 * j + c;
    const bool ok = m < A.M;
    float sq = 0.f;
    if (ok) {
      float rs = 1.f;
      if constexpr (NORM) rs = rsqrtf(A.ss_in[m] * inv_k + A.eps);
      if constexpr (pair_epi<EPI>()) {
#pragma unroll
        for (int i = 0; i < 8; i += 2)
          store_quad<EPI>(A, m, nt * 16 + wn * 8 + i, 4 * g, acc[i][j] * rs, acc[i + 1][j] * rs);
      } else {
#pragma unroll
        for (int i = 0; i < 8; i += 2)
          sq += store_pair_wide<EPI>(A, m, nt * 16 + wn * 8 + i, g, acc[i][j] * rs, acc[i + 1][j] * rs);
      }
    }
    if constexpr (EPI == EP_RESID) {
      if (A.ss_out) {
        sq += __shfl_xor(sq, 16, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (ok && g == 0) atomicAdd(A.ss_out + m, sq);
      }
    }
  }
}

template <int EPI, bool NORM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void w4_gemm_kernel(const Args A) {
  __shared__ __attribute__((aligned(1024))) char smem[W4_SMEM];
  w4_tile<EPI, NORM>(A, blockIdx.x, gridDim.x, smem);
}

}  // namespace pf
}  // namespace pa
