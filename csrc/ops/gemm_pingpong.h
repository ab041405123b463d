// Ping-pong 256 x 256 MFMA GEMM for the large-M projections (included by
// gemm_prefill.hip, which owns the argument struct, the planner and the launcher).
//
//     y[M, N] = epi( rownorm(x)[M, K] · W[N, K]^T )      bf16 in/out, fp32 accumulate
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", re-derived for the
// operands this engine holds):
//
//   * 512 threads = two wave GROUPS of 4 (waves 0-3, 4-7; a SIMD hosts one wave of each).
//     Group G owns W rows [128 G, 128 G + 128) of the tile, wave wc = wid & 3 owns tokens
//     [64 wc, 64 wc + 64): 128 x 64 outputs per wave, acc[8 n-frags][4 m-frags] of
//     v_mfma_f32_16x16x32_bf16 run as C^T = W · x^T, so each lane ends with 4 consecutive
//     output columns of one token (the packed_epi.h register epilogues).
//   * the groups run half a phase apart (one extra s_barrier for group 1 up front): while
//     group 0 runs its MFMA segment, group 1 issues its LDS reads and LDS-DMA pieces, and
//     vice versa, so every SIMD pairs one matrix-bound wave with one memory-bound wave.
//   * a 64-k tile lives in one of two 64-KiB LDS buffers as four 16-KiB PARTS:
//       A0 = W n-frags 0-3 of both groups, A1 = W n-frags 4-7 (packed fragment-major W:
//            one 1-KiB chunk per LDS-DMA wave instruction, lane-linear, conflict-free reads),
//       B0 = token frags 0-1 of every wave, B1 = token frags 2-3 (x rows in full 128-B lines,
//            16-B units XOR-swizzled by (row >> 1) on the SOURCE address).
//   * schedule (`body2`): one 64-k tile = 2 phases of 32 MFMAs; each load segment retires
//     its own LDS reads (lgkmcnt(0)) before its barrier, so a part is restaged one phase after
//     its last read, and the counted vmcnt before a phase's first barrier retires exactly the
//     part(s) the next phase reads (guide: "read a staged buffer one phase after the wait that
//     retires it"). No vmcnt(0) and no __syncthreads() inside the loop. (A four-phase
//     schedule of 16-MFMA quadrants ran 9 % more loop cycles and was removed:
//     profiles/r3_pingpong_ph2_ab.jsonl.)
//   * s_setprio(1) around every MFMA cluster (guide §5.5 T5).
//
// Work items are those of the prefill launcher: whole tiles (XCD-aware bijective remap, row
// tiles of one W panel on one XCD) and, for the remainder, K-slices whose fp32 partials
// are handed to the tile's last arriver through common.h handoff_last.
#pragma once
#include "common.h"
#include "packed_epi.h"

namespace pa {
namespace pf {

constexpr int PP_PART = 16384;
// non-pair epilogues: 16-B stores of 8 columns per lane (packed_epi.h store_pair_wide)
// instead of 8-B quads
constexpr bool kPpWideStores = true;
constexpr int PP_BUF = 4 * PP_PART;

// STAMP (diagnostic build, whole tiles only): workgroup b's thread 0 writes s_memtime at
// entry / after the prologue / after the k-loop / after the epilogue and s_memrealtime at
// entry and exit to A.ws[8 b ..] (as uint64) -- a buffer no output is computed from.
// F = W n-frags per wave: 8 -> 256 x 256 tiles (two 64-KiB buffers of parts A0 A1 B0 B1,
// schedule at `body2`); 6 -> 256 x 192 tiles (two 56-KiB buffers of [W: 24 KiB | B0 | B1],
// schedule at `body6`: N = 6,144, Llama-3-8B qkv, is 32 column tiles, so M in
// (1,280, 2,048] fills the 256 CUs in one round instead of 144-192 256 x 256 tiles);
// 4 -> 256 x 128 tiles (three 48-KiB buffers of parts A B0 B1, schedule at `body4`).
template <int EPI, bool NORM, bool STAMP = false, int F = 8>
__device__ __forceinline__ void pingpong_tile(const Args& A, const int bid, const int nblocks, char* smem) {
  static_assert(F == 8 || F == 6 || F == 4, "256-, 192- or 128-wide tiles");
  constexpr int NA = F / 4;                 // W parts per 64-k tile (F = 8, 4)
  constexpr int WB = F == 6 ? 24 * 1024 : NA * PP_PART;  // W bytes per tile buffer
  constexpr int BUFB = WB + 2 * PP_PART;    // bytes per tile buffer
  constexpr int NBUF = F == 4 ? 3 : 2;
  constexpr int SLABF = 256 * 32 * F;       // floats per split slab
  uint64_t st0 = 0, st1 = 0, st2 = 0, rt0 = 0;
  if constexpr (STAMP) {
    st0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = wid >> 2, wc = wid & 3;
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
  const int nk = kt1 - kt0;  // >= 2 (launcher)

  if (A.ss_zero && bid == 0)
    for (int i = threadIdx.x; i < A.M; i += 512) A.ss_zero[i] = 0.f;

  // ---- LDS-DMA sources. Every part is 16 wave instructions, two per wave.
  // W part r: chunk q = 2 wid + h (h = 0, 1) is n-frag (wid & 3) of group (wid >> 2),
  // k-half h of the 64-k tile: n16 tile nt * 16 + (wid >> 2) * 8 + r * 4 + (wid & 3).
  const int KS = A.K >> 5;
  // x part c: LDS row lr = (2 wid + h) * 8 + (lane >> 3) holds token (lr >> 5) * 64 + 32 c +
  // (lr & 31); its 16-B unit (lane & 7) is the row's logical unit (lane & 7) ^ ((lr >> 1) & 7).
  int xrow[2][2], xunit[2][2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lr = (2 * wid + h) * 8 + (lane >> 3);
      xrow[cc][h] = min(row0 + (lr >> 5) * 64 + cc * 32 + (lr & 31), A.M - 1);
      xunit[cc][h] = (lane & 7) ^ ((lr >> 1) & 7);
    }
  char* const sbase = smem;
  auto buf = [&](int t) -> char* { return sbase + (NBUF == 2 ? (t & 1) : (t % 3)) * BUFB; };

  const bf16* wsrc[F == 6 ? 3 : 2];
  const bf16* xsrc[2][2];
  if constexpr (F == 6) {
    // 24 W chunks per 64-k tile, three per wave: chunk q = 3 wid + j is k-half (q & 1) of
    // n-frag (q % 12) >> 1 of group q / 12, at LDS offset q KiB
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int q = 3 * wid + j;
      wsrc[j] = A.wp + ((size_t)(nt * 12 + (q / 12) * 6 + ((q % 12) >> 1)) * KS + (q & 1)) * 512 + lane * 8;
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int h = 0; h < 2; ++h) xsrc[cc][h] = A.x + (size_t)xrow[cc][h] * A.ldx + xunit[cc][h] * 8;
  } else {
#pragma unroll
    for (int r = 0; r < NA; ++r)
      wsrc[r] = A.wp + ((size_t)(nt * 2 * F + G * F + r * 4 + wc) * KS) * 512 + lane * 8;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int h = 0; h < 2; ++h) xsrc[cc][h] = A.x + (size_t)xrow[cc][h] * A.ldx + xunit[cc][h] * 8;
  }
  auto issue_w = [&](int r, int t) {
    char* dst = buf(t) + r * PP_PART + (2 * wid) * 1024;
    const bf16* s = wsrc[r] + (size_t)(2 * (kt0 + t)) * 512;
    glds16(s, dst);
    glds16(s + 512, dst + 1024);
  };
  auto issue_x = [&](int cc, int t) {
    char* dst = buf(t) + WB + cc * PP_PART + (2 * wid) * 1024;
    const size_t ko = (size_t)(kt0 + t) * 64;
    glds16(xsrc[cc][0] + ko, dst);
    glds16(xsrc[cc][1] + ko, dst + 1024);
  };
  // fragment reads: W frags of part r (4 n-frags x 2 k-halves), x frags of part cc
  // (2 token frags x 2 k-halves)
  auto read_w = [&](int r, int t, bf16x8(&af)[4][2]) {
    const char* p = buf(t) + r * PP_PART + (G * 8) * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) af[i][h] = *reinterpret_cast<const bf16x8*>(p + (2 * i + h) * 1024);
  };
  // F = 6: all 24 W chunks of tile t, three per wave
  auto issue_w6 = [&](int t) {
    char* dst = buf(t) + (3 * wid) * 1024;
    const size_t ko = (size_t)(2 * (kt0 + t)) * 512;
#pragma unroll
    for (int j = 0; j < 3; ++j) glds16(wsrc[j] + ko, dst + j * 1024);
  };
  // F = 6: n-frags 3 p .. 3 p + 2 of this wave's group (x 2 k-halves)
  auto read_w6 = [&](int p, int t, bf16x8(&af)[3][2]) {
    const char* s = buf(t) + (G * 12 + 6 * p) * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) af[i][h] = *reinterpret_cast<const bf16x8*>(s + (2 * i + h) * 1024);
  };
  auto read_x = [&](int cc, int t, bf16x8(&bfr)[2][2]) {
    const char* p = buf(t) + WB + cc * PP_PART;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lr = wc * 32 + 16 * j + c;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int u = 4 * h + g;
        bfr[j][h] = *reinterpret_cast<const bf16x8*>(p + lr * 128 + ((u ^ ((lr >> 1) & 7)) << 4));
      }
    }
  };

  f32x4 acc[F][4];
#pragma unroll
  for (int i = 0; i < F; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 16 MFMAs of quadrant (W part r, x part cc)
  auto mma = [&](auto rr, auto ccc, const bf16x8(&af)[4][2], const bf16x8(&bfr)[2][2]) {
    constexpr int r = decltype(rr)::value, cc = decltype(ccc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[r * 4 + i][cc * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][h], bfr[j][h], acc[r * 4 + i][cc * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [] { __builtin_amdgcn_s_waitcnt(0xC07F); };
  // 32 MFMAs: W part r (4 n-frags) x all 4 token frags x K = 64
  auto mma32 = [&](auto rr, const bf16x8(&af)[4][2], const bf16x8(&b0)[2][2], const bf16x8(&b1)[2][2]) {
    constexpr int r = decltype(rr)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[r * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][h], j < 2 ? b0[j][h] : b1[j - 2][h],
                                                                      acc[r * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // 24 MFMAs: n-frags 3 p .. 3 p + 2 x all 4 token frags x K = 64 (F = 6)
  auto mma24 = [&](auto pp, const bf16x8(&af)[3][2], const bf16x8(&b0)[2][2], const bf16x8(&b1)[2][2]) {
    constexpr int p = decltype(pp)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[3 * p + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][h], j < 2 ? b0[j][h] : b1[j - 2][h],
                                                                      acc[3 * p + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  bf16x8 af[4][2], bx0[2][2], bx1[2][2];
  bf16x8 a6[3][2];

  // 256 x 128 tiles: one 64-k tile = 2 phases, three buffers
  //     phase  reads (tile t)   MFMA        LDS-DMA issued            vmcnt
  //     0      A (8), B0 (4)    A x B0      A, B0 of tile t + 2       10
  //     1      B1 (4)           A x B1      B1 of tile t + 2           8
  // (a part is restaged two phases after its last read; the wait before a phase's first
  // barrier retires exactly what the next phase reads)
  auto body4 = [&](int t, auto st) {
    constexpr int S = decltype(st)::value;  // 0 steady, 1 tile nk - 2, 2 the last tile
    read_w(0, t, af);
    read_x(0, t, bx0);
    if constexpr (S == 0) {
      issue_w(0, t + 2);
      issue_x(0, t + 2);
      wait_vm<10>();
    } else if constexpr (S == 1) {
      wait_vm<6>();
    } else {
      wait_vm<0>();
    }
    raw_barrier();
    lgkm0();
    mma(ic<0>{}, ic<0>{}, af, bx0);
    raw_barrier();
    read_x(1, t, bx1);
    if constexpr (S == 0) {
      issue_x(1, t + 2);
      wait_vm<8>();
    } else if constexpr (S == 1) {
      wait_vm<2>();
    }
    raw_barrier();
    lgkm0();
    mma(ic<0>{}, ic<1>{}, af, bx1);
    raw_barrier();
  };

  // 256 x 256 tiles, two phases per 64-k tile:
  //     phase  reads (tile t)          MFMA              LDS-DMA issued          vmcnt
  //     0      A0 (8), B0 (4), B1 (4)  A0 x (B0, B1)     B1, A1 of tile t + 1      8
  //     1      A1 (8)                  A1 x (B0, B1)     A0, B0 of tile t + 2      6
  // lgkmcnt(0) before each load segment's barrier, so a part is restaged one phase after its
  // last read (the partner group's reads of that phase are retired behind the same barrier).
  auto body2 = [&](int t, auto st) {
    constexpr int S = decltype(st)::value;  // 0 steady, 1 tile nk - 2, 2 the last tile
    read_w(0, t, af);
    read_x(0, t, bx0);
    read_x(1, t, bx1);
    if constexpr (S < 2) {
      issue_x(1, t + 1);
      issue_w(1, t + 1);
      wait_vm<8>();
    } else {
      wait_vm<0>();
    }
    lgkm0();
    raw_barrier();
    mma32(ic<0>{}, af, bx0, bx1);
    raw_barrier();
    read_w(1, t, af);
    if constexpr (S == 0) {
      issue_w(0, t + 2);
      issue_x(0, t + 2);
      wait_vm<6>();
    } else if constexpr (S == 1) {
      wait_vm<2>();
    }
    lgkm0();
    raw_barrier();
    mma32(ic<1>{}, af, bx0, bx1);
    raw_barrier();
  };

  // 256 x 192 tiles, two phases per 64-k tile (F = 6):
  //     phase  reads (tile t)               MFMA                  LDS-DMA issued       vmcnt
  //     0      W n 0-2 (6), B0 (4), B1 (4)  n 0-2 x (B0, B1)      W of tile t + 1        -
  //     1      W n 3-5 (6)                  n 3-5 x (B0, B1)      B0, B1 of tile t + 2   4
  // W of a tile is read in both phases, so W(t + 1) goes into the other buffer after the
  // barrier that ends tile t - 1; B0 / B1 are read in phase 0 only, so B(t + 2) is restaged
  // in phase 1. The phase-1 wait leaves only B(t + 2) in flight: W(t + 1) and B(t + 1),
  // read by the next phase 0, have landed. Every wave issues 3 + 4 LDS-DMA instructions per
  // tile, so the counted waits hold for all eight.
  auto body6 = [&](int t, auto st) {
    constexpr int S = decltype(st)::value;  // 0 steady, 1 tile nk - 2, 2 the last tile
    read_w6(0, t, a6);
    read_x(0, t, bx0);
    read_x(1, t, bx1);
    if constexpr (S < 2) issue_w6(t + 1);
    lgkm0();
    raw_barrier();
    mma24(ic<0>{}, a6, bx0, bx1);
    raw_barrier();
    read_w6(1, t, a6);
    if constexpr (S == 0) {
      issue_x(0, t + 2);
      issue_x(1, t + 2);
      wait_vm<4>();
    } else if constexpr (S == 1) {
      wait_vm<0>();
    }
    lgkm0();
    raw_barrier();
    mma24(ic<1>{}, a6, bx0, bx1);
    raw_barrier();
  };

  int t = 0;
  if constexpr (F == 6) {
    issue_x(0, 0);
    issue_x(1, 0);
    issue_w6(0);
    issue_x(0, 1);
    issue_x(1, 1);
    wait_vm<4>();  // B0, B1 and W of tile 0 landed
    raw_barrier();
    if (G == 1) raw_barrier();
    if constexpr (STAMP) st1 = __builtin_amdgcn_s_memtime();
    for (; t + 2 < nk; ++t) body6(t, ic<0>{});
    body6(t, ic<1>{});
    body6(t + 1, ic<2>{});
  } else if constexpr (F == 8) {
    issue_w(0, 0);
    issue_x(0, 0);
    issue_x(1, 0);
    issue_w(1, 0);
    issue_w(0, 1);
    issue_x(0, 1);
    wait_vm<6>();  // A0, B0 and B1 of tile 0 landed
    raw_barrier();
    if (G == 1) raw_barrier();
    if constexpr (STAMP) st1 = __builtin_amdgcn_s_memtime();
    for (; t + 2 < nk; ++t) body2(t, ic<0>{});
    body2(t, ic<1>{});
    body2(t + 1, ic<2>{});
  } else {
    issue_w(0, 0);
    issue_x(0, 0);
    issue_x(1, 0);
    issue_w(0, 1);
    issue_x(0, 1);
    issue_x(1, 1);
    wait_vm<8>();  // A and B0 of tile 0 landed
    raw_barrier();
    if (G == 1) raw_barrier();
    if constexpr (STAMP) st1 = __builtin_amdgcn_s_memtime();
    for (; t + 2 < nk; ++t) body4(t, ic<0>{});
    body4(t, ic<1>{});
    body4(t + 1, ic<2>{});
  }
  if (G == 0) raw_barrier();  // balance the stagger
  if constexpr (STAMP) st2 = __builtin_amdgcn_s_memtime();

  // ---- split tiles: publish, the last arriver sums the other slices into its registers
  if (slice >= 0) {
    float* base = A.ws + (size_t)(tile - A.full) * A.S * SLABF;
    {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(base + (size_t)slice * SLABF, 0, SLABF * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < F; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                 (((wid * F + i) * 4 + j) * 64 + lane) * 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(A.counters + (tile - A.full), A.S, reinterpret_cast<int*>(smem), A.acq)) return;
    for (int p = 0; p < A.S; ++p) {
      if (p == slice) continue;
      const __amdgpu_buffer_rsrc_t rp =
          __builtin_amdgcn_make_buffer_rsrc(base + (size_t)p * SLABF, 0, SLABF * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < F; i += 2) {
        f32x4 tt[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            tt[h][j] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, (((wid * F + i + h) * 4 + j) * 64 + lane) * 16, 0, 16));
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i + h][j] += tt[h][j];
      }
    }
  }

  // ---- register epilogue: acc[i][j] holds token row0 + 64 wc + 16 j + c, columns
  // 4 g .. 4 g + 3 of 16-column tile nt * 2F + F G + i
  const float inv_k = 1.f / (float)A.K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = row0 + wc * 64 + 16 * j + c;
    const bool ok = m < A.M;
    float sq = 0.f;
    if (ok) {
      float rs = 1.f;
      if constexpr (NORM) rs = rsqrtf(A.ss_in[m] * inv_k + A.eps);
      if constexpr (pair_epi<EPI>()) {
#pragma unroll
        for (int i = 0; i < F; i += 2)
          store_quad<EPI>(A, m, nt * 2 * F + G * F + i, 4 * g, acc[i][j] * rs, acc[i + 1][j] * rs);
      } else {
        if constexpr (kPpWideStores) {
#pragma unroll
          for (int i = 0; i < F; i += 2)
            sq += store_pair_wide<EPI>(A, m, nt * 2 * F + G * F + i, g, acc[i][j] * rs, acc[i + 1][j] * rs);
        } else {
#pragma unroll
          for (int i = 0; i < F; ++i)
            sq += store_quad<EPI>(A, m, nt * 2 * F + G * F + i, 4 * g, acc[i][j] * rs, acc[i][j]);
        }
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
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t st3 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      uint64_t* d = reinterpret_cast<uint64_t*>(A.ws) + (size_t)bid * 8;
      const uint64_t v[8] = {st0, st1, st2, st3, rt0, rt1, (uint64_t)tile, 0};
#pragma unroll
      for (int q = 0; q < 8; ++q) __hip_atomic_store(d + q, v[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// One tile family per launch: the whole grid runs pingpong_tile.
template <int EPI, bool NORM, bool STAMP = false, int F = 8>
__global__ __launch_bounds__(512) void pingpong_gemm_kernel(const Args A) {
  __shared__ __attribute__((aligned(1024))) char smem[(F == 8 ? 2 * 4 : F == 6 ? 7 : 3 * 3) * PP_PART];
  pingpong_tile<EPI, NORM, STAMP, F>(A, blockIdx.x, gridDim.x, smem);
}

// Full rounds of 256 x 256 tiles, then the remaining columns as 256 x 128 tiles in the same
// launch (workgroups [0, nbig) run A's 256-wide tiles, the rest B's 128-wide tiles of the
// columns A leaves out): a tail of r <= 128 wide tiles costs one round of half-size tiles
// (~60 % of a wide-tile round) instead of a whole wide-tile round.
template <int EPI, bool NORM>
__global__ __launch_bounds__(512) void pingpong_mixed_kernel(const Args A, const Args B, const int nbig) {
  __shared__ __attribute__((aligned(1024))) char smem[9 * PP_PART];
  if ((int)blockIdx.x < nbig)
    pingpong_tile<EPI, NORM, false, 8>(A, blockIdx.x, nbig, smem);
  else
    pingpong_tile<EPI, NORM, false, 4>(B, blockIdx.x - nbig, gridDim.x - nbig, smem);
}

}  // namespace pf
}  // namespace pa
