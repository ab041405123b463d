// Mid-size projections (48 < M <= 512 tokens) on the packed weights.
//
//     y[M, N] = epi( rownorm(x)[M, K] · W[N, K]^T )      bf16 in/out, fp32 accumulate
//
// These are the steps that carry prefill chunks beside the decode rows of 64
// concurrent agents (BASELINE config 3: 49-512-token steps are a third of the
// GPU time). hipBLASLt runs them at 1.4-2.5 TB/s of weight traffic
// (profiles/r2_midm_hipblaslt.jsonl: down 58.7 us at M = 128 for 117 MB), i.e.
// neither at the HBM roofline nor at the MFMA roofline. This kernel is built for
// that regime:
//
//   * a workgroup (4 waves, 2 x 2) owns a BM x BN output tile (BM = 32 FM token
//     rows, BN = 32 FN columns) and one K slice; the grid is (K slices) x (column
//     tiles) x (row tiles), mapped XCD-aware so the row tiles of one column tile
//     (same weights) and the column tiles of one slice (same x panel) share an L2;
//   * BOTH operands are staged global -> LDS with global_load_lds (no VGPR round
//     trip, no ds_write), 64 k per stage, 3-4 stages in flight, drained with a
//     counted vmcnt and raw s_barrier (guide §5 "pipelining across barriers") —
//     one barrier per 64 k;
//   * the weights are the fragment-major packed copy (ops.pack_decode_weight), so a
//     weight stage is whole 1-KiB wave loads and a lane-linear, conflict-free LDS
//     image; x rows are 128-B lines whose 16-B units are XOR-swizzled by (row >> 1)
//     on the SOURCE address (LDS-DMA writes lane-linear), which makes every 16-row
//     fragment read conflict-free under the ds_read_b128 lane groups;
//   * the MFMA runs with the weights as the A operand (C^T = W · x^T), so each lane
//     ends with 4 CONSECUTIVE output columns of one token: 8-byte stores, and the
//     epilogues (RMSNorm row scale, SwiGLU over interleaved gate/up tiles, residual
//     add, RoPE + paged KV write over the (i, i + 64) tile pairs of the rope-packed
//     QKV) run on registers;
//   * RMSNorm costs the main loop nothing: the norm weight is folded into the packed
//     weights and the row statistics come from the PRODUCER of x — the residual-add
//     epilogue that writes h accumulates sum(h^2) per row (LDS, then one fp32 atomic
//     per row and workgroup) into a buffer the next projection reads;
//   * split-K partials go to fp32 slabs with write-through (sc1) stores; the last
//     slice to take the tile's ticket reduces them and runs the epilogue — one launch.
#include "common.h"
#include "packed_epi.h"

#include <algorithm>

namespace pa {
namespace mid {

using pk::EP_PLAIN;
using pk::EP_SILU;
using pk::EP_RESID;
using pk::EP_ROPEPERM;
using pk::EP_ROPEKV;

struct Args {
  bf16* y;
  const bf16* x;
  const bf16* wp;
  const bf16* resid;
  float* ws;      // split-K slabs: [tiles][S][BM][BN] fp32
  int* counters;  // [tiles] arrival tickets, zero between launches (the last arriver resets)
  int M, N, K, ldx, ldy, ldr;
  int S, per;     // K slices, 64-k chunks per slice
  int MT, NT;     // row tiles, column tiles
  float eps;
  const float* ss_in;  // NORM: [M] row sum(x^2) over K (rows scaled by rsqrt(ss / K + eps))
  float* ss_out;       // EP_RESID (optional): [M] += row sum(y^2) of the written (bf16) output
  float* ss_zero;      // optional: [M] zeroed by workgroup 0 (the buffer the NEXT residual fills)
  // EP_ROPEKV
  bf16* q_out;           // [M, H, 128]
  bf16* k_cache;         // [NB, KV, 16, 16, 8]  fragment-major pages (rope_cache.hip)
  bf16* v_cache;         // [NB, KV, 128, 16]
  const int* positions;  // [M]
  const int* slots;      // [M], < 0 = no cache write
  const float* cos_sin;  // [max_pos, 128] (cos | sin)
  int H, KV;
  int acq;  // hand-off consumer mode (common.h handoff_last)
};

typedef __attribute__((address_space(3))) void lds_t;
typedef __attribute__((address_space(1))) void gbl_t;

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at "no wait"); gfx9 encoding.
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void glds16(const bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_t*)src, (lds_t*)lds, 16, 0, 0);
}
// gate_up's weight stream when one row tile covers M (each weight byte read once per step):
// non-temporal, 1-3 % faster at M = 64-256. The other projections keep the default policy:
// with nt o_proj at M = 256 ran 34.4 -> 37.9 us, down and qkv 1-3 % slower
// (profiles/r2_nt_weights_ab.jsonl).
__device__ __forceinline__ void glds16_nt(const bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_t*)src, (lds_t*)lds, 16, 0, 2);
}

using pk::ropeperm_tile;
using pk::store_quad;
using pk::pair_epi;

template <int FM, int FN, int EPI, bool NORM, bool WNT>
__global__ __launch_bounds__(256) void mid_gemm_kernel(const Args A) {
  constexpr int BM = 32 * FM, BN = 32 * FN, NTL = BN / 16;  // tiles per block
  constexpr int XB = BM * 128, WB = BN * 128, SB = XB + WB;  // bytes per stage
  // stages: as many as fit 160 KiB (<= 8); PF = chunks in flight beyond the one being read
  constexpr int STAGES = (160 * 1024 / SB) < 8 ? (160 * 1024 / SB) : 8;
  constexpr int PF = STAGES - 2;
  static_assert(PF >= 1, "tile too large for the LDS pipeline");
  constexpr int NPC = FM + FN;                                 // LDS-DMA loads per wave per stage
  static_assert(!pair_epi<EPI>() || FN % 2 == 0, "pair epilogues need an even tile count per wave");
  // the only LDS object (guide §5 trap 4a): the stages, reused after the k-loop
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SB];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  // XCD-aware bijective remap: consecutive work ids share an XCD (and its L2)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int mt = work % A.MT;
  const int nt = (work / A.MT) % A.NT;
  const int s = work / (A.MT * A.NT);
  const int KS = A.K >> 5;
  const int c0 = s * A.per;
  const int nch = min(A.per, (KS >> 1) - c0);
  const int row0 = mt * BM;

  // per-lane LDS-DMA sources; stage image: [x: BM rows x 128 B][w: NTL tiles x 2 k-steps x 1 KiB]
  const bf16* xsrc[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r = (wid * FM + i) * 8 + (lane >> 3);
    const int gr = min(row0 + r, A.M - 1);
    const int unit = (lane & 7) ^ ((r >> 1) & 7);
    xsrc[i] = A.x + (size_t)gr * A.ldx + c0 * 64 + unit * 8;
  }
  const bf16* wsrc[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int p = wid * FN + i;  // piece: local tile p >> 1, k-step p & 1
    wsrc[i] = A.wp + ((size_t)(nt * NTL + (p >> 1)) * KS + c0 * 2 + (p & 1)) * 512 + lane * 8;
  }
  auto issue = [&](int c, int b) {
    char* st = smem + b * SB;
#pragma unroll
    for (int i = 0; i < FM; ++i) glds16(xsrc[i] + c * 64, st + (wid * FM + i) * 1024);
    if constexpr (WNT) {
#pragma unroll
      for (int i = 0; i < FN; ++i) glds16_nt(wsrc[i] + (size_t)c * 1024, st + XB + (wid * FN + i) * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < FN; ++i) glds16(wsrc[i] + (size_t)c * 1024, st + XB + (wid * FN + i) * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (A.ss_zero && blockIdx.x == 0)
    for (int i = threadIdx.x; i < A.M; i += 256) A.ss_zero[i] = 0.f;

  // Fragments of one k-step (32 k) of stage b.
  auto read_frags = [&](int b, int ks, bf16x8 (&xf)[FM], bf16x8 (&wf)[FN]) {
    const char* st = smem + b * SB;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int row = (wm * FM + fm) * 16 + (lane & 15);
      const int u = 4 * ks + (lane >> 4);
      xf[fm] = *reinterpret_cast<const bf16x8*>(st + row * 128 + ((u ^ ((row >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
      wf[fn] = *reinterpret_cast<const bf16x8*>(st + XB + ((2 * (wn * FN + fn) + ks) * 64 + lane) * 16);
  };
  auto mma = [&](const bf16x8 (&xf)[FM], const bf16x8 (&wf)[FN]) {
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[fn], xf[fm], acc[fm][fn], 0, 0, 0);
  };
  // wait until chunk c has landed: `after` = chunks issued after it (<= PF - 1)
  auto wait_chunk = [&](int after) {
    if constexpr (PF >= 4) { if (after >= 3) { wait_vm<3 * NPC>(); return; } }
    if constexpr (PF >= 3) { if (after == 2) { wait_vm<2 * NPC>(); return; } }
    if constexpr (PF >= 2) { if (after == 1) { wait_vm<NPC>(); return; } }
    wait_vm<0>();
  };

  // Software pipeline: the fragment reads of the next k-step are in flight while the
  // current one's MFMAs run, and the barrier that publishes chunk c + 1 sits between the
  // two k-steps of chunk c. Stage (c + 1 + PF) % STAGES = (c - 1) % STAGES is refilled
  // right after that barrier: every wave finished reading chunk c - 1 before it.
  for (int p = 0; p < PF; ++p)
    if (p < nch) issue(p, p);
  bf16x8 xa[FM], wa[FN], xb[FM], wb[FN];
  if (nch > 0) {
    wait_chunk(min(PF, nch) - 1);
    raw_barrier();
    if (PF < nch) issue(PF, PF % STAGES);
    read_frags(0, 0, xa, wa);
  }
  int st = 0, c = 0;
  // steady state: branch-free body (a branch between the two MFMA groups makes hipcc
  // shuffle the accumulators through v_accvgpr moves every iteration)
  for (; c + 1 + PF < nch; ++c) {
    read_frags(st, 1, xb, wb);
    mma(xa, wa);
    wait_vm<(PF - 1) * NPC>();
    raw_barrier();
    const int nxt = c + 1 + PF;
    issue(nxt, nxt % STAGES);
    st = st + 1 == STAGES ? 0 : st + 1;
    read_frags(st, 0, xa, wa);
    mma(xb, wb);
  }
  for (; c + 1 < nch; ++c) {  // drain: nothing left to issue
    read_frags(st, 1, xb, wb);
    mma(xa, wa);
    wait_chunk(nch - 2 - c);
    raw_barrier();
    st = st + 1 == STAGES ? 0 : st + 1;
    read_frags(st, 0, xa, wa);
    mma(xb, wb);
  }
  if (nch > 0) {
    read_frags(st, 1, xb, wb);
    mma(xa, wa);
    mma(xb, wb);
  }

  const float inv_k = 1.f / (float)A.K;
  const int g = lane >> 4, cl = lane & 15;
  auto row_scale = [&](int m) -> float {
    if constexpr (NORM) return rsqrtf(A.ss_in[m] * inv_k + A.eps);
    else return 1.f;
  };

  if (A.S == 1) {
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int tl = (wm * FM + fm) * 16 + cl;
      const int m = row0 + tl;
      const bool ok = m < A.M;
      float sq = 0.f;
      if (ok) {
        const float rs = row_scale(m);
        if constexpr (pair_epi<EPI>()) {
#pragma unroll
          for (int fn = 0; fn < FN; fn += 2)
            store_quad<EPI>(A, m, nt * NTL + wn * FN + fn, 4 * g, acc[fm][fn] * rs, acc[fm][fn + 1] * rs);
        } else {
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            sq += store_quad<EPI>(A, m, nt * NTL + wn * FN + fn, 4 * g, acc[fm][fn] * rs, acc[fm][fn]);
        }
      }
      if constexpr (EPI == EP_RESID) {
        if (A.ss_out) {  // the 4 lane groups hold the 4 column quads of each row: reduce, 1 atomic
          sq += __shfl_xor(sq, 16, 64);
          sq += __shfl_xor(sq, 32, 64);
          if (ok && g == 0) atomicAdd(A.ss_out + m, sq);
        }
      }
    }
    return;
  }

  // ---- split-K: publish this slice's partial tile (write-through), the last arriver reduces
  const int tile_id = mt * A.NT + nt;
  float* slab_base = A.ws + (size_t)tile_id * A.S * BM * BN;
  {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slab_base + (size_t)s * BM * BN, 0, BM * BN * 4, 0x00020000);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int tl = (wm * FM + fm) * 16 + cl;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[fm][fn]), rs,
                                               (tl * BN + (wn * FN + fn) * 16 + 4 * g) * 4, 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is past its last LDS read of the stages
  int* lflag = reinterpret_cast<int*>(smem);
  float* rsq = reinterpret_cast<float*>(smem) + 4;  // [BM] row sum(y^2) of this tile (EP_RESID)
  if constexpr (EPI == EP_RESID)
    for (int i = threadIdx.x; i < BM; i += 256) rsq[i] = 0.f;
  if (!pa::handoff_last(A.counters + tile_id, A.S, lflag, A.acq)) return;
  const __amdgpu_buffer_rsrc_t rall =
      __builtin_amdgcn_make_buffer_rsrc(slab_base, 0, A.S * BM * BN * 4, 0x00020000);
  // thread -> (token row, 4 consecutive columns of one tile; pair epilogues: of an even tile).
  // RU quads per thread per pass with every slab load of the pass issued before the first
  // add (the slabs come from memory: one quad at a time put ~1.5 us of load latency per quad
  // on the critical path -- 16 quads per thread at BM = BN = 128 -- and made split-K tiles
  // slower than whole-K ones, profiles/r5_mid_splitk_reduce.jsonl)
  constexpr int QPR = BN / 4;                          // column quads per row
  constexpr int QW = pair_epi<EPI>() ? QPR / 2 : QPR;  // quads of work per row
  constexpr int NQ = BM * QW;
  constexpr int RU = 4;
  for (int e0 = threadIdx.x; e0 < NQ; e0 += 256 * RU) {
    int tl[RU], q4[RU];
    f32x4 sum[RU], sum2[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int e = min(e0 + u * 256, NQ - 1);
      tl[u] = e / QW;
      const int k = e % QW;
      q4[u] = pair_epi<EPI>() ? (k >> 2) * 32 + (k & 3) * 4 : k * 4;
      sum[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      sum2[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int p0 = 0; p0 < A.S; p0 += 4) {
      f32x4 v[4][RU], v2[4][RU];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int pp = min(p0 + p, A.S - 1);
          v[p][u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rall, ((pp * BM + tl[u]) * BN + q4[u]) * 4, 0, 16));
          if constexpr (pair_epi<EPI>())
            v2[p][u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rall, ((pp * BM + tl[u]) * BN + q4[u] + 16) * 4, 0, 16));
        }
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (p0 + p < A.S) {
#pragma unroll
          for (int u = 0; u < RU; ++u) {
            sum[u] += v[p][u];
            if constexpr (pair_epi<EPI>()) sum2[u] += v2[p][u];
          }
        }
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int m = row0 + tl[u];
      if (e0 + u * 256 >= NQ || m >= A.M) continue;
      const int lt = q4[u] >> 4, cq = q4[u] & 15;
      const float rs = row_scale(m);
      const float sq = store_quad<EPI>(A, m, nt * NTL + lt, cq, sum[u] * rs, sum2[u] * rs);
      if constexpr (EPI == EP_RESID) {
        if (A.ss_out) atomicAdd(rsq + tl[u], sq);  // LDS
      }
    }
  }
  if constexpr (EPI == EP_RESID) {
    if (A.ss_out) {
      __syncthreads();
      for (int i = threadIdx.x; i < BM; i += 256)
        if (row0 + i < A.M) atomicAdd(A.ss_out + row0 + i, rsq[i]);
    }
  }
}

// ---------------------------------------------------------------------------------
template <int FM, int FN>
static int launch_f(const Args& a, int epi, bool norm, int grid, hipStream_t st) {
#define PA_MID(E, NRM)                                                                                \
  do {                                                                                                \
    if (E == EP_SILU && a.MT == 1) hipLaunchKernelGGL((mid_gemm_kernel<FM, FN, E, NRM, true>), dim3(grid), dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((mid_gemm_kernel<FM, FN, E, NRM, false>), dim3(grid), dim3(256), 0, st, a);          \
  } while (0)
  switch (epi) {
    case EP_PLAIN:
      if (norm) PA_MID(EP_PLAIN, true); else PA_MID(EP_PLAIN, false);
      return 0;
    case EP_RESID:
      if (norm) return 1;
      PA_MID(EP_RESID, false);
      return 0;
    case EP_ROPEPERM:
      if (norm) PA_MID(EP_ROPEPERM, true); else PA_MID(EP_ROPEPERM, false);
      return 0;
    case EP_SILU:
      if constexpr (FN % 2 == 0) {
        if (norm) PA_MID(EP_SILU, true); else PA_MID(EP_SILU, false);
        return 0;
      }
      return 1;
    case EP_ROPEKV:
      if constexpr (FN % 2 == 0) {
        if (norm) PA_MID(EP_ROPEKV, true); else PA_MID(EP_ROPEKV, false);
        return 0;
      }
      return 1;
    default:
      return 1;
  }
#undef PA_MID
}

// Default decomposition. Tiles: the token tile covers M when it can (FM = 2/4/8 for
// M <= 64/128/256, row tiles of 256 above); the column tile is 128 wide (FN = 4), or 64
// (FN = 2) when 128-wide tiles leave fewer than 128 tiles x row tiles. Then split K until
// the grid reaches ~256 workgroups, keeping >= 8 chunks (512 k) per slice.
static void plan_default(int M, int N, int K, int epi, int& fm, int& fn, int& S) {
  fm = M <= 64 ? 2 : (M <= 128 ? 4 : 8);
  const int MT = (M + 32 * fm - 1) / (32 * fm);
  fn = 4;
  if ((N / 128) * MT < 128 && epi != EP_SILU && epi != EP_ROPEKV) fn = 2;
  const int NT = N / (32 * fn);
  const int tiles = MT * NT;
  const int chunks = K / 64;
  S = 1;
  while (tiles * S < 224 && chunks / (S + 1) >= 8) ++S;
}

}  // namespace mid
}  // namespace pa

extern "C" int pa_mid_gemm_plan(int M, int N, int K, int epi, int* fm, int* fn, int* S) {
  pa::mid::plan_default(M, N, K, epi, *fm, *fn, *S);
  return 0;
}

extern "C" long long pa_mid_gemm_ws_floats(int M, int N, int K, int fm, int fn, int S) {
  const int BM = 32 * fm, BN = 32 * fn;
  const long long MT = (M + BM - 1) / BM, NT = N / BN;
  (void)K;
  return S > 1 ? MT * NT * S * (long long)BM * BN : 0;
}

// out[m] = sum_k x[m, k]^2 in fp32 (the row statistics of the first norm of a step; every
// later one comes from a residual epilogue).
__global__ __launch_bounds__(256) void row_sumsq_kernel(float* __restrict__ out, const pa::bf16* __restrict__ x,
                                                        int M, int K, int ldx) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m = blockIdx.x * 4 + w;
  if (m >= M) return;
  const pa::bf16x8* row = reinterpret_cast<const pa::bf16x8*>(x + (size_t)m * ldx);
  float acc = 0.f;
  for (int i = lane; i < K / 8; i += 64) {
    const pa::bf16x8 v = row[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf((float)v[e], (float)v[e], acc);
  }
  acc = pa::wave_sum(acc);
  if (lane == 0) out[m] = acc;
}

extern "C" int pa_row_sumsq(float* out, const void* x, int M, int K, int ldx, hipStream_t st) {
  if (M <= 0) return 0;
  if (K % 8 || ldx % 8) return 1;
  hipLaunchKernelGGL(row_sumsq_kernel, dim3((M + 3) / 4), dim3(256), 0, st, out, (const pa::bf16*)x, M, K, ldx);
  return (int)hipGetLastError() == 0 ? 0 : -2;
}

// Returns 1 if the shape/config is not handled, 0 on success, -2 on a launch error.
// fm/fn/splits <= 0 pick the defaults. For epi 4 (RoPE + paged KV write) y is unused.
extern "C" int pa_mid_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws,
                           long long ws_floats, int* counters, int n_counters, int M, int N, int K, int ldx,
                           int ldy, int ldr, int epi, const float* ss_in, float* ss_out, float* ss_zero, float eps,
                           int fm, int fn, int splits, void* q_out, void* k_cache, void* v_cache,
                           const int* positions, const int* slots, const float* cos_sin, int H, int KV,
                           hipStream_t st) {
  using namespace pa::mid;
  if (M <= 0) return 0;
  if (K % 64 != 0 || N % 16 != 0 || epi < 0 || epi > 4) return 1;
  const int norm = ss_in != nullptr;
  if (epi == EP_RESID && (!resid || norm)) return 1;
  if (ss_out && epi != EP_RESID) return 1;
  if (epi == EP_ROPEKV && (!q_out || !k_cache || !v_cache || !positions || !slots || !cos_sin ||
                           N != (H + 2 * KV) * 128))
    return 1;
  int dfm, dfn, dS;
  plan_default(M, N, K, epi, dfm, dfn, dS);
  if (fm <= 0) fm = dfm;
  if (fn <= 0) fn = dfn;
  int S = splits > 0 ? splits : dS;
  const int BM = 32 * fm, BN = 32 * fn;
  if (N % BN) return 1;
  const int MT = (M + BM - 1) / BM, NT = N / BN;
  const int chunks = K / 64;
  S = std::max(1, std::min(S, chunks));
  int per = (chunks + S - 1) / S;
  S = (chunks + per - 1) / per;  // no empty slices
  if (S > 1) {
    const long long need = (long long)MT * NT * S * BM * BN;
    if (!ws || !counters || n_counters < MT * NT || need > ws_floats) return 1;
  }
  Args a{(pa::bf16*)y, (const pa::bf16*)x, (const pa::bf16*)wp, (const pa::bf16*)resid, ws, counters, M, N, K,
         ldx, ldy, ldr, S, per, MT, NT, eps, ss_in, ss_out, ss_zero, (pa::bf16*)q_out, (pa::bf16*)k_cache, (pa::bf16*)v_cache, positions,
         slots, cos_sin, H, KV, pa::g_handoff_acquire};
  const int grid = MT * NT * S;
  int rc;
  if (fm == 1 && fn == 1) rc = launch_f<1, 1>(a, epi, norm != 0, grid, st);
  else if (fm == 2 && fn == 1) rc = launch_f<2, 1>(a, epi, norm != 0, grid, st);
  else if (fm == 1 && fn == 2) rc = launch_f<1, 2>(a, epi, norm != 0, grid, st);
  else if (fm == 1 && fn == 4) rc = launch_f<1, 4>(a, epi, norm != 0, grid, st);
  else if (fm == 2 && fn == 2) rc = launch_f<2, 2>(a, epi, norm != 0, grid, st);
  else if (fm == 2 && fn == 4) rc = launch_f<2, 4>(a, epi, norm != 0, grid, st);
  else if (fm == 4 && fn == 2) rc = launch_f<4, 2>(a, epi, norm != 0, grid, st);
  else if (fm == 4 && fn == 4) rc = launch_f<4, 4>(a, epi, norm != 0, grid, st);
  else if (fm == 8 && fn == 2) rc = launch_f<8, 2>(a, epi, norm != 0, grid, st);
  else if (fm == 8 && fn == 4) rc = launch_f<8, 4>(a, epi, norm != 0, grid, st);
  else return 1;
  if (rc) return rc;
  return (int)hipGetLastError() == 0 ? 0 : -2;
}
