// Weight-streaming projections for mid-size steps (16 < M <= 256 tokens) on the packed
// weights (VERDICT r3 "next round" item 1).
//
//     y[M, N] = epi( rownorm(x)[M, K] · W[N, K]^T )      bf16 in/out, fp32 accumulate
//
// At 17-256 rows a Llama-3-8B projection is bound by what each CU can TAKE IN, not by the
// MFMA: the per-CU intake is  x_rows·K_slice·2  (activations, L2-resident)  +  the CU's share
// of the weights  (+ the fp32 partials of a K split). The round-3 kernels (gemm_mid.hip,
// gemm_prefill.hip) ran 192 workgroups of 32-256-row x panels over the whole K and reached
// 30-38 GB/s per CU (qkv at 64 rows: 768 KB per workgroup in 23.3 us). This kernel is laid
// out so that the per-CU intake is the minimum the shape allows and every CU works:
//
//   * decomposition: G column groups (CT tiles of 16 outputs) x S K-slices x RG row groups
//     = ~256 workgroups (one per CU), chosen per shape by the host (plan_default): the K
//     split keeps the x panel of a workgroup about as large as its weight share
//     (qkv / o at 64 rows: 128 KB of x + 196 / 128 KB of weights per CU instead of 768 KB);
//   * the weights (fragment-major packed, ops.pack_decode_weight: one 1-KiB wave load per
//     16 x 32 fragment) stream straight into VGPRs with non-temporal loads — every weight
//     byte is read once per step by one wave, so it needs no LDS round trip and must not
//     displace x in L2 (guide: "GEMV / decode weights: load straight to VGPRs");
//   * x is staged once per workgroup through LDS in full 128-B lines (16-B units XOR-
//     swizzled by (row >> 1) so the 16-row fragment reads are conflict-free), shared by all
//     waves; both streams are plain loads in one in-order register ring D chunks deep, so
//     hipcc's counted vmcnt covers both (no glds / register-load mix, guide §5 trap 4b);
//   * waves split the workgroup's tiles (TPW per wave) and optionally the k-steps of each
//     chunk (WK), so 4-8 waves keep >= 48 KB of weights in flight per CU;
//   * the K split is reduced by the workgroups of a group TOGETHER (not by a last arriver):
//     each writes its fp32 partial fragments to an uncached slab (ops.empty_handoff), arrives
//     on a per-group counter and waits for the others (all S slices of a group are resident:
//     the grid is at most one workgroup per CU), then reduces 1/S of the group's fragments
//     and runs the epilogue on them (RMSNorm row scale, SwiGLU, residual + the next norm's row
//     statistics, RoPE + paged KV write: packed_epi.h). Publish = 16-B sc1 slab stores, every
//     wave's vmcnt(0), the workgroup barrier, one lane's relaxed agent-scope arrive (optionally
//     behind an agent release, rel bit 0); consume = relaxed poll, agent-scope acquire + drain,
//     barrier, sc1 loads (MI355X_MICROARCH.md hand-off table row 1, plus the acquire). A
//     departure counter resets both counters, so they are zero between launches (hipGraph
//     replay safe). Every spin is bounded: a timed-out group barrier sets the err word, which
//     the engine reads back with every step and fails on (LLMEngine._health_check).
//
// Why the shipping form (rel = 0, no producer release) is ordered -- the ISA program order of
// one group member's publish and every member's consume:
//   P1  every wave: buffer_store_dwordx4 ... sc1 (cache-policy aux 16) of its fragments into
//       the slab, which is hipDeviceMallocUncached memory (MTYPE UC: neither a
//       CU's L1 nor any XCD's L2 may hold its lines, so there is no cached copy to write back
//       or to go stale -- the reason the release (buffer_wbl2 sc1) has nothing left to do here);
//   P2  every wave: asm volatile "s_waitcnt vmcnt(0)" -- the wave stalls until each of its
//       stores is acknowledged; an uncached write is acknowledged by the memory-side point that
//       orders it (the data fabric / memory channel), not by a cache;
//   P3  s_barrier (group_barrier's __syncthreads) -- no lane passes it before every wave of the
//       workgroup has passed P2;
//   P4  lane 0: global_atomic_add (relaxed, agent scope; executed at the L2/memory side) -- in
//       program order after P3, hence after every store of the workgroup was acknowledged;
//   C1  lane 0: relaxed agent-scope (sc1) polls of the same counter until it reads S -- a value
//       that exists only after all S members executed their P4;
//   C2  lane 0: fence(acquire, agent) = buffer_inv sc1 + s_waitcnt vmcnt(0), then s_barrier;
//   C3  every wave: buffer_load_dwordx4 sc1 of the slabs -- issued after C2 in program order,
//       bypassing L1 and reading the UC lines at the same memory-side point that acknowledged P2.
// So each slab load is issued after an acknowledgement of the store it reads (P2 < P3 < P4 <
// C1 < C2 < C3, each link a program-order or value dependence); this is row 1 of the measured
// hand-off table in MI355X_MICROARCH.md (one lane per storing workgroup signals with an agent
// atomic after every storing wave's vmcnt(0) and a barrier; the consumer polls with sc1 loads,
// its other waves load after a barrier; 16-B sc1 stores and loads), plus the acquire. The one
// hardware assumption is that P2's acknowledgement of an uncached write comes from its ordering
// point. Evidence: 0 bad runs in 1,200,000 poisoned repetitions with the release and, at rel = 0,
// 100,000 per engine plan (profiles/r6_stream_handoff_rel0.jsonl) plus 2,000 per plan in the GPU
// tier (tests/test_stream_gemm_gpu.py::test_stream_handoff_shipping_default_no_release).
// The round-4 failure (5 / 10,000 without a release) was the OTHER form, in gemm_decode /
// gemm_mid: the last arriver read its partners' slabs right after its own add returned, with no
// poll-then-acquire and 4-byte stores; those kernels keep the release.
#include "common.h"
#include "packed_epi.h"

#include <algorithm>
#include <type_traits>

namespace pa {
namespace sg {

using pk::EP_PLAIN;
using pk::EP_SILU;
using pk::EP_RESID;
using pk::EP_ROPEPERM;
using pk::EP_ROPEKV;
using pk::store_quad;

struct Args {
  bf16* y;
  const bf16* x;
  const bf16* wp;
  const bf16* resid;
  float* ws;      // slabs: [groups][S * WK][CT * MG fragments][64 lanes][4] fp32 (uncached)
  int* counters;  // [groups][2] arrive / depart, zero between launches
  int* err;       // set to 1 if a group barrier timed out (never in a healthy run)
  int M, N, K, ldx, ldy, ldr;
  int S, RG, G;   // K slices, row groups, column groups
  int KSW;        // k-steps (32 k) per K slice
  int epi;        // pk::EP_*
  float eps;
  const float* ss_in;  // NORM: [M] row sum(x^2) over K (rows scaled by rsqrt(ss / K + eps)); null = none
  float* ss_out;       // EP_RESID (optional): [M] += row sum(y^2) of the written (bf16) output
  float* ss_zero;      // optional: [M] zeroed by workgroup 0
  bf16* q_out;         // EP_ROPEKV
  bf16* k_cache;
  bf16* v_cache;
  const int* positions;
  const int* slots;
  const float* cos_sin;
  int H, KV;
  // bit 0: agent-scope release (buffer_wbl2 sc1 + drain) before arriving (off by default:
  // ops.STREAM_REL -- the sc1 form below passed 1.2M poisoned repetitions and the release costs
  // 2.5-5 us per launch); bit 1: each workgroup starts its K slice at a different chunk
  // (rotated order; HBM channel spread)
  int rel;
  // diagnostics (null in the engine): per workgroup 8 wall-clock stamps (s_memrealtime, 100 MHz):
  // [0] start, [1] first chunk in LDS, [2] main loop done, [3] group barrier passed, [4] end
  unsigned long long* stamps;
};

typedef __attribute__((address_space(1))) int gi32;

template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  // vmcnt / expcnt left at "no wait" (gfx9 encoding: vmcnt 63 = 0xF | 3 << 14, expcnt 7)
  __builtin_amdgcn_s_waitcnt(0xF | (7 << 4) | (N << 8) | (3 << 14));
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Arrive on the group counter and wait until all n workgroups of the group have arrived.
// Every storing wave has drained its slab stores (vmcnt(0)) before the barrier in here.
__device__ __forceinline__ void group_barrier(int* arrive, int n, int* err, int rel) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (rel) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int tk = __hip_atomic_fetch_add((gi32*)arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk != n - 1) {
      // bounded by wall time (s_memrealtime runs at 100 MHz): after 1 s a partner never ran;
      // give up and raise the err word (the engine fails the step) rather than hang
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load((gi32*)arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
          __hip_atomic_store((gi32*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    // the slabs are uncached and read with sc1 loads; the acquire also drops this CU's L1
    // copy of anything else a partner wrote (nothing here reads such data, kept for safety)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int EPI>
__device__ __forceinline__ float epi_quad(const Args& A, int m, int tile, int cq, f32x4 v, f32x4 v2) {
  return store_quad<EPI>(A, m, tile, cq, v, v2);
}

// Epilogue inputs that do not depend on the GEMM result (the row's norm scale, the residual
// quad, the RoPE angle and the KV slot), loaded BEFORE the group barrier so that the split-K
// epilogue after it waits on one memory round trip (the slab gather) instead of two or three.
struct Pre {
  float rs;
  bf16x4 rv;
  f32x4 c, sn;
  int slot;
};

__device__ __forceinline__ Pre preload(const Args& A, int m, int tile, int cq) {
  Pre p;
  p.rs = 1.f;
  p.slot = -1;
  p.c = f32x4{1.f, 1.f, 1.f, 1.f};
  p.sn = f32x4{0.f, 0.f, 0.f, 0.f};
  if (m >= A.M) return p;
  if (A.ss_in) p.rs = rsqrtf(A.ss_in[m] * (1.f / (float)A.K) + A.eps);
  if (A.epi == EP_RESID) {
    p.rv = *reinterpret_cast<const bf16x4*>(A.resid + (size_t)m * A.ldr + tile * 16 + cq);
  } else if (A.epi == EP_ROPEKV) {
    const int hh = tile >> 3;
    const int d = 16 * ((tile & 7) >> 1) + cq;
    if (hh < A.H + A.KV) {
      const float* cs = A.cos_sin + (size_t)A.positions[m] * 128;
      p.c = *reinterpret_cast<const f32x4*>(cs + d);
      p.sn = *reinterpret_cast<const f32x4*>(cs + 64 + d);
    }
    if (hh >= A.H) p.slot = A.slots[m];
  }
  return p;
}

// store_quad (packed_epi.h) on preloaded inputs: v / v2 already scaled by p.rs
__device__ __forceinline__ float epi_pre(const Args& A, int m, int tile, int cq, f32x4 v, f32x4 v2, const Pre& p) {
  if (A.epi == EP_SILU) return store_quad<EP_SILU>(A, m, tile, cq, v, v2);
  if (A.epi == EP_PLAIN) return store_quad<EP_PLAIN>(A, m, tile, cq, v, v2);
  if (A.epi == EP_ROPEPERM) return store_quad<EP_ROPEPERM>(A, m, tile, cq, v, v2);
  if (A.epi == EP_RESID) {
    bf16x4 o;
    float sq = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = (bf16)(v[r] + (float)p.rv[r]);
      const float f = (float)o[r];
      sq = fmaf(f, f, sq);
    }
    *reinterpret_cast<bf16x4*>(A.y + (size_t)m * A.ldy + tile * 16 + cq) = o;
    return sq;
  }
  // EP_ROPEKV: tile even = original head tile i (dims 16 i + cq ..), v2 = tile i + 4 (dims + 64)
  const int hh = tile >> 3;
  const int d = 16 * ((tile & 7) >> 1) + cq;
  f32x4 o1 = v, o2 = v2;
  if (hh < A.H + A.KV) {
    o1 = v * p.c - v2 * p.sn;
    o2 = v2 * p.c + v * p.sn;
  }
  bf16x4 b1, b2;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    b1[r] = (bf16)o1[r];
    b2[r] = (bf16)o2[r];
  }
  if (hh < A.H) {
    bf16* dst = A.q_out + ((size_t)m * A.H + hh) * 128;
    *reinterpret_cast<bf16x4*>(dst + d) = b1;
    *reinterpret_cast<bf16x4*>(dst + d + 64) = b2;
  } else if (p.slot >= 0) {
    const int blk = p.slot >> 4, off = p.slot & 15;
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
  return 0.f;
}

// MG: 16-row groups per workgroup (m_t = 16 MG rows); TPW: 16-column tiles per wave;
// WT x WK waves (tile groups x k-step groups); D: register-ring depth in chunks.
// A chunk is KC = 2 WK k-steps (64 WK k); each wave runs KW = 2 k-steps of every chunk.
template <int MG, int TPW, int WT, int WK, int D>
__global__ __launch_bounds__(WT * WK * 64) void stream_gemm_kernel(const Args A) {
  constexpr int W = WT * WK, NTH = W * 64;
  constexpr int MT = 16 * MG;          // rows per workgroup
  constexpr int CT = WT * TPW;         // tiles per workgroup
  constexpr int KW = 2, KC = 2 * WK;   // k-steps per wave / per chunk
  constexpr int XCH = WK * MT * 128;   // x bytes per chunk (LDS slot)
  constexpr int XU = WK * MT * 8;      // 16-B units per chunk
  constexpr int LX = (XU + NTH - 1) / NTH;  // x loads per thread per chunk (duplicates wrap)
  static_assert(D == 2 || D == 4 || D == 8 || D == 16, "even ring depth (LDS slot = chunk & 1)");
  // one LDS object only (guide §5 trap 4a): [2 x-slots][row sums of squares][flag]
  __shared__ __attribute__((aligned(1024))) char smem[2 * XCH + MT * 4 + 16];
  float* rsq = reinterpret_cast<float*>(smem + 2 * XCH);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wt = wid % WT, wk = wid / WT;
  // XCD-aware bijective remap: consecutive work ids share an XCD (row groups of one
  // (column group, slice) read the same weights from one L2)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int rg = work % A.RG;
  const int s = (work / A.RG) % A.S;
  const int grp = work / (A.RG * A.S);
  const int gid = grp * A.RG + rg;
  const int row0 = rg * MT;
  const int t0 = grp * CT;
  const int KS = A.K >> 5;
  const int kb0 = s * A.KSW;
  const int nch = A.KSW / KC;  // host: nch % D == 0, nch >= D
  // rotated chunk order (rel bit 1): chunk c of this workgroup is K chunk (c + rot) % nch
  const int rot = (A.rel & 2) ? (work * 5) % nch : 0;

  auto stamp = [&](int i) {
    if (A.stamps && threadIdx.x == 0) A.stamps[(size_t)bid * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (A.ss_zero && bid == 0)
    for (int i = threadIdx.x; i < A.M; i += NTH) A.ss_zero[i] = 0.f;
  for (int i = threadIdx.x; i < MT; i += NTH) rsq[i] = 0.f;

  // ---- sources
  const bf16x8* wsrc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
    wsrc[j] = reinterpret_cast<const bf16x8*>(A.wp + ((size_t)(t0 + wt * TPW + j) * KS + kb0 + wk * KW) * 512) + lane;
  const bf16* xsrc[LX];
  int xdst[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int e = (threadIdx.x + i * NTH) % XU;
    const int h = e / (MT * 8), r = (e >> 3) % MT, u = e & 7;
    const int gr = min(row0 + r, A.M - 1);
    xsrc[i] = A.x + (size_t)gr * A.ldx + kb0 * 32 + h * 64 + u * 8;
    xdst[i] = h * MT * 128 + r * 128 + ((u ^ ((r >> 1) & 7)) << 4);
  }

  bf16x8 wr[D][KW][TPW];
  bf16x8 xr[D][LX];
  f32x4 acc[MG][TPW];
#pragma unroll
  for (int i = 0; i < MG; ++i)
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One chunk's loads in a fixed order (x first, then the weights by k-step): the scheduling
  // barriers keep every chunk's loads in issue order, so the prologue and the loop body leave
  // the same per-register vmcnt distances and hipcc's counted waits stay at (D - 1) chunks
  // (without them it reordered the prologue and fell back to vmcnt(0) inside the loop).
  auto issue = [&](int c0, int d) {
    const int c = rot ? (c0 + rot) % nch : c0;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < LX; ++i) xr[d][i] = *reinterpret_cast<const bf16x8*>(xsrc[i] + (size_t)c * KC * 32);
#pragma unroll
    for (int i = 0; i < KW; ++i)
#pragma unroll
      for (int j = 0; j < TPW; ++j) wr[d][i][j] = __builtin_nontemporal_load(wsrc[j] + (size_t)(c * KC + i) * 64);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto consume = [&](int d, int slot) {
    char* st = smem + slot * XCH;
#pragma unroll
    for (int i = 0; i < LX; ++i) *reinterpret_cast<bf16x8*>(st + xdst[i]) = xr[d][i];
    wait_lgkm<0>();
    raw_barrier();
#pragma unroll
    for (int i = 0; i < KW; ++i) {
      const int kk = wk * KW + i;
      const int hb = (kk >> 1) * MT * 128, ks = kk & 1;
      bf16x8 xf[MG];
#pragma unroll
      for (int mg = 0; mg < MG; ++mg) {
        const int row = mg * 16 + (lane & 15);
        const int u = 4 * ks + (lane >> 4);
        xf[mg] = *reinterpret_cast<const bf16x8*>(st + hb + row * 128 + ((u ^ ((row >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int mg = 0; mg < MG; ++mg)
#pragma unroll
        for (int j = 0; j < TPW; ++j)
          acc[mg][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[d][i][j], xf[mg], acc[mg][j], 0, 0, 0);
    }
  };

#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d);
  int c = 0;
  for (; c + D < nch; c += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      consume(d, d & 1);
      if (c == 0 && d == 0) stamp(1);
      issue(c + d + D, d);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) {
    consume(d, d & 1);
    if (c == 0 && d == 0) stamp(1);
  }
  stamp(2);

  const bool pair = A.epi == EP_SILU || A.epi == EP_ROPEKV;
  const float inv_k = 1.f / (float)A.K;
  const int g = lane >> 4, cl = lane & 15;
  auto epi_any = [&](int m, int tile, f32x4 v, f32x4 v2) -> float {
    switch (A.epi) {
      case EP_PLAIN: return epi_quad<EP_PLAIN>(A, m, tile, 4 * g, v, v2);
      case EP_SILU: return epi_quad<EP_SILU>(A, m, tile, 4 * g, v, v2);
      case EP_RESID: return epi_quad<EP_RESID>(A, m, tile, 4 * g, v, v2);
      case EP_ROPEPERM: return epi_quad<EP_ROPEPERM>(A, m, tile, 4 * g, v, v2);
      default: return epi_quad<EP_ROPEKV>(A, m, tile, 4 * g, v, v2);
    }
  };
  auto row_stat = [&](int mg, int m, float sq) {  // the 4 lane groups hold a row's 4 column quads
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    if (g == 0 && m < A.M) atomicAdd(rsq + mg * 16 + cl, sq);  // LDS
  };
  auto flush_row_stats = [&]() {
    __syncthreads();
    if (A.ss_out)
      for (int i = threadIdx.x; i < MT; i += NTH) {
        const float v = rsq[i];
        if (v != 0.f && row0 + i < A.M) atomicAdd(A.ss_out + row0 + i, v);
      }
  };

  // ---- no K split anywhere: the epilogue straight from the accumulators (pair epilogues
  // need both tiles of a pair in one wave: TPW even)
  if (A.S * WK == 1 && (!pair || TPW % 2 == 0)) {
#pragma unroll
    for (int mg = 0; mg < MG; ++mg) {
      const int m = row0 + mg * 16 + cl;
      float sq = 0.f;
      if (m < A.M) {
        const float rs = A.ss_in ? rsqrtf(A.ss_in[m] * inv_k + A.eps) : 1.f;
        if (pair) {
#pragma unroll
          for (int j = 0; j + 1 < TPW; j += 2) epi_any(m, t0 + wt * TPW + j, acc[mg][j] * rs, acc[mg][j + 1] * rs);
        } else {
#pragma unroll
          for (int j = 0; j < TPW; ++j) sq += epi_any(m, t0 + wt * TPW + j, acc[mg][j] * rs, acc[mg][j]);
        }
      }
      if (A.ss_out) row_stat(mg, m, sq);
    }
    flush_row_stats();
    stamp(3);
    stamp(4);
    return;
  }

  // ---- this wave's first reduction unit (most waves have exactly one): its epilogue inputs
  // are loaded now, behind the slab stores and the barrier, not after the gather
  const int TU = pair ? CT / 2 : CT;  // tile units
  const int U = TU * MG;
  const int u0 = s + A.S * wid;
  Pre pre0{};
  if (u0 < U) {
    const int tl = pair ? 2 * (u0 / MG) : u0 / MG;
    pre0 = preload(A, row0 + (u0 % MG) * 16 + cl, t0 + tl, 4 * g);
  }

  // ---- publish this wave's partial fragments: slab (gid, s * WK + wk), fragment
  // f = tile_local * MG + mg, 1 KiB each (16 B per lane), write-through into uncached memory
  const int SV = A.S * WK;
  float* gslab = A.ws + (size_t)gid * SV * CT * MG * 256;
  {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(gslab, 0, SV * CT * MG * 1024, 0x00020000);
    const int sv = s * WK + wk;
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int mg = 0; mg < MG; ++mg) {
        const int f = (wt * TPW + j) * MG + mg;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mg][j]), rs,
                                               ((sv * CT * MG + f) * 64 + lane) * 16, 0, 16);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int* ctr = A.counters + 2 * gid;
  group_barrier(ctr, A.S, A.err, A.rel & 1);
  stamp(3);

  // ---- reduce 1/S of the group's fragments and run the epilogue on them
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(gslab, 0, SV * CT * MG * 1024, 0x00020000);
  for (int u = s + A.S * wid; u < U; u += A.S * W) {
    const int tu = u / MG, mg = u % MG;
    const int tl = pair ? 2 * tu : tu;
    const int f = tl * MG + mg;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f}, v2 = f32x4{0.f, 0.f, 0.f, 0.f};
    // every slab's fragment is loaded before the first add (up to 8 at a time, unconditional
    // loads of a clamped index; the surplus is masked out): the uncached round trips overlap
    // instead of running one after the other (a load under a runtime condition, or a loop
    // hipcc does not unroll, made it wait per slab: 2-5 us per launch, tools/stream_stamps.py)
    auto gather = [&](auto two) {
      constexpr bool TWO = decltype(two)::value;
      for (int p0 = 0; p0 < SV; p0 += 8) {
        f32x4 ta[8], tb[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int p = min(p0 + q, SV - 1);
          ta[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, ((p * CT * MG + f) * 64 + lane) * 16, 0, 16));
          if constexpr (TWO)
            tb[q] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, ((p * CT * MG + f + MG) * 64 + lane) * 16, 0, 16));
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float keep = p0 + q < SV ? 1.f : 0.f;
          v += ta[q] * keep;
          if constexpr (TWO) v2 += tb[q] * keep;
        }
      }
    };
    if (pair) gather(std::true_type{});
    else gather(std::false_type{});
    const int m = row0 + mg * 16 + cl;
    float sq = 0.f;
    if (m < A.M) {
      if (u == u0) {
        sq = epi_pre(A, m, t0 + tl, 4 * g, v * pre0.rs, v2 * pre0.rs, pre0);
      } else {
        const float rs = A.ss_in ? rsqrtf(A.ss_in[m] * inv_k + A.eps) : 1.f;
        sq = epi_any(m, t0 + tl, v * rs, v2 * rs);
      }
    }
    if (A.ss_out) row_stat(mg, m, sq);
  }
  flush_row_stats();  // also: every slab read of this workgroup is done
  stamp(4);
  if (threadIdx.x == 0) {  // the last to leave resets the group's counters for the next launch
    const int left = __hip_atomic_fetch_add((gi32*)(ctr + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (left == A.S - 1) {
      __hip_atomic_store((gi32*)ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gi32*)(ctr + 1), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------------
// Instantiated shapes: (TPW, WT, WK) x MG x D. The host picks one per projection shape.
struct Shape {
  int tpw, wt, wk;
};
static const Shape kShapes[] = {
    {1, 4, 1}, {2, 4, 1}, {3, 4, 1}, {4, 4, 1}, {1, 4, 2}, {2, 2, 2}, {3, 2, 2},
    {1, 6, 1}, {2, 6, 1}, {2, 7, 1}, {2, 8, 1}, {1, 8, 1},
};

template <int MG, int TPW, int WT, int WK>
static bool launch_d(const Args& a, int D, int grid, hipStream_t st) {
  switch (D) {
    case 2: hipLaunchKernelGGL((stream_gemm_kernel<MG, TPW, WT, WK, 2>), dim3(grid), dim3(WT * WK * 64), 0, st, a); return true;
    case 4: hipLaunchKernelGGL((stream_gemm_kernel<MG, TPW, WT, WK, 4>), dim3(grid), dim3(WT * WK * 64), 0, st, a); return true;
    case 8: hipLaunchKernelGGL((stream_gemm_kernel<MG, TPW, WT, WK, 8>), dim3(grid), dim3(WT * WK * 64), 0, st, a); return true;
    case 16: hipLaunchKernelGGL((stream_gemm_kernel<MG, TPW, WT, WK, 16>), dim3(grid), dim3(WT * WK * 64), 0, st, a); return true;
    default: return false;
  }
}

template <int MG>
static bool launch_mg(const Args& a, int tpw, int wt, int wk, int D, int grid, hipStream_t st) {
#define PA_SG(T_, W_, K_) \
  if (tpw == T_ && wt == W_ && wk == K_) return launch_d<MG, T_, W_, K_>(a, D, grid, st);
  PA_SG(1, 4, 1) PA_SG(2, 4, 1) PA_SG(3, 4, 1) PA_SG(4, 4, 1) PA_SG(1, 4, 2) PA_SG(2, 2, 2) PA_SG(3, 2, 2)
  PA_SG(1, 6, 1) PA_SG(2, 6, 1) PA_SG(2, 7, 1) PA_SG(2, 8, 1) PA_SG(1, 8, 1)
#undef PA_SG
  return false;
}

// A decomposition: MG (16-row groups per workgroup), RG row groups, (tpw, wt, wk) wave
// shape (CT = tpw * wt tiles per workgroup), S K-slices, D ring depth.
struct Plan {
  int mg, rg, tpw, wt, wk, S, D;
};

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

static bool plan_ok(const Plan& p, int M, int N, int K, int epi) {
  const int tiles = N / 16, KS = K / 32;
  const int CT = p.tpw * p.wt;
  if (p.mg != 2 && p.mg != 4 && p.mg != 8) return false;
  if (p.rg < 1 || 16 * p.mg * p.rg < M || 16 * p.mg * (p.rg - 1) >= M) return false;
  if (tiles % CT) return false;
  if ((epi == EP_SILU || epi == EP_ROPEKV) && CT % 2) return false;
  if (p.S < 1 || KS % p.S) return false;
  const int KC = 2 * p.wk;
  const int ksw = KS / p.S;
  if (ksw % KC) return false;
  const int nch = ksw / KC;
  if (nch < p.D || nch % p.D) return false;
  // the S workgroups of a group wait for each other: the whole grid must be resident at once
  // (at most one workgroup per CU is guaranteed)
  if (p.S > 1 && (tiles / CT) * p.rg * p.S > num_cus()) return false;
  return true;
}

// Default decomposition per shape (starting points from the per-CU intake model in the file
// header; tools/stream_gemm_bench.py on MI355X decides the final table). One row group up to
// 128 rows, two (sharing the weights through one XCD's L2) up to 256; ~256 workgroups.
static Plan plan_default(int M, int N, int K, int epi) {
  Plan p{};
  p.mg = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
  p.rg = (M + 16 * p.mg - 1) / (16 * p.mg);
  const int tiles = N / 16;
  const bool two = p.rg > 1;
  p.wk = 1;
  p.D = 4;
  if (tiles == 1792) {                 // gate_up (interleaved gate / up tiles): 14 tiles
    p.tpw = 2; p.wt = 7; p.S = two ? 1 : 2;
  } else if (K >= 8192) {              // down: 8 tiles x 8 slices (x 4 with two row groups)
    p.tpw = 2; p.wt = 4; p.S = two ? 4 : 8;
  } else if (tiles == 384) {           // qkv: 6 tiles x 4 slices / 12 tiles x 4 slices
    if (two) { p.tpw = 3; p.wt = 4; p.S = 4; }
    else { p.tpw = 3; p.wt = 2; p.wk = 2; p.S = 4; }
  } else if (tiles == 256) {           // o: 4 tiles x 4 slices / 8 tiles x 4 slices
    if (two) { p.tpw = 2; p.wt = 4; p.S = 4; }
    else { p.tpw = 1; p.wt = 4; p.wk = 2; p.S = 4; }
  } else if (tiles % 16 == 0 && tiles >= 4096) {  // LM head: 16 tiles, no K split
    p.tpw = 4; p.wt = 4; p.S = 1;
  } else {
    p.tpw = 1; p.wt = 4; p.S = 1; p.D = 2;
  }
  if (!plan_ok(p, M, N, K, epi)) {  // generic fallback: 4 tiles per workgroup, no K split
    p.tpw = 1; p.wt = 4; p.wk = 1; p.S = 1; p.D = 2;
  }
  return p;
}

}  // namespace sg
}  // namespace pa

extern "C" long long pa_stream_gemm_ws_floats(int M, int N, int K, int mg, int rg, int tpw, int wt, int wk, int S) {
  (void)M; (void)K;
  const long long CT = (long long)tpw * wt, G = N / 16 / CT;
  return G * rg * S * wk * CT * mg * 256;
}

// Fill *plan (7 ints: mg, rg, tpw, wt, wk, S, D) with the default decomposition.
extern "C" void pa_stream_gemm_plan(int M, int N, int K, int epi, int* plan) {
  const pa::sg::Plan p = pa::sg::plan_default(M, N, K, epi);
  plan[0] = p.mg; plan[1] = p.rg; plan[2] = p.tpw; plan[3] = p.wt; plan[4] = p.wk; plan[5] = p.S; plan[6] = p.D;
}

// Returns 1 if the shape / plan is not handled, 0 on success, -2 on a launch error.
// plan: 7 ints (mg, rg, tpw, wt, wk, S, D); any entry <= 0 -> the whole default plan.
extern "C" int pa_stream_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws,
                              long long ws_floats, int* counters, int n_counters, int* err, int M, int N, int K,
                              int ldx, int ldy, int ldr, int epi, const float* ss_in, float* ss_out, float* ss_zero,
                              float eps, const int* plan, void* q_out, void* k_cache, void* v_cache,
                              const int* positions, const int* slots, const float* cos_sin, int H, int KV, int rel,
                              unsigned long long* stamps, hipStream_t st) {
  using namespace pa::sg;
  if (M <= 0) return 0;
  if (M > 256 || K % 64 != 0 || N % 16 != 0 || epi < 0 || epi > 4) return 1;
  if (epi == EP_RESID && !resid) return 1;
  if (ss_out && epi != EP_RESID) return 1;
  if (epi == EP_ROPEKV && (!q_out || !k_cache || !v_cache || !positions || !slots || !cos_sin ||
                           N != (H + 2 * KV) * 128))
    return 1;
  Plan p = plan_default(M, N, K, epi);
  if (plan && plan[0] > 0 && plan[1] > 0 && plan[2] > 0 && plan[3] > 0 && plan[4] > 0 && plan[5] > 0 && plan[6] > 0)
    p = Plan{plan[0], plan[1], plan[2], plan[3], plan[4], plan[5], plan[6]};
  if (!plan_ok(p, M, N, K, epi)) return 1;
  const int CT = p.tpw * p.wt;
  const int G = N / 16 / CT;
  const int groups = G * p.rg;
  if (!ws || !counters || !err || n_counters < 2 * groups) return 1;
  // slabs only off the direct epilogue (a K split, or pair epilogues split over waves)
  const bool direct = p.S * p.wk == 1 && (!(epi == EP_SILU || epi == EP_ROPEKV) || p.tpw % 2 == 0);
  if (!direct && pa_stream_gemm_ws_floats(M, N, K, p.mg, p.rg, p.tpw, p.wt, p.wk, p.S) > ws_floats) return 1;
  const int grid = groups * p.S;
  Args a{(pa::bf16*)y, (const pa::bf16*)x, (const pa::bf16*)wp, (const pa::bf16*)resid, ws, counters, err,
         M, N, K, ldx, ldy, ldr, p.S, p.rg, G, K / 32 / p.S, epi, eps, ss_in, ss_out, ss_zero,
         (pa::bf16*)q_out, (pa::bf16*)k_cache, (pa::bf16*)v_cache, positions, slots, cos_sin, H, KV, rel,
         stamps};
  bool ok = false;
  switch (p.mg) {
    case 2: ok = launch_mg<2>(a, p.tpw, p.wt, p.wk, p.D, grid, st); break;
    case 4: ok = launch_mg<4>(a, p.tpw, p.wt, p.wk, p.D, grid, st); break;
    case 8: ok = launch_mg<8>(a, p.tpw, p.wt, p.wk, p.D, grid, st); break;
    default: ok = false;
  }
  if (!ok) return 1;
  return (int)hipGetLastError() == 0 ? 0 : -2;
}
