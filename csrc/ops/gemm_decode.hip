// Decode-step projections on pre-packed weights (fused):
//
//     y[M, N] = epi( r[m] * x[M, K] · W[N, K]^T )        bf16 in/out, fp32 accumulate, M <= 64
//
// At decode batch sizes every projection is bound by streaming W from HBM once
// (Llama-3-8B: 14 GB of layer weights per step), so this kernel is organised
// around the W stream and fuses the small per-layer kernels that would
// otherwise each cost a launch + a few microseconds at M <= 16:
//
//   * W is stored "fragment-major" (packed once at model load, pa_decode_pack):
//     Wp[N/16][K/32][64 lanes][8] with lane l = 16*g + c holding
//     W[16t + c][32s + 8g .. 8g+7] — exactly the B operand of
//     v_mfma_f32_16x16x32_bf16. One wave load is 1 KiB of CONTIGUOUS memory
//     (8 full 128-B lines) instead of 16 rows x 64 B (16 half lines), which
//     halves the texture-path work per streamed byte (guide §5: fragment-shaped
//     loads cost 2x TA at identical HBM traffic);
//   * a workgroup owns NT column tiles (16*NT outputs) and ALL rows; its WAVES
//     waves split K, each streaming a contiguous run of its tiles' fragments;
//     x (<= 512 KB, L2-resident) feeds the A operand and is re-used across the
//     NT tiles; per-wave partials are summed through LDS;
//   * NORM: RMSNorm folded in — the norm weight is pre-multiplied into W's
//     columns at load time, the kernel accumulates sum(x^2) from the same x
//     fragments it feeds to the MFMAs and scales each output row by
//     rsqrt(mean + eps) (no separate norm kernel, no normalised-x round trip);
//   * EPI_SILU: gate/up tiles are interleaved in the packed layout, so the
//     workgroup holds gate and up for the same 16 outputs and writes
//     silu(gate) * up directly (no [M, 2F] intermediate, no SwiGLU kernel);
//   * EPI_RESID: y = resid + acc (in place on the residual stream).
//   * grid = N / (16*NT) workgroups, XCD-aware bijective remap so consecutive
//     column groups share one XCD's L2 copy of x.
//
// Replaces the norm -> GEMM -> SwiGLU -> GEMM -> add chain of the reference
// model path (models/llama.py forward) for decode-sized steps.
#include "common.h"

#include <algorithm>

namespace pa {

enum { EPI_PLAIN = 0, EPI_SILU = 1, EPI_RESID = 2, EPI_ROPE = 3 };

// EPI_ROPE: the QKV projection with RoPE + paged KV write in its epilogue
// (replaces rope_cache.hip on decode steps). The packed QKV columns are permuted
// per 128-wide head to tile order [0,4,1,5,2,6,3,7], so a workgroup of NT = 2
// tiles holds rotary dims i and i + 64 of one head for 16 consecutive i.
struct RopeArgs {
  bf16* q_out;           // [M, H, 128]
  bf16* k_cache;         // [NB, KV, 16, 16, 8]  fragment-major pages (rope_cache.hip)
  bf16* v_cache;         // [NB, KV, 128, 16]
  const int* positions;  // [M]
  const int* slots;      // [M], < 0 = no cache write
  const float* cos_sin;  // [max_pos, 128] (cos | sin)
  int H, KV;
};

struct DgArgs {
  bf16* y;
  const bf16* x;
  const bf16* wp;
  const bf16* resid;
  int M, N, K, ldx, ldy, ldr;
  float eps;
  RopeArgs rope;
  int S;          // K slices (split-K across workgroups; 1 = none)
  float* ws;      // split-K slabs [groups][S][TM*TN + TM] fp32
  int* counters;  // [groups] arrival tickets, zero between launches
  int acq;        // hand-off consumer mode (common.h handoff_last)
};

template <int MT, int NT, int WAVES, int U, int EPI, bool NORM, bool NTW>
__global__ __launch_bounds__(WAVES * 64) void decode_gemm_kernel(const DgArgs A) {
  bf16* __restrict__ y = A.y;
  const bf16* __restrict__ x = A.x;
  const bf16* __restrict__ wp = A.wp;
  const bf16* resid = A.resid;
  const int M = A.M, K = A.K, ldx = A.ldx, ldy = A.ldy, ldr = A.ldr;
  const float eps = A.eps;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TM = MT * 16, TN = NT * 16;
  float* red = reinterpret_cast<float*>(smem);  // [WAVES][TM][TN]
  float* ssq = red + WAVES * TM * TN;            // [WAVES][TM]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int N = A.N;
  (void)N;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = bid % 8;
  const int work = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int S = A.S, G = nwg / S;
  const int sl = work / G, grp = work % G;  // slice-major: workgroups sharing a K slice of x share an XCD
  const int tile0 = grp * NT;

  const int KS = K / 32;
  const int perS = (KS + S - 1) / S;
  const int kb0 = min(KS, sl * perS), kb1 = min(KS, kb0 + perS);
  const int per = (kb1 - kb0 + WAVES - 1) / WAVES;
  const int ks0 = min(kb1, kb0 + wid * per);
  const int ks1 = min(kb1, ks0 + per);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ss[i] = 0.f;

  // NTW: the weight stream (read once per step, by one wave) is loaded non-temporal
  auto ldw = [](const bf16x8* p) -> bf16x8 {
    if constexpr (NTW) return __builtin_nontemporal_load(p);
    else return *p;
  };
  const bf16x8* wt[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    wt[j] = reinterpret_cast<const bf16x8*>(wp + ((size_t)(tile0 + j) * KS) * 512) + lane;
  const bf16* xr[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = 16 * i + c;
    xr[i] = x + (size_t)(m < M ? m : 0) * ldx + 8 * g;
  }

  auto step = [&](const bf16x8 (&bw)[NT], const bf16x8 (&ax)[MT]) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const bf16x8 a = ax[i];
      if constexpr (NORM) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (float)a[e];
          ss[i] = fmaf(v, v, ss[i]);
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[j], acc[i][j], 0, 0, 0);
    }
  };

  // Every load of a round (U chunks of W from HBM and the matching x fragments from L2)
  // is issued before the first MFMA: left to itself the scheduler interleaved them with
  // the MFMAs and kept only 2-5 loads in flight per wave, so each round paid several
  // dependent L2 round trips for x (down_proj at M=8 streamed 4.6 TB/s). Loads are
  // ordered chunk by chunk, so chunk u waits only for its own operands.
  auto load_x = [&](bf16x8 (&ax)[MT], int k) {
#pragma unroll
    for (int i = 0; i < MT; ++i) ax[i] = *reinterpret_cast<const bf16x8*>(xr[i] + 32 * k);
  };
  // (sub-batches of UB chunks where a whole round would not fit the wave's registers:
  // 16-wave workgroups leave 128 VGPRs per wave)
  constexpr int LOAD_REGS = WAVES >= 16 ? 80 : 192;
  constexpr int UB0 = LOAD_REGS / (4 * (NT + MT));
  constexpr int UB = UB0 >= U ? U : (UB0 < 1 ? 1 : UB0);
  int ks = ks0;
  for (; ks + U <= ks1; ks += U) {
#pragma unroll
    for (int u0 = 0; u0 < U; u0 += UB) {
      bf16x8 bw[UB][NT], ax[UB][MT];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        if (u0 + u < U) {
#pragma unroll
          for (int j = 0; j < NT; ++j) bw[u][j] = ldw(wt[j] + (size_t)(ks + u0 + u) * 64);
          load_x(ax[u], ks + u0 + u);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < UB; ++u)
        if (u0 + u < U) step(bw[u], ax[u]);
    }
  }
  for (; ks < ks1; ++ks) {
    bf16x8 bw[NT], ax[MT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bw[j] = ldw(wt[j] + (size_t)ks * 64);
    load_x(ax, ks);
    step(bw, ax);
  }

  // C layout of a 16x16 tile: lane (g, c) holds rows 4g + r, column c.
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wid * TM + 16 * i + 4 * g + r) * TN + 16 * j + c] = acc[i][j][r];
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) ssq[wid * TM + 16 * i + c] = v;
    }
  }
  __syncthreads();
  // workgroup sum over waves -> fin [TM][TN], fss [TM] (row sums of squares)
  float* fin = ssq + WAVES * TM;
  float* fss = fin + TM * TN;
  int* lflag = reinterpret_cast<int*>(fss + TM);
  for (int e = threadIdx.x; e < TM * TN; e += WAVES * 64) {
    float t = 0.f;
#pragma unroll
    for (int wv = 0; wv < WAVES; ++wv) t += red[wv * TM * TN + e];
    fin[e] = t;
  }
  if constexpr (NORM) {
    for (int m = threadIdx.x; m < TM; m += WAVES * 64) {
      float t = 0.f;
#pragma unroll
      for (int wv = 0; wv < WAVES; ++wv) t += ssq[wv * TM + m];
      fss[m] = t;
    }
  }
  __syncthreads();
  if (S > 1) {
    // split-K hand-off (common.h handoff_last): publish the slice's partial tile
    // write-through, take a ticket; the last slice acquires at agent scope and reduces.
    // Slabs padded to 64 floats: each wave's b32 store instruction writes two whole 128-B lines.
    constexpr int SLAB = (TM * TN + TM + 63) / 64 * 64;
    float* gslab = A.ws + (size_t)grp * S * SLAB;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(gslab + (size_t)sl * SLAB, 0, SLAB * 4, 0x00020000);
    for (int e = threadIdx.x; e < SLAB; e += WAVES * 64)
      __builtin_amdgcn_raw_buffer_store_b32(
          __float_as_uint(e < TM * TN ? fin[e] : (e < TM * TN + TM ? fss[e - TM * TN] : 0.f)), rs, e * 4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(A.counters + grp, S, lflag, A.acq)) return;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(gslab, 0, S * SLAB * 4, 0x00020000);
    for (int e = threadIdx.x; e < TM * TN + TM; e += WAVES * 64) {  // (padding not read)
      float t = 0.f;
      for (int p = 0; p < S; ++p) t += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, (p * SLAB + e) * 4, 0, 16));
      if (e < TM * TN) fin[e] = t;
      else fss[e - TM * TN] = t;
    }
    __syncthreads();
  }
  if constexpr (EPI == EPI_ROPE) {
    static_assert(NT == 2, "EPI_ROPE pairs the two tiles of a workgroup");
    const RopeArgs& R = A.rope;
    const int hh = tile0 >> 3, i0 = 16 * ((tile0 & 7) >> 1);
    for (int e = threadIdx.x; e < TM * 16; e += WAVES * 64) {
      const int m = e >> 4, cc = e & 15;
      if (m >= M) continue;
      float rs = 1.f;
      if constexpr (NORM) rs = rsqrtf(fss[m] / (float)K + eps);
      const float a = fin[m * TN + cc] * rs, b = fin[m * TN + 16 + cc] * rs;
      const int i = i0 + cc;
      float o1 = a, o2 = b;
      if (hh < R.H + R.KV) {
        const float* cs = R.cos_sin + (size_t)R.positions[m] * 128;
        const float c = cs[i], sn = cs[64 + i];
        o1 = a * c - b * sn;
        o2 = b * c + a * sn;
      }
      if (hh < R.H) {
        bf16* dst = R.q_out + ((size_t)m * R.H + hh) * 128;
        dst[i] = (bf16)o1;
        dst[i + 64] = (bf16)o2;
      } else {
        const int slot = R.slots[m];
        if (slot >= 0) {
          const int blk = slot >> 4, off = slot & 15;
          if (hh < R.H + R.KV) {
            bf16* page = R.k_cache + ((size_t)blk * R.KV + (hh - R.H)) * 128 * 16;
            page[((size_t)(i >> 3) * 16 + off) * 8 + (i & 7)] = (bf16)o1;
            page[((size_t)((i + 64) >> 3) * 16 + off) * 8 + (i & 7)] = (bf16)o2;
          } else {
            bf16* page = R.v_cache + ((size_t)blk * R.KV + (hh - R.H - R.KV)) * 128 * 16 + off;
            page[(size_t)i * 16] = (bf16)o1;
            page[(size_t)(i + 64) * 16] = (bf16)o2;
          }
        }
      }
    }
    return;
  }
  constexpr int TNO = EPI == EPI_SILU ? TN / 2 : TN;
  const int n0 = (EPI == EPI_SILU ? tile0 / 2 : tile0) * 16;
  const float inv_k = 1.f / (float)K;
  for (int e = threadIdx.x; e < TM * TNO; e += WAVES * 64) {
    const int m = e / TNO, n = e % TNO;
    if (m >= M) continue;
    float rs = 1.f;
    if constexpr (NORM) rs = rsqrtf(fss[m] * inv_k + eps);
    if constexpr (EPI == EPI_SILU) {
      const int p = n >> 4, cc = n & 15;
      const float gs = fin[m * TN + 32 * p + cc] * rs, us = fin[m * TN + 32 * p + 16 + cc] * rs;
      y[(size_t)m * ldy + n0 + n] = (bf16)(gs / (1.f + __expf(-gs)) * us);
    } else {
      float s = fin[m * TN + n] * rs;
      if constexpr (EPI == EPI_RESID) s += (float)resid[(size_t)m * ldr + n0 + n];
      y[(size_t)m * ldy + n0 + n] = (bf16)s;
    }
  }
}

// bit 0: non-temporal weight loads (default on: the weight stream is read once per step by one
// wave, so it should not displace x and the KV cache in L2 / MALL; 5-9 % faster on every
// projection at M = 8-32, 8-token decode steps 3.49 -> 3.33 ms: profiles/r2_decode_nt_ab.jsonl)
static int g_dg_variant = 1;

// protocol of the in-launch hand-offs, common.h handoff_last (tools/splitk_check.py: fresh
// inputs, NaN-poisoned slabs and outputs; tools/handoff_cost.py; profiles/r3_splitk_handoff.md):
//   GEMM split-K slabs (decode / wide / mid / prefill): 2 = producer agent release + last-arriver
//     agent acquire. Decode qkv_rope at M = 9 with 3 K-slices mismatched in 46 of 3,000 runs
//     with the round-2 sc1-only form (mode 0) and in 4 of 10,000 with the acquire alone
//     (mode 1); none with mode 2 (+2-3 us per split launch). Round 4: with the slabs in
//     uncached memory (ops.empty_handoff) mode 1 still mismatched 5 of 10,000 (finite values),
//     so the cause is not a stale L2 copy of the slab; mode 2 stays
//     (profiles/r4_handoff_uncached.md).
//   attention partition merge: 1 = last-arriver agent acquire on uncached partials: 0 bad runs
//     in 10,000 poisoned repetitions for each of ten 256/512-key, 4/8-wave cases (round 4); the
//     release costs +77 us at 64 rows x 1,000 keys there (it writes back every dirty L2 line of
//     the XCD, and this launch leaves many).
int g_handoff_acquire = 2;
int g_handoff_attn = 1;

template <int MT, int NT, int WAVES, int EPI, bool NORM>
static int launch_dg(const DgArgs& a, hipStream_t st) {
  constexpr int U = MT == 1 ? 8 : (MT == 2 ? 4 : 2);  // chunks per round (16 per round for 8-wave groups was slower)
  const size_t lds = ((size_t)(WAVES + 1) * MT * 16 * (NT * 16 + 1) + 16) * sizeof(float);
  auto kern = g_dg_variant & 1 ? decode_gemm_kernel<MT, NT, WAVES, U, EPI, NORM, true>
                                : decode_gemm_kernel<MT, NT, WAVES, U, EPI, NORM, false>;
  static bool attr[2] = {false, false};
  if (!attr[g_dg_variant & 1]) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr[g_dg_variant & 1] = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.N / (16 * NT) * a.S), dim3(WAVES * 64), lds, st, a);
  return 0;
}

template <int MT, int EPI, bool NORM>
static int pick_nw(int nt, int waves, const DgArgs& a, hipStream_t st) {
#define PA_DG(NT_, W_) \
  if (nt == NT_ && waves == W_) return launch_dg<MT, NT_, W_, EPI, NORM>(a, st);
  if constexpr (EPI == EPI_ROPE) {
    PA_DG(2, 4) PA_DG(2, 8) PA_DG(2, 16)
    return 1;
  } else {
    if constexpr (EPI != EPI_SILU) {
      PA_DG(1, 8) PA_DG(1, 16)
    }
    PA_DG(2, 4) PA_DG(2, 8) PA_DG(2, 16)
    if constexpr (MT <= 2) {
      PA_DG(4, 4) PA_DG(4, 8) PA_DG(4, 16)
    } else {
      PA_DG(4, 8)
    }
  }
#undef PA_DG
  return 1;
}

// Default (tile width, waves, K slices) per shape, from tools/decode_gemm_bench.py on
// MI355X (profiles/r1_decode_gemm.md, r1_decode_gemm_splitk.jsonl): 2 column tiles per
// workgroup once there are >= 384 tiles (x fragments re-used across both), 4 for wide
// matrices at M > 8 (the x stream grows with M); K split over 16 waves when a
// workgroup is alone on its CU. Split-K across workgroups is available (splits > 0)
// but off by default: it won only on down in isolation and lost inside the engine.
static void default_cfg(int MT, int M, int N, int K, int epi, int& nt, int& waves, int& S) {
  const int tiles = N / 16;
  if (epi == EPI_ROPE) nt = 2;
  else if (epi == EPI_SILU) nt = (M > 8 && tiles % 4 == 0) ? 4 : 2;
  else if (MT >= 2 && tiles >= 1792 && tiles % 4 == 0) nt = 4;
  else nt = (tiles >= 384 && tiles % 2 == 0) ? 2 : 1;
  waves = (tiles / nt <= 256 && M <= 8) ? 16 : 8;
  S = 1;
  (void)K;  // split-K (S > 1) measured no faster inside the engine: r1_decode_gemm.md
}

static int dispatch(DgArgs a, int epi, int norm, int nt, int waves, int splits, long long ws_floats,
                    int n_counters, hipStream_t st) {
  const int M = a.M, N = a.N;
  if (M <= 0) return 0;
  if (M > 64 || a.K % 32 != 0 || N % 16 != 0 || epi < 0 || epi > 3) return 1;
  if ((epi == EPI_SILU || epi == EPI_ROPE) && (N / 16) % 2) return 1;
  if (epi == EPI_RESID && !a.resid) return 1;
  const int MT = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  int dn, dw, dS;
  default_cfg(MT, M, N, a.K, epi, dn, dw, dS);
  if (nt <= 0) nt = dn;
  if (waves <= 0) waves = dw;
  int S = splits > 0 ? splits : dS;
  if ((N / 16) % nt) return 1;
  S = std::max(1, std::min(S, a.K / 32));
  const int G = N / 16 / nt;
  if (S > 1) {
    const long long slab = ((long long)MT * 16 * (nt * 16 + 1) + 63) / 64 * 64;  // kernel's padded SLAB
    if (!a.ws || !a.counters || n_counters < G || (long long)G * S * slab > ws_floats) {
      if (splits > 0) return 1;
      S = 1;  // default split without a workspace: run unsplit
    }
  }
  a.S = S;
  a.acq = g_handoff_acquire;
  int rc = 1;
#define PA_DGE(MT_)                                                                 \
  switch (epi * 2 + (norm ? 1 : 0)) {                                               \
    case 0: rc = pick_nw<MT_, EPI_PLAIN, false>(nt, waves, a, st); break;           \
    case 1: rc = pick_nw<MT_, EPI_PLAIN, true>(nt, waves, a, st); break;            \
    case 3: rc = pick_nw<MT_, EPI_SILU, true>(nt, waves, a, st); break;             \
    case 4: rc = pick_nw<MT_, EPI_RESID, false>(nt, waves, a, st); break;           \
    case 7: rc = pick_nw<MT_, EPI_ROPE, true>(nt, waves, a, st); break;             \
    default: rc = 1;                                                                \
  }
  switch (MT) {
    case 1: PA_DGE(1) break;
    case 2: PA_DGE(2) break;
    default: PA_DGE(4) break;
  }
#undef PA_DGE
  if (rc != 0) return rc;
  return (int)hipGetLastError() == 0 ? 0 : -2;
}

}  // namespace pa

// Returns 1 if the shape/config is not handled, 0 on success, -2 on a launch error.
// epi: 0 plain, 1 silu(gate)*up over interleaved tile pairs, 2 residual add.
// nt/waves/splits <= 0 pick the defaults; ws/counters: split-K slabs and zeroed tickets.
extern "C" void pa_decode_set_variant(int v) { pa::g_dg_variant = v; }
extern "C" void pa_handoff_set_acquire(int v) { pa::g_handoff_acquire = pa::g_handoff_attn = v; }
extern "C" void pa_handoff_set_modes(int gemm, int attn) {
  pa::g_handoff_acquire = gemm;
  pa::g_handoff_attn = attn;
}

extern "C" int pa_decode_gemm(void* y, const void* x, const void* wp, const void* resid, int M, int N, int K,
                              int ldx, int ldy, int ldr, int epi, int norm, float eps, int nt, int waves,
                              int splits, float* ws, long long ws_floats, int* counters, int n_counters,
                              hipStream_t st) {
  using namespace pa;
  if (epi == EPI_ROPE) return 1;
  DgArgs a{(bf16*)y, (const bf16*)x, (const bf16*)wp, (const bf16*)resid, M, N, K, ldx, ldy, ldr, eps, RopeArgs{},
           1, ws, counters};
  return dispatch(a, epi, norm, nt, waves, splits, ws_floats, n_counters, st);
}

// QKV projection (RMSNorm folded, rope-permuted packed weights) + RoPE + paged KV
// write: q -> q_out [M, H, 128], k/v -> the layer's cache pages at slots[m].
extern "C" int pa_decode_qkv_rope(const void* x, const void* wp, int M, int N, int K, int ldx, float eps,
                                  void* q_out, void* k_cache, void* v_cache, const int* positions,
                                  const int* slots, const float* cos_sin, int H, int KV, int nt, int waves,
                                  int splits, float* ws, long long ws_floats, int* counters, int n_counters,
                                  hipStream_t st) {
  using namespace pa;
  if (N != (H + 2 * KV) * 128) return 1;
  DgArgs a{nullptr, (const bf16*)x, (const bf16*)wp, nullptr, M, N, K, ldx, 0, 0, eps,
           RopeArgs{(bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, positions, slots, cos_sin, H, KV},
           1, ws, counters};
  return dispatch(a, EPI_ROPE, 1, nt, waves, splits, ws_floats, n_counters, st);
}
