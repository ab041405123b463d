// Small-batch projections (16 < M <= 128 tokens) on the packed weights:
// the steps that carry 64 decode rows plus grammar jump-forward runs or a short
// prefill chunk (BASELINE config 3: ~40 % of engine steps sit at 96-256 tokens).
//
//     y[M, N] = epi( x[M, K] · W[N, K]^T )       bf16 in/out, fp32 accumulate
//
// hipBLASLt runs these at 1-2.5 TB/s of weight traffic (tools/prefill_gemm_bench.py:
// o at M = 128 20 us for 33 MB, down 58 us for 117 MB) — too few output tiles for
// 256 CUs. At M <= 256 the weight stream is still the bound, so this kernel is built
// around it:
//
//   * a workgroup owns WAVES * NTW packed column tiles x ALL rows x one K slice;
//     narrow projections are split over K so the grid fills 256 CUs; the split-K
//     partials go to fp32 slabs (write-through sc1 stores) and the last slice to
//     arrive (agent-scope ticket, self-resetting) reduces them — one launch;
//   * x is staged once per workgroup through LDS in FULL 128-B lines (128 k per row
//     per chunk, two chunks in flight, 16-B units XOR-swizzled by row so the
//     16-row A-fragment reads are conflict-free), and shared by all waves — the
//     fragment-shaped direct loads cost twice the load-path work (guide §5) and
//     were the bound of a first version that let every wave fetch its own x;
//   * each wave streams its own NTW weight tiles (fragment-major, 1 KiB contiguous
//     per wave load) straight into registers one chunk ahead, so every weight byte
//     is read from HBM exactly once;
//   * epilogues as the decode kernel: plain, RoPE-permuted QKV columns restored,
//     SwiGLU over interleaved gate/up tiles (in registers with two tiles per wave, or
//     handed from the up wave to the gate wave through LDS with one), residual add.
#include "common.h"

#include <algorithm>

namespace pa {

enum { WG_PLAIN = 0, WG_SILU = 1, WG_RESID = 2, WG_ROPEPERM = 3 };

struct WgArgs {
  bf16* y;
  const bf16* x;
  const bf16* wp;
  const bf16* resid;
  float* ws;      // split-K slabs [groups][S][16*MT][cols per group] fp32
  int* counters;  // [groups], zero between launches
  int M, N, K, ldx, ldy, ldr, S, per;  // per = k-steps per slice (multiple of the chunk's k-steps)
  float eps;                           // NORM: rows scaled by rsqrt(mean(x^2) + eps)
  int acq;                             // hand-off consumer mode (common.h handoff_last)
};

__device__ __forceinline__ int ropeperm_col(int tile, int c) {
  const int p = tile & 7;  // packed position inside a head -> original tile (0,4,1,5,2,6,3,7)
  return (tile >> 3) * 128 + ((p & 1) ? 4 + (p >> 1) : (p >> 1)) * 16 + c;
}

template <int MT, int NTW, int WAVES, int EPI, bool NORM>
__global__ __launch_bounds__(WAVES * 64) void wide_gemm_kernel(const WgArgs A) {
  constexpr int NTH = WAVES * 64;
  constexpr int ROWS = MT * 16;
  // k-steps (32 k) per chunk = per barrier. The per-chunk barrier and x staging set the
  // pace (not LDS bandwidth: profiles/r1_wide_gemm_wavegrid_rejected.jsonl); 4 k-steps (128 k)
  // beat 2 at every M and 8 (profiles/r1_wide_gemm_chunks.jsonl). The register ring holds
  // D * KC = 8 k-steps of weights in flight either way.
  constexpr int KC = 4;
  constexpr int UPR = 4 * KC;                    // 16-B units per row of one x chunk
  constexpr int XU = ROWS * UPR;                 // 16-B units of one x chunk
  constexpr int XPT = (XU + NTH - 1) / NTH;      // units per thread
  constexpr int TPG = WAVES * NTW;               // tiles per column group
  __shared__ __attribute__((aligned(16))) bf16x8 xs[2][ROWS][UPR];  // the only LDS object (guide §5 trap 4a)
  static_assert(sizeof(xs) >= (256 + WAVES / 2 * ROWS * 16) * sizeof(float), "SiLU hand-off must fit the x staging");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int M = A.M, K = A.K, S = A.S;
  const int G = A.N / (16 * TPG);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = bid % 8;
  const int work = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int s = work / G, grp = work % G;
  const int KS = K / 32;
  const int ks0 = min(KS, s * A.per), ks1 = min(KS, ks0 + A.per);
  const int nch = (ks1 - ks0) / KC;  // chunks of KC k-steps (host: K and per multiples of 32 * KC)

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];  // NORM: wave i % WAVES accumulates sum(x^2) of rows 16i + c over its g-units
#pragma unroll
  for (int i = 0; i < MT; ++i) ss[i] = 0.f;

  const int tile0 = grp * TPG + wid * NTW;
  const bf16x8* wsrc[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) wsrc[j] = reinterpret_cast<const bf16x8*>(A.wp + ((size_t)(tile0 + j) * KS) * 512) + lane;

  // x staging: unit u -> (row u>>3, 16-B unit u&7) of a 64-k chunk. Chunk k of x and
  // of W lives in ring slot k % D (registers), D chunks in flight; the LDS image is
  // double-buffered and written one chunk ahead of its use.
  constexpr int D = 8 / KC;
  bf16x8 xring[D][XPT];
  bf16x8 wring[D][KC][NTW];
  auto load_x = [&](int ch, bf16x8 (&dst)[XPT]) {
    const int k0 = (ks0 + KC * ch) * 32;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int u = threadIdx.x + i * NTH;
      if (XU % NTH == 0 || u < XU) {
        const int row = u / UPR, unit = u % UPR;
        const int rsrc = row < M ? row : 0;
        dst[i] = *reinterpret_cast<const bf16x8*>(A.x + (size_t)rsrc * A.ldx + k0 + unit * 8);
      }
    }
  };
  auto store_x = [&](int buf, const bf16x8 (&src)[XPT]) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int u = threadIdx.x + i * NTH;
      if (XU % NTH == 0 || u < XU) {
        const int row = u / UPR, unit = u % UPR;
        xs[buf][row][unit ^ (row & 7)] = src[i];
      }
    }
  };
  // weights: non-temporal (streamed once per step by one wave; as in gemm_decode.hip)
  auto load_w = [&](int ch, bf16x8 (&dst)[KC][NTW]) {
#pragma unroll
    for (int kk = 0; kk < KC; ++kk)
#pragma unroll
      for (int j = 0; j < NTW; ++j) dst[kk][j] = __builtin_nontemporal_load(wsrc[j] + (size_t)(ks0 + KC * ch + kk) * 64);
  };

#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (d < nch) {
      load_x(d, xring[d]);
      load_w(d, wring[d]);
    }
  }
  if (nch > 0) {
    store_x(0, xring[0]);
    if (D < nch) load_x(D, xring[0]);  // slot 0 now waits for chunk D
  }
  __syncthreads();
  for (int cb = 0; cb < nch; cb += D) {
#pragma unroll
    for (int sub = 0; sub < D; ++sub) {
      const int ch = cb + sub;
      if (ch >= nch) break;
      const int buf = ch & 1;
      bf16x8 wcur[KC][NTW];
#pragma unroll
      for (int kk = 0; kk < KC; ++kk)
#pragma unroll
        for (int j = 0; j < NTW; ++j) wcur[kk][j] = wring[sub][kk][j];
      if (ch + D < nch) load_w(ch + D, wring[sub]);
#pragma unroll
      for (int kk = 0; kk < KC; ++kk) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const int row = 16 * i + c;
          const bf16x8 a = xs[buf][row][(4 * kk + g) ^ (row & 7)];
          if constexpr (NORM) {
            if (i % WAVES == wid) {  // row tile i's sum of squares: spread over the waves
#pragma unroll
              for (int e = 0; e < 8; ++e) ss[i] = fmaf((float)a[e], (float)a[e], ss[i]);
            }
          }
#pragma unroll
          for (int j = 0; j < NTW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wcur[kk][j], acc[i][j], 0, 0, 0);
        }
      }
      if (ch + 1 < nch) {
        store_x(buf ^ 1, xring[(sub + 1) % D]);
        if (ch + 1 + D < nch) load_x(ch + 1 + D, xring[(sub + 1) % D]);
      }
      __syncthreads();
    }
  }

  auto out_col = [&](int tile, int cc) -> int {
    if constexpr (EPI == WG_ROPEPERM) return ropeperm_col(tile, cc);
    else return tile * 16 + cc;
  };
  // LDS after the k-loop (x staging is dead): [0] split-K flag, [16, 16 + ROWS) row sum(x^2)
  float* lds_f = reinterpret_cast<float*>(&xs[0][0][0]);
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i % WAVES == wid) {
        float v = ss[i];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        ss[i] = v;
        if (g == 0) lds_f[16 + 16 * i + c] = v;
      }
    }
  }
  const float inv_k = 1.f / (float)K;

  if (S == 1) {
    if constexpr (NORM) __syncthreads();
    auto rsf = [&](int m) -> float {
      if constexpr (NORM) return rsqrtf(lds_f[16 + m] * inv_k + A.eps);
      else return 1.f;
    };
    if constexpr (EPI == WG_SILU && NTW == 1) {
      // one tile per wave: odd waves hold the up tiles of their even neighbours' gate
      // tiles (interleaved packing) and hand them over through LDS (x staging is dead;
      // [256, 256 + WAVES / 2 * ROWS * 16) floats, clear of the flag and row sums)
      float* xch = lds_f + 256 + (wid >> 1) * ROWS * 16;
      if (wid & 1) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) xch[(16 * i + 4 * g + r) * 16 + c] = acc[i][0][r];
      }
      __syncthreads();
      if (wid & 1) return;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * i + 4 * g + r;
          if (m >= M) continue;
          const float rs = rsf(m);
          const float gv = acc[i][0][r] * rs, uv = xch[m * 16 + c] * rs;
          A.y[(size_t)m * A.ldy + (tile0 >> 1) * 16 + c] = (bf16)(gv / (1.f + __expf(-gv)) * uv);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * g + r;
        if (m >= M) continue;
        const float rs = rsf(m);
        if constexpr (EPI == WG_SILU) {
#pragma unroll
          for (int j = 0; j + 1 < NTW; j += 2) {
            const float gv = acc[i][j][r] * rs, uv = acc[i][j + 1][r] * rs;
            const int col = ((tile0 + j) >> 1) * 16 + c;
            A.y[(size_t)m * A.ldy + col] = (bf16)(gv / (1.f + __expf(-gv)) * uv);
          }
        } else {
#pragma unroll
          for (int j = 0; j < NTW; ++j) {
            const int col = out_col(tile0 + j, c);
            float v = acc[i][j][r] * rs;
            if constexpr (EPI == WG_RESID) v += (float)A.resid[(size_t)m * A.ldr + col];
            A.y[(size_t)m * A.ldy + col] = (bf16)v;
          }
        }
      }
    }
    return;
  }

  // ---- split-K: publish this slice's partial tile, the last arriver reduces
  constexpr int GC = TPG * 16;  // columns per group
  float* slab_base = A.ws + (size_t)grp * S * ROWS * GC;
  {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slab_base + (size_t)s * ROWS * GC, 0, ROWS * GC * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * g + r;
#pragma unroll
        for (int j = 0; j < NTW; ++j)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rs,
                                                (m * GC + (wid * NTW + j) * 16 + c) * 4, 0, 16);
      }
  }
  // NORM: this slice's row sums of squares go to their own slab after the tile slabs
  const int Gt = A.N / (16 * TPG);
  float* ss_base = A.ws + (size_t)Gt * S * ROWS * GC + (size_t)grp * S * ROWS;
  if constexpr (NORM) {
    if (g == 0) {
      const __amdgpu_buffer_rsrc_t rq =
          __builtin_amdgcn_make_buffer_rsrc(ss_base + (size_t)s * ROWS, 0, ROWS * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < MT; ++i)
        if (i % WAVES == wid) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ss[i]), rq, (16 * i + c) * 4, 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int* lflag = reinterpret_cast<int*>(lds_f);
  if (!handoff_last(A.counters + grp, S, lflag, A.acq)) return;
  const __amdgpu_buffer_rsrc_t rall =
      __builtin_amdgcn_make_buffer_rsrc(slab_base, 0, S * ROWS * GC * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rqall = __builtin_amdgcn_make_buffer_rsrc(ss_base, 0, S * ROWS * 4, 0x00020000);
  // thread -> (row m, 4 consecutive columns of one tile); SILU: gate tile + its up tile
  constexpr int C4 = GC / 4;
  for (int e = threadIdx.x; e < ROWS * C4; e += NTH) {
    const int m = e / C4, c4 = (e % C4) * 4;
    if (m >= M) continue;
    const int lt = c4 >> 4, cc = c4 & 15;  // local tile within the group
    if constexpr (EPI == WG_SILU) {
      if (lt & 1) continue;
    }
    f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < S; ++p)
      sum += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rall, ((p * ROWS + m) * GC + c4) * 4, 0, 16));
    float rs = 1.f;
    if constexpr (NORM) {
      float t = 0.f;
      for (int p = 0; p < S; ++p) t += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rqall, (p * ROWS + m) * 4, 0, 16));
      rs = rsqrtf(t * inv_k + A.eps);
    }
    sum *= rs;
    const int tile = grp * TPG + lt;
    if constexpr (EPI == WG_SILU) {
      f32x4 up = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < S; ++p)
        up += __builtin_bit_cast(f32x4,
                                 __builtin_amdgcn_raw_buffer_load_b128(rall, ((p * ROWS + m) * GC + c4 + 16) * 4, 0, 16));
      up *= rs;
      const int col0 = (tile >> 1) * 16 + cc;
#pragma unroll
      for (int t = 0; t < 4; ++t) A.y[(size_t)m * A.ldy + col0 + t] = (bf16)(sum[t] / (1.f + __expf(-sum[t])) * up[t]);
    } else {
      const int col0 = out_col(tile, cc);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v = sum[t];
        if constexpr (EPI == WG_RESID) v += (float)A.resid[(size_t)m * A.ldr + col0 + t];
        A.y[(size_t)m * A.ldy + col0 + t] = (bf16)v;
      }
    }
  }
}

template <int MT, int NTW, int WAVES>
static int launch_wg_e(const WgArgs& a, int epi, bool norm, hipStream_t st) {
  const int G = a.N / (16 * WAVES * NTW);
  const dim3 grid(G * a.S), block(WAVES * 64);
#define PA_WG(E, NRM) hipLaunchKernelGGL((wide_gemm_kernel<MT, NTW, WAVES, E, NRM>), grid, block, 0, st, a)
  if (!norm) {
    switch (epi) {
      case WG_PLAIN: PA_WG(WG_PLAIN, false); return 0;
      case WG_RESID: PA_WG(WG_RESID, false); return 0;
      case WG_ROPEPERM: PA_WG(WG_ROPEPERM, false); return 0;
      default:
        PA_WG(WG_SILU, false);
        return 0;
    }
  }
  switch (epi) {
    case WG_PLAIN: PA_WG(WG_PLAIN, true); return 0;
    case WG_ROPEPERM: PA_WG(WG_ROPEPERM, true); return 0;
    case WG_SILU:
      PA_WG(WG_SILU, true);
      return 0;
    default: return 1;
  }
#undef PA_WG
}

template <int MT>
static int launch_wg_mt(const WgArgs& a, int epi, bool norm, int ntw, int waves, hipStream_t st) {
  if (ntw == 1 && waves == 4) return launch_wg_e<MT, 1, 4>(a, epi, norm, st);
  if (ntw == 2 && waves == 4) return launch_wg_e<MT, 2, 4>(a, epi, norm, st);
  if (ntw == 1 && waves == 8) return launch_wg_e<MT, 1, 8>(a, epi, norm, st);
  if (ntw == 2 && waves == 8) return launch_wg_e<MT, 2, 8>(a, epi, norm, st);
  return 1;
}

// Default decomposition: the widest column group that still gives >= 256
// workgroups without split-K, else split K so that groups x slices >= 256.
static void wide_default(int M, int N, int K, int epi, int& ntw, int& waves, int& S) {
  const int tiles = N / 16;
  waves = M > 128 ? 8 : 4;
  // SiLU on one tile per wave too (gate/up pairs meet through LDS): twice the workgroups
  // of the paired form, 1792 / 4 = 448 for gate_up
  ntw = 1;
  if (epi != WG_SILU && M <= 128 && tiles / 8 >= 256 && tiles % 8 == 0) ntw = 2;
  const int G = tiles / (waves * ntw);
  S = G >= 192 ? 1 : std::max(1, (256 + G - 1) / G);
  // down_proj (K = 14,336) at M <= 32: 512 workgroups (8 K-slices) beat 256 with the
  // non-temporal weight stream, 25.8 vs 28.0 us at M = 24 (profiles/r2_nt_weights_ab.jsonl
  // sweep); at M = 48 the two tie.
  if (K >= 8192 && M <= 32) S = std::max(S, (512 + G - 1) / G);
  S = std::min(S, std::max(1, K / 64 / 8));  // keep >= 8 chunks per slice
}

}  // namespace pa

extern "C" int pa_wide_gemm_plan(int M, int N, int K, int epi, int* ntw, int* waves, int* S) {
  pa::wide_default(M, N, K, epi, *ntw, *waves, *S);
  return 0;
}

// Returns 1 if the shape/config is not handled, 0 on success, -2 on a launch error.
// ntw/waves/splits <= 0 pick the defaults.
extern "C" int pa_wide_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws,
                            long long ws_floats, int* counters, int n_counters, int M, int N, int K, int ldx,
                            int ldy, int ldr, int epi, int norm, float eps, int ntw, int waves, int splits,
                            hipStream_t st) {
  using namespace pa;
  if (M <= 0) return 0;
  if (M > 128 || K % 64 != 0 || N % 16 != 0 || epi < 0 || epi > 3) return 1;
  if (epi == WG_RESID && (!resid || norm)) return 1;
  int dn, dw, dS;
  wide_default(M, N, K, epi, dn, dw, dS);
  if (ntw <= 0) ntw = dn;
  if (waves <= 0) waves = dw;
  int S = splits > 0 ? splits : dS;
  if (epi == WG_SILU && (waves * ntw) % 2) return 1;  // gate/up tile pairs within a group
  const int TPG = waves * ntw;
  if ((N / 16) % TPG) return 1;
  const int G = N / 16 / TPG;
  const int MT = (M + 15) / 16;
  const int MTp = MT <= 2 ? 2 : (MT <= 4 ? 4 : 8);
  const int KC = 4;  // k-steps per chunk (kernel constexpr)
  if ((K / 32) % KC) return 1;
  auto ws_need = [&](int s_) { return (long long)G * s_ * MTp * 16 * (TPG * 16 + 1); };
  const int KS = K / 32;
  S = std::max(1, std::min(S, KS / KC));
  int per = (KS + S - 1) / S;
  per = (per + KC - 1) / KC * KC;
  S = (KS + per - 1) / per;  // no empty slices
  if (S > 1 && splits <= 0) {  // default split: shrink to the workspace
    while (S > 1 && ws_need(S) > ws_floats) {
      --S;
      per = ((KS + S - 1) / S + KC - 1) / KC * KC;
      S = (KS + per - 1) / per;
    }
  }
  if (S > 1) {
    if (!ws || !counters || n_counters < G) return 1;
    if (ws_need(S) > ws_floats) return 1;
  }
  WgArgs a{(bf16*)y, (const bf16*)x, (const bf16*)wp, (const bf16*)resid, ws, counters, M, N, K, ldx, ldy, ldr,
           S, per, eps, g_handoff_acquire};
  int rc;
  switch (MTp) {
    case 2: rc = launch_wg_mt<2>(a, epi, norm != 0, ntw, waves, st); break;
    case 4: rc = launch_wg_mt<4>(a, epi, norm != 0, ntw, waves, st); break;
    default: rc = launch_wg_mt<8>(a, epi, norm != 0, ntw, waves, st); break;
  }
  if (rc) return rc;
  return (int)hipGetLastError() == 0 ? 0 : -2;
}
