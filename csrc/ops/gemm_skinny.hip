// Weight-streaming "skinny" GEMM for decode-shaped projections:
//
//     y[M, N] = x[M, K] · W[N, K]^T      bf16 in/out, fp32 accumulate, M <= 128
//
// At decode batch sizes every projection is HBM-bound on W (QKV 50 MB, gate_up
// 235 MB, down 117 MB, O 33 MB, LM head 1 GB for Llama-3-8B), so the kernel is
// built to stream W exactly once at full rate:
//   * one workgroup = 8 waves owns a tile of 16*NT output columns and ALL M rows;
//     the 8 waves split K into contiguous slices, so every W byte is read by
//     exactly one lane and there is no cross-workgroup reduction;
//   * W goes straight from HBM into the B operand of v_mfma_f32_16x16x32_bf16
//     (lane l loads 16 contiguous bytes of row n0 + (l & 15)), no LDS staging —
//     the guide's "GEMV / M <= 16" rule, extended to M <= 128 by reusing each W
//     fragment across MT = M/16 MFMAs;
//   * x (<= 1 MB) stays L2-resident and feeds the A operand;
//   * the 8 per-wave partial tiles are summed through LDS and written as bf16;
//   * grid = N / (16*NT) workgroups, remapped so consecutive column tiles land
//     on one XCD (bijective remap, guide §5 T1) — all share x in that XCD's L2.
#include "common.h"

namespace pa {

template <int MT, int NT, int UNROLL, bool NTL>
__global__ __launch_bounds__(512) void skinny_gemm_kernel(bf16* __restrict__ y,
                                                          const bf16* __restrict__ x,
                                                          const bf16* __restrict__ w, int M, int N,
                                                          int K, int ldy) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);  // [8][MT*16][NT*16]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  // XCD-aware bijective remap of the column tile index
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = bid % 8;
  const int tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int n0 = tile * 16 * NT;
  // K slice of this wave (multiple of 32)
  const int ksteps_total = K / 32;
  const int per = (ksteps_total + 7) / 8;
  const int ks0 = wid * per;
  const int ks1 = min(ksteps_total, ks0 + per);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* wrow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wrow[j] = w + (size_t)(n0 + 16 * j + c) * K + 8 * g;
  const bf16* xrow[MT];
  bool mval[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = 16 * i + c;
    mval[i] = m < M;
    xrow[i] = x + (size_t)(mval[i] ? m : 0) * K + 8 * g;
  }

  int ks = ks0;
  for (; ks + UNROLL <= ks1; ks += UNROLL) {
    bf16x8 bw[UNROLL][NT];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bw[u][j] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wrow[j] + 32 * (ks + u)))
                       : *reinterpret_cast<const bf16x8*>(wrow[j] + 32 * (ks + u));
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        bf16x8 a = *reinterpret_cast<const bf16x8*>(xrow[i] + 32 * (ks + u));
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[u][j], acc[i][j], 0, 0, 0);
      }
    }
  }
  for (; ks < ks1; ++ks) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(wrow[j] + 32 * ks);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(xrow[i] + 32 * ks);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i][j], 0, 0, 0);
      }
    }
  }
  // C layout: lane (g, c): rows 4g + r (m), column c (n) of each 16x16 tile
  constexpr int TM = MT * 16, TN = NT * 16;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wid * TM + 16 * i + 4 * g + r) * TN + 16 * j + c] = acc[i][j][r];
  __syncthreads();
  for (int e = threadIdx.x; e < TM * TN; e += 512) {
    const int m = e / TN, n = e % TN;
    if (m >= M) continue;
    float s = 0.f;
#pragma unroll
    for (int wv = 0; wv < 8; ++wv) s += red[(wv * TM + m) * TN + n];
    y[(size_t)m * ldy + n0 + n] = (bf16)s;
  }
}

template <int MT, int NT, int UNROLL, bool NTL>
static void launch_skinny_v(bf16* y, const bf16* x, const bf16* w, int M, int N, int K, int ldy,
                            hipStream_t st) {
  const size_t lds = (size_t)8 * MT * 16 * NT * 16 * sizeof(float);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)skinny_gemm_kernel<MT, NT, UNROLL, NTL>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, UNROLL, NTL>), dim3(N / (16 * NT)), dim3(512), lds, st, y,
                     x, w, M, N, K, ldy);
}

// variant (benchmarking knob): 0 = default (temporal loads), 1 = deep unroll,
// 2 = nontemporal loads, 3 = deep + nontemporal. Cache-cold measurements on
// MI355X (profiles/r1_skinny_gemm_cold.md): temporal loads win by 5-15%.
static int g_variant = 0;

template <int MT, int NT>
static void launch_skinny(bf16* y, const bf16* x, const bf16* w, int M, int N, int K, int ldy,
                          hipStream_t st) {
  constexpr int U = MT <= 2 ? 8 : (MT <= 4 ? 4 : 2);
  constexpr int UD = MT <= 2 ? 16 : (MT <= 4 ? 8 : 4);
  switch (g_variant) {
    case 1: launch_skinny_v<MT, NT, UD, false>(y, x, w, M, N, K, ldy, st); break;
    case 2: launch_skinny_v<MT, NT, U, true>(y, x, w, M, N, K, ldy, st); break;
    case 3: launch_skinny_v<MT, NT, UD, true>(y, x, w, M, N, K, ldy, st); break;
    default: launch_skinny_v<MT, NT, U, false>(y, x, w, M, N, K, ldy, st); break;
  }
}

}  // namespace pa

extern "C" void pa_skinny_set_variant(int v) { pa::g_variant = v; }

// Returns 1 if the shape is not handled (caller falls back to the library GEMM).
extern "C" int pa_skinny_gemm(void* y, const void* x, const void* w, int M, int N, int K, int ldy,
                              hipStream_t st) {
  using namespace pa;
  if (M <= 0) return 0;
  if (M > 128 || K % 256 != 0 || N % 16 != 0) return 1;
  bf16* Y = (bf16*)y;
  const bf16* X = (const bf16*)x;
  const bf16* W = (const bf16*)w;
  const int MT = (M + 15) / 16;
  // wider column tiles only when there are still >= 512 workgroups to fill 256 CUs
  const bool wide = N % 32 == 0 && N / 32 >= 512 && MT <= 4;
#define PA_SK(mt)                                                     \
  if (wide) launch_skinny<mt, 2>(Y, X, W, M, N, K, ldy, st);          \
  else launch_skinny<mt, 1>(Y, X, W, M, N, K, ldy, st);
  switch (MT) {
    case 1: PA_SK(1) break;
    case 2: PA_SK(2) break;
    case 3: PA_SK(3) break;
    case 4: PA_SK(4) break;
    case 5: launch_skinny<5, 1>(Y, X, W, M, N, K, ldy, st); break;
    case 6: launch_skinny<6, 1>(Y, X, W, M, N, K, ldy, st); break;
    case 7: launch_skinny<7, 1>(Y, X, W, M, N, K, ldy, st); break;
    default: launch_skinny<8, 1>(Y, X, W, M, N, K, ldy, st); break;
  }
#undef PA_SK
  return (int)hipGetLastError() == 0 ? 0 : -2;
}
