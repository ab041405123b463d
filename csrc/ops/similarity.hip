// HBM-resident semantic index: fused filter + cosine similarity + top-k
// (backs EnhancedMemory.semantic_search,
// reference pilott/memory/enhanced_memory.py:93-131).
//
// index   [N, D] bf16, rows L2-normalised on insert (so cosine == dot)
// queries [Q, D] bf16, L2-normalised
// per-row filter metadata: priority (int32), tag bitmask (uint64), expiry (f32
// seconds, 0 = never); per-query: min priority, required tag bitmask.
// A row qualifies for query q iff prio >= minp[q] && (tags & qtags[q]) == qtags[q]
// && (expiry == 0 || expiry > now) — the reference's candidate-index semantics
// (priority index range, tag-set intersection, is_expired) evaluated in-kernel.
//
// Stage 1 (grid = row-slices x query-tiles of 16): each wave multiplies 16 index
// rows by the 16-query tile with v_mfma_f32_16x16x32_bf16 (rows stream from HBM
// straight into the A operand, the query tile sits in LDS as the B operand), so
// a [Q<=16, 1024] x [1024, N] scan is one pass over the index at HBM rate.
// Scores above the per-query running threshold are appended to an LDS candidate
// buffer; when a buffer nears capacity the workgroup sorts it (bitonic) and
// raises the threshold to the current k-th best. Each slice writes its top-k.
// Stage 2 (one WG per query) merges the slices' top-k lists the same way.
#include "common.h"

namespace pa {

constexpr int SIM_CAND = 256;     // candidate buffer per query (power of two)
constexpr int SIM_MAXK = 64;
constexpr int SIM_QT = 16;        // queries per tile (MFMA N)
constexpr int SIM_MAXD = 1024;    // LDS query tile capacity (bf16)
constexpr int SIM_MIN_ROWS_PER_WG = 1024;
constexpr int SIM_MAX_WG = 1024;

__device__ __forceinline__ int sim_num_wg(int N) {
  int nwg = (N + SIM_MIN_ROWS_PER_WG - 1) / SIM_MIN_ROWS_PER_WG;
  if (nwg > SIM_MAX_WG) nwg = SIM_MAX_WG;
  if (nwg < 1) nwg = 1;
  return nwg;
}

// Sort cand_s/cand_r[0..SIM_CAND) descending by score (whole workgroup, 256 threads).
__device__ void bitonic_desc(float* cs, int* cr) {
  for (int k = 2; k <= SIM_CAND; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      __syncthreads();
      const int i = threadIdx.x;  // SIM_CAND == 256 threads
      const int p = i ^ j;
      if (p > i) {
        const bool desc = (i & k) == 0;
        const float a = cs[i], b = cs[p];
        const bool swap = desc ? (a < b) : (a > b);
        if (swap) {
          cs[i] = b; cs[p] = a;
          const int t = cr[i]; cr[i] = cr[p]; cr[p] = t;
        }
      }
    }
  }
  __syncthreads();
}

// Compact query c's buffer to its best K entries and update its threshold.
__device__ void compact_query(float* cs, int* cr, int* cnt, float* theta, int K) {
  const int n = min(*cnt, SIM_CAND);
  if (threadIdx.x >= n) { cs[threadIdx.x] = -INFINITY; cr[threadIdx.x] = -1; }
  bitonic_desc(cs, cr);
  if (threadIdx.x == 0) {
    const int keep = min(n, K);
    *cnt = keep;
    if (keep == K) *theta = cs[K - 1];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void cosine_stage1_kernel(
    float* __restrict__ ws_s, int* __restrict__ ws_r, const bf16* __restrict__ queries,
    const bf16* __restrict__ index, int Q, int N, int D, int K, const int* __restrict__ row_prio,
    const uint64_t* __restrict__ row_tags, const float* __restrict__ row_exp,
    const int* __restrict__ q_minp, const uint64_t* __restrict__ q_tags, float now) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* qt = reinterpret_cast<bf16*>(smem);                                  // [16][D]
  float* cand_s = reinterpret_cast<float*>(smem + SIM_QT * SIM_MAXD * 2);    // [16][CAND]
  int* cand_r = reinterpret_cast<int*>(cand_s + SIM_QT * SIM_CAND);          // [16][CAND]
  int* cnt = cand_r + SIM_QT * SIM_CAND;                                     // [16]
  float* theta = reinterpret_cast<float*>(cnt + SIM_QT);                     // [16]
  int* flag = reinterpret_cast<int*>(theta + SIM_QT);                        // [1]

  const int nwg = gridDim.x, wg = blockIdx.x, qtile = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int qi = qtile * SIM_QT + col;
  const bool qvalid = qi < Q;
  // stage the query tile into LDS (zero rows for missing queries)
  for (int v = threadIdx.x; v < SIM_QT * D / 8; v += 256) {
    const int r = (v * 8) / D, c = (v * 8) % D;
    const int qq = qtile * SIM_QT + r;
    bf16x8 x;
    if (qq < Q) x = *reinterpret_cast<const bf16x8*>(queries + (size_t)qq * D + c);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(qt + r * D + c) = x;
  }
  if (threadIdx.x < SIM_QT) { cnt[threadIdx.x] = 0; theta[threadIdx.x] = -INFINITY; }
  __syncthreads();

  const int minp = qvalid ? q_minp[qi] : 0x7fffffff;
  const uint64_t qtag = qvalid ? q_tags[qi] : 0ull;
  // rows of this slice
  const int per = (N + nwg - 1) / nwg;
  const int r0 = wg * per, r1 = min(N, r0 + per);
  const int ngroups = (max(0, r1 - r0) + 15) / 16;
  const int nrounds = (ngroups + 3) / 4;
  const int ksteps = D / 32;

  for (int round = 0; round < nrounds; ++round) {
    const int grp = round * 4 + wid;
    if (grp < ngroups) {
      const int gbase = r0 + grp * 16;
      // A operand: row gbase + col (clamped), dims 32m + 8g
      const int arow = min(gbase + col, N - 1);
      const bf16* ap = index + (size_t)arow * D + 8 * g;
      const bf16* bp = qt + col * D + 8 * g;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int m = 0; m < ksteps; ++m) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(ap + 32 * m);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(bp + 32 * m);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
      }
      // lane holds rows gbase + 4g + r for query col
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = gbase + 4 * g + r;
        if (!qvalid || row >= r1) continue;
        const float sc = acc[r];
        if (!(sc > theta[col])) continue;
        if (row_prio[row] < minp) continue;
        if ((row_tags[row] & qtag) != qtag) continue;
        const float ex = row_exp[row];
        if (ex != 0.f && !(ex > now)) continue;
        const int pos = atomicAdd(&cnt[col], 1);
        if (pos < SIM_CAND) {
          cand_s[col * SIM_CAND + pos] = sc;
          cand_r[col * SIM_CAND + pos] = row;
        }
      }
    }
    __syncthreads();
    // compaction when a buffer cannot absorb another round (64 rows)
    for (int c = 0; c < SIM_QT; ++c) {
      if (cnt[c] > SIM_CAND - 64)
        compact_query(cand_s + c * SIM_CAND, cand_r + c * SIM_CAND, &cnt[c], &theta[c], K);
    }
  }
  __syncthreads();
  // final: sort every valid query's buffer and emit its top-K
  for (int c = 0; c < SIM_QT; ++c) {
    const int qq = qtile * SIM_QT + c;
    if (qq >= Q) break;
    compact_query(cand_s + c * SIM_CAND, cand_r + c * SIM_CAND, &cnt[c], &theta[c], K);
    const int n = cnt[c];
    if (threadIdx.x < K) {
      const size_t o = ((size_t)qq * nwg + wg) * K + threadIdx.x;
      ws_s[o] = threadIdx.x < n ? cand_s[c * SIM_CAND + threadIdx.x] : -INFINITY;
      ws_r[o] = threadIdx.x < n ? cand_r[c * SIM_CAND + threadIdx.x] : -1;
    }
    __syncthreads();
  }
  (void)flag;
}

__global__ __launch_bounds__(256) void cosine_stage2_kernel(float* __restrict__ out_s,
                                                            int* __restrict__ out_r,
                                                            const float* __restrict__ ws_s,
                                                            const int* __restrict__ ws_r,
                                                            int nwg, int K) {
  __shared__ float cs[SIM_CAND];
  __shared__ int cr[SIM_CAND];
  __shared__ int cnt;
  __shared__ float theta;
  const int q = blockIdx.x;
  if (threadIdx.x == 0) { cnt = 0; theta = -INFINITY; }
  __syncthreads();
  const int total = nwg * K;
  const float* s = ws_s + (size_t)q * total;
  const int* r = ws_r + (size_t)q * total;
  for (int base = 0; base < total; base += 64) {
    if (threadIdx.x < 64) {
      const int i = base + threadIdx.x;
      if (i < total && r[i] >= 0 && s[i] > theta) {
        const int pos = atomicAdd(&cnt, 1);
        if (pos < SIM_CAND) { cs[pos] = s[i]; cr[pos] = r[i]; }
      }
    }
    __syncthreads();
    if (cnt > SIM_CAND - 64) compact_query(cs, cr, &cnt, &theta, K);
  }
  compact_query(cs, cr, &cnt, &theta, K);
  if (threadIdx.x < K) {
    out_s[(size_t)q * K + threadIdx.x] = threadIdx.x < cnt ? cs[threadIdx.x] : -INFINITY;
    out_r[(size_t)q * K + threadIdx.x] = threadIdx.x < cnt ? cr[threadIdx.x] : -1;
  }
}

}  // namespace pa

extern "C" int pa_cosine_topk_workspace_bytes(int Q, int N, int K) {
  const int nwg = (N + pa::SIM_MIN_ROWS_PER_WG - 1) / pa::SIM_MIN_ROWS_PER_WG;
  const int w = nwg > pa::SIM_MAX_WG ? pa::SIM_MAX_WG : (nwg < 1 ? 1 : nwg);
  return Q * w * K * 8;
}

extern "C" int pa_cosine_topk(float* out_scores, int* out_rows, void* workspace,
                              const void* queries, const void* index, int Q, int N, int D, int K,
                              const int* row_priority, const uint64_t* row_tags,
                              const float* row_expiry, const int* q_min_priority,
                              const uint64_t* q_tags, float now, int n_valid, hipStream_t st) {
  (void)n_valid;
  if (Q <= 0) return 0;
  if (D % 32 != 0 || D > pa::SIM_MAXD || K < 1 || K > pa::SIM_MAXK) return -1;
  if (N <= 0) {
    // empty index: every query gets an empty result (the reference raised here;
    // SURVEY App. A #26)
    hipMemsetAsync(out_rows, 0xff, (size_t)Q * K * sizeof(int), st);
    return (int)hipGetLastError();
  }
  int nwg = (N + pa::SIM_MIN_ROWS_PER_WG - 1) / pa::SIM_MIN_ROWS_PER_WG;
  nwg = nwg > pa::SIM_MAX_WG ? pa::SIM_MAX_WG : (nwg < 1 ? 1 : nwg);
  float* ws_s = reinterpret_cast<float*>(workspace);
  int* ws_r = reinterpret_cast<int*>(ws_s + (size_t)Q * nwg * K);
  const size_t lds = pa::SIM_QT * pa::SIM_MAXD * 2 + pa::SIM_QT * pa::SIM_CAND * 8 +
                     pa::SIM_QT * 8 + 16;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)pa::cosine_stage1_kernel,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  dim3 g1(nwg, (Q + pa::SIM_QT - 1) / pa::SIM_QT);
  hipLaunchKernelGGL(pa::cosine_stage1_kernel, g1, dim3(256), lds, st, ws_s, ws_r,
                     (const pa::bf16*)queries, (const pa::bf16*)index, Q, N, D, K, row_priority,
                     row_tags, row_expiry, q_min_priority, q_tags, now);
  hipLaunchKernelGGL(pa::cosine_stage2_kernel, dim3(Q), dim3(256), 0, st, out_scores, out_rows,
                     ws_s, ws_r, nwg, K);
  return (int)hipGetLastError();
}
