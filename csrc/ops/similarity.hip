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
// Stage 1 (one pass over the index for up to 64 queries): each workgroup owns a
// slice of rows; its 16 waves take 16-row groups and multiply them by EVERY query
// tile with v_mfma_f32_16x16x32_bf16 — index rows stream from HBM straight into
// the A operand once (the index is stored in 16-row tiles, fragment-major:
// [N/16][D/32][64 lanes][8], so each wave load is 1 KiB contiguous instead of
// 16 rows x 64 B — half the load-path work per streamed byte), the (<= 64) queries sit in LDS as B operands, so a 205 GB
// 100M x 1024 index is read exactly once per batch of agent queries. Scores
// above a query's running threshold (and passing the filters) are appended to
// that query's candidate buffer (global workspace, per workgroup); a full buffer
// is sorted (bitonic, in LDS) and the threshold raised to its k-th best. Each
// slice writes its top-k. Stage 2 (one WG per query) merges the slices' lists.
#include "common.h"

namespace pa {

constexpr int SIM_CAND = 512;     // candidate buffer per (slice, query), power of two
constexpr int SIM_MAXK = 64;
constexpr int SIM_QT = 16;        // queries per MFMA tile (N = 16)
constexpr int SIM_MAXQ = 64;      // queries per pass (4 tiles resident in LDS)
constexpr int SIM_MAXD = 1024;    // LDS query capacity per query (bf16)
constexpr int SIM_THREADS = 1024; // 16 waves: 128 KB of row loads in flight per CU
constexpr int SIM_MIN_ROWS_PER_WG = 2048;
constexpr int SIM_KB = 8;         // k-steps per row-load batch (two batches in flight)
constexpr int SIM_MAX_WG = 256;    // one resident workgroup per CU: the threshold warm-up is paid once per CU

__host__ __device__ inline int sim_num_wg(int N) {
  int nwg = (N + SIM_MIN_ROWS_PER_WG - 1) / SIM_MIN_ROWS_PER_WG;
  if (nwg > SIM_MAX_WG) nwg = SIM_MAX_WG;
  if (nwg < 1) nwg = 1;
  return nwg;
}

// Sort cand_s/cand_r[0..SIM_CAND) descending by score (whole workgroup, >= SIM_CAND threads).
__device__ void bitonic_desc(float* cs, int* cr) {
  for (int k = 2; k <= SIM_CAND; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      __syncthreads();
      const int i = threadIdx.x;
      const int p = i ^ j;
      if (i < SIM_CAND && p > i) {
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
  if (threadIdx.x < SIM_CAND && threadIdx.x >= n) { cs[threadIdx.x] = -INFINITY; cr[threadIdx.x] = -1; }
  bitonic_desc(cs, cr);
  if (threadIdx.x == 0) {
    const int keep = min(n, K);
    *cnt = keep;
    if (keep == K) *theta = cs[K - 1];
  }
  __syncthreads();
}

// Sort the global candidate buffer `gs/gr` of one query through the LDS scratch,
// keep the best K, raise the threshold.
__device__ void compact_global(float* gs, int* gr, float* cs, int* cr, int* cnt, float* theta, int K) {
  const int n = min(*cnt, SIM_CAND);
  if (threadIdx.x < SIM_CAND) {
    cs[threadIdx.x] = threadIdx.x < n ? gs[threadIdx.x] : -INFINITY;
    cr[threadIdx.x] = threadIdx.x < n ? gr[threadIdx.x] : -1;
  }
  bitonic_desc(cs, cr);  // begins and ends with a barrier
  if (threadIdx.x < K) {
    gs[threadIdx.x] = cs[threadIdx.x];
    gr[threadIdx.x] = cr[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    const int keep = min(n, K);
    *cnt = keep;
    if (keep == K) *theta = cs[K - 1];
  }
  __syncthreads();
}

__global__ __launch_bounds__(SIM_THREADS) void cosine_stage1_kernel(
    float* __restrict__ ws_s, int* __restrict__ ws_r, float* __restrict__ cand_s, int* __restrict__ cand_r,
    const bf16* __restrict__ queries, const bf16* __restrict__ index, int Q, int N, int D, int K,
    const int* __restrict__ row_prio, const uint64_t* __restrict__ row_tags,
    const float* __restrict__ row_exp, const int* __restrict__ q_minp, const uint64_t* __restrict__ q_tags,
    float now) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int NQT = (Q + SIM_QT - 1) / SIM_QT;
  const int QLD = D + 8;  // padded LDS row: the 16 query rows of a B fragment hit distinct bank slots
  bf16* qt = reinterpret_cast<bf16*>(smem);                                     // [NQT*16][QLD]
  float* cs = reinterpret_cast<float*>(smem + (size_t)NQT * SIM_QT * QLD * 2);  // sort scratch [CAND]
  int* cr = reinterpret_cast<int*>(cs + SIM_CAND);                            // [CAND]
  int* cnt = cr + SIM_CAND;                                                   // [MAXQ]
  float* theta = reinterpret_cast<float*>(cnt + SIM_MAXQ);                    // [MAXQ]
  int* minp = reinterpret_cast<int*>(theta + SIM_MAXQ);                       // [MAXQ]
  uint64_t* qtag = reinterpret_cast<uint64_t*>(minp + SIM_MAXQ);              // [MAXQ]

  const int nwg = gridDim.x, wg = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  for (int v = threadIdx.x; v < NQT * SIM_QT * D / 8; v += SIM_THREADS) {
    const int r = (v * 8) / D, c = (v * 8) % D;
    bf16x8 x;
    if (r < Q) x = *reinterpret_cast<const bf16x8*>(queries + (size_t)r * D + c);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(qt + (size_t)r * QLD + c) = x;
  }
  if (threadIdx.x < SIM_MAXQ) {
    const int q = threadIdx.x;
    cnt[q] = 0;
    theta[q] = -INFINITY;
    minp[q] = q < Q ? q_minp[q] : 0x7fffffff;
    qtag[q] = q < Q ? q_tags[q] : 0ull;
  }
  __syncthreads();

  float* my_s = cand_s + (size_t)wg * SIM_MAXQ * SIM_CAND;
  int* my_r = cand_r + (size_t)wg * SIM_MAXQ * SIM_CAND;
  const int per = ((N + nwg - 1) / nwg + 15) / 16 * 16;  // slices start on 16-row tiles
  const int r0 = wg * per, r1 = min(N, r0 + per);
  const int ngroups = (max(0, r1 - r0) + 15) / 16;
  constexpr int NW = SIM_THREADS / 64;
  const int nrounds = (ngroups + NW - 1) / NW;
  const int ksteps = D / 32;

  // Row loads are double-buffered in batches of SIM_KB k-steps (bufA / bufB) and
  // the first batch of a wave's NEXT 16-row group is issued before the round's
  // candidate work and barrier, so ~2 x SIM_KB KiB per wave stay in flight across
  // group and round boundaries (a round-synchronous loop drains the stream at
  // every barrier: 3.5-3.8 TB/s before).
  auto tile_ptr = [&](int grp_) {
    return index + ((size_t)((r0 + grp_ * 16) >> 4) * ksteps) * 512 + lane * 8;
  };
  auto load_batch = [&](const bf16* ap, int m, bf16x8 (&dst)[SIM_KB]) {
#pragma unroll
    for (int u = 0; u < SIM_KB; ++u)
      dst[u] = (m + u < ksteps) ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(ap + 512 * (m + u)))
                                : bf16x8{};
  };
  bf16x8 bufA[SIM_KB], bufB[SIM_KB];
  if (wid < ngroups) load_batch(tile_ptr(wid), 0, bufA);

  for (int round = 0; round < nrounds; ++round) {
    const int grp = round * NW + wid;
    if (grp < ngroups) {
      const int gbase = r0 + grp * 16;
      // packed tile gbase/16: k-step m is 64 lanes x 16 B contiguous (1 KiB per wave load)
      const bf16* ap = tile_ptr(grp);
      f32x4 acc[SIM_MAXQ / SIM_QT];
#pragma unroll
      for (int t = 0; t < SIM_MAXQ / SIM_QT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto compute = [&](const bf16x8 (&av)[SIM_KB], int m) {
#pragma unroll
        for (int u = 0; u < SIM_KB; ++u) {
          if (m + u >= ksteps) break;
#pragma unroll
          for (int t = 0; t < SIM_MAXQ / SIM_QT; ++t) {
            if (t < NQT) {
              const bf16x8 b = *reinterpret_cast<const bf16x8*>(qt + (size_t)(t * SIM_QT + col) * QLD + 32 * (m + u) + 8 * g);
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[u], b, acc[t], 0, 0, 0);
            }
          }
        }
      };
      for (int m = 0; m < ksteps; m += 2 * SIM_KB) {
        if (m + SIM_KB < ksteps) load_batch(ap, m + SIM_KB, bufB);
        compute(bufA, m);
        if (m + 2 * SIM_KB < ksteps) load_batch(ap, m + 2 * SIM_KB, bufA);
        else if (grp + NW < ngroups) load_batch(tile_ptr(grp + NW), 0, bufA);  // next group's first batch
        if (m + SIM_KB < ksteps) compute(bufB, m + SIM_KB);
      }
      // lane holds rows gbase + 4g + r for queries t*16 + col
#pragma unroll
      for (int t = 0; t < SIM_MAXQ / SIM_QT; ++t) {
        const int q = t * SIM_QT + col;
        if (t >= NQT || q >= Q) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = gbase + 4 * g + r;
          const float sc = acc[t][r];
          if (row >= r1 || !(sc > theta[q])) continue;
          if (row_prio[row] < minp[q]) continue;
          if ((row_tags[row] & qtag[q]) != qtag[q]) continue;
          const float ex = row_exp[row];
          if (ex != 0.f && !(ex > now)) continue;
          const int pos = atomicAdd(&cnt[q], 1);
          if (pos < SIM_CAND) {
            my_s[q * SIM_CAND + pos] = sc;
            my_r[q * SIM_CAND + pos] = row;
          }
        }
      }
    }
    __syncthreads();
    // a buffer must absorb the next round (NW waves x 16 rows)
    for (int q = 0; q < Q; ++q)
      if (cnt[q] > SIM_CAND - NW * 16)
        compact_global(my_s + q * SIM_CAND, my_r + q * SIM_CAND, cs, cr, &cnt[q], &theta[q], K);
  }
  __syncthreads();
  for (int q = 0; q < Q; ++q) {
    compact_global(my_s + q * SIM_CAND, my_r + q * SIM_CAND, cs, cr, &cnt[q], &theta[q], K);
    const int n = cnt[q];
    if (threadIdx.x < K) {
      const size_t o = ((size_t)q * nwg + wg) * K + threadIdx.x;
      ws_s[o] = threadIdx.x < n ? cs[threadIdx.x] : -INFINITY;
      ws_r[o] = threadIdx.x < n ? cr[threadIdx.x] : -1;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(SIM_CAND) void cosine_stage2_kernel(float* __restrict__ out_s,
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

// workspace = stage-1 top-k lists [Q][nwg][K] (score, row) + per-(slice, query)
// candidate buffers [nwg][64][CAND] (score, row)
extern "C" long long pa_cosine_topk_workspace_bytes(int Q, int N, int K) {
  const long long w = pa::sim_num_wg(N);
  return (long long)Q * w * K * 8 + w * pa::SIM_MAXQ * pa::SIM_CAND * 8;
}

extern "C" int pa_cosine_topk(float* out_scores, int* out_rows, void* workspace,
                              const void* queries, const void* index, int Q, int N, int D, int K,
                              const int* row_priority, const uint64_t* row_tags,
                              const float* row_expiry, const int* q_min_priority,
                              const uint64_t* q_tags, float now, int n_valid, hipStream_t st) {
  (void)n_valid;
  if (Q <= 0) return 0;
  if (D % 32 != 0 || D > pa::SIM_MAXD || K < 1 || K > pa::SIM_MAXK || Q > pa::SIM_MAXQ) return -1;
  if (N <= 0) {
    // empty index: every query gets an empty result (the reference raised here;
    // SURVEY App. A #26)
    (void)hipMemsetAsync(out_rows, 0xff, (size_t)Q * K * sizeof(int), st);
    return (int)hipGetLastError();
  }
  const int nwg = pa::sim_num_wg(N);
  float* ws_s = reinterpret_cast<float*>(workspace);
  int* ws_r = reinterpret_cast<int*>(ws_s + (size_t)Q * nwg * K);
  float* cand_s = reinterpret_cast<float*>(ws_r + (size_t)Q * nwg * K);
  int* cand_r = reinterpret_cast<int*>(cand_s + (size_t)nwg * pa::SIM_MAXQ * pa::SIM_CAND);
  const int nqt = (Q + pa::SIM_QT - 1) / pa::SIM_QT;
  const size_t lds = (size_t)nqt * pa::SIM_QT * (D + 8) * 2 + pa::SIM_CAND * 8 + pa::SIM_MAXQ * (4 + 4 + 4 + 8);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)pa::cosine_stage1_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(pa::cosine_stage1_kernel, dim3(nwg), dim3(pa::SIM_THREADS), lds, st, ws_s, ws_r,
                     cand_s, cand_r, (const pa::bf16*)queries, (const pa::bf16*)index, Q, N, D, K,
                     row_priority, row_tags, row_expiry, q_min_priority, q_tags, now);
  hipLaunchKernelGGL(pa::cosine_stage2_kernel, dim3(Q), dim3(pa::SIM_CAND), 0, st, out_scores, out_rows,
                     ws_s, ws_r, nwg, K);
  return (int)hipGetLastError();
}
