// Paged, GQA-packed flash attention for CDNA4 — one kernel for prefill chunks,
// decode tokens and mixed batches (SURVEY §2.5 N3 + N4).
//
// Layout (written by rope_cache.hip):
//   q        [T, H, 128] bf16 (already rotated)
//   k_cache  [num_blocks, KV, 16, 128]   keys row-major inside a 16-token page
//   v_cache  [num_blocks, KV, 128, 16]   values transposed inside a page
//
// MFMA formulation (v_mfma_f32_16x16x32_bf16, wave64):
//   The 16 MFMA columns are (G query heads of one KV head) x (16/G query tokens),
//   so a decode step of Llama-3-8B (G=4) packs 4 heads of 1 token, and a prefill
//   wave packs 4 heads x 4 tokens — the GQA group is the N dimension.
//   S^T = K · Q^T   A = K rows (keys) straight from the page, B = Q^T in registers
//   O^T = V^T · P^T A = V^T rows straight from the page, B = P^T = the S^T
//                   accumulator itself (no LDS round trip, no lane shuffle)
//   The row permutation key(i,c) = 8*(i>>2) + 4c + (i&3) on the K load makes the
//   S^T accumulator of lane group g hold exactly keys 8g..8g+7 of a 32-key tile,
//   i.e. the B fragment PV needs, and makes V^T one 16-byte load per lane.
//   Softmax is per column = per lane&15: the max needs two xor-shuffles across the
//   four lane groups; the rescale of O is lane-local.
//
// Work decomposition (built by the host scheduler, see runtime/scheduler.cpp):
//   item = (seq, q_begin, nq | part<<8 | nparts<<20, partial_slot)
//   nq <= 16/G : "kv-split" — the 4 waves of the workgroup share the query
//                columns and interleave 32-key tiles; merged through LDS. Long
//                contexts are further split into 512-key partitions (flash-
//                decoding); partitions are combined by attn_reduce_kernel.
//   nq >  16/G : "q-split" — wave w owns tokens [q_begin + w*16/G, ...) and
//                walks its causal key range alone.
// The grid is (max_items, KV) with a device-side item count so the launch is
// shape-stable under hipGraph capture.
#include "common.h"

namespace pa {

constexpr int ATT_HD = 128;
constexpr int ATT_BLK = 16;
constexpr int ATT_PART = 512;  // keys per decode partition (multiple of 32)
constexpr float NEG_BIG = -1.0e30f;

template <int G>
__global__ __launch_bounds__(256) void paged_attn_kernel(
    bf16* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml,
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int4* __restrict__ items,
    const int* __restrict__ n_items, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len,
    const int* __restrict__ block_table, int max_blocks, int H, int KV, float scale_log2) {
  constexpr int TPW = 16 / G;
  const int item = blockIdx.x;
  if (item >= n_items[0]) return;
  const int kvh = blockIdx.y;
  const int4 it = items[item];
  const int s = it.x, qb = it.y;
  const int nq = it.z & 0xff, part = (it.z >> 8) & 0xfff, nparts = it.z >> 20;
  const int pidx = it.w;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int hg = col % G, tq = col / G;
  const int ctx = ctx_len[s], ql = q_len[s], q0 = q_start[s];
  const bool kvsplit = nq <= TPW;
  if (!kvsplit && wid * TPW >= nq) return;  // idle wave in a short q-split tile (no barrier follows)

  const int tokbase = kvsplit ? qb : qb + wid * TPW;
  const int ncols_tok = kvsplit ? nq : min(TPW, nq - wid * TPW);
  const bool colvalid = tq < ncols_tok;
  const int tok = tokbase + tq;
  const int key_limit = colvalid ? (ctx - ql + tok + 1) : 0;
  const int head = kvh * G + hg;

  int kv_begin, kv_end;
  if (kvsplit) {
    const int causal_end = ctx - ql + qb + nq;
    kv_begin = nparts > 1 ? part * ATT_PART : 0;
    kv_end = nparts > 1 ? min(causal_end, kv_begin + ATT_PART) : causal_end;
  } else {
    kv_begin = 0;
    kv_end = ctx - ql + tokbase + ncols_tok;
  }
  const int t_first = kv_begin >> 5;
  const int t_last = (kv_end + 31) >> 5;
  const int t_step = kvsplit ? 4 : 1;

  // Q^T fragments (B operand): column col, dims 32m + 8g + j.
  bf16x8 qf[4];
  {
    const bf16* qrow = q + ((size_t)(q0 + (colvalid ? tok : 0)) * H + head) * ATT_HD + 8 * g;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + 32 * m);
      if (!colvalid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)0.f;
      }
      qf[m] = v;
    }
  }

  const int* bt = block_table + (size_t)s * max_blocks;
  const int nblk = (ctx + ATT_BLK - 1) / ATT_BLK;
  // lane-constant parts of the K / V addresses
  const int kin = 8 * (col >> 2) + (col & 3);  // key within tile for chunk 0 (chunk 1: +4)
  const size_t kv_stride_blk = (size_t)KV * ATT_BLK * ATT_HD;  // elements per page (all heads)

  f32x4 o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = NEG_BIG, l_run = 0.f;

  for (int t = t_first + (kvsplit ? wid : 0); t < t_last; t += t_step) {
    const int b0 = min(2 * t, nblk - 1), b1 = min(2 * t + 1, nblk - 1);
    const int pb0 = bt[b0], pb1 = bt[b1];
    // K fragments: key = 32t + kin + 4c  -> page (kin >= 16), slot (kin & 15) + 4c
    const int pk = (kin >= 16) ? pb1 : pb0;
    const bf16* kbase =
        k_cache + (size_t)pk * kv_stride_blk + ((size_t)kvh * ATT_BLK + (kin & 15)) * ATT_HD + 8 * g;
    bf16x8 kf[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        kf[c][m] = *reinterpret_cast<const bf16x8*>(kbase + 4 * c * ATT_HD + 32 * m);
    // V^T fragments: dim 16n + col, keys 8g..8g+7 -> page (g >> 1), slot 8*(g&1)
    const int pv = (g >> 1) ? pb1 : pb0;
    const bf16* vbase =
        v_cache + (size_t)pv * kv_stride_blk + ((size_t)kvh * ATT_HD + col) * ATT_BLK + 8 * (g & 1);
    bf16x8 vf[8];
#pragma unroll
    for (int n = 0; n < 8; ++n)
      vf[n] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)16 * n * ATT_BLK);

    // S^T for the two 16-key chunks
    f32x4 sc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 4; ++m)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[c][m], qf[m], acc, 0, 0, 0);
      sc[c] = acc;
    }
    // scale + causal/length mask; lane holds keys 32t + 8g + 4c + r
    float tmax = NEG_BIG;
    const int kb = 32 * t + 8 * g;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb + 4 * c + r;
        float v = sc[c][r] * scale_log2;
        v = (key < key_limit && key >= kv_begin) ? v : NEG_BIG;
        sc[c][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    bf16x8 pf;
    float psum = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(sc[c][r] - m_new);
        psum += p;
        pf[4 * c + r] = (bf16)p;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      o[n] *= alpha;
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[n], pf, o[n], 0, 0, 0);
    }
  }
  // per-column denominator: sum the four lane groups' partial sums
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);

  if (!kvsplit) {
    if (!colvalid) return;
    const float inv = 1.f / l_run;
    bf16* orow = out + ((size_t)(q0 + tok) * H + head) * ATT_HD + 4 * g;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[n][r] * inv);
      *reinterpret_cast<bf16x4*>(orow + 16 * n) = w;
    }
    return;
  }

  // kv-split: merge the four waves through LDS
  __shared__ float lds_o[4][16][ATT_HD + 4];
  __shared__ float lds_m[4][16];
  __shared__ float lds_l[4][16];
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) lds_o[wid][col][16 * n + 4 * g + r] = o[n][r];
  if (g == 0) {
    lds_m[wid][col] = m_run;
    lds_l[wid][col] = l_run;
  }
  __syncthreads();
  const int ccol = threadIdx.x >> 4;
  const int d0 = (threadIdx.x & 15) * 8;
  float mt = NEG_BIG;
#pragma unroll
  for (int w = 0; w < 4; ++w) mt = fmaxf(mt, lds_m[w][ccol]);
  float wgt[4], L = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    wgt[w] = exp2f(lds_m[w][ccol] - mt);
    L += wgt[w] * lds_l[w][ccol];
  }
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) a += wgt[w] * lds_o[w][ccol][d0 + j];
    acc[j] = a;
  }
  const int ctq = ccol / G, chg = ccol % G;
  if (nparts > 1) {
    float* po = part_o + (((size_t)pidx * KV + kvh) * 16 + ccol) * ATT_HD + d0;
#pragma unroll
    for (int j = 0; j < 8; ++j) po[j] = acc[j];
    if ((threadIdx.x & 15) == 0) {
      float* pm = part_ml + (((size_t)pidx * KV + kvh) * 16 + ccol) * 2;
      pm[0] = mt;
      pm[1] = L;
    }
    return;
  }
  if (ctq >= nq) return;
  const float inv = 1.f / L;
  bf16x8 w8;
#pragma unroll
  for (int j = 0; j < 8; ++j) w8[j] = (bf16)(acc[j] * inv);
  *reinterpret_cast<bf16x8*>(out + ((size_t)(q0 + qb + ctq) * H + kvh * G + chg) * ATT_HD + d0) = w8;
}

// Combine decode partitions: ritem = (seq, first partial slot, nparts, q_begin | nq << 16)
template <int G>
__global__ __launch_bounds__(256) void attn_reduce_kernel(
    bf16* __restrict__ out, const float* __restrict__ part_o, const float* __restrict__ part_ml,
    const int4* __restrict__ ritems, const int* __restrict__ n_ritems,
    const int* __restrict__ q_start, int H, int KV) {
  const int item = blockIdx.x;
  if (item >= n_ritems[0]) return;
  const int kvh = blockIdx.y;
  const int4 it = ritems[item];
  const int s = it.x, p0 = it.y, np = it.z, qb = it.w & 0xffff, nq = it.w >> 16;
  const int ccol = threadIdx.x >> 4, d0 = (threadIdx.x & 15) * 8;
  const int ctq = ccol / G, chg = ccol % G;
  if (ctq >= nq) return;
  float mt = NEG_BIG;
  for (int p = 0; p < np; ++p)
    mt = fmaxf(mt, part_ml[(((size_t)(p0 + p) * KV + kvh) * 16 + ccol) * 2]);
  float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < np; ++p) {
    const size_t base = ((size_t)(p0 + p) * KV + kvh) * 16 + ccol;
    const float w = exp2f(part_ml[base * 2] - mt);
    L += w * part_ml[base * 2 + 1];
    const f32x4* po = reinterpret_cast<const f32x4*>(part_o + base * ATT_HD + d0);
    const f32x4 a = po[0], b = po[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += w * a[j];
      acc[4 + j] += w * b[j];
    }
  }
  const float inv = 1.f / L;
  bf16x8 w8;
#pragma unroll
  for (int j = 0; j < 8; ++j) w8[j] = (bf16)(acc[j] * inv);
  *reinterpret_cast<bf16x8*>(out + ((size_t)(q_start[s] + qb + ctq) * H + kvh * G + chg) * ATT_HD +
                             d0) = w8;
}

}  // namespace pa

extern "C" int pa_paged_attention(void* out, float* part_o, float* part_ml, const void* q,
                                  const void* k_cache, const void* v_cache, const int* items,
                                  const int* n_items, int max_items, const int* ritems,
                                  const int* n_ritems, int max_ritems, const int* q_start,
                                  const int* q_len, const int* ctx_len, const int* block_table,
                                  int max_blocks, int H, int KV, float scale_log2,
                                  hipStream_t st) {
  if (H % KV != 0) return -1;
  const int G = H / KV;
  dim3 grid(max_items, KV), rgrid(max_ritems, KV);
#define PA_ATT(GG)                                                                          \
  do {                                                                                      \
    if (max_items > 0)                                                                      \
      hipLaunchKernelGGL(pa::paged_attn_kernel<GG>, grid, dim3(256), 0, st, (pa::bf16*)out, \
                         part_o, part_ml, (const pa::bf16*)q, (const pa::bf16*)k_cache,      \
                         (const pa::bf16*)v_cache, (const int4*)items, n_items, q_start,     \
                         q_len, ctx_len, block_table, max_blocks, H, KV, scale_log2);       \
    if (max_ritems > 0)                                                                     \
      hipLaunchKernelGGL(pa::attn_reduce_kernel<GG>, rgrid, dim3(256), 0, st,               \
                         (pa::bf16*)out, part_o, part_ml, (const int4*)ritems, n_ritems,     \
                         q_start, H, KV);                                                   \
  } while (0)
  switch (G) {
    case 1: PA_ATT(1); break;
    case 2: PA_ATT(2); break;
    case 4: PA_ATT(4); break;
    case 8: PA_ATT(8); break;
    case 16: PA_ATT(16); break;
    default: return -2;
  }
#undef PA_ATT
  return (int)hipGetLastError();
}
