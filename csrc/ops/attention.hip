// Paged, GQA-packed flash attention for CDNA4 — one kernel for prefill chunks,
// decode tokens and mixed batches (SURVEY §2.5 N3 + N4).
//
// Layout (written by rope_cache.hip):
//   q        [T, H, 128] bf16 (already rotated)
//   k_cache  [num_blocks, KV, 16, 16, 8] keys fragment-major: [dim/8][key][dim%8]
//   v_cache  [num_blocks, KV, 128, 16]   values transposed inside a page
// so that each MFMA A-fragment load (8 dims x 16 keys of K, 8 keys x 16 dims of
// V^T) is one contiguous 256-B run: whole cache lines per load instruction.
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
//                decoding); the last partition to finish merges them (ticket
//                counter per (sequence, KV head), no second launch).
//   nq >  16/G : "prefill" — items of 32/G tokens = 32 columns on 32x32x16
//                MFMAs; the 4 waves interleave key tiles and merge through LDS.
// The grid is (max_items, KV) with a device-side item count so the launch is
// shape-stable under hipGraph capture.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace pa {

constexpr int ATT_HD = 128;
constexpr int ATT_BLK = 16;
constexpr int ATT_PART = 512;  // default keys per decode partition (the step may choose 256/128)
constexpr float NEG_BIG = -1.0e30f;

// ---------------------------------------------------------------------------
// kv-split path (decode tokens / short runs, nq <= 16/G): 16x16x32 MFMA, the 4
// waves interleave 32-key tiles and merge through LDS.
// NW waves per workgroup (4, or 8 for small decode batches: each wave's chain of 32-key
// tiles halves, which is what a latency-bound 8-row decode step waits on)
template <int NW>
constexpr int att_lds_decode_bytes() { return (NW * 16 * (ATT_HD + 4) + 2 * NW * 16) * 4; }
constexpr int ATT_LDS_DECODE_BYTES = att_lds_decode_bytes<4>();
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;

// An attention output store (8 bf16, one 16-B vector store)
__device__ __forceinline__ void att_store8(bf16* p, const bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }

template <int G, int NW = 4>
__device__ __forceinline__ void decode_item(
    const int4 it, char* smem, bf16* __restrict__ out, float* __restrict__ part_o,
    float* __restrict__ part_ml, int* __restrict__ counters, const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int* __restrict__ q_start, const int* __restrict__ q_len,
    const int* __restrict__ ctx_len, const int* __restrict__ block_table, int max_blocks, int H,
    int KV, int kvh, float scale_log2, int psz, int acq) {
  const int s = it.x, qb = it.y;
  const int nq = it.z & 0xff, part = (it.z >> 8) & 0xfff, nparts = it.z >> 20;
  const int pidx = it.w;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int hg = col % G, tq = col / G;
  const int ctx = ctx_len[s], ql = q_len[s], q0 = q_start[s];

  const bool colvalid = tq < nq;
  const int tok = qb + tq;
  const int key_limit = colvalid ? (ctx - ql + tok + 1) : 0;
  const int head = kvh * G + hg;
  const int causal_end = ctx - ql + qb + nq;
  const int kv_begin = nparts > 1 ? part * psz : 0;
  const int kv_end = nparts > 1 ? min(causal_end, kv_begin + psz) : causal_end;
  const int t_first = kv_begin >> 5;
  const int t_last = (kv_end + 31) >> 5;

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
  const int kin = 8 * (col >> 2) + (col & 3);  // key within tile for chunk 0 (chunk 1: +4)
  const size_t kv_stride_blk = (size_t)KV * ATT_BLK * ATT_HD;  // elements per page (all heads)

  f32x4 o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = NEG_BIG, l_run = 0.f;

  // K/V fragments of one 32-key tile; the loop keeps the next tile's loads in flight
  // while computing this one (small decode batches have too few workgroups to hide
  // HBM latency by occupancy alone: 8 sequences x 8 KV heads x 2 partitions).
  auto load_tile = [&](int t, bf16x8 (&kf)[2][4], bf16x8 (&vf)[8]) {
    const int b0 = min(2 * t, nblk - 1), b1 = min(2 * t + 1, nblk - 1);
    const int pb0 = bt[b0], pb1 = bt[b1];
    const int pk = (kin >= 16) ? pb1 : pb0;
    // dims 32m + 8g = chunk 4m + g; key (kin & 15) + 4c
    const bf16* kbase = k_cache + (size_t)pk * kv_stride_blk +
                        (((size_t)kvh * 16 + g) * ATT_BLK + (kin & 15)) * 8;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        kf[c][m] = *reinterpret_cast<const bf16x8*>(kbase + (4 * m * ATT_BLK + 4 * c) * 8);
    const int pv = (g >> 1) ? pb1 : pb0;
    const bf16* vbase =
        v_cache + (size_t)pv * kv_stride_blk + ((size_t)kvh * ATT_HD + col) * ATT_BLK + 8 * (g & 1);
#pragma unroll
    for (int n = 0; n < 8; ++n)
      vf[n] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)16 * n * ATT_BLK);
  };
  bf16x8 kf[2][4], vf[8];
  if (t_first + wid < t_last) load_tile(t_first + wid, kf, vf);
  for (int t = t_first + wid; t < t_last; t += NW) {
    bf16x8 kn[2][4], vn[8];
    if (t + NW < t_last) load_tile(t + NW, kn, vn);

    f32x4 sc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 4; ++m)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[c][m], qf[m], acc, 0, 0, 0);
      sc[c] = acc;
    }
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
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int m = 0; m < 4; ++m) kf[c][m] = kn[c][m];
#pragma unroll
    for (int n = 0; n < 8; ++n) vf[n] = vn[n];
  }
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);

  // merge the NW waves through LDS
  float(*lds_o)[16][ATT_HD + 4] = reinterpret_cast<float(*)[16][ATT_HD + 4]>(smem);
  float(*lds_m)[16] = reinterpret_cast<float(*)[16]>(smem + NW * 16 * (ATT_HD + 4) * sizeof(float));
  float(*lds_l)[16] = lds_m + NW;
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) lds_o[wid][col][16 * n + 4 * g + r] = o[n][r];
  if (g == 0) {
    lds_m[wid][col] = m_run;
    lds_l[wid][col] = l_run;
  }
  __syncthreads();
  // the first 256 threads merge (16 columns x 16 threads x 8 dims); with NW = 8 the others
  // only join the workgroup-wide steps (the partition hand-off)
  const bool mthr = NW == 4 || threadIdx.x < 256;
  const int ccol = (threadIdx.x >> 4) & 15;
  const int d0 = (threadIdx.x & 15) * 8;
  float mt = NEG_BIG;
#pragma unroll
  for (int w = 0; w < NW; ++w) mt = fmaxf(mt, lds_m[w][ccol]);
  float wgt[NW], L = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wgt[w] = exp2f(lds_m[w][ccol] - mt);
    L += wgt[w] * lds_l[w][ccol];
  }
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += wgt[w] * lds_o[w][ccol][d0 + j];
    acc[j] = a;
  }
  const int ctq = ccol / G, chg = ccol % G;
  if (nparts > 1) {
    // Partition hand-off inside the launch (cdna_hip_programming.md §6 G16, common.h
    // handoff_last): part_o / part_ml live in UNCACHED device memory (ops.empty_handoff), the
    // slab is stored write-through (sc1) and (m, l) as one relaxed agent-scope 64-bit atomic,
    // every wave drains, then one lane takes a relaxed ticket; the holder of ticket nparts-1
    // runs ONE agent-scope acquire (mode g_handoff_attn = 1) and merges all partitions with sc1
    // loads. No producer release (its L2 write-back cost +77 us on a 64 x 1,000-key launch);
    // 0 bad runs in 10,000 poisoned repetitions for every 256/512-key, 4/8-wave case
    // (profiles/r4_handoff_uncached.md). No second launch.
    const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
        part_o + ((size_t)pidx * KV + kvh) * 16 * ATT_HD, 0, 16 * ATT_HD * 4, 0x00020000);
    const int soff = (ccol * ATT_HD + d0) * 4;
    if (mthr) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{acc[0], acc[1], acc[2], acc[3]}),
                                             ps, soff, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{acc[4], acc[5], acc[6], acc[7]}),
                                             ps, soff + 16, 0, 16);
    }
    if (mthr && (threadIdx.x & 15) == 0) {
      const unsigned long long mlv =
          ((unsigned long long)__float_as_uint(L) << 32) | (unsigned long long)__float_as_uint(mt);
      __hip_atomic_store((gu64*)(part_ml + (((size_t)pidx * KV + kvh) * 16 + ccol) * 2), mlv,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int* lflag = reinterpret_cast<int*>(smem + att_lds_decode_bytes<NW>());
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(counters + (size_t)s * KV + kvh, nparts, lflag, acq) || ctq >= nq || !mthr) return;
    const int p0 = pidx - part;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        part_o + (size_t)p0 * KV * 16 * ATT_HD, 0, nparts * KV * 16 * ATT_HD * 4, 0x00020000);
    auto load_ml = [&](int p) {
      return __hip_atomic_load((gu64*)(part_ml + (((size_t)(p0 + p) * KV + kvh) * 16 + ccol) * 2),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    float gm = NEG_BIG;
    for (int p = 0; p < nparts; ++p) gm = fmaxf(gm, __uint_as_float((unsigned)load_ml(p)));
    float GL = 0.f, ga[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < nparts; ++p) {
      const unsigned long long v = load_ml(p);
      const float pmv = __uint_as_float((unsigned)v), plv = __uint_as_float((unsigned)(v >> 32));
      const float w = exp2f(pmv - gm);
      GL += w * plv;
      const int roff = (((p * KV + kvh) * 16 + ccol) * ATT_HD + d0) * 4;
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, roff, 0, 16));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, roff + 16, 0, 16));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ga[j] += w * a[j];
        ga[4 + j] += w * b[j];
      }
    }
    const float ginv = 1.f / GL;
    bf16x8 g8;
#pragma unroll
    for (int j = 0; j < 8; ++j) g8[j] = (bf16)(ga[j] * ginv);
    att_store8(out + ((size_t)(q0 + qb + ctq) * H + kvh * G + chg) * ATT_HD + d0, g8);
    return;
  }
  if (ctq >= nq || !mthr) return;
  const float inv = 1.f / L;
  bf16x8 w8;
#pragma unroll
  for (int j = 0; j < 8; ++j) w8[j] = (bf16)(acc[j] * inv);
  att_store8(out + ((size_t)(q0 + qb + ctq) * H + kvh * G + chg) * ATT_HD + d0, w8);
}

// ---------------------------------------------------------------------------
// prefill path (nq > 16/G): 32x32x16 MFMA, an item is 32/G tokens = 32 columns
// (G heads x 32/G tokens); like the decode path, the 4 waves of the workgroup
// interleave the item's 32-key tiles (loaded straight into registers) and merge
// through LDS, so a chunk of n tokens yields n*G/32 items per KV head with
// short per-wave chains, and each K/V byte serves 32 columns.
//
//   S^T[32 keys x 32 cols] = K · Q^T    A = K rows, B = Q^T (registers)
//   O^T[128 x 32 cols]    += V^T · P^T  A = V^T rows, B = P^T = the S^T registers
//
// 32x32 accumulator row rho of lane (r, h), register g: rho = (g&3) + 8(g>>2) + 4h.
// Lane r loads K row pi(r) = r with bits 2 and 3 swapped, so registers 8s..8s+7
// of a lane hold keys 16s + 8h + 0..7 — exactly the B fragment of the PV MFMA
// for k-step s, whose V^T A fragment is one 16-B load (keys 8h..8h+7 of page s).
__device__ __forceinline__ int swap23(int x) { return (x & ~12) | ((x & 4) << 1) | ((x & 8) >> 1); }
constexpr int PF_LD = ATT_HD + 4;  // padded LDS row (floats) of the merge image

// One 32-key tile of the online softmax + its PV product, shared by both prefill
// paths. The tile is VALU-bound if written naively (the r2 counters showed ~25 VALU
// instructions per MFMA): the scale is folded into one FMA feeding v_exp, the causal
// mask runs only on tiles that cross some column's end (`mask`, wave-uniform), and the
// O rescale (64 multiplies) only when some column's running max actually grew.
// s: raw scores of S^T (lane column, registers g -> keys key0 + 16(g>>3) + (g&7),
// key0 = 32t + 8h); m_run is kept in scaled log2 units.
__device__ __forceinline__ void softmax_pv_tile(f32x16 s, bool mask, int key0, int key_limit, float scale_log2,
                                                float& m_run, float& l_run, f32x16 (&o)[4],
                                                const bf16x8 (&vf)[2][4]) {
  if (mask) {  // wave-uniform
    const int lim = key_limit - key0;
#pragma unroll
    for (int g = 0; g < 16; ++g) s[g] = (16 * (g >> 3) + (g & 7)) < lim ? s[g] : NEG_BIG;
  }
  float tmax = s[0];
#pragma unroll
  for (int g = 1; g < 16; ++g) tmax = fmaxf(tmax, s[g]);
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
  const float m_new = fmaxf(m_run, tmax * scale_log2);
  if (__any(m_new > m_run)) {  // wave-uniform: lanes whose max did not grow get alpha = 1
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    l_run *= alpha;
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] *= alpha;
    m_run = m_new;
  }
  const float nm = -m_run;
  float psum = 0.f;
  bf16x8 pf[2];
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float p = __builtin_amdgcn_exp2f(fmaf(s[g], scale_log2, nm));
    psum += p;
    pf[g >> 3][g & 7] = (bf16)p;
  }
  l_run += psum;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[st][m], pf[st], o[m], 0, 0, 0);
}

// S^T tile = K · Q^T over the 128-dim head: one accumulation chain (the 32x32x16
// MFMA's dependent-issue rate equals its independent one, so a second chain only
// adds 16 zeroing moves and 16 adds per tile).
__device__ __forceinline__ f32x16 qk_tile(const bf16x8 (&kf)[8], const bf16x8 (&qf)[8]) {
  f32x16 s;
#pragma unroll
  for (int j = 0; j < 16; ++j) s[j] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[i], qf[i], s, 0, 0, 0);
  return s;
}

template <int G, int NW = 4>
__device__ __forceinline__ void prefill_item(
    const int4 it, char* smem, bf16* __restrict__ out, const bf16* __restrict__ q,
    const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ q_start, const int* __restrict__ q_len, const int* __restrict__ ctx_len,
    const int* __restrict__ block_table, int max_blocks, int H, int KV, int kvh, float scale_log2) {
  const int s = it.x, qb = it.y, nq = it.z & 0xff;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int hg = r % G, tq = r / G;
  const int ctx = ctx_len[s], ql = q_len[s], q0 = q_start[s];
  const bool colvalid = tq < nq;
  const int tok = qb + tq;
  const int key_limit = colvalid ? (ctx - ql + tok + 1) : 0;
  const int head = kvh * G + hg;
  const int ntiles = (ctx - ql + qb + nq + 31) >> 5;
  const int kmin = ctx - ql + qb + 1;  // smallest causal end of the item's columns

  bf16x8 qf[8];
  {
    const bf16* qrow = q + ((size_t)(q0 + (colvalid ? tok : 0)) * H + head) * ATT_HD + 8 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + 16 * i);
      if (!colvalid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)0.f;
      }
      qf[i] = v;
    }
  }
  const int* bt = block_table + (size_t)s * max_blocks;
  const int nblk = (ctx + ATT_BLK - 1) / ATT_BLK;
  const size_t kv_stride_blk = (size_t)KV * ATT_BLK * ATT_HD;
  const int krow = swap23(r);

  f32x16 o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 16; ++j) o[m][j] = 0.f;
  float m_run = NEG_BIG, l_run = 0.f;

  for (int t = wid; t < ntiles; t += NW) {
    const int pb0 = bt[min(2 * t, nblk - 1)], pb1 = bt[min(2 * t + 1, nblk - 1)];
    // dims 16i + 8h = chunk 2i + h; key krow & 15 of page krow >> 4
    const bf16* kbase = k_cache + (size_t)(krow >= 16 ? pb1 : pb0) * kv_stride_blk +
                        (((size_t)kvh * 16 + h) * ATT_BLK + (krow & 15)) * 8;
    bf16x8 kf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) kf[i] = *reinterpret_cast<const bf16x8*>(kbase + (size_t)2 * i * ATT_BLK * 8);
    bf16x8 vf[2][4];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16* vbase = v_cache + (size_t)(st ? pb1 : pb0) * kv_stride_blk +
                          ((size_t)kvh * ATT_HD + r) * ATT_BLK + 8 * h;
#pragma unroll
      for (int m = 0; m < 4; ++m) vf[st][m] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)32 * m * ATT_BLK);
    }
    const f32x16 sc = qk_tile(kf, qf);
    softmax_pv_tile(sc, 32 * t + 32 > kmin, 32 * t + 8 * h, key_limit, scale_log2, m_run, l_run, o, vf);
  }
  l_run += __shfl_xor(l_run, 32, 64);

  // merge the NW waves: O^T images [wave][col][dim] (fp32) + per-column (m, l)
  float* lo = reinterpret_cast<float*>(smem);
  float* lm = lo + NW * 32 * PF_LD;
  float* ll = lm + NW * 32;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      f32x4 v = {o[m][4 * gq], o[m][4 * gq + 1], o[m][4 * gq + 2], o[m][4 * gq + 3]};
      *reinterpret_cast<f32x4*>(lo + (wid * 32 + r) * PF_LD + 32 * m + 8 * gq + 4 * h) = v;
    }
  if (h == 0) {
    lm[wid * 32 + r] = m_run;
    ll[wid * 32 + r] = l_run;
  }
  __syncthreads();
  const int ccol = threadIdx.x >> 3, d0 = (threadIdx.x & 7) * 16;
  const int ctq = ccol / G, chg = ccol % G;
  if (ctq >= nq || (NW == 8 && threadIdx.x >= 256)) return;
  float mt = NEG_BIG;
#pragma unroll
  for (int w = 0; w < NW; ++w) mt = fmaxf(mt, lm[w * 32 + ccol]);
  float wgt[NW], L = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wgt[w] = exp2f(lm[w * 32 + ccol] - mt);
    L += wgt[w] * ll[w * 32 + ccol];
  }
  const float inv = 1.f / L;
  bf16* orow = out + ((size_t)(q0 + qb + ctq) * H + kvh * G + chg) * ATT_HD + d0;
#pragma unroll
  for (int c8 = 0; c8 < 2; ++c8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const f32x4* src = reinterpret_cast<const f32x4*>(lo + (w * 32 + ccol) * PF_LD + d0 + 8 * c8);
      const f32x4 a = src[0], b = src[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] += wgt[w] * a[j];
        acc[4 + j] += wgt[w] * b[j];
      }
    }
    bf16x8 w8;
#pragma unroll
    for (int j = 0; j < 8; ++j) w8[j] = (bf16)(acc[j] * inv);
    att_store8(orow + 8 * c8, w8);
  }
}

// ---------------------------------------------------------------------------
// wide prefill path (nq > 32/G): an item is 4 waves x 32 columns = 128/G tokens. The
// 32-key K/V tiles (two 16-key pages; a page of one KV head is 4 KiB contiguous in both
// caches) are staged ONCE per workgroup into LDS by LDS-DMA and read by all 4 waves,
// double-buffered (tile t+1 lands while tile t is computed): 4x less K/V traffic per
// query column than the one-wave-per-tile path above, whose 32-column items made every
// CU pull ~4x the L2 bandwidth it has (the prefill microbenchmark ran at 160-170
// TFLOP/s, profiles/r1_attention_microbench_final.jsonl). Each wave owns its columns
// outright: no cross-wave merge; the O^T tile is transposed through LDS for 16-B stores.
// 64 KiB of LDS per workgroup (4 staged tiles): two workgroups per CU.
constexpr int PW_TILE = 16384;  // bytes per staged tile: K pb0 | K pb1 | V pb0 | V pb1

typedef __attribute__((address_space(3))) void att_lds_t;
typedef __attribute__((address_space(1))) void att_gbl_t;

constexpr int PW_NBUF = 4;     // staged tiles (3 in flight while one is computed)
template <int N>
__device__ __forceinline__ void att_wait_vm() { __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8)); }

// Split wide items: the scheduler cuts the longest causal items' key range
// into nparts partitions of whole 32-key tiles (item.z bits 8-19 = part, 20+ = nparts; item.w =
// the partition's first partial slot, 8 slots = 64 KiB of fp32 per KV head, partitions p0 + 8p).
// Each partition keeps its unnormalised O accumulators in their 32x32 register layout and the
// per-column (running max, summed denominator), stores them write-through into the uncached
// partial slab and takes a ticket; the last partition merges lane by lane (same register layout,
// no transpose) and runs the normal epilogue -- the decode path's partition hand-off
// (common.h handoff_last), with its own counter per split item (pf_counters).
constexpr int PW_PART_SLOTS = 8;

template <int G, bool SPLIT>
__device__ __forceinline__ void prefill_item_wg(
    const int4 it, char* smem, bf16* __restrict__ out, const bf16* __restrict__ q,
    const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ q_start, const int* __restrict__ q_len, const int* __restrict__ ctx_len,
    const int* __restrict__ block_table, int max_blocks, int H, int KV, int kvh, float scale_log2,
    float* __restrict__ part_o, float* __restrict__ part_ml, int* __restrict__ pf_counters, int acq) {
  constexpr int TPWV = 32 / G;  // tokens per wave
  const int s = it.x, qb = it.y, nq = it.z & 0xff;
  // without ticket room (pf_counters null) a split item computes its whole key range; SPLIT =
  // false (the engine's default, prefill_split_keys = 0) compiles the partition hand-off out --
  // it cost 8 spilled registers in every prefill item
  const int part = SPLIT && pf_counters ? (it.z >> 8) & 0xfff : 0;
  const int nparts = SPLIT && pf_counters ? max(1, it.z >> 20) : 1;
  const int pidx = it.w;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int hg = r % G, tq = wid * TPWV + r / G;
  const int ctx = ctx_len[s], ql = q_len[s], q0 = q_start[s];
  const bool colvalid = tq < nq;
  const int tok = qb + tq;
  const int key_limit = colvalid ? (ctx - ql + tok + 1) : 0;
  const int head = kvh * G + hg;
  const int wave_keys = wid * TPWV < nq ? ctx - ql + qb + min(nq, (wid + 1) * TPWV) : 0;  // wave's causal end
  const int ntiles_all = (ctx - ql + qb + nq + 31) >> 5;
  const int tpp = (ntiles_all + nparts - 1) / nparts;  // this partition: tiles [t_begin, t_begin + ntiles)
  const int t_begin = min(ntiles_all, part * tpp);
  const int ntiles = min(ntiles_all, t_begin + tpp) - t_begin;
  const int kmin = ctx - ql + qb + wid * TPWV + 1;  // smallest causal end of the wave's columns

  bf16x8 qf[8];
  {
    const bf16* qrow = q + ((size_t)(q0 + (colvalid ? tok : 0)) * H + head) * ATT_HD + 8 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + 16 * i);
      if (!colvalid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)0.f;
      }
      qf[i] = v;
    }
  }
  const int* bt = block_table + (size_t)s * max_blocks;
  const int nblk = (ctx + ATT_BLK - 1) / ATT_BLK;
  const size_t kv_stride_blk = (size_t)KV * ATT_BLK * ATT_HD;
  const int krow = swap23(r);
  // wave w stages the 1-KiB pieces 4w..4w+3 of a tile: K pb0, K pb1, V pb0, V pb1 in order
  auto stage = [&](int t, int buf) {
    const int pb0 = bt[min(2 * t, nblk - 1)], pb1 = bt[min(2 * t + 1, nblk - 1)];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = wid * 4 + i;
      // V^T pieces land with 16-B chunks c and c ^ 1 swapped where bit 4 of c is set:
      // the PV fragment reads of dims r and r + 8 then fall in different banks
      const int chunk = p < 8 ? lane : lane ^ ((lane >> 4) & 1);
      const bf16* src = (p < 8 ? k_cache : v_cache) + (size_t)(((p >> 2) & 1) ? pb1 : pb0) * kv_stride_blk +
                        (size_t)kvh * ATT_BLK * ATT_HD + (p & 3) * 512 + chunk * 8;
      __builtin_amdgcn_global_load_lds((att_gbl_t*)src, (att_lds_t*)(smem + buf * PW_TILE + p * 1024), 16, 0, 0);
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 16; ++j) o[m][j] = 0.f;
  float m_run = NEG_BIG, l_run = 0.f;

  // PW_NBUF buffers, PW_NBUF - 1 tiles in flight: a tile's DMA is issued three compute
  // phases before its use (one phase in flight left each tile ~1.5 us of L2/HBM latency
  // to wait out: the 2048-token case ran at 0.3 PFLOP/s).
#pragma unroll
  for (int p = 0; p < PW_NBUF - 1; ++p)
    if (p < ntiles) stage(t_begin + p, p);
  for (int u = 0; u < ntiles; ++u) {
    const int t = t_begin + u;
    const int buf = u % PW_NBUF;
    const int after = min(PW_NBUF - 2, ntiles - 1 - u);  // tiles issued after t, still in flight
    if (after >= 2) att_wait_vm<8>();  // this wave's pieces of tile t have landed ...
    else if (after == 1) att_wait_vm<4>();
    else att_wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... and everyone's; every wave is also done with tile t-1
    asm volatile("" ::: "memory");
    if (u + PW_NBUF - 1 < ntiles) stage(t + PW_NBUF - 1, (u + PW_NBUF - 1) % PW_NBUF);  // tile t-1's buffer
    if (32 * t >= wave_keys) continue;  // wave-uniform: beyond this wave's causal end
    const char* tb = smem + buf * PW_TILE;
    // K rows: dims 16i + 8h = chunk 2i + h; key krow & 15 of page krow >> 4
    const char* kb = tb + (krow >= 16 ? 4096 : 0) + ((h * ATT_BLK + (krow & 15)) << 4);
    bf16x8 kf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) kf[i] = *reinterpret_cast<const bf16x8*>(kb + i * 2 * ATT_BLK * 16);
    bf16x8 vf[2][4];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        vf[st][m] = *reinterpret_cast<const bf16x8*>(tb + 8192 + st * 4096 + (32 * m + r) * 32 +
                                                     16 * (h ^ ((r >> 3) & 1)));
    const f32x16 sc = qk_tile(kf, qf);
    softmax_pv_tile(sc, 32 * t + 32 > kmin, 32 * t + 8 * h, key_limit, scale_log2, m_run, l_run, o, vf);
  }
  l_run += __shfl_xor(l_run, 32, 64);
  if (SPLIT && nparts > 1) {
    // ---- partition hand-off: slab chunk j = 2 wid + (m >> 1) of the partition's 8 slots holds
    // registers o[m] of the wave's 64 lanes; (m, l) of column 32 wid + r in slot (32 wid + r) / 16
    const int p0 = pidx - PW_PART_SLOTS * part;
    auto chunk = [&](int slot0, int j) { return part_o + ((size_t)(slot0 + j) * KV + kvh) * 16 * ATT_HD; };
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(chunk(pidx, 2 * wid + (m >> 1)), 0,
                                                                          16 * ATT_HD * 4, 0x00020000);
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, f32x4{o[m][4 * c4], o[m][4 * c4 + 1], o[m][4 * c4 + 2], o[m][4 * c4 + 3]}), ps,
            ((((m & 1) * 64 + lane) * 16) + 4 * c4) * 4, 0, 16);
    }
    const int pcol = 32 * wid + r;
    if (h == 0) {
      const unsigned long long mlv =
          ((unsigned long long)__float_as_uint(l_run) << 32) | (unsigned long long)__float_as_uint(m_run);
      __hip_atomic_store((gu64*)(part_ml + ((size_t)(pidx + pcol / 16) * KV + kvh) * 32 + (pcol % 16) * 2), mlv,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int* lflag = reinterpret_cast<int*>(smem + PW_NBUF * PW_TILE);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(pf_counters + (size_t)p0 * KV + kvh, nparts, lflag, acq)) return;
    // ---- the last partition: merge every partition lane by lane (sc1 loads, after the acquire)
    float gm = NEG_BIG;
    for (int p = 0; p < nparts; ++p) {
      const unsigned long long v = __hip_atomic_load(
          (gu64*)(part_ml + ((size_t)(p0 + PW_PART_SLOTS * p + pcol / 16) * KV + kvh) * 32 + (pcol % 16) * 2),
          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      gm = fmaxf(gm, __uint_as_float((unsigned)v));
    }
    float GL = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] = f32x16{};
    for (int p = 0; p < nparts; ++p) {
      const int sp = p0 + PW_PART_SLOTS * p;
      const unsigned long long v = __hip_atomic_load(
          (gu64*)(part_ml + ((size_t)(sp + pcol / 16) * KV + kvh) * 32 + (pcol % 16) * 2), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT);
      const float w = __builtin_amdgcn_exp2f(__uint_as_float((unsigned)v) - gm);
      GL += w * __uint_as_float((unsigned)(v >> 32));
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(chunk(sp, 2 * wid + (m >> 1)), 0,
                                                                            16 * ATT_HD * 4, 0x00020000);
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const f32x4 a = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((((m & 1) * 64 + lane) * 16) + 4 * c4) * 4, 0, 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) o[m][4 * c4 + e] += w * a[e];
        }
      }
    }
    l_run = GL;
  }
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;

  // transpose O^T through LDS (the tile buffers are free once every wave passed here):
  // wave image [32 columns][128 dims] bf16, 8 KiB per wave
  __syncthreads();
  char* img = smem + wid * 8192;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[m][4 * gq + j] * inv);
      *reinterpret_cast<bf16x4*>(img + (r * ATT_HD + 32 * m + 8 * gq + 4 * h) * 2) = v;
    }
  __syncthreads();
  const int ccol = lane >> 1, dhalf = (lane & 1) * 64;
  const int ctq = wid * TPWV + ccol / G, chg = ccol % G;
  if (ctq < nq) {
    bf16* orow = out + ((size_t)(q0 + qb + ctq) * H + kvh * G + chg) * ATT_HD + dhalf;
#pragma unroll
    for (int c8 = 0; c8 < 8; ++c8)
      *reinterpret_cast<bf16x8*>(orow + 8 * c8) =
          *reinterpret_cast<const bf16x8*>(img + (ccol * ATT_HD + dhalf + 8 * c8) * 2);
  }
}

// A q-split item of either width. 8-wave workgroups run no LDS-staged wide items (their 4-wave
// image layout): a wide item (128/G tokens) runs there as its 32-column sub-items.
template <int G, int NW, bool SPLIT>
__device__ __forceinline__ void prefill_any(
    const int4 it, char* smem, bf16* __restrict__ out, const bf16* __restrict__ q,
    const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ q_start, const int* __restrict__ q_len, const int* __restrict__ ctx_len,
    const int* __restrict__ block_table, int max_blocks, int H, int KV, int kvh, float scale_log2,
    float* __restrict__ part_o, float* __restrict__ part_ml, int* __restrict__ pf_counters, int acq) {
  const int nq = it.z & 0xff;
  if (nq <= 32 / G) {
    prefill_item<G, NW>(it, smem, out, q, k_cache, v_cache, q_start, q_len, ctx_len, block_table, max_blocks,
                            H, KV, kvh, scale_log2);
  } else if constexpr (NW == 4) {
    prefill_item_wg<G, SPLIT>(it, smem, out, q, k_cache, v_cache, q_start, q_len, ctx_len, block_table, max_blocks, H, KV,
                       kvh, scale_log2, part_o, part_ml, pf_counters, acq);
  } else {
    for (int sb = 0; sb < nq; sb += 32 / G) {
      const int4 sub = {it.x, it.y + sb, min(32 / G, nq - sb) | (it.z & ~0xff), it.w};
      prefill_item<G, NW>(sub, smem, out, q, k_cache, v_cache, q_start, q_len, ctx_len, block_table,
                              max_blocks, H, KV, kvh, scale_log2);
      __syncthreads();  // LDS reuse by the next sub-item
    }
  }
}

constexpr int ATT_LDS_DECODE = ATT_LDS_DECODE_BYTES + 16;  // + last-arriver flag
// 8-wave workgroups (decode-sized steps: decode and narrow prefill items only)
constexpr int ATT_LDS_BYTES8 = std::max(att_lds_decode_bytes<8>() + 16, (8 * 32 * PF_LD + 2 * 8 * 32) * 4);
constexpr int ATT_LDS_PREFILL = (4 * 32 * PF_LD + 2 * 4 * 32) * 4;
constexpr int ATT_LDS_BYTES0 = ATT_LDS_PREFILL > ATT_LDS_DECODE ? ATT_LDS_PREFILL : ATT_LDS_DECODE;
constexpr int ATT_LDS_BYTES0W = ATT_LDS_BYTES0 > PW_NBUF * PW_TILE + 16 ? ATT_LDS_BYTES0 : PW_NBUF * PW_TILE + 16;
constexpr int ATT_LDS_BYTES = ATT_LDS_BYTES0W;  // + the split items' last-arriver flag after the tiles

// One launch serves a whole ragged step: items (seq, q_begin, nq | part<<8 |
// nparts<<20, partial slot) are strided over the grid, so the shape-stable
// (graph-captured) grid can be sized to the chip rather than to the worst case.
// (Round 4 measured and removed two alternatives: a persistent work-queue launch and idle
// workgroups warming the next projection's weights into the Infinity Cache; neither paid
// end to end, BENCHMARKS.md.)
template <int G, int NW = 4, bool SPLIT = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void paged_attn_kernel(
    bf16* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml,
    int* __restrict__ counters, const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int4* __restrict__ items,
    const int* __restrict__ n_items, const int* __restrict__ part_size, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len,
    const int* __restrict__ block_table, int max_blocks, int H, int KV, float scale_log2, int acq,
    int* __restrict__ pf_counters) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TPW = 16 / G;
  const int psz_q = part_size ? part_size[0] : ATT_PART;
  // Grid (KV, slots): the KV head is the fastest-varying workgroup index, so workgroups are
  // dispatched item by item over all KV heads -- the heaviest-first item order the scheduler
  // builds holds across the heads (with the head as the slow index, head 7's heaviest items
  // were dispatched after heads 0-6's lightest) -- and the round-robin XCD assignment keeps a
  // KV head's workgroups on one XCD (KV = 8), whose L2 then holds only that head's K/V.
  // tools/attn_bench.py: the bench's 2,048-token step 54.8 -> 45.3 us, a 2,048-token prompt
  // 79.6 -> 67.3 us (profiles/r5_attention_grid_ab.jsonl).
  const int kvh = blockIdx.x;
  const int slot = blockIdx.y;
  const int nslots = gridDim.y;
  // The first item is loaded together with the item count, not after it: one dependent
  // memory round trip less before the K/V stream starts (decode steps with few rows are
  // latency-bound). In bounds: the host sizes the grid to nslots <= max_items, the
  // length of `items`.
  const int n = n_items[0];
  int4 it_next = items[min(slot, max(n - 1, 0))];
  if (slot >= n) return;  // the grid is sized for the bucket's largest item list
  const int psz = psz_q;  // decode partition (keys), per step
  for (int item = slot; item < n; item += nslots) {
    const int4 it = it_next;
    if (item + nslots < n) it_next = items[item + nslots];
    const int nq = it.z & 0xff;
    if (nq <= TPW)
      decode_item<G, NW>(it, smem, out, part_o, part_ml, counters, q, k_cache, v_cache, q_start, q_len, ctx_len,
                         block_table, max_blocks, H, KV, kvh, scale_log2, psz, acq);
    else
      prefill_any<G, NW, SPLIT>(it, smem, out, q, k_cache, v_cache, q_start, q_len, ctx_len, block_table, max_blocks, H,
                         KV, kvh, scale_log2, part_o, part_ml, pf_counters, acq);
    __syncthreads();  // LDS reuse by the next item
  }
}

}  // namespace pa

extern "C" int pa_paged_attention(void* out, float* part_o, float* part_ml, const void* q,
                                  const void* k_cache, const void* v_cache, const int* items,
                                  const int* n_items, int max_items, const int* part_size, int* counters,
                                  const int* q_start, const int* q_len, const int* ctx_len, const int* block_table,
                                  int max_blocks, int H, int KV, float scale_log2, int waves, int* pf_counters,
                                  hipStream_t st) {
  if (H % KV != 0) return -1;
  if (waves != 4 && waves != 8) return -1;
  const int G = H / KV;
  // items are strided over the grid: ~8 resident workgroups per CU over all KV heads
  const int gx = max_items < 1 ? 1 : (max_items < 2048 / KV ? max_items : (2048 / KV > 0 ? 2048 / KV : 1));
  const dim3 grid(KV, gx);
#define PA_ATT(GG)                                                                              \
  do {                                                                                          \
    if (max_items <= 0) break;                                                                  \
    if (waves == 8) {                                                                           \
      static bool attr8 = false;                                                                \
      if (!attr8) {                                                                             \
        (void)hipFuncSetAttribute((const void*)pa::paged_attn_kernel<GG, 8>,                    \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, pa::ATT_LDS_BYTES8); \
        attr8 = true;                                                                           \
      }                                                                                         \
      hipLaunchKernelGGL((pa::paged_attn_kernel<GG, 8>), grid, dim3(512), pa::ATT_LDS_BYTES8, st, \
                         (pa::bf16*)out, part_o, part_ml, counters, (const pa::bf16*)q,         \
                         (const pa::bf16*)k_cache, (const pa::bf16*)v_cache, (const int4*)items, \
                         n_items, part_size, q_start, q_len, ctx_len, block_table, max_blocks, H, \
                         KV, scale_log2, pa::g_handoff_attn, pf_counters);                      \
      break;                                                                                    \
    }                                                                                           \
    static bool attr4 = false;                                                                  \
    if (!attr4) {                                                                               \
      (void)hipFuncSetAttribute((const void*)pa::paged_attn_kernel<GG, 4, false>,               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, pa::ATT_LDS_BYTES); \
      (void)hipFuncSetAttribute((const void*)pa::paged_attn_kernel<GG, 4, true>,                \
                                hipFuncAttributeMaxDynamicSharedMemorySize, pa::ATT_LDS_BYTES); \
      attr4 = true;                                                                             \
    }                                                                                           \
    if (pf_counters)  /* ticket room for split prefill items: the SPLIT instantiation */        \
      hipLaunchKernelGGL((pa::paged_attn_kernel<GG, 4, true>), grid, dim3(256), pa::ATT_LDS_BYTES, st, \
                         (pa::bf16*)out, part_o, part_ml, counters, (const pa::bf16*)q,         \
                         (const pa::bf16*)k_cache, (const pa::bf16*)v_cache, (const int4*)items, \
                         n_items, part_size, q_start, q_len, ctx_len, block_table, max_blocks, H, \
                         KV, scale_log2, pa::g_handoff_attn, pf_counters);                      \
    else                                                                                        \
      hipLaunchKernelGGL((pa::paged_attn_kernel<GG, 4, false>), grid, dim3(256), pa::ATT_LDS_BYTES, st, \
                         (pa::bf16*)out, part_o, part_ml, counters, (const pa::bf16*)q,         \
                         (const pa::bf16*)k_cache, (const pa::bf16*)v_cache, (const int4*)items, \
                         n_items, part_size, q_start, q_len, ctx_len, block_table, max_blocks, H, \
                         KV, scale_log2, pa::g_handoff_attn, nullptr);                          \
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
