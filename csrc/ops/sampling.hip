// Token sampling with grammar masks.
//
// Temperature sampling uses the Gumbel-max identity
//     argmax_i (logit_i / T + G_i),  G_i = -log(-log(U_i))   ~  softmax(logit / T)
// so one streaming pass over the vocabulary replaces softmax + cumsum + search,
// and the vocabulary can be split over many workgroups (a 128K-entry row is
// 32 workgroups of 4096 entries; a decode batch of 64 rows fills 2048 WGs).
// T == 0 selects greedy argmax. top-k / top-p truncation is a per-row logit
// threshold tau computed exactly by topkp_threshold_kernel (radix select on the
// bf16 order key, below); the sampler then keeps logit >= tau, and Gumbel-max
// over the kept set samples the renormalised truncated distribution.
// U_i comes from a counter-based hash of (row seed, row offset, vocab index),
// so a request samples the same token regardless of how it was batched, and the
// vocab-parallel (TP) variant produces the identical token after an all-gather
// of the per-shard winners.
// The JSON grammar is applied as a per-row mask class: bit i of
// class_masks[class][i/32] says whether token i may follow; a row may instead be
// forced to one token (structural JSON text), which skips the stochastic part.
#include "common.h"

namespace pa {

constexpr int SMP_CHUNK = 4096;  // vocab entries per workgroup (256 threads x 16)

struct KeyIdx {
  float k;
  int i;
};

__device__ __forceinline__ KeyIdx better(KeyIdx a, KeyIdx b) {
  // larger key wins; ties -> smaller index (deterministic)
  if (b.k > a.k || (b.k == a.k && b.i < a.i)) return b;
  return a;
}

__global__ __launch_bounds__(256) void sample_chunk_kernel(
    float* __restrict__ part_k, int* __restrict__ part_i, const bf16* __restrict__ logits,
    int V, int ld, int vocab_offset, const float* __restrict__ temperature,
    const int* __restrict__ mask_class, const uint32_t* __restrict__ class_masks, int mask_words,
    const int64_t* __restrict__ seeds, const int* __restrict__ offsets, int nchunk,
    const float* __restrict__ tau) {
  const int row = blockIdx.y, chunk = blockIdx.x;
  const float T = temperature[row];
  const float thr = tau ? tau[row] : -INFINITY;
  const bool greedy = T <= 0.f;
  const float invT = greedy ? 1.f : 1.f / T;
  const int mc = mask_class[row];
  const uint64_t seed = (uint64_t)seeds[row];
  const uint32_t off = (uint32_t)offsets[row];
  const bf16* lr = logits + (size_t)row * ld;
  KeyIdx best{-INFINITY, 0x7fffffff};
  const int base = chunk * SMP_CHUNK + threadIdx.x * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i0 = base + h * 2048;
    if (i0 >= V) break;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(lr + i0);
    uint32_t bits = 0xffffffffu;
    if (mc >= 0) {
      const int gi = vocab_offset + i0;  // global vocab index (TP shards)
      bits = class_masks[(size_t)mc * mask_words + (gi >> 5)] >> (gi & 31);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + j;
      if (i >= V || !((bits >> j) & 1u)) continue;
      const float lv = bf2f(v[j]);
      if (lv < thr) continue;
      float key = lv * invT;
      if (!greedy) {
        const float u = uniform01(seed, off, (uint32_t)(vocab_offset + i));
        key += -__logf(-__logf(u));
      }
      best = better(best, KeyIdx{key, vocab_offset + i});
    }
  }
  // wave reduce
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    KeyIdx other{__shfl_xor(best.k, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, other);
  }
  __shared__ float sk[4];
  __shared__ int si[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sk[wid] = best.k;
    si[wid] = best.i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    KeyIdx b{sk[0], si[0]};
#pragma unroll
    for (int w = 1; w < 4; ++w) b = better(b, KeyIdx{sk[w], si[w]});
    part_k[row * nchunk + chunk] = b.k;
    part_i[row * nchunk + chunk] = b.i;
  }
}

__global__ __launch_bounds__(64) void sample_final_kernel(int* __restrict__ out_tokens,
                                                          float* __restrict__ out_keys,
                                                          const float* __restrict__ part_k,
                                                          const int* __restrict__ part_i,
                                                          const int* __restrict__ forced,
                                                          int nchunk) {
  const int row = blockIdx.x;
  KeyIdx best{-INFINITY, 0x7fffffff};
  for (int c = threadIdx.x; c < nchunk; c += 64)
    best = better(best, KeyIdx{part_k[row * nchunk + c], part_i[row * nchunk + c]});
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    KeyIdx other{__shfl_xor(best.k, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, other);
  }
  if (threadIdx.x == 0) {
    const int f = forced ? forced[row] : -1;
    out_tokens[row] = f >= 0 ? f : (best.i == 0x7fffffff ? 0 : best.i);
    if (out_keys) out_keys[row] = best.k;
  }
}

// ---------------------------------------------------------------------------
// top-k / top-p threshold. One 1024-thread workgroup per row; the row is read
// from L2 once per pass (4 passes). bf16 values map to a monotone 16-bit order
// key; the threshold key is found byte by byte from 256-bin histograms of
// (count, softmax mass at the row's temperature) in LDS, so the kept set is
// exactly {allowed i : logit_i >= tau} with
//   top-k: the k-th largest allowed logit, top-p: the smallest top set whose
//   mass reaches p (ties at the boundary value are kept), tau = the larger.
// The logits may be a TP all-gather: `shards` slices of V/shards columns
// each, `shard_stride` elements apart.
__device__ __forceinline__ uint32_t bf16_order_key(uint16_t b) {
  return (b & 0x8000u) ? (~(uint32_t)b & 0xffffu) : ((uint32_t)b | 0x8000u);
}
__device__ __forceinline__ float order_key_value(uint32_t k) {
  const uint16_t b = (k & 0x8000u) ? (uint16_t)(k & 0x7fffu) : (uint16_t)(~k & 0xffffu);
  return __uint_as_float((uint32_t)b << 16);
}

constexpr int TKP_THREADS = 1024;

__global__ __launch_bounds__(TKP_THREADS) void topkp_threshold_kernel(
    float* __restrict__ tau, const uint16_t* __restrict__ logits, int V, int ld, int shards,
    size_t shard_stride, const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const int* __restrict__ mask_class,
    const uint32_t* __restrict__ class_masks, int mask_words) {
  const int row = blockIdx.x;
  const int k = top_k[row];
  const float p = top_p[row];
  const float T = temperature[row];
  if (T <= 0.f || ((k <= 0 || k >= V) && !(p < 1.f))) {  // nothing to truncate
    if (threadIdx.x == 0) tau[row] = -INFINITY;
    return;
  }
  const int vs = V / shards;
  const int mc = mask_class[row];
  const float invT_log2 = 1.4426950408889634f / T;
  __shared__ float s_cnt[256], s_mass[256];
  __shared__ float red[TKP_THREADS / 64];
  __shared__ uint32_t s_sel[2];
  __shared__ float s_carry[2];
  auto value_at = [&](int g, uint32_t* key) -> bool {
    if (mc >= 0 && !((class_masks[(size_t)mc * mask_words + (g >> 5)] >> (g & 31)) & 1u)) return false;
    const int sh = g / vs, li = g - sh * vs;
    *key = bf16_order_key(logits[sh * shard_stride + (size_t)row * ld + li]);
    return true;
  };
  // pass 1: max allowed logit
  float mx = -INFINITY;
  for (int g = threadIdx.x; g < V; g += TKP_THREADS) {
    uint32_t kk;
    if (value_at(g, &kk)) mx = fmaxf(mx, order_key_value(kk));
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int w = 1; w < TKP_THREADS / 64; ++w) mx = fmaxf(mx, red[w]);
  if (mx == -INFINITY) {  // no allowed token: leave the row to the sampler's fallback
    if (threadIdx.x == 0) tau[row] = -INFINITY;
    return;
  }
  // passes 2/3: histogram of the high byte, then of the low byte inside the
  // selected high bin; each followed by a top-down scan of the 256 bins
  uint32_t prefix = 0;
  float above_cnt = 0.f, above_mass = 0.f, total_mass = 0.f;
  for (int level = 0; level < 2; ++level) {
    if (threadIdx.x < 256) { s_cnt[threadIdx.x] = 0.f; s_mass[threadIdx.x] = 0.f; }
    __syncthreads();
    for (int g = threadIdx.x; g < V; g += TKP_THREADS) {
      uint32_t kk;
      if (!value_at(g, &kk)) continue;
      if (level == 1 && (kk >> 8) != prefix) continue;
      const int bin = level == 0 ? (int)(kk >> 8) : (int)(kk & 0xff);
      atomicAdd(&s_cnt[bin], 1.f);
      atomicAdd(&s_mass[bin], exp2f((order_key_value(kk) - mx) * invT_log2));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (level == 0) {
        for (int b = 0; b < 256; ++b) total_mass += s_mass[b];
        s_carry[0] = total_mass;
      }
      const float tm = level == 0 ? total_mass : s_carry[0];
      const float need_mass = p < 1.f ? p * tm : INFINITY;
      const float need_cnt = (k > 0 && k < V) ? (float)k : INFINITY;
      float c = above_cnt, m = above_mass;
      int sel = 0;
      for (int b = 255; b >= 0; --b) {
        const float c2 = c + s_cnt[b], m2 = m + s_mass[b];
        if (c2 >= need_cnt || m2 >= need_mass) { sel = b; break; }
        c = c2; m = m2;
        sel = b;
      }
      s_sel[0] = (uint32_t)sel;
      s_carry[1] = c;  // count strictly above the selected bin
      red[0] = m;      // mass strictly above the selected bin
    }
    __syncthreads();
    const uint32_t sel = s_sel[0];
    above_cnt = s_carry[1];
    above_mass = red[0];
    prefix = level == 0 ? sel : ((prefix << 8) | sel);
    __syncthreads();
  }
  if (threadIdx.x == 0) tau[row] = order_key_value(prefix);
}

// ---------------------------------------------------------------------------
// The same threshold for a vocab-parallel LM head (TP > 1) without gathering the logits: each
// rank runs the passes on its own V/tp slice and the group combines the partial results
// between them with the custom P2P collectives (parallel/custom_ar.py; no RCCL in the step
// graph). Histograms ADD across shards, maxima MAX, so every rank ends with the tau the
// single-GPU kernel computes on the whole row:
//   phase 0  mx[row]            = max allowed logit of the slice         -> MAX over ranks
//   phase 1  h0[row][0:256/256:512] = (count, mass) per high byte         -> SUM over ranks
//   phase 2  scan h0 (identical on every rank) -> st[row] = (hi, count / mass above hi, total);
//            h1[row] = (count, mass) per low byte inside bin hi          -> SUM over ranks
//   phase 3  scan h1 with the carries -> tau[row]
// mass = exp2((logit - mx) * log2(e) / T) of the allowed tokens (as the single-GPU kernel).
struct TkpArgs {
  const uint16_t* logits;  // [rows, ld] this rank's slice (v_local valid columns)
  int v_local, ld, vocab_offset, V;
  const float* temperature;
  const int* top_k;
  const float* top_p;
  const int* mask_class;
  const uint32_t* class_masks;
  int mask_words;
  float* mx;   // [rows]
  float* h0;   // [rows, 512]
  float* h1;   // [rows, 512]
  float* st;   // [rows, 4]
  float* tau;  // [rows]
};

__device__ __forceinline__ bool tkp_active(const TkpArgs& A, int row) {
  const int k = A.top_k[row];
  const float p = A.top_p[row];
  return A.temperature[row] > 0.f && !((k <= 0 || k >= A.V) && !(p < 1.f));
}

// top-down scan of 256 (count, mass) bins (thread 0): the highest bin where the count or the
// mass from the top reaches its need (bin 0 if none), and the count / mass strictly above it
__device__ __forceinline__ int tkp_scan(const float* cnt, const float* mass, float need_cnt, float need_mass,
                                        float* c_io, float* m_io) {
  float c = *c_io, m = *m_io;
  int sel = 0;
  for (int b = 255; b >= 0; --b) {
    const float c2 = c + cnt[b], m2 = m + mass[b];
    if (c2 >= need_cnt || m2 >= need_mass) { sel = b; break; }
    c = c2; m = m2;
    sel = b;
  }
  *c_io = c;
  *m_io = m;
  return sel;
}

template <int PHASE>
__global__ __launch_bounds__(TKP_THREADS) void tp_topkp_kernel(const TkpArgs A) {
  const int row = blockIdx.x;
  const bool act = tkp_active(A, row);
  const int mc = A.mask_class[row];
  const uint16_t* lr = A.logits + (size_t)row * A.ld;
  auto allowed = [&](int li) -> bool {
    if (mc < 0) return true;
    const int g = A.vocab_offset + li;
    return (A.class_masks[(size_t)mc * A.mask_words + (g >> 5)] >> (g & 31)) & 1u;
  };
  __shared__ float s_cnt[256], s_mass[256];
  __shared__ float red[TKP_THREADS / 64];
  if constexpr (PHASE == 0) {
    float m = -INFINITY;
    if (act)
      for (int li = threadIdx.x; li < A.v_local; li += TKP_THREADS)
        if (allowed(li)) m = fmaxf(m, order_key_value(bf16_order_key(lr[li])));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      float r = red[0];
      for (int w = 1; w < TKP_THREADS / 64; ++w) r = fmaxf(r, red[w]);
      A.mx[row] = r;
    }
    return;
  }
  if constexpr (PHASE == 3) {
    if (threadIdx.x == 0) {
      const float* st = A.st + (size_t)row * 4;
      float tau = -INFINITY;
      if (act && A.mx[row] > -INFINITY) {
        const int k = A.top_k[row];
        const float p = A.top_p[row];
        const float need_mass = p < 1.f ? p * st[3] : INFINITY;
        const float need_cnt = (k > 0 && k < A.V) ? (float)k : INFINITY;
        float c = st[1], m = st[2];
        const float* h = A.h1 + (size_t)row * 512;
        const int lo = tkp_scan(h, h + 256, need_cnt, need_mass, &c, &m);
        tau = order_key_value(((uint32_t)st[0] << 8) | (uint32_t)lo);
      }
      A.tau[row] = tau;
    }
    return;
  }
  // phases 1 and 2: a histogram of this slice
  if (threadIdx.x < 256) { s_cnt[threadIdx.x] = 0.f; s_mass[threadIdx.x] = 0.f; }
  __shared__ int s_hi;
  const float mx = A.mx[row];
  const bool live = act && mx > -INFINITY;
  if constexpr (PHASE == 2) {
    if (threadIdx.x == 0) {
      int hi = 0;
      float c = 0.f, m = 0.f, total = 0.f;
      if (live) {
        const float* h = A.h0 + (size_t)row * 512;
        for (int b = 0; b < 256; ++b) total += h[256 + b];
        const int k = A.top_k[row];
        const float p = A.top_p[row];
        const float need_mass = p < 1.f ? p * total : INFINITY;
        const float need_cnt = (k > 0 && k < A.V) ? (float)k : INFINITY;
        hi = tkp_scan(h, h + 256, need_cnt, need_mass, &c, &m);
      }
      float* st = A.st + (size_t)row * 4;
      st[0] = (float)hi;
      st[1] = c;
      st[2] = m;
      st[3] = total;
      s_hi = hi;
    }
  }
  __syncthreads();
  if (live) {
    const float invT_log2 = 1.4426950408889634f / A.temperature[row];
    const int hi = PHASE == 2 ? s_hi : -1;
    for (int li = threadIdx.x; li < A.v_local; li += TKP_THREADS) {
      if (!allowed(li)) continue;
      const uint32_t kk = bf16_order_key(lr[li]);
      if (PHASE == 2 && (int)(kk >> 8) != hi) continue;
      const int bin = PHASE == 1 ? (int)(kk >> 8) : (int)(kk & 0xff);
      atomicAdd(&s_cnt[bin], 1.f);
      atomicAdd(&s_mass[bin], exp2f((order_key_value(kk) - mx) * invT_log2));
    }
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    float* h = (PHASE == 1 ? A.h0 : A.h1) + (size_t)row * 512;
    h[threadIdx.x] = s_cnt[threadIdx.x];
    h[256 + threadIdx.x] = s_mass[threadIdx.x];
  }
}

}  // namespace pa

// TP top-k / top-p threshold, one phase per call (the caller combines mx / h0 / h1 over the TP
// group between phases). ws: [ceil4(rows) + rows * 1028] floats: mx | h0 | h1 | st.
extern "C" int pa_tp_topkp_phase(int phase, float* tau, float* ws, const void* logits, int rows, int v_local,
                                 int ld, int vocab_offset, int V, const float* temperature, const int* top_k,
                                 const float* top_p, const int* mask_class, const uint32_t* class_masks,
                                 int mask_words, hipStream_t st) {
  if (rows <= 0) return 0;
  if (phase < 0 || phase > 3 || v_local <= 0 || ld < v_local) return -1;
  // mx is padded to a multiple of 4 rows, so every segment the TP group reduces starts 16-byte
  // aligned and holds a multiple of 4 floats (the custom collectives move 16-byte vectors)
  const size_t r4 = ((size_t)rows + 3) & ~(size_t)3;
  pa::TkpArgs a{(const uint16_t*)logits, v_local, ld, vocab_offset, V, temperature, top_k, top_p, mask_class,
                class_masks, mask_words, ws, ws + r4, ws + r4 + (size_t)rows * 512, ws + r4 + (size_t)rows * 1024,
                tau};
  switch (phase) {
    case 0: hipLaunchKernelGGL(pa::tp_topkp_kernel<0>, dim3(rows), dim3(pa::TKP_THREADS), 0, st, a); break;
    case 1: hipLaunchKernelGGL(pa::tp_topkp_kernel<1>, dim3(rows), dim3(pa::TKP_THREADS), 0, st, a); break;
    case 2: hipLaunchKernelGGL(pa::tp_topkp_kernel<2>, dim3(rows), dim3(pa::TKP_THREADS), 0, st, a); break;
    default: hipLaunchKernelGGL(pa::tp_topkp_kernel<3>, dim3(rows), dim3(pa::TKP_THREADS), 0, st, a); break;
  }
  return (int)hipGetLastError();
}

extern "C" int pa_topkp_threshold(float* tau, const void* logits, int rows, int V, int ld, int shards,
                                  long long shard_stride, const float* temperature, const int* top_k,
                                  const float* top_p, const int* mask_class, const uint32_t* class_masks,
                                  int mask_words, hipStream_t st) {
  if (rows <= 0) return 0;
  if (shards <= 0 || V % shards != 0) return -1;
  hipLaunchKernelGGL(pa::topkp_threshold_kernel, dim3(rows), dim3(pa::TKP_THREADS), 0, st, tau,
                     (const uint16_t*)logits, V, ld, shards, (size_t)shard_stride, temperature, top_k,
                     top_p, mask_class, class_masks, mask_words);
  return (int)hipGetLastError();
}

extern "C" int pa_sample_workspace_floats(int rows, int V) {
  const int nchunk = (V + pa::SMP_CHUNK - 1) / pa::SMP_CHUNK;
  return rows * nchunk * 2;
}

// workspace: float[rows * nchunk] keys followed by int[rows * nchunk] indices.
// out_keys (optional) receives the winning perturbed key per row, used by the
// tensor-parallel sampler to pick the global winner across vocab shards.
extern "C" int pa_sample(int* out_tokens, float* out_keys, float* workspace, const void* logits,
                         int rows, int V, int ld, int vocab_offset, const float* temperature,
                         const int* mask_class, const uint32_t* class_masks, int mask_words,
                         const int64_t* seeds, const int* offsets, const int* forced,
                         const float* tau, hipStream_t st) {
  if (rows <= 0) return 0;
  if (V % 8 != 0 || ld % 8 != 0) return -1;
  const int nchunk = (V + pa::SMP_CHUNK - 1) / pa::SMP_CHUNK;
  float* pk = workspace;
  int* pi = reinterpret_cast<int*>(workspace + (size_t)rows * nchunk);
  hipLaunchKernelGGL(pa::sample_chunk_kernel, dim3(nchunk, rows), dim3(256), 0, st, pk, pi,
                     (const pa::bf16*)logits, V, ld, vocab_offset, temperature, mask_class,
                     class_masks, mask_words, seeds, offsets, nchunk, tau);
  hipLaunchKernelGGL(pa::sample_final_kernel, dim3(rows), dim3(64), 0, st, out_tokens, out_keys,
                     pk, pi, forced, nchunk);
  return (int)hipGetLastError();
}

// Pipelined engine steps (engine.py, async_steps): a row whose previous token is still
// being sampled by the step in flight enters the next step with input id -(r + 1), r =
// its sampling row there. This runs first in the next step's graph, after the previous
// step's sampler (same stream), and replaces each such id by the sampled token.
namespace pa {
__global__ __launch_bounds__(256) void patch_pending_ids_kernel(int* __restrict__ ids,
                                                                const int* __restrict__ sampled, int T,
                                                                int n_sampled) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  const int v = ids[t];
  if (v < 0) {
    const int r = -v - 1;
    ids[t] = r < n_sampled ? sampled[r] : 0;
  }
}
}  // namespace pa

extern "C" int pa_patch_pending_ids(int* ids, const int* sampled, int T, int n_sampled, hipStream_t st) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(pa::patch_pending_ids_kernel, dim3((T + 255) / 256), dim3(256), 0, st, ids, sampled, T,
                     n_sampled);
  return (int)hipGetLastError();
}
