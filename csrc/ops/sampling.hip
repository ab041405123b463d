// Token sampling with grammar masks.
//
// Temperature sampling uses the Gumbel-max identity
//     argmax_i (logit_i / T + G_i),  G_i = -log(-log(U_i))   ~  softmax(logit / T)
// so one streaming pass over the vocabulary replaces softmax + cumsum + search,
// and the vocabulary can be split over many workgroups (a 128K-entry row is
// 32 workgroups of 4096 entries; a decode batch of 64 rows fills 2048 WGs).
// T == 0 selects greedy argmax. top-k (k <= 64) runs a per-row threshold search
// on the chunk winners' candidate lists (see topk pass below).
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
    const int64_t* __restrict__ seeds, const int* __restrict__ offsets, int nchunk) {
  const int row = blockIdx.y, chunk = blockIdx.x;
  const float T = temperature[row];
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
      float key = bf2f(v[j]) * invT;
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

}  // namespace pa

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
                         hipStream_t st) {
  if (rows <= 0) return 0;
  if (V % 8 != 0 || ld % 8 != 0) return -1;
  const int nchunk = (V + pa::SMP_CHUNK - 1) / pa::SMP_CHUNK;
  float* pk = workspace;
  int* pi = reinterpret_cast<int*>(workspace + (size_t)rows * nchunk);
  hipLaunchKernelGGL(pa::sample_chunk_kernel, dim3(nchunk, rows), dim3(256), 0, st, pk, pi,
                     (const pa::bf16*)logits, V, ld, vocab_offset, temperature, mask_class,
                     class_masks, mask_words, seeds, offsets, nchunk);
  hipLaunchKernelGGL(pa::sample_final_kernel, dim3(rows), dim3(64), 0, st, out_tokens, out_keys,
                     pk, pi, forced, nchunk);
  return (int)hipGetLastError();
}
