// Custom all-reduce over P2P IPC buffers for small/medium tensor-parallel messages
// (160 all-reduces per 70B TP=8 decode step at 16 KiB x B).
//
// Why not RCCL for these: xGMI is point-to-point (7 links per GPU). A ring moves a
// message through W-1 hops, one link per direction, so a 16-256 KiB decode message
// pays W-1 hop latencies. Here every rank reads its peers' buffers directly over
// all 7 links at once:
//
//   one-shot (<= ~512 KiB): stage local input -> own IPC buffer, signal peers, then
//            every rank reads all W buffers and sums (W-1 remote reads per element,
//            one cross-rank barrier).
//   two-shot (larger):      after staging, rank j/W reduces the 1/W share of chunks it
//            owns (reading W-1 peers) in place, signals again, then every rank gathers
//            each reduced chunk from its owner: 2(W-1)/W of the bytes over the links
//            instead of (W-1), for one more barrier.
//
// Buffer of each rank (hipExtMallocWithFlags(..., hipDeviceMallocUncached), exported
// by hipIpcGetMemHandle and opened by every peer):
//   [flags1: AR_G x 8 u32][flags2: AR_G x 8 u32] (padded to AR_FLAG_BYTES)
//   [data parity 0: cap bytes][data parity 1: cap bytes]
//
// Ownership is fixed per workgroup, independent of the message size: 16-byte
// vector v belongs to chunk c = v / AR_VPB, chunk c to workgroup c % AR_G (and, in
// two-shot, to rank (c / AR_G) % W). Workgroup b of every rank therefore touches
// only its own chunks, and the cross-rank barriers are per workgroup (flag slot
// [b][src]). Each workgroup keeps a private epoch counter in device memory, so the
// launch has no per-call arguments and captures into a hipGraph. Calls alternate
// between the two data parities: a rank can only reuse a parity after passing the
// next call's barrier, which every peer reaches only after finishing its reads of
// this one — so no trailing barrier is needed.
//
// Every spin-wait is bounded (AR_TIMEOUT_TICKS of the 100 MHz wall clock): a lost
// peer sets `err` and the grid still drains instead of hanging the GPU.
#include "common.h"

namespace pa {

constexpr int AR_G = 128;            // workgroups per rank: flag / epoch slots (ownership must not depend on size)
// Workgroups actually launched per rank: AR_G, or PILOTTAI_CAR_WG (1..AR_G, the same on every rank
// of a group: chunk c belongs to workgroup c % G). A share-GPU rehearsal of TP=4/8 lowers it: each
// rank's all-reduce workgroups spin until their peers arrive, and with 3-7 peers' worth of
// spinning workgroups on the card a peer's GEMM that needs a whole CU finds none free.
static int car_wg() {
  static int g = 0;
  if (g == 0) {
    const char* e = getenv("PILOTTAI_CAR_WG");
    const int v = e ? atoi(e) : AR_G;
    g = v >= 1 && v <= AR_G ? v : AR_G;
  }
  return g;
}
constexpr int AR_THREADS = 256;      // one 16-byte vector per thread per chunk
constexpr int AR_VPB = AR_THREADS;   // vectors per chunk (4 KiB)
constexpr int AR_MAXW = 8;
constexpr long long AR_FLAG_BYTES = 65536;
constexpr unsigned long long AR_TIMEOUT_TICKS = 500000000ull;  // ~5 s at 100 MHz

struct ArPeers {
  char* base[AR_MAXW];   // every rank's buffer, mapped into this process
};

struct ArIO {            // input/output per rank handled by this launch (blockIdx.y)
  const u32x4* in[AR_MAXW];
  u32x4* out[AR_MAXW];
  // fused residual epilogue (RES): out = resid + sum(in); ss[row] += sum(out^2) over the
  // written bf16 values (the next RMSNorm's row statistics); ss_zero[0 .. nrows) <- 0 (the
  // buffer the NEXT fused all-reduce fills, consumed before this launch). resid may alias out.
  const u32x4* resid[AR_MAXW];
  float* ss[AR_MAXW];
  float* ss_zero[AR_MAXW];
  int row_vec;  // 16-byte vectors per row (hidden / 8); a 4-KiB chunk never straddles rows
  int nrows;
};

__device__ __forceinline__ uint32_t* ar_flags(char* base, int which) {
  return reinterpret_cast<uint32_t*>(base) + which * (AR_G * AR_MAXW);
}

// Wait until this thread's stores are acknowledged (gfx9: vmcnt counts stores too).
// The data and flags live in uncached memory, so an acknowledged store is visible to
// every peer; no L2 writeback/invalidate (a system-scope fence would write back and
// invalidate the whole L2 under the concurrently running GEMMs) is needed.
__device__ __forceinline__ void ar_stores_done() { __builtin_amdgcn_s_waitcnt(0); }

__device__ __forceinline__ void ar_signal_wait(const ArPeers& P, int rank, int W, int b, int which, uint32_t ep,
                                               int* err) {
  // caller: every thread ran ar_stores_done() and the workgroup passed a barrier
  const int t = threadIdx.x;
  if (t < W && t != rank) {
    uint32_t* dst = ar_flags(P.base[t], which) + b * AR_MAXW + rank;
    __hip_atomic_store(dst, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = ar_flags(P.base[rank], which) + b * AR_MAXW + t;
    const unsigned long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - ep) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > AR_TIMEOUT_TICKS) {
        atomicOr(err, 1);
        break;
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void acc8(float* a, const u32x4 v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[2 * i] += __uint_as_float(v[i] << 16);
    a[2 * i + 1] += __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* a) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = f2bf(a[i]);
  return __builtin_bit_cast(u32x4, r);
}

// sum of squares of the 8 bf16 values of v
__device__ __forceinline__ float sq8(const u32x4 v) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(v[i] << 16), hi = __uint_as_float(v[i] & 0xffff0000u);
    s = fmaf(lo, lo, fmaf(hi, hi, s));
  }
  return s;
}

// one chunk's row statistic: the workgroup's 256 vectors lie in one row (host: row_vec % 256
// == 0); every thread of the workgroup calls it (sq = 0 past the message end)
__device__ __forceinline__ void chunk_row_stat(float* ss, long long c, int row_vec, float sq, float* red) {
  sq = wave_sum(sq);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = sq;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(ss + (c * AR_VPB) / row_vec, red[0] + red[1] + red[2] + red[3]);
  __syncthreads();
}

// blockIdx.y selects the rank when several "ranks" share one launch (single-process
// test mode: rank = rank0 + blockIdx.y, ins/outs indexed by blockIdx.y).
// RES: the fused residual epilogue (ArIO.resid / ss / ss_zero): replaces the all-reduce ->
// h.add_ -> row_sumsq chain of a row-parallel projection under TP with one launch.
template <int W, bool TWO, bool RES>
__global__ __launch_bounds__(AR_THREADS) void ar_kernel(ArPeers P, ArIO io, int rank0, long long nvec,
                                                         long long cap_vec, uint32_t* epochs, int* err) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int rank = rank0 + blockIdx.y;
  const u32x4* in = io.in[blockIdx.y];
  u32x4* out = io.out[blockIdx.y];
  const u32x4* resid = io.resid[blockIdx.y];
  float* ss = io.ss[blockIdx.y];
  __shared__ float red[4];
  if (RES && b == 0 && io.ss_zero[blockIdx.y])
    for (int i = t; i < io.nrows; i += AR_THREADS) io.ss_zero[blockIdx.y][i] = 0.f;
  // out = (resid +) sum, rounded to bf16 once; returns the written vector
  auto finish = [&](float* a, long long v) -> u32x4 {
    if constexpr (RES) acc8(a, resid[v]);
    return pack8(a);
  };
  uint32_t* ep_slot = epochs + blockIdx.y * AR_G + b;
  const uint32_t ep = *ep_slot + 1;
  const long long par_off = (long long)(ep & 1) * cap_vec;
  const long long nchunk = (nvec + AR_VPB - 1) / AR_VPB;
  auto data = [&](int r) {
    return reinterpret_cast<u32x4*>(P.base[r] + AR_FLAG_BYTES) + par_off;
  };

  // 1) stage this rank's input into its own (uncached) buffer
  u32x4* mine = data(rank);
  for (long long c = b; c < nchunk; c += (long long)gridDim.x) {
    const long long v = c * AR_VPB + t;
    if (v < nvec) __builtin_nontemporal_store(in[v], mine + v);
  }
  ar_stores_done();
  __syncthreads();
  ar_signal_wait(P, rank, W, b, 0, ep, err);

  if (!TWO) {
    // 2) one-shot: every rank sums all W buffers for the chunks this workgroup owns
    for (long long c = b; c < nchunk; c += (long long)gridDim.x) {
      const long long v = c * AR_VPB + t;
      float sq = 0.f;
      if (v < nvec) {
        u32x4 x[W];
#pragma unroll
        for (int r = 0; r < W; ++r) x[r] = __builtin_nontemporal_load(data(r) + v);
        float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < W; ++r) acc8(a, x[r]);  // rank order on every rank: bit-identical results
        const u32x4 o = finish(a, v);
        out[v] = o;
        if constexpr (RES) sq = sq8(o);
      }
      if constexpr (RES) {
        if (ss) chunk_row_stat(ss, c, io.row_vec, sq, red);
      }
    }
  } else {
    // 2a) reduce-scatter: reduce the chunks this rank owns, write the sum back in place
    // (with RES the owner adds the residual: h is replicated, so h + sum is the same on every
    // rank and the gathered chunks are final)
    long long j = 0;
    for (long long c = b; c < nchunk; c += (long long)gridDim.x, ++j) {
      if ((int)(j % W) != rank) continue;
      const long long v = c * AR_VPB + t;
      float sq = 0.f;
      if (v < nvec) {
        u32x4 x[W];
#pragma unroll
        for (int r = 0; r < W; ++r) x[r] = __builtin_nontemporal_load(data(r) + v);
        float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < W; ++r) acc8(a, x[r]);
        const u32x4 s = finish(a, v);
        __builtin_nontemporal_store(s, mine + v);
        out[v] = s;
        if constexpr (RES) sq = sq8(s);
      }
      if constexpr (RES) {
        if (ss) chunk_row_stat(ss, c, io.row_vec, sq, red);
      }
    }
    ar_stores_done();
    __syncthreads();
    ar_signal_wait(P, rank, W, b, 1, ep, err);
    // 2b) all-gather: copy every other rank's reduced chunks
    j = 0;
    for (long long c = b; c < nchunk; c += (long long)gridDim.x, ++j) {
      const int owner = (int)(j % W);
      if (owner == rank) continue;
      const long long v = c * AR_VPB + t;
      float sq = 0.f;
      if (v < nvec) {
        const u32x4 o = __builtin_nontemporal_load(data(owner) + v);
        out[v] = o;
        if constexpr (RES) sq = sq8(o);
      }
      if constexpr (RES) {
        if (ss) chunk_row_stat(ss, c, io.row_vec, sq, red);
      }
    }
  }
  if (t == 0) *ep_slot = ep;
}

// ---------------------------------------------------------------------------------------
// Small collectives of the TP step graph on the same buffers, flags and epochs (VERDICT r4
// item 4: no RCCL call inside a captured graph): the sampler's all-gather of per-shard winners
// (keys, token ids) and the top-k / top-p threshold's MAX / SUM all-reduces of fp32 row maxima
// and radix histograms. One-shot: stage, one cross-rank barrier, every rank reads every
// peer's chunk. Elements are 4 bytes moved as 16-byte vectors; SUM adds in rank order, so
// every rank holds bit-identical results. Sharing the epochs with ar_kernel keeps the
// parity argument above: a workgroup's calls, of any kind, alternate parities in one order.
enum { CO_SUM_F32 = 0, CO_MAX_F32 = 1, CO_GATHER = 2 };

template <int W, int OP>
__global__ __launch_bounds__(AR_THREADS) void co_kernel(ArPeers P, ArIO io, int rank0, long long nvec,
                                                         long long cap_vec, uint32_t* epochs, int* err) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int rank = rank0 + blockIdx.y;
  const u32x4* in = io.in[blockIdx.y];
  u32x4* out = io.out[blockIdx.y];
  uint32_t* ep_slot = epochs + blockIdx.y * AR_G + b;
  const uint32_t ep = *ep_slot + 1;
  const long long par_off = (long long)(ep & 1) * cap_vec;
  const long long nchunk = (nvec + AR_VPB - 1) / AR_VPB;
  auto data = [&](int r) { return reinterpret_cast<u32x4*>(P.base[r] + AR_FLAG_BYTES) + par_off; };
  u32x4* mine = data(rank);
  for (long long c = b; c < nchunk; c += (long long)gridDim.x) {
    const long long v = c * AR_VPB + t;
    if (v < nvec) __builtin_nontemporal_store(in[v], mine + v);
  }
  ar_stores_done();
  __syncthreads();
  ar_signal_wait(P, rank, W, b, 0, ep, err);
  for (long long c = b; c < nchunk; c += (long long)gridDim.x) {
    const long long v = c * AR_VPB + t;
    if (v >= nvec) continue;
    u32x4 x[W];
#pragma unroll
    for (int r = 0; r < W; ++r) x[r] = __builtin_nontemporal_load(data(r) + v);
    if constexpr (OP == CO_GATHER) {
#pragma unroll
      for (int r = 0; r < W; ++r) out[(long long)r * nvec + v] = x[r];
    } else {
      f32x4 a = __builtin_bit_cast(f32x4, x[0]);
#pragma unroll
      for (int r = 1; r < W; ++r) {
        const f32x4 y = __builtin_bit_cast(f32x4, x[r]);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = OP == CO_SUM_F32 ? a[i] + y[i] : fmaxf(a[i], y[i]);
      }
      out[v] = __builtin_bit_cast(u32x4, a);
    }
  }
  if (t == 0) *ep_slot = ep;
}

}  // namespace pa

using namespace pa;

extern "C" {

int pa_car_group() { return AR_G; }
long long pa_car_flag_bytes() { return AR_FLAG_BYTES; }

// Allocate an uncached, IPC-exportable buffer: returns the device pointer and
// writes the 64-byte IPC handle to `handle_out`.
void* pa_car_alloc(long long bytes, void* handle_out) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  __builtin_memcpy(handle_out, &h, sizeof(h));
  return p;
}

void* pa_car_open(const void* handle) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  return p;
}

int pa_car_close(void* p) { return hipIpcCloseMemHandle(p) == hipSuccess ? 0 : -1; }
int pa_car_free(void* p) { return hipFree(p) == hipSuccess ? 0 : -1; }

// bases: W buffer pointers (this process's mapping of every rank's buffer).
// nranks_local: ranks handled by this launch — 1 in real use; up to W in the
// single-process test, where ranks rank0.. share one launch (ins/outs per rank,
// epochs holds nranks_local x AR_G counters).
// resids / ss / ss_zero (nullable): the fused residual epilogue (ArIO); row_len = hidden size.
int pa_car_all_reduce(void* const* bases, int W, int rank0, int nranks_local, const void* const* ins,
                      void* const* outs, long long nelem, long long cap_bytes, uint32_t* epochs, int* err,
                      int two_shot, const void* const* resids, float* const* ss, float* const* ss_zero,
                      int row_len, hipStream_t st) {
  if (W < 2 || W > AR_MAXW || nelem % 8 || nelem * 2 > cap_bytes || nranks_local < 1 ||
      rank0 + nranks_local > W)
    return -1;
  const bool res = resids != nullptr;
  if (res && (row_len <= 0 || (row_len / 8) % AR_VPB || row_len % 8 || nelem % row_len)) return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAXW; ++i) P.base[i] = i < W ? (char*)bases[i] : nullptr;
  const long long nvec = nelem / 8, cap_vec = cap_bytes / 16;
  dim3 grid(car_wg(), nranks_local);
  ArIO io;
  for (int i = 0; i < AR_MAXW; ++i) {
    const bool on = i < nranks_local;
    io.in[i] = on ? (const u32x4*)ins[i] : nullptr;
    io.out[i] = on ? (u32x4*)outs[i] : nullptr;
    io.resid[i] = on && res ? (const u32x4*)resids[i] : nullptr;
    io.ss[i] = on && res && ss ? ss[i] : nullptr;
    io.ss_zero[i] = on && res && ss_zero ? ss_zero[i] : nullptr;
  }
  io.row_vec = res ? row_len / 8 : 0;
  io.nrows = res ? (int)(nelem / row_len) : 0;
#define AR_KERN(WW, TT, RR) \
  hipLaunchKernelGGL((ar_kernel<WW, TT, RR>), grid, dim3(AR_THREADS), 0, st, P, io, rank0, nvec, cap_vec, epochs, err)
#define AR_LAUNCH(WW)                        \
  case WW:                                   \
    if (two_shot) {                          \
      if (res) AR_KERN(WW, true, true);      \
      else AR_KERN(WW, true, false);         \
    } else {                                 \
      if (res) AR_KERN(WW, false, true);     \
      else AR_KERN(WW, false, false);        \
    }                                        \
    break;
  switch (W) {
    AR_LAUNCH(2)
    AR_LAUNCH(3)
    AR_LAUNCH(4)
    AR_LAUNCH(5)
    AR_LAUNCH(6)
    AR_LAUNCH(7)
    AR_LAUNCH(8)
    default:
      return -1;
  }
#undef AR_LAUNCH
#undef AR_KERN
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Small collectives (co_kernel): n4 4-byte elements per rank (a multiple of 4), op CO_*; for
// CO_GATHER outs[i] receives W x n4 elements (rank-major). Same buffers / epochs / err as
// pa_car_all_reduce, so the two kinds of call may be interleaved in any order every rank shares.
int pa_car_collective(void* const* bases, int W, int rank0, int nranks_local, const void* const* ins,
                      void* const* outs, long long n4, long long cap_bytes, uint32_t* epochs, int* err, int op,
                      hipStream_t st) {
  if (W < 2 || W > AR_MAXW || n4 <= 0 || n4 % 4 || n4 * 4 > cap_bytes || nranks_local < 1 ||
      rank0 + nranks_local > W || op < CO_SUM_F32 || op > CO_GATHER)
    return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAXW; ++i) P.base[i] = i < W ? (char*)bases[i] : nullptr;
  ArIO io{};
  for (int i = 0; i < AR_MAXW; ++i) {
    const bool on = i < nranks_local;
    io.in[i] = on ? (const u32x4*)ins[i] : nullptr;
    io.out[i] = on ? (u32x4*)outs[i] : nullptr;
  }
  const long long nvec = n4 / 4, cap_vec = cap_bytes / 16;
  dim3 grid(car_wg(), nranks_local);
#define CO_KERN(WW, OO) \
  hipLaunchKernelGGL((co_kernel<WW, OO>), grid, dim3(AR_THREADS), 0, st, P, io, rank0, nvec, cap_vec, epochs, err)
#define CO_LAUNCH(WW)                                  \
  case WW:                                             \
    if (op == CO_SUM_F32) CO_KERN(WW, CO_SUM_F32);     \
    else if (op == CO_MAX_F32) CO_KERN(WW, CO_MAX_F32); \
    else CO_KERN(WW, CO_GATHER);                       \
    break;
  switch (W) {
    CO_LAUNCH(2)
    CO_LAUNCH(3)
    CO_LAUNCH(4)
    CO_LAUNCH(5)
    CO_LAUNCH(6)
    CO_LAUNCH(7)
    CO_LAUNCH(8)
    default:
      return -1;
  }
#undef CO_LAUNCH
#undef CO_KERN
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
