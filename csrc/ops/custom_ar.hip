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

constexpr int AR_G = 128;            // workgroups per rank (fixed: ownership must not depend on size)
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

// blockIdx.y selects the rank when several "ranks" share one launch (single-process
// test mode: rank = rank0 + blockIdx.y, ins/outs indexed by blockIdx.y).
template <int W, bool TWO>
__global__ __launch_bounds__(AR_THREADS) void ar_kernel(ArPeers P, ArIO io, int rank0, long long nvec,
                                                         long long cap_vec, uint32_t* epochs, int* err) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int rank = rank0 + blockIdx.y;
  const u32x4* in = io.in[blockIdx.y];
  u32x4* out = io.out[blockIdx.y];
  uint32_t* ep_slot = epochs + blockIdx.y * AR_G + b;
  const uint32_t ep = *ep_slot + 1;
  const long long par_off = (long long)(ep & 1) * cap_vec;
  const long long nchunk = (nvec + AR_VPB - 1) / AR_VPB;
  auto data = [&](int r) {
    return reinterpret_cast<u32x4*>(P.base[r] + AR_FLAG_BYTES) + par_off;
  };

  // 1) stage this rank's input into its own (uncached) buffer
  u32x4* mine = data(rank);
  for (long long c = b; c < nchunk; c += AR_G) {
    const long long v = c * AR_VPB + t;
    if (v < nvec) __builtin_nontemporal_store(in[v], mine + v);
  }
  ar_stores_done();
  __syncthreads();
  ar_signal_wait(P, rank, W, b, 0, ep, err);

  if (!TWO) {
    // 2) one-shot: every rank sums all W buffers for the chunks this workgroup owns
    for (long long c = b; c < nchunk; c += AR_G) {
      const long long v = c * AR_VPB + t;
      if (v >= nvec) continue;
      u32x4 x[W];
#pragma unroll
      for (int r = 0; r < W; ++r) x[r] = __builtin_nontemporal_load(data(r) + v);
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < W; ++r) acc8(a, x[r]);  // rank order on every rank: bit-identical results
      out[v] = pack8(a);
    }
  } else {
    // 2a) reduce-scatter: reduce the chunks this rank owns, write the sum back in place
    long long j = 0;
    for (long long c = b; c < nchunk; c += AR_G, ++j) {
      if ((int)(j % W) != rank) continue;
      const long long v = c * AR_VPB + t;
      if (v >= nvec) continue;
      u32x4 x[W];
#pragma unroll
      for (int r = 0; r < W; ++r) x[r] = __builtin_nontemporal_load(data(r) + v);
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < W; ++r) acc8(a, x[r]);
      const u32x4 s = pack8(a);
      __builtin_nontemporal_store(s, mine + v);
      out[v] = s;
    }
    ar_stores_done();
    __syncthreads();
    ar_signal_wait(P, rank, W, b, 1, ep, err);
    // 2b) all-gather: copy every other rank's reduced chunks
    j = 0;
    for (long long c = b; c < nchunk; c += AR_G, ++j) {
      const int owner = (int)(j % W);
      if (owner == rank) continue;
      const long long v = c * AR_VPB + t;
      if (v < nvec) out[v] = __builtin_nontemporal_load(data(owner) + v);
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
int pa_car_all_reduce(void* const* bases, int W, int rank0, int nranks_local, const void* const* ins,
                      void* const* outs, long long nelem, long long cap_bytes, uint32_t* epochs, int* err,
                      int two_shot, hipStream_t st) {
  if (W < 2 || W > AR_MAXW || nelem % 8 || nelem * 2 > cap_bytes || nranks_local < 1 ||
      rank0 + nranks_local > W)
    return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAXW; ++i) P.base[i] = i < W ? (char*)bases[i] : nullptr;
  const long long nvec = nelem / 8, cap_vec = cap_bytes / 16;
  dim3 grid(AR_G, nranks_local);
  ArIO io;
  for (int i = 0; i < AR_MAXW; ++i) {
    io.in[i] = i < nranks_local ? (const u32x4*)ins[i] : nullptr;
    io.out[i] = i < nranks_local ? (u32x4*)outs[i] : nullptr;
  }
#define AR_LAUNCH(WW)                                                                                      \
  case WW:                                                                                                 \
    if (two_shot)                                                                                          \
      hipLaunchKernelGGL((ar_kernel<WW, true>), grid, dim3(AR_THREADS), 0, st, P, io, rank0, nvec,  \
                         cap_vec, epochs, err);                                                            \
    else                                                                                                   \
      hipLaunchKernelGGL((ar_kernel<WW, false>), grid, dim3(AR_THREADS), 0, st, P, io, rank0, nvec, \
                         cap_vec, epochs, err);                                                            \
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
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
