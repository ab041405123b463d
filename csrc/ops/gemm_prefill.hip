// Large-M projections (prefill-heavy steps, M > 256 tokens) on the packed weights
// (replaces hipBLASLt + rmsnorm + silu_mul + rope_cache on those steps).
//
//     y[M, N] = epi( rownorm(x)[M, K] · W[N, K]^T )      bf16 in/out, fp32 accumulate
//
// At 64 concurrent agents most engine time sits in 512-2,048-token steps (prefill chunks
// beside the decode rows). Their projections are compute-bound: 2·M·N·K FLOPs on MFMA.
// The kernel is the CDNA4 256x256 tile of cdna_hip_programming.md §5, built around the
// operands this engine already has in memory:
//
//   * 512 threads = 8 waves as 2 (rows) x 4 (columns); a wave owns 128 x 64 outputs
//     (8 x 4 tiles of v_mfma_f32_16x16x32_bf16, 128 accumulator VGPRs). The MFMA runs as
//     C^T = W · x^T, so each lane ends with 4 consecutive output columns of one token:
//     the norm / SwiGLU / residual / RoPE + KV-write epilogues of packed_epi.h run on
//     registers (no separate rmsnorm / silu_mul / rope_cache launches);
//   * W is the fragment-major packed copy (ops.pack_decode_weight): a 16-column x 32-k
//     chunk is 1 KiB contiguous, so one global_load_lds wave instruction moves one chunk
//     and the LDS image is lane-linear and conflict-free for the B-fragment ds_read_b128;
//   * x rows are staged in full 128-B lines (64 k); the 16-B units are XOR-swizzled by
//     (row >> 1) on the SOURCE address (LDS-DMA writes lane-linear), which makes every
//     16-row fragment read conflict-free under the ds_read_b128 lane groups;
//   * a 64-k tile is four 16-KiB "pieces" [x rows lo | x rows hi | W k0 | W k1] in one of
//     two buffers (128 KiB LDS, one workgroup per CU). Each of the tile's four phases
//     (rows lo/hi x k halves, 16 MFMAs per wave) reads the NEXT phase's fragments ahead and
//     issues one piece of tile i + 2 with a counted vmcnt — pieces stay in flight across the
//     raw s_barrier of every phase (schedule table at the read-ahead body below). This is
//     the fallback family (variant 1: work items of one k-tile) next to the ping-pong
//     kernels of gemm_pingpong.h;
//   * s_setprio(1) around each MFMA cluster keeps hipcc from moving the MFMAs across the
//     barriers (guide §5.5 T5);
//   * tiles are numbered row-tile fastest and mapped XCD-aware, so the 8 row tiles that
//     share a W panel at M = 2,048 run on one XCD (W read once from HBM per panel);
//   * wave quantisation: tiles [0, full) run whole, the remaining tiles are split over S
//     K-slices (one more round of shorter items instead of a half-empty round). The slices
//     publish fp32 partials write-through in the accumulators' own fragment order and the
//     last arriver adds them to its registers after the agent-scope acquire of
//     common.h handoff_last.
#include "common.h"
#include "packed_epi.h"

#include <algorithm>
#include <type_traits>

namespace pa {
namespace pf {

using namespace pk;

struct Args {
  bf16* y;
  const bf16* x;
  const bf16* wp;
  const bf16* resid;
  float* ws;      // split slabs: [(tiles - full) * S][256 * 256] fp32, fragment order
  int* counters;  // [tiles - full] arrival tickets, zero between launches
  int M, N, K, ldx, ldy, ldr;
  int MT, NT;     // 256-row / 256-column tiles
  int full;       // tiles [0, full) run whole
  int S, per;     // tiles [full, MT * NT): S K-slices of `per` 64-k tiles
  float eps;
  const float* ss_in;  // NORM: [M] row sum(x^2) over K
  float* ss_out;       // EP_RESID (optional): [M] += row sum(y^2) of the written bf16 output
  float* ss_zero;      // optional: [M] zeroed by workgroup 0
  bf16* q_out;
  bf16* k_cache;
  bf16* v_cache;
  const int* positions;
  const int* slots;
  const float* cos_sin;
  int H, KV;
  int acq;
};

typedef __attribute__((address_space(3))) void lds_t;
typedef __attribute__((address_space(1))) void gbl_t;

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at "no wait"); gfx9 encoding.
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void glds16(const bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_t*)src, (lds_t*)lds, 16, 0, 0);
}

constexpr int PIECE = 16384;          // bytes
constexpr int BUF = 4 * PIECE;        // one 64-k tile: [A-p0 | A-p1 | B-k0 | B-k1]
constexpr int OFF_B = 2 * PIECE;
constexpr int SLAB = 256 * 256;       // floats per split slab

template <int V>
using ic = std::integral_constant<int, V>;

template <int EPI, bool NORM>
__global__ __launch_bounds__(512) void prefill_gemm_kernel(const Args A) {
  constexpr int NW = 8;           // 2 x 4 waves of 128 x 64 outputs
  constexpr int WCN = NW / 2;     // wave columns
  constexpr int CPW = 16 / WCN;   // 16-column fragments per wave
  constexpr int LPW = 16 / NW;    // LDS-DMA loads per lane per 16-KiB piece
  constexpr int NTH = NW * 64;
  // the only LDS object (guide §5 trap 4a): two tile buffers, reused by the hand-off flag
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / WCN, wc = wid % WCN;
  const int g = lane >> 4, c = lane & 15;

  // ---- work item: a whole tile, or one K-slice of a tail tile
  const int bid = blockIdx.x;
  const int KT = A.K >> 6;
  int tile, kt0, kt1, slice = -1;
  if (bid < A.full) {  // XCD-aware bijective remap: consecutive tiles share an XCD
    const int q8 = A.full >> 3, r8 = A.full & 7, xcd = bid & 7;
    tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    kt0 = 0;
    kt1 = KT;
  } else {
    const int w2 = bid - A.full;
    tile = A.full + w2 / A.S;
    slice = w2 % A.S;
    kt0 = slice * A.per;
    kt1 = min(KT, kt0 + A.per);
  }
  const int mt = tile % A.MT, nt = tile / A.MT;
  const int row0 = mt * 256;
  const int nk = kt1 - kt0;

  if (A.ss_zero && blockIdx.x == 0)
    for (int i = threadIdx.x; i < A.M; i += NTH) A.ss_zero[i] = 0.f;

  // ---- per-lane LDS-DMA sources
  // x piece p (rows lo / hi of each wave row): LDS row lr = (LPW wid + q) * 8 + (lane >> 3)
  // holds tile row (lr >> 6) * 128 + 64 p + (lr & 63); its 16-B unit (lane & 7) is the
  // row's logical unit (lane & 7) ^ ((lr >> 1) & 7).
  const bf16* xs[2][LPW];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < LPW; ++q) {
      const int lr = (wid * LPW + q) * 8 + (lane >> 3);
      const int trow = (lr >> 6) * 128 + p * 64 + (lr & 63);
      const int gr = min(row0 + trow, A.M - 1);
      const int unit = (lane & 7) ^ ((lr >> 1) & 7);
      xs[p][q] = A.x + (size_t)gr * A.ldx + unit * 8;
    }
  const int KS = A.K >> 5;
  const bf16* wsrc[LPW];
#pragma unroll
  for (int q = 0; q < LPW; ++q) wsrc[q] = A.wp + ((size_t)(nt * 16 + wid * LPW + q) * KS) * 512 + lane * 8;

  auto issue_a = [&](int p, int kt, char* buf) {
#pragma unroll
    for (int q = 0; q < LPW; ++q) glds16(xs[p][q] + (size_t)kt * 64, buf + p * PIECE + (wid * LPW + q) * 1024);
  };
  auto issue_b = [&](int kh, int kt, char* buf) {
#pragma unroll
    for (int q = 0; q < LPW; ++q)
      glds16(wsrc[q] + (size_t)(2 * kt + kh) * 512, buf + OFF_B + kh * PIECE + (wid * LPW + q) * 1024);
  };
  auto read_b = [&](const char* buf, int kh, bf16x8(&bf)[CPW]) {
#pragma unroll
    for (int j = 0; j < CPW; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(buf + OFF_B + kh * PIECE + (wc * CPW + j) * 1024 + lane * 16);
  };
  auto read_a = [&](const char* buf, int p, int kh, bf16x8(&af)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = wr * 64 + 16 * i + c;
      const int u = 4 * kh + g;
      af[i] = *reinterpret_cast<const bf16x8*>(buf + p * PIECE + lr * 128 + ((u ^ ((lr >> 1) & 7)) << 4));
    }
  };

  f32x4 acc[8][CPW];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < CPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](auto half, const bf16x8(&af)[4], const bf16x8(&bf)[CPW]) {
    constexpr int h = decltype(half)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < CPW; ++j)
        acc[h * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[h * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  char* const b0 = smem;
  char* const b1 = smem + BUF;
  bf16x8 bk0[CPW], bk1[CPW];

  {
    // Read-ahead schedule: each phase's window (between two barriers) issues the LDS reads
    // of the NEXT phase into the other register set, one piece of tile i + 2 (into the
    // current buffer: its region's last reads completed before the window's barrier), then
    // the phase's 16 MFMAs on registers read one window earlier; every wave retires its
    // LDS reads (lgkmcnt(0)) and the counted vmcnt before the barrier. Pieces stay in flight
    // ~5 phases (vmcnt(10): 5 pieces x 2 LDS-DMA loads per lane).
    //   window  reads (for next phase)        MFMA          issue           wait
    //   ph0     B-k1(i) -> bk1, x-lo k1 -> afB  afA x bk0    B-k0(i + 2)     10
    //   ph1     x-hi k0 -> afA                  afB x bk1    x-lo(i + 2)     -
    //   ph2     x-hi k1 -> afB                  afA x bk0    B-k1(i + 2)     10
    //   ph3     B-k0(i+1) -> bk0, x-lo(i+1) -> afA  afB x bk1  x-hi(i + 2)   10
    bf16x8 afA[4], afB[4];
    auto body = [&](int i, auto iss, auto nxt, auto w0, auto w2, auto w3) {
      char* cur = (i & 1) ? b1 : b0;
      char* oth = (i & 1) ? b0 : b1;
      // ph0
      read_b(cur, 1, bk1);
      read_a(cur, 0, 1, afB);
      if constexpr (decltype(iss)::value) issue_b(0, kt0 + i + 2, cur);
      mma(ic<0>{}, afA, bk0);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this window's LDS reads are done
      if constexpr (decltype(w0)::value >= 0) wait_vm<decltype(w0)::value * LPW / 2>();
      raw_barrier();
      // ph1
      read_a(cur, 1, 0, afA);
      if constexpr (decltype(iss)::value) issue_a(0, kt0 + i + 2, cur);
      mma(ic<0>{}, afB, bk1);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      raw_barrier();
      // ph2
      read_a(cur, 1, 1, afB);
      if constexpr (decltype(iss)::value) issue_b(1, kt0 + i + 2, cur);
      mma(ic<1>{}, afA, bk0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if constexpr (decltype(w2)::value >= 0) wait_vm<decltype(w2)::value * LPW / 2>();
      raw_barrier();
      // ph3
      if constexpr (decltype(nxt)::value) {
        read_b(oth, 0, bk0);
        read_a(oth, 0, 0, afA);
      }
      if constexpr (decltype(iss)::value) issue_a(1, kt0 + i + 2, cur);
      mma(ic<1>{}, afB, bk1);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if constexpr (decltype(w3)::value >= 0) wait_vm<decltype(w3)::value * LPW / 2>();
      raw_barrier();
    };
    // prologue: the pieces of tiles 0 and 1 in steady-state order, then phase 0's registers
    issue_b(0, kt0, b0);
    issue_a(0, kt0, b0);
    issue_b(1, kt0, b0);
    issue_a(1, kt0, b0);
    if (nk >= 2) {
      issue_b(0, kt0 + 1, b1);
      issue_a(0, kt0 + 1, b1);
      issue_b(1, kt0 + 1, b1);
      issue_a(1, kt0 + 1, b1);
      wait_vm<10 * LPW / 2>();  // tile 0's B-k0, x-lo and B-k1 landed
    } else {
      wait_vm<2 * LPW / 2>();
    }
    raw_barrier();
    read_b(b0, 0, bk0);
    read_a(b0, 0, 0, afA);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // no LDS read pending at the loop head (else hipcc waits
                                         // lgkmcnt(0) before phase 0's MFMAs on every iteration)
    if (nk >= 2) {
      int i = 0;
      for (; i + 2 < nk; ++i) body(i, ic<1>{}, ic<1>{}, ic<10>{}, ic<10>{}, ic<10>{});
      body(i, ic<0>{}, ic<1>{}, ic<8>{}, ic<4>{}, ic<2>{});       // tile nk - 2: nothing left to issue
      body(i + 1, ic<0>{}, ic<0>{}, ic<0>{}, ic<-1>{}, ic<-1>{});  // tile nk - 1
    } else {
      body(0, ic<0>{}, ic<0>{}, ic<0>{}, ic<-1>{}, ic<-1>{});
    }
  }

  // ---- split tiles: publish, last arriver sums the other slices into its registers
  if (slice >= 0) {
    float* base = A.ws + (size_t)(tile - A.full) * A.S * SLAB;
    {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)slice * SLAB, 0, SLAB * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < CPW; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                 (((wid * 8 + i) * CPW + j) * 64 + lane) * 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(A.counters + (tile - A.full), A.S, reinterpret_cast<int*>(smem), A.acq)) return;
    for (int p = 0; p < A.S; ++p) {
      if (p == slice) continue;
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)p * SLAB, 0, SLAB * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; i += 8 / CPW) {  // 8 loads in flight per lane (the accumulators hold the rest)
        f32x4 t[8 / CPW][CPW];
#pragma unroll
        for (int h = 0; h < 8 / CPW; ++h)
#pragma unroll
          for (int j = 0; j < CPW; ++j)
            t[h][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rp, (((wid * 8 + i + h) * CPW + j) * 64 + lane) * 16, 0, 16));
#pragma unroll
        for (int h = 0; h < 8 / CPW; ++h)
#pragma unroll
          for (int j = 0; j < CPW; ++j) acc[i + h][j] += t[h][j];
      }
    }
  }

  // ---- register epilogue: lane (g, c) of tile (i, j) holds token row 16 i + c (of its
  // wave's 128), columns 4 g .. 4 g + 3 of 16-column tile nt * 16 + wc * 4 + j
  const float inv_k = 1.f / (float)A.K;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = row0 + wr * 128 + 16 * i + c;
    const bool ok = m < A.M;
    float sq = 0.f;
    if (ok) {
      float rs = 1.f;
      if constexpr (NORM) rs = rsqrtf(A.ss_in[m] * inv_k + A.eps);
      if constexpr (pair_epi<EPI>()) {
#pragma unroll
        for (int j = 0; j < CPW; j += 2)
          store_quad<EPI>(A, m, nt * 16 + wc * CPW + j, 4 * g, acc[i][j] * rs, acc[i][j + 1] * rs);
      } else {
#pragma unroll
        for (int j = 0; j < CPW; ++j)
          sq += store_quad<EPI>(A, m, nt * 16 + wc * CPW + j, 4 * g, acc[i][j] * rs, acc[i][j]);
      }
    }
    if constexpr (EPI == EP_RESID) {
      if (A.ss_out) {
        sq += __shfl_xor(sq, 16, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (ok && g == 0) atomicAdd(A.ss_out + m, sq);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256 x 128 tiles (N = 4,096 / 6,144 projections, and gate_up where 128-wide tiles fill
// whole rounds: 1,792 tiles = 7 x 256 CUs at M = 2,048). One tile stage is 48 KiB
// ([x 256 rows x 64 k | W-k0 8 chunks | W-k1 8 chunks]), so THREE stages fit (144 KiB):
// two tiles are in flight while one is computed, with ONE barrier per 64-k tile (the
// schedule is at `body` below).
//
// 8 waves as 4 (rows) x 2 (columns), 64 x 64 outputs per wave (acc[4][4], 64 VGPRs); the
// per-wave fragment reads (4 x-rows + 4 W per 32 k) keep the LDS array under half busy.
// The x image and its (row >> 1) unit swizzle are those of the 256-wide kernel.
constexpr int BUF128 = 49152;
constexpr int OFFB128 = 32768;
constexpr int SLAB128 = 256 * 128;

template <int EPI, bool NORM>
__global__ __launch_bounds__(512) void prefill_gemm_n128_kernel(const Args A) {
  __shared__ __attribute__((aligned(1024))) char smem[3 * BUF128];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int g = lane >> 4, c = lane & 15;

  const int bid = blockIdx.x;
  const int KT = A.K >> 6;
  int tile, kt0, kt1, slice = -1;
  if (bid < A.full) {
    const int q8 = A.full >> 3, r8 = A.full & 7, xcd = bid & 7;
    tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    kt0 = 0;
    kt1 = KT;
  } else {
    const int w2 = bid - A.full;
    tile = A.full + w2 / A.S;
    slice = w2 % A.S;
    kt0 = slice * A.per;
    kt1 = min(KT, kt0 + A.per);
  }
  const int mt = tile % A.MT, nt = tile / A.MT;
  const int row0 = mt * 256;
  const int nk = kt1 - kt0;

  if (A.ss_zero && blockIdx.x == 0)
    for (int i = threadIdx.x; i < A.M; i += 512) A.ss_zero[i] = 0.f;

  // wave w stages x rows 32 w .. 32 w + 31 (four 8-row x 128-B pieces) and W chunk w of
  // both k halves; 6 LDS-DMA loads per lane per tile
  const bf16* xs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int lr = (wid * 4 + q) * 8 + (lane >> 3);
    const int gr = min(row0 + lr, A.M - 1);
    xs[q] = A.x + (size_t)gr * A.ldx + ((lane & 7) ^ ((lr >> 1) & 7)) * 8;
  }
  const int KS = A.K >> 5;
  const bf16* wsrc = A.wp + ((size_t)(nt * 8 + wid) * KS) * 512 + lane * 8;

  auto stage = [&](int i) { return smem + (i % 3) * BUF128; };
  auto issue = [&](int kt, char* buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) glds16(xs[q] + (size_t)kt * 64, buf + (wid * 4 + q) * 1024);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) glds16(wsrc + (size_t)(2 * kt + kh) * 512, buf + OFFB128 + kh * 8192 + wid * 1024);
  };
  auto read_frags = [&](const char* buf, int kh, bf16x8(&af)[4], bf16x8(&bf)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(buf + OFFB128 + kh * 8192 + (wn * 4 + j) * 1024 + lane * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = wm * 64 + 16 * i + c;
      af[i] = *reinterpret_cast<const bf16x8*>(buf + lr * 128 + (((4 * kh + g) ^ ((lr >> 1) & 7)) << 4));
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8(&af)[4], const bf16x8(&bf)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  bf16x8 aA[4], bA[4], aB[4], bB[4];
  // Tile i in two phases; each phase issues the fragment reads of the NEXT phase into the
  // other register set, runs its 16 MFMAs on registers read one phase earlier and ends with
  // lgkmcnt(0) (so no LDS read is in flight at a phase boundary and hipcc never has to wait
  // for a read issued in the same phase before an MFMA):
  //   A: k1 of tile i -> set B | MFMAs set A (k0 of i) | lgkmcnt(0), vmcnt retiring tile
  //      i + 1, s_barrier
  //   B: k0 of tile i + 1 -> set A | LDS-DMA tile i + 3 into tile i's stage (every read of
  //      it finished before the barrier) | MFMAs set B (k1 of i) | lgkmcnt(0)
  // ISS: issue tile i + 3; W: that vmcnt (-1: last tile, no barrier); NXT: tile i + 1 exists
  auto body = [&](int i, auto iss, auto w, auto nxt) {
    char* cur = stage(i);
    read_frags(cur, 1, aB, bB);
    mma(aA, bA);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if constexpr (decltype(w)::value >= 0) {
      wait_vm<decltype(w)::value>();
      raw_barrier();
    }
    if constexpr (decltype(nxt)::value) read_frags(stage(i + 1), 0, aA, bA);
    if constexpr (decltype(iss)::value) issue(kt0 + i + 3, cur);
    mma(aB, bB);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  };

  issue(kt0, stage(0));
  if (nk > 1) issue(kt0 + 1, stage(1));
  if (nk > 2) issue(kt0 + 2, stage(2));
  if (nk > 2) wait_vm<12>();
  else if (nk == 2) wait_vm<6>();
  else wait_vm<0>();
  raw_barrier();
  read_frags(stage(0), 0, aA, bA);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  int i = 0;
  for (; i + 3 < nk; ++i) body(i, ic<1>{}, ic<6>{}, ic<1>{});
  if (nk >= 3) body(nk - 3, ic<0>{}, ic<6>{}, ic<1>{});
  if (nk >= 2) body(nk - 2, ic<0>{}, ic<0>{}, ic<1>{});
  body(nk - 1, ic<0>{}, ic<-1>{}, ic<0>{});

  if (slice >= 0) {
    float* base = A.ws + (size_t)(tile - A.full) * A.S * SLAB128;
    {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(base + (size_t)slice * SLAB128, 0, SLAB128 * 4, 0x00020000);
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i2][j]), rs,
                                                 (((wid * 4 + i2) * 4 + j) * 64 + lane) * 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!handoff_last(A.counters + (tile - A.full), A.S, reinterpret_cast<int*>(smem), A.acq)) return;
    for (int p = 0; p < A.S; ++p) {
      if (p == slice) continue;
      const __amdgpu_buffer_rsrc_t rp =
          __builtin_amdgcn_make_buffer_rsrc(base + (size_t)p * SLAB128, 0, SLAB128 * 4, 0x00020000);
      f32x4 t[4][4];
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          t[i2][j] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, (((wid * 4 + i2) * 4 + j) * 64 + lane) * 16, 0, 16));
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i2][j] += t[i2][j];
    }
  }

  const float inv_k = 1.f / (float)A.K;
#pragma unroll
  for (int i2 = 0; i2 < 4; ++i2) {
    const int m = row0 + wm * 64 + 16 * i2 + c;
    const bool ok = m < A.M;
    float sq = 0.f;
    if (ok) {
      float rs = 1.f;
      if constexpr (NORM) rs = rsqrtf(A.ss_in[m] * inv_k + A.eps);
      if constexpr (pair_epi<EPI>()) {
#pragma unroll
        for (int j = 0; j < 4; j += 2)
          store_quad<EPI>(A, m, nt * 8 + wn * 4 + j, 4 * g, acc[i2][j] * rs, acc[i2][j + 1] * rs);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          sq += store_quad<EPI>(A, m, nt * 8 + wn * 4 + j, 4 * g, acc[i2][j] * rs, acc[i2][j]);
      }
    }
    if constexpr (EPI == EP_RESID) {
      if (A.ss_out) {
        sq += __shfl_xor(sq, 16, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (ok && g == 0) atomicAdd(A.ss_out + m, sq);
      }
    }
  }
}

}  // namespace pf
}  // namespace pa

#include "gemm_pingpong.h"

namespace pa {
namespace pf {

// Kernel family: 3 = ping-pong wave groups (gemm_pingpong.h; default; 256-wide tiles on the
// two-phase schedule with the mixed 128-wide tail when it applies, 192- and 128-wide tiles
// on their own schedules; items of < 2 k-tiles fall back to 1); 9 = 3 without the mixed
// tail; 4 = its cycle-stamp build; 1 = read-ahead 8-wave 256 x 256 / 3-stage 256 x 128.
// (Measured and removed: the four-phase ping-pong schedule, buffer_load staging, 4-wave
// 128 x 128 kernels -- profiles/r3_pingpong_ph2_ab.jsonl, profiles/r5_w4_experiment.md.)
constexpr int kPfDefaultVariant = 3;
static int g_pf_variant = kPfDefaultVariant;

// Default decomposition: whole tiles while they fill complete rounds of 256 CUs; a
// remainder of at most half a round is split over K so that the last round is (nearly)
// full. Measured on MI355X (profiles/r3_prefill_gemm_variants.jsonl): a split slice costs
// far more than its MFMA share — a 256 KiB fp32 slab written per item and read serially
// by the tile's last arriver at one CU's bandwidth — so 192 leftover tiles run whole (one
// 75 %-full round: qkv at M = 2,048 106 us) rather than as 768 quarter items (190 us, and
// the tail items regrouped per XCD did not recover it).
constexpr long long kWsFloats = 64ll << 20;  // the workspace ops.prefill_workspace allocates

static void plan_default(int M, int N, int K, int bn, int& full, int& S) {
  const int tiles = ((M + 255) / 256) * (N / bn);
  const int KT = K / 64;
  const int rem = tiles % 256;
  full = tiles - rem;
  S = 1;
  if (rem) {
    S = std::max(1, std::min(4, 256 / rem));
    while (S > 1 && (KT / S < 8 || (long long)rem * S * 256 * bn > kWsFloats)) --S;
    if (S == 1) full = tiles;
  }
}

// Tile width when the caller leaves it open: 256 x 128 tiles for the narrow projections
// (N <= 6,144: qkv / o / down of Llama-3-8B, 0.6-0.85x the 256-wide kernel's time at
// M <= 1,024), 256 x 256 for wide ones (gate_up: 1.08x faster).
static int pick_bn(int M, int N) {
  (void)M;
  return (N % 256 || N <= 6144) ? 128 : 256;
}

}  // namespace pf
}  // namespace pa

extern "C" void pa_prefill_set_variant(int v) { pa::pf::g_pf_variant = v < 0 ? pa::pf::kPfDefaultVariant : v; }

extern "C" int pa_prefill_pick_bn(int M, int N) { return pa::pf::pick_bn(M, N); }

extern "C" void pa_prefill_gemm_plan(int M, int N, int K, int bn, int* full, int* S) {
  if (bn <= 0) bn = pa::pf::pick_bn(M, N);
  pa::pf::plan_default(M, N, K, bn, *full, *S);
}

extern "C" long long pa_prefill_gemm_ws_floats(int M, int N, int bn, int full, int S) {
  if (bn <= 0) bn = pa::pf::pick_bn(M, N);
  const long long tiles = (long long)((M + 255) / 256) * (N / bn);
  return S > 1 ? (tiles - full) * S * (long long)(256 * bn) : 0;
}

// Returns 1 if the shape/config is not handled, 0 on success, -2 on a launch error.
// kernel_variant >= 0 picks the kernel family for this call (3: ping-pong, 1: read-ahead /
// 3-stage 256 x 128), < 0 the process default (pa_prefill_set_variant).
// full < 0 / splits <= 0 / bn <= 0 pick the defaults. For epi 4 (RoPE + paged KV write) y
// is unused.
extern "C" int pa_prefill_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws,
                               long long ws_floats, int* counters, int n_counters, int M, int N, int K, int ldx,
                               int ldy, int ldr, int epi, const float* ss_in, float* ss_out, float* ss_zero,
                               float eps, int full, int splits, int bn, void* q_out, void* k_cache, void* v_cache,
                               const int* positions, const int* slots, const float* cos_sin, int H, int KV,
                               int kernel_variant, hipStream_t st) {
  using namespace pa::pf;
  if (M <= 0) return 0;
  if (bn <= 0) bn = pick_bn(M, N);
  if (bn != 128 && bn != 192 && bn != 256) return 1;
  if (K % 64 != 0 || N % bn != 0 || epi < 0 || epi > 4 || ldx % 8 != 0) return 1;
  const int norm = ss_in != nullptr;
  if (epi == EP_RESID && (!resid || norm)) return 1;
  if (ss_out && epi != EP_RESID) return 1;
  if (epi == EP_ROPEKV && (!q_out || !k_cache || !v_cache || !positions || !slots || !cos_sin ||
                           N != (H + 2 * KV) * 128))
    return 1;
  const int MT = (M + 255) / 256, NT = N / bn, tiles = MT * NT;
  const bool default_plan = full < 0 && splits <= 0;
  int dfull, dS;
  plan_default(M, N, K, bn, dfull, dS);
  if (full < 0) full = dfull;
  int S = splits > 0 ? splits : (full == dfull ? dS : 1);
  full = std::min(std::max(full, 0), tiles);
  const int KT = K / 64;
  S = std::max(1, std::min(S, KT));
  int per = (KT + S - 1) / S;
  S = (KT + per - 1) / per;  // no empty slices
  if (S == 1) full = tiles;
  // the ping-pong kernel's schedule needs >= 2 k-tiles per work item
  int variant = kernel_variant >= 0 ? kernel_variant : g_pf_variant;
  if (variant >= 3 && (KT < 2 || (S > 1 && (per < 2 || KT - (S - 1) * per < 2)))) variant = 1;
  if (bn == 192 && variant < 3) return 1;  // 256 x 192 tiles: ping-pong schedule only
  if (full < tiles) {
    const long long need = (long long)(tiles - full) * S * (256 * bn);
    if (!ws || !counters || n_counters < tiles - full || need > ws_floats) return 1;
  }
  Args a{(pa::bf16*)y, (const pa::bf16*)x, (const pa::bf16*)wp, (const pa::bf16*)resid, ws, counters,
         M, N, K, ldx, ldy, ldr, MT, NT, full, S, per, eps, ss_in, ss_out, ss_zero,
         (pa::bf16*)q_out, (pa::bf16*)k_cache, (pa::bf16*)v_cache, positions, slots, cos_sin, H, KV,
         pa::g_handoff_acquire};
  const int grid = full + (tiles - full) * S;
  // Mixed tail (variant 3, the default, and 8; 9 = without it): full rounds of 256 x 256
  // tiles over the first c1 column tiles,
  // the remaining columns as 256 x 128 tiles in the same launch, when that tail fits one
  // round of half-size tiles (pingpong_mixed_kernel). Not for the RoPE + KV-write epilogue
  // (its head index comes from the absolute column tile).
  if (variant == 3 || variant == 8) {
    const int r = tiles % 256, c1 = (tiles - r) / MT, nsmall = MT * 2 * (NT - c1);
    if (!(bn == 256 && default_plan && r > 0 && c1 > 0 && nsmall <= 256 && epi != EP_ROPEKV)) {
      variant = 3;
    } else {
      const int nbig = c1 * MT;
      Args big = a;
      big.full = nbig;
      big.S = 1;
      big.per = KT;
      Args sm = a;
      const int co = c1 * 256;  // first column (packed) of the 128-wide tiles
      sm.wp = a.wp + (size_t)c1 * 16 * (K / 32) * 512;
      sm.y = a.y ? a.y + (epi == EP_SILU ? co / 2 : co) : nullptr;
      sm.resid = a.resid ? a.resid + co : nullptr;
      sm.N = N - co;
      sm.NT = sm.N / 128;
      sm.full = nsmall;
      sm.S = 1;
      sm.per = KT;
      sm.ss_zero = nullptr;
#define PA_MIX(E, NRM) hipLaunchKernelGGL((pingpong_mixed_kernel<E, NRM>), dim3(nbig + nsmall), dim3(512), 0, st, big, sm, nbig)
      switch (epi) {
        case EP_PLAIN: if (norm) PA_MIX(EP_PLAIN, true); else PA_MIX(EP_PLAIN, false); break;
        case EP_RESID: PA_MIX(EP_RESID, false); break;
        case EP_ROPEPERM: if (norm) PA_MIX(EP_ROPEPERM, true); else PA_MIX(EP_ROPEPERM, false); break;
        case EP_SILU: if (norm) PA_MIX(EP_SILU, true); else PA_MIX(EP_SILU, false); break;
        default: return 1;
      }
#undef PA_MIX
      return (int)hipGetLastError() == 0 ? 0 : -2;
    }
  }
#define PA_PF(E, NRM)                                                                                \
  do {                                                                                               \
    const bool stamp = E == EP_PLAIN && !NRM && full == tiles;                                       \
    if (bn == 192) hipLaunchKernelGGL((pingpong_gemm_kernel<E, NRM, false, 6>), dim3(grid), dim3(512), 0, st, a); \
    else if (bn == 128 && variant == 4 && stamp)                                                     \
      hipLaunchKernelGGL((pingpong_gemm_kernel<EP_PLAIN, false, true, 4>), dim3(grid), dim3(512), 0, st, a); \
    else if (bn == 128 && variant >= 3) hipLaunchKernelGGL((pingpong_gemm_kernel<E, NRM, false, 4>), dim3(grid), dim3(512), 0, st, a); \
    else if (bn == 128) hipLaunchKernelGGL((prefill_gemm_n128_kernel<E, NRM>), dim3(grid), dim3(512), 0, st, a); \
    else if (variant == 4 && stamp)                                                                  \
      hipLaunchKernelGGL((pingpong_gemm_kernel<EP_PLAIN, false, true, 8>), dim3(grid), dim3(512), 0, st, a); \
    else if (variant >= 3) hipLaunchKernelGGL((pingpong_gemm_kernel<E, NRM, false, 8>), dim3(grid), dim3(512), 0, st, a); \
    else hipLaunchKernelGGL((prefill_gemm_kernel<E, NRM>), dim3(grid), dim3(512), 0, st, a);          \
  } while (0)
  switch (epi) {
    case EP_PLAIN:
      if (norm) PA_PF(EP_PLAIN, true); else PA_PF(EP_PLAIN, false);
      break;
    case EP_RESID:
      PA_PF(EP_RESID, false);
      break;
    case EP_ROPEPERM:
      if (norm) PA_PF(EP_ROPEPERM, true); else PA_PF(EP_ROPEPERM, false);
      break;
    case EP_SILU:
      if (norm) PA_PF(EP_SILU, true); else PA_PF(EP_SILU, false);
      break;
    case EP_ROPEKV:
      if (norm) PA_PF(EP_ROPEKV, true); else PA_PF(EP_ROPEKV, false);
      break;
    default:
      return 1;
  }
#undef PA_PF
  return (int)hipGetLastError() == 0 ? 0 : -2;
}
