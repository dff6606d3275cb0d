// Exact ring GEMM over Z_2^64 / Z_2^128 on the gfx950 int8 matrix cores.
//
// There is no 64-bit integer MFMA, so every ring element is split into L signed 8-bit
// limbs (L = 8 for Z_2^64, 16 for Z_2^128) in the *balanced* representation
// x = sum_l d_l 256^l, d_l in [-128, 127] (carry propagated low to high; the carry out of
// the top limb vanishes mod 2^(8L)).  Then
//
//     x . y  =  sum_{d < L} 256^d  sum_{i + j = d} (X_i . Y_j)      (mod 2^(8L))
//
// so the product needs the L(L+1)/2 limb-pair GEMMs on or below the anti-diagonal (36 for
// Z_2^64, 136 for Z_2^128), each an i8 x i8 -> i32 MFMA (v_mfma_i32_32x32x32_i8).  Pairs on
// the same anti-diagonal d accumulate into ONE i32 accumulator tile, so a wave holds L
// accumulator tiles (16 regs each).  Diagonal d contributes S_d * 2^(8d) and only needs S_d
// mod 2^(8(L-d)); for the low diagonals |S_d| <= (d+1) K' 2^14 < 2^31 whenever K' <= 8192
// (Z_2^128) / 16384 (Z_2^64), and the high diagonals (8(L-d) <= 32) may wrap freely.
// Longer K is split into chunks accumulated in the output.
//
// The RSS multiplication needs z_i = x_i.(y_i + y_{i+1}) + x_{i+1}.y_i per party.  That is
// ONE GEMM with a doubled K: A' = [x_i | x_{i+1}], B' = [y_i + y_{i+1} ; y_i]  (mode 1).
// The three parties of a stacked session are the batch dimension of one launch.
//
// Pipeline per call:
//   1. prep_a / prep_b (memory-bound): limb-split A' and B' into a blocked, swizzled int8
//      layout [batch][tile][k-step][limb][64 rows][32 bytes] so that each 64x32 tile of a
//      limb plane is a contiguous 2 KB image whose 16-byte fragment reads are LDS
//      bank-conflict free (halves of rows r and r+8 are swapped).
//   2. gemm (MFMA-bound): 256-thread blocks (4 waves as 2x2), 64x64 output tile, each wave
//      32x32 with L diagonal accumulators; K advances 32 limb-bytes per step, streamed
//      global->LDS by LDS-DMA (global_load_lds) into a double buffer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>

#include "hip_attr.h"
#include "moosex.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

namespace {

// MX_SETPRIO=1: raise the wave priority for the MFMA section of each k-step (tuning knob)
#ifndef MX_SETPRIO
#define MX_SETPRIO 0
#endif
#if MX_SETPRIO
#define MX_PRIO_HI() __builtin_amdgcn_s_setprio(1)
#define MX_PRIO_LO() __builtin_amdgcn_s_setprio(0)
#else
#define MX_PRIO_HI() ((void)0)
#define MX_PRIO_LO() ((void)0)
#endif

constexpr int TM = 64;  // rows of the block tile (A side)
constexpr int TN = 64;  // cols of the block tile (B side)
constexpr int TK = 32;  // limb-bytes per k-step (one MFMA K)
constexpr int kTileBytes = 64 * TK;  // one limb plane of one tile per k-step: 2 KB
constexpr int kGroupM = 4;           // row bands per L2 tile group

__device__ __host__ inline int swz(int r, int h) { return r * TK + 16 * (h ^ ((r >> 3) & 1)); }

template <class T>
struct Limbs;
template <>
struct Limbs<u64> {
  static constexpr int L = 8;
};
template <>
struct Limbs<u128> {
  static constexpr int L = 16;
};

// Pack the balanced limbs of 16 consecutive k' of one tile row into L 16-byte vectors
// (word j/4, byte j%4); fully unrolled so everything stays in registers.
template <class T, class Load>
__device__ inline void split16(Load load, v4i (&w)[Limbs<T>::L]) {
  constexpr int L = Limbs<T>::L;
#pragma unroll
  for (int l = 0; l < L; ++l) w[l] = v4i{0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    T x = load(j);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      int v = (int)(x & 0xff);
      x >>= 8;
      if (v >= 128) x += 1;  // balanced digit v - 256, carry one into the next limb
      w[l][j >> 2] |= (v & 0xff) << (8 * (j & 3));
    }
  }
}

// One thread = (tile, k-step, tile row r, k-half h); a wave covers 32 rows x both halves of
// one (tile, k-step), so every limb-plane store of the wave is one contiguous 1 KB run.
__device__ inline void prep_coords(int64_t g, int64_t nkb, int64_t& t, int64_t& kb, int& r,
                                   int& h) {
  h = (int)(g & 1);
  r = (int)((g >> 1) & 63);
  const int64_t q = g >> 7;
  kb = q % nkb;
  t = q / nkb;
}

// A' [batch, M, K'] (K' = K or 2K: mode 1 concatenates A0 | A1) -> blocked limbs.
template <class T>
__global__ void __launch_bounds__(256) k_prep_a(const T* __restrict__ A0, const T* __restrict__ A1,
                                                int64_t M, int64_t K, int64_t a_bstride, int mode,
                                                int8_t* __restrict__ out, int64_t Mp, int64_t Kp) {
  constexpr int L = Limbs<T>::L;
  const int64_t nkb = Kp / TK;
  const int64_t total = (Mp / TM) * nkb * 128;
  const int64_t b = blockIdx.y;
  const T* a0 = A0 + b * a_bstride;
  const T* a1 = mode ? A1 + b * a_bstride : a0;
  int8_t* ob = out + b * (Mp / TM) * nkb * (int64_t)L * kTileBytes;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    int64_t mb, kb;
    int r, h;
    prep_coords(g, nkb, mb, kb, r, h);
    const int64_t m = mb * TM + r;
    const int64_t k0 = kb * TK + h * 16;
    v4i w[L];
    split16<T>(
        [&](int j) -> T {
          const int64_t k = k0 + j;
          if (m >= M) return 0;
          if (k < K) return a0[m * K + k];
          if (mode && k < 2 * K) return a1[m * K + (k - K)];
          return 0;
        },
        w);
    int8_t* base = ob + (mb * nkb + kb) * (int64_t)L * kTileBytes + swz(r, h);
#pragma unroll
    for (int l = 0; l < L; ++l) *(v4i*)(base + l * kTileBytes) = w[l];
  }
}

// B' [batch, K', N] -> blocked limbs with n as the tile row.  mode 1: rows k < K hold
// B0 + B1, rows K <= k < 2K hold B0.  Lanes of a wave read 32 consecutive columns.
template <class T>
__global__ void __launch_bounds__(256) k_prep_b(const T* __restrict__ B0, const T* __restrict__ B1,
                                                int64_t K, int64_t N, int64_t b_bstride, int mode,
                                                int8_t* __restrict__ out, int64_t Np, int64_t Kp) {
  constexpr int L = Limbs<T>::L;
  const int64_t nkb = Kp / TK;
  const int64_t total = (Np / TN) * nkb * 128;
  const int64_t b = blockIdx.y;
  const T* b0 = B0 + b * b_bstride;
  const T* b1 = mode ? B1 + b * b_bstride : b0;
  int8_t* ob = out + b * (Np / TN) * nkb * (int64_t)L * kTileBytes;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    int64_t nb, kb;
    int r, h;
    prep_coords(g, nkb, nb, kb, r, h);
    const int64_t n = nb * TN + r;
    const int64_t k0 = kb * TK + h * 16;
    v4i w[L];
    split16<T>(
        [&](int j) -> T {
          const int64_t k = k0 + j;
          if (n >= N) return 0;
          if (k < K) return mode ? (T)(b0[k * N + n] + b1[k * N + n]) : b0[k * N + n];
          if (mode && k < 2 * K) return b0[(k - K) * N + n];
          return 0;
        },
        w);
    int8_t* base = ob + (nb * nkb + kb) * (int64_t)L * kTileBytes + swz(r, h);
#pragma unroll
    for (int l = 0; l < L; ++l) *(v4i*)(base + l * kTileBytes) = w[l];
  }
}

// XCD-aware remap of the flattened tile index: consecutive tiles of the same row band
// land on the same XCD (blocks b and b+8 share an XCD under round-robin dispatch).
__device__ inline int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8;
  const int64_t x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <class T>
__global__ void __launch_bounds__(256, Limbs<T>::L == 8 ? 2 : 1)
    k_gemm_limb(const int8_t* __restrict__ LA, const int8_t* __restrict__ LB,
                T* __restrict__ C, int64_t M, int64_t N, int64_t Mp, int64_t Np, int64_t Kp,
                int accumulate, int gM, int xcd) {
  constexpr int L = Limbs<T>::L;
  constexpr int STAGE = L * kTileBytes;  // bytes per operand per k-step
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  // two LDS buffers, each holding the A and B stage of one k-step
  auto buf = [&](int i) -> int8_t* { return smem + i * 2 * STAGE; };

  const int64_t tiles_n = Np / TN, tiles_m = Mp / TM;
  const int64_t ntiles = tiles_n * tiles_m;
  // XCD-contiguous tile ranges, walked in groups of kGroupM row bands so the ~32 blocks
  // co-resident on one XCD cover a 4 x 8 patch of output tiles: they share 4 A and 8 B
  // k-streams in that XCD's L2 instead of 1 A and 32 B streams.
  const int64_t tid_flat = xcd ? xcd_remap(blockIdx.x, ntiles) : (int64_t)blockIdx.x;
  const int64_t group = tid_flat / (gM * tiles_n);
  const int64_t first_m = group * gM;
  const int64_t gm = tiles_m - first_m < gM ? tiles_m - first_m : gM;
  const int64_t in_group = tid_flat % (gM * tiles_n);
  const int64_t tm = first_m + in_group % gm, tn = in_group / gm;
  const int64_t b = blockIdx.y;
  const int64_t nkb = Kp / TK;

  const int8_t* ga = LA + (b * tiles_m + tm) * nkb * (int64_t)STAGE;
  const int8_t* gb = LB + (b * tiles_n + tn) * nkb * (int64_t)STAGE;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int arow = wr * 32 + (lane & 31);
  const int brow = wc * 32 + (lane & 31);
  const int half = lane >> 5;

  v16i acc[L];
#pragma unroll
  for (int d = 0; d < L; ++d) acc[d] = v16i{0};

  // Stage k-step kb of both operands straight into LDS with global_load_lds (16 B per
  // lane, 1 KiB per wave-instruction): the blocked limb layout makes each stage one
  // contiguous image, so the lane-linear LDS destination of LDS-DMA matches exactly and no
  // VGPRs are spent on staging (they hold the 2 x L MFMA fragments instead).
  constexpr int PIECES = STAGE / 1024;  // 1 KiB pieces per operand per stage
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto issue_stage = [&](int64_t kb, int8_t* dst) {
    const int8_t* sa = ga + kb * STAGE + lane * 16;
    const int8_t* sb = gb + kb * STAGE + lane * 16;
#pragma unroll
    for (int c = wave_u; c < PIECES; c += 4) {
      __builtin_amdgcn_global_load_lds((const void*)(sa + c * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + c * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(sb + c * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + STAGE + c * 1024),
                                       16, 0, 0);
    }
  };
  // Two LDS buffers; the DMA of stage kb+1 is in flight while stage kb is multiplied.  One
  // barrier per k-step: after it every wave has finished reading buffer kb&1 (so it may be
  // refilled with stage kb+2) and every wave's DMA of stage kb+1 has landed (vmcnt(0)).
  // (Commit 221b0c9 moved the barrier before the last A-limb's MFMA run and prefetched
  // the next step's fragments into a second register set: 4% slower, 43.6 vs 42.0 ms at
  // 3 x 4096 x 8192 x 4096 -- the extra live VGPRs cost more than the hidden LDS latency.)
  const int aoff = swz(arow, half), boff = swz(brow, half);
  issue_stage(0, buf(0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nkb > 1) issue_stage(1, buf(1));
  for (int64_t kb = 0; kb < nkb; ++kb) {
    const int cur = (int)(kb & 1);
    const int8_t* As = buf(cur);
    const int8_t* Bs = As + STAGE;
    // B fragments of the step stay resident; A limbs are consumed one per round, so only
    // two are requested ahead of their round (the rest stream in behind the MFMAs).
    v4i bf[L], af[L];
#pragma unroll
    for (int j = 0; j < L; ++j) bf[j] = *(const v4i*)(Bs + j * kTileBytes + boff);
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *(const v4i*)(As + i * kTileBytes + aoff);
    // Issue order: round i multiplies A limb i into diagonals d = L-1 .. i (j = d - i),
    // so consecutive MFMAs never share an accumulator and two updates of the same
    // diagonal are >= 2 MFMAs apart (no back-to-back SrcC dependency); the scheduling
    // barriers keep the compiler from regrouping them.
#pragma unroll
    for (int i = 0; i < L; ++i) {
      if (i + 2 < L) af[i + 2] = *(const v4i*)(As + (i + 2) * kTileBytes + aoff);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = L - 1; d >= i; --d) {
        acc[d] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[d - i], acc[d], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kb + 2 < nkb) issue_stage(kb + 2, buf(cur));
  }

  // epilogue: C[row][col] = sum_d sext(acc_d) << 8d
  const int col = lane & 31;
  const int64_t gcol = tn * TN + wc * 32 + col;
  T* cb = C + b * M * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int64_t grow = tm * TM + wr * 32 + row;
    T v = 0;
#pragma unroll
    for (int d = 0; d < L; ++d) v += ((T)(int64_t)acc[d][r]) << (8 * d);
    if (grow < M && gcol < N) {
      T* p = cb + grow * N + gcol;
      *p = accumulate ? (T)(*p + v) : v;
    }
  }
}

// Z_2^128 variant with TWO waves per SIMD.  The 16 diagonal accumulators of a 32x32 tile
// (256 registers) pin k_gemm_limb to one wave per SIMD, so every LDS wait and barrier
// idles the matrix core.  Here each 32x32 tile is owned by a pair of waves that split the
// anti-diagonals: the "low" wave sums d = 0..kSplit-1 (55 MFMAs, 10 accumulators), the
// "high" wave d = kSplit..15 (81 MFMAs, 6 accumulators), each within 256 registers, so
// 8 waves share the CU and one wave's MFMAs cover the other's waits.  B fragments a wave
// needs stay resident; A fragments stream limb by limb.  The high wave hands its partial
// sums to the low wave through LDS at the end.
constexpr int kSplit = 10;

__global__ void __launch_bounds__(512, 1)
    k_gemm_limb128_split(const int8_t* __restrict__ LA, const int8_t* __restrict__ LB,
                         u128* __restrict__ C, int64_t M, int64_t N, int64_t Mp, int64_t Np,
                         int64_t Kp, int accumulate, int gM, int xcd) {
  constexpr int L = 16;
  constexpr int STAGE = L * kTileBytes;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  auto buf = [&](int i) -> int8_t* { return smem + i * 2 * STAGE; };

  const int64_t tiles_n = Np / TN, tiles_m = Mp / TM;
  const int64_t ntiles = tiles_n * tiles_m;
  const int64_t tid_flat = xcd ? xcd_remap(blockIdx.x, ntiles) : (int64_t)blockIdx.x;
  const int64_t group = tid_flat / (gM * tiles_n);
  const int64_t first_m = group * gM;
  const int64_t gm = tiles_m - first_m < gM ? tiles_m - first_m : gM;
  const int64_t in_group = tid_flat % (gM * tiles_n);
  const int64_t tm = first_m + in_group % gm, tn = in_group / gm;
  const int64_t b = blockIdx.y;
  const int64_t nkb = Kp / TK;
  const int8_t* ga = LA + (b * tiles_m + tm) * nkb * (int64_t)STAGE;
  const int8_t* gb = LB + (b * tiles_n + tn) * nkb * (int64_t)STAGE;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;  // 0..7
  const int tile = wave & 3;          // which 32x32 quarter of the 64x64 block tile
  const bool high = wave >= 4;        // diagonal half
  const int wr = tile >> 1, wc = tile & 1;
  const int half = lane >> 5;
  const int aoff = swz(wr * 32 + (lane & 31), half);
  const int boff = swz(wc * 32 + (lane & 31), half);

  constexpr int PIECES = STAGE / 1024;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto issue_stage = [&](int64_t kb, int8_t* dst) {
    const int8_t* sa = ga + kb * STAGE + lane * 16;
    const int8_t* sb = gb + kb * STAGE + lane * 16;
#pragma unroll
    for (int c = wave_u; c < PIECES; c += 8) {
      __builtin_amdgcn_global_load_lds((const void*)(sa + c * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + c * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(sb + c * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + STAGE + c * 1024),
                                       16, 0, 0);
    }
  };

  constexpr int NLO = kSplit, NHI = L - kSplit;
  v16i acc[NLO > NHI ? NLO : NHI];
#pragma unroll
  for (int d = 0; d < (NLO > NHI ? NLO : NHI); ++d) acc[d] = v16i{0};

  issue_stage(0, buf(0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nkb > 1) issue_stage(1, buf(1));
  for (int64_t kb = 0; kb < nkb; ++kb) {
    const int cur = (int)(kb & 1);
    const int8_t* As = buf(cur);
    const int8_t* Bs = As + STAGE;
    if (!high) {
      v4i bf[NLO];
#pragma unroll
      for (int j = 0; j < NLO; ++j) bf[j] = *(const v4i*)(Bs + j * kTileBytes + boff);
      MX_PRIO_HI();
#pragma unroll
      for (int i = 0; i < NLO; ++i) {
        const v4i a = *(const v4i*)(As + i * kTileBytes + aoff);
#pragma unroll
        for (int j = 0; j < NLO - i; ++j)
          acc[i + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bf[j], acc[i + j], 0, 0, 0);
      }
    } else {
      v4i bf[L];
#pragma unroll
      for (int j = 0; j < L; ++j) bf[j] = *(const v4i*)(Bs + j * kTileBytes + boff);
      MX_PRIO_HI();
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const v4i a = *(const v4i*)(As + i * kTileBytes + aoff);
#pragma unroll
        for (int j = (kSplit - i > 0 ? kSplit - i : 0); j < L - i; ++j)
          acc[i + j - kSplit] =
              __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bf[j], acc[i + j - kSplit], 0, 0, 0);
      }
    }
    MX_PRIO_LO();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kb + 2 < nkb) issue_stage(kb + 2, buf(cur));
  }

  // epilogue: the high wave parks its partial sums in LDS (free now), the low wave adds
  // its own and writes C.  16 rows x 64 lanes x 16 B = 16 KB per tile.
  u128* part = (u128*)smem + tile * (16 * 64);
  if (high) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      u128 v = 0;
#pragma unroll
      for (int d = 0; d < NHI; ++d) v += ((u128)(int64_t)acc[d][r]) << (8 * (d + kSplit));
      part[r * 64 + lane] = v;
    }
  }
  __syncthreads();
  if (!high) {
    const int col = lane & 31;
    const int64_t gcol = tn * TN + wc * 32 + col;
    u128* cb = C + b * M * N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t grow = tm * TM + wr * 32 + row;
      u128 v = part[r * 64 + lane];
#pragma unroll
      for (int d = 0; d < NLO; ++d) v += ((u128)(int64_t)acc[d][r]) << (8 * d);
      if (grow < M && gcol < N) {
        u128* p = cb + grow * N + gcol;
        *p = accumulate ? (u128)(*p + v) : v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// v2 kernels: software-pipelined across the k-step boundary.
//
// PMC on the kernels above (profiles/r2_v0_gemm_pmc.md): the matrix pipes idle ~26 % of
// the time.  After each k-step barrier every wave first issues its LDS-DMA pieces, then a
// burst of fragment reads, and waits for them before its first MFMA -- with both waves of a
// SIMD doing the same thing at the same moment, the pipe drains at every step.
//
// Here each wave's share of a k-step is a static schedule of "rounds" (round i multiplies
// A limb i into its diagonals) split in two phases around ONE barrier:
//   phase 1 (rounds < SPLIT): fragments of the current stage are read >= 2 rounds ahead of
//            use; every read of the stage is issued (and waited for) before the barrier;
//   barrier: all waves have finished reading stage k and their DMA of stage k+1 landed;
//   phase 2 (rounds >= SPLIT): operands already in registers.  Interleaved with these MFMAs
//            the wave issues its share of the DMA of stage k+2 (into stage k's buffer) and
//            reads the fragments that step k+1 needs first ("carried": A_0, A_1 and the B
//            limbs used in rounds 0-1) from stage k+1.
// So right after the barrier every wave has MFMAs ready, and the next step starts with its
// first operands already in registers: the pipe never waits on LDS at a step boundary.
// Two LDS stages (A + B per stage).  The k-loop is unrolled by two so the carried register
// sets swap roles without moves.
// ---------------------------------------------------------------------------------------
template <int L_, int DLO_, int DHI_, int SPLIT_>
struct TriWave {
  static constexpr int L = L_, DLO = DLO_, DHI = DHI_, SPLIT = SPLIT_;
  static constexpr int LAST = DHI < L - 1 ? DHI : L - 1;  // last round (= last A limb)
  static constexpr int ND = DHI - DLO + 1;                // accumulators
  __host__ __device__ static constexpr int jlo(int i) { return DLO - i > 0 ? DLO - i : 0; }
  __host__ __device__ static constexpr int jhi(int i) { return DHI - i < L - 1 ? DHI - i : L - 1; }
  __host__ __device__ static constexpr int bfirst(int j) { return DLO - j > 0 ? DLO - j : 0; }
  // Operands used in rounds 0 and 1 are "carried" (read during the previous step); any
  // other operand first used in round `use` is read right after the MFMAs of round
  // rd(use) = use - 2, so a whole round of MFMAs covers its latency (the compiler waits
  // with lgkmcnt(0) before a consumer, so a read must not be issued just before one), and
  // never after the step's barrier.
  __host__ __device__ static constexpr bool carried(int j) { return bfirst(j) <= 1; }
  __host__ __device__ static constexpr int rd(int use) {
    return use - 2 < SPLIT - 1 ? use - 2 : SPLIT - 1;
  }
  __host__ __device__ static constexpr int mfmas() {
    int n = 0;
    for (int i = 0; i <= LAST; ++i) n += jhi(i) - jlo(i) + 1;
    return n;
  }
  __host__ __device__ static constexpr int phase2_mfmas() {
    int n = 0;
    for (int i = SPLIT; i <= LAST; ++i) n += jhi(i) - jlo(i) + 1;
    return n;
  }
  static_assert(SPLIT >= 2 && SPLIT <= LAST, "phase 2 must exist and start after round 1");
};

// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(0) in the gfx9 encoding
constexpr int kWaitVmLgkm0 = 0x0070;

__device__ __forceinline__ v4i lds_frag(const int8_t* base, int limb, int off) {
  return *(const v4i*)(base + limb * kTileBytes + off);
}

// One k-step of one wave.  `dma(t)` issues this wave's t-th DMA piece of stage k+2 (past
// the last stage it re-reads the last stage into a buffer nobody reads any more, so the
// schedule has no branches); the carried fragments of stage k+1 are read unconditionally
// (past the end they are never used).
template <class W, int NPIECE, class Dma>
__device__ __forceinline__ void tri_step(const int8_t* As, const int8_t* Bs,
                                         const int8_t* Asn, const int8_t* Bsn, int aoff,
                                         int boff, v16i (&acc)[W::ND], const v4i (&Ac)[2],
                                         const v4i (&Bc)[W::L], v4i (&An)[2], v4i (&Bn)[W::L],
                                         Dma&& dma) {
  constexpr int L = W::L;
  v4i A[L], B[L];
  A[0] = Ac[0];
  A[1] = Ac[1];
#pragma unroll
  for (int j = 0; j <= W::LAST; ++j)
    if (W::carried(j)) B[j] = Bc[j];
  int piece = 0;  // DMA pieces issued in phase 2 (compile-time after unrolling)
#pragma unroll
  for (int r = 0; r <= W::LAST; ++r) {
    if (r == W::SPLIT) {
      // all reads of this stage done, my DMA of the next stage landed (a builtin, so the
      // compiler's wait-count model knows the pre-barrier reads are complete)
      __builtin_amdgcn_s_waitcnt(kWaitVmLgkm0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = W::jlo(r); j <= W::jhi(r); ++j) {
      acc[r + j - W::DLO] =
          __builtin_amdgcn_mfma_i32_32x32x32_i8(A[r], B[j], acc[r + j - W::DLO], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (r == W::SPLIT && j == W::jlo(r)) {  // carried fragments of the next step
        An[0] = lds_frag(Asn, 0, aoff);
        An[1] = lds_frag(Asn, 1, aoff);
#pragma unroll
        for (int jj = 0; jj <= W::LAST; ++jj)
          if (W::carried(jj)) Bn[jj] = lds_frag(Bsn, jj, boff);
        __builtin_amdgcn_sched_barrier(0);
      } else if (r >= W::SPLIT && piece < NPIECE) {
        dma(piece);
        ++piece;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // reads issued after this round's MFMAs
#pragma unroll
    for (int i = 2; i <= W::LAST; ++i)
      if (W::rd(i) == r) A[i] = lds_frag(As, i, aoff);
#pragma unroll
    for (int j = 0; j <= W::LAST; ++j)
      if (!W::carried(j) && W::rd(W::bfirst(j)) == r) B[j] = lds_frag(Bs, j, boff);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (; piece < NPIECE; ++piece) dma(piece);  // phase 2 shorter than the DMA share
}

// The whole k-loop of one wave: prologue (stage 0 landed, carried fragments read, DMA of
// stage 1 in flight), then steps unrolled by two.  Ends with every DMA landed and a
// barrier, so the caller may reuse the LDS.
template <class W, int NPIECE, class Dma>
__device__ __forceinline__ void tri_loop(const int8_t* smem, int stage_bytes, int a_bytes,
                                         int aoff, int boff, int64_t nkb,
                                         v16i (&acc)[W::ND], Dma&& dma_stage) {
  constexpr int L = W::L;
  v4i A0[2], B0[L], A1[2], B1[L];
  auto As = [&](int64_t kb) { return smem + (kb & 1) * stage_bytes; };
  auto Bs = [&](int64_t kb) { return smem + (kb & 1) * stage_bytes + a_bytes; };
  auto clampk = [&](int64_t kb) { return kb < nkb ? kb : nkb - 1; };
#pragma unroll
  for (int t = 0; t < NPIECE; ++t) dma_stage(0, t, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  A0[0] = lds_frag(As(0), 0, aoff);
  A0[1] = lds_frag(As(0), 1, aoff);
#pragma unroll
  for (int j = 0; j <= W::LAST; ++j)
    if (W::carried(j)) B0[j] = lds_frag(Bs(0), j, boff);
#pragma unroll
  for (int t = 0; t < NPIECE; ++t) dma_stage(clampk(1), t, 1);
  for (int64_t kb = 0; kb < nkb; kb += 2) {
    const int64_t s2 = clampk(kb + 2), s3 = clampk(kb + 3);
    tri_step<W, NPIECE>(As(kb), Bs(kb), As(kb + 1), Bs(kb + 1), aoff, boff, acc, A0, B0, A1,
                        B1, [&](int t) { dma_stage(s2, t, (int)(kb & 1)); });
    if (kb + 1 < nkb)
      tri_step<W, NPIECE>(As(kb + 1), Bs(kb + 1), As(kb + 2), Bs(kb + 2), aoff, boff, acc,
                          A1, B1, A0, B0, [&](int t) { dma_stage(s3, t, (int)((kb + 1) & 1)); });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Z_2^128, 64x64 block tile, 8 waves: wave w owns 32x32 quarter (w & 3); waves 0-3 sum the
// anti-diagonals 0..kLo-1, waves 4-7 the rest (register budget: 2 waves per SIMD).
constexpr int kLo = 9;
using Lo128 = TriWave<16, 0, kLo - 1, 5>;
using Hi128 = TriWave<16, kLo, 15, 11>;

__global__ void __launch_bounds__(512, 1)
    k_gemm128_v2(const int8_t* __restrict__ LA, const int8_t* __restrict__ LB,
                 u128* __restrict__ C, int64_t M, int64_t N, int64_t Mp, int64_t Np, int64_t Kp,
                 int accumulate, int gM, int xcd) {
  constexpr int L = 16;
  constexpr int SA = L * kTileBytes;  // A stage bytes (32 KB); B the same
  constexpr int STAGE = 2 * SA;
  constexpr int NPIECE = STAGE / 1024 / 8;  // DMA pieces per wave per stage
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const int64_t tiles_n = Np / TN, tiles_m = Mp / TM;
  const int64_t ntiles = tiles_n * tiles_m;
  const int64_t tid_flat = xcd ? xcd_remap(blockIdx.x, ntiles) : (int64_t)blockIdx.x;
  const int64_t group = tid_flat / (gM * tiles_n);
  const int64_t first_m = group * gM;
  const int64_t gm = tiles_m - first_m < gM ? tiles_m - first_m : gM;
  const int64_t in_group = tid_flat % (gM * tiles_n);
  const int64_t tm = first_m + in_group % gm, tn = in_group / gm;
  const int64_t b = blockIdx.y;
  const int64_t nkb = Kp / TK;
  const int8_t* ga = LA + (b * tiles_m + tm) * nkb * (int64_t)SA;
  const int8_t* gb = LB + (b * tiles_n + tn) * nkb * (int64_t)SA;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = wave & 3;
  const bool high = wave >= 4;
  const int wr = tile >> 1, wc = tile & 1;
  const int half = lane >> 5;
  const int aoff = swz(wr * 32 + (lane & 31), half);
  const int boff = swz(wc * 32 + (lane & 31), half);

  // piece c = wave + 8 t of a stage: A pieces 0..31, B pieces 32..63
  auto dma_stage = [&](int64_t kb, int t, int bufi) {
    const int c = wave + 8 * t;
    const bool is_b = t >= 4;  // wave < 8
    const int cc = is_b ? c - 32 : c;
    const int8_t* src = (is_b ? gb : ga) + kb * SA + cc * 1024 + lane * 16;
    int8_t* dst = smem + bufi * STAGE + (is_b ? SA : 0) + cc * 1024;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };

  v16i acc[Lo128::ND > Hi128::ND ? Lo128::ND : Hi128::ND];
#pragma unroll
  for (int d = 0; d < (Lo128::ND > Hi128::ND ? Lo128::ND : Hi128::ND); ++d) acc[d] = v16i{0};
  if (high) {
    v16i (&a)[Hi128::ND] = *reinterpret_cast<v16i(*)[Hi128::ND]>(&acc);
    tri_loop<Hi128, NPIECE>(smem, STAGE, SA, aoff, boff, nkb, a, dma_stage);
  } else {
    v16i (&a)[Lo128::ND] = *reinterpret_cast<v16i(*)[Lo128::ND]>(&acc);
    tri_loop<Lo128, NPIECE>(smem, STAGE, SA, aoff, boff, nkb, a, dma_stage);
  }

  // epilogue: high waves park their partial sums in LDS, low waves add and store
  u128* part = (u128*)smem + tile * (16 * 64);
  if (high) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      u128 v = 0;
#pragma unroll
      for (int d = 0; d < Hi128::ND; ++d) v += ((u128)(int64_t)acc[d][r]) << (8 * (d + kLo));
      part[r * 64 + lane] = v;
    }
  }
  __syncthreads();
  if (!high) {
    const int col = lane & 31;
    const int64_t gcol = tn * TN + wc * 32 + col;
    u128* cb = C + b * M * N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t grow = tm * TM + wr * 32 + row;
      u128 v = part[r * 64 + lane];
#pragma unroll
      for (int d = 0; d < Lo128::ND; ++d) v += ((u128)(int64_t)acc[d][r]) << (8 * d);
      if (grow < M && gcol < N) {
        u128* p = cb + grow * N + gcol;
        *p = accumulate ? (u128)(*p + v) : v;
      }
    }
  }
}

// Z_2^64, 64x128 block tile (two 64-column B tiles), 8 waves = 2 x 4 quarters of 32x32,
// every wave all 8 diagonals (128 accumulator registers; 2 waves per SIMD).  Versus the
// 64x64 / 4-wave kernel this cuts the L2->LDS stream per MFMA by a quarter.
using W64 = TriWave<8, 0, 7, 4>;

__global__ void __launch_bounds__(512, 1)
    k_gemm64_v2(const int8_t* __restrict__ LA, const int8_t* __restrict__ LB,
                u64* __restrict__ C, int64_t M, int64_t N, int64_t Mp, int64_t Np, int64_t Kp,
                int accumulate, int gM, int xcd) {
  constexpr int L = 8;
  constexpr int SA = L * kTileBytes;  // 16 KB: one 64-row tile of A
  constexpr int SB = 2 * SA;          // two 64-column tiles of B
  constexpr int STAGE = SA + SB;
  constexpr int NPIECE = STAGE / 1024 / 8;  // 6
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const int64_t tiles_n2 = Np / (2 * TN), tiles_m = Mp / TM;  // block tiles
  const int64_t ntiles = tiles_n2 * tiles_m;
  const int64_t tid_flat = xcd ? xcd_remap(blockIdx.x, ntiles) : (int64_t)blockIdx.x;
  const int64_t group = tid_flat / (gM * tiles_n2);
  const int64_t first_m = group * gM;
  const int64_t gm = tiles_m - first_m < gM ? tiles_m - first_m : gM;
  const int64_t in_group = tid_flat % (gM * tiles_n2);
  const int64_t tm = first_m + in_group % gm, tn2 = in_group / gm;
  const int64_t b = blockIdx.y;
  const int64_t nkb = Kp / TK;
  const int8_t* ga = LA + (b * tiles_m + tm) * nkb * (int64_t)SA;
  const int8_t* gb = LB + (b * (Np / TN) + 2 * tn2) * nkb * (int64_t)SA;  // first of two

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // 2 x 4 quarters
  const int half = lane >> 5;
  const int aoff = swz(wr * 32 + (lane & 31), half);
  const int boff = (wc >> 1) * SA + swz((wc & 1) * 32 + (lane & 31), half);

  // piece c = wave + 8 t: A pieces 0..15, B pieces 16..47 (16 per 64-column tile)
  auto dma_stage = [&](int64_t kb, int t, int bufi) {
    const int c = wave + 8 * t;
    const int8_t* src;
    if (t < 2) {
      src = ga + kb * SA + c * 1024;
    } else {
      const int cb = c - 16, h = cb >> 4;
      src = gb + (h * nkb + kb) * SA + (cb & 15) * 1024;
    }
    int8_t* dst = smem + bufi * STAGE + c * 1024;
    __builtin_amdgcn_global_load_lds((const void*)(src + lane * 16),
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };

  v16i acc[W64::ND];
#pragma unroll
  for (int d = 0; d < W64::ND; ++d) acc[d] = v16i{0};
  tri_loop<W64, NPIECE>(smem, STAGE, SA, aoff, boff, nkb, acc, dma_stage);

  const int col = lane & 31;
  const int64_t gcol = tn2 * 2 * TN + wc * 32 + col;
  u64* cbase = C + b * M * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int64_t grow = tm * TM + wr * 32 + row;
    u64 v = 0;
#pragma unroll
    for (int d = 0; d < W64::ND; ++d) v += ((u64)(int64_t)acc[d][r]) << (8 * d);
    if (grow < M && gcol < N) {
      u64* p = cbase + grow * N + gcol;
      *p = accumulate ? (u64)(*p + v) : v;
    }
  }
}

// MOOSEX_GEMM_V=1 selects the round-1 kernels (A/B measurements)
bool use_v1_kernels() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_GEMM_V");
    return e && e[0] == '1';
  }();
  return on;
}

// MOOSEX_GEMM_SPLIT=0 selects the one-wave-per-SIMD kernel for Z_2^128 (A/B testing)
// Tile-order knobs (tuning experiments): MOOSEX_GEMM_GROUPM row bands per L2 group
// (default kGroupM), MOOSEX_GEMM_XCD=0 disables the XCD-contiguous block remap.
int gemm_group_m() {
  const char* e = std::getenv("MOOSEX_GEMM_GROUPM");
  int v = e ? std::atoi(e) : kGroupM;
  return v >= 1 && v <= 64 ? v : kGroupM;
}

int gemm_xcd() {
  const char* e = std::getenv("MOOSEX_GEMM_XCD");
  return e && e[0] == '0' ? 0 : 1;
}

bool use_split_kernel() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_GEMM_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace

// Workspace bookkeeping shared with gemm_crt.hip: the size of the last failed allocation
// (reported by the Python wrapper when a GEMM returns -4) and the bytes held per device.
std::atomic<int64_t> g_ws_failed{0};
std::atomic<int64_t> g_ws_held[16];
std::atomic<int64_t> g_ws_shared{0};

void mx_ws_shared_note(void) { ++g_ws_shared; }

// lookups that found every per-stream slot taken and fell back to a shared one (0 expected)
extern "C" int64_t mx_workspace_shared_count(void) { return g_ws_shared.load(); }

// A workspace that grows while its stream is being captured (a taped evaluation's first
// product of a size, on the tape's own stream): the allocation is not a stream operation,
// so it runs in relaxed capture mode (as PyTorch's caching allocator allocates inside
// captures); the buffer is never freed, so the captured kernels' pointer stays valid.
bool mx_ws_malloc(void** p, int64_t bytes) {
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
  const bool ok = hipMalloc(p, bytes) == hipSuccess;
  if (swapped) hipThreadExchangeStreamCaptureMode(&mode);
  if (!ok) (void)hipGetLastError();
  return ok;
}

void mx_ws_note(int dev, int64_t want, bool ok) {
  if (ok) {
    if (dev >= 0 && dev < 16) g_ws_held[dev] += want;
  } else {
    g_ws_failed = want;
    (void)hipGetLastError();  // do not leave the OOM as the sticky error of later launches
  }
}

extern "C" int64_t mx_workspace_failed_bytes(void) { return g_ws_failed.exchange(0); }

extern "C" int64_t mx_workspace_held_bytes(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  return g_ws_held[dev].load();
}

namespace {

struct Workspace {
  void* ptr = nullptr;
  int64_t bytes = 0;
  hipStream_t stream = nullptr;
  bool used = false;
};
std::mutex g_ws_mu;
constexpr int kWsPerDev = 128;
Workspace g_ws[16][kWsPerDev];

// Grow-only scratch per (device, stream) -- see gemm_crt.hip workspace(): concurrent GEMMs
// on different streams get different buffers.  A replaced buffer is retired, never freed: a
// captured hipGraph may still reference it, and freeing would need a device-wide sync.
void* get_workspace(int64_t bytes, hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) return nullptr;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Workspace* slot = nullptr;
  for (int i = 0; i < kWsPerDev && !slot; ++i)
    if (g_ws[dev][i].used && g_ws[dev][i].stream == st) slot = &g_ws[dev][i];
  for (int i = 0; i < kWsPerDev && !slot; ++i)
    if (!g_ws[dev][i].used) {
      slot = &g_ws[dev][i];
      slot->used = true;
      slot->stream = st;
    }
  if (!slot) {
    slot = &g_ws[dev][kWsPerDev - 1];
    mx_ws_shared_note();
  }
  Workspace& w = *slot;
  if (w.bytes < bytes) {
    int64_t want = 1 << 20;
    while (want < bytes) want <<= 1;
    void* p = nullptr;
    const bool ok = mx_ws_malloc(&p, want);
    mx_ws_note(dev, want, ok);
    if (!ok) return nullptr;
    w.ptr = p;  // the previous buffer (if any) stays allocated
    w.bytes = want;
  }
  return w.ptr;
}

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct Plan {
  int L;
  int64_t Mp, Np, Kp, la_bytes, lb_bytes;
};

Plan make_plan(int words, int64_t batch, int64_t M, int64_t N, int64_t Kchunk, int mode) {
  Plan p;
  p.L = words == 1 ? 8 : 16;
  p.Mp = round_up(M, TM);
  p.Np = round_up(N, words == 1 ? 2 * TN : TN);
  p.Kp = round_up(mode ? 2 * Kchunk : Kchunk, TK);
  p.la_bytes = batch * p.Mp * p.Kp * p.L;
  p.lb_bytes = batch * p.Np * p.Kp * p.L;
  return p;
}

int64_t max_k_chunk(int words, int mode) {
  // K' limit keeping the low diagonals exact in i32 (see header comment)
  int64_t kp = words == 1 ? 16384 : 8192;
  return mode ? kp / 2 : kp;
}

template <class T>
void launch_prep_a(const Plan& p, int64_t batch, int64_t M, int64_t K, const T* A0,
                   const T* A1, int64_t a_bstride, int mode, int8_t* la, hipStream_t st) {
  const int threads = 256;
  const int64_t work = p.Mp * (p.Kp / 16);
  const int gx = (int)std::min<int64_t>((work + threads - 1) / threads, 8192);
  hipLaunchKernelGGL(k_prep_a<T>, dim3(gx, (unsigned)batch), dim3(threads), 0, st, A0, A1, M, K,
                     a_bstride, mode, la, p.Mp, p.Kp);
}

template <class T>
void launch_prep_b(const Plan& p, int64_t batch, int64_t K, int64_t N, const T* B0,
                   const T* B1, int mode, int8_t* lb, hipStream_t st, int64_t b_bstride = -1) {
  const int threads = 256;
  const int64_t work = p.Np * (p.Kp / 16);
  const int gx = (int)std::min<int64_t>((work + threads - 1) / threads, 8192);
  hipLaunchKernelGGL(k_prep_b<T>, dim3(gx, (unsigned)batch), dim3(threads), 0, st, B0, B1, K, N,
                     b_bstride < 0 ? K * N : b_bstride, mode, lb, p.Np, p.Kp);
}

template <class T>
void launch_gemm(const Plan& p, int64_t batch, int64_t M, int64_t N, const int8_t* la,
                 const int8_t* lb, T* C, int accumulate, hipStream_t st) {
  constexpr int L = Limbs<T>::L;
  const int64_t ntiles = (p.Mp / TM) * (p.Np / TN);
  const size_t lds = 4 * (size_t)L * kTileBytes;  // 2 buffers x (A + B) stages
  ensure_lds_attr((const void*)k_gemm_limb<T>, (int)lds, st);
  ensure_lds_attr((const void*)k_gemm_limb128_split, (int)lds, st);
  ensure_lds_attr((const void*)k_gemm128_v2, 4 * 16 * kTileBytes, st);
  ensure_lds_attr((const void*)k_gemm64_v2, 2 * 3 * 8 * kTileBytes, st);
  if (!use_v1_kernels()) {
    if constexpr (sizeof(T) == 16) {
      hipLaunchKernelGGL(k_gemm128_v2, dim3((unsigned)ntiles, (unsigned)batch), dim3(512),
                         4 * 16 * kTileBytes, st, la, lb, (u128*)C, M, N, p.Mp, p.Np, p.Kp,
                         accumulate, gemm_group_m(), gemm_xcd());
    } else {
      hipLaunchKernelGGL(k_gemm64_v2, dim3((unsigned)(ntiles / 2), (unsigned)batch), dim3(512),
                         2 * 3 * 8 * kTileBytes, st, la, lb, (u64*)C, M, N, p.Mp, p.Np, p.Kp,
                         accumulate, gemm_group_m(), gemm_xcd());
    }
  } else if (sizeof(T) == 16 && use_split_kernel()) {
    hipLaunchKernelGGL(k_gemm_limb128_split, dim3((unsigned)ntiles, (unsigned)batch), dim3(512),
                       lds, st, la, lb, (u128*)C, M, N, p.Mp, p.Np, p.Kp, accumulate,
                       gemm_group_m(), gemm_xcd());
  } else {
    hipLaunchKernelGGL(k_gemm_limb<T>, dim3((unsigned)ntiles, (unsigned)batch), dim3(256), lds,
                       st, la, lb, C, M, N, p.Mp, p.Np, p.Kp, accumulate, gemm_group_m(),
                       gemm_xcd());
  }
}

template <class T>
int run(int64_t batch, int64_t M, int64_t N, int64_t K, const T* A0, const T* A1, const T* B0,
        const T* B1, int mode, T* C, int accumulate, void* ws, int64_t ws_bytes,
        hipStream_t st) {
  if (K > max_k_chunk(sizeof(T) == 8 ? 1 : 2, mode)) return -6;  // caller splits long K
  Plan p = make_plan(sizeof(T) == 8 ? 1 : 2, batch, M, N, K, mode);
  if (p.la_bytes + p.lb_bytes > ws_bytes) return -5;
  int8_t* la = (int8_t*)ws;
  int8_t* lb = la + p.la_bytes;
  launch_prep_a<T>(p, batch, M, K, A0, A1, M * K, mode, la, st);
  launch_prep_b<T>(p, batch, K, N, B0, B1, mode, lb, st);
  launch_gemm<T>(p, batch, M, N, la, lb, C, accumulate, st);
  hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

}  // namespace

namespace {

// Register-only MFMA throughput probe: the ceiling the limb GEMM is measured against
// (same instruction, same clock behaviour, no memory traffic).
__global__ void __launch_bounds__(256, 1) k_mfma_peak(int iters, int* __restrict__ sink) {
  v16i acc[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) acc[d] = v16i{0};
  v4i a = v4i{(int)threadIdx.x, 1, 2, 3}, b = v4i{3, 2, 1, (int)blockIdx.x};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int d = 0; d < 8; ++d) acc[d] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[d], 0, 0, 0);
  }
  int s = 0;
#pragma unroll
  for (int d = 0; d < 8; ++d) s += acc[d][threadIdx.x & 15];
  if (s == 0x7fffffff) sink[0] = s;
}

}  // namespace

extern "C" {

int mx_mfma_peak(int blocks, int iters, void* sink, void* stream) {
  hipLaunchKernelGGL(k_mfma_peak, dim3(blocks), dim3(256), 0, (hipStream_t)stream, iters,
                     (int*)sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"

// multi-modular (CRT) GEMM, gemm_crt.hip
extern "C" int mxh_gemm_crt(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                            const void* A0, const void* A1, const void* B0, const void* B1,
                            int mode, void* C, int accumulate, void* stream);
extern "C" int64_t mxh_crt_b_bytes(int words, int64_t batch, int64_t N, int64_t K, int mode);
extern "C" int mxh_crt_prep_b(int words, int64_t batch, int64_t K, int64_t N, const void* B0,
                              const void* B1, int mode, void* rb, void* stream);
extern "C" int mxh_gemm_crt_strided(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                                    const void* A0, const void* A1, int64_t a_bstride,
                                    const void* B0, const void* B1, int64_t b_bstride, int mode,
                                    void* C, int accumulate, void* stream);
extern "C" int mxh_crt_with_b(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                              const void* A0, const void* A1, int64_t a_bstride, int mode,
                              const void* rb, void* C, int accumulate, void* stream);
extern "C" int mxh_crt_roll(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                            const void* A0, int64_t a_bstride, int64_t roll, const void* B0,
                            const void* B1, const void* rb, void* C, int accumulate,
                            void* stream);

namespace {
// 0 = auto (CRT for products with at least one full 256x256 output tile and K' >= 512),
// 1 = CRT whenever K' allows, 2 = limb GEMM only.  MOOSEX_GEMM_CRT overrides the default.
int g_crt_mode = -1;

int crt_mode() {
  if (g_crt_mode < 0) {
    const char* e = std::getenv("MOOSEX_GEMM_CRT");
    g_crt_mode = !e ? 0 : (e[0] == '0' ? 2 : (e[0] == '1' ? 1 : 0));
  }
  return g_crt_mode;
}

bool use_crt(int64_t M, int64_t N, int64_t K, int mode) {
  const int64_t kp = mode ? 2 * K : K;
  const int m = crt_mode();
  if (m == 2 || kp > 32768) return false;
  if (m == 1) return true;
  return M >= 256 && N >= 256 && kp >= 512;
}
}  // namespace

extern "C" {

void mx_set_gemm_crt(int mode) { g_crt_mode = mode; }

int64_t mx_gemm_workspace_bytes(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                                int mode) {
  if (words != 1 && words != 2) return 0;
  int64_t kk = std::min(K, max_k_chunk(words, mode));
  Plan p = make_plan(words, batch, M, N, kk, mode);
  return p.la_bytes + p.lb_bytes;
}

int mx_gemm_ws(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
               const void* A1, const void* B0, const void* B1, int mode, void* C,
               int accumulate, void* workspace, int64_t ws_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    return run<u64>(batch, M, N, K, (const u64*)A0, (const u64*)A1, (const u64*)B0,
                    (const u64*)B1, mode, (u64*)C, accumulate, workspace, ws_bytes, st);
  if (words == 2)
    return run<u128>(batch, M, N, K, (const u128*)A0, (const u128*)A1, (const u128*)B0,
                     (const u128*)B1, mode, (u128*)C, accumulate, workspace, ws_bytes, st);
  return -2;
}

// Prepared-B GEMM: the B' operand's limb planes are built once (mx_gemm_prep_b into a
// caller buffer of mx_gemm_b_bytes) and reused by several products with different A row
// blocks (mx_gemm_with_b; A given with a batch stride, so row blocks of a stacked
// [batch, M, K] tensor need no copy).  Used by the row-chunked dot pipeline.
int64_t mx_gemm_b_bytes(int words, int64_t batch, int64_t N, int64_t K, int mode) {
  if (words != 1 && words != 2) return 0;
  if (use_crt(256, N, K, mode)) return mxh_crt_b_bytes(words, batch, N, K, mode);
  if (K > max_k_chunk(words, mode)) return 0;
  return make_plan(words, batch, 64, N, K, mode).lb_bytes;
}

int mx_gemm_prep_b(int words, int64_t batch, int64_t K, int64_t N, const void* B0,
                   const void* B1, int mode, void* lb, void* stream) {
  if (use_crt(256, N, K, mode)) return mxh_crt_prep_b(words, batch, K, N, B0, B1, mode, lb, stream);
  if (K > max_k_chunk(words, mode)) return -6;
  Plan p = make_plan(words, batch, 64, N, K, mode);
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    launch_prep_b<u64>(p, batch, K, N, (const u64*)B0, (const u64*)B1, mode, (int8_t*)lb, st);
  else if (words == 2)
    launch_prep_b<u128>(p, batch, K, N, (const u128*)B0, (const u128*)B1, mode, (int8_t*)lb,
                        st);
  else
    return -2;
  hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

int mx_gemm_with_b(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                   const void* A1, int64_t a_bstride, int mode, const void* lb, void* C,
                   int accumulate, void* stream) {
  if (use_crt(256, N, K, mode))  // the prepared B' holds residues (same test as prep_b)
    return mxh_crt_with_b(words, batch, M, N, K, A0, A1, a_bstride, mode, lb, C, accumulate,
                          stream);
  if (K > max_k_chunk(words, mode)) return -6;
  Plan p = make_plan(words, batch, M, N, K, mode);
  void* la = get_workspace(p.la_bytes, (hipStream_t)stream);
  if (!la) return -4;
  hipStream_t st = (hipStream_t)stream;
  if (words == 1) {
    launch_prep_a<u64>(p, batch, M, K, (const u64*)A0, (const u64*)A1, a_bstride, mode,
                       (int8_t*)la, st);
    launch_gemm<u64>(p, batch, M, N, (const int8_t*)la, (const int8_t*)lb, (u64*)C, accumulate,
                     st);
  } else if (words == 2) {
    launch_prep_a<u128>(p, batch, M, K, (const u128*)A0, (const u128*)A1, a_bstride, mode,
                        (int8_t*)la, st);
    launch_gemm<u128>(p, batch, M, N, (const int8_t*)la, (const int8_t*)lb, (u128*)C,
                      accumulate, st);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

// Mode-1 product whose second A operand is the first rolled over the batch (a stacked RSS
// pair: A1[b] = A0[(b + roll) % batch]); lb: prepared B' (mx_gemm_prep_b) or null.  Runs
// on the CRT GEMM only; -7 (the caller falls back to the two-operand form) otherwise.
int mx_gemm_roll(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                 int64_t a_bstride, int64_t roll, const void* B0, const void* B1, const void* lb,
                 void* C, int accumulate, void* stream) {
  if (M == 0 || N == 0 || batch == 0) return 0;
  if ((words != 1 && words != 2) || !use_crt(lb ? 256 : M, N, K, 1)) return -7;
  return mxh_crt_roll(words, batch, M, N, K, A0, a_bstride, roll, B0, B1, lb, C, accumulate,
                      stream);
}

// Batched product with explicit batch strides (elements) for A and B (0 broadcasts).
int mx_gemm_strided(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                    const void* A1, int64_t a_bstride, const void* B0, const void* B1,
                    int64_t b_bstride, int mode, void* C, int accumulate, void* stream) {
  if (M == 0 || N == 0 || batch == 0) return 0;
  if (words != 1 && words != 2) return -2;
  if (use_crt(M, N, K, mode))
    return mxh_gemm_crt_strided(words, batch, M, N, K, A0, A1, a_bstride, B0, B1, b_bstride,
                                mode, C, accumulate, stream);
  if (K > max_k_chunk(words, mode)) return -6;
  Plan p = make_plan(words, batch, M, N, K, mode);
  void* ws = get_workspace(p.la_bytes + p.lb_bytes, (hipStream_t)stream);
  if (!ws) return -4;
  int8_t* la = (int8_t*)ws;
  int8_t* lb = la + p.la_bytes;
  hipStream_t st = (hipStream_t)stream;
  if (words == 1) {
    launch_prep_a<u64>(p, batch, M, K, (const u64*)A0, (const u64*)A1, a_bstride, mode, la, st);
    launch_prep_b<u64>(p, batch, K, N, (const u64*)B0, (const u64*)B1, mode, lb, st, b_bstride);
    launch_gemm<u64>(p, batch, M, N, la, lb, (u64*)C, accumulate, st);
  } else {
    launch_prep_a<u128>(p, batch, M, K, (const u128*)A0, (const u128*)A1, a_bstride, mode, la,
                        st);
    launch_prep_b<u128>(p, batch, K, N, (const u128*)B0, (const u128*)B1, mode, lb, st,
                        b_bstride);
    launch_gemm<u128>(p, batch, M, N, la, lb, (u128*)C, accumulate, st);
  }
  hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

int mxh_gemm_mfma(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                  const void* A1, const void* B0, const void* B1, int mode, void* C,
                  int accumulate, void* stream) {
  if (use_crt(M, N, K, mode))
    return mxh_gemm_crt(words, batch, M, N, K, A0, A1, B0, B1, mode, C, accumulate, stream);
  if (K > max_k_chunk(words, mode)) return -6;  // caller splits long K
  int64_t bytes = mx_gemm_workspace_bytes(words, batch, M, N, K, mode);
  void* ws = get_workspace(bytes, (hipStream_t)stream);
  if (!ws) return -4;
  return mx_gemm_ws(words, batch, M, N, K, A0, A1, B0, B1, mode, C, accumulate, ws, bytes,
                    stream);
}

}  // extern "C"
