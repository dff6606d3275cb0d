// gfx950 kernels for the moosex ring dialect: elementwise Z_2^64 / Z_2^128 / Z_2 ops,
// the ChaCha12 correlated-randomness generator (prf_core.h), the fused RSS local step
// (cross terms + zero share in one pass), fixed-point encode/decode, reductions.
//
// Design notes (MI355X):
//  * every elementwise kernel is a grid-stride loop over 16-byte elements (one u128, two
//    u64) so each lane issues dwordx4 loads; the grid is capped at 256 CUs x 8 blocks.
//  * the PRF is ChaCha12 (VALU add/rotate/xor, no tables): a thread computes one 64-byte
//    block and hands its four 16-byte chunks to elements 64 chunks apart; one chunk yields
//    one u128 / two u64 / sixteen bits.
//  * the fused RSS kernel (mxh_rss_cross) reads the four share streams once and writes
//    z_i + alpha_i once: the whole local half of an RSS multiplication is one launch, for
//    all three parties at once when they are stacked on one device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "prf_dev.h"
#include "moosex.h"
#include "party_batch.h"
#include "ring_common.h"
#include "rss_fused.h"

using mxr::u128;
using u64 = uint64_t;

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n, int per_thread = 1) {
  int64_t blocks = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
  return (int)std::max<int64_t>(1, std::min<int64_t>(blocks, 256 * 8));
}

inline hipStream_t S(void* s) { return (hipStream_t)s; }

#define MX_LAUNCH_CHECK()                               \
  do {                                                  \
    hipError_t _e = hipGetLastError();                  \
    if (_e != hipSuccess) return -100 - (int)_e;        \
  } while (0)

template <class T>
__device__ __forceinline__ void d_binary(int op, const T* __restrict__ a, int64_t na,
                                         const T* __restrict__ b, int64_t nb, T* __restrict__ out,
                                         int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = mxr::binop<T>(op, a[na == 1 ? 0 : i], b[nb == 1 ? 0 : i]);
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_binary(int op, const T* __restrict__ a, int64_t na,
                                                const T* __restrict__ b, int64_t nb,
                                                T* __restrict__ out, int64_t n) {
  d_binary<T>(op, a, na, b, nb, out, n);
}

template <class T>
__device__ __forceinline__ void d_binary_slot(int op, const T* __restrict__ a,
                                              const T* __restrict__ b, int64_t nb,
                                              T* __restrict__ out, int64_t m, int np, int which) {
  const int64_t n = m * np;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = g / m, i = g - p * m;
    out[g] = p == which ? mxr::binop<T>(op, a[g], b[nb == 1 ? 0 : i % nb]) : a[g];
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_binary_slot(int op, const T* __restrict__ a,
                                                     const T* __restrict__ b, int64_t nb,
                                                     T* __restrict__ out, int64_t m, int np,
                                                     int which) {
  d_binary_slot<T>(op, a, b, nb, out, m, np, which);
}

// Share-pair forms: both replicated share vectors (s0, s1) of a share-wise op in ONE launch,
// blockIdx.y picks the pair member.
template <class T>
struct Pair {
  const T* a[2];
  const T* b[2];
  T* o[2];
  int which[2];
};

template <class T>
__device__ __forceinline__ void d_binary2(int op, const Pair<T>& p, int64_t na, int64_t nb,
                                          int64_t n) {
  const int y = blockIdx.y;
  const T* __restrict__ a = p.a[y];
  const T* __restrict__ b = p.b[y];
  T* __restrict__ out = p.o[y];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mxr::binop<T>(op, a[na == 1 ? 0 : i], b[nb == 1 ? 0 : i]);
}

template <class T>
__global__ void __launch_bounds__(256) k_binary2(int op, Pair<T> p, int64_t na, int64_t nb,
                                                 int64_t n) {
  d_binary2<T>(op, p, na, nb, n);
}

template <class T>
__device__ __forceinline__ void d_unary2(int op, const Pair<T>& p, int64_t n, int k) {
  const int y = blockIdx.y;
  const T* __restrict__ a = p.a[y];
  T* __restrict__ out = p.o[y];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mxr::unop<T>(op, a[i], k);
}

template <class T>
__global__ void __launch_bounds__(256) k_unary2(int op, Pair<T> p, int64_t n, int k) {
  d_unary2<T>(op, p, n, k);
}

// out_y = a_y^T for a party's two share components ([rows, cols] -> [cols, rows]): 32 x 32
// tiles through LDS (rows read and written whole); tile = blockIdx.x, component = blockIdx.y
// (blockIdx.z stays free for the party-batched twin)
template <class T>
__device__ __forceinline__ void d_transpose2(const Pair<T>& p, int64_t rows, int64_t cols) {
  __shared__ T tile[32][33];
  const T* __restrict__ a = p.a[blockIdx.y];
  T* __restrict__ out = p.o[blockIdx.y];
  const int64_t tiles_c = (cols + 31) / 32;
  const int64_t r0 = (blockIdx.x / tiles_c) * 32, c0 = (blockIdx.x % tiles_c) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 lanes: 8 rows per pass
  for (int r = ty; r < 32; r += 8)
    if (r0 + r < rows && c0 + tx < cols) tile[r][tx] = a[(r0 + r) * cols + c0 + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8)
    if (c0 + r < cols && r0 + tx < rows) out[(c0 + r) * rows + r0 + tx] = tile[tx][r];
}

template <class T>
__global__ void __launch_bounds__(256) k_transpose2(Pair<T> p, int64_t rows, int64_t cols) {
  d_transpose2<T>(p, rows, cols);
}

// public b applied to party slot which[y] of stacked a[y] ([np, m]), other slots copied
template <class T>
__device__ __forceinline__ void d_binary_slot2(int op, const Pair<T>& p, int64_t nb, int64_t m,
                                               int np) {
  const int y = blockIdx.y;
  const T* __restrict__ a = p.a[y];
  const T* __restrict__ b = p.b[0];
  T* __restrict__ out = p.o[y];
  const int which = p.which[y];
  const int64_t n = m * np;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = g / m, i = g - q * m;
    out[g] = q == which ? mxr::binop<T>(op, a[g], b[nb == 1 ? 0 : i % nb]) : a[g];
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_binary_slot2(int op, Pair<T> p, int64_t nb, int64_t m,
                                                      int np) {
  d_binary_slot2<T>(op, p, nb, m, np);
}

// out = a + b + c (a reveal: the holder's two shares plus the received third)
template <class T>
__global__ void __launch_bounds__(256) k_add3(const T* __restrict__ a, const T* __restrict__ b,
                                              const T* __restrict__ c, T* __restrict__ out,
                                              int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a[i] + b[i] + c[i];
}

// Share-wise linear combination of up to three replicated values, both share vectors in one
// launch: out_y = sum_t coef[t] * in_t[y] (+ public b at party slot which[y], period nb).
template <class T>
struct Lin3 {
  const T* a[3][2];
  T* o[2];
  int64_t coef[3];
  int which[2];
};

template <class T>
__device__ __forceinline__ void d_lincomb2(const Lin3<T>& p, int nin, const T* __restrict__ b,
                                           int64_t nb, int64_t m, int np) {
  const int y = blockIdx.y;
  T* __restrict__ out = p.o[y];
  const int which = p.which[y];
  const int64_t n = m * np;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    T v = (T)(int64_t)p.coef[0] * p.a[0][y][g];
    if (nin > 1) v += (T)(int64_t)p.coef[1] * p.a[1][y][g];
    if (nin > 2) v += (T)(int64_t)p.coef[2] * p.a[2][y][g];
    if (b != nullptr) {
      const int64_t q = g / m, i = g - q * m;
      if (q == which) v += b[nb == 1 ? 0 : i % nb];
    }
    out[g] = v;
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_lincomb2(Lin3<T> p, int nin, const T* __restrict__ b,
                                                  int64_t nb, int64_t m, int np) {
  d_lincomb2<T>(p, nin, b, nb, m, np);
}

// AddN of k replicated values that are evenly spaced views of one stack (the products of a
// batched Dot): out_y[p, e] = sum_t base_y[t * is_y + p * ps_y + e], both share vectors in
// one launch.
template <class T>
struct SumViews {
  const T* base[2];
  T* o[2];
  int64_t is[2];
  int64_t ps[2];
};

template <class T>
__device__ __forceinline__ void d_sum_views2(const SumViews<T>& p, int k, int64_t m, int np) {
  const int y = blockIdx.y;
  const T* __restrict__ base = p.base[y];
  T* __restrict__ out = p.o[y];
  const int64_t is = p.is[y], ps = p.ps[y];
  const int64_t n = m * np;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = g / m, e = g - q * m;
    const T* src = base + q * ps + e;
    T acc = 0;
    for (int t = 0; t < k; ++t) acc += src[(int64_t)t * is];
    out[g] = acc;
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_sum_views2(SumViews<T> p, int k, int64_t m, int np) {
  d_sum_views2<T>(p, k, m, np);
}

// trivial sharings in the stacked layout: out_y[q, i] = q == which[y] ? a[y][i] : 0
template <class T>
__device__ __forceinline__ void d_slot_place2(const Pair<T>& p, int64_t m, int np) {
  const int y = blockIdx.y;
  const T* __restrict__ a = p.a[y];
  T* __restrict__ out = p.o[y];
  const int which = p.which[y];
  const int64_t n = m * np;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = g / m, i = g - q * m;
    out[g] = q == which ? a[i] : (T)0;
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_slot_place2(Pair<T> p, int64_t m, int np) {
  d_slot_place2<T>(p, m, np);
}

template <class T>
__global__ void __launch_bounds__(256) k_add_zs3(const T* __restrict__ v, const T* __restrict__ r,
                                                 T* __restrict__ out0, T* __restrict__ out1,
                                                 int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const T r0 = r[e], r1 = r[n + e], r2 = r[2 * n + e];
    const T z0 = v[e] + r0 - r1, z1 = v[n + e] + r1 - r2, z2 = v[2 * n + e] + r2 - r0;
    out0[e] = z0;
    out0[n + e] = z1;
    out0[2 * n + e] = z2;
    out1[e] = z1;
    out1[n + e] = z2;
    out1[2 * n + e] = z0;
  }
}

template <class T>
__device__ __forceinline__ void d_unary(int op, const T* __restrict__ a, T* __restrict__ out,
                                        int64_t n, int k) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mxr::unop<T>(op, a[i], k);
}

template <class T>
__global__ void __launch_bounds__(256) k_unary(int op, const T* __restrict__ a, T* __restrict__ out,
                                               int64_t n, int k) {
  d_unary<T>(op, a, out, n, k);
}

template <class T>
__device__ __forceinline__ void d_fill(T* __restrict__ out, int64_t n, uint64_t lo, uint64_t hi) {
  T v;
  if constexpr (sizeof(T) == 16) {
    v = ((T)hi << 64) | (T)lo;
  } else {
    v = (T)lo;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = v;
}

template <class T>
__global__ void __launch_bounds__(256) k_fill(T* __restrict__ out, int64_t n, uint64_t lo,
                                              uint64_t hi) {
  d_fill<T>(out, n, lo, hi);
}

// out[o, j, i] = bit (start + j) of a[o, i] as a 0/1 byte (bit decomposition / split)
template <class T>
__device__ __forceinline__ void d_bit_planes(const T* __restrict__ a, uint8_t* __restrict__ out,
                                             int64_t outer, int64_t inner, int start, int count) {
  const int64_t n = outer * inner;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = g / inner, i = g - o * inner;
    const T v = a[g];
    uint8_t* dst = out + o * count * inner + i;
    for (int j = 0; j < count; ++j) dst[(int64_t)j * inner] = (uint8_t)((v >> (start + j)) & 1);
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_bit_planes(const T* __restrict__ a,
                                                    uint8_t* __restrict__ out, int64_t outer,
                                                    int64_t inner, int start, int count) {
  d_bit_planes<T>(a, out, outer, inner, start, count);
}

// out[o, i] = sum_j w[j] * a[o, j, i]  (public ring weights, bit composition)
template <class T>
__global__ void __launch_bounds__(256) k_weighted_sum(const T* __restrict__ a,
                                                      const T* __restrict__ w, 
                               T* __restrict__ out, int64_t outer, int64_t k, int64_t inner) {
  const int64_t n = outer * inner;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = g / inner, i = g - o * inner;
    const T* src = a + o * k * inner + i;
    // independent partial sums so the k loads of a thread are in flight together
    T acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t j = 0;
    for (; j + 8 <= k; j += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += w[j + u] * src[(j + u) * inner];
    }
    for (; j < k; ++j) acc[0] += w[j] * src[j * inner];
    out[g] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
}

// k_weighted_sum for latency-bound launches with a long reduction: G threads per output,
// each summing every G-th term (all k loads of an output in flight at once), then a
// tree over the G partials in LDS.  Ring sums: any order gives the same value.
template <class T, int G = 8>
__global__ void __launch_bounds__(256) k_weighted_sum_wide(const T* __restrict__ a,
                                                           const T* __restrict__ w,
                                                           T* __restrict__ out, int64_t outer,
                                                           int64_t k, int64_t inner) {
  __shared__ T part[256];
  const int64_t n = outer * inner;
  const int lane = threadIdx.x % G;
  for (int64_t g0 = (int64_t)blockIdx.x * (256 / G); g0 < n; g0 += (int64_t)gridDim.x * (256 / G)) {
    const int64_t g = g0 + threadIdx.x / G;
    T acc = 0;
    if (g < n) {
      const int64_t o = g / inner, i = g - o * inner;
      const T* src = a + o * k * inner + i;
      for (int64_t j = lane; j < k; j += G) acc += w[j] * src[j * inner];
    }
    part[threadIdx.x] = acc;
    __syncthreads();
#pragma unroll
    for (int h = G / 2; h > 0; h /= 2) {
      if (lane < h) part[threadIdx.x] += part[threadIdx.x + h];
      __syncthreads();
    }
    if (lane == 0 && g < n) out[g] = part[threadIdx.x];
    __syncthreads();
  }
}

template <class T>
__device__ __forceinline__ void d_compare(int op, const T* __restrict__ a, int64_t na,
                                          const T* __restrict__ b, int64_t nb,
                                          uint8_t* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mxr::cmpop<T>(op, a[na == 1 ? 0 : i], b ? b[nb == 1 ? 0 : i] : (T)0);
}

template <class T>
__global__ void __launch_bounds__(256) k_compare(int op, const T* __restrict__ a, int64_t na,
                                                 const T* __restrict__ b, int64_t nb,
                                                 uint8_t* __restrict__ out, int64_t n) {
  d_compare<T>(op, a, na, b, nb, out, n);
}

template <class T>
__device__ __forceinline__ void d_bit_extract(const T* __restrict__ a, uint8_t* __restrict__ out,
                                              int64_t n, int bit) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint8_t)((a[i] >> bit) & 1);
}

template <class T>
__global__ void __launch_bounds__(256) k_bit_extract(const T* __restrict__ a,
                                                     uint8_t* __restrict__ out, int64_t n,
                                                     int bit) {
  d_bit_extract<T>(a, out, n, bit);
}

template <class T>
__device__ __forceinline__ void d_ring_inject(const uint8_t* __restrict__ bits, T* __restrict__ out,
                                              int64_t n, int bit) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = ((T)(bits[i] & 1)) << bit;
}

template <class T>
__global__ void __launch_bounds__(256) k_ring_inject(const uint8_t* __restrict__ bits,
                                                     T* __restrict__ out, int64_t n, int bit) {
  d_ring_inject<T>(bits, out, n, bit);
}

// The local half of rep.b2a for three stacked parties, one launch: from the bit sharing
// (s0, s1 party vectors [3][n], P_p holding (b_p, b_{p+1})) P0's a = b_0 ^ b_1 as a ring
// value (to be shared by P0) and the trivial sharing B of b_2 (slot 2: P2's s0 and P1's s1)
// -- the values of the Xor + RingInject x 3 + slot placement it replaces.
template <class T>
__global__ void __launch_bounds__(256) k_b2a_prep3(const uint8_t* __restrict__ s0,
                                                   const uint8_t* __restrict__ s1, int64_t n,
                                                   T* __restrict__ a, T* __restrict__ b0,
                                                   T* __restrict__ b1) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    a[e] = (T)((s0[e] ^ s1[e]) & 1);
    const T x2 = (T)(s0[2 * n + e] & 1), x2b = (T)(s1[n + e] & 1);
    b0[e] = 0;
    b0[n + e] = 0;
    b0[2 * n + e] = x2;
    b1[e] = 0;
    b1[n + e] = x2b;
    b1[2 * n + e] = 0;
  }
}

// The whole of rep.b2a for three stacked parties in ONE launch: P0 shares a = b_0 ^ b_1
// (the sharing mask r = PRF(k_mir, n1); slots (r, a - r, 0), mirrored (a - r, r, 0)), the
// product of that sharing with the trivial sharing of b_2 (slot 2) and its zero share
// PRF(k_p, nmul) - PRF(k_{p+1}, nmul), and the lincomb A + B - 2 AB.  With A_2 = B_0 = B_1 =
// 0 the cross terms are c_0 = 0, c_1 = A_1 b_2, c_2 = A_0 b_2.  Four keystream chunks per
// chunk position, one per thread into LDS (as k_rss_cross_ring3_lat), then EPB threads
// finish the elements: bitwise the shares of b2a_prep3 + share3 + rss_mul3 + lincomb2.
// With pw0 (k_b2a3 over bit planes): the bits are read from packed boolean share words
// [3][m] (T) instead of bit tensors -- element e = j * m + i is bit start + j of word i (the
// BitSplit planes [3][count][m] it replaces).
template <class T>
__global__ void __launch_bounds__(256) k_b2a3(const uint8_t* __restrict__ s0,
                                              const uint8_t* __restrict__ s1,
                                              T* __restrict__ out0, T* __restrict__ out1,
                                              int64_t n, mxd::KeySrc keys, int mir, uint64_t n1,
                                              uint64_t nmul, const T* __restrict__ pw0 = nullptr,
                                              const T* __restrict__ pw1 = nullptr,
                                              int start = 0, int64_t m = 1) {
  constexpr int EPB = 64;
  __shared__ uint32_t rks[3][mxd::kKeyWords];
  __shared__ uint64_t kl[4][EPB], kh[4][EPB];
  mxd::stage_keys(rks, keys, 3);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  const int key_of = s < 3 ? s : mir;  // s < 3: the product's zero share; 3: the mask
  const uint64_t nonce_of = s < 3 ? nmul : n1;
  const bool r4 = out1 == out0 + n;  // 4-slot ring: out1's slots 0, 1 are out0's 1, 2
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    // the finishing threads' bits first: their loads overlap the keystream work
    const bool fin = tid < EPB && b0 + tid < nb;
    uint8_t ba[P], bx[P], by[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t e = (b0 + tid) * P + j;
      const bool ok = fin && e < n;
      if (pw0 != nullptr) {  // bit start + e / m of packed word e % m
        const int64_t pj = ok ? e / m : 0, pi = ok ? e - pj * m : 0;
        const int sh = start + (int)pj;
        ba[j] = ok ? (uint8_t)(((pw0[pi] ^ pw1[pi]) >> sh) & 1) : 0;
        bx[j] = ok ? (uint8_t)((pw0[2 * m + pi] >> sh) & 1) : 0;
        by[j] = ok ? (uint8_t)((pw1[m + pi] >> sh) & 1) : 0;
      } else {
        ba[j] = ok ? (uint8_t)(s0[e] ^ s1[e]) : 0;
        bx[j] = ok ? s0[2 * n + e] : 0;
        by[j] = ok ? s1[n + e] : 0;
      }
    }
    if (b0 + lb < nb) {
      uint64_t lo, hi;
      mxd::prf_chunk(rks[key_of], nonce_of, (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    __syncthreads();
    if (fin) {
      const int64_t b = b0 + tid;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t e = b * P + j;
        if (e >= n) break;
        const T a = (T)(ba[j] & 1);
        const T x2 = (T)(bx[j] & 1), x2b = (T)(by[j] & 1);  // P2's, P1's b_2
        const T r = mxd::pick<T>(kl[3][tid], kh[3][tid], j);
        const T v = a - r;
        const T A0 = mir ? v : r, A1 = mir ? r : v;
        const T k0 = mxd::pick<T>(kl[0][tid], kh[0][tid], j);
        const T k1 = mxd::pick<T>(kl[1][tid], kh[1][tid], j);
        const T k2 = mxd::pick<T>(kl[2][tid], kh[2][tid], j);
        const T z0 = k0 - k1, z1 = A1 * x2b + k1 - k2, z2 = A0 * x2 + k2 - k0;
        const T o[3] = {(T)(A0 - (z0 << 1)), (T)(A1 - (z1 << 1)), (T)(x2 - (z2 << 1))};
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          out0[p * n + e] = o[p];
          if (!r4 || p == 2) out1[p * n + e] = o[p == 2 ? 0 : p + 1];
        }
      }
    }
    __syncthreads();
  }
}

template <class T>
__device__ __forceinline__ void d_encode(const double* __restrict__ x, T* __restrict__ out,
                                         int64_t n, double scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (T)mxr::f64_to_i128(x[i] * scale);
}

template <class T>
__global__ void __launch_bounds__(256) k_encode(const double* __restrict__ x, T* __restrict__ out,
                                                int64_t n, double scale) {
  d_encode<T>(x, out, n, scale);
}

template <class T>
__device__ __forceinline__ void d_decode(const T* __restrict__ x, double* __restrict__ out,
                                         int64_t n, double scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (sizeof(T) == 8)
      out[i] = (double)(int64_t)x[i] * scale;
    else
      out[i] = mxr::i128_to_f64(x[i]) * scale;
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_decode(const T* __restrict__ x, double* __restrict__ out,
                                                int64_t n, double scale) {
  d_decode<T>(x, out, n, scale);
}

// decode(a + b + c [+ d]): the reveal's add and the decode in one pass (no ring-valued sum in
// HBM); d may be null
template <class T>
__device__ __forceinline__ void d_addn_decode(const T* __restrict__ a, const T* __restrict__ b,
                                              const T* __restrict__ c, const T* __restrict__ d,
                                              double* __restrict__ out, int64_t n, double scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    T v = a[i] + b[i] + c[i];
    if (d != nullptr) v += d[i];
    if constexpr (sizeof(T) == 8)
      out[i] = (double)(int64_t)v * scale;
    else
      out[i] = mxr::i128_to_f64(v) * scale;
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_addn_decode(const T* __restrict__ a,
                                                     const T* __restrict__ b,
                                                     const T* __restrict__ c,
                                                     const T* __restrict__ d,
                                                     double* __restrict__ out, int64_t n,
                                                     double scale) {
  d_addn_decode<T>(a, b, c, d, out, n, scale);
}

// one thread per output when the reduced axis is short; a block per output otherwise
template <class T>
__device__ __forceinline__ void d_sum_axis(const T* __restrict__ a, T* __restrict__ out,
                                           int64_t outer, int64_t red, int64_t inner) {
  int64_t total = outer * inner;
  for (int64_t oi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; oi < total;
       oi += (int64_t)gridDim.x * blockDim.x) {
    int64_t o = oi / inner, i = oi % inner;
    const T* p = a + o * red * inner + i;
    T acc[4] = {0, 0, 0, 0};
    int64_t r = 0;
    for (; r + 4 <= red; r += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += p[(r + u) * inner];
    }
    for (; r < red; ++r) acc[0] += p[r * inner];
    out[oi] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_sum_axis(const T* __restrict__ a, T* __restrict__ out,
                                                  int64_t outer, int64_t red, int64_t inner) {
  d_sum_axis<T>(a, out, outer, red, inner);
}

template <class T>
__global__ void __launch_bounds__(256) k_sum_axis_wide(const T* __restrict__ a, T* __restrict__ out,
                                                       int64_t red, 
                                int64_t inner) {
  __shared__ T part[kBlock];
  int64_t oi = blockIdx.x;
  int64_t o = oi / inner, i = oi % inner;
  const T* p = a + o * red * inner + i;
  T acc = 0;
  for (int64_t r = threadIdx.x; r < red; r += blockDim.x) acc += p[r * inner];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[oi] = part[0];
}

// ---------------------------------------------------------------------------
// PRF (ChaCha12 keystream, prf_core.h / prf_dev.h)
// ---------------------------------------------------------------------------
using mxd::KeySrc;
using mxd::Lane;
using mxd::pick;
using mxd::stage_keys;
using mxd::prf_chunk;
using mxd::kKeyWords;

struct RawKey {
  uint32_t k[kKeyWords];
};

// raw keystream bytes from chunk ctr0 on (random access per chunk; tests and tools only)
__global__ void __launch_bounds__(256) k_prg(RawKey key, uint64_t nonce, uint64_t ctr0,
                                             uint8_t* __restrict__ out, int64_t nbytes) {
  int64_t nblocks = (nbytes + 15) / 16;
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nblocks;
       b += (int64_t)gridDim.x * blockDim.x) {
    uint64_t lo, hi;
    prf_chunk(key.k, nonce, ctr0 + b, &lo, &hi);
    if ((b + 1) * 16 <= nbytes) {
      uint64_t* o = (uint64_t*)(out + b * 16);
      o[0] = lo;
      o[1] = hi;
    } else {
      uint8_t tmp[16];
      memcpy(tmp, &lo, 8);
      memcpy(tmp + 8, &hi, 8);
      for (int64_t j = 0; j < nbytes - b * 16; ++j) out[b * 16 + j] = tmp[j];
    }
  }
}

// Element e of type T lives in keystream chunk e / (16 / sizeof(T)).  A thread computes one
// ChaCha block per key and finishes the block's four chunks (64 chunks apart); g walks
// (party, block).  Keys are staged in LDS (from launch parameters or from key slots in
// device memory, see prf_dev.h).
template <class T>
__device__ __forceinline__ void d_rss_cross(int kind, const T* __restrict__ x0,
                                            const T* __restrict__ x1, const T* __restrict__ y0,
                                            const T* __restrict__ y1, T* __restrict__ out,
                                            int64_t n, int nparties, int has_keys,
                                            const KeySrc& keys, uint64_t nonce, int pairs) {
  // pairs == 0: party p uses keys p and p+1 (one session, shared ring of keys);
  // pairs == 1: party p uses keys 2p and 2p+1 (parties of independent sessions)
  __shared__ uint32_t rks[mxd::kMaxKeySlots][kKeyWords];
  if (has_keys) stage_keys(rks, keys, pairs ? 2 * nparties : nparties + 1);
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;  // keystream chunks per party
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)nb);
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nblk * nparties;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - p * nblk);
    uint32_t wa[16], wb[16];
    if (has_keys) {
      const int ka = pairs ? 2 * p : p;
      mx::chacha_block(rks[ka], nonce, B, wa);
      mx::chacha_block(rks[ka + 1], nonce, B, wb);
    }
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int64_t b = (int64_t)mx::ks_chunk(B, part);
      if (b >= nb) break;
      uint64_t alo = 0, ahi = 0, blo = 0, bhi = 0;
      if (has_keys) {
        mx::part_u64(wa, part, &alo, &ahi);
        mx::part_u64(wb, part, &blo, &bhi);
      }
#pragma unroll
      for (int j = 0; j < P; ++j) {
        int64_t e = b * P + j;
        if (e >= n) break;
        int64_t i = (int64_t)p * n + e;
        T v = 0;
        if (x0 != nullptr && y0 != nullptr)
          v = mxr::cross<T>(kind, x0[i], x1 ? x1[i] : (T)0, y0[i], y1 ? y1[i] : (T)0,
                            x1 != nullptr, y1 != nullptr);
        else if (x0 != nullptr)
          v = x0[i];  // add-zero-share mode
        if (has_keys) v = mxr::zs_combine<T>(kind, v, pick<T>(alo, ahi, j), pick<T>(blo, bhi, j));
        out[i] = v;
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_rss_cross(int kind, const T* __restrict__ x0,
                                                   const T* __restrict__ x1,
                                                   const T* __restrict__ y0,
                                                   const T* __restrict__ y1, T* __restrict__ out,
                                                   int64_t n, int nparties, int has_keys,
                                                   KeySrc keys, uint64_t nonce, int pairs) {
  d_rss_cross<T>(kind, x0, x1, y0, y1, out, n, nparties, has_keys, keys, nonce, pairs);
}

// Operand layouts of the stacked multiplication kernels: operand k of party p, element e is
// ptr_k[p * ps[k] + e % per[k]] -- a slice along the first logical axis (party stride !=
// n) or a broadcast of one row over it (per = row size) without materialising the view.
// strided == 0: every operand is a contiguous [3, n] vector (ps = per = n).
struct Views {
  int64_t ps[4];
  int64_t per[4];
  int strided;
};

template <class T>
__device__ __forceinline__ T ld_view(const T* __restrict__ a, const Views& v, int k, int p,
                                     int64_t e, int64_t n) {
  if (!v.strided) return a[(int64_t)p * n + e];
  return a[(int64_t)p * v.ps[k] + (v.per[k] == n ? e : e % v.per[k])];
}

// Stacked three-party ring (keys k0, k1, k2, k3 == k0): party p needs PRF(k_p) and
// PRF(k_{p+1}), so each of the three keystreams is used by two parties.  One thread per
// ChaCha block evaluates the three keys' blocks once and finishes all three parties'
// elements of the block's chunks (the shares are identical to k_rss_cross).
template <class T>
__global__ void __launch_bounds__(256) k_rss_cross_ring3(int kind, const T* __restrict__ x0,
                                                         const T* __restrict__ x1, 
                                  const T* __restrict__ y0, const T* __restrict__ y1,
                                  T* __restrict__ out, T* __restrict__ out1, int64_t n,
                                  KeySrc keys, uint64_t nonce, Views vw) {
  __shared__ uint32_t rks[3][kKeyWords];
  stage_keys(rks, keys, 3);
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const uint32_t* const key[3] = {rks[0], rks[1], rks[2]};
  const uint64_t nn[3] = {nonce, nonce, nonce};
  mxd::walk_chunks<3>(nb, key, nn, [&](int64_t b, const uint64_t (&lo)[3], const uint64_t (&hi)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int q = p == 2 ? 0 : p + 1;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t e = b * P + j;
        if (e >= n) break;
        const int64_t i = (int64_t)p * n + e;
        T v = 0;
        if (x0 != nullptr && y0 != nullptr)
          v = mxr::cross<T>(kind, ld_view(x0, vw, 0, p, e, n), x1 ? ld_view(x1, vw, 1, p, e, n) : (T)0,
                            ld_view(y0, vw, 2, p, e, n), y1 ? ld_view(y1, vw, 3, p, e, n) : (T)0,
                            x1 != nullptr, y1 != nullptr);
        else if (x0 != nullptr)
          v = ld_view(x0, vw, 0, p, e, n);
        const T z = mxr::zs_combine<T>(kind, v, pick<T>(lo[p], hi[p], j), pick<T>(lo[q], hi[q], j));
        out[i] = z;
        // fused reshare: z_p is party p-1's second share
        if (out1 != nullptr) out1[(int64_t)(p == 0 ? 2 : p - 1) * n + e] = z;
      }
    }
  });
}

// One Kogge-Stone level for the three stacked parties (see mx_ks_level3_k).  A block
// handles EPB elements: its NS = 3 (t) or 6 (t and pk') keystream values per element are
// computed one PRF chunk per thread into LDS (one PRF on the critical path), then EPB
// threads finish all three parties' shares and write the reshared outputs directly.
template <class T>
__global__ void __launch_bounds__(256) k_ks_level3(const T* __restrict__ g0,
                                                   const T* __restrict__ g1, 
                                                   const T* __restrict__ p0, const T* __restrict__ p1,
                                                   T* __restrict__ og0, T* __restrict__ og1,
                                                   T* __restrict__ op0, T* __restrict__ op1,
                                                   int64_t n, int d, int both, KeySrc keys,
                                                   uint64_t nonce) {
  constexpr int EPB = 256 / 6;
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ T ks[6][EPB];
  stage_keys(rks, keys, 3);
  constexpr int P = Lane<T>::kPer;
  const int NS = both ? 6 : 3;
  const int tid = threadIdx.x, s = tid / EPB, le = tid % EPB;
  for (int64_t e0 = (int64_t)blockIdx.x * EPB; e0 < n; e0 += (int64_t)gridDim.x * EPB) {
    if (s < NS && e0 + le < n) {
      const int64_t c = (s < 3 ? 0 : n) + e0 + le;  // t at e, pk' at n + e
      uint64_t lo, hi;
      prf_chunk(rks[s % 3], nonce, (uint64_t)(c / P), &lo, &hi);
      ks[s][le] = pick<T>(lo, hi, (int)(c % P));
    }
    __syncthreads();
    const int64_t e = e0 + tid;
    if (tid < EPB && e < n) {
      T t[3], q[3], gv0[3], gv1[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int64_t i = (int64_t)p * n + e;
        gv0[p] = g0[i];
        gv1[p] = g1[i];
        const T a0 = p0[i], a1 = p1[i];
        const T s0 = gv0[p] << d, s1 = gv1[p] << d;
        const int pn = p == 2 ? 0 : p + 1;
        t[p] = (a0 & s0) ^ (a0 & s1) ^ (a1 & s0) ^ ks[p][tid] ^ ks[pn][tid];
        if (both) {
          const T u0 = a0 << d, u1 = a1 << d;
          q[p] = (a0 & u0) ^ (a0 & u1) ^ (a1 & u0) ^ ks[3 + p][tid] ^ ks[3 + pn][tid];
        } else {
          q[p] = 0;
        }
      }
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int64_t i = (int64_t)p * n + e;
        const int pn = p == 2 ? 0 : p + 1;
        og0[i] = gv0[p] ^ t[p];
        og1[i] = gv1[p] ^ t[pn];
        if (both) {
          op0[i] = q[p];
          op1[i] = q[pn];
        }
      }
    }
    __syncthreads();
  }
}

// The whole Kogge-Stone carry chain of rep.binary_adder for three stacked parties: the
// levels d = 1, 2, 4, ... of k_ks_level3 in ONE launch (a level is element-local: its
// shifts stay inside an element's packed bits, its reshare inside the stack), g and p held
// in registers between levels; level l draws its masks at nonce nn[l] exactly as
// k_ks_level3 does, so the result is bitwise the per-level chain's.  Returns the final g.
struct Nonces8 {
  uint64_t v[8];
};

template <class T>
__global__ void __launch_bounds__(256) k_ks_adder3(const T* __restrict__ g0,
                                                   const T* __restrict__ g1, 
                                                   const T* __restrict__ p0, const T* __restrict__ p1,
                                                   T* __restrict__ og0, T* __restrict__ og1,
                                                   int64_t n, int nlev, KeySrc keys, Nonces8 nn,
                                                   int sum_out) {
  constexpr int EPB = 256 / 6;
  constexpr int W = 8 * (int)sizeof(T);
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ T ks[6][EPB];
  stage_keys(rks, keys, 3);
  constexpr int P = Lane<T>::kPer;
  const int tid = threadIdx.x, s = tid / EPB, le = tid % EPB;
  for (int64_t e0 = (int64_t)blockIdx.x * EPB; e0 < n; e0 += (int64_t)gridDim.x * EPB) {
    const int64_t e = e0 + tid;
    const bool act = tid < EPB && e < n;
    T G0[3], G1[3], A0[3], A1[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int64_t i = (int64_t)p * n + e;
      G0[p] = act ? g0[i] : (T)0;
      G1[p] = act ? g1[i] : (T)0;
      A0[p] = act ? p0[i] : (T)0;
      A1[p] = act ? p1[i] : (T)0;
    }
    int d = 1;
    for (int lev = 0; lev < nlev; ++lev, d *= 2) {
      const bool both = 2 * d < W;
      const int NS = both ? 6 : 3;
      if (s < NS && e0 + le < n) {
        const int64_t c = (s < 3 ? 0 : n) + e0 + le;  // t at e, pk' at n + e
        uint64_t lo, hi;
        prf_chunk(rks[s % 3], nn.v[lev], (uint64_t)(c / P), &lo, &hi);
        ks[s][le] = pick<T>(lo, hi, (int)(c % P));
      }
      __syncthreads();
      if (act) {
        T t[3], q[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const int pn = p == 2 ? 0 : p + 1;
          const T s0 = G0[p] << d, s1 = G1[p] << d;
          t[p] = (A0[p] & s0) ^ (A0[p] & s1) ^ (A1[p] & s0) ^ ks[p][tid] ^ ks[pn][tid];
          if (both) {
            const T u0 = A0[p] << d, u1 = A1[p] << d;
            q[p] = (A0[p] & u0) ^ (A0[p] & u1) ^ (A1[p] & u0) ^ ks[3 + p][tid] ^ ks[3 + pn][tid];
          } else {
            q[p] = 0;
          }
        }
        T nG1[3], nA1[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const int pn = p == 2 ? 0 : p + 1;
          nG1[p] = G1[p] ^ t[pn];
          nA1[p] = q[pn];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          G0[p] ^= t[p];
          G1[p] = nG1[p];
          if (both) {
            A0[p] = q[p];
            A1[p] = nA1[p];
          }
        }
      }
      __syncthreads();
    }
    if (act) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int64_t i = (int64_t)p * n + e;
        // sum_out: the adder's result p ^ (g << 1) (share-wise) instead of the carries
        og0[i] = sum_out ? (T)(p0[i] ^ (G0[p] << 1)) : G0[p];
        og1[i] = sum_out ? (T)(p1[i] ^ (G1[p] << 1)) : G1[p];
      }
    }
  }
}

// k_ks_adder3 for latency-bound launches: a block takes E = 6 elements and first computes
// EVERY level's mask chunks in parallel (up to 8 levels x 6 streams x 6 elements, one
// ChaCha block per thread), then three threads per element (one per party, exchanging t
// and pk' through LDS) run the whole carry chain from LDS -- one keystream latency instead
// of one per level.  Same masks, same logic: bitwise k_ks_adder3's result.
template <class T>
__global__ void __launch_bounds__(256) k_ks_adder3p(const T* __restrict__ g0,
                                                    const T* __restrict__ g1, 
                                                    const T* __restrict__ p0, const T* __restrict__ p1,
                                                    T* __restrict__ og0, T* __restrict__ og1,
                                                    int64_t n, int nlev, KeySrc keys, Nonces8 nn,
                                                   int sum_out) {
  constexpr int E = 6;
  constexpr int W = 8 * (int)sizeof(T);
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ T ks[8][6][E];
  __shared__ T xt[2][3 * E], xq[2][3 * E];
  stage_keys(rks, keys, 3);
  constexpr int P = Lane<T>::kPer;
  const int tid = threadIdx.x;
  for (int64_t e0 = (int64_t)blockIdx.x * E; e0 < n; e0 += (int64_t)gridDim.x * E) {
    // the chain: one thread per (element, party), E x 3 threads (its operands are loaded
    // first, so their latency hides behind the keystream work); each level's t and pk'
    // of party p + 1 come through LDS (double-buffered by level parity: one barrier per
    // level); levels unrolled, so every shift is by a constant
    const int le = tid / 3, p = tid - 3 * (tid / 3), pn = p == 2 ? 0 : p + 1;
    const int64_t e = e0 + le;
    const bool act = tid < 3 * E && e < n;
    const int64_t i = (int64_t)p * n + e;
    T G0 = act ? g0[i] : (T)0, G1 = act ? g1[i] : (T)0;
    T A0 = act ? p0[i] : (T)0, A1 = act ? p1[i] : (T)0;
    for (int q = tid; q < nlev * 6 * E; q += blockDim.x) {
      const int lev = q / (6 * E), s = (q / E) % 6, lq = q % E;
      const bool both = 2 * (1 << lev) < W;
      if (s >= (both ? 6 : 3) || e0 + lq >= n) continue;
      const int64_t c = (s < 3 ? 0 : n) + e0 + lq;  // t at e, pk' at n + e
      uint64_t lo, hi;
      prf_chunk(rks[s % 3], nn.v[lev], (uint64_t)(c / P), &lo, &hi);
      ks[lev][s][lq] = pick<T>(lo, hi, (int)(c % P));
    }
    __syncthreads();
#pragma unroll
    for (int lev = 0; lev < 8; ++lev) {
      if (lev >= nlev) break;  // uniform over the block
      const int d = 1 << lev;
      const bool both = 2 * d < W;
      T t = 0, q = 0;
      if (act) {
        const T s0 = G0 << d, s1 = G1 << d;
        t = (A0 & s0) ^ (A0 & s1) ^ (A1 & s0) ^ ks[lev][p][le] ^ ks[lev][pn][le];
        if (both) {
          const T u0 = A0 << d, u1 = A1 << d;
          q = (A0 & u0) ^ (A0 & u1) ^ (A1 & u0) ^ ks[lev][3 + p][le] ^ ks[lev][3 + pn][le];
        }
        xt[lev & 1][tid] = t;
        xq[lev & 1][tid] = q;
      }
      __syncthreads();
      if (act) {
        const int src = 3 * le + pn;
        G1 ^= xt[lev & 1][src];
        G0 ^= t;
        if (both) {
          A1 = xq[lev & 1][src];
          A0 = q;
        }
      }
    }
    if (act) {
      // sum_out: the adder's result p ^ (g << 1) (share-wise) instead of the carries
      og0[i] = sum_out ? (T)(p0[i] ^ (G0 << 1)) : G0;
      og1[i] = sum_out ? (T)(p1[i] ^ (G1 << 1)) : G1;
    }
    __syncthreads();
  }
}

// The whole of rep.bit_decompose for three stacked parties in ONE launch (latency form):
// P0's y = x_0 + x_1 boolean-shared (mask PRF(k_mir, n1): slots (r, y ^ r, 0), mirrored
// (y ^ r, r, 0)), the trivial sharing of x_2 (slot 2: P2's s0, P1's s1), the adder's
// p = a ^ b and g = a AND b (zero share PRF(k_q, nmul) ^ PRF(k_{q+1}, nmul); with
// A_2 = B_0 = B_1 = 0 the cross terms are c_0 = 0, c_1 = A_1 & b_2, c_2 = A_0 & b_2), then
// the Kogge-Stone chain as k_ks_adder3p and the sum p ^ (g << 1).  Every keystream chunk is
// computed in parallel first (4 + 6 per level per element), then three threads per
// element (one per party) run the chain.  Bitwise the shares of the share + slot placement
// + xor + AND + adder kernels it replaces.
template <class T, bool SIGN>
__global__ void __launch_bounds__(256) k_bitdec3(const T* __restrict__ x0, const T* __restrict__ x1,
                                                 T* __restrict__ o0, T* __restrict__ o1,
                                                 int64_t n, int nlev, KeySrc keys, int mir,
                                                 uint64_t n1, uint64_t nmul, Nonces8 nn,
                                                 uint64_t n1b, uint64_t nmulb) {
  constexpr int E = 5;
  constexpr int W = 8 * (int)sizeof(T);
  constexpr int P = Lane<T>::kPer;
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ T ks[8][6][E];
  __shared__ T kr[E], kz[3][E], kr2[E], kz2[3][E];
  __shared__ uint8_t bs0[3 * E], bs1[3 * E];
  constexpr int NB = SIGN ? 8 : 4;  // per element: sharing mask + AND zero share (+ b2a's)
  __shared__ T xt[2][3 * E], xq[2][3 * E];
  stage_keys(rks, keys, 3);
  const int tid = threadIdx.x;
  for (int64_t e0 = (int64_t)blockIdx.x * E; e0 < n; e0 += (int64_t)gridDim.x * E) {
    const int le = tid / 3, p = tid - 3 * (tid / 3), pn = p == 2 ? 0 : p + 1;
    const int64_t e = e0 + le;
    const bool act = tid < 3 * E && e < n;
    // operands first: their loads overlap the keystream work
    T y = 0, b2 = 0, b2b = 0;
    if (act) {
      y = x0[e] + x1[e];  // P0's x_0 + x_1
      b2 = x0[2 * n + e];  // x_2 as P2 holds it (s0)
      b2b = x1[n + e];     // x_2 as P1 holds it (s1)
    }
    for (int q = tid; q < NB * E + nlev * 6 * E; q += blockDim.x) {
      uint64_t lo, hi;
      if (q < NB * E) {  // 0: the sharing mask; 1..3: the AND's zero share (k0, k1, k2);
                         // 4..7 (SIGN): the same two for the b2a of the sign bit
        const int s = q / E, lq = q % E;
        if (e0 + lq >= n) continue;
        const int64_t c = e0 + lq;
        const int sl = s & 3;
        const uint64_t non = s < 4 ? (sl == 0 ? n1 : nmul) : (sl == 0 ? n1b : nmulb);
        prf_chunk(rks[sl == 0 ? mir : sl - 1], non, (uint64_t)(c / P), &lo, &hi);
        const T v = pick<T>(lo, hi, (int)(c % P));
        if (s == 0)
          kr[lq] = v;
        else if (s < 4)
          kz[s - 1][lq] = v;
        else if (s == 4)
          kr2[lq] = v;
        else
          kz2[s - 5][lq] = v;
      } else {
        const int r = q - NB * E;
        const int lev = r / (6 * E), s = (r / E) % 6, lq = r % E;
        const bool both = 2 * (1 << lev) < W;
        if (s >= (both ? 6 : 3) || e0 + lq >= n) continue;
        const int64_t c = (s < 3 ? 0 : n) + e0 + lq;  // t at e, pk' at n + e
        prf_chunk(rks[s % 3], nn.v[lev], (uint64_t)(c / P), &lo, &hi);
        ks[lev][s][lq] = pick<T>(lo, hi, (int)(c % P));
      }
    }
    __syncthreads();
    T G0 = 0, G1 = 0, A0 = 0, A1 = 0, S0 = 0, S1 = 0;
    if (act) {
      const T r = kr[le], v = y ^ r;
      const T As[3] = {mir ? v : r, mir ? r : v, (T)0};
      S0 = As[p] ^ (p == 2 ? b2 : (T)0);    // p's s0 = slot p of a ^ b
      S1 = As[pn] ^ (p == 1 ? b2b : (T)0);  // p's s1 = slot p + 1
      const T c[3] = {(T)0, (T)(As[1] & b2b), (T)(As[0] & b2)};
      const int pnn = pn == 2 ? 0 : pn + 1;
      G0 = c[p] ^ kz[p][le] ^ kz[pn][le];     // z_p
      G1 = c[pn] ^ kz[pn][le] ^ kz[pnn][le];  // z_{p+1}, reshared to p
      A0 = S0;
      A1 = S1;
    }
#pragma unroll
    for (int lev = 0; lev < 8; ++lev) {
      if (lev >= nlev) break;  // uniform over the block
      const int d = 1 << lev;
      const bool both = 2 * d < W;
      T t = 0, q = 0;
      if (act) {
        const T s0 = G0 << d, s1 = G1 << d;
        t = (A0 & s0) ^ (A0 & s1) ^ (A1 & s0) ^ ks[lev][p][le] ^ ks[lev][pn][le];
        if (both) {
          const T u0 = A0 << d, u1 = A1 << d;
          q = (A0 & u0) ^ (A0 & u1) ^ (A1 & u0) ^ ks[lev][3 + p][le] ^ ks[lev][3 + pn][le];
        }
        xt[lev & 1][tid] = t;
        xq[lev & 1][tid] = q;
      }
      __syncthreads();
      if (act) {
        const int src = 3 * le + pn;
        G1 ^= xt[lev & 1][src];
        G0 ^= t;
        if (both) {
          A1 = xq[lev & 1][src];
          A0 = q;
        }
      }
    }
    if constexpr (!SIGN) {
      if (act) {
        o0[(int64_t)p * n + e] = S0 ^ (T)(G0 << 1);
        o1[(int64_t)p * n + e] = S1 ^ (T)(G1 << 1);
      }
    } else {
      // the sign bit of every component (msb), then its b2a as k_b2a3 (one thread per
      // element): P0's a = b_0 ^ b_1 shared, times the trivial sharing of b_2, lincomb
      if (act) {
        bs0[tid] = (uint8_t)((S0 ^ (T)(G0 << 1)) >> (W - 1)) & 1;
        bs1[tid] = (uint8_t)((S1 ^ (T)(G1 << 1)) >> (W - 1)) & 1;
      }
      __syncthreads();
      if (act && p == 0) {
        const T a = (T)((bs0[tid] ^ bs1[tid]) & 1);
        const T x2 = (T)bs0[tid + 2], x2b = (T)bs1[tid + 1];  // P2's, P1's b_2
        const T r = kr2[le];
        const T v = a - r;
        const T B0 = mir ? v : r, B1 = mir ? r : v;
        const T k0 = kz2[0][le], k1 = kz2[1][le], k2 = kz2[2][le];
        const T z0 = k0 - k1, z1 = B1 * x2b + k1 - k2, z2 = B0 * x2 + k2 - k0;
        const T o[3] = {(T)(B0 - (z0 << 1)), (T)(B1 - (z1 << 1)), (T)(x2 - (z2 << 1))};
        const bool r4 = o1 == o0 + n;  // 4-slot ring: out1's slots 0, 1 are out0's 1, 2
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          o0[(int64_t)q * n + e] = o[q];
          if (!r4 || q == 2) o1[(int64_t)q * n + e] = o[q == 2 ? 0 : q + 1];
        }
      }
    }
    __syncthreads();
  }
}

// rep.mux(s, x, y) = s * (x - y) + y for arithmetic sharings, three stacked parties, ONE
// launch: the share-wise differences, the RSS product with its zero share
// PRF(k_p, nonce) - PRF(k_{p+1}, nonce) and reshare (as k_rss_cross_ring3_lat), and the
// share-wise add of y -- bitwise the sub + mul + add kernels it replaces.  Latency form:
// the block's 3 x EPB keystream chunks one per thread, then EPB threads finish.
template <class T>
__global__ void __launch_bounds__(256) k_mux3_lat(const T* __restrict__ s0,
                                                  const T* __restrict__ s1, 
                                                  const T* __restrict__ x0, const T* __restrict__ x1,
                                                  const T* __restrict__ y0, const T* __restrict__ y1,
                                                  T* __restrict__ out0, T* __restrict__ out1,
                                                  int64_t n, KeySrc keys, uint64_t nonce,
                                                  int absv = 0) {
  constexpr int EPB = 256 / 3;
  constexpr int P = Lane<T>::kPer;
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ uint64_t kl[3][EPB], kh[3][EPB];
  stage_keys(rks, keys, 3);
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  const bool r4 = out1 == out0 + n;  // 4-slot ring: out1's slots 0, 1 are out0's 1, 2
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    const bool fin = tid < EPB && b0 + tid < nb;
    T v[3][P], ya[3][P], yb[3][P];  // operands first: their loads overlap the keystream work
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t e = (b0 + tid) * P + j, i = (int64_t)p * n + e;
        if (fin && e < n) {
          // absv: x - 2 s x (rep.lincomb of x and the product) -- operand x, added x
          const T a0 = s0[i], a1 = s1[i];
          const T d0 = absv ? x0[i] : (T)(x0[i] - y0[i]), d1 = absv ? x1[i] : (T)(x1[i] - y1[i]);
          v[p][j] = a0 * d0 + a0 * d1 + a1 * d0;
          ya[p][j] = absv ? x0[i] : y0[i];
          yb[p][j] = absv ? x1[i] : y1[i];
        } else {
          v[p][j] = ya[p][j] = yb[p][j] = 0;
        }
      }
    }
    if (s < 3 && b0 + lb < nb) {
      uint64_t lo, hi;
      prf_chunk(rks[s], nonce, (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    __syncthreads();
    if (fin) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int q = p == 2 ? 0 : p + 1, pm = p == 0 ? 2 : p - 1;
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t e = (b0 + tid) * P + j;
          if (e >= n) break;
          const T z = v[p][j] + pick<T>(kl[p][tid], kh[p][tid], j) - pick<T>(kl[q][tid], kh[q][tid], j);
          const T zz = absv ? (T)(0 - (z << 1)) : z;
          out0[(int64_t)p * n + e] = zz + ya[p][j];
          // z_p is party p-1's second share: out1[p-1] = z_p + y1[p-1]
          if (!r4 || pm == 2) out1[(int64_t)pm * n + e] = zz + yb[pm][j];
        }
      }
    }
    __syncthreads();
  }
}

// a * f + (batch row in {ra, rb} ? c : 0), elementwise over a [rows][per] stack with f of
// the same shape and c a scalar on the device: exp's integer-part factors (MulLeading by the
// public vector's broadcast, then add_public of 1 on slot 0 of s0 and slot 2 of s1, here the
// pair buffer's rows ra, rb) in one launch instead of two.
template <class T>
__global__ void __launch_bounds__(256) k_mul_rows_add(const T* __restrict__ a,
                                                      const T* __restrict__ f,
                                                      T* __restrict__ out, int64_t n,
                                                      int64_t per, const T* __restrict__ c,
                                                      int ra, int rb) {
  const T cv = c[0];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per;
    out[i] = a[i] * f[i] + ((r == ra || r == rb) ? cv : (T)0);
  }
}

// Share-pair form of k_mul_rows_add for one party's two components (per-party sessions):
// o_y = a_y * f + (which[y] ? c : 0) -- the scaled integer-part factors plus the public 1
// on this party's copies of x_0, one launch instead of two multiplies and an add.
template <class T>
__device__ __forceinline__ void d_mul_add2(const Pair<T>& p, int64_t n, const T* __restrict__ c) {
  const int y = blockIdx.y;
  const T* __restrict__ a = p.a[y];
  const T* __restrict__ f = p.b[0];
  T* __restrict__ out = p.o[y];
  const T cv = p.which[y] ? c[0] : (T)0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a[i] * f[i] + cv;
}

template <class T>
__global__ void __launch_bounds__(256) k_mul_add2(Pair<T> p, int64_t n, const T* __restrict__ c) {
  d_mul_add2<T>(p, n, c);
}

// The adder's sum after the last level, both share components: p ^ ((g ^ t) << 1).
template <class T>
__device__ __forceinline__ void d_ks_sum2(const T* __restrict__ p0, const T* __restrict__ p1,
                                          const T* __restrict__ g0, const T* __restrict__ g1,
                                          const T* __restrict__ t0, const T* __restrict__ t1,
                                          T* __restrict__ o0, T* __restrict__ o1, int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    o0[e] = p0[e] ^ (T)((g0[e] ^ t0[e]) << 1);
    o1[e] = p1[e] ^ (T)((g1[e] ^ t1[e]) << 1);
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_ks_sum2(const T* __restrict__ p0, const T* __restrict__ p1,
                                                 const T* __restrict__ g0, const T* __restrict__ g1,
                                                 const T* __restrict__ t0, const T* __restrict__ t1,
                                                 T* __restrict__ o0, T* __restrict__ o1,
                                                 int64_t n) {
  d_ks_sum2<T>(p0, p1, g0, g1, t0, t1, o0, o1, n);
}

// One party's cross terms of a Kogge-Stone level (mx_ks_cross1): thread per element.  With
// t0 (mx_ks_cross1x_s) the level's g is g ^ t -- the previous level's xor, folded in --
// and is written to go0 / go1 for the next level.
template <class T>
__device__ __forceinline__ void d_ks_cross1(const T* __restrict__ g0, const T* __restrict__ g1,
                                            const T* __restrict__ p0, const T* __restrict__ p1,
                                            T* __restrict__ z, int64_t n, int d, int both,
                                            const KeySrc& keys, uint64_t nonce,
                                            const T* __restrict__ t0 = nullptr,
                                            const T* __restrict__ t1 = nullptr,
                                            T* __restrict__ go0 = nullptr,
                                            T* __restrict__ go1 = nullptr) {
  __shared__ uint32_t rks[2][kKeyWords];
  stage_keys(rks, keys, 2);
  constexpr int P = Lane<T>::kPer;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    uint64_t l0, h0, l1, h1;
    prf_chunk(rks[0], nonce, (uint64_t)(e / P), &l0, &h0);
    prf_chunk(rks[1], nonce, (uint64_t)(e / P), &l1, &h1);
    const T a0 = p0[e], a1 = p1[e];
    T G0 = g0[e], G1 = g1[e];
    if (t0 != nullptr) {
      G0 ^= t0[e];
      G1 ^= t1[e];
      go0[e] = G0;
      go1[e] = G1;
    }
    const T s0 = G0 << d, s1 = G1 << d;
    z[e] = (a0 & s0) ^ (a0 & s1) ^ (a1 & s0) ^ pick<T>(l0, h0, (int)(e % P)) ^
           pick<T>(l1, h1, (int)(e % P));
    if (both) {
      const int64_t c = n + e;
      prf_chunk(rks[0], nonce, (uint64_t)(c / P), &l0, &h0);
      prf_chunk(rks[1], nonce, (uint64_t)(c / P), &l1, &h1);
      const T u0 = a0 << d, u1 = a1 << d;
      z[c] = (a0 & u0) ^ (a0 & u1) ^ (a1 & u0) ^ pick<T>(l0, h0, (int)(c % P)) ^
             pick<T>(l1, h1, (int)(c % P));
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_ks_cross1(const T* __restrict__ g0,
                                                   const T* __restrict__ g1,
                                                   const T* __restrict__ p0,
                                                   const T* __restrict__ p1, T* __restrict__ z,
                                                   int64_t n, int d, int both, KeySrc keys,
                                                   uint64_t nonce,
                                                   const T* __restrict__ t0 = nullptr,
                                                   const T* __restrict__ t1 = nullptr,
                                                   T* __restrict__ go0 = nullptr,
                                                   T* __restrict__ go1 = nullptr) {
  d_ks_cross1<T>(g0, g1, p0, p1, z, n, d, both, keys, nonce, nullptr, nullptr, nullptr, nullptr);
}

// Latency form of k_ks_cross1 (a per-party level of the LR inference's adders: a few
// hundred elements): the block's 2 x EPB keystream chunks (both keys, one nonce) one per
// thread into LDS, then every thread finishes elements -- one ChaCha block on the critical
// path instead of two (four with both ANDs) in sequence.  Same chunks, same values.
template <class T>
__device__ __forceinline__ void d_ks_cross1_lat(const T* __restrict__ g0, const T* __restrict__ g1,
                                                const T* __restrict__ p0, const T* __restrict__ p1,
                                                T* __restrict__ z, int64_t n, int d, int both,
                                                const KeySrc& keys, uint64_t nonce,
                                                const T* __restrict__ t0, const T* __restrict__ t1,
                                                T* __restrict__ go0, T* __restrict__ go1) {
  constexpr int EPB = 128;
  __shared__ uint32_t rks[2][kKeyWords];
  __shared__ uint64_t kl[2][EPB], kh[2][EPB];
  stage_keys(rks, keys, 2);
  constexpr int P = Lane<T>::kPer;
  const int64_t ntot = both ? 2 * n : n;
  const int64_t nb = (ntot + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    if (b0 + lb < nb) {
      uint64_t lo, hi;
      prf_chunk(rks[s], nonce, (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    __syncthreads();
    for (int q = tid; q < EPB * P; q += blockDim.x) {
      const int64_t c = b0 * P + q;
      if (c >= ntot) break;
      const int lc = q / P, j = q % P;
      const T k = pick<T>(kl[0][lc], kh[0][lc], j) ^ pick<T>(kl[1][lc], kh[1][lc], j);
      const int64_t e = c < n ? c : c - n;
      const T a0 = p0[e], a1 = p1[e];
      if (c < n) {
        T G0 = g0[e], G1 = g1[e];
        if (t0 != nullptr) {
          G0 ^= t0[e];
          G1 ^= t1[e];
          go0[e] = G0;
          go1[e] = G1;
        }
        const T s0 = G0 << d, s1 = G1 << d;
        z[c] = (a0 & s0) ^ (a0 & s1) ^ (a1 & s0) ^ k;
      } else {
        const T u0 = a0 << d, u1 = a1 << d;
        z[c] = (a0 & u0) ^ (a0 & u1) ^ (a1 & u0) ^ k;
      }
    }
    __syncthreads();
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_ks_cross1_lat(const T* __restrict__ g0,
                                                       const T* __restrict__ g1,
                                                       const T* __restrict__ p0,
                                                       const T* __restrict__ p1, T* __restrict__ z,
                                                       int64_t n, int d, int both, KeySrc keys,
                                                       uint64_t nonce, const T* __restrict__ t0,
                                                       const T* __restrict__ t1,
                                                       T* __restrict__ go0, T* __restrict__ go1) {
  d_ks_cross1_lat<T>(g0, g1, p0, p1, z, n, d, both, keys, nonce, t0, t1, go0, go1);
}

// party-batched twins for the composed one-GPU replay (party_batch.h)
MX_X3_GS(k_binary<u64>, d_binary<u64>);
MX_X3_GS(k_binary<u128>, d_binary<u128>);
MX_X3(k_lincomb2<u64>, d_lincomb2<u64>);
MX_X3(k_lincomb2<u128>, d_lincomb2<u128>);
MX_X3(k_addn_decode<u64>, d_addn_decode<u64>);
MX_X3(k_addn_decode<u128>, d_addn_decode<u128>);
MX_X3(k_rss_cross<u64>, d_rss_cross<u64>);
MX_X3(k_rss_cross<u128>, d_rss_cross<u128>);
MX_X3(k_mul_add2<u64>, d_mul_add2<u64>);
MX_X3(k_mul_add2<u128>, d_mul_add2<u128>);
MX_X3(k_ks_cross1_lat<u64>, d_ks_cross1_lat<u64>);
MX_X3(k_ks_cross1_lat<u128>, d_ks_cross1_lat<u128>);

template <class T>
bool ks_lat_launch(const void* g0, const void* g1, const void* t0, const void* t1, void* go0,
                   void* go1, const void* p0, const void* p1, void* z, int64_t n, int d, int both,
                   const KeySrc& k, uint64_t nonce, hipStream_t st) {
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = ((both ? 2 * n : n) + P - 1) / P;
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_KS_LAT");
    return !(e && e[0] == '0');
  }();
  if (!on || nb > (1 << 14)) return false;
  hipLaunchKernelGGL(k_ks_cross1_lat<T>, dim3((unsigned)((nb + 127) / 128)), dim3(256), 0, st,
                     (const T*)g0, (const T*)g1, (const T*)p0, (const T*)p1, (T*)z, n, d, both, k,
                     nonce, (const T*)t0, (const T*)t1, (T*)go0, (T*)go1);
  return true;
}

// Latency variant for small launches (few keystream chunks): the block's 3 x EPB chunks are
// computed one per thread into LDS, then EPB threads finish the elements -- one PRF on the
// critical path instead of three.
template <class T>
__global__ void __launch_bounds__(256) k_rss_cross_ring3_lat(int kind, const T* __restrict__ x0,
                                                             const T* __restrict__ x1,
                                                             const T* __restrict__ y0,
                                                             const T* __restrict__ y1,
                                                             T* __restrict__ out,
                                                             T* __restrict__ out1, int64_t n,
                                                             KeySrc keys, uint64_t nonce, Views vw) {
  constexpr int EPB = 256 / 3;
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ uint64_t kl[3][EPB], kh[3][EPB];
  stage_keys(rks, keys, 3);
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    // the finishing threads' cross terms first: their loads overlap the keystream work
    const bool fin = tid < EPB && b0 + tid < nb;
    T vv[3][P];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t e = (b0 + tid) * P + j;
        T v = 0;
        if (fin && e < n) {
          if (x0 != nullptr && y0 != nullptr)
            v = mxr::cross<T>(kind, ld_view(x0, vw, 0, p, e, n),
                              x1 ? ld_view(x1, vw, 1, p, e, n) : (T)0, ld_view(y0, vw, 2, p, e, n),
                              y1 ? ld_view(y1, vw, 3, p, e, n) : (T)0, x1 != nullptr, y1 != nullptr);
          else if (x0 != nullptr)
            v = ld_view(x0, vw, 0, p, e, n);
        }
        vv[p][j] = v;
      }
    }
    if (s < 3 && b0 + lb < nb) {
      uint64_t lo, hi;
      prf_chunk(rks[s], nonce, (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    __syncthreads();
    if (fin) {
      const int64_t b = b0 + tid;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int q = p == 2 ? 0 : p + 1;
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t e = b * P + j;
          if (e >= n) break;
          const int64_t i = (int64_t)p * n + e;
          const T v = vv[p][j];
          const T z = mxr::zs_combine<T>(kind, v, pick<T>(kl[p][tid], kh[p][tid], j),
                                         pick<T>(kl[q][tid], kh[q][tid], j));
          out[i] = z;
          if (out1 != nullptr) out1[(int64_t)(p == 0 ? 2 : p - 1) * n + e] = z;
        }
      }
    }
    __syncthreads();
  }
}

// Fixed-point product of a latency-bound launch in ONE kernel: the stacked RSS product
// with its zero share (as k_rss_cross_ring3_lat) and the TruncPr of the reshared product
// (as k_trunc_pr3_lat) -- the product never leaves registers.  Nine keystream chunks per
// chunk position: the product's zero share (k0, k1, k2 at nmul) and the TruncPr's r0, r1,
// t, m, z0, z2 (keys k0 / k2, as in k_trunc_pr3).  Bitwise equal to the two kernels.
template <class T, int EPB>
__device__ __forceinline__ void mul_trunc3_lat_body(
    const T* __restrict__ x0, const T* __restrict__ x1, const T* __restrict__ y0,
    const T* __restrict__ y1, T* __restrict__ out0, T* __restrict__ out1, int64_t n, int64_t os,
    const uint32_t (&rks)[3][kKeyWords], uint64_t (&kl)[9][EPB], uint64_t (&kh)[9][EPB],
    uint64_t nmul, int m, uint64_t nr0, uint64_t nr1, uint64_t nt, uint64_t nm, uint64_t nz0,
    uint64_t nz2, const Views& vw) {
  constexpr int NS = 9;
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  // stream s: 0..2 product zero share (k_s), 3 r0 (k0), 4 r1 (k2), 5 t (k0), 6 m (k0),
  // 7 z0 (k0), 8 z2 (k2)
  const int key_of = s < 3 ? s : (s == 4 || s == 8) ? 2 : 0;
  const uint64_t nonce_of = s < 3 ? nmul : s == 3 ? nr0 : s == 4 ? nr1 : s == 5 ? nt
                            : s == 6 ? nm : s == 7 ? nz0 : nz2;
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    // the finishing threads' cross products first: their loads overlap the keystream work
    const bool fin = tid < EPB && b0 + tid < nb;
    T vv[P][3];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t e = (b0 + tid) * P + j;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        vv[j][p] = !fin || e >= n ? (T)0
                   : y0 == nullptr ? ld_view(x0, vw, 0, p, e, n)
                   : mxr::cross<T>(MX_CROSS_ARITH, ld_view(x0, vw, 0, p, e, n),
                                   ld_view(x1, vw, 1, p, e, n), ld_view(y0, vw, 2, p, e, n),
                                   ld_view(y1, vw, 3, p, e, n), true, true);
    }
    if (s < NS && b0 + lb < nb) {
      uint64_t lo, hi;
      prf_chunk(rks[key_of], nonce_of, (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    __syncthreads();
    if (fin) {
      const int64_t b = b0 + tid;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t e = b * P + j;
        if (e >= n) break;
        T z[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const int q = p == 2 ? 0 : p + 1;
          z[p] = mxr::zs_combine<T>(MX_CROSS_ARITH, vv[j][p], pick<T>(kl[p][tid], kh[p][tid], j),
                                    pick<T>(kl[q][tid], kh[q][tid], j));
        }
        const T Z0 = pick<T>(kl[7][tid], kh[7][tid], j);
        const T Z2 = pick<T>(kl[8][tid], kh[8][tid], j);
        const T Z1 = mxf::trunc_pr_z1<T>(
            z[0], z[1], z[2], pick<T>(kl[3][tid], kh[3][tid], j),
            pick<T>(kl[4][tid], kh[4][tid], j), pick<T>(kl[5][tid], kh[5][tid], j),
            pick<T>(kl[6][tid], kh[6][tid], j), Z0, Z2, m);
        out0[e] = Z0;
        out0[os + e] = Z1;
        out0[2 * os + e] = Z2;
        if (out1 != out0 + os) {  // else a 4-slot ring: out1's slots 0, 1 are out0's 1, 2
          out1[e] = Z1;
          out1[os + e] = Z2;
        }
        out1[2 * os + e] = Z0;
      }
    }
    __syncthreads();
  }
}

// Fixed-point product of a latency-bound launch in ONE kernel: the stacked RSS product
// with its zero share (as k_rss_cross_ring3_lat) and the TruncPr of the reshared product
// (as k_trunc_pr3_lat) -- the product never leaves registers.  Nine keystream chunks per
// chunk position: the product's zero share (k0, k1, k2 at nmul) and the TruncPr's r0, r1,
// t, m, z0, z2 (keys k0 / k2, as in k_trunc_pr3).  Bitwise equal to the two kernels.
template <class T>
__global__ void __launch_bounds__(256) k_mul_trunc3_lat(
    const T* __restrict__ x0, const T* __restrict__ x1, const T* __restrict__ y0,
    const T* __restrict__ y1, T* __restrict__ out0, T* __restrict__ out1, int64_t n, int64_t os,
    KeySrc keys, uint64_t nmul, int m, uint64_t nr0, uint64_t nr1, uint64_t nt, uint64_t nm,
    uint64_t nz0, uint64_t nz2, Views vw) {
  constexpr int EPB = 256 / 9;
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ uint64_t kl[9][EPB], kh[9][EPB];
  stage_keys(rks, keys, 3);
  mul_trunc3_lat_body<T, EPB>(x0, x1, y0, y1, out0, out1, n, os, rks, kl, kh, nmul, m, nr0,
                              nr1, nt, nm, nz0, nz2, vw);
}

// Two independent products of one placement (same keys) in one launch: blockIdx.y picks the
// problem (the rounds of two computations that run side by side, e.g. a polynomial level
// and a product-tree level).  Each is exactly k_mul_trunc3_lat's.
template <class T>
struct MT2 {
  const T* x0[2];
  const T* x1[2];
  const T* y0[2];
  const T* y1[2];
  T* out0[2];
  T* out1[2];
  int64_t n[2], os[2];
  uint64_t nmul[2], nn[2][6];
  int m[2];
  Views vw[2];
};

template <class T>
__global__ void __launch_bounds__(256) k_mul_trunc3_lat2(MT2<T> a, KeySrc keys) {
  constexpr int EPB = 256 / 9;
  __shared__ uint32_t rks[3][kKeyWords];
  __shared__ uint64_t kl[9][EPB], kh[9][EPB];
  stage_keys(rks, keys, 3);
  const int y = blockIdx.y;
  mul_trunc3_lat_body<T, EPB>(a.x0[y], a.x1[y], a.y0[y], a.y1[y], a.out0[y], a.out1[y], a.n[y],
                              a.os[y], rks, kl, kh, a.nmul[y], a.m[y], a.nn[y][0], a.nn[y][1],
                              a.nn[y][2], a.nn[y][3], a.nn[y][4], a.nn[y][5], a.vw[y]);
}

// Throughput form of k_mul_trunc3_lat: one ChaCha block of each of the nine streams per
// thread (walk_chunks), same shares.  y0 == nullptr: x0 already holds the three parties'
// local products (a GEMM's) -- the zero share + reshare + TruncPr tail of a fixed-point dot
// in one pass, the reshared product never written.
template <class T>
__global__ void __launch_bounds__(256) k_mul_trunc3(
    const T* __restrict__ x0, const T* __restrict__ x1, const T* __restrict__ y0,
    const T* __restrict__ y1, T* __restrict__ out0, T* __restrict__ out1, int64_t n, int64_t os,
    KeySrc keys, uint64_t nmul, int m, uint64_t nr0, uint64_t nr1, uint64_t nt, uint64_t nm,
    uint64_t nz0, uint64_t nz2, Views vw) {
  __shared__ uint32_t rks[3][kKeyWords];
  stage_keys(rks, keys, 3);
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  // streams as k_mul_trunc3_lat: product zero share (k0, k1, k2), r0 (k0), r1 (k2), t (k0),
  // m (k0), z0 (k0), z2 (k2)
  const uint32_t* const key[9] = {rks[0], rks[1], rks[2], rks[0], rks[2],
                                  rks[0], rks[0], rks[0], rks[2]};
  const uint64_t nonce[9] = {nmul, nmul, nmul, nr0, nr1, nt, nm, nz0, nz2};
  mxd::walk_chunks<9>(nb, key, nonce, [&](int64_t b, const uint64_t (&lo)[9],
                                          const uint64_t (&hi)[9]) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t e = b * P + j;
      if (e >= n) break;
      T z[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int q = p == 2 ? 0 : p + 1;
        const T v = y0 == nullptr ? ld_view(x0, vw, 0, p, e, n)
                    : mxr::cross<T>(MX_CROSS_ARITH, ld_view(x0, vw, 0, p, e, n),
                                    ld_view(x1, vw, 1, p, e, n), ld_view(y0, vw, 2, p, e, n),
                                    ld_view(y1, vw, 3, p, e, n), true, true);
        z[p] = mxr::zs_combine<T>(MX_CROSS_ARITH, v, pick<T>(lo[p], hi[p], j),
                                  pick<T>(lo[q], hi[q], j));
      }
      const T Z0 = pick<T>(lo[7], hi[7], j);
      const T Z2 = pick<T>(lo[8], hi[8], j);
      const T Z1 = mxf::trunc_pr_z1<T>(z[0], z[1], z[2], pick<T>(lo[3], hi[3], j),
                                       pick<T>(lo[4], hi[4], j), pick<T>(lo[5], hi[5], j),
                                       pick<T>(lo[6], hi[6], j), Z0, Z2, m);
      out0[e] = Z0;
      out0[os + e] = Z1;
      out0[2 * os + e] = Z2;
      if (out1 != out0 + os) {
        out1[e] = Z1;
        out1[os + e] = Z2;
      }
      out1[2 * os + e] = Z0;
    }
  });
}

template <class T>
__device__ __forceinline__ void d_prf_expand(T* __restrict__ out, int64_t n, int nkeys,
                                             const KeySrc& keys, uint64_t nonce) {
  __shared__ uint32_t rks[4][kKeyWords];
  stage_keys(rks, keys, nkeys);
  constexpr int P = Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)nb);
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nblk * nkeys;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - p * nblk);
    uint32_t w[16];
    mx::chacha_block(rks[p], nonce, B, w);
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int64_t b = (int64_t)mx::ks_chunk(B, part);
      if (b >= nb) break;
      uint64_t lo, hi;
      mx::part_u64(w, part, &lo, &hi);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        int64_t e = b * P + j;
        if (e < n) out[(int64_t)p * n + e] = pick<T>(lo, hi, j);
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_prf_expand(T* __restrict__ out, int64_t n, int nkeys,
                                                    KeySrc keys, uint64_t nonce) {
  d_prf_expand<T>(out, n, nkeys, keys, nonce);
}

// party-batched twins of the per-party sessions' local kernels (party_batch.h)
MX_X3_GS(k_binary2<u64>, d_binary2<u64>);
MX_X3_GS(k_binary2<u128>, d_binary2<u128>);
MX_X3_GS(k_unary2<u64>, d_unary2<u64>);
MX_X3_GS(k_unary2<u128>, d_unary2<u128>);
MX_X3(k_transpose2<u64>, d_transpose2<u64>);
MX_X3(k_transpose2<u128>, d_transpose2<u128>);
MX_X3_GS(k_unary<u64>, d_unary<u64>);
MX_X3_GS(k_unary<u128>, d_unary<u128>);
MX_X3(k_binary_slot<u64>, d_binary_slot<u64>);
MX_X3(k_binary_slot<u128>, d_binary_slot<u128>);
MX_X3(k_binary_slot2<u64>, d_binary_slot2<u64>);
MX_X3(k_binary_slot2<u128>, d_binary_slot2<u128>);
MX_X3(k_sum_axis<u64>, d_sum_axis<u64>);
MX_X3(k_sum_axis<u128>, d_sum_axis<u128>);
MX_X3(k_fill<u64>, d_fill<u64>);
MX_X3(k_fill<u128>, d_fill<u128>);
MX_X3(k_encode<u64>, d_encode<u64>);
MX_X3(k_encode<u128>, d_encode<u128>);
MX_X3(k_decode<u64>, d_decode<u64>);
MX_X3(k_decode<u128>, d_decode<u128>);
MX_X3(k_ks_cross1<u64>, d_ks_cross1<u64>);
MX_X3(k_ks_cross1<u128>, d_ks_cross1<u128>);
MX_X3(k_ks_sum2<u64>, d_ks_sum2<u64>);
MX_X3(k_ks_sum2<u128>, d_ks_sum2<u128>);
MX_X3(k_slot_place2<u64>, d_slot_place2<u64>);
MX_X3(k_slot_place2<u128>, d_slot_place2<u128>);
MX_X3(k_sum_views2<u64>, d_sum_views2<u64>);
MX_X3(k_sum_views2<u128>, d_sum_views2<u128>);
MX_X3(k_bit_extract<u64>, d_bit_extract<u64>);
MX_X3(k_bit_extract<u128>, d_bit_extract<u128>);
MX_X3(k_bit_planes<u64>, d_bit_planes<u64>);
MX_X3(k_bit_planes<u128>, d_bit_planes<u128>);
MX_X3(k_compare<u64>, d_compare<u64>);
MX_X3(k_compare<u128>, d_compare<u128>);
MX_X3(k_prf_expand<u64>, d_prf_expand<u64>);
MX_X3(k_prf_expand<u128>, d_prf_expand<u128>);
MX_X3(k_ring_inject<u64>, d_ring_inject<u64>);
MX_X3(k_ring_inject<u128>, d_ring_inject<u128>);

// Reference (VALU) ring GEMM: 16x16 output tile per block, K staged through LDS.
// a_bs / b_bs: batch strides in elements (0: one operand broadcast over the batch).
template <class T, int TS>
__device__ __forceinline__ void d_gemm_valu(int64_t M, int64_t N, int64_t K,
                                            const T* __restrict__ A0, const T* __restrict__ A1,
                                            const T* __restrict__ B0, const T* __restrict__ B1,
                                            int mode, T* __restrict__ C, int accumulate,
                                            int64_t a_bs, int64_t b_bs, int zb) {
  __shared__ T As[TS][TS + 1];
  __shared__ T Bs[TS][TS + 1];
  const int64_t b = zb >= 0 ? zb : blockIdx.z;  // zb >= 0: an unbatched launch's only product
  const int64_t row = blockIdx.y * TS + threadIdx.y;
  const int64_t col = blockIdx.x * TS + threadIdx.x;
  const T* a0 = A0 + b * a_bs;
  const T* b0 = B0 + b * b_bs;
  const T* a1 = mode ? A1 + b * a_bs : nullptr;
  const T* b1 = mode ? B1 + b * b_bs : nullptr;
  T acc = 0;
  const int passes = mode ? 2 : 1;
  for (int pass = 0; pass < passes; ++pass) {
    for (int64_t k0 = 0; k0 < K; k0 += TS) {
      int64_t ka = k0 + threadIdx.x, kb = k0 + threadIdx.y;
      T av = 0, bv = 0;
      if (row < M && ka < K) av = (pass == 0 ? a0 : a1)[row * K + ka];
      if (col < N && kb < K) {
        bv = b0[kb * N + col];
        if (mode && pass == 0) bv += b1[kb * N + col];
      }
      As[threadIdx.y][threadIdx.x] = av;
      Bs[threadIdx.y][threadIdx.x] = bv;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < TS; ++k) acc += As[threadIdx.y][k] * Bs[k][threadIdx.x];
      __syncthreads();
    }
  }
  if (row < M && col < N) {
    T* c = C + b * M * N + row * N + col;
    *c = accumulate ? (T)(*c + acc) : acc;
  }
}

template <class T, int TS>
__global__ void __launch_bounds__(256) k_gemm_valu(int64_t M, int64_t N, int64_t K,
                                                   const T* __restrict__ A0,
                                                   const T* __restrict__ A1,
                                                   const T* __restrict__ B0,
                                                   const T* __restrict__ B1, int mode,
                                                   T* __restrict__ C, int accumulate,
                                                   int64_t a_bs, int64_t b_bs, int zb) {
  d_gemm_valu<T, TS>(M, N, K, A0, A1, B0, B1, mode, C, accumulate, a_bs, b_bs, zb);
}

// an unbatched product (grid z = 1, zb = 0) of several parties: one party-batched launch
MX_X3((k_gemm_valu<u64, 16>), (d_gemm_valu<u64, 16>));
MX_X3((k_gemm_valu<u128, 16>), (d_gemm_valu<u128, 16>));

// Skinny products (N <= 4: a matrix times a vector or a few columns -- the per-party
// LogReg and LR dots): one wave per output row, its lanes splitting K, then a butterfly over
// whole ring elements.  One pass of coalesced loads instead of the tiled kernel's serial
// k-tiles with two barriers each (a 100 x 128 by 128 x 1 product: ~25 us there).  The same
// ring sums (addition mod 2^w is associative), so the same products.
template <class T>
__device__ __forceinline__ T shfl_xor_wave(T v, int m) {
  constexpr int W = (int)(sizeof(T) / 4);
  uint32_t w[W];
#pragma unroll
  for (int q = 0; q < W; ++q) w[q] = (uint32_t)(v >> (32 * q));
#pragma unroll
  for (int q = 0; q < W; ++q) w[q] = (uint32_t)__shfl_xor((int)w[q], m, 64);
  T r = 0;
#pragma unroll
  for (int q = 0; q < W; ++q) r |= (T)w[q] << (32 * q);
  return r;
}

template <class T>
__device__ __forceinline__ void d_gemv_valu(int64_t M, int64_t N, int64_t K,
                                            const T* __restrict__ A0, const T* __restrict__ A1,
                                            const T* __restrict__ B0, const T* __restrict__ B1,
                                            int mode, T* __restrict__ C, int accumulate,
                                            int64_t a_bs, int64_t b_bs, int zb) {
  const int64_t b = zb >= 0 ? zb : blockIdx.z;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;  // uniform per wave: the butterfly below sees whole waves
  const T* a0 = A0 + b * a_bs + row * K;
  const T* a1 = mode ? A1 + b * a_bs + row * K : nullptr;
  const T* b0 = B0 + b * b_bs;
  const T* b1 = mode ? B1 + b * b_bs : nullptr;
  for (int64_t n = 0; n < N; ++n) {
    T acc = 0;
    for (int64_t k = lane; k < K; k += 64) {
      const T y0 = b0[k * N + n];
      if (mode) {
        acc += a0[k] * (y0 + b1[k * N + n]) + a1[k] * y0;
      } else {
        acc += a0[k] * y0;
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc += shfl_xor_wave(acc, m);
    if (lane == 0) {
      T* c = C + b * M * N + row * N + n;
      *c = accumulate ? (T)(*c + acc) : acc;
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_gemv_valu(int64_t M, int64_t N, int64_t K,
                                                   const T* __restrict__ A0,
                                                   const T* __restrict__ A1,
                                                   const T* __restrict__ B0,
                                                   const T* __restrict__ B1, int mode,
                                                   T* __restrict__ C, int accumulate,
                                                   int64_t a_bs, int64_t b_bs, int zb) {
  d_gemv_valu<T>(M, N, K, A0, A1, B0, B1, mode, C, accumulate, a_bs, b_bs, zb);
}

MX_X3(k_gemv_valu<u64>, d_gemv_valu<u64>);
MX_X3(k_gemv_valu<u128>, d_gemv_valu<u128>);

// MOOSEX_GEMV=0: skinny products on the tiled kernel too
bool gemv_on() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_GEMV");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <class T>
int launch_gemm_valu(int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                     const void* A1, const void* B0, const void* B1, int mode, void* C,
                     int accumulate, hipStream_t st, int64_t a_bs = -1, int64_t b_bs = -1) {
  if (N <= 4 && gemv_on()) {
    const dim3 grid((unsigned)((M + 3) / 4), 1, (unsigned)batch);
    hipLaunchKernelGGL((k_gemv_valu<T>), grid, dim3(256), 0, st, M, N, K, (const T*)A0,
                       (const T*)A1, (const T*)B0, (const T*)B1, mode, (T*)C, accumulate,
                       a_bs < 0 ? M * K : a_bs, b_bs < 0 ? K * N : b_bs, batch == 1 ? 0 : -1);
    MX_LAUNCH_CHECK();
    return 0;
  }
  constexpr int TS = 16;
  dim3 grid((unsigned)((N + TS - 1) / TS), (unsigned)((M + TS - 1) / TS), (unsigned)batch);
  dim3 block(TS, TS);
  hipLaunchKernelGGL((k_gemm_valu<T, TS>), grid, block, 0, st, M, N, K, (const T*)A0,
                     (const T*)A1, (const T*)B0, (const T*)B1, mode, (T*)C, accumulate,
                     a_bs < 0 ? M * K : a_bs, b_bs < 0 ? K * N : b_bs, batch == 1 ? 0 : -1);
  MX_LAUNCH_CHECK();
  return 0;
}


}  // namespace

// from gemm_mfma.hip
extern "C" int mxh_gemm_mfma(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                             const void* A0, const void* A1, const void* B0, const void* B1,
                             int mode, void* C, int accumulate, void* stream);

static int g_gemm_impl = 0;

#define DEV_DISPATCH(words, T, ...)            \
  switch (words) {                             \
    case 0: { using T = uint8_t; __VA_ARGS__; } \
    case 1: { using T = u64; __VA_ARGS__; }     \
    case 2: { using T = u128; __VA_ARGS__; }    \
    default: return -2;                        \
  }

extern "C" {

void mx_set_gemm_impl(int impl) { g_gemm_impl = impl; }

int mx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mxh_ew_binary(int op, int words, const void* a, int64_t na, const void* b, int64_t nb,
                  void* out, int64_t n, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_binary<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), op,
                       (const T*)a, na, (const T*)b, nb, (T*)out, n);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_binary2(int op, int words, const void* a0, const void* b0, void* out0,
                   const void* a1, const void* b1, void* out1, int64_t na, int64_t nb, int64_t n,
                   void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    Pair<T> p{{(const T*)a0, (const T*)a1}, {(const T*)b0, (const T*)b1}, {(T*)out0, (T*)out1},
              {0, 0}};
    hipLaunchKernelGGL(k_binary2<T>, dim3(grid_for(n), 2), dim3(kBlock), 0, S(stream), op, p,
                       na, nb, n);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_unary2(int op, int words, const void* a0, void* out0, const void* a1, void* out1,
                  int64_t n, int64_t param, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    Pair<T> p{{(const T*)a0, (const T*)a1}, {nullptr, nullptr}, {(T*)out0, (T*)out1}, {0, 0}};
    hipLaunchKernelGGL(k_unary2<T>, dim3(grid_for(n), 2), dim3(kBlock), 0, S(stream), op, p, n,
                       (int)param);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_transpose2(int words, const void* a0, void* out0, const void* a1, void* out1,
                   int64_t rows, int64_t cols, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t tiles = ((rows + 31) / 32) * ((cols + 31) / 32);
  if (tiles > 0x7fffffff) return -3;
  DEV_DISPATCH(words, T, {
    Pair<T> p{{(const T*)a0, (const T*)a1}, {nullptr, nullptr}, {(T*)out0, (T*)out1}, {0, 0}};
    hipLaunchKernelGGL(k_transpose2<T>, dim3((unsigned)tiles, 2), dim3(256), 0, S(stream), p,
                       rows, cols);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_binary_slot2(int op, int words, const void* a0, const void* a1, const void* b,
                        int64_t nb, void* out0, void* out1, int64_t m, int nparties, int which0,
                        int which1, void* stream) {
  if (m == 0) return 0;
  DEV_DISPATCH(words, T, {
    Pair<T> p{{(const T*)a0, (const T*)a1}, {(const T*)b, (const T*)b}, {(T*)out0, (T*)out1},
              {which0, which1}};
    hipLaunchKernelGGL(k_binary_slot2<T>, dim3(grid_for(m * nparties), 2), dim3(kBlock), 0,
                       S(stream), op, p, nb, m, nparties);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_mul_add2(int words, const void* a0, const void* a1, const void* f, const void* c,
                 int add0, int add1, void* out0, void* out1, int64_t n, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    Pair<T> p{{(const T*)a0, (const T*)a1}, {(const T*)f, (const T*)f}, {(T*)out0, (T*)out1},
              {add0, add1}};
    hipLaunchKernelGGL(k_mul_add2<T>, dim3(grid_for(n), 2), dim3(kBlock), 0, S(stream), p, n,
                       (const T*)c);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_add3(int words, const void* a, const void* b, const void* c, void* out, int64_t n,
                void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_add3<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), (const T*)a,
                       (const T*)b, (const T*)c, (T*)out, n);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_lincomb2(int words, int nin, const void* const* ins, const int64_t* coef, const void* b,
                 int64_t nb, void* out0, void* out1, int64_t m, int nparties, int which0,
                 int which1, void* stream) {
  if (m == 0) return 0;
  if (nin < 1 || nin > 3) return -3;
  DEV_DISPATCH(words, T, {
    Lin3<T> p{};
    for (int t = 0; t < nin; ++t) {
      p.a[t][0] = (const T*)ins[2 * t];
      p.a[t][1] = (const T*)ins[2 * t + 1];
      p.coef[t] = coef[t];
    }
    p.o[0] = (T*)out0;
    p.o[1] = (T*)out1;
    p.which[0] = which0;
    p.which[1] = which1;
    hipLaunchKernelGGL(k_lincomb2<T>, dim3(grid_for(m * nparties), 2), dim3(kBlock), 0,
                       S(stream), p, nin, (const T*)b, nb, m, nparties);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_sum_views2(int words, const void* base0, const void* base1, int64_t is0, int64_t is1,
                   int64_t ps0, int64_t ps1, int k, void* out0, void* out1, int64_t m,
                   int nparties, void* stream) {
  if (m == 0) return 0;
  DEV_DISPATCH(words, T, {
    SumViews<T> p{{(const T*)base0, (const T*)base1}, {(T*)out0, (T*)out1}, {is0, is1},
                  {ps0, ps1}};
    hipLaunchKernelGGL(k_sum_views2<T>, dim3(grid_for(m * nparties), 2), dim3(kBlock), 0,
                       S(stream), p, k, m, nparties);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_slot_place2(int words, const void* x0, const void* x1, void* out0, void* out1,
                    int64_t m, int nparties, int which0, int which1, void* stream) {
  if (m == 0) return 0;
  DEV_DISPATCH(words, T, {
    Pair<T> p{{(const T*)x0, (const T*)x1}, {nullptr, nullptr}, {(T*)out0, (T*)out1},
              {which0, which1}};
    hipLaunchKernelGGL(k_slot_place2<T>, dim3(grid_for(m * nparties), 2), dim3(kBlock), 0,
                       S(stream), p, m, nparties);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_add_zs3(int words, const void* v, const void* r, void* out0, void* out1, int64_t n,
                void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_add_zs3<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const T*)v, (const T*)r, (T*)out0, (T*)out1, n);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_binary_slot(int op, int words, const void* a, const void* b, int64_t nb, void* out,
                       int64_t m, int nparties, int which, void* stream) {
  if (m == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_binary_slot<T>, dim3(grid_for(m * nparties)), dim3(kBlock), 0,
                       S(stream), op, (const T*)a, (const T*)b, nb, (T*)out, m, nparties,
                       which);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_unary(int op, int words, const void* a, void* out, int64_t n, int64_t param,
                 void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_unary<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), op,
                       (const T*)a, (T*)out, n, (int)param);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ew_compare(int op, int words, const void* a, int64_t na, const void* b, int64_t nb,
                   uint8_t* out, int64_t n, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_compare<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), op,
                       (const T*)a, na, (const T*)b, nb, out, n);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_bit_extract(int words, const void* a, uint8_t* out, int64_t n, int bit, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_bit_extract<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const T*)a, out, n, bit);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_b2a_prep3(int words, const uint8_t* s0, const uint8_t* s1, int64_t n, void* a,
                  void* b0, void* b1, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_b2a_prep3<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), s0, s1,
                       n, (T*)a, (T*)b0, (T*)b1);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

// slots: three consecutive key slots (k0, k1, k2 of the placement)
int mxh_b2a3(int words, const uint8_t* s0, const uint8_t* s1, int64_t n, void* out0,
             void* out1, const uint32_t* slots, int mir, uint64_t n1, uint64_t nmul,
             void* stream) {
  if (n == 0) return 0;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    const int64_t g = std::min<int64_t>(((n + P - 1) / P + 63) / 64, 16384);
    hipLaunchKernelGGL(k_b2a3<T>, dim3((unsigned)g), dim3(256), 0, S(stream), s0, s1,
                       (T*)out0, (T*)out1, n, mxd::keysrc_slots(ptrs, 3), mir ? 1 : 0, n1, nmul);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ring_inject(int words, const uint8_t* bits, void* out, int64_t n, int bit,
                    void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_ring_inject<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), bits,
                       (T*)out, n, bit);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_encode(int words, const double* x, void* out, int64_t n, int frac, void* stream) {
  if (n == 0) return 0;
  double scale = ldexp(1.0, frac);
  if (words == 1)
    hipLaunchKernelGGL(k_encode<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), x,
                       (u64*)out, n, scale);
  else if (words == 2)
    hipLaunchKernelGGL(k_encode<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), x,
                       (u128*)out, n, scale);
  else
    return -2;
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_addn_decode(int words, const void* a, const void* b, const void* c, const void* d,
                    double* out, int64_t n, int frac, void* stream) {
  if (n == 0) return 0;
  const double scale = ldexp(1.0, -frac);
  if (words == 1)
    hipLaunchKernelGGL(k_addn_decode<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)a, (const u64*)b, (const u64*)c, (const u64*)d, out, n, scale);
  else if (words == 2)
    hipLaunchKernelGGL(k_addn_decode<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)a, (const u128*)b, (const u128*)c, (const u128*)d, out, n,
                       scale);
  else
    return -2;
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_decode(int words, const void* x, double* out, int64_t n, int frac, void* stream) {
  if (n == 0) return 0;
  double scale = ldexp(1.0, -frac);
  if (words == 1)
    hipLaunchKernelGGL(k_decode<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)x, out, n, scale);
  else if (words == 2)
    hipLaunchKernelGGL(k_decode<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)x, out, n, scale);
  else
    return -2;
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_fill(int words, void* out, int64_t n, uint64_t lo, uint64_t hi, void* stream) {
  if (n == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_fill<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream), (T*)out, n,
                       lo, hi);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_bit_planes(int words, const void* a, uint8_t* out, int64_t outer, int64_t inner,
                   int start, int count, void* stream) {
  if (outer * inner == 0 || count == 0) return 0;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_bit_planes<T>, dim3(grid_for(outer * inner)), dim3(kBlock), 0,
                       S(stream), (const T*)a, out, outer, inner, start, count);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_weighted_sum(int words, const void* a, const void* w, void* out, int64_t outer,
                     int64_t k, int64_t inner, void* stream) {
  if (outer * inner == 0) return 0;
  DEV_DISPATCH(words, T, {
    if (k >= 16 && outer * inner <= 65536) {  // latency-bound: 8 threads per output
      const int64_t blocks = (outer * inner + 31) / 32;
      hipLaunchKernelGGL(k_weighted_sum_wide<T>, dim3((unsigned)blocks), dim3(kBlock), 0,
                         S(stream), (const T*)a, (const T*)w, (T*)out, outer, k, inner);
    } else {
      hipLaunchKernelGGL(k_weighted_sum<T>, dim3(grid_for(outer * inner)), dim3(kBlock), 0,
                         S(stream), (const T*)a, (const T*)w, (T*)out, outer, k, inner);
    }
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_sum_axis(int words, const void* a, void* out, int64_t outer, int64_t red, int64_t inner,
                 void* stream) {
  int64_t total = outer * inner;
  if (total == 0) return 0;
  DEV_DISPATCH(words, T, {
    if (red >= 1024 && total <= 65536) {
      hipLaunchKernelGGL(k_sum_axis_wide<T>, dim3((unsigned)total), dim3(kBlock), 0, S(stream),
                         (const T*)a, (T*)out, red, inner);
    } else {
      hipLaunchKernelGGL(k_sum_axis<T>, dim3(grid_for(total)), dim3(kBlock), 0, S(stream),
                         (const T*)a, (T*)out, outer, red, inner);
    }
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_prg(const uint8_t* key16, uint64_t nonce, uint64_t ctr0, void* out, int64_t nbytes,
            void* stream) {
  if (nbytes == 0) return 0;
  RawKey k;
  mx::key_words(key16, k.k);
  hipLaunchKernelGGL(k_prg, dim3(grid_for((nbytes + 15) / 16)), dim3(kBlock), 0, S(stream), k,
                     nonce, ctr0, (uint8_t*)out, nbytes);
  MX_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"

namespace {

int launch_rss_cross(int kind, int words, const void* x0, const void* x1, const void* y0,
                     const void* y1, void* out, int64_t n, int nparties, bool has_keys,
                     bool ring3, const KeySrc& k, uint64_t nonce, void* stream,
                     void* out1 = nullptr, int pairs = 0, const Views* views = nullptr) {
  Views vw{};
  if (views) vw = *views;
  if (n == 0) return 0;
  if (nparties < 1 || nparties > 3) return -3;
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    if (ring3) {
      const int64_t blocks = (n + P - 1) / P;
      if (blocks <= 65536) {  // latency-bound launch: one PRF chunk per thread, via LDS
        const int64_t g = (blocks + 84) / 85;
        hipLaunchKernelGGL(k_rss_cross_ring3_lat<T>, dim3((unsigned)g), dim3(kBlock), 0,
                           S(stream), kind, (const T*)x0, (const T*)x1, (const T*)y0,
                           (const T*)y1, (T*)out, (T*)out1, n, k, nonce, vw);
        MX_LAUNCH_CHECK();
        return 0;
      }
      hipLaunchKernelGGL(k_rss_cross_ring3<T>, dim3(mxd::grid_for_chunks(blocks)), dim3(kBlock), 0,
                         S(stream), kind, (const T*)x0, (const T*)x1, (const T*)y0,
                         (const T*)y1, (T*)out, (T*)out1, n, k, nonce, vw);
      MX_LAUNCH_CHECK();
      return 0;
    }
    const int64_t work = (int64_t)mx::ks_blocks_for((n + P - 1) / P) * nparties;
    hipLaunchKernelGGL(k_rss_cross<T>, dim3(grid_for(work)), dim3(kBlock), 0, S(stream), kind,
                       (const T*)x0, (const T*)x1, (const T*)y0, (const T*)y1, (T*)out, n,
                       nparties, has_keys ? 1 : 0, k, nonce, pairs);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int launch_prf_expand(int words, void* out, int64_t n, int nkeys, const KeySrc& k,
                      uint64_t nonce, void* stream) {
  if (n == 0) return 0;
  if (nkeys < 1 || nkeys > 4) return -3;
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    const int64_t work = (int64_t)mx::ks_blocks_for((n + P - 1) / P) * nkeys;
    hipLaunchKernelGGL(k_prf_expand<T>, dim3(grid_for(work)), dim3(kBlock), 0, S(stream),
                       (T*)out, n, nkeys, k, nonce);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

}  // namespace

extern "C" {

int mxh_rss_cross(int kind, int words, const void* x0, const void* x1, const void* y0,
                  const void* y1, void* out, int64_t n, int nparties, const uint8_t* keys16,
                  uint64_t nonce, void* stream) {
  KeySrc k = keys16 ? mxd::keysrc_host(keys16, nparties + 1) : mxd::keysrc_slots(nullptr, 0);
  const bool ring3 = keys16 && nparties == 3 && std::memcmp(keys16, keys16 + 48, 16) == 0;
  return launch_rss_cross(kind, words, x0, x1, y0, y1, out, n, nparties, keys16 != nullptr,
                          ring3, k, nonce, stream);
}

int mxh_rss_cross_k(int kind, int words, const void* x0, const void* x1, const void* y0,
                    const void* y1, void* out, int64_t n, int nparties, const uint32_t* slots,
                    int nslots, uint64_t nonce, void* stream) {
  if (nslots < 1 || nparties + 1 > 4) return -3;
  const uint32_t* ptrs[4];
  for (int i = 0; i <= nparties; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * (i % nslots);
  const bool ring3 = nparties == 3 && nslots == 3;
  KeySrc k = mxd::keysrc_slots(ptrs, ring3 ? 3 : nparties + 1);
  return launch_rss_cross(kind, words, x0, x1, y0, y1, out, n, nparties, true, ring3, k, nonce,
                          stream);
}

int mxh_rss_cross_kp(int kind, int words, const void* x0, const void* x1, const void* y0,
                     const void* y1, void* out, int64_t n, int nparties,
                     const uint32_t* const* slot_ptrs, uint64_t nonce, void* stream) {
  if (nparties < 1 || 2 * nparties > mxd::kMaxKeySlots) return -3;
  KeySrc k = mxd::keysrc_slots(slot_ptrs, 2 * nparties);
  return launch_rss_cross(kind, words, x0, x1, y0, y1, out, n, nparties, true, false, k, nonce,
                          stream, nullptr, 1);
}

int mxh_rss_mul3_k(int kind, int words, const void* x0, const void* x1, const void* y0,
                   const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                   uint64_t nonce, void* stream) {
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  return launch_rss_cross(kind, words, x0, x1, y0, y1, out0, n, 3, true, true,
                          mxd::keysrc_slots(ptrs, 3), nonce, stream, out1);
}

// mxh_rss_mul3_k with operand views: views = {ps[4], per[4]} in elements (see Views)
int mxh_rss_mul3_kv(int kind, int words, const void* x0, const void* x1, const void* y0,
                    const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                    uint64_t nonce, const int64_t* views, void* stream) {
  if (words != 1 && words != 2) return -2;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  Views vw;
  for (int i = 0; i < 4; ++i) {
    vw.ps[i] = views[i];
    vw.per[i] = views[4 + i] > 0 ? views[4 + i] : n;
  }
  vw.strided = 1;
  return launch_rss_cross(kind, words, x0, x1, y0, y1, out0, n, 3, true, true,
                          mxd::keysrc_slots(ptrs, 3), nonce, stream, out1, 0, &vw);
}

// k_mul_trunc3_lat for latency-bound launches, k_mul_trunc3 above.  x1 == y0 == y1 == null:
// x0 holds the parties' local products (the dot's tail).  views: {ps[4], per[4]} or null.
int mxh_mul_trunc3_kv(int words, const void* x0, const void* x1, const void* y0, const void* y1,
                      void* out0, void* out1, int64_t n, int64_t ostride, const uint32_t* slots,
                      uint64_t nmul, int m, const uint64_t* nn, const int64_t* views,
                      void* stream) {
  if (n == 0) return 0;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  Views vw{};
  if (views) {
    for (int i = 0; i < 4; ++i) {
      vw.ps[i] = views[i];
      vw.per[i] = views[4 + i] > 0 ? views[4 + i] : n;
    }
    vw.strided = 1;
  }
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    const int64_t blocks = (n + P - 1) / P;
    if (blocks > 8192) {
      hipLaunchKernelGGL(k_mul_trunc3<T>, dim3(mxd::grid_for_chunks(blocks)), dim3(kBlock), 0,
                         S(stream), (const T*)x0, (const T*)x1, (const T*)y0, (const T*)y1,
                         (T*)out0, (T*)out1, n, ostride, mxd::keysrc_slots(ptrs, 3), nmul, m,
                         nn[0], nn[1], nn[2], nn[3], nn[4], nn[5], vw);
      MX_LAUNCH_CHECK();
      return 0;
    }
    constexpr int EPB = 256 / 9;
    const int64_t g = (blocks + EPB - 1) / EPB;
    hipLaunchKernelGGL(k_mul_trunc3_lat<T>, dim3((unsigned)g), dim3(kBlock), 0, S(stream),
                       (const T*)x0, (const T*)x1, (const T*)y0, (const T*)y1, (T*)out0,
                       (T*)out1, n, ostride, mxd::keysrc_slots(ptrs, 3), nmul, m, nn[0], nn[1],
                       nn[2], nn[3], nn[4], nn[5], vw);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

// Two k_mul_trunc3_lat problems of one placement in one launch (k_mul_trunc3_lat2): per
// problem i the arguments of mxh_mul_trunc3_kv at index i of each array; nn: 6 nonces per
// problem; views: 8 int64 per problem or a null pointer per problem.  Only for latency-bound
// sizes (the throughput kernel has no two-problem form): -1 otherwise.
int mxh_mul_trunc3_kv2(int words, const void* const* x0, const void* const* x1,
                       const void* const* y0, const void* const* y1, void* const* out0,
                       void* const* out1, const int64_t* n, const int64_t* ostride,
                       const uint32_t* slots, const uint64_t* nmul, const int* m,
                       const uint64_t* nn, const int64_t* const* views, void* stream) {
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    constexpr int EPB = 256 / 9;
    MT2<T> a{};
    int64_t g = 1;
    for (int i = 0; i < 2; ++i) {
      const int64_t blocks = (n[i] + P - 1) / P;
      if (n[i] <= 0 || blocks > 8192) return -1;
      g = std::max<int64_t>(g, (blocks + EPB - 1) / EPB);
      a.x0[i] = (const T*)x0[i];
      a.x1[i] = (const T*)x1[i];
      a.y0[i] = (const T*)y0[i];
      a.y1[i] = (const T*)y1[i];
      a.out0[i] = (T*)out0[i];
      a.out1[i] = (T*)out1[i];
      a.n[i] = n[i];
      a.os[i] = ostride[i];
      a.nmul[i] = nmul[i];
      a.m[i] = m[i];
      for (int k = 0; k < 6; ++k) a.nn[i][k] = nn[6 * i + k];
      a.vw[i] = Views{};
      if (views[i]) {
        for (int k = 0; k < 4; ++k) {
          a.vw[i].ps[k] = views[i][k];
          a.vw[i].per[k] = views[i][4 + k] > 0 ? views[i][4 + k] : n[i];
        }
        a.vw[i].strided = 1;
      }
    }
    hipLaunchKernelGGL(k_mul_trunc3_lat2<T>, dim3((unsigned)g, 2), dim3(kBlock), 0, S(stream), a,
                       mxd::keysrc_slots(ptrs, 3));
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_ks_cross1(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                  void* z, int64_t n, int d, int both, const uint8_t* keys16, uint64_t nonce,
                  void* stream) {
  if (n == 0) return 0;
  KeySrc k = mxd::keysrc_host(keys16, 2);
  if (words == 1) {
    hipLaunchKernelGGL(k_ks_cross1<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)g0, (const u64*)g1, (const u64*)p0, (const u64*)p1, (u64*)z,
                       n, d, both, k, nonce);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_ks_cross1<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)g0, (const u128*)g1, (const u128*)p0, (const u128*)p1,
                       (u128*)z, n, d, both, k, nonce);
  } else {
    return -2;
  }
  MX_LAUNCH_CHECK();
  return 0;
}

// mxh_b2a3 over bit planes start..start+count-1 of packed boolean share words w0, w1
// ([3][m] ring words): out [3][count * m] (plane-major per party, as BitSplit lays them)
int mxh_b2a3_planes(int words, const void* w0, const void* w1, int64_t m, int start, int count,
                    void* out0, void* out1, const uint32_t* slots, int mir, uint64_t n1,
                    uint64_t nmul, void* stream) {
  const int64_t n = m * count;
  if (n == 0) return 0;
  if (words != 1 && words != 2) return -2;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    const int64_t g = std::min<int64_t>(((n + P - 1) / P + 63) / 64, 16384);
    hipLaunchKernelGGL(k_b2a3<T>, dim3((unsigned)g), dim3(256), 0, S(stream), nullptr, nullptr,
                       (T*)out0, (T*)out1, n, mxd::keysrc_slots(ptrs, 3), mir ? 1 : 0, n1, nmul,
                       (const T*)w0, (const T*)w1, start, m);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

int mxh_mul_rows_add(int words, const void* a, const void* f, void* out, int64_t n,
                     int64_t per, const void* c, int ra, int rb, void* stream) {
  if (n == 0) return 0;
  if (words != 1 && words != 2) return -2;
  DEV_DISPATCH(words, T, {
    hipLaunchKernelGGL(k_mul_rows_add<T>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const T*)a, (const T*)f, (T*)out, n, per, (const T*)c, ra, rb);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

// slots: k0, k1, k2 of the placement
// absv: x - 2 s x instead (y unused)
int mxh_mux3(int words, const void* s0, const void* s1, const void* x0, const void* x1,
             const void* y0, const void* y1, void* out0, void* out1, int64_t n,
             const uint32_t* slots, uint64_t nonce, int absv, void* stream) {
  if (n == 0) return 0;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  DEV_DISPATCH(words, T, {
    constexpr int P = 16 / (int)sizeof(T);
    const int64_t g = std::min<int64_t>(((n + P - 1) / P + 84) / 85, 16384);
    hipLaunchKernelGGL(k_mux3_lat<T>, dim3((unsigned)g), dim3(256), 0, S(stream), (const T*)s0,
                       (const T*)s1, (const T*)x0, (const T*)x1, (const T*)y0, (const T*)y1,
                       (T*)out0, (T*)out1, n, mxd::keysrc_slots(ptrs, 3), nonce, absv);
    MX_LAUNCH_CHECK();
    return 0;
  });
}

// slots: k0, k1, k2 of the placement; nonces: one per adder level (nlev <= 8)
int mxh_bitdec3(int words, const void* x0, const void* x1, void* o0, void* o1, int64_t n,
                int nlev, const uint32_t* slots, int mir, uint64_t n1, uint64_t nmul,
                const uint64_t* nonces, int sign, uint64_t n1b, uint64_t nmulb, void* stream) {
  if (n == 0) return 0;
  if (n > 65536 || nlev < 1 || nlev > 8) return -1;  // latency sizes only
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  Nonces8 nn{};
  for (int i = 0; i < nlev; ++i) nn.v[i] = nonces[i];
  const unsigned g = (unsigned)((n + 4) / 5);
  const KeySrc ks = mxd::keysrc_slots(ptrs, 3);
  const int m = mir ? 1 : 0;
  if (words == 1 && !sign)
    hipLaunchKernelGGL((k_bitdec3<u64, false>), dim3(g), dim3(256), 0, S(stream), (const u64*)x0,
                       (const u64*)x1, (u64*)o0, (u64*)o1, n, nlev, ks, m, n1, nmul, nn, n1b,
                       nmulb);
  else if (words == 1)
    hipLaunchKernelGGL((k_bitdec3<u64, true>), dim3(g), dim3(256), 0, S(stream), (const u64*)x0,
                       (const u64*)x1, (u64*)o0, (u64*)o1, n, nlev, ks, m, n1, nmul, nn, n1b,
                       nmulb);
  else if (words == 2 && !sign)
    hipLaunchKernelGGL((k_bitdec3<u128, false>), dim3(g), dim3(256), 0, S(stream),
                       (const u128*)x0, (const u128*)x1, (u128*)o0, (u128*)o1, n, nlev, ks, m,
                       n1, nmul, nn, n1b, nmulb);
  else if (words == 2)
    hipLaunchKernelGGL((k_bitdec3<u128, true>), dim3(g), dim3(256), 0, S(stream),
                       (const u128*)x0, (const u128*)x1, (u128*)o0, (u128*)o1, n, nlev, ks, m,
                       n1, nmul, nn, n1b, nmulb);
  else
    return -2;
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_ks_cross1x_s(int words, const void* g0, const void* g1, const void* t0, const void* t1,
                     void* go0, void* go1, const void* p0, const void* p1, void* z, int64_t n,
                     int d, int both, const uint32_t* const* slots, uint64_t nonce,
                     void* stream) {
  if (n == 0) return 0;
  KeySrc k = mxd::keysrc_slots(slots, 2);
  if ((words == 1 && ks_lat_launch<u64>(g0, g1, t0, t1, go0, go1, p0, p1, z, n, d, both, k,
                                        nonce, S(stream))) ||
      (words == 2 && ks_lat_launch<u128>(g0, g1, t0, t1, go0, go1, p0, p1, z, n, d, both, k,
                                         nonce, S(stream)))) {
    MX_LAUNCH_CHECK();
    return 0;
  }
  if (words == 1) {
    hipLaunchKernelGGL(k_ks_cross1<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)g0, (const u64*)g1, (const u64*)p0, (const u64*)p1, (u64*)z,
                       n, d, both, k, nonce, (const u64*)t0, (const u64*)t1, (u64*)go0,
                       (u64*)go1);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_ks_cross1<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)g0, (const u128*)g1, (const u128*)p0, (const u128*)p1,
                       (u128*)z, n, d, both, k, nonce, (const u128*)t0, (const u128*)t1,
                       (u128*)go0, (u128*)go1);
  } else {
    return -2;
  }
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_ks_sum2(int words, const void* p0, const void* p1, const void* g0, const void* g1,
                const void* t0, const void* t1, void* o0, void* o1, int64_t n, void* stream) {
  if (n == 0) return 0;
  if (words == 1) {
    hipLaunchKernelGGL(k_ks_sum2<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)p0, (const u64*)p1, (const u64*)g0, (const u64*)g1,
                       (const u64*)t0, (const u64*)t1, (u64*)o0, (u64*)o1, n);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_ks_sum2<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)p0, (const u128*)p1, (const u128*)g0, (const u128*)g1,
                       (const u128*)t0, (const u128*)t1, (u128*)o0, (u128*)o1, n);
  } else {
    return -2;
  }
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_ks_cross1_s(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                    void* z, int64_t n, int d, int both, const uint32_t* const* slots,
                    uint64_t nonce, void* stream) {
  if (n == 0) return 0;
  KeySrc k = mxd::keysrc_slots(slots, 2);
  if ((words == 1 && ks_lat_launch<u64>(g0, g1, nullptr, nullptr, nullptr, nullptr, p0, p1, z,
                                        n, d, both, k, nonce, S(stream))) ||
      (words == 2 && ks_lat_launch<u128>(g0, g1, nullptr, nullptr, nullptr, nullptr, p0, p1, z,
                                         n, d, both, k, nonce, S(stream)))) {
    MX_LAUNCH_CHECK();
    return 0;
  }
  if (words == 1) {
    hipLaunchKernelGGL(k_ks_cross1<u64>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)g0, (const u64*)g1, (const u64*)p0, (const u64*)p1, (u64*)z,
                       n, d, both, k, nonce);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_ks_cross1<u128>, dim3(grid_for(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)g0, (const u128*)g1, (const u128*)p0, (const u128*)p1,
                       (u128*)z, n, d, both, k, nonce);
  } else {
    return -2;
  }
  MX_LAUNCH_CHECK();
  return 0;
}

inline int ks_grid(int64_t items, int per_block = 256 / 6) {
  int64_t b = (items + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 8192));
}

int mxh_ks_level3_k(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                    void* og0, void* og1, void* op0, void* op1, int64_t n, int d, int both,
                    const uint32_t* slots, uint64_t nonce, void* stream) {
  if (n == 0) return 0;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  KeySrc k = mxd::keysrc_slots(ptrs, 3);
  if (words == 1) {
    hipLaunchKernelGGL(k_ks_level3<u64>, dim3(ks_grid(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)g0, (const u64*)g1, (const u64*)p0, (const u64*)p1,
                       (u64*)og0, (u64*)og1, (u64*)op0, (u64*)op1, n, d, both, k, nonce);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_ks_level3<u128>, dim3(ks_grid(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)g0, (const u128*)g1, (const u128*)p0, (const u128*)p1,
                       (u128*)og0, (u128*)og1, (u128*)op0, (u128*)op1, n, d, both, k, nonce);
  } else {
    return -2;
  }
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_ks_adder3_sum(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                      void* og0, void* og1, int64_t n, int nlev, const uint32_t* slots,
                      const uint64_t* nonces, void* stream, int sum_out);

int mxh_ks_adder3_k(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                    void* og0, void* og1, int64_t n, int nlev, const uint32_t* slots,
                    const uint64_t* nonces, void* stream) {
  return mxh_ks_adder3_sum(words, g0, g1, p0, p1, og0, og1, n, nlev, slots, nonces, stream, 0);
}

// The chain, returning the adder's sum p ^ (g << 1) when ``sum_out`` (the carries otherwise).
int mxh_ks_adder3_sum(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                      void* og0, void* og1, int64_t n, int nlev, const uint32_t* slots,
                      const uint64_t* nonces, void* stream, int sum_out) {
  if (n == 0) return 0;
  if (nlev < 1 || nlev > 8) return -3;
  const uint32_t* ptrs[3];
  for (int i = 0; i < 3; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  KeySrc k = mxd::keysrc_slots(ptrs, 3);
  Nonces8 nn{};
  for (int l = 0; l < nlev; ++l) nn.v[l] = nonces[l];
  if (n <= 65536 && (words == 1 || words == 2)) {  // latency-bound: masks first
    if (words == 1)
      hipLaunchKernelGGL(k_ks_adder3p<u64>, dim3(ks_grid(n, 6)), dim3(kBlock), 0, S(stream),
                         (const u64*)g0, (const u64*)g1, (const u64*)p0, (const u64*)p1,
                         (u64*)og0, (u64*)og1, n, nlev, k, nn, sum_out);
    else
      hipLaunchKernelGGL(k_ks_adder3p<u128>, dim3(ks_grid(n, 6)), dim3(kBlock), 0, S(stream),
                         (const u128*)g0, (const u128*)g1, (const u128*)p0, (const u128*)p1,
                         (u128*)og0, (u128*)og1, n, nlev, k, nn, sum_out);
  } else if (words == 1) {
    hipLaunchKernelGGL(k_ks_adder3<u64>, dim3(ks_grid(n)), dim3(kBlock), 0, S(stream),
                       (const u64*)g0, (const u64*)g1, (const u64*)p0, (const u64*)p1,
                       (u64*)og0, (u64*)og1, n, nlev, k, nn, sum_out);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_ks_adder3<u128>, dim3(ks_grid(n)), dim3(kBlock), 0, S(stream),
                       (const u128*)g0, (const u128*)g1, (const u128*)p0, (const u128*)p1,
                       (u128*)og0, (u128*)og1, n, nlev, k, nn, sum_out);
  } else {
    return -2;
  }
  MX_LAUNCH_CHECK();
  return 0;
}

int mxh_prf_expand(int words, void* out, int64_t n, int nkeys, const uint8_t* keys16,
                   uint64_t nonce, void* stream) {
  return launch_prf_expand(words, out, n, nkeys, mxd::keysrc_host(keys16, nkeys), nonce, stream);
}

int mxh_prf_expand_k(int words, void* out, int64_t n, int nkeys, const uint32_t* slots,
                     uint64_t nonce, void* stream) {
  if (nkeys < 1 || nkeys > 4) return -3;
  const uint32_t* ptrs[4];
  for (int i = 0; i < nkeys; ++i) ptrs[i] = slots + MX_KEY_SLOT_WORDS * i;
  return launch_prf_expand(words, out, n, nkeys, mxd::keysrc_slots(ptrs, nkeys), nonce, stream);
}

int mxh_gemm(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
             const void* A1, const void* B0, const void* B1, int mode, void* C, int accumulate,
             void* stream) {
  if (M == 0 || N == 0 || batch == 0) return 0;
  bool big = M >= 64 && N >= 64 && K >= 32;
  if ((g_gemm_impl == 2 || (g_gemm_impl == 0 && big)) && (words == 1 || words == 2))
    return mxh_gemm_mfma(words, batch, M, N, K, A0, A1, B0, B1, mode, C, accumulate, stream);
  if (words == 1)
    return launch_gemm_valu<u64>(batch, M, N, K, A0, A1, B0, B1, mode, C, accumulate,
                                 S(stream));
  if (words == 2)
    return launch_gemm_valu<u128>(batch, M, N, K, A0, A1, B0, B1, mode, C, accumulate,
                                  S(stream));
  return -2;
}

// Plain batched product with explicit batch strides (elements; 0 broadcasts an operand):
// the small-product (VALU) kernel, or the strided MFMA/CRT GEMM for large ones.
extern "C" int mx_gemm_strided(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                               const void* A0, const void* A1, int64_t a_bstride, const void* B0,
                               const void* B1, int64_t b_bstride, int mode, void* C,
                               int accumulate, void* stream);

int mxh_gemm_bs(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                int64_t a_bs, const void* B0, int64_t b_bs, void* C, void* stream) {
  if (M == 0 || N == 0 || batch == 0) return 0;
  const bool big = M >= 64 && N >= 64 && K >= 32;
  if (big && g_gemm_impl != 1)
    return mx_gemm_strided(words, batch, M, N, K, A0, nullptr, a_bs, B0, nullptr, b_bs, 0, C, 0,
                           stream);
  if (words == 1)
    return launch_gemm_valu<u64>(batch, M, N, K, A0, nullptr, B0, nullptr, 0, C, 0, S(stream),
                                 a_bs, b_bs);
  if (words == 2)
    return launch_gemm_valu<u128>(batch, M, N, K, A0, nullptr, B0, nullptr, 0, C, 0, S(stream),
                                  a_bs, b_bs);
  return -2;
}

}  // extern "C"
