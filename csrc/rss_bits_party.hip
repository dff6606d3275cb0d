// Per-party bit decomposition front and B2A kernels (bits_party.h has the protocol): one
// party per GPU / process / thread.  Latency form only -- these run on the LR inference's
// few-hundred-element values: the keystream chunks of a block's EPB positions, for every
// stream the role draws, are computed one per thread into LDS, then the elements finished.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "bits_party.h"
#include "moosex.h"
#include "party_batch.h"
#include "prf_dev.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

namespace {

constexpr int EPB = 64;

struct Str {
  int n;
  int key[3];  // 0 = own, 1 = next
  uint64_t nonce[3];
};

// stage the block's chunks [b0, b0 + EPB) of ss.n streams into kl / kh
__device__ inline void stage(const uint32_t (*rks)[mxd::kKeyWords], const Str& ss, int64_t b0,
                             int64_t nb, uint64_t (*kl)[EPB], uint64_t (*kh)[EPB]) {
  const int s = threadIdx.x / EPB, lb = threadIdx.x % EPB;
  if (s < ss.n && b0 + lb < nb) {
    uint64_t lo, hi;
    mxd::prf_chunk(rks[ss.key[s]], ss.nonce[s], (uint64_t)(b0 + lb), &lo, &hi);
    kl[s][lb] = lo;
    kh[s][lb] = hi;
  }
}

template <class T>
__device__ __forceinline__ void d_front(int role, int64_t n, const T* __restrict__ xa,
                                        const T* __restrict__ xb, const T* __restrict__ arecv,
                                        T* __restrict__ msg, T* __restrict__ z, T* __restrict__ p0,
                                        T* __restrict__ p1, const mxd::KeySrc& keys,
                                        const Str& ss) {
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  __shared__ uint64_t kl[3][EPB], kh[3][EPB];
  mxd::stage_keys(rks, keys, 2);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    stage(rks, ss, b0, nb, kl, kh);
    __syncthreads();
    for (int q = threadIdx.x; q < EPB * P; q += blockDim.x) {
      const int64_t i = b0 * P + q;
      if (i >= n) break;
      const int lc = q / P, j = q % P;
      // streams: role 0 / 2: fa, fo, fn; role 1: fo, fn
      const int o = role == 1 ? 0 : 1;
      const T fa = role == 1 ? (T)0 : mxd::pick<T>(kl[0][lc], kh[0][lc], j);
      const T fo = mxd::pick<T>(kl[o][lc], kh[o][lc], j);
      const T fn = mxd::pick<T>(kl[o + 1][lc], kh[o + 1][lc], j);
      const mxb::Front<T> r = mxb::front<T>(role, role == 1 ? (T)0 : xa[i], role == 2 ? (T)0 : xb[i],
                                            role == 1 ? arecv[i] : (T)0, fa, fo, fn);
      if (role == 0) msg[i] = r.msg;
      z[i] = r.z;
      p0[i] = r.p0;
      p1[i] = r.p1;
    }
    __syncthreads();
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_front(int role, int64_t n, const T* __restrict__ xa,
                                               const T* __restrict__ xb,
                                               const T* __restrict__ arecv, T* __restrict__ msg,
                                               T* __restrict__ z, T* __restrict__ p0,
                                               T* __restrict__ p1, mxd::KeySrc keys, Str ss) {
  d_front<T>(role, n, xa, xb, arecv, msg, z, p0, p1, keys, ss);
}

// source bit of component c at (plane row, element e): from the adder's sum words, or from
// its raw (p, g, t) of the last level (g == null: s are sum words)
template <class T>
__device__ __forceinline__ T src_bit(const T* s, const T* g, const T* t, int64_t e, int qbit) {
  if (g == nullptr) return (s[e] >> qbit) & (T)1;
  return mxb::sum_bit<T>(s[e], g[e], t ? t[e] : (T)0, qbit);
}

template <class T>
__device__ __forceinline__ void d_b2a(int phase, int role, int64_t S, int start, int count,
                                      int xbit, int blocks, const T* __restrict__ s0,
                                      const T* __restrict__ s1, const T* __restrict__ g0,
                                      const T* __restrict__ g1, const T* __restrict__ t0,
                                      const T* __restrict__ t1, const T* __restrict__ arecv,
                                      T* __restrict__ msg, T* __restrict__ z, T* __restrict__ base0,
                                      T* __restrict__ base1, const T* __restrict__ zr,
                                      T* __restrict__ out0, T* __restrict__ out1,
                                      const mxd::KeySrc& keys, const Str& ss) {
  const int64_t n = S * count;
  if (phase == 2) {  // out = base - 2 (z, z_received)
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
      out0[i] = base0[i] - (T)2 * z[i];
      out1[i] = base1[i] - (T)2 * zr[i];
    }
    return;
  }
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  __shared__ uint64_t kl[3][EPB], kh[3][EPB];
  mxd::stage_keys(rks, keys, 2);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    stage(rks, ss, b0, nb, kl, kh);
    __syncthreads();
    for (int q = threadIdx.x; q < EPB * P; q += blockDim.x) {
      const int64_t i = b0 * P + q;
      if (i >= n) break;
      const int lc = q / P, j = q % P;
      const int64_t row = i / S, e = i - row * S;
      int qbit, xq, blk, neg;
      mxb::plane_of((int)row, start, count, xbit, blocks, &qbit, &xq, &blk, &neg);
      const int64_t es = e + blk * S;  // the element in the adder's blocks
      const int o = role == 1 ? 0 : 1;
      const T fa = role == 1 ? (T)0 : mxd::pick<T>(kl[0][lc], kh[0][lc], j);
      const T fo = mxd::pick<T>(kl[o][lc], kh[o][lc], j);
      const T fn = mxd::pick<T>(kl[o + 1][lc], kh[o + 1][lc], j);
      T c0 = role == 1 ? (T)0 : src_bit<T>(s0, g0, t0, es, qbit);
      T c1 = role == 2 ? (T)0 : src_bit<T>(s1, g1, t1, es, qbit);
      if (xq >= 0) {  // share-wise XOR with plane xq (local on boolean shares)
        if (role != 1) c0 ^= src_bit<T>(s0, g0, t0, es, xq);
        if (role != 2) c1 ^= src_bit<T>(s1, g1, t1, es, xq);
      }
      if (neg && role == 0) c0 ^= (T)1;  // NOT: component 0 (P0's first) flipped
      const mxb::B2a<T> r = mxb::b2a<T>(role, c0, c1, role == 1 ? arecv[i] : (T)0, fa, fo, fn);
      if (role == 0) msg[i] = r.msg;
      z[i] = r.z;
      base0[i] = r.base0;
      base1[i] = r.base1;
    }
    __syncthreads();
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_b2a(int phase, int role, int64_t S, int start, int count,
                                             int xbit, int blocks, const T* __restrict__ s0,
                                             const T* __restrict__ s1, const T* __restrict__ g0,
                                             const T* __restrict__ g1, const T* __restrict__ t0,
                                             const T* __restrict__ t1, const T* __restrict__ arecv,
                                             T* __restrict__ msg, T* __restrict__ z,
                                             T* __restrict__ base0, T* __restrict__ base1,
                                             const T* __restrict__ zr, T* __restrict__ out0,
                                             T* __restrict__ out1, mxd::KeySrc keys, Str ss) {
  d_b2a<T>(phase, role, S, start, count, xbit, blocks, s0, s1, g0, g1, t0, t1, arecv, msg, z, base0,
           base1, zr, out0, out1, keys, ss);
}

// Throughput form of phases 0 / 1 (larger B2As, e.g. all bit planes of a decomposition): one
// thread per ChaCha block index of every stream the role draws, its 4 chunks' elements
// finished from registers -- a quarter of the latency form's keystream work (which computes a
// whole block for each chunk), the same chunk -> element mapping (so bitwise the same).
template <class T>
__device__ __forceinline__ void d_b2a_tp(int role, int64_t S, int start, int count, int xbit,
                                         int blocks, const T* __restrict__ s0,
                                         const T* __restrict__ s1, const T* __restrict__ g0,
                                         const T* __restrict__ g1, const T* __restrict__ t0,
                                         const T* __restrict__ t1, const T* __restrict__ arecv,
                                         T* __restrict__ msg, T* __restrict__ z,
                                         T* __restrict__ base0, T* __restrict__ base1,
                                         const mxd::KeySrc& keys, const Str& ss) {
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t n = S * count;
  const int64_t nch = (n + P - 1) / P;
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)nch);
  const int o = role == 1 ? 0 : 1;
  for (int64_t B = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; B < nblk;
       B += (int64_t)gridDim.x * blockDim.x) {
    uint32_t w[3][16];
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < ss.n) mx::chacha_block(rks[ss.key[q]], ss.nonce[q], (uint64_t)B, w[q]);
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int64_t c = (int64_t)mx::ks_chunk((uint64_t)B, part);
      if (c >= nch) break;
      uint64_t lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q < ss.n) mx::part_u64(w[q], part, &lo[q], &hi[q]);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = c * P + j;
        if (i >= n) break;
        const int64_t row = i / S, e = i - row * S;
        int qbit, xq, blk, neg;
        mxb::plane_of((int)row, start, count, xbit, blocks, &qbit, &xq, &blk, &neg);
        const int64_t es = e + blk * S;
        const T fa = role == 1 ? (T)0 : mxd::pick<T>(lo[0], hi[0], j);
        const T fo = mxd::pick<T>(lo[o], hi[o], j);
        const T fn = mxd::pick<T>(lo[o + 1], hi[o + 1], j);
        T c0 = role == 1 ? (T)0 : src_bit<T>(s0, g0, t0, es, qbit);
        T c1 = role == 2 ? (T)0 : src_bit<T>(s1, g1, t1, es, qbit);
        if (xq >= 0) {
          if (role != 1) c0 ^= src_bit<T>(s0, g0, t0, es, xq);
          if (role != 2) c1 ^= src_bit<T>(s1, g1, t1, es, xq);
        }
        if (neg && role == 0) c0 ^= (T)1;
        const mxb::B2a<T> r = mxb::b2a<T>(role, c0, c1, role == 1 ? arecv[i] : (T)0, fa, fo, fn);
        if (role == 0) msg[i] = r.msg;
        z[i] = r.z;
        base0[i] = r.base0;
        base1[i] = r.base1;
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_b2a_tp(int role, int64_t S, int start, int count, int xbit,
                                                int blocks, const T* __restrict__ s0,
                                                const T* __restrict__ s1, const T* __restrict__ g0,
                                                const T* __restrict__ g1, const T* __restrict__ t0,
                                                const T* __restrict__ t1,
                                                const T* __restrict__ arecv, T* __restrict__ msg,
                                                T* __restrict__ z, T* __restrict__ base0,
                                                T* __restrict__ base1, mxd::KeySrc keys, Str ss) {
  d_b2a_tp<T>(role, S, start, count, xbit, blocks, s0, s1, g0, g1, t0, t1, arecv, msg, z, base0,
              base1, keys, ss);
}

// party-batched twins for the composed one-GPU replay (party_batch.h)
MX_X3(k_front<u64>, d_front<u64>);
MX_X3(k_front<u128>, d_front<u128>);
MX_X3(k_b2a<u64>, d_b2a<u64>);
MX_X3(k_b2a<u128>, d_b2a<u128>);
MX_X3(k_b2a_tp<u64>, d_b2a_tp<u64>);
MX_X3(k_b2a_tp<u128>, d_b2a_tp<u128>);

Str streams(int role, const uint64_t* nn) {
  // nn = (n1, n_g); role 0: (own, n1), role 2: (next, n1); then (own, n_g), (next, n_g)
  Str s{};
  int k = 0;
  if (role != 1) {
    s.key[k] = role == 0 ? 0 : 1;
    s.nonce[k++] = nn[0];
  }
  s.key[k] = 0;
  s.nonce[k++] = nn[1];
  s.key[k] = 1;
  s.nonce[k++] = nn[1];
  s.n = k;
  return s;
}

template <class T>
unsigned grid_of(int64_t n) {
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  int64_t g = (nb + EPB - 1) / EPB;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (unsigned)g;
}

}  // namespace

extern "C" {

int mxh_bits_front(int words, int role, int64_t n, const void* xa, const void* xb,
                   const void* arecv, void* msg, void* z, void* p0, void* p1,
                   const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  if (n == 0) return 0;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2);
  const Str ss = streams(role, nn);
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    hipLaunchKernelGGL(k_front<u64>, dim3(grid_of<u64>(n)), dim3(256), 0, st, role, n,
                       (const u64*)xa, (const u64*)xb, (const u64*)arecv, (u64*)msg, (u64*)z,
                       (u64*)p0, (u64*)p1, k, ss);
  else if (words == 2)
    hipLaunchKernelGGL(k_front<u128>, dim3(grid_of<u128>(n)), dim3(256), 0, st, role, n,
                       (const u128*)xa, (const u128*)xb, (const u128*)arecv, (u128*)msg,
                       (u128*)z, (u128*)p0, (u128*)p1, k, ss);
  else
    return -2;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_bits_b2a(int words, int phase, int role, int64_t S, int start, int count, int xbit,
                 int blocks, const void* const* src, const void* arecv, void* msg, void* z, void* base0,
                 void* base1, const void* zr, void* out0, void* out1,
                 const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  const int64_t n = S * count;
  if (n == 0) return 0;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2);
  const Str ss = streams(role, nn);
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = phase == 2 ? (unsigned)mxd::grid_for(n) : 0;
  const void* none[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (src == nullptr) src = none;  // phase 2 reads no source
  // phases 0 / 1 over more than a few thousand chunks: the throughput form
  const int64_t nch_ = words == 2 ? n : (n + 1) / 2;
  if (phase != 2 && nch_ >= 2048 && getenv("MOOSEX_B2A_TP") == nullptr) {
#define MX_B2A_TP(T)                                                                         \
  hipLaunchKernelGGL(k_b2a_tp<T>, dim3(mxd::grid_for_chunks(nch_)), dim3(256), 0, st, role, S, \
                     start, count, xbit, blocks, (const T*)src[0], (const T*)src[1],          \
                     (const T*)src[2], (const T*)src[3], (const T*)src[4], (const T*)src[5],  \
                     (const T*)arecv, (T*)msg, (T*)z, (T*)base0, (T*)base1, k, ss)
    if (words == 1)
      MX_B2A_TP(u64);
    else if (words == 2)
      MX_B2A_TP(u128);
    else
      return -2;
#undef MX_B2A_TP
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -100 - (int)e;
  }
#define MX_B2A_LAUNCH(T)                                                                   \
  hipLaunchKernelGGL(k_b2a<T>, dim3(phase == 2 ? g : grid_of<T>(n)), dim3(256), 0, st, phase, \
                     role, S, start, count, xbit, blocks, (const T*)src[0], (const T*)src[1],            \
                     (const T*)src[2], (const T*)src[3], (const T*)src[4], (const T*)src[5], \
                     (const T*)arecv, (T*)msg, (T*)z, (T*)base0, (T*)base1, (const T*)zr,  \
                     (T*)out0, (T*)out1, k, ss)
  if (words == 1)
    MX_B2A_LAUNCH(u64);
  else if (words == 2)
    MX_B2A_LAUNCH(u128);
  else
    return -2;
#undef MX_B2A_LAUNCH
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

}  // extern "C"
