// gfx950 versions of the fused stacked-session protocol kernels (rss_fused.h).
//
// trunc_pr3: one pass per element computes the dealer's masks, both parties' masked
// openings, the local truncation and the additive->replicated conversion for all three
// parties -- six keystream chunks (prf_core.h) and ~40 integer ops per element, one read of
// the three input slots, one write of the two output share vectors.
// share3: input sharing by a member party (two keystream chunks per element).
#include <hip/hip_runtime.h>

#include "prf_dev.h"
#include "moosex.h"
#include "ring_common.h"
#include "rss_fused.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

namespace {

template <class T>
__global__ void __launch_bounds__(256) k_trunc_pr3(const T* __restrict__ s0, T* __restrict__ out0, T* __restrict__ out1,
                            int64_t n, int64_t os, T cm, int m, mxd::KeySrc keys, uint64_t n_r0, uint64_t n_r1,
                            uint64_t n_t, uint64_t n_m, uint64_t n_z0, uint64_t n_z2) {
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  // streams r0, r1, t, m, z0, z2 (dealer keys k0 / k2)
  const uint32_t* const key[6] = {rks[0], rks[1], rks[0], rks[0], rks[0], rks[1]};
  const uint64_t nonce[6] = {n_r0, n_r1, n_t, n_m, n_z0, n_z2};
  mxd::walk_chunks<6>(nb, key, nonce, [&](int64_t b, const uint64_t (&lo)[6], const uint64_t (&hi)[6]) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t i = b * P + j;
      if (i >= n) break;
      const T z0 = mxd::pick<T>(lo[4], hi[4], j);
      const T z2 = mxd::pick<T>(lo[5], hi[5], j);
      const T z1 = mxf::trunc_pr_z1<T>(cm * s0[i], cm * s0[n + i], cm * s0[2 * n + i], mxd::pick<T>(lo[0], hi[0], j),
                                       mxd::pick<T>(lo[1], hi[1], j), mxd::pick<T>(lo[2], hi[2], j),
                                       mxd::pick<T>(lo[3], hi[3], j), z0, z2, m);
      out0[i] = z0;
      out0[os + i] = z1;
      out0[2 * os + i] = z2;
      if (out1 != out0 + os) {  // else out1 = out0 + os: a 4-slot ring, slots 1, 2 shared
        out1[i] = z1;
        out1[os + i] = z2;
      }
      out1[2 * os + i] = z0;
    }
  });
}

// Latency variant (small n): the six keystream chunks of each of the block's EPB chunk
// positions are computed one per thread into LDS; then EPB threads finish the elements.
template <class T>
__global__ void __launch_bounds__(256) k_trunc_pr3_lat(const T* __restrict__ s0, T* __restrict__ out0,
                                                       T* __restrict__ out1, int64_t n,
                                                       int64_t os, T cm, int m, mxd::KeySrc keys, uint64_t n_r0,
                                                       uint64_t n_r1, uint64_t n_t, uint64_t n_m,
                                                       uint64_t n_z0, uint64_t n_z2) {
  constexpr int EPB = 256 / 6;
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  __shared__ uint64_t kl[6][EPB], kh[6][EPB];
  mxd::stage_keys(rks, keys, 2);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  // stream s: (key, nonce) of r0, r1, t, m, z0, z2 -- as in k_trunc_pr3
  const int key_of = (s == 1 || s == 5) ? 1 : 0;
  const uint64_t nonce_of = s == 0 ? n_r0 : s == 1 ? n_r1 : s == 2 ? n_t : s == 3 ? n_m
                            : s == 4 ? n_z0 : n_z2;
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    // the finishing threads' operands first: their loads overlap the keystream work
    const bool fin = tid < EPB && b0 + tid < nb;
    T xv[P][3];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t i = (b0 + tid) * P + j;
#pragma unroll
      for (int p = 0; p < 3; ++p) xv[j][p] = fin && i < n ? cm * s0[p * n + i] : (T)0;
    }
    if (s < 6 && b0 + lb < nb) {
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
        const int64_t i = b * P + j;
        if (i >= n) break;
        const T z0 = mxd::pick<T>(kl[4][tid], kh[4][tid], j);
        const T z2 = mxd::pick<T>(kl[5][tid], kh[5][tid], j);
        const T z1 = mxf::trunc_pr_z1<T>(
            xv[j][0], xv[j][1], xv[j][2], mxd::pick<T>(kl[0][tid], kh[0][tid], j),
            mxd::pick<T>(kl[1][tid], kh[1][tid], j), mxd::pick<T>(kl[2][tid], kh[2][tid], j),
            mxd::pick<T>(kl[3][tid], kh[3][tid], j), z0, z2, m);
        out0[i] = z0;
        out0[os + i] = z1;
        out0[2 * os + i] = z2;
        if (out1 != out0 + os) {
          out1[i] = z1;
          out1[os + i] = z2;
        }
        out1[2 * os + i] = z0;
      }
    }
    __syncthreads();
  }
}

// A polynomial's tail in one launch: the public weighted sum of the powers stack S
// ([3 parties][R rows][n], party stride ps, row stride rs, weights w[R] on the device), the
// TruncPr of that sum (as k_trunc_pr3_lat: same streams, same nonces) and the public
// constant c added to party 0's share (slot 0 of out0, slot 2 of out1) -- the values of
// weighted_sum + trunc_pr + add_public.
template <class T>
__global__ void __launch_bounds__(256) k_wsum_trunc3_lat(
    const T* __restrict__ S, int64_t ps, int64_t rs, int R, const T* __restrict__ w,
    T* __restrict__ out0, T* __restrict__ out1, int64_t n, int64_t os, T cadd, int m,
    mxd::KeySrc keys, uint64_t n_r0, uint64_t n_r1, uint64_t n_t, uint64_t n_m, uint64_t n_z0,
    uint64_t n_z2) {
  constexpr int EPB = 256 / 6;
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  __shared__ uint64_t kl[6][EPB], kh[6][EPB];
  mxd::stage_keys(rks, keys, 2);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / EPB, lb = tid % EPB;
  const int key_of = (s == 1 || s == 5) ? 1 : 0;
  const uint64_t nonce_of = s == 0 ? n_r0 : s == 1 ? n_r1 : s == 2 ? n_t : s == 3 ? n_m
                            : s == 4 ? n_z0 : n_z2;
  __shared__ T xs[3][EPB][P];
  for (int64_t b0 = (int64_t)blockIdx.x * EPB; b0 < nb; b0 += (int64_t)gridDim.x * EPB) {
    if (s < 6 && b0 + lb < nb) {
      uint64_t lo, hi;
      mxd::prf_chunk(rks[key_of], nonce_of, (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    // the weighted sums, one (party, chunk) per thread (3 x EPB of the 256), into LDS
    if (tid < 3 * EPB && b0 + (tid % EPB) < nb) {
      const int p = tid / EPB, c = tid % EPB;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = (b0 + c) * P + j;
        T acc = 0;
        if (i < n)
          for (int r = 0; r < R; ++r) acc += w[r] * S[p * ps + r * rs + i];
        xs[p][c][j] = acc;
      }
    }
    __syncthreads();
    if (tid < EPB && b0 + tid < nb) {
      const int64_t b = b0 + tid;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = b * P + j;
        if (i >= n) break;
        const T x[3] = {xs[0][tid][j], xs[1][tid][j], xs[2][tid][j]};
        const T z0 = mxd::pick<T>(kl[4][tid], kh[4][tid], j);
        const T z2 = mxd::pick<T>(kl[5][tid], kh[5][tid], j);
        const T z1 = mxf::trunc_pr_z1<T>(
            x[0], x[1], x[2], mxd::pick<T>(kl[0][tid], kh[0][tid], j),
            mxd::pick<T>(kl[1][tid], kh[1][tid], j), mxd::pick<T>(kl[2][tid], kh[2][tid], j),
            mxd::pick<T>(kl[3][tid], kh[3][tid], j), z0, z2, m);
        const T a0 = z0 + cadd;
        out0[i] = a0;
        out0[os + i] = z1;
        out0[2 * os + i] = z2;
        if (out1 != out0 + os) {
          out1[i] = z1;
          out1[os + i] = z2;
        }
        out1[2 * os + i] = a0;
      }
    }
    __syncthreads();
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_share3(int kind, const void* __restrict__ xv, T* __restrict__ out0,
                         T* __restrict__ out1, int64_t n, int j0, mxd::KeySrc keys, uint64_t n1,
                         uint64_t na) {
  const bool mir = kind & MX_SHARE_MIRROR;
  kind &= ~MX_SHARE_MIRROR;
  const T* x = (const T*)xv;
  const double* xf = (const double*)xv;  // kind MX_SHARE_F64: encode in the kernel
  const double scale = kind == MX_SHARE_F64 ? ldexp(1.0, (int)na) : 0.0;
  __shared__ uint32_t rks[1][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 1);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const uint32_t* const key[1] = {rks[0]};
  const uint64_t nonce[1] = {n1};
  mxd::walk_chunks<1>(nb, key, nonce, [&](int64_t b, const uint64_t (&lo)[1], const uint64_t (&hi)[1]) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t i = b * P + j;
      if (i >= n) break;
      const T r = mxd::pick<T>(lo[0], hi[0], j);
      const T xi = kind == MX_SHARE_F64 ? (T)mxr::f64_to_i128(xf[i] * scale) : x[i];
      const T v = kind == MX_CROSS_BOOL ? (T)(xi ^ r) : (T)(xi - r);
      T slot[3];
      slot[j0] = mir ? v : r;
      slot[(j0 + 1) % 3] = mir ? r : v;
      slot[(j0 + 2) % 3] = 0;
      const bool ring4 = out1 == out0 + n;  // 4-slot ring: out1's slots 0, 1 are out0's 1, 2
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        out0[p * n + i] = slot[p];
        if (!ring4 || p == 2) out1[p * n + i] = slot[(p + 1) % 3];
      }
    }
  });
}

// out0 / out1: party p's slot at out + p * os (os = n: dense stacks; larger: row views);
// cm: public premultiplier of the input shares (words little-endian; null = 1)
int launch_trunc_pr3(int words, const void* s0, void* out0, void* out1, int64_t n, int64_t os,
                     int m, const mxd::KeySrc& keys, const uint64_t* nn, void* stream,
                     const uint64_t* cm = nullptr) {
  const u64 c64 = cm ? cm[0] : 1;
  const u128 c128 = cm ? (((u128)cm[1] << 64) | cm[0]) : (u128)1;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int64_t nblk = words == 1 ? (n + 1) / 2 : n;
  if (nblk <= 8192 && (words == 1 || words == 2)) {  // latency-bound: one PRF per thread
    const unsigned g = (unsigned)((nblk + 41) / 42);
    if (words == 1)
      hipLaunchKernelGGL(k_trunc_pr3_lat<u64>, dim3(g), dim3(256), 0, st, (const u64*)s0,
                         (u64*)out0, (u64*)out1, n, os, c64, m, keys, nn[0], nn[1], nn[2], nn[3], nn[4],
                         nn[5]);
    else
      hipLaunchKernelGGL(k_trunc_pr3_lat<u128>, dim3(g), dim3(256), 0, st, (const u128*)s0,
                         (u128*)out0, (u128*)out1, n, os, c128, m, keys, nn[0], nn[1], nn[2], nn[3],
                         nn[4], nn[5]);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -100 - (int)e;
  }
  if (words == 1) {
    int64_t nb = (n + 1) / 2;
    hipLaunchKernelGGL(k_trunc_pr3<u64>, dim3(mxd::grid_for_chunks(nb)), dim3(256), 0, st,
                       (const u64*)s0, (u64*)out0, (u64*)out1, n, os, c64, m, keys, nn[0], nn[1], nn[2],
                       nn[3], nn[4], nn[5]);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_trunc_pr3<u128>, dim3(mxd::grid_for_chunks(n)), dim3(256), 0, st,
                       (const u128*)s0, (u128*)out0, (u128*)out1, n, os, c128, m, keys, nn[0], nn[1], nn[2],
                       nn[3], nn[4], nn[5]);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int launch_share3(int kind, int words, const void* x, void* out0, void* out1, int64_t n, int j,
                  const mxd::KeySrc& keys, uint64_t n1, uint64_t na, void* stream) {
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (words) {
    case 0:
      hipLaunchKernelGGL(k_share3<uint8_t>, dim3(mxd::grid_for_chunks((n + 15) / 16)), dim3(256), 0, st,
                         kind, x, (uint8_t*)out0, (uint8_t*)out1, n, j, keys, n1,
                         na);
      break;
    case 1:
      hipLaunchKernelGGL(k_share3<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2)), dim3(256), 0, st, kind,
                         x, (u64*)out0, (u64*)out1, n, j, keys, n1, na);
      break;
    case 2:
      hipLaunchKernelGGL(k_share3<u128>, dim3(mxd::grid_for_chunks(n)), dim3(256), 0, st, kind,
                         x, (u128*)out0, (u128*)out1, n, j, keys, n1, na);
      break;
    default:
      return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

}  // namespace

extern "C" {

// k_wsum_trunc3_lat (latency-bound sizes only; -1 otherwise).  Strides in elements; cadd
// little-endian words.
int mxh_wsum_trunc3(int words, const void* S, int64_t ps, int64_t rs, int R,
                               const void* w, void* out0, void* out1, int64_t n, int m,
                               const uint32_t* k0, const uint32_t* k2, const uint64_t* nn,
                               const uint64_t* cadd, void* stream) {
  const int64_t nblk = words == 1 ? (n + 1) / 2 : n;
  if (n <= 0 || R < 1 || nblk > 8192 || (words != 1 && words != 2)) return -1;
  const uint32_t* ptrs[2] = {k0, k2};
  const mxd::KeySrc keys = mxd::keysrc_slots(ptrs, 2);
  const unsigned g = (unsigned)((nblk + 41) / 42);
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    hipLaunchKernelGGL(k_wsum_trunc3_lat<u64>, dim3(g), dim3(256), 0, st, (const u64*)S, ps, rs,
                       R, (const u64*)w, (u64*)out0, (u64*)out1, n, n, (u64)cadd[0], m, keys,
                       nn[0], nn[1], nn[2], nn[3], nn[4], nn[5]);
  else
    hipLaunchKernelGGL(k_wsum_trunc3_lat<u128>, dim3(g), dim3(256), 0, st, (const u128*)S, ps,
                       rs, R, (const u128*)w, (u128*)out0, (u128*)out1, n, n,
                       (((u128)cadd[1]) << 64) | cadd[0], m, keys, nn[0], nn[1], nn[2], nn[3],
                       nn[4], nn[5]);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}


int mxh_trunc_pr3(int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                  const uint8_t* k0, const uint8_t* k2, const uint64_t* nn, void* stream) {
  uint8_t kk[32];
  memcpy(kk, k0, 16);
  memcpy(kk + 16, k2, 16);
  return launch_trunc_pr3(words, s0, out0, out1, n, n, m, mxd::keysrc_host(kk, 2), nn, stream);
}

int mxh_trunc_pr3_k(int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                    const uint32_t* slot_k0, const uint32_t* slot_k2, const uint64_t* nn,
                    void* stream) {
  const uint32_t* ptrs[2] = {slot_k0, slot_k2};
  return launch_trunc_pr3(words, s0, out0, out1, n, n, m, mxd::keysrc_slots(ptrs, 2), nn, stream);
}

int mxh_trunc_pr3_ko(int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                     const uint32_t* slot_k0, const uint32_t* slot_k2, const uint64_t* nn,
                     int64_t ostride, void* stream) {
  const uint32_t* ptrs[2] = {slot_k0, slot_k2};
  return launch_trunc_pr3(words, s0, out0, out1, n, ostride, m, mxd::keysrc_slots(ptrs, 2), nn,
                          stream);
}

int mxh_trunc_pr3_kmo(int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                      const uint32_t* slot_k0, const uint32_t* slot_k2, const uint64_t* nn,
                      int64_t ostride, const uint64_t* cm, void* stream) {
  const uint32_t* ptrs[2] = {slot_k0, slot_k2};
  return launch_trunc_pr3(words, s0, out0, out1, n, ostride, m, mxd::keysrc_slots(ptrs, 2), nn,
                          stream, cm);
}

int mxh_share3(int kind, int words, const void* x, void* out0, void* out1, int64_t n, int j,
               const uint8_t* k_next, const uint8_t* k_all, uint64_t n1, uint64_t na,
               void* stream) {
  uint8_t kk[32];
  memcpy(kk, k_next, 16);
  memcpy(kk + 16, k_all, 16);
  return launch_share3(kind, words, x, out0, out1, n, j, mxd::keysrc_host(kk, 2), n1, na,
                       stream);
}

int mxh_share3_k(int kind, int words, const void* x, void* out0, void* out1, int64_t n, int j,
                 const uint32_t* slot_next, const uint32_t* slot_all, uint64_t n1, uint64_t na,
                 void* stream) {
  const uint32_t* ptrs[2] = {slot_next, slot_all};
  return launch_share3(kind, words, x, out0, out1, n, j, mxd::keysrc_slots(ptrs, 2), n1, na,
                       stream);
}

}  // extern "C"
