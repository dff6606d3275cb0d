// Device side of the per-party fused weighted sums (wsum_pair.h).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "moosex.h"
#include "party_batch.h"
#include "prf_dev.h"
#include "wsum_pair.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

namespace {

template <class T>
__device__ __forceinline__ void d_wsum_pair(const mxw::WsumArgs<T>& a, const T* __restrict__ r0,
                                            const T* __restrict__ r1, const T* __restrict__ x0,
                                            const T* __restrict__ x1, T* __restrict__ o0,
                                            T* __restrict__ o1, T* __restrict__ q0,
                                            T* __restrict__ q1) {
  const int64_t n = 2 * a.L;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int c = g >= a.L;
    const int64_t i = g - (c ? a.L : 0);
    const T s = mxw::wsum_at<T>(a, c ? r1 : r0, c ? x1 : x0, i);
    const bool pub = c ? a.pub1 : a.pub0;
    T* o = c ? o1 : o0;
    for (int b = 0; b < a.nblk; ++b) o[(int64_t)b * a.L + i] = s + (pub ? a.cb[b] : (T)0);
    if (a.has2) (c ? q1 : q0)[i] = a.m2 * s + (pub ? a.c2 : (T)0);
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_wsum_pair(mxw::WsumArgs<T> a, const T* __restrict__ r0,
                                                   const T* __restrict__ r1,
                                                   const T* __restrict__ x0,
                                                   const T* __restrict__ x1, T* __restrict__ o0,
                                                   T* __restrict__ o1, T* __restrict__ q0,
                                                   T* __restrict__ q1) {
  d_wsum_pair<T>(a, r0, r1, x0, x1, o0, o1, q0, q1);
}

// Group form: kGroup lanes per output element, lane j summing rows j, j + kGroup, ... (a
// dependent chain of nrows / kGroup loads instead of nrows), then a butterfly over the
// group's lanes (whole ring elements: carries included) and lane 0 writes.  Same ring
// sums in another association order -- addition mod 2^w is associative, so bitwise equal.
constexpr int kGroup = 8;

template <class T>
__device__ __forceinline__ T shfl_xor_ring(T v, int m) {
  constexpr int W = (int)(sizeof(T) / 4);
  uint32_t w[W];
#pragma unroll
  for (int q = 0; q < W; ++q) w[q] = (uint32_t)(v >> (32 * q));
#pragma unroll
  for (int q = 0; q < W; ++q) w[q] = (uint32_t)__shfl_xor((int)w[q], m, kGroup);
  T r = 0;
#pragma unroll
  for (int q = 0; q < W; ++q) r |= (T)w[q] << (32 * q);
  return r;
}

template <class T>
__device__ __forceinline__ void d_wsum_pair_g(const mxw::WsumArgs<T>& a, const T* __restrict__ r0,
                                              const T* __restrict__ r1, const T* __restrict__ x0,
                                              const T* __restrict__ x1, T* __restrict__ o0,
                                              T* __restrict__ o1, T* __restrict__ q0,
                                              T* __restrict__ q1) {
  // the grid covers every element once (kGroup lanes each): no stride loop, so all lanes
  // of a group reach the butterfly
  const int64_t n = 2 * a.L;
  const int lane = threadIdx.x % kGroup;
  const int64_t gb = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kGroup;
  const bool live = gb < n;
  const int c = live && gb >= a.L;
  const int64_t i = live ? gb - (c ? a.L : 0) : 0;
  const T* rows = c ? r1 : r0;
  T s = (T)0;
  if (live) {
    for (int k = lane; k < a.nrows; k += kGroup) s += a.w[k] * rows[(int64_t)k * a.rs + i];
    const T* x = c ? x1 : x0;
    if (lane == 0 && x != nullptr) s += a.wx * x[i];
  }
#pragma unroll
  for (int m = kGroup / 2; m >= 1; m >>= 1) s += shfl_xor_ring<T>(s, m);
  if (live && lane == 0) {
    const bool pub = c ? a.pub1 : a.pub0;
    T* o = c ? o1 : o0;
    for (int b = 0; b < a.nblk; ++b) o[(int64_t)b * a.L + i] = s + (pub ? a.cb[b] : (T)0);
    if (a.has2) (c ? q1 : q0)[i] = a.m2 * s + (pub ? a.c2 : (T)0);
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_wsum_pair_g(mxw::WsumArgs<T> a, const T* __restrict__ r0,
                                                     const T* __restrict__ r1,
                                                     const T* __restrict__ x0,
                                                     const T* __restrict__ x1, T* __restrict__ o0,
                                                     T* __restrict__ o1, T* __restrict__ q0,
                                                     T* __restrict__ q1) {
  d_wsum_pair_g<T>(a, r0, r1, x0, x1, o0, o1, q0, q1);
}

// party-batched twins for the composed one-GPU replay (party_batch.h)
MX_X3(k_wsum_pair<u64>, d_wsum_pair<u64>);
MX_X3(k_wsum_pair<u128>, d_wsum_pair<u128>);
MX_X3(k_wsum_pair_g<u64>, d_wsum_pair_g<u64>);
MX_X3(k_wsum_pair_g<u128>, d_wsum_pair_g<u128>);

}  // namespace

extern "C" int mxh_wsum_pair(int words, const void* args, const void* r0, const void* r1,
                             const void* x0, const void* x1, void* o0, void* o1, void* q0,
                             void* q1, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  // many rows over few elements (the per-party sums: 8-64 rows of a few hundred elements):
  // the group form; else one thread per element
  const int nrows = words == 1 ? ((const mxw::WsumArgs<u64>*)args)->nrows
                               : ((const mxw::WsumArgs<u128>*)args)->nrows;
  const int64_t L = words == 1 ? ((const mxw::WsumArgs<u64>*)args)->L
                               : ((const mxw::WsumArgs<u128>*)args)->L;
  static const bool group_on = [] {
    const char* e = std::getenv("MOOSEX_WSUM_GROUP");
    return !(e && e[0] == '0');
  }();
  if (group_on && nrows >= 2 * kGroup && 2 * L * kGroup <= (int64_t)1 << 22) {
    const unsigned grid = (unsigned)((2 * L * kGroup + 255) / 256);
    if (words == 1)
      hipLaunchKernelGGL(k_wsum_pair_g<u64>, dim3(grid), dim3(256), 0, st,
                         *(const mxw::WsumArgs<u64>*)args, (const u64*)r0, (const u64*)r1,
                         (const u64*)x0, (const u64*)x1, (u64*)o0, (u64*)o1, (u64*)q0, (u64*)q1);
    else
      hipLaunchKernelGGL(k_wsum_pair_g<u128>, dim3(grid), dim3(256), 0, st,
                         *(const mxw::WsumArgs<u128>*)args, (const u128*)r0, (const u128*)r1,
                         (const u128*)x0, (const u128*)x1, (u128*)o0, (u128*)o1, (u128*)q0,
                         (u128*)q1);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -100 - (int)e;
  }
  if (words == 1) {
    const auto& a = *(const mxw::WsumArgs<u64>*)args;
    hipLaunchKernelGGL(k_wsum_pair<u64>, dim3(mxd::grid_for(2 * a.L)), dim3(256), 0, st, a,
                       (const u64*)r0, (const u64*)r1, (const u64*)x0, (const u64*)x1,
                       (u64*)o0, (u64*)o1, (u64*)q0, (u64*)q1);
  } else if (words == 2) {
    const auto& a = *(const mxw::WsumArgs<u128>*)args;
    hipLaunchKernelGGL(k_wsum_pair<u128>, dim3(mxd::grid_for(2 * a.L)), dim3(256), 0, st, a,
                       (const u128*)r0, (const u128*)r1, (const u128*)x0, (const u128*)x1,
                       (u128*)o0, (u128*)o1, (u128*)q0, (u128*)q1);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}
