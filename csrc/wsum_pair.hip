// Device side of the per-party fused weighted sums (wsum_pair.h).
#include <hip/hip_runtime.h>

#include "moosex.h"
#include "prf_dev.h"
#include "wsum_pair.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

namespace {

template <class T>
__global__ void __launch_bounds__(256)
    k_wsum_pair(mxw::WsumArgs<T> a, const T* __restrict__ r0, const T* __restrict__ r1,
                const T* __restrict__ x0, const T* __restrict__ x1, T* __restrict__ o0,
                T* __restrict__ o1, T* __restrict__ q0, T* __restrict__ q1) {
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

}  // namespace

extern "C" int mxh_wsum_pair(int words, const void* args, const void* r0, const void* r1,
                             const void* x0, const void* x1, void* o0, void* o1, void* q0,
                             void* q1, void* stream) {
  hipStream_t st = (hipStream_t)stream;
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
