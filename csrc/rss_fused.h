// Fused single-pass kernels for a stacked 3-party session (all parties on one device).
//
// They compute exactly the same shares as the generic protocol code in
// moose_amd/protocols/replicated.py (same PRF keys, nonces and element->keystream
// mapping), but do every party's local work of a whole protocol in ONE pass over
// memory: TruncPr (dealer masks, masked openings, additive->replicated) and Share.
#pragma once
#include <stdint.h>

#include "aes_core.h"
#include "ring_common.h"

namespace mxf {

template <class T>
MX_HD inline T shl(T x, int k) {
  constexpr int W = 8 * sizeof(T);
  return k >= W ? (T)0 : (T)(x << k);
}
template <class T>
MX_HD inline T shr(T x, int k) {
  constexpr int W = 8 * sizeof(T);
  return k >= W ? (T)0 : (T)(x >> k);
}

// inputs: slots x0, x1, x2 and the six PRF values (dealer key k0: r0, rt0, rm0, z0;
// dealer key k2: r1, z2).  Returns the new slots z0, z1, z2 (z0, z2 are the PRF values).
template <class T>
MX_HD inline T trunc_pr_z1(T x0, T x1, T x2, T r0, T r1, T rt0, T rm0, T z0, T z2, int m) {
  constexpr int W = 8 * sizeof(T);
  const int k = W - 1;
  T r = r0 + r1;
  T r_msb = shr<T>(r, W - 1);
  T r_top = shr<T>(shl<T>(r, 1), m + 1);
  T rt1 = r_top - rt0;
  T rm1 = r_msb - rm0;
  T mk0 = x0 + x1 + shl<T>((T)1, k - 1) + r0;
  T mk1 = x2 + r1;
  T c = mk0 + mk1;
  T c_msb = shr<T>(c, W - 1);
  T c_top = shr<T>(shl<T>(c, 1), m + 1);
  T ov0 = rm0 - shl<T>(c_msb * rm0, 1) + c_msb;
  T y0 = shl<T>(ov0, k - m) - rt0 + c_top - shl<T>((T)1, k - 1 - m);
  T ov1 = rm1 - shl<T>(c_msb * rm1, 1);
  T y1 = shl<T>(ov1, k - m) - rt1;
  return (y0 - z0) + (y1 - z2);
}

}  // namespace mxf

// ---------------------------------------------------------------------------------------
// Per-party TruncPr rounds (one party per stacked component, parties on different GPUs;
// see rss_party.hip).  Same arithmetic as trunc_pr_z1, split at the two message rounds.
// The dealer's msb-mask share only matters modulo 2^(m+1) (it is shifted left by k - m),
// so it travels as a u64 (m <= 63).
// ---------------------------------------------------------------------------------------
namespace mxf {

// dealer P2: r = r0 + r1 -> (rt1, rm1) for P1
template <class T>
MX_HD inline void trunc_dealer(T r0, T r1, T rt0, T rm0, int m, T* rt1, uint64_t* rm1) {
  constexpr int W = 8 * sizeof(T);
  const T r = r0 + r1;
  *rt1 = shr<T>(shl<T>(r, 1), m + 1) - rt0;
  *rm1 = (uint64_t)(shr<T>(r, W - 1) - rm0);
}

// P0's masked opening share: x0 + x1 + 2^(k-1) + r0
template <class T>
MX_HD inline T trunc_mask0(T x0, T x1, T r0) {
  constexpr int W = 8 * sizeof(T);
  return x0 + x1 + shl<T>((T)1, W - 2) + r0;
}

// P0's (first) / P1's truncated additive share from the opened c
template <class T>
MX_HD inline T trunc_y(T c, T rt, T rm, int m, bool first) {
  constexpr int W = 8 * sizeof(T);
  const int k = W - 1;
  const T c_msb = shr<T>(c, W - 1);
  T ov = rm - shl<T>(c_msb * rm, 1);
  if (!first) return shl<T>(ov, k - m) - rt;
  ov = ov + c_msb;
  const T c_top = shr<T>(shl<T>(c, 1), m + 1);
  return shl<T>(ov, k - m) - rt + c_top - shl<T>((T)1, k - 1 - m);
}

}  // namespace mxf
