// Per-party fused local step over both share components (one party per GPU / process /
// thread): the weighted sums of stacked rows that a per-party protocol forms between its
// rounds (a fraction from bit planes, a polynomial's sum of powers), with the public terms
// added on the slots this party holds of x_0, in ONE pass instead of weighted_sum +
// multiply + add + lincomb launches:
//
//   s_c[i]          = sum_k w_k rows_c[k * rs + i] + wx x_c[i]             (c = 0, 1)
//   out_c[b L + i]  = s_c[i] + (pub_c ? cb[b] : 0)                         (b < nblk)
//   out2_c[i]       = m2 s_c[i] + (pub_c ? c2 : 0)                         (optional)
//
// pub_c: component c of this party is a copy of x_0 (P0's s0, P2's s1), where a public
// constant is added.  All arithmetic is in the ring (wrapping), so the result is bitwise
// the composition of the separate steps.
#pragma once
#include <stdint.h>

#include "ring_common.h"

namespace mxw {

constexpr int kMaxRows = 64;
constexpr int kMaxBlk = 3;

template <class T>
struct WsumArgs {
  int nrows, nblk, has2, pub0, pub1;
  int64_t L, rs;
  T w[kMaxRows];
  T wx, m2, c2;
  T cb[kMaxBlk];
};

template <class T>
MX_HD inline T wsum_at(const WsumArgs<T>& a, const T* rows, const T* x, int64_t i) {
  T s = (T)0;
  for (int k = 0; k < a.nrows; ++k) s += a.w[k] * rows[(int64_t)k * a.rs + i];
  if (x != nullptr) s += a.wx * x[i];
  return s;
}

}  // namespace mxw
