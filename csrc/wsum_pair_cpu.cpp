// Host side and C ABI of the per-party fused weighted sums (wsum_pair.h).
#include <cstring>

#include "moosex.h"
#include "wsum_pair.h"

extern "C" int mxh_wsum_pair(int words, const void* args, const void* r0, const void* r1,
                             const void* x0, const void* x1, void* o0, void* o1, void* q0,
                             void* q1, void* stream);

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;

template <class T>
void fill_args(mxw::WsumArgs<T>& a, int nrows, int nblk, int has2, int pub0, int pub1,
               int64_t L, int64_t rs, const int64_t* w, const int64_t* wx, const int64_t* m2,
               const int64_t* c2, const int64_t* cb) {
  constexpr int W = sizeof(T) / 8;
  std::memset(&a, 0, sizeof a);
  a.nrows = nrows;
  a.nblk = nblk;
  a.has2 = has2;
  a.pub0 = pub0;
  a.pub1 = pub1;
  a.L = L;
  a.rs = rs;
  auto rd = [](const int64_t* p) {  // W little-endian 64-bit words -> T
    T v = 0;
    for (int j = W - 1; j >= 0; --j) v = (T)((v << 32) << 32) | (T)(uint64_t)p[j];
    return v;
  };
  for (int k = 0; k < nrows; ++k) a.w[k] = rd(w + W * k);
  a.wx = rd(wx);
  a.m2 = rd(m2);
  a.c2 = rd(c2);
  for (int b = 0; b < nblk; ++b) a.cb[b] = rd(cb + W * b);
}

template <class T>
void run_host(const mxw::WsumArgs<T>& a, const T* r0, const T* r1, const T* x0, const T* x1,
              T* o0, T* o1, T* q0, T* q1) {
  for (int c = 0; c < 2; ++c) {
    const T* r = c ? r1 : r0;
    const T* x = c ? x1 : x0;
    T* o = c ? o1 : o0;
    T* q = c ? q1 : q0;
    const bool pub = c ? a.pub1 : a.pub0;
    for (int64_t i = 0; i < a.L; ++i) {
      const T s = mxw::wsum_at<T>(a, r, x, i);
      for (int b = 0; b < a.nblk; ++b) o[(int64_t)b * a.L + i] = s + (pub ? a.cb[b] : (T)0);
      if (a.has2) q[i] = a.m2 * s + (pub ? a.c2 : (T)0);
    }
  }
}

}  // namespace

extern "C" int mx_wsum_pair(int dev, int words, int nrows, int nblk, int has2, int pub0,
                            int pub1, int64_t L, int64_t rs, const int64_t* w,
                            const int64_t* wx, const int64_t* m2, const int64_t* c2,
                            const int64_t* cb, const void* r0, const void* r1, const void* x0,
                            const void* x1, void* o0, void* o1, void* q0, void* q1,
                            void* stream) {
  if (nrows < 0 || nrows > mxw::kMaxRows || nblk < 1 || nblk > mxw::kMaxBlk || L < 0 ||
      (nrows > 0 && (r0 == nullptr || r1 == nullptr)) || (has2 && (!q0 || !q1)))
    return -3;
  if (L == 0) return 0;
  if (words == 1) {
    mxw::WsumArgs<u64> a;
    fill_args(a, nrows, nblk, has2, pub0, pub1, L, rs, w, wx, m2, c2, cb);
    if (dev) return mxh_wsum_pair(1, &a, r0, r1, x0, x1, o0, o1, q0, q1, stream);
    run_host(a, (const u64*)r0, (const u64*)r1, (const u64*)x0, (const u64*)x1, (u64*)o0,
             (u64*)o1, (u64*)q0, (u64*)q1);
    return 0;
  }
  if (words == 2) {
    mxw::WsumArgs<u128> a;
    fill_args(a, nrows, nblk, has2, pub0, pub1, L, rs, w, wx, m2, c2, cb);
    if (dev) return mxh_wsum_pair(2, &a, r0, r1, x0, x1, o0, o1, q0, q1, stream);
    run_host(a, (const u128*)r0, (const u128*)r1, (const u128*)x0, (const u128*)x1,
             (u128*)o0, (u128*)o1, (u128*)q0, (u128*)q1);
    return 0;
  }
  return -2;
}
