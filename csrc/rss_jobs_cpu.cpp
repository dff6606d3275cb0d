// Host versions of the per-party job tail (rss_jobs.hip) and the C ABI entry points that
// dispatch host / device.  Same PRF streams and element order as the device kernels.
#include <algorithm>
#include <climits>
#include <functional>
#include <vector>

#include "moosex.h"
#include "ring_common.h"
#include "rss_fused.h"

void mx_cpu_prf_range(const uint8_t* key, uint64_t nonce, int words, int64_t i0, int64_t n,
                      void* out);
void mx_cpu_parallel_for(int64_t n, int64_t grain,
                         const std::function<void(int64_t, int64_t)>& f);

extern "C" {
int mxh_jobs_r0(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                int m, int role, int main, int dealer, void* msg, void* msg_rt, void* msg_rm,
                const uint32_t* const* slots, const uint64_t* nn, void* stream);
int mxh_jobs_r0p(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                 int m, int role, int main, int dealer, void* msg, void* msg_rt, void* msg_rm,
                 const uint32_t* const* slots, const uint64_t* nn, int npend,
                 const void* const* pend, const int64_t* pend_len, void* stream);
int mxh_jobs_r1(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                int m, int role, const void* msg, const void* rmk, const void* rz,
                const void* rrt, const void* rrm, void* w, const uint32_t* const* slots,
                const uint64_t* nn, void* stream);
int mxh_jobs_r2(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                int role, const void* a, const void* b, void* stream);
}

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;

struct Job {
  const void* p[8];  // x0 x1 y0 y1 a a2 o0 o1
  int64_t rows, sx, sy, sa, sa2, ca, ca2, cb, start;
};

int make(int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
         std::vector<Job>* js, int64_t* n) {
  if (njobs < 1 || njobs > MX_MAX_JOBS || L < 1) return -3;
  int64_t at = 0;
  for (int q = 0; q < njobs; ++q) {
    Job J;
    for (int k = 0; k < 8; ++k) J.p[k] = ptrs[8 * q + k];
    const int64_t* dq = dims + 8 * q;
    J.rows = dq[0];
    J.sx = dq[1];
    J.sy = dq[2];
    J.sa = dq[3];
    J.sa2 = dq[4];
    J.ca = dq[5];
    J.ca2 = dq[6];
    J.cb = dq[7];
    J.start = at;
    at += J.rows * L;
    js->push_back(J);
  }
  *n = at;
  return 0;
}

struct Loc {
  int q;
  int64_t r, e;
};

// pending round-2 sums of the previous level (rss_jobs.hip Pend): o[k][i] = a[k][i] + b[k][i]
struct Pending {
  int n = 0;
  const void* o[MX_MAX_JOBS];
  const void* a[MX_MAX_JOBS];
  const void* b[MX_MAX_JOBS];
  int64_t len[MX_MAX_JOBS];
};

template <class T>
T ld(const Pending& pd, const void* p, int64_t idx) {
  const T* q = (const T*)p + idx;
  for (int k = 0; k < pd.n; ++k) {
    const T* o = (const T*)pd.o[k];
    if (q >= o && q < o + pd.len[k]) {
      const int64_t off = q - o;
      return ((const T*)pd.a[k])[off] + ((const T*)pd.b[k])[off];
    }
  }
  return *q;
}

Loc locate(const std::vector<Job>& js, int64_t L, int64_t i) {
  int q = (int)js.size() - 1;
  while (q > 0 && i < js[q].start) --q;
  const int64_t k = i - js[q].start;
  return {q, k / L, k % L};
}

template <class T>
T value(const std::vector<Job>& js, const Loc& l, const Pending& pd) {
  const Job& J = js[l.q];
  T v = 0;
  if (J.cb != 0) {
    const int64_t ix = l.r * J.sx + l.e, iy = l.r * J.sy + l.e;
    const T x0 = ld<T>(pd, J.p[0], ix), x1 = ld<T>(pd, J.p[1], ix);
    const T y0 = ld<T>(pd, J.p[2], iy), y1 = ld<T>(pd, J.p[3], iy);
    v = (T)J.cb * (x0 * y0 + x0 * y1 + x1 * y0);
  }
  if (J.p[4] != nullptr) v += (T)J.ca * ld<T>(pd, J.p[4], l.r * J.sa + l.e);
  if (J.p[5] != nullptr) v += (T)J.ca2 * ld<T>(pd, J.p[5], l.r * J.sa2 + l.e);
  return v;
}

template <class T>
T* out(const std::vector<Job>& js, int64_t L, const Loc& l, int which) {
  return (T*)js[l.q].p[6 + which] + l.r * L + l.e;
}

template <class F>
void for_chunks(int64_t n, F&& f) {
  mx_cpu_parallel_for(n, 1 << 12, [&](int64_t s, int64_t e) {
    const int64_t CH = 512;
    for (int64_t c = s; c < e; c += CH) f(c, std::min(CH, e - c));
  });
}

template <class T>
void prf(const uint32_t* slot, uint64_t nonce, int64_t i0, int64_t len, T* o) {
  mx_cpu_prf_range((const uint8_t*)slot, nonce, (int)(sizeof(T) / 8), i0, len, o);
}

template <class T>
int r0(const std::vector<Job>& js, int64_t L, int64_t n, int m, int role, int main, int dealer,
       T* msg, T* msg_rt, u64* msg_rm, const uint32_t* const* slots, const uint64_t* nn,
       const Pending& pd) {
  const uint32_t* own = slots[0];
  const uint32_t* nxt = slots[1];
  for_chunks(n, [&](int64_t i0, int64_t len) {
    if (main) {
      std::vector<T> a(len, (T)0), b(len, (T)0), r(len);
      if (role != 1) prf<T>(own, nn[0], i0, len, a.data());
      if (role != 0) prf<T>(nxt, nn[0], i0, len, b.data());
      if (role == 0) prf<T>(own, nn[1], i0, len, r.data());
      if (role == 1) prf<T>(nxt, nn[2], i0, len, r.data());
      for (int64_t q = 0; q < len; ++q) {
        const int64_t i = i0 + q;
        const T z = value<T>(js, locate(js, L, i), pd) + a[q] - b[q];
        msg[i] = role == 0 ? mxf::trunc_mask0<T>(z, (T)0, r[q]) : role == 1 ? (T)(z + r[q]) : z;
      }
    }
    if (role == 2 && dealer) {
      std::vector<T> v0(len), v1(len), t(len), mm(len), z0(len), z2(len);
      prf<T>(nxt, nn[1], i0, len, v0.data());
      prf<T>(own, nn[2], i0, len, v1.data());
      prf<T>(nxt, nn[3], i0, len, t.data());
      prf<T>(nxt, nn[4], i0, len, mm.data());
      prf<T>(nxt, nn[5], i0, len, z0.data());
      prf<T>(own, nn[6], i0, len, z2.data());
      for (int64_t q = 0; q < len; ++q) {
        const int64_t i = i0 + q;
        mxf::trunc_dealer<T>(v0[q], v1[q], t[q], mm[q], m, &msg_rt[i], &msg_rm[i]);
        const Loc l = locate(js, L, i);
        *out<T>(js, L, l, 0) = z2[q];
        *out<T>(js, L, l, 1) = z0[q];
      }
    }
  });
  // the pending sums, materialised after every read above went through ld()
  for (int k = 0; k < pd.n; ++k)
    for (int64_t i = 0; i < pd.len[k]; ++i)
      ((T*)pd.o[k])[i] = ((const T*)pd.a[k])[i] + ((const T*)pd.b[k])[i];
  return 0;
}

template <class T>
int r1(const std::vector<Job>& js, int64_t L, int64_t n, int m, int role, const T* mine,
       const T* other, const T* z2m, const T* rt, const u64* rm, T* wo,
       const uint32_t* const* slots, const uint64_t* nn) {
  if (role != 0 && role != 1) return 0;
  for_chunks(n, [&](int64_t i0, int64_t len) {
    std::vector<T> t(len), mm(len), z(len);
    if (role == 0) {
      prf<T>(slots[0], nn[3], i0, len, t.data());
      prf<T>(slots[0], nn[4], i0, len, mm.data());
      prf<T>(slots[0], nn[5], i0, len, z.data());
    } else {
      prf<T>(slots[1], nn[6], i0, len, z.data());
    }
    for (int64_t q = 0; q < len; ++q) {
      const int64_t i = i0 + q;
      T cc = mine[i] + other[i];
      if (z2m) cc += z2m[i];
      const T y = role == 0 ? mxf::trunc_y<T>(cc, t[q], mm[q], m, true)
                            : mxf::trunc_y<T>(cc, rt[i], (T)rm[i], m, false);
      wo[i] = y - z[q];
      *out<T>(js, L, locate(js, L, i), role == 0 ? 0 : 1) = z[q];
    }
  });
  return 0;
}

template <class T>
int r2(const std::vector<Job>& js, int64_t L, int64_t n, int role, const T* a, const T* b) {
  if (role != 0 && role != 1) return 0;
  for (int64_t i = 0; i < n; ++i) *out<T>(js, L, locate(js, L, i), role == 0 ? 1 : 0) = a[i] + b[i];
  return 0;
}

}  // namespace

extern "C" {

int mx_jobs_r0p(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
                int64_t L, int m, int role, int main, int dealer, void* msg, void* msg_rt,
                void* msg_rm, const uint32_t* const* slots, const uint64_t* nn, int npend,
                const void* const* pend, const int64_t* pend_len, void* stream) {
  if (m < 1 || m > 63 || role < 0 || role > 2) return -3;
  if (npend < 0 || npend > MX_MAX_JOBS) return -3;
  if (dev)
    return mxh_jobs_r0p(words, njobs, ptrs, dims, L, m, role, main, dealer, msg, msg_rt, msg_rm,
                        slots, nn, npend, pend, pend_len, stream);
  std::vector<Job> js;
  int64_t n = 0;
  int rc = make(njobs, ptrs, dims, L, &js, &n);
  if (rc) return rc;
  Pending pd;
  pd.n = npend;
  for (int k = 0; k < npend; ++k) {
    pd.o[k] = pend[3 * k];
    pd.a[k] = pend[3 * k + 1];
    pd.b[k] = pend[3 * k + 2];
    pd.len[k] = pend_len[k];
  }
  if (words == 1)
    return r0<u64>(js, L, n, m, role, main, dealer, (u64*)msg, (u64*)msg_rt, (u64*)msg_rm, slots,
                   nn, pd);
  if (words == 2)
    return r0<u128>(js, L, n, m, role, main, dealer, (u128*)msg, (u128*)msg_rt, (u64*)msg_rm,
                    slots, nn, pd);
  return -2;
}

int mx_jobs_r0(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
               int64_t L, int m, int role, int main, int dealer, void* msg, void* msg_rt,
               void* msg_rm, const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  return mx_jobs_r0p(dev, words, njobs, ptrs, dims, L, m, role, main, dealer, msg, msg_rt,
                     msg_rm, slots, nn, 0, nullptr, nullptr, stream);
}

int mx_jobs_r1(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
               int64_t L, int m, int role, const void* msg, const void* rmk, const void* rz,
               const void* rrt, const void* rrm, void* w, const uint32_t* const* slots,
               const uint64_t* nn, void* stream) {
  if (m < 1 || m > 63 || role < 0 || role > 2) return -3;
  if (dev)
    return mxh_jobs_r1(words, njobs, ptrs, dims, L, m, role, msg, rmk, rz, rrt, rrm, w, slots,
                       nn, stream);
  std::vector<Job> js;
  int64_t n = 0;
  int rc = make(njobs, ptrs, dims, L, &js, &n);
  if (rc) return rc;
  if (words == 1)
    return r1<u64>(js, L, n, m, role, (const u64*)msg, (const u64*)rmk, (const u64*)rz,
                   (const u64*)rrt, (const u64*)rrm, (u64*)w, slots, nn);
  if (words == 2)
    return r1<u128>(js, L, n, m, role, (const u128*)msg, (const u128*)rmk, (const u128*)rz,
                    (const u128*)rrt, (const u64*)rrm, (u128*)w, slots, nn);
  return -2;
}

int mx_jobs_r2(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
               int64_t L, int role, const void* a, const void* b, void* stream) {
  if (role < 0 || role > 2) return -3;
  if (dev) return mxh_jobs_r2(words, njobs, ptrs, dims, L, role, a, b, stream);
  std::vector<Job> js;
  int64_t n = 0;
  int rc = make(njobs, ptrs, dims, L, &js, &n);
  if (rc) return rc;
  if (words == 1) return r2<u64>(js, L, n, role, (const u64*)a, (const u64*)b);
  if (words == 2) return r2<u128>(js, L, n, role, (const u128*)a, (const u128*)b);
  return -2;
}

}  // extern "C"
