// Host versions of the fused stacked-session kernels (see rss_fused.h) and the C ABI
// entry points that dispatch host / device.
#include <cmath>
#include <cstring>
#include <functional>
#include <vector>

#include "moosex.h"
#include "ring_common.h"
#include "rss_fused.h"

void mx_cpu_prf_range(const uint8_t* key, uint64_t nonce, int words, int64_t i0, int64_t n,
                      void* out);
void mx_cpu_parallel_for(int64_t n, int64_t grain,
                         const std::function<void(int64_t, int64_t)>& f);

extern "C" int mxh_trunc_pr3(int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                             const uint8_t* k0, const uint8_t* k2, const uint64_t* nonces,
                             void* stream);
extern "C" int mxh_share3(int kind, int words, const void* x, void* out0, void* out1, int64_t n,
                          int j, const uint8_t* k_next, const uint8_t* k_all, uint64_t n1,
                          uint64_t na, void* stream);
extern "C" int mxh_trunc_pr3_k(int words, const void* s0, void* out0, void* out1, int64_t n,
                               int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                               const uint64_t* nonces, void* stream);
extern "C" int mxh_trunc_pr3_kmo(int words, const void* s0, void* out0, void* out1, int64_t n,
                                 int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                                 const uint64_t* nonces, int64_t ostride, const uint64_t* cm,
                                 void* stream);
extern "C" int mxh_trunc_pr3_ko(int words, const void* s0, void* out0, void* out1, int64_t n,
                                int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                                const uint64_t* nonces, int64_t ostride, void* stream);
extern "C" int mxh_share3_k(int kind, int words, const void* x, void* out0, void* out1,
                            int64_t n, int j, const uint32_t* slot_next,
                            const uint32_t* slot_all, uint64_t n1, uint64_t na, void* stream);

namespace {

template <class T>
int trunc3_host(const T* s0, T* out0, T* out1, int64_t n, int m, const uint8_t* k0,
                const uint8_t* k2, const uint64_t* nn) {
  const int words = sizeof(T) / 8;
  mx_cpu_parallel_for(n, 1 << 12, [&](int64_t s, int64_t e) {
    const int64_t CH = 512;
    std::vector<T> r0(CH), r1(CH), rt0(CH), rm0(CH), z0(CH), z2(CH);
    for (int64_t c = s; c < e; c += CH) {
      int64_t len = std::min(CH, e - c);
      mx_cpu_prf_range(k0, nn[0], words, c, len, r0.data());
      mx_cpu_prf_range(k2, nn[1], words, c, len, r1.data());
      mx_cpu_prf_range(k0, nn[2], words, c, len, rt0.data());
      mx_cpu_prf_range(k0, nn[3], words, c, len, rm0.data());
      mx_cpu_prf_range(k0, nn[4], words, c, len, z0.data());
      mx_cpu_prf_range(k2, nn[5], words, c, len, z2.data());
      for (int64_t t = 0; t < len; ++t) {
        int64_t i = c + t;
        T z1 = mxf::trunc_pr_z1<T>(s0[i], s0[n + i], s0[2 * n + i], r0[t], r1[t], rt0[t], rm0[t],
                                   z0[t], z2[t], m);
        out0[i] = z0[t];
        out0[n + i] = z1;
        out0[2 * n + i] = z2[t];
        out1[i] = z1;
        out1[n + i] = z2[t];
        out1[2 * n + i] = z0[t];
      }
    }
  });
  return 0;
}

template <class T>
int share3_host(int kind, const void* xv, T* out0, T* out1, int64_t n, int j, const uint8_t* kn,
                const uint8_t* /*ka: unused*/, uint64_t n1, uint64_t na) {
  const bool mir = kind & MX_SHARE_MIRROR;
  kind &= ~MX_SHARE_MIRROR;
  const int words = sizeof(T) == 1 ? 0 : (int)(sizeof(T) / 8);
  const T* x = (const T*)xv;
  const double* xf = (const double*)xv;  // kind MX_SHARE_F64 (moosex.h)
  const double scale = kind == MX_SHARE_F64 ? std::ldexp(1.0, (int)na) : 0.0;
  mx_cpu_parallel_for(n, 1 << 12, [&](int64_t s, int64_t e) {
    const int64_t CH = 512;
    std::vector<T> r1(CH);
    for (int64_t c = s; c < e; c += CH) {
      int64_t len = std::min(CH, e - c);
      mx_cpu_prf_range(kn, n1, words, c, len, r1.data());
      for (int64_t t = 0; t < len; ++t) {
        int64_t i = c + t;
        const T xi = kind == MX_SHARE_F64 ? (T)mxr::f64_to_i128(xf[i] * scale) : x[i];
        const T v = kind == MX_CROSS_BOOL ? (T)(xi ^ r1[t]) : (T)(xi - r1[t]);
        T slot[3];
        slot[j] = mir ? v : r1[t];
        slot[(j + 1) % 3] = mir ? r1[t] : v;
        slot[(j + 2) % 3] = 0;
        for (int p = 0; p < 3; ++p) {
          out0[p * n + i] = slot[p];
          out1[p * n + i] = slot[(p + 1) % 3];
        }
      }
    }
  });
  return 0;
}

}  // namespace

extern "C" {

int mx_trunc_pr3(int dev, int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                 const uint8_t* k0, const uint8_t* k2, const uint64_t* nonces, void* stream) {
  if (dev) return mxh_trunc_pr3(words, s0, out0, out1, n, m, k0, k2, nonces, stream);
  if (words == 1)
    return trunc3_host<uint64_t>((const uint64_t*)s0, (uint64_t*)out0, (uint64_t*)out1, n, m, k0,
                                 k2, nonces);
  if (words == 2)
    return trunc3_host<unsigned __int128>((const unsigned __int128*)s0, (unsigned __int128*)out0,
                                          (unsigned __int128*)out1, n, m, k0, k2, nonces);
  return -2;
}

int mx_share3(int dev, int kind, int words, const void* x, void* out0, void* out1, int64_t n,
              int j, const uint8_t* k_next, const uint8_t* k_all, uint64_t n1, uint64_t na,
              void* stream) {
  if (dev) return mxh_share3(kind, words, x, out0, out1, n, j, k_next, k_all, n1, na, stream);
  switch (words) {
    case 0:
      return share3_host<uint8_t>(kind, (const uint8_t*)x, (uint8_t*)out0, (uint8_t*)out1, n, j,
                                  k_next, k_all, n1, na);
    case 1:
      return share3_host<uint64_t>(kind, (const uint64_t*)x, (uint64_t*)out0, (uint64_t*)out1, n,
                                   j, k_next, k_all, n1, na);
    case 2:
      return share3_host<unsigned __int128>(kind, (const unsigned __int128*)x,
                                            (unsigned __int128*)out0, (unsigned __int128*)out1, n,
                                            j, k_next, k_all, n1, na);
  }
  return -2;
}

// key-slot variants: host slots lead with the raw key (moosex.h)
int mx_trunc_pr3_k(int dev, int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                   const uint32_t* slot_k0, const uint32_t* slot_k2, const uint64_t* nonces,
                   void* stream) {
  if (dev)
    return mxh_trunc_pr3_k(words, s0, out0, out1, n, m, slot_k0, slot_k2, nonces, stream);
  return mx_trunc_pr3(0, words, s0, out0, out1, n, m, (const uint8_t*)slot_k0,
                      (const uint8_t*)slot_k2, nonces, stream);
}

// mx_trunc_pr3_k writing party p's output slot at out + p * ostride (row views of a
// larger stack); the host path computes dense slots and copies them out
int mx_trunc_pr3_ko(int dev, int words, const void* s0, void* out0, void* out1, int64_t n,
                    int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                    const uint64_t* nonces, int64_t ostride, void* stream) {
  if (dev)
    return mxh_trunc_pr3_ko(words, s0, out0, out1, n, m, slot_k0, slot_k2, nonces, ostride,
                            stream);
  if (words != 1 && words != 2) return -2;
  const size_t es = 8 * (size_t)words;
  std::vector<uint8_t> t0(3 * n * es), t1(3 * n * es);
  int rc = mx_trunc_pr3_k(0, words, s0, t0.data(), t1.data(), n, m, slot_k0, slot_k2, nonces,
                          stream);
  if (rc) return rc;
  for (int p = 0; p < 3; ++p) {
    std::memcpy((uint8_t*)out0 + p * ostride * es, t0.data() + p * n * es, n * es);
    std::memcpy((uint8_t*)out1 + p * ostride * es, t1.data() + p * n * es, n * es);
  }
  return 0;
}

// mx_trunc_pr3_ko of cm * s0 (cm: public multiplier, words little-endian)
int mx_trunc_pr3_kmo(int dev, int words, const void* s0, void* out0, void* out1, int64_t n,
                     int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                     const uint64_t* nonces, int64_t ostride, const uint64_t* cm, void* stream) {
  if (dev)
    return mxh_trunc_pr3_kmo(words, s0, out0, out1, n, m, slot_k0, slot_k2, nonces, ostride, cm,
                             stream);
  if (words == 1) {
    std::vector<uint64_t> t(3 * n);
    for (int64_t i = 0; i < 3 * n; ++i) t[i] = ((const uint64_t*)s0)[i] * cm[0];
    return mx_trunc_pr3_ko(0, words, t.data(), out0, out1, n, m, slot_k0, slot_k2, nonces,
                           ostride, stream);
  }
  if (words == 2) {
    using u128 = unsigned __int128;
    const u128 c = ((u128)cm[1] << 64) | cm[0];
    std::vector<u128> t(3 * n);
    for (int64_t i = 0; i < 3 * n; ++i) t[i] = ((const u128*)s0)[i] * c;
    return mx_trunc_pr3_ko(0, words, t.data(), out0, out1, n, m, slot_k0, slot_k2, nonces,
                           ostride, stream);
  }
  return -2;
}

int mx_share3_k(int dev, int kind, int words, const void* x, void* out0, void* out1, int64_t n,
                int j, const uint32_t* slot_next, const uint32_t* slot_all, uint64_t n1,
                uint64_t na, void* stream) {
  if (dev)
    return mxh_share3_k(kind, words, x, out0, out1, n, j, slot_next, slot_all, n1, na, stream);
  return mx_share3(0, kind, words, x, out0, out1, n, j, (const uint8_t*)slot_next,
                   (const uint8_t*)slot_all, n1, na, stream);
}

}  // extern "C"
