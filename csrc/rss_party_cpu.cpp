// Host versions of the per-party protocol kernels (rss_party.hip) and the C ABI entry
// points that dispatch host / device.  Key slots are MX_KEY_SLOT_WORDS-word images whose
// first four words are the raw AES key.
#include <cmath>
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
int mxh_trunc_party_r0(int words, int64_t n, int m, int ncomp, const int* roles,
                       const void* s0, const void* s1, void* msg, void* msg_rm, void* out0,
                       void* out1, const uint32_t* const* slots, const uint64_t* nn,
                       void* stream);
int mxh_trunc_party_r1(int words, int64_t n, int m, int ncomp, const int* roles,
                       const void* msg, const void* rmk, const void* rrt, const void* rrm,
                       void* w, void* out0, void* out1, const uint32_t* const* slots,
                       const uint64_t* nn, void* stream);
int mxh_share_party(int kind, int words, int64_t n, int ncomp, const int* rel, const void* x,
                    void* out0, void* out1, const uint32_t* const* slots, uint64_t n1,
                    uint64_t na, void* stream);
int mxh_dot_tail_r0(int words, int64_t n, int m, int ncomp, const int* roles,
                    const void* const* cross, void* const* msg, void* const* msg_rt,
                    void* const* msg_rm, void* const* out0, void* const* out1,
                    const uint32_t* const* slots, const uint64_t* nn, void* stream);
int mxh_dot_tail_r1(int words, int64_t n, int m, int ncomp, const int* roles,
                    const void* const* msg, const void* const* rmk, const void* const* rz,
                    const void* const* rrt, const void* const* rrm, void* const* w,
                    void* const* out0, void* const* out1, const uint32_t* const* slots,
                    const uint64_t* nn, void* stream);
int mxh_dot_tail_r2(int words, int64_t n, int ncomp, const int* roles, const void* const* a,
                    const void* const* b, void* const* out, void* stream);
}

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;

const uint8_t* key_of(const uint32_t* slot) { return (const uint8_t*)slot; }

// chunked element loop with up to six PRF streams per chunk
template <class T, class F>
void for_chunks(int64_t n, F&& f) {
  mx_cpu_parallel_for(n, 1 << 12, [&](int64_t s, int64_t e) {
    const int64_t CH = 512;
    for (int64_t c = s; c < e; c += CH) f(c, std::min(CH, e - c));
  });
}

template <class T>
void prf(const uint32_t* slot, uint64_t nonce, int64_t i0, int64_t len, T* out) {
  const int words = sizeof(T) == 1 ? 0 : (int)(sizeof(T) / 8);
  mx_cpu_prf_range(key_of(slot), nonce, words, i0, len, out);
}

template <class T>
int trunc_r0(int64_t n, int m, int ncomp, const int* roles, const T* s0, const T* s1, T* msg,
             u64* msg_rm, T* out0, T* out1, const uint32_t* const* slots, const uint64_t* nn) {
  for (int c = 0; c < ncomp; ++c) {
    const int role = roles[c];
    const uint32_t* own = slots[2 * c];
    const uint32_t* nxt = slots[2 * c + 1];
    const int64_t base = (int64_t)c * n;
    for_chunks<T>(n, [&](int64_t i0, int64_t len) {
      std::vector<T> a(len), b(len), t(len), mm(len), z0(len), z2(len);
      if (role == 0) {
        prf<T>(own, nn[0], i0, len, a.data());
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = base + i0 + q;
          msg[i] = mxf::trunc_mask0<T>(s0[i], s1[i], a[q]);
        }
      } else if (role == 1) {
        prf<T>(nxt, nn[1], i0, len, a.data());
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = base + i0 + q;
          msg[i] = s1[i] + a[q];
        }
      } else if (role == 2) {
        prf<T>(nxt, nn[0], i0, len, a.data());
        prf<T>(own, nn[1], i0, len, b.data());
        prf<T>(nxt, nn[2], i0, len, t.data());
        prf<T>(nxt, nn[3], i0, len, mm.data());
        prf<T>(nxt, nn[4], i0, len, z0.data());
        prf<T>(own, nn[5], i0, len, z2.data());
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = base + i0 + q;
          mxf::trunc_dealer<T>(a[q], b[q], t[q], mm[q], m, &msg[i], &msg_rm[i]);
          out0[i] = z2[q];
          out1[i] = z0[q];
        }
      }
    });
  }
  return 0;
}

template <class T>
int trunc_r1(int64_t n, int m, int ncomp, const int* roles, const T* msg, const T* rmk,
             const T* rrt, const u64* rrm, T* w, T* out0, T* out1,
             const uint32_t* const* slots, const uint64_t* nn) {
  for (int c = 0; c < ncomp; ++c) {
    const int role = roles[c];
    const int64_t base = (int64_t)c * n;
    for_chunks<T>(n, [&](int64_t i0, int64_t len) {
      std::vector<T> t(len), mm(len), z(len);
      if (role == 0) {
        const uint32_t* k0 = slots[2 * c];
        prf<T>(k0, nn[2], i0, len, t.data());
        prf<T>(k0, nn[3], i0, len, mm.data());
        prf<T>(k0, nn[4], i0, len, z.data());
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = base + i0 + q;
          const T y0 = mxf::trunc_y<T>(msg[i] + rmk[i], t[q], mm[q], m, true);
          w[i] = y0 - z[q];
          out0[i] = z[q];
        }
      } else if (role == 1) {
        prf<T>(slots[2 * c + 1], nn[5], i0, len, z.data());
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = base + i0 + q;
          const T y1 = mxf::trunc_y<T>(msg[i] + rmk[i], rrt[i], (T)rrm[i], m, false);
          w[i] = y1 - z[q];
          out1[i] = z[q];
        }
      }
    });
  }
  return 0;
}

template <class T>
int share_party(int kind, int64_t n, int ncomp, const int* rel, const void* xp, T* out0, T* out1,
                const uint32_t* const* slots, uint64_t n1, uint64_t na) {
  const bool mir = kind & MX_SHARE_MIRROR;
  kind &= ~MX_SHARE_MIRROR;
  const T* x = (const T*)xp;
  const double* xf = (const double*)xp;  // kind MX_SHARE_F64 (moosex.h)
  const double scale = kind == MX_SHARE_F64 ? std::ldexp(1.0, (int)na) : 0.0;
  for (int c = 0; c < ncomp; ++c) {
    const int code = rel[c];  // as k_share_party: role + 4 * (1 + local P_{j+1} component)
    if (code < 0) continue;
    const int r = code & 3, fwd = (code >> 2) - 1;
    const int64_t base = (int64_t)c * n;
    if (r > 2) continue;
    for_chunks<T>(n, [&](int64_t i0, int64_t len) {
      std::vector<T> a(len);
      if (mir ? r != 2 : r != 1) prf<T>(slots[2 * c], n1, i0, len, a.data());
      for (int64_t q = 0; q < len; ++q) {
        const int64_t i = base + i0 + q;
        if (r == 0) {
          const T xv =
              kind == MX_SHARE_F64 ? (T)mxr::f64_to_i128(xf[i0 + q] * scale) : x[i0 + q];
          const T v = kind == MX_CROSS_BOOL ? (T)(xv ^ a[q]) : (T)(xv - a[q]);
          out0[i] = mir ? v : a[q];
          out1[i] = mir ? a[q] : v;
          if (fwd >= 0) (mir ? out1 : out0)[(int64_t)fwd * n + i0 + q] = v;
        } else if (r == 1) {
          if (mir) out0[i] = a[q];
          out1[i] = 0;  // s0 arrives from the owner (mirrored: zero slot j+2)
        } else {
          out0[i] = 0;
          if (!mir) out1[i] = a[q];  // mirrored: s1 arrives from the owner
        }
      }
    });
  }
  return 0;
}


// ---- fixed-point dot tail (see rss_party.hip: reshare folded into TruncPr round A) ----
template <class T>
int dot_tail_r0(int64_t n, int m, int ncomp, const int* roles, const void* const* cross,
                void* const* msg, void* const* msg_rt, void* const* msg_rm, void* const* out0,
                void* const* out1, const uint32_t* const* slots, const uint64_t* nn) {
  for (int c = 0; c < ncomp; ++c) {
    const int role = roles[c];
    if (role < 0 || role > 2) continue;
    const uint32_t* own = slots[2 * c];
    const uint32_t* nxt = slots[2 * c + 1];
    const T* x = (const T*)cross[c];
    T* mo = (T*)msg[c];
    // as k_dot_tail_r0: no cross -> the dealer part only; no msg_rt -> no dealer part
    const bool main_part = x != nullptr;
    const bool dealer = role == 2 && msg_rt[c] != nullptr;
    for_chunks<T>(n, [&](int64_t i0, int64_t len) {
      if (main_part) {
        // zero share: P0 f(k0), P1 -f(k2), P2 f(k2) - f(k0) (rss_party.hip)
        std::vector<T> a(len, (T)0), b(len, (T)0), r(len);
        if (role != 1) prf<T>(own, nn[0], i0, len, a.data());
        if (role != 0) prf<T>(nxt, nn[0], i0, len, b.data());
        if (role == 0) prf<T>(own, nn[1], i0, len, r.data());
        if (role == 1) prf<T>(nxt, nn[2], i0, len, r.data());
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = i0 + q;
          const T z = x[i] + a[q] - b[q];
          mo[i] = role == 0 ? mxf::trunc_mask0<T>(z, (T)0, r[q]) : role == 1 ? (T)(z + r[q]) : z;
        }
      }
      if (dealer) {
        std::vector<T> r0(len), r1(len), t(len), mm(len), z0(len), z2(len);
        prf<T>(nxt, nn[1], i0, len, r0.data());
        prf<T>(own, nn[2], i0, len, r1.data());
        prf<T>(nxt, nn[3], i0, len, t.data());
        prf<T>(nxt, nn[4], i0, len, mm.data());
        prf<T>(nxt, nn[5], i0, len, z0.data());
        prf<T>(own, nn[6], i0, len, z2.data());
        T* rt = (T*)msg_rt[c];
        u64* rm = (u64*)msg_rm[c];
        for (int64_t q = 0; q < len; ++q) {
          const int64_t i = i0 + q;
          mxf::trunc_dealer<T>(r0[q], r1[q], t[q], mm[q], m, &rt[i], &rm[i]);
          ((T*)out0[c])[i] = z2[q];
          ((T*)out1[c])[i] = z0[q];
        }
      }
    });
  }
  return 0;
}

template <class T>
int dot_tail_r1(int64_t n, int m, int ncomp, const int* roles, const void* const* msg,
                const void* const* rmk, const void* const* rz, const void* const* rrt,
                const void* const* rrm, void* const* w, void* const* out0, void* const* out1,
                const uint32_t* const* slots, const uint64_t* nn) {
  for (int c = 0; c < ncomp; ++c) {
    const int role = roles[c];
    if (role != 0 && role != 1) continue;
    const T* mine = (const T*)msg[c];
    const T* other = (const T*)rmk[c];
    const T* z2m = rz ? (const T*)rz[c] : nullptr;
    T* wo = (T*)w[c];
    T* o = role == 0 ? (T*)out0[c] : (T*)out1[c];
    for_chunks<T>(n, [&](int64_t i0, int64_t len) {
      std::vector<T> t(len), mm(len), z(len);
      if (role == 0) {
        prf<T>(slots[2 * c], nn[3], i0, len, t.data());
        prf<T>(slots[2 * c], nn[4], i0, len, mm.data());
        prf<T>(slots[2 * c], nn[5], i0, len, z.data());
      } else {
        prf<T>(slots[2 * c + 1], nn[6], i0, len, z.data());
      }
      for (int64_t q = 0; q < len; ++q) {
        const int64_t i = i0 + q;
        T cc = mine[i] + other[i];
        if (z2m) cc += z2m[i];
        const T y = role == 0 ? mxf::trunc_y<T>(cc, t[q], mm[q], m, true)
                              : mxf::trunc_y<T>(cc, ((const T*)rrt[c])[i],
                                                (T)((const u64*)rrm[c])[i], m, false);
        wo[i] = y - z[q];
        o[i] = z[q];
      }
    });
  }
  return 0;
}

template <class T>
int dot_tail_r2(int64_t n, int ncomp, const int* roles, const void* const* a,
                const void* const* b, void* const* out) {
  for (int c = 0; c < ncomp; ++c) {
    if (roles[c] != 0 && roles[c] != 1) continue;
    const T* x = (const T*)a[c];
    const T* y = (const T*)b[c];
    T* o = (T*)out[c];
    mx_cpu_parallel_for(n, 1 << 14, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) o[i] = x[i] + y[i];
    });
  }
  return 0;
}

}  // namespace

extern "C" {

int mx_trunc_party_r0(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                      const void* s0, const void* s1, void* msg, void* msg_rm, void* out0,
                      void* out1, const uint32_t* const* slots, const uint64_t* nn,
                      void* stream) {
  if (m < 1 || m > 63) return -3;
  if (dev)
    return mxh_trunc_party_r0(words, n, m, ncomp, roles, s0, s1, msg, msg_rm, out0, out1,
                              slots, nn, stream);
  if (words == 1)
    return trunc_r0<u64>(n, m, ncomp, roles, (const u64*)s0, (const u64*)s1, (u64*)msg,
                         (u64*)msg_rm, (u64*)out0, (u64*)out1, slots, nn);
  if (words == 2)
    return trunc_r0<u128>(n, m, ncomp, roles, (const u128*)s0, (const u128*)s1, (u128*)msg,
                          (u64*)msg_rm, (u128*)out0, (u128*)out1, slots, nn);
  return -2;
}

int mx_trunc_party_r1(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                      const void* msg, const void* rmk, const void* rrt, const void* rrm,
                      void* w, void* out0, void* out1, const uint32_t* const* slots,
                      const uint64_t* nn, void* stream) {
  if (m < 1 || m > 63) return -3;
  if (dev)
    return mxh_trunc_party_r1(words, n, m, ncomp, roles, msg, rmk, rrt, rrm, w, out0, out1,
                              slots, nn, stream);
  if (words == 1)
    return trunc_r1<u64>(n, m, ncomp, roles, (const u64*)msg, (const u64*)rmk,
                         (const u64*)rrt, (const u64*)rrm, (u64*)w, (u64*)out0, (u64*)out1,
                         slots, nn);
  if (words == 2)
    return trunc_r1<u128>(n, m, ncomp, roles, (const u128*)msg, (const u128*)rmk,
                          (const u128*)rrt, (const u64*)rrm, (u128*)w, (u128*)out0,
                          (u128*)out1, slots, nn);
  return -2;
}

int mx_share_party(int dev, int kind, int words, int64_t n, int ncomp, const int* rel,
                   const void* x, void* out0, void* out1, const uint32_t* const* slots,
                   uint64_t n1, uint64_t na, void* stream) {
  if (dev)
    return mxh_share_party(kind, words, n, ncomp, rel, x, out0, out1, slots, n1, na, stream);
  switch (words) {
    case 0:
      return share_party<uint8_t>(kind, n, ncomp, rel, (const uint8_t*)x, (uint8_t*)out0,
                                  (uint8_t*)out1, slots, n1, na);
    case 1:
      return share_party<u64>(kind, n, ncomp, rel, (const u64*)x, (u64*)out0, (u64*)out1,
                              slots, n1, na);
    case 2:
      return share_party<u128>(kind, n, ncomp, rel, (const u128*)x, (u128*)out0, (u128*)out1,
                               slots, n1, na);
    default:
      return -2;
  }
}


int mx_dot_tail_r0(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                   const void* const* cross, void* const* msg, void* const* msg_rt,
                   void* const* msg_rm, void* const* out0, void* const* out1,
                   const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  if (m < 1 || m > 63) return -3;
  if (ncomp < 1 || ncomp > 3) return -3;
  if (dev)
    return mxh_dot_tail_r0(words, n, m, ncomp, roles, cross, msg, msg_rt, msg_rm, out0, out1,
                           slots, nn, stream);
  if (words == 1)
    return dot_tail_r0<u64>(n, m, ncomp, roles, cross, msg, msg_rt, msg_rm, out0, out1, slots,
                            nn);
  if (words == 2)
    return dot_tail_r0<u128>(n, m, ncomp, roles, cross, msg, msg_rt, msg_rm, out0, out1, slots,
                             nn);
  return -2;
}

int mx_dot_tail_r1(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                   const void* const* msg, const void* const* rmk, const void* const* rz,
                   const void* const* rrt, const void* const* rrm, void* const* w,
                   void* const* out0, void* const* out1, const uint32_t* const* slots,
                   const uint64_t* nn, void* stream) {
  if (m < 1 || m > 63) return -3;
  if (ncomp < 1 || ncomp > 3) return -3;
  if (dev)
    return mxh_dot_tail_r1(words, n, m, ncomp, roles, msg, rmk, rz, rrt, rrm, w, out0, out1,
                           slots, nn, stream);
  if (words == 1)
    return dot_tail_r1<u64>(n, m, ncomp, roles, msg, rmk, rz, rrt, rrm, w, out0, out1, slots,
                            nn);
  if (words == 2)
    return dot_tail_r1<u128>(n, m, ncomp, roles, msg, rmk, rz, rrt, rrm, w, out0, out1, slots,
                             nn);
  return -2;
}

int mx_dot_tail_r2(int dev, int words, int64_t n, int ncomp, const int* roles,
                   const void* const* a, const void* const* b, void* const* out, void* stream) {
  if (ncomp < 1 || ncomp > 3) return -3;
  if (dev) return mxh_dot_tail_r2(words, n, ncomp, roles, a, b, out, stream);
  if (words == 1) return dot_tail_r2<u64>(n, ncomp, roles, a, b, out);
  if (words == 2) return dot_tail_r2<u128>(n, ncomp, roles, a, b, out);
  return -2;
}

}  // extern "C"
