// Host versions of the per-party bit decomposition front and B2A (rss_bits_party.hip,
// protocol in bits_party.h) and the C ABI entry points that dispatch host / device.
#include <algorithm>
#include <functional>
#include <vector>

#include "bits_party.h"
#include "moosex.h"

void mx_cpu_prf_range(const uint8_t* key, uint64_t nonce, int words, int64_t i0, int64_t n,
                      void* out);

extern "C" {
int mxh_bits_front(int words, int role, int64_t n, const void* xa, const void* xb,
                   const void* arecv, void* msg, void* z, void* p0, void* p1,
                   const uint32_t* const* slots, const uint64_t* nn, void* stream);
int mxh_bits_b2a(int words, int phase, int role, int64_t S, int start, int count, int xbit,
                 int blocks, const void* const* src, const void* arecv, void* msg, void* z, void* base0,
                 void* base1, const void* zr, void* out0, void* out1,
                 const uint32_t* const* slots, const uint64_t* nn, void* stream);
}

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;

template <class T>
std::vector<T> prf(const uint32_t* slot, uint64_t nonce, int64_t n) {
  std::vector<T> v(n);
  mx_cpu_prf_range((const uint8_t*)slot, nonce, (int)(sizeof(T) / 8), 0, n, v.data());
  return v;
}

template <class T>
int front(int role, int64_t n, const T* xa, const T* xb, const T* arecv, T* msg, T* z, T* p0,
          T* p1, const uint32_t* const* slots, const uint64_t* nn) {
  std::vector<T> fa(n, (T)0);
  if (role == 0) fa = prf<T>(slots[0], nn[0], n);
  if (role == 2) fa = prf<T>(slots[1], nn[0], n);
  const std::vector<T> fo = prf<T>(slots[0], nn[1], n), fn = prf<T>(slots[1], nn[1], n);
  for (int64_t i = 0; i < n; ++i) {
    const mxb::Front<T> r = mxb::front<T>(role, role == 1 ? (T)0 : xa[i],
                                          role == 2 ? (T)0 : xb[i],
                                          role == 1 ? arecv[i] : (T)0, fa[i], fo[i], fn[i]);
    if (role == 0) msg[i] = r.msg;
    z[i] = r.z;
    p0[i] = r.p0;
    p1[i] = r.p1;
  }
  return 0;
}

template <class T>
T src_bit(const T* s, const T* g, const T* t, int64_t e, int q) {
  if (g == nullptr) return (s[e] >> q) & (T)1;
  return mxb::sum_bit<T>(s[e], g[e], t ? t[e] : (T)0, q);
}

template <class T>
int b2a(int phase, int role, int64_t S, int start, int count, int xbit, int blocks,
        const void* const* src,
        const T* arecv, T* msg, T* z, T* base0, T* base1, const T* zr, T* out0, T* out1,
        const uint32_t* const* slots, const uint64_t* nn) {
  const int64_t n = S * count;
  if (phase == 2) {
    for (int64_t i = 0; i < n; ++i) {
      out0[i] = base0[i] - (T)2 * z[i];
      out1[i] = base1[i] - (T)2 * zr[i];
    }
    return 0;
  }
  std::vector<T> fa(n, (T)0);
  if (role == 0) fa = prf<T>(slots[0], nn[0], n);
  if (role == 2) fa = prf<T>(slots[1], nn[0], n);
  const std::vector<T> fo = prf<T>(slots[0], nn[1], n), fn = prf<T>(slots[1], nn[1], n);
  const T* s0 = (const T*)src[0];
  const T* s1 = (const T*)src[1];
  const T* g0 = (const T*)src[2];
  const T* g1 = (const T*)src[3];
  const T* t0 = (const T*)src[4];
  const T* t1 = (const T*)src[5];
  for (int64_t i = 0; i < n; ++i) {
    const int64_t row = i / S, e = i - row * S;
    int q, xq, blk, neg;
    mxb::plane_of((int)row, start, count, xbit, blocks, &q, &xq, &blk, &neg);
    const int64_t es = e + blk * S;  // the element in the adder's blocks
    T c0 = role == 1 ? (T)0 : src_bit<T>(s0, g0, t0, es, q);
    T c1 = role == 2 ? (T)0 : src_bit<T>(s1, g1, t1, es, q);
    if (neg && role == 0) c0 ^= (T)1;  // NOT: component 0 (P0's first) flipped
    if (xq >= 0) {
      if (role != 1) c0 ^= src_bit<T>(s0, g0, t0, e, xq);
      if (role != 2) c1 ^= src_bit<T>(s1, g1, t1, e, xq);
    }
    const mxb::B2a<T> r = mxb::b2a<T>(role, c0, c1, role == 1 ? arecv[i] : (T)0, fa[i], fo[i],
                                      fn[i]);
    if (role == 0) msg[i] = r.msg;
    z[i] = r.z;
    base0[i] = r.base0;
    base1[i] = r.base1;
  }
  return 0;
}

}  // namespace

extern "C" {

int mx_bits_front(int dev, int words, int role, int64_t n, const void* xa, const void* xb,
                  const void* arecv, void* msg, void* z, void* p0, void* p1,
                  const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  if (role < 0 || role > 2) return -3;
  if (dev) return mxh_bits_front(words, role, n, xa, xb, arecv, msg, z, p0, p1, slots, nn, stream);
  if (words == 1)
    return front<u64>(role, n, (const u64*)xa, (const u64*)xb, (const u64*)arecv, (u64*)msg,
                      (u64*)z, (u64*)p0, (u64*)p1, slots, nn);
  if (words == 2)
    return front<u128>(role, n, (const u128*)xa, (const u128*)xb, (const u128*)arecv,
                       (u128*)msg, (u128*)z, (u128*)p0, (u128*)p1, slots, nn);
  return -2;
}

int mx_bits_b2a(int dev, int words, int phase, int role, int64_t S, int start, int count,
                int xbit, int blocks, const void* const* src, const void* arecv, void* msg,
                void* z, void* base0, void* base1, const void* zr, void* out0, void* out1,
                const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  if (xbit < 0) blocks = 1;
  const int nb = blocks & 0xff, sbit = blocks >> 8;
  const int planes = count - mxb::tail_rows(xbit, blocks);  // rows read from start..
  if (role < 0 || role > 2 || phase < 0 || phase > 2 || start < 0 || count < 1 ||
      start + planes > 64 * words || xbit >= 64 * words || nb < 1 || nb > 4 ||
      sbit >= 64 * words || (sbit > 0) != (nb == 2 || nb == 4) || (xbit >= 0 && planes < 1))
    return -3;
  if (dev)
    return mxh_bits_b2a(words, phase, role, S, start, count, xbit, blocks, src, arecv, msg, z,
                        base0, base1, zr, out0, out1, slots, nn, stream);
  if (words == 1)
    return b2a<u64>(phase, role, S, start, count, xbit, blocks, src, (const u64*)arecv, (u64*)msg, (u64*)z,
                    (u64*)base0, (u64*)base1, (const u64*)zr, (u64*)out0, (u64*)out1, slots, nn);
  if (words == 2)
    return b2a<u128>(phase, role, S, start, count, xbit, blocks, src, (const u128*)arecv, (u128*)msg,
                     (u128*)z, (u128*)base0, (u128*)base1, (const u128*)zr, (u128*)out0,
                     (u128*)out1, slots, nn);
  return -2;
}

}  // extern "C"
