// Per-party bit decomposition front and B2A (one party per GPU / process / thread): the
// element arithmetic shared by the device kernels (rss_bits_party.hip) and the host twins
// (rss_bits_party_cpu.cpp).
//
// Bit decomposition of an arithmetic sharing x (replicated: P_p holds (x_p, x_{p+1})),
// reference replicated/bits.rs + misc.rs:181-243, as the generic protocol code
// (protocols/replicated.py bit_decompose): P0 boolean-shares y = x0 + x1 (a = (a0, a1, 0)
// with a0 = PRF(k0, n1), a1 = y ^ a0), x2 is the trivial sharing b = (0, 0, x2), and the
// packed Kogge-Stone adder starts from p = a ^ b and g = a & b.  The front below gives every
// party its p pair and its zero-shared cross term z_p of g = a & b:
//   P0 (before any message):  p = (a0, a1), z0 = 0            ^ F(k0) ^ F(k1);  a1 -> P1
//   P2 (before any message):  p = (x2, a0), z2 = (a0 & x2)    ^ F(k2) ^ F(k0)
//   P1 (after a1 arrives):    p = (a1, x2), z1 = (a1 & x2)    ^ F(k1) ^ F(k2)
// (F(k) = PRF(k, n_g)); g = (z_p, z_{p+1}) after one reshare -- P0's z0 and P2's z2 travel
// with the share message, P1's z1 one round later.  Same PRF streams and nonces as share +
// from_slot_holders + xor + and_, so the same shares, in 1 kernel per party instead of 5.
//
// B2A of bit planes of a boolean sharing s (packed words; plane j = bit start + j), as
// rep.b2a (convert.rs:316-390): A = P0's arithmetic sharing of a = s0 ^ s1 (A0 = PRF(k0, n1),
// A1 = a - A0, A2 = 0), B = the trivial sharing of s2, AB zero-shared (arith), result
// A + B - 2 AB:
//   P0 (phase 0): base = (A0, A1), z0 = 0      + F(k0) - F(k1);  A1 -> P1
//   P2 (phase 0): base = (s2, A0), z2 = A0 s2  + F(k2) - F(k0)
//   P1 (phase 1): base = (A1, s2), z1 = A1 s2  + F(k1) - F(k2)
//   all (phase 2, after the reshare of z): out = base - 2 (z_p, z_{p+1}).
#pragma once
#include <stdint.h>

#include "aes_core.h"

namespace mxb {

template <class T>
struct Front {
  T msg, z, p0, p1;
};

// xa, xb: this party's two arithmetic components; arecv: P1's received a1; fa = PRF(k0, n1)
// (P0: own key, P2: next key), fo / fn = PRF(own / next key, n_g)
template <class T>
MX_HD inline Front<T> front(int role, T xa, T xb, T arecv, T fa, T fo, T fn) {
  Front<T> r{};
  if (role == 0) {
    const T y = xa + xb;
    r.msg = y ^ fa;
    r.p0 = fa;
    r.p1 = r.msg;
    r.z = fo ^ fn;
  } else if (role == 2) {
    r.p0 = xa;
    r.p1 = fa;
    r.z = (fa & xa) ^ fo ^ fn;
  } else {
    r.p0 = arecv;
    r.p1 = xb;
    r.z = (arecv & xb) ^ fo ^ fn;
  }
  return r;
}

template <class T>
struct B2a {
  T msg, z, base0, base1;
};

// c0, c1: this party's two boolean components' bit (0 / 1); Arecv: P1's received A1
template <class T>
MX_HD inline B2a<T> b2a(int role, T c0, T c1, T Arecv, T fa, T fo, T fn) {
  B2a<T> r{};
  if (role == 0) {
    const T a = c0 ^ c1;
    r.base0 = fa;
    r.base1 = a - fa;
    r.msg = r.base1;
    r.z = fo - fn;
  } else if (role == 2) {
    r.base0 = c0;
    r.base1 = fa;
    r.z = fa * c0 + fo - fn;
  } else {
    r.base0 = Arecv;
    r.base1 = c1;
    r.z = Arecv * c1 + fo - fn;
  }
  return r;
}

// bit q of a sum word of the packed adder: (p ^ ((g ^ t) << 1)) >> q & 1
template <class T>
MX_HD inline T sum_bit(T p, T g, T t, int q) {
  T v = (p >> q) & (T)1;
  if (q > 0) v ^= ((g ^ t) >> (q - 1)) & (T)1;
  return v;
}

// the bit plane of B2A row ``row``: plane start + row of element block 0.  With ``xbit`` >= 0
// the rows before the last tail rows are XORed (locally, share-wise) with plane xbit of block
// 0 -- the planes of |z| up to one ulp -- and the tail rows are sign planes.  ``blocks``
// packs the block layout: nb = blocks & 0xff blocks concatenated along the elements, and
// sbit = blocks >> 8 the sign plane of the tail rows (0: xbit).
//   nb == 1: one tail row, the sign of z (block 0);
//   nb == 3 (the adder ran over z, z - T, z + T): NOT sign(z - T) = [z >= T],
//            sign(z + T) = [z < -T], then sign(z);
//   nb == 2 (z, x): one tail row, sign(x) at plane sbit -- the ring's msb when sbit is the
//            top bit, so the sign holds for every representable x, whatever bound z's
//            planes assume;
//   nb == 4 (z, x - T', x + T', x): [x >= T'] = NOT sign(x - T'), [x < -T'] = sign(x + T'),
//            sign(x), all at plane sbit.
// ``neg``: the row is the complement (boolean NOT: share component 0 flipped).
MX_HD inline int tail_rows(int xbit, int blocks) {
  if (xbit < 0) return 0;
  const int nb = blocks & 0xff;
  return (nb == 2 || nb == 4) ? nb - 1 : nb;
}

MX_HD inline void plane_of(int row, int start, int count, int xbit, int blocks, int* q, int* xq,
                           int* blk, int* neg) {
  *blk = 0;
  *neg = 0;
  const int nb = blocks & 0xff, sbit = blocks >> 8;
  const int tail = tail_rows(xbit, blocks);
  if (row < count - tail) {
    *q = start + row;
    *xq = xbit;
    return;
  }
  *q = sbit > 0 ? sbit : xbit;
  *xq = -1;
  const int k = row - (count - tail);  // 0 .. tail - 1
  if (nb == 3) {
    *blk = k == 0 ? 1 : (k == 1 ? 2 : 0);
    *neg = k == 0;
  } else if (nb == 2) {
    *blk = 1;
  } else if (nb == 4) {
    *blk = k + 1;
    *neg = k == 0;
  }
}

}  // namespace mxb
