// Element-level ring semantics shared by the host and device kernels.
#pragma once
#include <stdint.h>
#include <string.h>

#include "aes_core.h"
#include "moosex.h"

namespace mxr {

using u64 = uint64_t;
using u128 = unsigned __int128;
using i128 = __int128;

template <class T>
struct Bits {
  static constexpr int value = 8 * sizeof(T);
};

template <class T>
MX_HD inline T binop(int op, T a, T b) {
  if constexpr (sizeof(T) == 1) {  // bit tensors: Z_2 (0/1 bytes)
    switch (op) {
      case MX_ADD:
      case MX_SUB:
      case MX_XOR: return (T)((a ^ b) & 1);
      case MX_MUL:
      case MX_AND: return (T)(a & b & 1);
      case MX_OR: return (T)((a | b) & 1);
    }
    return 0;
  } else {
    switch (op) {
      case MX_ADD: return a + b;
      case MX_SUB: return a - b;
      case MX_MUL: return a * b;
      case MX_AND: return a & b;
      case MX_OR: return a | b;
      case MX_XOR: return a ^ b;
    }
    return 0;
  }
}

template <class T>
MX_HD inline T unop(int op, T a, int k) {
  constexpr int W = Bits<T>::value;
  if constexpr (sizeof(T) == 1) {
    switch (op) {
      case MX_NEG: return (T)(a & 1);
      case MX_NOT: return (T)((a ^ 1) & 1);
      default: return k == 0 ? (T)(a & 1) : (T)0;
    }
  } else {
    switch (op) {
      case MX_NEG: return (T)0 - a;
      case MX_NOT: return ~a;
      case MX_SHL: return k >= W ? (T)0 : (T)(a << k);
      case MX_SHR: return k >= W ? (T)0 : (T)(a >> k);
      case MX_SAR: {
        if constexpr (sizeof(T) == 8) {
          int64_t s = (int64_t)a;
          return (T)(k >= 64 ? (s >> 63) : (s >> k));
        } else {
          i128 s = (i128)a;
          return (T)(k >= 128 ? (s >> 127) : (s >> k));
        }
      }
    }
    return 0;
  }
}

template <class T>
MX_HD inline uint8_t cmpop(int op, T a, T b) {
  if constexpr (sizeof(T) == 1) {
    switch (op) {
      case MX_LT: return a < b;
      case MX_GT: return a > b;
      case MX_EQ: return a == b;
      default: return a & 1;
    }
  } else if constexpr (sizeof(T) == 8) {
    int64_t x = (int64_t)a, y = (int64_t)b;
    switch (op) {
      case MX_LT: return x < y;
      case MX_GT: return x > y;
      case MX_EQ: return x == y;
      default: return (uint8_t)(a >> 63);
    }
  } else {
    i128 x = (i128)a, y = (i128)b;
    switch (op) {
      case MX_LT: return x < y;
      case MX_GT: return x > y;
      case MX_EQ: return x == y;
      default: return (uint8_t)(a >> 127);
    }
  }
}

template <class T>
MX_HD inline T cross(int kind, T x0, T x1, T y0, T y1, bool has_x1, bool has_y1) {
  if (kind == MX_CROSS_BOOL) {
    T v = x0 & y0;
    if (has_y1) v ^= x0 & y1;
    if (has_x1) v ^= x1 & y0;
    return v;
  }
  T v = x0 * y0;
  if (has_y1) v += x0 * y1;
  if (has_x1) v += x1 * y0;
  return v;
}

template <class T>
MX_HD inline T zs_combine(int kind, T v, T ra, T rb) {
  if (kind == MX_CROSS_BOOL) return (T)(v ^ ra ^ rb);
  return (T)(v + ra - rb);
}

// double -> two's complement integer, truncating toward zero (Rust `as i128`
// semantics, saturating at the range limits; NaN -> 0)
MX_HD inline i128 f64_to_i128(double x) {
  uint64_t bits;
  memcpy(&bits, &x, 8);
  int neg = (int)(bits >> 63);
  int e = (int)((bits >> 52) & 0x7ff);
  uint64_t mant = bits & ((1ull << 52) - 1);
  if (e == 0x7ff) return mant ? (i128)0 : (neg ? (i128)((u128)1 << 127) : ~(i128)((u128)1 << 127));
  if (e == 0) return 0;  // subnormals truncate to 0
  mant |= (1ull << 52);
  int sh = e - 1075;  // value = mant * 2^sh
  u128 mag;
  if (sh >= 0) {
    if (sh > 127 - 53) return neg ? (i128)((u128)1 << 127) : ~(i128)((u128)1 << 127);
    mag = (u128)mant << sh;
  } else if (sh <= -53) {
    mag = 0;
  } else {
    mag = (u128)(mant >> (-sh));
  }
  return neg ? -(i128)mag : (i128)mag;
}

MX_HD inline double i128_to_f64(u128 v) {
  i128 s = (i128)v;
  int neg = s < 0;
  u128 m = neg ? (u128)(-s) : (u128)s;
  uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
  double r = (double)hi * 18446744073709551616.0 + (double)lo;
  return neg ? -r : r;
}

}  // namespace mxr

// Device launchers (ring_hip.hip / gemm_mfma.hip)
extern "C" {
int mxh_ew_binary(int op, int words, const void* a, int64_t na, const void* b, int64_t nb,
                  void* out, int64_t n, void* stream);
int mxh_ew_unary(int op, int words, const void* a, void* out, int64_t n, int64_t param,
                 void* stream);
int mxh_ew_compare(int op, int words, const void* a, int64_t na, const void* b, int64_t nb,
                   uint8_t* out, int64_t n, void* stream);
int mxh_bit_extract(int words, const void* a, uint8_t* out, int64_t n, int bit, void* stream);
int mxh_ring_inject(int words, const uint8_t* bits, void* out, int64_t n, int bit,
                    void* stream);
int mxh_encode(int words, const double* x, void* out, int64_t n, int frac, void* stream);
int mxh_decode(int words, const void* x, double* out, int64_t n, int frac, void* stream);
int mxh_addn_decode(int words, const void* a, const void* b, const void* c, const void* d,
                    double* out, int64_t n, int frac, void* stream);
int mxh_fill(int words, void* out, int64_t n, uint64_t lo, uint64_t hi, void* stream);
int mxh_bit_planes(int words, const void* a, uint8_t* out, int64_t outer, int64_t inner,
                   int start, int count, void* stream);
int mxh_weighted_sum(int words, const void* a, const void* w, void* out, int64_t outer,
                     int64_t k, int64_t inner, void* stream);
int mxh_sum_axis(int words, const void* a, void* out, int64_t outer, int64_t red, int64_t inner,
                 void* stream);
int mxh_prg(const uint8_t* key16, uint64_t nonce, uint64_t ctr0, void* out, int64_t nbytes,
            void* stream);
int mxh_rss_cross(int kind, int words, const void* x0, const void* x1, const void* y0,
                  const void* y1, void* out, int64_t n, int nparties, const uint8_t* keys16,
                  uint64_t nonce, void* stream);
int mxh_prf_expand(int words, void* out, int64_t n, int nkeys, const uint8_t* keys16,
                   uint64_t nonce, void* stream);
int mxh_rss_cross_kp(int kind, int words, const void* x0, const void* x1, const void* y0,
                     const void* y1, void* out, int64_t n, int nparties,
                     const uint32_t* const* slot_ptrs, uint64_t nonce, void* stream);
int mxh_rss_cross_k(int kind, int words, const void* x0, const void* x1, const void* y0,
                    const void* y1, void* out, int64_t n, int nparties, const uint32_t* slots,
                    int nslots, uint64_t nonce, void* stream);
int mxh_rss_mul3_kv(int kind, int words, const void* x0, const void* x1, const void* y0,
                    const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                    uint64_t nonce, const int64_t* views, void* stream);
int mxh_rss_mul3_k(int kind, int words, const void* x0, const void* x1, const void* y0,
                   const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                   uint64_t nonce, void* stream);
int mxh_ew_binary_slot(int op, int words, const void* a, const void* b, int64_t nb, void* out,
                       int64_t m, int nparties, int which, void* stream);
int mxh_add_zs3(int words, const void* v, const void* r, void* out0, void* out1, int64_t n,
                void* stream);
int mxh_ew_binary2(int op, int words, const void* a0, const void* b0, void* out0,
                   const void* a1, const void* b1, void* out1, int64_t na, int64_t nb, int64_t n,
                   void* stream);
int mxh_mul_add2(int words, const void* a0, const void* a1, const void* f, const void* c,
                 int add0, int add1, void* out0, void* out1, int64_t n, void* stream);
int mxh_ew_add3(int words, const void* a, const void* b, const void* c, void* out, int64_t n,
                void* stream);
int mxh_lincomb2(int words, int nin, const void* const* ins, const int64_t* coef, const void* b,
                 int64_t nb, void* out0, void* out1, int64_t m, int nparties, int which0,
                 int which1, void* stream);
int mxh_sum_views2(int words, const void* base0, const void* base1, int64_t is0, int64_t is1,
                   int64_t ps0, int64_t ps1, int k, void* out0, void* out1, int64_t m,
                   int nparties, void* stream);
int mxh_slot_place2(int words, const void* x0, const void* x1, void* out0, void* out1,
                    int64_t m, int nparties, int which0, int which1, void* stream);
int mxh_mul_trunc3_kv(int words, const void* x0, const void* x1, const void* y0, const void* y1,
                      void* out0, void* out1, int64_t n, int64_t ostride, const uint32_t* slots,
                      uint64_t nmul, int m, const uint64_t* nn, const int64_t* views,
                      void* stream);
int mxh_ew_unary2(int op, int words, const void* a0, void* out0, const void* a1, void* out1,
                  int64_t n, int64_t param, void* stream);
int mxh_transpose2(int words, const void* a0, void* out0, const void* a1, void* out1,
                   int64_t rows, int64_t cols, void* stream);
int mxh_ew_binary_slot2(int op, int words, const void* a0, const void* a1, const void* b,
                        int64_t nb, void* out0, void* out1, int64_t m, int nparties, int which0,
                        int which1, void* stream);
int mxh_ks_cross1(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                  void* z, int64_t n, int d, int both, const uint8_t* keys16, uint64_t nonce,
                  void* stream);
int mxh_ks_cross1_s(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                    void* z, int64_t n, int d, int both, const uint32_t* const* slots,
                    uint64_t nonce, void* stream);
int mxh_ks_cross1x_s(int words, const void* g0, const void* g1, const void* t0, const void* t1,
                     void* go0, void* go1, const void* p0, const void* p1, void* z, int64_t n,
                     int d, int both, const uint32_t* const* slots, uint64_t nonce,
                     void* stream);
int mxh_ks_sum2(int words, const void* p0, const void* p1, const void* g0, const void* g1,
                const void* t0, const void* t1, void* o0, void* o1, int64_t n, void* stream);
int mxh_ks_adder3_k(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                    void* og0, void* og1, int64_t n, int nlev, const uint32_t* slots,
                    const uint64_t* nonces, void* stream);
int mxh_ks_level3_k(int words, const void* g0, const void* g1, const void* p0, const void* p1,
                    void* og0, void* og1, void* op0, void* op1, int64_t n, int d, int both,
                    const uint32_t* slots, uint64_t nonce, void* stream);
int mxh_prf_expand_k(int words, void* out, int64_t n, int nkeys, const uint32_t* slots,
                     uint64_t nonce, void* stream);
int mxh_gemm(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
             const void* A1, const void* B0, const void* B1, int mode, void* C, int accumulate,
             void* stream);
}
