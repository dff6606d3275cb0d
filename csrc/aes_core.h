// AES-128 (FIPS-197) building blocks: the AES dialect (AES-GCM decryption of host
// ciphertexts, protocols/aes.py) encrypts blocks with AES-NI when available and with the
// portable T-table implementation below otherwise; the unit tests check both against the
// FIPS-197 appendix vector.  (The protocols' PRF is ChaCha12, prf_core.h.)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MX_HD __host__ __device__
#else
#define MX_HD
#endif

namespace mx {

#define MX_SBOX_INIT { \
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, \
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, \
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, \
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, \
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84, \
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf, \
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, \
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, \
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, \
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, \
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79, \
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08, \
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, \
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, \
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, \
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16, \
  }

static const uint8_t kSbox[256] = MX_SBOX_INIT;

MX_HD inline uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

// T0[x] = (2s, s, s, 3s) packed big-endian, s = S(x); T_k = ror(T0, 8k)
MX_HD inline uint32_t t0_entry(uint8_t s) {
  uint8_t s2 = xtime(s);
  uint8_t s3 = (uint8_t)(s2 ^ s);
  return ((uint32_t)s2 << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) | (uint32_t)s3;
}

MX_HD inline uint32_t ror32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

inline void expand_key(const uint8_t* key, uint32_t rk[44]) {
  static const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
  for (int i = 0; i < 4; ++i)
    rk[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
            ((uint32_t)key[4 * i + 2] << 8) | (uint32_t)key[4 * i + 3];
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = (t << 8) | (t >> 24);
      t = ((uint32_t)kSbox[t >> 24] << 24) | ((uint32_t)kSbox[(t >> 16) & 255] << 16) |
          ((uint32_t)kSbox[(t >> 8) & 255] << 8) | (uint32_t)kSbox[t & 255];
      t ^= (uint32_t)rcon[i / 4 - 1] << 24;
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

// Portable table-driven block encryption: T is a 256-entry T0 table, S the S-box.
template <typename TT, typename ST>
MX_HD inline void encrypt_block_tt(const uint32_t* rk, const TT& T, const ST& S,
                                   uint32_t in0, uint32_t in1, uint32_t in2, uint32_t in3,
                                   uint32_t out[4]) {
  uint32_t s0 = in0 ^ rk[0], s1 = in1 ^ rk[1], s2 = in2 ^ rk[2], s3 = in3 ^ rk[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t t0 = T[s0 >> 24] ^ ror32(T[(s1 >> 16) & 255], 8) ^ ror32(T[(s2 >> 8) & 255], 16) ^
                  ror32(T[s3 & 255], 24) ^ rk[4 * r];
    uint32_t t1 = T[s1 >> 24] ^ ror32(T[(s2 >> 16) & 255], 8) ^ ror32(T[(s3 >> 8) & 255], 16) ^
                  ror32(T[s0 & 255], 24) ^ rk[4 * r + 1];
    uint32_t t2 = T[s2 >> 24] ^ ror32(T[(s3 >> 16) & 255], 8) ^ ror32(T[(s0 >> 8) & 255], 16) ^
                  ror32(T[s1 & 255], 24) ^ rk[4 * r + 2];
    uint32_t t3 = T[s3 >> 24] ^ ror32(T[(s0 >> 16) & 255], 8) ^ ror32(T[(s1 >> 8) & 255], 16) ^
                  ror32(T[s2 & 255], 24) ^ rk[4 * r + 3];
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
  out[0] = (((uint32_t)S[s0 >> 24] << 24) | ((uint32_t)S[(s1 >> 16) & 255] << 16) |
            ((uint32_t)S[(s2 >> 8) & 255] << 8) | (uint32_t)S[s3 & 255]) ^ rk[40];
  out[1] = (((uint32_t)S[s1 >> 24] << 24) | ((uint32_t)S[(s2 >> 16) & 255] << 16) |
            ((uint32_t)S[(s3 >> 8) & 255] << 8) | (uint32_t)S[s0 & 255]) ^ rk[41];
  out[2] = (((uint32_t)S[s2 >> 24] << 24) | ((uint32_t)S[(s3 >> 16) & 255] << 16) |
            ((uint32_t)S[(s0 >> 8) & 255] << 8) | (uint32_t)S[s1 & 255]) ^ rk[42];
  out[3] = (((uint32_t)S[s3 >> 24] << 24) | ((uint32_t)S[(s0 >> 16) & 255] << 16) |
            ((uint32_t)S[(s1 >> 8) & 255] << 8) | (uint32_t)S[s2 & 255]) ^ rk[43];
}

MX_HD inline uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// CTR input block (nonce_le64 || ctr_le64) as four big-endian words
MX_HD inline void ctr_block_words(uint64_t nonce, uint64_t ctr, uint32_t w[4]) {
  w[0] = bswap32((uint32_t)nonce);
  w[1] = bswap32((uint32_t)(nonce >> 32));
  w[2] = bswap32((uint32_t)ctr);
  w[3] = bswap32((uint32_t)(ctr >> 32));
}

// Output words (big-endian packed) -> little-endian u64 pair (bytes 0..7, 8..15)
MX_HD inline void block_to_u64(const uint32_t o[4], uint64_t* lo, uint64_t* hi) {
  *lo = (uint64_t)bswap32(o[0]) | ((uint64_t)bswap32(o[1]) << 32);
  *hi = (uint64_t)bswap32(o[2]) | ((uint64_t)bswap32(o[3]) << 32);
}

}  // namespace mx
