// The PRF of moosex: ChaCha12 keystream, shared by the host and the gfx950 kernels.
//
// Every seeded draw in the protocols (zero shares, share masks, TruncPr dealer masks, PRF
// expansion of replicated setups) is keystream of PRF(key, nonce): a sequence of 16-byte
// chunks.  The reference's PRG is AES-128-CTR (AES-NI on CPU); on gfx950 an AES round is 16
// data-dependent table lookups, so an AES keystream is bound by LDS bank throughput
// (~49 G blocks/s measured for the replicated-T-table kernels).  ChaCha is add/rotate/xor on
// 32-bit words -- pure VALU, no tables, no LDS -- and one block yields 64 bytes, so the same
// keystream costs a fraction of the issue slots and the PRF-heavy kernels become bound by
// their HBM traffic.  ChaCha12 is the round count of the Rust rand crate's StdRng.
//
// Definition (all words little-endian):
//   state = "expand 16-byte k" constants, key[0..3], key[0..3], blk_lo, blk_hi, nonce_lo,
//           nonce_hi;  block(blk) = state + 12 rounds of ChaCha(state)   (16 words).
//   Chunk c of the stream (words lo64 = w0 | w1 << 32, hi64 = w2 | w3 << 32) is the 16-byte
//   part s = (c >> 6) & 3 of block ((c >> 8) << 6) | (c & 63): the four parts of one block
//   are 64 chunks apart, so a thread that computes block B = (its global index) hands
//   chunks to 64 consecutive lanes -- element accesses stay fully coalesced.
// Element i of a ring with 16-byte elements is chunk i, of 8-byte elements half i & 1 of
// chunk i >> 1, of bits byte (i & 15) & 1 of chunk i >> 4 (as before with AES blocks).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define MX_PRF_HD __host__ __device__
#else
#define MX_PRF_HD
#endif

namespace mx {

constexpr int kPrfRounds = 12;

MX_PRF_HD inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define MX_QR(a, b, c, d)      \
  a += b; d ^= a; d = rotl32(d, 16); \
  c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  \
  c += d; b ^= c; b = rotl32(b, 7);

MX_PRF_HD inline void chacha_block(const uint32_t key[4], uint64_t nonce, uint64_t blk,
                                   uint32_t out[16]) {
  uint32_t x0 = 0x61707865u, x1 = 0x3120646eu, x2 = 0x79622d36u, x3 = 0x6b206574u;
  uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
  uint32_t x8 = key[0], x9 = key[1], x10 = key[2], x11 = key[3];
  uint32_t x12 = (uint32_t)blk, x13 = (uint32_t)(blk >> 32);
  uint32_t x14 = (uint32_t)nonce, x15 = (uint32_t)(nonce >> 32);
  for (int r = 0; r < kPrfRounds; r += 2) {
    MX_QR(x0, x4, x8, x12)
    MX_QR(x1, x5, x9, x13)
    MX_QR(x2, x6, x10, x14)
    MX_QR(x3, x7, x11, x15)
    MX_QR(x0, x5, x10, x15)
    MX_QR(x1, x6, x11, x12)
    MX_QR(x2, x7, x8, x13)
    MX_QR(x3, x4, x9, x14)
  }
  out[0] = x0 + 0x61707865u;
  out[1] = x1 + 0x3120646eu;
  out[2] = x2 + 0x79622d36u;
  out[3] = x3 + 0x6b206574u;
  out[4] = x4 + key[0];
  out[5] = x5 + key[1];
  out[6] = x6 + key[2];
  out[7] = x7 + key[3];
  out[8] = x8 + key[0];
  out[9] = x9 + key[1];
  out[10] = x10 + key[2];
  out[11] = x11 + key[3];
  out[12] = x12 + (uint32_t)blk;
  out[13] = x13 + (uint32_t)(blk >> 32);
  out[14] = x14 + (uint32_t)nonce;
  out[15] = x15 + (uint32_t)(nonce >> 32);
}
#undef MX_QR

// chunk c <-> (block, part)
MX_PRF_HD inline uint64_t ks_block_of(uint64_t c) { return ((c >> 8) << 6) | (c & 63); }
MX_PRF_HD inline int ks_part_of(uint64_t c) { return (int)((c >> 6) & 3); }
MX_PRF_HD inline uint64_t ks_chunk(uint64_t blk, int part) {
  return ((blk >> 6) << 8) | ((uint64_t)part << 6) | (blk & 63);
}
// blocks to walk for chunks [0, nchunks): whole groups of 64 blocks
MX_PRF_HD inline uint64_t ks_blocks_for(uint64_t nchunks) { return ((nchunks + 255) >> 8) << 6; }

MX_PRF_HD inline void part_u64(const uint32_t w[16], int part, uint64_t* lo, uint64_t* hi) {
  *lo = (uint64_t)w[4 * part] | ((uint64_t)w[4 * part + 1] << 32);
  *hi = (uint64_t)w[4 * part + 2] | ((uint64_t)w[4 * part + 3] << 32);
}

// one chunk by random access (computes its whole block)
MX_PRF_HD inline void prf_chunk(const uint32_t key[4], uint64_t nonce, uint64_t c, uint64_t* lo,
                                uint64_t* hi) {
  uint32_t w[16];
  chacha_block(key, nonce, ks_block_of(c), w);
  part_u64(w, ks_part_of(c), lo, hi);
}

inline void key_words(const uint8_t* key16, uint32_t k[4]) { memcpy(k, key16, 16); }

}  // namespace mx
