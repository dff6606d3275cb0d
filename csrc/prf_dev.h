// Device-side PRF helpers shared by the gfx950 translation units (keystream definition in
// prf_core.h).  Throughput kernels walk the keystream one ChaCha block per thread and get
// the block's four 16-byte chunks for four element groups 64 chunks apart (walk_chunks);
// latency kernels that need an arbitrary chunk use prf_chunk.
#pragma once
#include <hip/hip_runtime.h>
#include <string.h>

#include "prf_core.h"

namespace mxd {

constexpr int kKeyWords = 4;  // a PRF key: 128 bits

struct Keys4 {
  uint32_t k[4][kKeyWords];
};

// elements of type T per 16-byte keystream chunk
template <class T>
struct Lane {
  static constexpr int kPer = 16 / (int)sizeof(T);
};

template <class T>
__device__ inline T pick(uint64_t lo, uint64_t hi, int j) {
  if constexpr (sizeof(T) == 16) {
    return ((T)hi << 64) | (T)lo;
  } else if constexpr (sizeof(T) == 8) {
    return j == 0 ? lo : hi;
  } else {
    uint64_t w = j < 8 ? lo : hi;
    return (T)((w >> (8 * (j & 7))) & 1);
  }
}

inline Keys4 load_keys(const uint8_t* keys16, int nkeys) {
  Keys4 k;
  memset(&k, 0, sizeof(k));
  for (int i = 0; i < nkeys && i < 4; ++i) mx::key_words(keys16 + 16 * i, k.k[i]);
  return k;
}

// PRF key source of a launch: raw keys passed by value, or pointers to key slots in device
// memory (MX_KEY_SLOT_WORDS words, raw key in words 0..3).  Slots keep the keys out of the
// launch parameters, so a captured hipGraph replays with whatever keys the slots hold at
// replay time (fresh per evaluation).
constexpr int kMaxKeySlots = 6;  // pairs mode: (k_p, k_p') for up to 3 parties
struct KeySrc {
  Keys4 k;
  const uint32_t* slot[kMaxKeySlots];
};

inline KeySrc keysrc_host(const uint8_t* keys16, int nkeys) {
  KeySrc s;
  s.k = load_keys(keys16, nkeys);
  for (int i = 0; i < kMaxKeySlots; ++i) s.slot[i] = nullptr;
  return s;
}

inline KeySrc keysrc_slots(const uint32_t* const* slots, int nkeys) {
  KeySrc s;
  memset(&s.k, 0, sizeof(s.k));
  for (int i = 0; i < kMaxKeySlots; ++i) s.slot[i] = i < nkeys ? slots[i] : nullptr;
  return s;
}

// Copy nkeys raw keys into LDS, then a barrier.
__device__ inline void stage_keys(uint32_t (*rks)[kKeyWords], const KeySrc& src, int nkeys) {
  for (int i = threadIdx.x; i < nkeys * kKeyWords; i += blockDim.x) {
    const int q = i / kKeyWords, w = i - q * kKeyWords;
    rks[q][w] = src.slot[q] ? src.slot[q][w] : (q < 4 ? src.k.k[q][w] : 0u);
  }
  __syncthreads();
}

// Walk the chunks [0, nchunks) of NS keystreams (key[q], nonce[q]): per thread, one ChaCha
// block of every stream per iteration, then body(chunk, lo[NS], hi[NS]) for the block's
// chunks in increasing order.  The grid stride is a multiple of 64, so lane l of a wave owns
// chunks = l (mod 64) and the body's element accesses are coalesced.
template <int NS, class Body>
__device__ inline void walk_chunks(int64_t nchunks, const uint32_t* const (&key)[NS],
                                   const uint64_t (&nonce)[NS], Body&& body) {
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)nchunks);
  for (int64_t B = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; B < nblk;
       B += (int64_t)gridDim.x * blockDim.x) {
    uint32_t w[NS][16];
#pragma unroll
    for (int q = 0; q < NS; ++q) mx::chacha_block(key[q], nonce[q], (uint64_t)B, w[q]);
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int64_t c = (int64_t)mx::ks_chunk((uint64_t)B, part);
      if (c >= nchunks) break;
      uint64_t lo[NS], hi[NS];
#pragma unroll
      for (int q = 0; q < NS; ++q) mx::part_u64(w[q], part, &lo[q], &hi[q]);
      body(c, lo, hi);
    }
  }
}

__device__ inline void prf_chunk(const uint32_t* key, uint64_t nonce, uint64_t c, uint64_t* lo,
                                 uint64_t* hi) {
  mx::prf_chunk(key, nonce, c, lo, hi);
}

inline int grid_for(int64_t n, int block = 256) {
  int64_t blocks = (n + block - 1) / block;
  if (blocks < 1) blocks = 1;
  if (blocks > 256 * 8) blocks = 256 * 8;
  return (int)blocks;
}

// grid for a walk over nchunks keystream chunks (one thread per ChaCha block)
inline int grid_for_chunks(int64_t nchunks) {
  return grid_for((int64_t)mx::ks_blocks_for((uint64_t)nchunks));
}

}  // namespace mxd
