// Device-side AES-128-CTR helpers shared by the gfx950 translation units.
//
// Each block stages the T0 table into LDS once (replicated for conflict-free lookups, see
// kTTWords); T1..T3 are byte rotations of T0.  A keystream block yields one u128, two u64 or sixteen bits.
#pragma once
#include <hip/hip_runtime.h>
#include <string.h>

#include "aes_core.h"

namespace mxd {

static __constant__ uint8_t c_sbox[256] = MX_SBOX_INIT;

struct RK {
  uint32_t rk[44];
};
struct Keys4 {
  uint32_t rk[4][44];
};

// The T0 table is replicated 32 times in LDS, word i*32 + c for copy c: lane L of a
// 32-lane ds_read_b32 group reads copy L & 31, so the 32 lanes of a group always hit 32
// different banks ((a/4) mod 32 = c) -- random table lookups are bank-conflict free.
// The S-box (last round) is byte 2 of T0.  32 KB of LDS per block.
constexpr int kTTWords = 256 * 32;

struct TRep {
  const uint32_t* b;
  int c;
  __device__ uint32_t operator[](uint32_t i) const { return b[i * 32 + c]; }
};
struct SRep {
  TRep t;
  __device__ uint8_t operator[](uint32_t i) const { return (uint8_t)(t[i] >> 16); }
};

__device__ inline void stage_tables_rep(uint32_t* T) {
  for (int i = threadIdx.x; i < kTTWords; i += blockDim.x) T[i] = mx::t0_entry(c_sbox[i >> 5]);
  __syncthreads();
}

__device__ inline void aes_ctr_rep(const uint32_t* rk, const uint32_t* T, uint64_t nonce,
                                   uint64_t ctr, uint64_t* lo, uint64_t* hi) {
  uint32_t w[4], o[4];
  mx::ctr_block_words(nonce, ctr, w);
  const TRep tr{T, (int)(threadIdx.x & 31)};
  mx::encrypt_block_tt(rk, tr, SRep{tr}, w[0], w[1], w[2], w[3], o);
  mx::block_to_u64(o, lo, hi);
}

// Compact variant (1.25 KB: one T0 copy + S-box) for latency-bound launches that run one
// AES per thread, where staging 32 KB would cost more than the bank conflicts.
__device__ inline void stage_tables(uint32_t* T, uint8_t* Sb) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint8_t s = c_sbox[i];
    Sb[i] = s;
    T[i] = mx::t0_entry(s);
  }
  __syncthreads();
}

__device__ inline void aes_ctr(const uint32_t* rk, const uint32_t* T, const uint8_t* Sb,
                               uint64_t nonce, uint64_t ctr, uint64_t* lo, uint64_t* hi) {
  uint32_t w[4], o[4];
  mx::ctr_block_words(nonce, ctr, w);
  mx::encrypt_block_tt(rk, T, Sb, w[0], w[1], w[2], w[3], o);
  mx::block_to_u64(o, lo, hi);
}

// elements of type T per AES block
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
  for (int i = 0; i < nkeys && i < 4; ++i) mx::expand_key(keys16 + 16 * i, k.rk[i]);
  return k;
}

// PRF key source of a launch: expanded schedules passed by value, or pointers to key
// slots in device memory (MX_KEY_SLOT_WORDS words: raw key in words 0..3, schedule in
// 4..47).  Slots keep the keys out of the launch parameters, so a captured hipGraph
// replays with whatever keys the slots hold at replay time (fresh per evaluation).
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

// Copy nkeys schedules into LDS.  Call before stage_tables: its barrier publishes them.
__device__ inline void stage_keys(uint32_t (*rks)[44], const KeySrc& src, int nkeys) {
  for (int i = threadIdx.x; i < nkeys * 44; i += blockDim.x) {
    const int q = i / 44, w = i - q * 44;
    rks[q][w] = src.slot[q] ? src.slot[q][4 + w] : (q < 4 ? src.k.rk[q][w] : 0u);
  }
}

inline int grid_for(int64_t n, int block = 256) {
  int64_t blocks = (n + block - 1) / block;
  if (blocks < 1) blocks = 1;
  if (blocks > 256 * 8) blocks = 256 * 8;
  return (int)blocks;
}

}  // namespace mxd
