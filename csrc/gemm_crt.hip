// Exact ring GEMM over Z_2^64 / Z_2^128 by multi-modular (CRT) int8 MFMA products.
//
// The limb GEMM (gemm_mfma.hip) splits every ring element into L 8-bit limbs and needs the
// L(L+1)/2 limb-pair products on or below the anti-diagonal: 136 int8 GEMMs for Z_2^128,
// 36 for Z_2^64.  Here the exact INTEGER product is computed instead, in residues:
//
//   * every ring element x is read as its signed representative X in [-2^(w-1), 2^(w-1));
//     the integer product Z = sum_k X_k Y_k then satisfies |Z| <= K' 2^(2w-2);
//   * n pairwise-coprime moduli p_i <= 256 (256, 253, 251, 249, ...) with product
//     M > |Z| / 0.45 are chosen -- 36 for Z_2^128 at K' = 8192, 18 for Z_2^64;
//   * each operand is reduced to centered int8 residues (prep kernels, one udot4 per 4 bytes
//     of the element + one fp32 rounding), and ONE int8 GEMM per modulus gives
//     acc_i = Z mod p_i exactly in i32 (K' <= 2^15 keeps the epilogue's fp32 rounding exact);
//   * the CRT reconstruction  Z = sum_i c_i (M/p_i) - q M,  c_i = Z (M/p_i)^-1 mod p_i,
//     q = round(sum_i c_i / p_i), is evaluated mod 2^w:  z = sum_i c_i W_i - q (M mod 2^w)
//     with W_i = (M/p_i) mod 2^w.  The inverse (M/p_i)^-1 is folded into A's residues, so
//     the GEMM epilogue only reduces acc_i mod p_i (centered, stored as one byte).
//
// So a Z_2^128 product costs 36 int8 GEMMs instead of 136 (3.8x fewer MFMAs), Z_2^64 18
// instead of 36, at the price of wider operand prep and one reconstruction pass.  (The same
// idea as the Ozaki-II / multi-modular emulation of high-precision GEMM on integer matrix
// units; here the target is modular rather than floating-point arithmetic.)
//
// Kernels:
//   k_crt_prep<T, TRANS>  operand -> n residue planes in a blocked, swizzled int8 image
//                         [g = batch*n + i][tile][k-step][256 rows][64 bytes] (one 16 KB
//                         image per (tile, k-step), LDS-DMA ready, ds_read_b128 conflict free)
//   k_crt_gemm            256x256 block tile, 8 waves (2 per SIMD) of 128x64, K-step 64,
//                         3-stage LDS-DMA ring, one barrier per step; epilogue reduces the
//                         i32 accumulators mod p_i and stores one byte per output element in
//                         MFMA register order (16 B per lane per 32x32 block)
//   k_crt_recon<T>        n residue bytes per element -> ring element (sum c_i W_i - q Mw),
//                         optionally accumulated into C
// Mode 1 (RSS cross GEMM, as in gemm_mfma.hip): A' = [A0 | A1], B' = [B0 + B1 ; B0].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "hip_attr.h"
#include "moosex.h"

void mx_ws_note(int dev, int64_t want, bool ok);  // gemm_mfma.hip: workspace bookkeeping
bool mx_ws_malloc(void** p, int64_t bytes);       // gemm_mfma.hip: allocation (capture-safe)
void mx_ws_shared_note(void);

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kMaxMod = 48;
// pairwise coprime, descending: 2^8, 3*5*17, 11*23, 13*19, primes, 7*31, primes
// Pairwise coprime, in the order they are used (a call takes the shortest prefix whose
// product is large enough).  The first 36 are the product-maximising set of 36 coprime
// integers <= 256 (exhaustive branch-and-bound over 61..256): 268.2 bits, just enough for an
// exact Z_2^128 product at K' = 8192 (268.15 bits), where the greedy descending set
// (256, 255, 253, ...) needs 37.  Their first 18 also cover Z_2^64 at K' = 8192.
constexpr int kModuli[kMaxMod] = {256, 253, 251, 249, 247, 241, 239, 235, 233, 229, 227, 223,
                                  217, 211, 199, 197, 193, 191, 181, 179, 173, 167, 163, 157,
                                  151, 149, 139, 137, 131, 127, 113, 109, 107, 103, 101, 97,
                                  89,  79,  73,  71,  67,  61,  59,  53,  43,  41,  37,  17};

constexpr int BM = 256;          // block tile rows (A side); the cols BN are 256 or 128
constexpr int BK = 64;           // k bytes per stage
constexpr int kImg = BM * BK;    // one A operand image per (tile, k-step): 16 KB
constexpr int kStages = 3;       // LDS ring depth

// byte offset of 16-byte chunk c (0..3) of image row r: chunks XOR-swizzled by
// f((r >> 2) & 3), f = [0, 2, 3, 1], so that the 16 lanes of each ds_read_b128 lane group hit
// 16 distinct 16-byte bank slots both for the 32x32x32 fragments (lane l: row l & 31, one
// chunk per half-wave) and for the 16x16x64 fragments (lane l: row l & 15, chunk l >> 4).
__device__ __host__ inline int swz(int q) { return (0x78 >> (2 * (q & 3))) & 3; }
__device__ __host__ inline int img_off(int r, int c) { return r * BK + 16 * (c ^ swz(r >> 2)); }

// --- tables ---------------------------------------------------------------------------------
struct PrepTab {  // operand residues
  int n;
  int p[kMaxMod];
  float rcp[kMaxMod];
  uint32_t w[kMaxMod][4];  // weight of byte j of the element = byte j%4 of word j/4
  uint32_t neg[kMaxMod];   // added when the element is negative: (p - 2^w mod p) [* inv] mod p
  uint32_t mul0;           // p = 256: residue = (byte0 * mul0) mod 256
};
struct EpiTab {  // GEMM epilogue
  int n;
  int p[kMaxMod];
  float pf[kMaxMod];
  float rcp[kMaxMod];
  int t16[kMaxMod];  // 2^16 mod p
};
struct RecTab {  // reconstruction
  int n;
  float rcp[kMaxMod];
  uint16_t W[kMaxMod][8];  // (M / p_i) mod 2^w, 16-bit words
  uint16_t Mw[8];          // M mod 2^w
};

// Reconstruction by v_dot4_i32_i8 over groups of 4 moduli: W_i and R_i = round(2^24 / p_i)
// as signed base-256 digits, packed per (group, digit) with modulus 4g + u in byte u, so one
// dot4 of an element's 4 residues with one (uniform, SGPR) word adds that digit's 4 terms.
struct RecTab4 {
  int groups;
  uint32_t wd[kMaxMod / 4][16];
  uint32_t rd[kMaxMod / 4][3];
};

struct Tables {
  int words = 0, n = 0;
  PrepTab pa, pb;
  EpiTab ep;
  RecTab rc;
  RecTab4 r4;
};

int modinv(int a, int m) {
  int t = 0, nt = 1, r = m, nr = ((a % m) + m) % m;
  while (nr) {
    int q = r / nr, x;
    x = t - q * nt; t = nt; nt = x;
    x = r - q * nr; r = nr; nr = x;
  }
  return r == 1 ? (t % m + m) % m : -1;
}

// smallest n with prod p_i >= |Z|max / 0.45, |Z| <= K' 2^(2w-2)
int moduli_needed(int words, int64_t kprime) {
  const double need = 2.0 * 64 * words - 2 + std::log2((double)std::max<int64_t>(kprime, 1)) +
                      std::log2(1 / 0.45);
  double have = 0;
  for (int i = 0; i < kMaxMod; ++i) {
    have += std::log2((double)kModuli[i]);
    if (have >= need) return i + 1;
  }
  return -1;
}

void build_tables(int words, int n, Tables& t) {
  t.words = words;
  t.n = n;
  const int wbits = 64 * words;
  const int nbytes = 8 * words;
  u128 Mw = 1;
  for (int i = 0; i < n; ++i) Mw *= (u128)kModuli[i];
  if (words == 1) Mw &= ~(u64)0;
  std::memset(&t.pa, 0, sizeof t.pa);
  std::memset(&t.pb, 0, sizeof t.pb);
  std::memset(&t.ep, 0, sizeof t.ep);
  std::memset(&t.rc, 0, sizeof t.rc);
  t.pa.n = t.pb.n = t.ep.n = t.rc.n = n;
  for (int i = 0; i < n; ++i) {
    const int p = kModuli[i];
    u128 W = 1;
    int rest = 1;  // (M / p) mod p
    for (int j = 0; j < n; ++j)
      if (j != i) {
        W *= (u128)kModuli[j];
        rest = (int)((int64_t)rest * kModuli[j] % p);
      }
    const int inv = modinv(rest, p);
    for (int k = 0; k < 8; ++k) t.rc.W[i][k] = (uint16_t)(W >> (16 * k));
    t.rc.rcp[i] = 1.0f / (float)p;
    t.ep.p[i] = p;
    t.ep.pf[i] = (float)p;
    t.ep.rcp[i] = 1.0f / (float)p;
    t.ep.t16[i] = (int)((1 << 16) % p);
    t.pa.p[i] = t.pb.p[i] = p;
    t.pa.rcp[i] = t.pb.rcp[i] = 1.0f / (float)p;
    int pw = 1 % p;  // 256^j mod p
    for (int j = 0; j < nbytes; ++j) {
      const int wb = pw, wa = (int)((int64_t)pw * inv % p);
      t.pb.w[i][j / 4] |= (uint32_t)wb << (8 * (j % 4));
      t.pa.w[i][j / 4] |= (uint32_t)wa << (8 * (j % 4));
      pw = pw * 256 % p;
    }
    // pw = 2^w mod p now; element negative => subtract 2^w, i.e. add p - 2^w mod p
    const int negb = (p - pw) % p;
    t.pb.neg[i] = (uint32_t)negb;
    t.pa.neg[i] = (uint32_t)((int64_t)negb * inv % p);
    if (i == 0) {
      t.pa.mul0 = (uint32_t)inv;
      t.pb.mul0 = 1;
    }
  }
  for (int k = 0; k < 8; ++k) t.rc.Mw[k] = (uint16_t)(Mw >> (16 * k));
  std::memset(&t.r4, 0, sizeof t.r4);
  t.r4.groups = (n + 3) / 4;
  for (int i = 0; i < n; ++i) {
    u128 W = 0;
    for (int k = 0; k < 8; ++k) W |= (u128)t.rc.W[i][k] << (16 * k);
    int carry = 0;
    for (int d = 0; d < nbytes; ++d) {  // W mod 2^w in signed digits (carry out dropped)
      int b = (int)((W >> (8 * d)) & 0xff) + carry;
      carry = b >= 128;
      b -= 256 * carry;
      t.r4.wd[i / 4][d] |= (uint32_t)(uint8_t)(int8_t)b << (8 * (i % 4));
    }
    int R = (int)std::lround(16777216.0 / kModuli[i]);
    for (int d = 0; d < 3; ++d) {  // R < 2^24: exact in three signed digits
      int b = (R & 0xff);
      R >>= 8;
      if (b >= 128) {
        b -= 256;
        R += 1;
      }
      t.r4.rd[i / 4][d] |= (uint32_t)(uint8_t)(int8_t)b << (8 * (i % 4));
    }
  }
  (void)wbits;
}

const Tables& tables_for(int words, int n) {
  static std::mutex mu;
  static Tables cache[3][kMaxMod + 1];
  std::lock_guard<std::mutex> lk(mu);
  Tables& t = cache[words][n];
  if (t.n != n || t.words != words) build_tables(words, n, t);
  return t;
}

// --- device helpers ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
  const uint32_t lo = __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm((uint32_t)d, (uint32_t)c, 0x0c0c0400u);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

template <class T>
struct Words;
template <>
struct Words<u64> {
  static constexpr int N = 2;
};
template <>
struct Words<u128> {
  static constexpr int N = 4;
};

// centered residue of the signed element whose little-endian 32-bit words are x[0..NW-1]
template <int NW>
__device__ __forceinline__ int residue(const uint32_t (&x)[NW], const uint32_t (&w)[4],
                                       uint32_t neg, float p, float rcp) {
  uint32_t s = (x[NW - 1] >> 31) * neg;
#pragma unroll
  for (int q = 0; q < NW; ++q) s = __builtin_amdgcn_udot4(x[q], w[q], s, false);
  const float fs = (float)s;  // < 2^20: exact
  const float qt = __builtin_rintf(fs * rcp);  // p odd: s/p is never within 1/(2p) of k + 1/2
  return (int)__builtin_fmaf(-qt, p, fs);      // in [-(p-1)/2, (p-1)/2]
}

// Two residues at once: the fp32 scaling and the multiply-subtract as packed instructions
// (v_pk_mul_f32, v_pk_fma_f32: one issue for both elements); the same values as residue().
typedef float f2 __attribute__((ext_vector_type(2)));
template <int NW>
__device__ __forceinline__ void residue2(const uint32_t (&xa)[NW], const uint32_t (&xb)[NW],
                                         const uint32_t (&w)[4], uint32_t neg, float p,
                                         float rcp, int& ra, int& rb) {
  uint32_t sa = 0, sb = 0;
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    sa = __builtin_amdgcn_udot4(xa[q], w[q], sa, false);
    sb = __builtin_amdgcn_udot4(xb[q], w[q], sb, false);
  }
  // the negative-element correction as one packed fma (the signs are per element, hoisted
  // out of the modulus loop): exact, the sum stays below 2^21
  const f2 sg = {(float)(xa[NW - 1] >> 31), (float)(xb[NW - 1] >> 31)};
  const float nf = (float)neg;
  const f2 fs = __builtin_elementwise_fma(sg, (f2){nf, nf}, (f2){(float)sa, (float)sb});
  f2 qt = fs * (f2){rcp, rcp};
  qt.x = __builtin_rintf(qt.x);
  qt.y = __builtin_rintf(qt.y);
  const f2 r = __builtin_elementwise_fma(-qt, (f2){p, p}, fs);
  ra = (int)r.x;
  rb = (int)r.y;
}

// One thread = (tile, k-step, image row r, 16-byte chunk c) of every residue plane.
// TRANS = false: A' rows are M rows of A0 (mode 0), [A0 | A1] (mode 1) or A0 + A1 (mode 2)
// (row-major [R][K] per batch, batch stride xs elements).  TRANS = true: B' rows are the N
// columns ([K][R]) of B0 (mode 0), [B0 + B1 ; B0] (1), [B0 ; B1] (2) or B0 + B1 (3).
// nkb k-steps are generated; the image is laid out with nkb_s k-steps per tile (>= nkb: a
// shorter operand placed in a longer operand's slot).
// src.n > 0: batch entry b takes its operands and mode from src instead (one launch for a
// set of images of different forms, e.g. run_crt_asym's sums beside plain shares).
// dual[b] != 0 (mode 0 only): the thread then adds x1 to the elements it holds and writes
// the sum's image too, at byte offset dual[b] from entry b's own image -- a share's image
// and the image of its sum with the next share from one read of the share.
struct PrepSrcs {
  int n = 0;
  int mode[6];
  const void* x0[6];
  const void* x1[6];
  int64_t dual[6];
};

template <class T, bool TRANS, int ROWS, bool PK = true>
__global__ void __launch_bounds__(256)
    k_crt_prep(const T* __restrict__ X0, const T* __restrict__ X1, int64_t R, int64_t K,
               int64_t xs, int mode_all, int8_t* __restrict__ out, int64_t tiles, int64_t nkb,
               int64_t nkb_s, const PrepTab tab, const PrepSrcs src) {
  constexpr int NW = Words<T>::N;
  const int64_t total = tiles * nkb * (ROWS * 4);
  const int64_t b = blockIdx.y;
  const int mode = src.n > 0 ? src.mode[b] : mode_all;
  const T* x0 = src.n > 0 ? (const T*)src.x0[b] : X0 + b * xs;
  const T* x1 = src.n > 0 ? (const T*)src.x1[b] : (mode ? X1 + b * xs : x0);
  const int n = tab.n;
  const int64_t plane = tiles * nkb_s * (int64_t)(ROWS * BK);
  int8_t* ob = out + b * n * plane;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(g & 3);
    const int r = (int)((g >> 2) & (ROWS - 1));
    const int64_t q = g / (ROWS * 4);
    const int64_t kb = q % nkb, t = q / nkb;
    const int64_t row = t * ROWS + r;
    const int64_t k0 = kb * BK + c * 16;
    uint32_t v[16][NW];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t k = k0 + j;
      T e = 0;
      if (row < R) {
        if (!TRANS) {
          if (k < K) e = mode == 2 ? (T)(x0[row * K + k] + x1[row * K + k]) : x0[row * K + k];
          else if (mode == 1 && k < 2 * K) e = x1[row * K + (k - K)];
        } else {
          if (k < K)
            e = (mode & 1) ? (T)(x0[k * R + row] + x1[k * R + row]) : x0[k * R + row];
          else if (mode == 1 && k < 2 * K) e = x0[(k - K) * R + row];
          else if (mode == 2 && k < 2 * K) e = x1[(k - K) * R + row];
        }
      }
#pragma unroll
      for (int w = 0; w < NW; ++w) v[j][w] = (uint32_t)(e >> (32 * w));
    }
    const int64_t boff = (t * nkb_s + kb) * (int64_t)(ROWS * BK) + img_off(r, c);
    auto emit = [&](int8_t* base) __attribute__((always_inline)) {
    {  // p = 256: the low byte (times the folded inverse)
      int rr[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) rr[j] = (int)(v[j][0] * tab.mul0);
      v4i o;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = (int)pack4(rr[4 * u], rr[4 * u + 1], rr[4 * u + 2], rr[4 * u + 3]);
      *(v4i*)base = o;
    }
    for (int i = 1; i < n; ++i) {
      const uint32_t w[4] = {tab.w[i][0], tab.w[i][1], tab.w[i][2], tab.w[i][3]};
      const uint32_t neg = tab.neg[i];
      const float p = (float)tab.p[i], rcp = tab.rcp[i];
      int rr[16];
      if constexpr (PK) {
#pragma unroll
        for (int j = 0; j < 16; j += 2)
          residue2<NW>(v[j], v[j + 1], w, neg, p, rcp, rr[j], rr[j + 1]);
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) rr[j] = residue<NW>(v[j], w, neg, p, rcp);
      }
      v4i o;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = (int)pack4(rr[4 * u], rr[4 * u + 1], rr[4 * u + 2], rr[4 * u + 3]);
      *(v4i*)(base + i * plane) = o;
    }
    };
    emit(ob + boff);
    if (src.n > 0 && src.dual[b]) {  // + x1: the sum's image from the same read of x0
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int64_t k = k0 + j;
        if (row < R && k < K) {
          T e = 0;
#pragma unroll
          for (int w = 0; w < NW; ++w) e |= (T)v[j][w] << (32 * w);
          e += TRANS ? x1[k * R + row] : x1[row * K + k];
#pragma unroll
          for (int w = 0; w < NW; ++w) v[j][w] = (uint32_t)(e >> (32 * w));
        }
      }
      emit(ob + src.dual[b] + boff);
    }
  }
}

// o = a + b over n ring elements (run_crt_asym's party-0 A' sum, written once so that its
// residue image streams one operand: the two-operand prep ran at ~2.4 plain images)
template <class T>
__global__ void __launch_bounds__(256)
    k_add_pair(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ o, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    o[i] = a[i] + b[i];
}

// XCD-aware remap (as gemm_mfma.hip): consecutive tile ids land on one XCD
__device__ inline int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8;
  const int64_t x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// s_waitcnt vmcnt(N) lgkmcnt(0) expcnt(7), gfx9 encoding (vmcnt split 4 + 2 bits)
constexpr int waitcnt_vm_lgkm0(int vm) { return (vm & 15) | ((vm >> 4) << 14) | (7 << 4); }

__device__ __forceinline__ int centered_mod(int acc, float pf, float rcp, int t16) {
  // acc = hi 2^16 + lo; s = hi (2^16 mod p) + lo is exact in fp32 (|s| < 2^24)
  const int hi = acc >> 16, lo = acc & 0xffff;
  const int s = __mul24(hi, t16) + lo;
  const float fs = (float)s;
  const float qt = __builtin_rintf(fs * rcp);
  return (int)__builtin_fmaf(-qt, pf, fs);
}

// WR x WC waves per 256x256 block tile; wave tile (256/WR) x (256/WC) = MI x NJ MFMA
// blocks of 32x32.  <2,2>: 4 waves of 128x128 (256 accumulator registers, one wave per
// SIMD); <2,4>: 8 waves of 128x64 (128 accumulators, two waves per SIMD, so one wave's
// LDS reads, address arithmetic and barrier waits hide behind its partner's MFMAs).
template <int WR, int WC, int BN, int MINW>
__global__ void __launch_bounds__(64 * WR * WC, MINW)
    k_crt_gemm(const int8_t* __restrict__ RA, const int8_t* __restrict__ RB,
               int8_t* __restrict__ CR, int tiles_m, int tiles_n, int nkb, int gM,
               const EpiTab ep, int dma_mask, int bcast) {
  constexpr int NW = WR * WC;
  constexpr int MI = BM / WR / 32, NJ = BN / WC / 32;
  constexpr int kImgB = BN * BK;                 // one B image per (tile, k-step)
  constexpr int kStageBytes = kImg + kImgB;
  constexpr int NPIECE = kStageBytes / 1024;     // 1 KB LDS-DMA pieces per stage
  constexpr int PPW = NPIECE / NW;               // DMA pieces per wave per stage
  static_assert(PPW * NW == NPIECE, "stage pieces must split evenly over the waves");
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int ntiles = tiles_m * tiles_n;
  const int tid_flat = (int)xcd_remap(blockIdx.x, ntiles);
  const int group = tid_flat / (gM * tiles_n);
  const int first_m = group * gM;
  const int gm = tiles_m - first_m < gM ? tiles_m - first_m : gM;
  const int in_group = tid_flat % (gM * tiles_n);
  const int tm = first_m + in_group % gm, tn = in_group / gm;
  const int g = blockIdx.y;  // batch * n + modulus
  const int mi = g % ep.n;
  // bcast bit 0 / 1: A / B residues were prepared once for every batch entry
  const int8_t* ga = RA + ((int64_t)((bcast & 1) ? mi : g) * tiles_m + tm) * nkb * (int64_t)kImg;
  const int8_t* gb = RB + ((int64_t)((bcast & 2) ? mi : g) * tiles_n + tn) * nkb * (int64_t)kImgB;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int half = lane >> 5;
  const int sw = swz(lane >> 2);  // row swizzle of every fragment row this lane reads
  const int rowa = (wr * (BM / WR) + (lane & 31)) * BK;
  const int rowb = kImg + (wc * (BN / WC) + (lane & 31)) * BK;
  const int co0 = 16 * (half ^ sw), co1 = 16 * ((2 + half) ^ sw);

  // wave w issues pieces w, w + NW, .. of the NPIECE 1-KB pieces of a stage (16 A, then
  // BN / 16 B); the sources advance by one image per k-step
  const int8_t* srcs[PPW];
  int dsts[PPW], steps[PPW];
#pragma unroll
  for (int t = 0; t < PPW; ++t) {
    const int pc = wave + NW * t;
    const bool is_b = pc >= 16;
    const int pp = is_b ? pc - 16 : pc;
    srcs[t] = (is_b ? gb : ga) + pp * 1024 + lane * 16;
    dsts[t] = (is_b ? kImg : 0) + pp * 1024;
    steps[t] = is_b ? kImgB : kImg;
  }
  auto dma = [&](int kb, int t, int8_t* dst_stage) {
    if (!((dma_mask >> (wave + NW * t >= 16 ? 1 : 0)) & 1)) return;  // timing experiments only
    __builtin_amdgcn_global_load_lds((const void*)(srcs[t] + (int64_t)kb * steps[t]),
                                     (__attribute__((address_space(3))) void*)(dst_stage + dsts[t]),
                                     16, 0, 0);
  };

  v16i acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v16i{0};

  v4i fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
  auto frags = [&](const int8_t* st, int co, v4i(&fa)[MI], v4i(&fb)[NJ]) {
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *(const v4i*)(st + rowa + i * 32 * BK + co);
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb[j] = *(const v4i*)(st + rowb + j * 32 * BK + co);
  };

  // prologue: stages 0, 1, 2 in flight; wait for stage 0
#pragma unroll
  for (int s = 0; s < kStages; ++s)
#pragma unroll
    for (int t = 0; t < PPW; ++t) dma(s < nkb ? s : nkb - 1, t, smem + s * kStageBytes);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(2 * PPW));
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  frags(smem, co0, fa0, fb0);
  if (dma_mask & 8) frags(smem, co1, fa1, fb1);

  int8_t* cur = smem;                    // stage kb
  int8_t* nxt = smem + kStageBytes;      // stage kb + 1
  int8_t* nn = smem + 2 * kStageBytes;   // stage kb + 2
  for (int kb = 0; kb < nkb; ++kb) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0[i], fb0[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (i == 0 && j == 1 && !(dma_mask & 8)) {  // second-half fragments, behind the
          frags(cur, co1, fa1, fb1);  // first MFMAs (the compiler waits for all LDS reads
          __builtin_amdgcn_sched_barrier(0);  // before an MFMA that follows any of them)
        }
      }
    // my DMA of stage kb+1 landed (only stage kb+2's pieces may be outstanding) and my
    // reads of stage kb are done; after the barrier, everyone's are
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(PPW));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (!(dma_mask & 8)) frags(nxt, co0, fa0, fb0);  // past the end: stale, never used
    __builtin_amdgcn_sched_barrier(0);
    const int kn = kb + kStages < nkb ? kb + kStages : nkb - 1;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // this wave's PPW pieces of stage kb+3 into the freed buffer, spread over the
        // MI * NJ MFMAs: piece t after MFMA floor((t + 1) MI NJ / PPW) - 1
        const int m = i * NJ + j;
#pragma unroll
        for (int t = 0; t < PPW; ++t)
          if (m == (t + 1) * MI * NJ / PPW - 1) {
            dma(kn, t, cur);
            __builtin_amdgcn_sched_barrier(0);
          }
      }
    int8_t* t = cur;
    cur = nxt;
    nxt = nn;
    nn = t;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: centered acc mod p, one byte per element, MFMA register order; 32x32 block
  // (bi, bj) of the tile at byte ((bi * BN / 32 + bj) * 64 + lane) * 16 of the tile's bytes
  const float pf = ep.pf[mi], rcp = ep.rcp[mi];
  const int t16 = ep.t16[mi];
  int8_t* cr = CR + ((int64_t)g * ntiles + tm * tiles_n + tn) * (int64_t)(BM * BN);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      // (p = 256 takes the same path: t16 = 0, exact power-of-two rounding, r in
      // [-128, 128] whose low byte is the residue)
      int rr[16];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        rr[e] = (dma_mask & 4) ? acc[i][j][e] : centered_mod(acc[i][j][e], pf, rcp, t16);
      v4i o;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = (int)pack4(rr[4 * u], rr[4 * u + 1], rr[4 * u + 2], rr[4 * u + 3]);
      const int bi = wr * MI + i, bj = wc * NJ + j;
      *(v4i*)(cr + ((bi * (BN / 32) + bj) * 64 + lane) * 16) = o;
    }
}

// One thread = 8 residue bytes (8 output elements of one MFMA block) of every modulus.
template <class T, int BN>
__global__ void __launch_bounds__(256)
    k_crt_recon(const int8_t* __restrict__ CR, T* __restrict__ C, int64_t M, int64_t N,
                int64_t tiles_m, int64_t tiles_n, int accumulate, const RecTab rc) {
  constexpr int NK = sizeof(T) / 2;  // 16-bit words of a ring element
  const int64_t ntiles = tiles_m * tiles_n;
  constexpr int kCrTile = BM * BN, NBJ = BN / 32, LOGB = BN == 256 ? 6 : 5;
  const int64_t total = ntiles * (kCrTile / 8);
  const int64_t b = blockIdx.y;
  const int n = rc.n;
  for (int64_t gt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gt < total;
       gt += (int64_t)gridDim.x * blockDim.x) {
    const int hf = (int)(gt & 1);
    const int lane = (int)((gt >> 1) & 63);
    const int64_t rest = gt >> 7;
    const int blk = (int)(rest & ((1 << LOGB) - 1));  // 32x32 block (blk / NBJ, blk % NBJ)
    const int64_t tile = rest >> LOGB;
    const int64_t off = tile * kCrTile + (blk * 64 + lane) * 16 + hf * 8;
    int acc[8][NK];
    float qs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      qs[e] = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k) acc[e][k] = 0;
    }
    const int8_t* src = CR + b * n * ntiles * (int64_t)kCrTile + off;
    for (int i = 0; i < n; ++i) {
      const uint2 v = *(const uint2*)(src + i * ntiles * (int64_t)kCrTile);
      const float rcp = rc.rcp[i];
      int wk[NK];
#pragma unroll
      for (int k = 0; k < NK; ++k) wk[k] = rc.W[i][k];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = (int)(int8_t)(((e < 4 ? v.x : v.y) >> (8 * (e & 3))) & 0xff);
        qs[e] = __builtin_fmaf((float)c, rcp, qs[e]);
#pragma unroll
        for (int k = 0; k < NK; ++k) acc[e][k] += __mul24(c, wk[k]);
      }
    }
    const int64_t tm = tile / tiles_n, tn = tile % tiles_n;
    const int bi = blk / NBJ, bj = blk % NBJ;
    const int64_t gcol = tn * BN + bj * 32 + (lane & 31);
    T mw = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) mw |= (T)rc.Mw[k] << (16 * k);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ee = hf * 8 + e;  // accumulator register index in the 32x32 block
      const int row = (ee & 3) + 8 * (ee >> 2) + 4 * (lane >> 5);
      const int64_t grow = tm * BM + bi * 32 + row;
      T z = 0;
#pragma unroll
      for (int k = 0; k < NK; ++k) z += (T)(int64_t)acc[e][k] << (16 * k);
      const int q = (int)__builtin_rintf(qs[e]);
      z -= (T)(int64_t)q * mw;
      if (grow < M && gcol < N) {
        T* pc = C + (b * M + grow) * N + gcol;
        *pc = accumulate ? (T)(*pc + z) : z;
      }
    }
  }
}

// 16x16x64 variant: one v_mfma_i32_16x16x64_i8 covers a whole 64-byte k-step, lane l reads
// row l & 15, chunk l >> 4 of the image.  WR x WC waves, wave tile (BM/WR) x (BN/WC) =
// MI x NJ MFMA blocks of 16x16 (4 accumulator registers each).  Fragments of stage kb+1 are
// read right after the step's barrier into the second register set (the k-loop is unrolled
// by two so the sets swap without moves), while the second half of stage kb's MFMAs runs.
// Output bytes: 16x16 block (bi, bj) at ((bi * BN / 16 + bj) * 64 + lane) * 4 of the tile.
template <int WR, int WC, int BN, int MINW, int STG = kStages, int IL = 0>
__global__ void __launch_bounds__(64 * WR * WC, MINW)
    k_crt_gemm16(const int8_t* __restrict__ RA, const int8_t* __restrict__ RB,
                 int8_t* __restrict__ CR, int tiles_m, int tiles_n, int nkb_all, int gM,
                 const EpiTab ep, int dma_mask, int bcast, int a_nkb, int roll, int amap,
                 int bmap) {
  constexpr int NW = WR * WC;
  constexpr int MI = BM / WR / 16, NJ = BN / WC / 16;
  constexpr int NM = MI * NJ;                    // MFMAs per wave per k-step
  constexpr int kImgB = BN * BK;
  constexpr int kStageBytes = kImg + kImgB;
  constexpr int NPIECE = kStageBytes / 1024;
  constexpr int PPW = NPIECE / NW;
  static_assert(PPW * NW == NPIECE, "stage pieces must split evenly over the waves");
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int ntiles = tiles_m * tiles_n;
  const int tid_flat = (int)xcd_remap(blockIdx.x, ntiles);
  const int group = tid_flat / (gM * tiles_n);
  const int first_m = group * gM;
  const int gm = tiles_m - first_m < gM ? tiles_m - first_m : gM;
  const int in_group = tid_flat % (gM * tiles_n);
  const int tm = first_m + in_group % gm, tn = in_group / gm;
  // amap < 0 (bit 31): the asymmetric three-party product (run_crt_asym) -- the parties with
  // the full K' (1 and 2) are dispatched first, party 0's half-length blocks fill the tail
  const int g = amap < 0 ? (int)((blockIdx.y + ep.n) % gridDim.y) : (int)blockIdx.y;
  const int mi = g % ep.n;
  int nkb = nkb_all;
  const int8_t* ga = RA + ((int64_t)((bcast & 1) ? mi : g) * tiles_m + tm) * a_nkb * (int64_t)kImg;
  const int8_t* gb = RB + ((int64_t)((bcast & 2) ? mi : g) * tiles_n + tn) * nkb_all * (int64_t)kImgB;
  // roll != 0: A' = [x_b | x_{b+roll}] (an RSS pair whose second share is the next party's
  // first) -- the image holds each batch entry's K residues once; k-blocks from a_nkb on
  // read entry b + roll's image (ga2 is biased so that ga2 + kb * kImg addresses it)
  const int8_t* ga2 = ga;
  const int8_t* gb2 = gb;
  int khalf = 1 << 30;
  if (roll) {
    const int nbt = (int)gridDim.y / ep.n;
    const int b2 = (g / ep.n + roll) % nbt;
    ga2 = RA + ((int64_t)(b2 * ep.n + mi) * tiles_m + tm) * a_nkb * (int64_t)kImg -
          (int64_t)a_nkb * kImg;
    khalf = a_nkb;
  } else if (amap < 0) {
    // party b reads A' = [entry e1 | entry e2] of the K-residue A image and
    // B' = [entry f1 ; entry f2] of the K-residue B image (bmap), or only (e1, f1)'s K
    // (k-steps [0, a_nkb): party 0's one-GEMM product) when its half bit is set
    const int sh = 8 * (g / ep.n);
    const int e1 = (amap >> sh) & 7, e2 = (amap >> (sh + 3)) & 7;
    const int f1 = (bmap >> sh) & 7, f2 = (bmap >> (sh + 3)) & 7;
    ga = RA + ((int64_t)(e1 * ep.n + mi) * tiles_m + tm) * a_nkb * (int64_t)kImg;
    ga2 = RA + ((int64_t)(e2 * ep.n + mi) * tiles_m + tm) * a_nkb * (int64_t)kImg -
          (int64_t)a_nkb * kImg;
    gb = RB + ((int64_t)(f1 * ep.n + mi) * tiles_n + tn) * a_nkb * (int64_t)kImgB;
    gb2 = RB + ((int64_t)(f2 * ep.n + mi) * tiles_n + tn) * a_nkb * (int64_t)kImgB -
          (int64_t)a_nkb * kImgB;
    khalf = a_nkb;
    if ((amap >> (sh + 6)) & 1) nkb = a_nkb;
  }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int co = 16 * ((lane >> 4) ^ swz((lane & 15) >> 2));
  const int rowa = (wr * (BM / WR) + (lane & 15)) * BK + co;
  const int rowb = kImg + (wc * (BN / WC) + (lane & 15)) * BK + co;

  const int8_t* srcs[PPW];
  const int8_t* srcs2[PPW];
  int dsts[PPW], steps[PPW];
#pragma unroll
  for (int t = 0; t < PPW; ++t) {
    const int pc = wave + NW * t;
    const bool is_b = pc >= 16;
    const int pp = is_b ? pc - 16 : pc;
    srcs[t] = (is_b ? gb : ga) + pp * 1024 + lane * 16;
    srcs2[t] = (is_b ? gb2 : ga2) + pp * 1024 + lane * 16;
    dsts[t] = (is_b ? kImg : 0) + pp * 1024;
    steps[t] = is_b ? kImgB : kImg;
  }
  bool dma_on[PPW];
#pragma unroll
  for (int t = 0; t < PPW; ++t) dma_on[t] = (dma_mask >> ((wave + NW * t) >= 16 ? 1 : 0)) & 1;
  auto dma = [&](int kb, int t, int8_t* dst_stage) {
    if (!dma_on[t]) return;  // MOOSEX_CRT_DMA_MASK timing experiments only
    const int8_t* src = kb >= khalf ? srcs2[t] : srcs[t];
    __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)kb * steps[t]),
                                     (__attribute__((address_space(3))) void*)(dst_stage + dsts[t]),
                                     16, 0, 0);
  };

  v4i acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  v4i fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
  const bool no_frags = (dma_mask & 8) != 0;  // timing experiments only
  auto frags = [&](const int8_t* st, v4i(&fa)[MI], v4i(&fb)[NJ]) {
    if (no_frags) return;
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *(const v4i*)(st + rowa + i * 16 * BK);
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb[j] = *(const v4i*)(st + rowb + j * 16 * BK);
  };

  // IL == 3 (STG == 5): one barrier per TWO k-steps; the prologue issues stages 0..3 and
  // waits for 0..2 (stage 3 may still be in flight)
  constexpr int PRO = IL == 3 ? 4 : STG;
#pragma unroll
  for (int s = 0; s < PRO; ++s)
#pragma unroll
    for (int t = 0; t < PPW; ++t) dma(s < nkb ? s : nkb - 1, t, smem + s * kStageBytes);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0((PRO - 1) * PPW));
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  frags(smem, fa0, fb0);

  // one k-step: MFMAs of the stage in registers (fa, fb); after the first half, the barrier
  // (stage kb+1 landed everywhere, stage kb no longer read) and the reads of stage kb+1 into
  // (na, nb); the DMA of stage kb+3 into the freed buffer runs beside the second half
  auto step = [&](int kb, int8_t* cur, int8_t* nxt, v4i(&fa)[MI], v4i(&fb)[NJ], v4i(&na)[MI],
                  v4i(&nbf)[NJ]) __attribute__((always_inline)) {
    const int kn = kb + STG < nkb ? kb + STG : nkb - 1;
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      if (i == MI / 2) {
        __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0((STG - 2) * PPW));
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        frags(nxt, na, nbf);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll NJ
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        const int h = (i - MI / 2) * NJ + j;  // MFMA index in the second half
#pragma unroll PPW
        for (int t = 0; t < PPW; ++t)
          if (h == (t + 1) * (NM / 2) / PPW - 1) {
            dma(kn, t, cur);
            __builtin_amdgcn_sched_barrier(0);
          }
      }
    }
  };

  // IL: one barrier at the START of each k-step (stage kb+1 landed everywhere, stage kb's
  // buffer no longer read), then the step's MFMAs with the next stage's fragment reads
  // spread one per GAP MFMAs and the DMAs of stage kb+STG in the last gaps -- instead of
  // every wave bursting its 12 fragment reads into the LDS right after a mid-step barrier
  auto rd_frag = [&](const int8_t* st, int q, v4i(&fa)[MI], v4i(&fb)[NJ])
                     __attribute__((always_inline)) {
    if (no_frags) return;
    if (q < MI)
      fa[q] = *(const v4i*)(st + rowa + q * 16 * BK);
    else
      fb[q - MI] = *(const v4i*)(st + rowb + (q - MI) * 16 * BK);
  };
  auto step_il = [&](int kb, int8_t* cur, int8_t* nxt, v4i(&fa)[MI], v4i(&fb)[NJ],
                     v4i(&na)[MI], v4i(&nbf)[NJ]) __attribute__((always_inline)) {
    const int kn = kb + STG < nkb ? kb + STG : nkb - 1;
    constexpr int NR = MI + NJ;
    constexpr int GAP = (NM - 2 * PPW) / NR > 0 ? (NM - 2 * PPW) / NR : 1;
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0((STG - 2) * PPW));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // IL == 2: the NR reads and PPW DMAs share the NM/2 odd gaps, a DMA in every
    // (NR + PPW)/PPW-th of them (so the DMAs spread over the whole step)
    constexpr int NMEM = NR + PPW, DEV = NMEM / PPW;
#pragma unroll
    for (int h = 0; h < NM; ++h) {
      const int i = h / NJ, j = h % NJ;
      acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (IL == 2) {
        if (h % 2 == 1 && h / 2 < NMEM) {
          const int u = h / 2;
          if (u % DEV == DEV - 1 && u / DEV < PPW) {
            dma(kn, u / DEV, cur);
          } else {
            const int q = u - (u / DEV < PPW ? u / DEV : PPW);
            if (q < NR) rd_frag(nxt, q, na, nbf);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        if (h % GAP == GAP - 1 && h / GAP < NR) {
          rd_frag(nxt, h / GAP, na, nbf);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll PPW
        for (int t = 0; t < PPW; ++t)
          if (h == NM - 2 * PPW + 2 * t + 1) {
            dma(kn, t, cur);
            __builtin_amdgcn_sched_barrier(0);
          }
      }
    }
  };

  // IL == 3: five 32 KB stage buffers (160 KB), stage s in buffer s % 5, a barrier only at
  // even k-steps.  Barrier B_k (even k) follows each wave's wait for its DMAs of stages
  // k+1 and k+2 (only stage k+3's may still be in flight), so step k reads stage k+1 and
  // step k+1 reads stage k+2 without a barrier of its own; and every wave has finished
  // step k-1, so the buffers of stages k-1 and k (fragments already in registers) are free
  // and take stages k+4 and k+5 -- issued in that order, the k+4 pieces first, so that
  // "all but the last PPW" is exactly "all but stage k+5".
  auto step_pair = [&](int kb, bool even, v4i(&fa)[MI], v4i(&fb)[NJ], v4i(&na)[MI],
                       v4i(&nbf)[NJ]) __attribute__((always_inline)) {
    constexpr int NR = MI + NJ;
    constexpr int GAP = (NM - 2 * PPW) / NR > 0 ? (NM - 2 * PPW) / NR : 1;
    const int8_t* nxt = smem + ((kb + 1) % STG) * kStageBytes;
    int8_t* d4 = smem + ((kb + 4) % STG) * kStageBytes;
    int8_t* d5 = smem + ((kb + 5) % STG) * kStageBytes;
    const int k4 = kb + 4 < nkb ? kb + 4 : nkb - 1;
    const int k5 = kb + 5 < nkb ? kb + 5 : nkb - 1;
    if (even) {
      __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(PPW));
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int h = 0; h < NM; ++h) {
      const int i = h / NJ, j = h % NJ;
      acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (h % GAP == GAP - 1 && h / GAP < NR) {
        rd_frag(nxt, h / GAP, na, nbf);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (even) {
#pragma unroll PPW
        for (int t = 0; t < PPW; ++t) {
          if (h == NM - 2 * PPW + t) {
            dma(k4, t, d4);
            __builtin_amdgcn_sched_barrier(0);
          }
          if (h == NM - PPW + t) {
            dma(k5, t, d5);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
  };

  auto buf = [&](int i) { return smem + i * kStageBytes; };
  int r = 0;  // stage kb lives in buf(r)
  if constexpr (IL == 3) {
    static_assert(STG == 5, "the paired schedule needs five stage buffers");
    for (int kb = 0; kb < nkb; kb += 2) {
      step_pair(kb, true, fa0, fb0, fa1, fb1);
      if (kb + 1 < nkb) step_pair(kb + 1, false, fa1, fb1, fa0, fb0);
    }
  } else
  for (int kb = 0; kb < nkb; kb += 2) {
    if constexpr (IL)
      step_il(kb, buf(r), buf(r == STG - 1 ? 0 : r + 1), fa0, fb0, fa1, fb1);
    else
      step(kb, buf(r), buf(r == STG - 1 ? 0 : r + 1), fa0, fb0, fa1, fb1);
    r = r == STG - 1 ? 0 : r + 1;
    if (kb + 1 < nkb) {
      if constexpr (IL)
        step_il(kb + 1, buf(r), buf(r == STG - 1 ? 0 : r + 1), fa1, fb1, fa0, fb0);
      else
        step(kb + 1, buf(r), buf(r == STG - 1 ? 0 : r + 1), fa1, fb1, fa0, fb0);
      r = r == STG - 1 ? 0 : r + 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const float pf = ep.pf[mi], rcp = ep.rcp[mi];
  const int t16 = ep.t16[mi];
  int8_t* cr = CR + ((int64_t)g * ntiles + tm * tiles_n + tn) * (int64_t)(BM * BN);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      int rr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        rr[e] = centered_mod(acc[i][j][e], pf, rcp, t16);
      const int bi = wr * MI + i, bj = wc * NJ + j;
      *(uint32_t*)(cr + ((bi * (BN / 16) + bj) * 64 + lane) * 4) = pack4(rr[0], rr[1], rr[2], rr[3]);
    }
}

// reconstruction for the 16x16 output layout: one thread = one lane's 4 bytes of a block
template <class T, int BN>
__global__ void __launch_bounds__(256)
    k_crt_recon16(const int8_t* __restrict__ CR, T* __restrict__ C, int64_t M, int64_t N,
                  int64_t tiles_m, int64_t tiles_n, int accumulate, const RecTab rc) {
  constexpr int NK = sizeof(T) / 2;
  constexpr int kCrTile = BM * BN, NBJ = BN / 16;
  const int64_t ntiles = tiles_m * tiles_n;
  const int64_t total = ntiles * (kCrTile / 4);
  const int64_t b = blockIdx.y;
  const int n = rc.n;
  for (int64_t gt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gt < total;
       gt += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(gt & 63);
    const int64_t rest = gt >> 6;
    const int blk = (int)(rest % (16 * NBJ));
    const int64_t tile = rest / (16 * NBJ);
    const int64_t off = tile * kCrTile + (blk * 64 + lane) * 4;
    int acc[4][NK];
    float qs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qs[e] = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k) acc[e][k] = 0;
    }
    const int8_t* src = CR + b * n * ntiles * (int64_t)kCrTile + off;
    for (int i = 0; i < n; ++i) {
      const uint32_t v = *(const uint32_t*)(src + i * ntiles * (int64_t)kCrTile);
      const float rcp = rc.rcp[i];
      int wk[NK];
#pragma unroll
      for (int k = 0; k < NK; ++k) wk[k] = rc.W[i][k];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = (int)(int8_t)((v >> (8 * e)) & 0xff);
        qs[e] = __builtin_fmaf((float)c, rcp, qs[e]);
#pragma unroll
        for (int k = 0; k < NK; ++k) acc[e][k] += __mul24(c, wk[k]);
      }
    }
    const int64_t tm = tile / tiles_n, tn = tile % tiles_n;
    const int bi = blk / NBJ, bj = blk % NBJ;
    const int64_t gcol = tn * BN + bj * 16 + (lane & 15);
    T mw = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) mw |= (T)rc.Mw[k] << (16 * k);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t grow = tm * BM + bi * 16 + 4 * (lane >> 4) + e;
      T z = 0;
#pragma unroll
      for (int k = 0; k < NK; ++k) z += (T)(int64_t)acc[e][k] << (16 * k);
      const int q = (int)__builtin_rintf(qs[e]);
      z -= (T)(int64_t)q * mw;
      if (grow < M && gcol < N) {
        T* pc = C + (b * M + grow) * N + gcol;
        *pc = accumulate ? (T)(*pc + z) : z;
      }
    }
  }
}

// k_crt_recon16 with the per-modulus multiply-adds done as v_dot4_i32_i8: a thread's 4
// elements x 4 moduli of residues (4 dwords, one per modulus plane) are transposed with 8
// v_perm_b32 into one dword of 4 moduli per element, then one dot4 per (element, W digit)
// and per (element, R digit) -- 19 dot4 for 4 moduli instead of 4 x (8 multiply-adds + a
// float convert and fma).  q = round(sum_i c_i R_i / 2^24) (error <= 36 * 128 / 2^25, far
// inside the 0.05 rounding margin of |Z| <= 0.45 M).  Same output as k_crt_recon16.
template <class T, int BN>
__global__ void __launch_bounds__(256)
    k_crt_recon16d(const int8_t* __restrict__ CR, T* __restrict__ C, int64_t M, int64_t N,
                   int64_t tiles_m, int64_t tiles_n, int accumulate, const RecTab4 r4, int n,
                   const RecTab rc) {
  constexpr int ND = (int)sizeof(T);  // W digits
  constexpr int NK = ND / 2;
  constexpr int kCrTile = BM * BN, NBJ = BN / 16;
  const int64_t ntiles = tiles_m * tiles_n;
  const int64_t total = ntiles * (kCrTile / 4);
  const int64_t b = blockIdx.y;
  for (int64_t gt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gt < total;
       gt += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(gt & 63);
    const int64_t rest = gt >> 6;
    const int blk = (int)(rest % (16 * NBJ));
    const int64_t tile = rest / (16 * NBJ);
    const int64_t off = tile * kCrTile + (blk * 64 + lane) * 4;
    int acc[4][ND], aq[4][3];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int d = 0; d < ND; ++d) acc[e][d] = 0;
#pragma unroll
      for (int d = 0; d < 3; ++d) aq[e][d] = 0;
    }
    const int8_t* src = CR + b * n * ntiles * (int64_t)kCrTile + off;
    const int64_t pstride = ntiles * (int64_t)kCrTile;
    for (int g = 0; g < r4.groups; ++g) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = 4 * g + u < n ? *(const uint32_t*)(src + (4 * g + u) * pstride) : 0u;
      const uint32_t a0 = __builtin_amdgcn_perm(v[1], v[0], 0x05010400u);
      const uint32_t a1 = __builtin_amdgcn_perm(v[1], v[0], 0x07030602u);
      const uint32_t c0 = __builtin_amdgcn_perm(v[3], v[2], 0x05010400u);
      const uint32_t c1 = __builtin_amdgcn_perm(v[3], v[2], 0x07030602u);
      const int t[4] = {(int)__builtin_amdgcn_perm(c0, a0, 0x05040100u),
                        (int)__builtin_amdgcn_perm(c0, a0, 0x07060302u),
                        (int)__builtin_amdgcn_perm(c1, a1, 0x05040100u),
                        (int)__builtin_amdgcn_perm(c1, a1, 0x07060302u)};
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int w = (int)r4.wd[g][d];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e][d] = __builtin_amdgcn_sdot4(t[e], w, acc[e][d], false);
      }
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int w = (int)r4.rd[g][d];
#pragma unroll
        for (int e = 0; e < 4; ++e) aq[e][d] = __builtin_amdgcn_sdot4(t[e], w, aq[e][d], false);
      }
    }
    const int64_t tm = tile / tiles_n, tn = tile % tiles_n;
    const int bi = blk / NBJ, bj = blk % NBJ;
    const int64_t gcol = tn * BN + bj * 16 + (lane & 15);
    T mw = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) mw |= (T)rc.Mw[k] << (16 * k);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t grow = tm * BM + bi * 16 + 4 * (lane >> 4) + e;
      T z = 0;
#pragma unroll
      for (int k = 0; k < NK; ++k)
        z += (T)(int64_t)(acc[e][2 * k] + acc[e][2 * k + 1] * 256) << (16 * k);
      const int64_t F = (int64_t)aq[e][0] + (int64_t)aq[e][1] * 256 + (int64_t)aq[e][2] * 65536;
      const int64_t q = (F + (1 << 23)) >> 24;
      z -= (T)q * mw;
      if (grow < M && gcol < N) {
        T* pc = C + (b * M + grow) * N + gcol;
        *pc = accumulate ? (T)(*pc + z) : z;
      }
    }
  }
}

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

int crt_kernel() {  // MOOSEX_CRT_KERNEL: 1 = 4 waves of 128x128, 2 = 8 waves of 128x64
  // (256x256 tiles, one block per CU), 3 = 4 waves of 128x64 in 256x128 tiles (two blocks
  // per CU, so one block's barrier waits, LDS bursts and epilogue overlap the other's MFMAs)
  // 4 = 16x16x64 MFMAs, 4 waves of 128x128 (256x256 tiles; the compiler spills: 71 ms),
  // 5 = 16x16x64, 4 waves of 128x64 in 256x128 tiles (72 KB LDS: two blocks per CU; 12 %
  // faster than 3 -- the chip holds a higher clock on the 16x16 shape), 6 = 16x16x64, 8
  // waves of 128x64 in 256x256 tiles (96 KB LDS and 242 VGPRs: ONE block per CU, two waves
  // per SIMD; 11.95 vs 12.12 ms for 5 on the 4096^2 Z_2^128 RSS product,
  // profiles/r2_crt_variant_ab.md), 7 = 6 with a 4-stage ring (no gain), 8 = 6 with one
  // barrier at the start of each k-step and the next stage's fragment reads spread over the
  // step's MFMAs (the default: 4-6 % faster than 6 on the same box, profiles/r3_crt_gemm.md),
  // 9 = 8 with 4 stages, 10 / 11 = 8 / 9 with the DMAs spread over the step too, 12 = 4
  // with 8's schedule, 13 = 12 with 4 stages, 14 / 15 = 12 / 13 with the DMAs spread (4 and
  // 12-15 need the VGPR-form MFMA flag of _native/build.py, else they spill), 16 = 8 with
  // one barrier per two k-steps over five stage buffers (160 KB LDS).  Tried and removed (profiles/r3_crt_gemm.md): DMAs through
  // buffer descriptors (16.2 vs 15.5 ms per step), a persistent one-block-per-CU kernel
  // streaming all its tiles' k-steps (16.2 vs 15.5 ms), B fragments loaded from global
  // memory straight into registers (hipcc drains every counter before their first use)
  const char* e = std::getenv("MOOSEX_CRT_KERNEL");
  const int v = e ? std::atoi(e) : 8;
  return v >= 1 && v <= 16 ? v : 8;
}
bool crt_mfma16() { return crt_kernel() >= 4; }
int recon_dot4() {  // MOOSEX_CRT_RECON=0: the multiply-add reconstruction
  static const int v = [] {
    const char* e = std::getenv("MOOSEX_CRT_RECON");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return v;
}

struct CPlan {
  int n, bn;
  int64_t tiles_m, tiles_n, nkb, a_nkb, ra_bytes, rb_bytes, cr_bytes;
};

// roll: the A' image holds each batch entry's K residues once (k_crt_gemm16's roll)
CPlan make_cplan(int words, int64_t batch, int64_t M, int64_t N, int64_t K, int mode,
                 bool roll = false) {
  CPlan p;
  p.bn = (crt_kernel() == 3 || crt_kernel() == 5) ? 128 : 256;  // B tile columns
  const int64_t kprime = mode ? 2 * K : K;
  p.n = moduli_needed(words, kprime);
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = (N + p.bn - 1) / p.bn;
  p.nkb = round_up(kprime, BK) / BK;
  p.a_nkb = roll ? p.nkb / 2 : p.nkb;
  p.ra_bytes = batch * p.n * p.tiles_m * p.a_nkb * (int64_t)kImg;
  p.rb_bytes = batch * p.n * p.tiles_n * p.nkb * (int64_t)(p.bn * BK);
  p.cr_bytes = batch * p.n * p.tiles_m * p.tiles_n * (int64_t)(BM * p.bn);
  return p;
}

int gemm_group_m() {  // 8: 0.02-0.07 ms per headline step faster than 4 (profiles/r6_asym_products.md)
  const char* e = std::getenv("MOOSEX_CRT_GROUPM");
  const int v = e ? std::atoi(e) : 8;
  return v >= 1 && v <= 64 ? v : 8;
}

bool prep_packed() {
  static const bool v = [] {
    const char* e = std::getenv("MOOSEX_CRT_PACKED");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <class T>
void launch_prep(const CPlan& p, const Tables& tb, bool is_b, int64_t batch, int64_t R,
                 int64_t K, int64_t xs, const T* X0, const T* X1, int mode, int8_t* out,
                 hipStream_t st, int64_t nkb = -1, int64_t nkb_s = -1,
                 const PrepSrcs& src = PrepSrcs()) {
  if (nkb < 0) nkb = p.nkb;
  if (nkb_s < nkb) nkb_s = nkb;
  const int64_t tiles = is_b ? p.tiles_n : p.tiles_m;
  const int rows = is_b ? p.bn : BM;
  const int64_t work = tiles * nkb * (rows * 4);
  const dim3 grid((unsigned)std::min<int64_t>((work + 255) / 256, 16384), (unsigned)batch);
  // packed residues pay on A' (0.626 -> 0.592 ms at 4096^2) but not on the B' image, which
  // streams 1.5x the bytes and loses more to the extra VGPRs (1.128 -> 1.163 ms)
  static const bool packed_b = [] {  // MOOSEX_CRT_PACKED_B=1: packed residues on B' too
    const char* e = std::getenv("MOOSEX_CRT_PACKED_B");
    return e && e[0] == '1';
  }();
  if (!prep_packed() || (is_b && !packed_b)) {  // MOOSEX_CRT_PACKED=0: one at a time everywhere
    if (!is_b)
      hipLaunchKernelGGL((k_crt_prep<T, false, BM, false>), grid, dim3(256), 0, st, X0, X1, R, K,
                         xs, mode, out, tiles, nkb, nkb_s, tb.pa, src);
    else if (rows == 256)
      hipLaunchKernelGGL((k_crt_prep<T, true, 256, false>), grid, dim3(256), 0, st, X0, X1, R, K,
                         xs, mode, out, tiles, nkb, nkb_s, tb.pb, src);
    else
      hipLaunchKernelGGL((k_crt_prep<T, true, 128, false>), grid, dim3(256), 0, st, X0, X1, R, K,
                         xs, mode, out, tiles, nkb, nkb_s, tb.pb, src);
    return;
  }
  if (!is_b)
    hipLaunchKernelGGL((k_crt_prep<T, false, BM>), grid, dim3(256), 0, st, X0, X1, R, K, xs, mode,
                       out, tiles, nkb, nkb_s, tb.pa, src);
  else if (rows == 256)
    hipLaunchKernelGGL((k_crt_prep<T, true, 256>), grid, dim3(256), 0, st, X0, X1, R, K, xs, mode,
                       out, tiles, nkb, nkb_s, tb.pb, src);
  else
    hipLaunchKernelGGL((k_crt_prep<T, true, 128>), grid, dim3(256), 0, st, X0, X1, R, K, xs, mode,
                       out, tiles, nkb, nkb_s, tb.pb, src);
}

// MOOSEX_CRT_DMA_MASK (timing experiments, wrong results): bit 0 = stream A, bit 1 = B,
// bit 2 = skip the epilogue reduction, bit 3 = no LDS fragment reads in the main loop
int dma_mask() {
  const char* e = std::getenv("MOOSEX_CRT_DMA_MASK");
  return e ? std::atoi(e) : 3;
}

template <int WR, int WC, int BN, int MINW, bool M16, int STG = kStages, int IL = 0>
void launch_variant(const CPlan& p, const Tables& tb, int64_t batch, const int8_t* ra,
                    const int8_t* rb, int8_t* cr, int bcast, int roll, hipStream_t st,
                    int amap = 0, int bmap = 0) {
  constexpr int lds = STG * (kImg + BN * BK);
  const void* fn = M16 ? (const void*)k_crt_gemm16<WR, WC, BN, MINW, STG, IL>
                       : (const void*)k_crt_gemm<WR, WC, BN, MINW>;
  ensure_lds_attr(fn, lds, st);
  const dim3 grid((unsigned)(p.tiles_m * p.tiles_n), (unsigned)(batch * p.n));
  if constexpr (M16)
    hipLaunchKernelGGL((k_crt_gemm16<WR, WC, BN, MINW, STG, IL>), grid, dim3(64 * WR * WC), lds, st, ra,
                       rb, cr, (int)p.tiles_m, (int)p.tiles_n, (int)p.nkb, gemm_group_m(), tb.ep,
                       dma_mask(), bcast, (int)p.a_nkb, roll, amap, bmap);
  else
    hipLaunchKernelGGL((k_crt_gemm<WR, WC, BN, MINW>), grid, dim3(64 * WR * WC), lds, st, ra, rb,
                       cr, (int)p.tiles_m, (int)p.tiles_n, (int)p.nkb, gemm_group_m(), tb.ep,
                       dma_mask(), bcast);
}

void launch_crt_gemm(const CPlan& p, const Tables& tb, int64_t batch, const int8_t* ra,
                     const int8_t* rb, int8_t* cr, int bcast, int roll, hipStream_t st,
                     int amap = 0, int bmap = 0) {
  switch (crt_kernel()) {  // roll, amap: 16x16x64 kernels only (run_crt* check)
    case 1: launch_variant<2, 2, 256, 1, false>(p, tb, batch, ra, rb, cr, bcast, 0, st); break;
    case 2: launch_variant<2, 4, 256, 2, false>(p, tb, batch, ra, rb, cr, bcast, 0, st); break;
    case 4: launch_variant<2, 2, 256, 1, true>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 3: launch_variant<2, 2, 128, 2, false>(p, tb, batch, ra, rb, cr, bcast, 0, st); break;
    case 6: launch_variant<2, 4, 256, 2, true>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 7: launch_variant<2, 4, 256, 2, true, 4>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 8: launch_variant<2, 4, 256, 2, true, 3, 1>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 9: launch_variant<2, 4, 256, 2, true, 4, 1>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 10: launch_variant<2, 4, 256, 2, true, 3, 2>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 11: launch_variant<2, 4, 256, 2, true, 4, 2>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 12: launch_variant<2, 2, 256, 1, true, 3, 1>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 13: launch_variant<2, 2, 256, 1, true, 4, 1>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 14: launch_variant<2, 2, 256, 1, true, 3, 2>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 15: launch_variant<2, 2, 256, 1, true, 4, 2>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    case 16: launch_variant<2, 4, 256, 2, true, 5, 3>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
    default: launch_variant<2, 2, 128, 2, true>(p, tb, batch, ra, rb, cr, bcast, roll, st, amap, bmap); break;
  }
}

template <class T>
void launch_recon(const CPlan& p, const Tables& tb, int64_t batch, int64_t M, int64_t N,
                  const int8_t* cr, T* C, int accumulate, hipStream_t st) {
  const int64_t work = p.tiles_m * p.tiles_n * (BM * p.bn / 8);
  const int gx = (int)std::min<int64_t>((work + 255) / 256, 16384);
  if (crt_mfma16() && recon_dot4()) {
    const int gx16 = (int)std::min<int64_t>((2 * work + 255) / 256, 16384);
    if (p.bn == 256)
      hipLaunchKernelGGL((k_crt_recon16d<T, 256>), dim3(gx16, (unsigned)batch), dim3(256), 0, st,
                         cr, C, M, N, p.tiles_m, p.tiles_n, accumulate, tb.r4, p.n, tb.rc);
    else
      hipLaunchKernelGGL((k_crt_recon16d<T, 128>), dim3(gx16, (unsigned)batch), dim3(256), 0, st,
                         cr, C, M, N, p.tiles_m, p.tiles_n, accumulate, tb.r4, p.n, tb.rc);
  } else if (crt_mfma16()) {
    const int gx16 = (int)std::min<int64_t>((2 * work + 255) / 256, 16384);
    if (p.bn == 256)
      hipLaunchKernelGGL((k_crt_recon16<T, 256>), dim3(gx16, (unsigned)batch), dim3(256), 0, st,
                         cr, C, M, N, p.tiles_m, p.tiles_n, accumulate, tb.rc);
    else
      hipLaunchKernelGGL((k_crt_recon16<T, 128>), dim3(gx16, (unsigned)batch), dim3(256), 0, st,
                         cr, C, M, N, p.tiles_m, p.tiles_n, accumulate, tb.rc);
  } else if (p.bn == 256)
    hipLaunchKernelGGL((k_crt_recon<T, 256>), dim3(gx, (unsigned)batch), dim3(256), 0, st, cr, C,
                       M, N, p.tiles_m, p.tiles_n, accumulate, tb.rc);
  else
    hipLaunchKernelGGL((k_crt_recon<T, 128>), dim3(gx, (unsigned)batch), dim3(256), 0, st, cr, C,
                       M, N, p.tiles_m, p.tiles_n, accumulate, tb.rc);
}

struct Ws {
  void* ptr = nullptr;
  int64_t bytes = 0;
  hipStream_t stream = nullptr;
  bool used = false;
};
std::mutex g_mu;
constexpr int kWsPerDev = 128;
Ws g_ws[16][kWsPerDev];

// Grow-only scratch per (device, stream): GEMMs issued on different streams (dataflow lanes,
// pipelined steps, the in-process parties' graphs replayed concurrently) may run at the same
// time and must not share residue buffers.  kWsPerDev exceeds the streams a process can hold
// (PyTorch's pools: 32 per priority, plus the null stream); past it streams would share the
// last slot (ordered only by the caller) -- counted, mx_workspace_shared_count.  Replaced
// buffers are retired, never freed (a captured graph may hold them).
void* workspace(int64_t bytes, hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  Ws* slot = nullptr;
  for (int i = 0; i < kWsPerDev && !slot; ++i)
    if (g_ws[dev][i].used && g_ws[dev][i].stream == st) slot = &g_ws[dev][i];
  for (int i = 0; i < kWsPerDev && !slot; ++i)
    if (!g_ws[dev][i].used) {
      slot = &g_ws[dev][i];
      slot->used = true;
      slot->stream = st;
    }
  if (!slot) {
    slot = &g_ws[dev][kWsPerDev - 1];
    mx_ws_shared_note();
  }
  Ws& w = *slot;
  if (w.bytes < bytes) {
    int64_t want = 1 << 20;
    while (want < bytes) want <<= 1;
    void* q = nullptr;
    const bool ok = mx_ws_malloc(&q, want);
    mx_ws_note(dev, want, ok);
    if (!ok) return nullptr;
    w.ptr = q;
    w.bytes = want;
  }
  return w.ptr;
}

template <class T>
int run_crt(int64_t batch, int64_t M, int64_t N, int64_t K, const T* A0, const T* A1,
            int64_t a_bstride, const T* B0, const T* B1, int64_t b_bstride,
            const int8_t* rb_pre, int mode, T* C, int accumulate, hipStream_t st,
            int64_t roll = 0) {
  constexpr int words = sizeof(T) / 8;
  if (roll && (mode != 1 || K % BK || !crt_mfma16() || a_bstride == 0 || batch < 2 ||
               roll % batch == 0))
    return -7;  // not applicable: the caller runs the two-operand form
  const CPlan p = make_cplan(words, batch, M, N, K, mode, roll != 0);
  if (p.n < 0) return -6;
  if ((mode ? 2 * K : K) > (1 << 15)) return -6;  // exact epilogue rounding bound
  const Tables& tb = tables_for(words, p.n);
  const int64_t need = p.ra_bytes + (rb_pre ? 0 : p.rb_bytes) + p.cr_bytes;
  int8_t* ws = (int8_t*)workspace(need, st);
  if (!ws) return -4;
  int8_t* ra = ws;
  int8_t* cr = ra + p.ra_bytes;
  const int8_t* rb = rb_pre;
  // an operand broadcast over the batch (stride 0) has its residues prepared once and read
  // by every batch entry's GEMM (every product is still computed)
  const bool a_bc = batch > 1 && a_bstride == 0;
  const bool b_bc = batch > 1 && b_bstride == 0 && !rb_pre;
  if (!rb) {
    int8_t* rbw = cr + p.cr_bytes;
    launch_prep<T>(p, tb, true, b_bc ? 1 : batch, N, K, b_bstride, B0, B1, mode, rbw, st);
    rb = rbw;
  }
  if (roll)  // each entry's own K residues; the GEMM reads entry b + roll's for the 2nd half
    launch_prep<T>(p, tb, false, batch, M, K, a_bstride, A0, A0, 0, ra, st, p.a_nkb);
  else
    launch_prep<T>(p, tb, false, a_bc ? 1 : batch, M, K, a_bstride, A0, A1, mode, ra, st);
  launch_crt_gemm(p, tb, batch, ra, rb, cr, (a_bc ? 1 : 0) | (b_bc ? 2 : 0),
                  (int)(((roll % batch) + batch) % batch), st);
  launch_recon<T>(p, tb, batch, M, N, cr, C, accumulate, st);
  const hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

// The three parties' local products of a replicated matrix product in the asymmetric
// form: with party p holding (a, b) = (x_p, x_{p+1}) and (c, d) = (y_p, y_{p+1}),
//   z_0 = (a + b)(c + d),   z_1 = b (c + d) + a d,   z_2 = a d + b c,
// which sum to x.y (all nine x_i y_j exactly once) with five K-long GEMMs instead of the
// symmetric form's six (z_p = a (c + d) + b c for every p).  S0/S1, T0/T1: [3][M][K] and
// [3][K][N] share stacks; rolled: S1[p] = S0[p + 1] and T1[p] = T0[p + 1] (a stacked
// session's pair; S1/T1 may be null) -- party 1's b and party 2's a are then the same
// share x_2, whose residues are prepared once (four K-long A' images instead of five).
template <class T>
int run_crt_asym(int64_t M, int64_t N, int64_t K, const T* S0, const T* S1, const T* T0,
                 const T* T1, int rolled, T* C, hipStream_t st) {
  constexpr int words = sizeof(T) / 8;
  if (K % BK || !crt_mfma16()) return -7;
  if (2 * K > (1 << 15)) return -6;  // exact epilogue rounding bound
  const CPlan p = make_cplan(words, 3, M, N, K, 1, true);  // nkb = 2K/64, a_nkb = K/64
  if (p.n < 0) return -6;
  const Tables& tb = tables_for(words, p.n);
  const int64_t sa = M * K, sb = K * N;
  const T* a[3];
  const T* b[3];
  const T* c[3];
  const T* d[3];
  for (int q = 0; q < 3; ++q) {
    a[q] = S0 + q * sa;
    b[q] = rolled ? S0 + ((q + 1) % 3) * sa : S1 + q * sa;
    c[q] = T0 + q * sb;
    d[q] = rolled ? T0 + ((q + 1) % 3) * sb : T1 + q * sb;
  }
  // K-residue images.  A: E0 = a_0 + b_0; party 1 reads [b_1 | a_1], party 2 [a_2 | b_2].
  // B: F0 = c_0 + d_0, F1 = c_1 + d_1; party 1 reads [F1 ; d_1], party 2 [d_2 ; c_2].
  // Rolled (a_p = x_p, b_p = x_{p+1}, c_p = y_p, d_p = y_{p+1}): b_1 = a_2 = x_2 and
  // d_1 = c_2 = y_2 are one image each -- A = [x_0 + x_1, x_2, x_1, x_0], B = [y_0 + y_1,
  // y_1 + y_2, y_2, y_0] -- and each image group is one batched launch.
  int na, nb, amap, bmap;
  const int64_t a_entry = p.n * p.tiles_m * p.a_nkb * (int64_t)kImg;
  const int64_t b_entry = p.n * p.tiles_n * p.a_nkb * (int64_t)(p.bn * BK);
  auto pmap = [](int e0, int e1, int e2, int e3, int e4) {  // party 0: (e0, -) half-length
    return (int)(0x80000000u | (unsigned)e0 | (1u << 6) | ((unsigned)(e1 | (e2 << 3)) << 8) |
                 ((unsigned)(e3 | (e4 << 3)) << 16));
  };
  if (rolled) {
    na = 4;
    nb = 4;
    amap = pmap(0, 1, 2, 1, 3);
    bmap = pmap(0, 1, 2, 3, 2);
  } else {
    na = 5;
    nb = 5;
    amap = pmap(0, 1, 2, 3, 4);
    bmap = pmap(0, 1, 2, 3, 4);
  }
  const int64_t ra_bytes = na * a_entry, rb_bytes = nb * b_entry;
  static const bool asum = [] {  // MOOSEX_CRT_ASUM=0: the sum inside the prep (mode 2)
    const char* e = std::getenv("MOOSEX_CRT_ASUM");
    return !(e && e[0] == '0');
  }();
  static const bool dual = [] {  // MOOSEX_CRT_DUAL=0: separate sum images
    const char* e = std::getenv("MOOSEX_CRT_DUAL");
    return !(e && e[0] == '0');
  }();
  // rolled: the sums ride on the share images' threads (dual) -- no separate sum pass
  const bool duals = rolled && dual;
  const int64_t sum_bytes = asum && !duals ? round_up(sa * (int64_t)sizeof(T), 256) : 0;
  int8_t* ws = (int8_t*)workspace(ra_bytes + rb_bytes + p.cr_bytes + sum_bytes, st);
  if (!ws) return -4;
  int8_t* ra = ws;
  int8_t* cr = ra + ra_bytes;
  int8_t* rb = cr + p.cr_bytes;
  T* a01 = sum_bytes ? (T*)(rb + rb_bytes) : nullptr;
  if (a01)
    hipLaunchKernelGGL((k_add_pair<T>), dim3((unsigned)std::min<int64_t>((sa + 255) / 256, 65536)),
                       dim3(256), 0, st, a[0], b[0], a01, sa);
  const int64_t kn = p.a_nkb;
  // every image of a side in one launch (a lone batch-1 launch of the sum ran at half the
  // bandwidth of the batched images)
  PrepSrcs sa_, sb_;
  auto put = [](PrepSrcs& q, const T* x0, const T* x1, int mode, int64_t dual = 0) {
    q.x0[q.n] = x0;
    q.x1[q.n] = x1;
    q.mode[q.n] = mode;
    q.dual[q.n] = dual;
    ++q.n;
  };
  if (duals) {
    // A = [x0 + x1, x2, x1, x0]: the x0 thread writes E3 and then E0 = x0 + x1.
    // B = [y0 + y1, y1 + y2, y2, y0]: the y2 thread writes F2 and then F1 = y2 + y1, the y0
    // thread F3 and then F0 = y0 + y1.  Launched as entries 1..3 / 2..3 of the image.
    put(sa_, a[2], a[2], 0);                  // E1 = x2
    put(sa_, a[1], a[1], 0);                  // E2 = x1
    put(sa_, a[0], b[0], 0, -3 * a_entry);    // E3 = x0, dual E0 = x0 + x1
    put(sb_, d[1], c[1], 0, -b_entry);        // F2 = y2, dual F1 = y2 + y1
    put(sb_, d[2], d[0], 0, -3 * b_entry);    // F3 = y0, dual F0 = y0 + y1
    launch_prep<T>(p, tb, true, sb_.n, N, K, 0, nullptr, nullptr, 0, rb + 2 * b_entry, st, kn,
                   kn, sb_);
    launch_prep<T>(p, tb, false, sa_.n, M, K, 0, nullptr, nullptr, 0, ra + a_entry, st, kn, kn,
                   sa_);
  } else {
    if (a01)
      put(sa_, a01, a01, 0);
    else
      put(sa_, a[0], b[0], 2);
    put(sb_, c[0], d[0], 3);
    put(sb_, c[1], d[1], 3);
    if (rolled) {
      for (const T* e : {a[2], a[1], a[0]}) put(sa_, e, e, 0);  // x2, x1, x0
      for (const T* f : {d[1], d[2]}) put(sb_, f, f, 0);        // y2, y0
    } else {
      for (const T* e : {b[1], a[1], a[2], b[2]}) put(sa_, e, e, 0);
      for (const T* f : {d[1], d[2], c[2]}) put(sb_, f, f, 0);
    }
    launch_prep<T>(p, tb, true, sb_.n, N, K, 0, nullptr, nullptr, 0, rb, st, kn, kn, sb_);
    launch_prep<T>(p, tb, false, sa_.n, M, K, 0, nullptr, nullptr, 0, ra, st, kn, kn, sa_);
  }
  launch_crt_gemm(p, tb, 3, ra, rb, cr, 0, 0, st, amap, bmap);
  launch_recon<T>(p, tb, 3, M, N, cr, C, 0, st);
  const hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

}  // namespace

extern "C" {

// Asymmetric three-party RSS product (run_crt_asym): C[p] = z_p for p = 0, 1, 2.  -7: not
// applicable (the caller runs the generic form of the same z_p).
int mx_gemm_asym(int words, int64_t M, int64_t N, int64_t K, const void* S0, const void* S1,
                 const void* T0, const void* T1, int rolled, void* C, void* stream) {
  if (M == 0 || N == 0) return 0;
  if (!rolled && (!S1 || !T1)) return -2;
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    return run_crt_asym<u64>(M, N, K, (const u64*)S0, (const u64*)S1, (const u64*)T0,
                             (const u64*)T1, rolled, (u64*)C, st);
  if (words == 2)
    return run_crt_asym<u128>(M, N, K, (const u128*)S0, (const u128*)S1, (const u128*)T0,
                              (const u128*)T1, rolled, (u128*)C, st);
  return -2;
}

// Moduli count for a K' (= K, or 2K in mode 1) inner dimension; -1 if out of range.
int mx_crt_moduli(int words, int64_t kprime) {
  if (words != 1 && words != 2) return -2;
  return moduli_needed(words, kprime);
}

// Host copy of the tables (tests re-run the arithmetic on the CPU): per modulus i
// p, inv-folded A byte weights, B byte weights, A/B negative corrections, W_i words; and Mw.
int mx_crt_tables(int words, int n, int32_t* p_out, uint8_t* wa_out, uint8_t* wb_out,
                  int32_t* nega_out, int32_t* negb_out, uint16_t* W_out, uint16_t* Mw_out) {
  if ((words != 1 && words != 2) || n < 1 || n > kMaxMod) return -2;
  const Tables& t = tables_for(words, n);
  for (int i = 0; i < n; ++i) {
    p_out[i] = t.ep.p[i];
    for (int j = 0; j < 16; ++j) {
      wa_out[i * 16 + j] = (uint8_t)(t.pa.w[i][j / 4] >> (8 * (j % 4)));
      wb_out[i * 16 + j] = (uint8_t)(t.pb.w[i][j / 4] >> (8 * (j % 4)));
    }
    nega_out[i] = (int32_t)t.pa.neg[i];
    negb_out[i] = (int32_t)t.pb.neg[i];
    if (i == 0) {
      nega_out[0] = (int32_t)t.pa.mul0;  // p = 256 uses the multiplier instead
      negb_out[0] = 1;
    }
    for (int k = 0; k < 8; ++k) W_out[i * 8 + k] = t.rc.W[i][k];
  }
  for (int k = 0; k < 8; ++k) Mw_out[k] = t.rc.Mw[k];
  return 0;
}

// Host copy of the dot4 reconstruction tables (tests recompose the digits): wd
// [groups][16], rd [groups][3] words, modulus 4g + u in byte u.  Returns the group count.
int mx_crt_tables4(int words, int n, uint32_t* wd_out, uint32_t* rd_out) {
  if ((words != 1 && words != 2) || n < 1 || n > kMaxMod) return -2;
  const Tables& t = tables_for(words, n);
  for (int g = 0; g < t.r4.groups; ++g) {
    for (int d = 0; d < 16; ++d) wd_out[g * 16 + d] = t.r4.wd[g][d];
    for (int d = 0; d < 3; ++d) rd_out[g * 3 + d] = t.r4.rd[g][d];
  }
  return t.r4.groups;
}

int mxh_gemm_crt(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                 const void* A1, const void* B0, const void* B1, int mode, void* C,
                 int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    return run_crt<u64>(batch, M, N, K, (const u64*)A0, (const u64*)A1, M * K, (const u64*)B0,
                        (const u64*)B1, K * N, nullptr, mode, (u64*)C, accumulate, st);
  if (words == 2)
    return run_crt<u128>(batch, M, N, K, (const u128*)A0, (const u128*)A1, M * K,
                         (const u128*)B0, (const u128*)B1, K * N, nullptr, mode, (u128*)C,
                         accumulate, st);
  return -2;
}

// Batch strides given (elements; 0 broadcasts one operand over the batch): the operands of a
// batched product may be views such as an expanded (stride-0) stack -- no copy is made.
int mxh_gemm_crt_strided(int words, int64_t batch, int64_t M, int64_t N, int64_t K,
                         const void* A0, const void* A1, int64_t a_bstride, const void* B0,
                         const void* B1, int64_t b_bstride, int mode, void* C, int accumulate,
                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    return run_crt<u64>(batch, M, N, K, (const u64*)A0, (const u64*)A1, a_bstride,
                        (const u64*)B0, (const u64*)B1, b_bstride, nullptr, mode, (u64*)C,
                        accumulate, st);
  if (words == 2)
    return run_crt<u128>(batch, M, N, K, (const u128*)A0, (const u128*)A1, a_bstride,
                         (const u128*)B0, (const u128*)B1, b_bstride, nullptr, mode, (u128*)C,
                         accumulate, st);
  return -2;
}

// RSS pair form of the mode-1 product: A1 is A0 rolled by ``roll`` batch entries
// (A1[b] = A0[(b + roll) % batch], as the second shares of a stacked replicated sharing are
// the next party's first), so A' residues are prepared once per share instead of twice.
// rb: prepared B' (mxh_crt_prep_b) or null (then B0, B1).  -7: not applicable.
int mxh_crt_roll(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                 int64_t a_bstride, int64_t roll, const void* B0, const void* B1, const void* rb,
                 void* C, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int64_t bs = K * N;
  if (words == 1)
    return run_crt<u64>(batch, M, N, K, (const u64*)A0, nullptr, a_bstride, (const u64*)B0,
                        (const u64*)B1, bs, (const int8_t*)rb, 1, (u64*)C, accumulate, st, roll);
  if (words == 2)
    return run_crt<u128>(batch, M, N, K, (const u128*)A0, nullptr, a_bstride, (const u128*)B0,
                         (const u128*)B1, bs, (const int8_t*)rb, 1, (u128*)C, accumulate, st,
                         roll);
  return -2;
}

// Prepared-B variant (row-chunked dot pipeline): B' residues built once into a caller buffer.
int64_t mxh_crt_b_bytes(int words, int64_t batch, int64_t N, int64_t K, int mode) {
  if (words != 1 && words != 2) return 0;
  const CPlan p = make_cplan(words, batch, BM, N, K, mode);
  return p.n < 0 ? 0 : p.rb_bytes;
}

int mxh_crt_prep_b(int words, int64_t batch, int64_t K, int64_t N, const void* B0,
                   const void* B1, int mode, void* rb, void* stream) {
  const CPlan p = make_cplan(words, batch, BM, N, K, mode);
  if (p.n < 0) return -6;
  const Tables& tb = tables_for(words, p.n);
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    launch_prep<u64>(p, tb, true, batch, N, K, K * N, (const u64*)B0, (const u64*)B1, mode,
                     (int8_t*)rb, st);
  else if (words == 2)
    launch_prep<u128>(p, tb, true, batch, N, K, K * N, (const u128*)B0, (const u128*)B1, mode,
                      (int8_t*)rb, st);
  else
    return -2;
  const hipError_t e = hipGetLastError();
  return e != hipSuccess ? -100 - (int)e : 0;
}

int mxh_crt_with_b(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                   const void* A1, int64_t a_bstride, int mode, const void* rb, void* C,
                   int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (words == 1)
    return run_crt<u64>(batch, M, N, K, (const u64*)A0, (const u64*)A1, a_bstride, nullptr,
                        nullptr, 0, (const int8_t*)rb, mode, (u64*)C, accumulate, st);
  if (words == 2)
    return run_crt<u128>(batch, M, N, K, (const u128*)A0, (const u128*)A1, a_bstride, nullptr,
                         nullptr, 0, (const int8_t*)rb, mode, (u128*)C, accumulate, st);
  return -2;
}

}  // extern "C"
