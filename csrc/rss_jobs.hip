// Batched fixed-point products of ONE party (one party per GPU / process / thread: SPMD,
// in-process parties) -- the per-party dot tail (rss_party.hip k_dot_tail_r*) over a list
// of "jobs" instead of one dense product.
//
// A round of a per-party protocol often multiplies several independent pairs at once (the
// exp's polynomial level and product-tree level, moose_amd/protocols/fixedpoint.py
// _merged_exp_tail).  The generic path computed each pair's local cross terms in its own
// kernel, concatenated them, ran the tail on the concatenation and sliced / concatenated
// the results into the power stacks -- ~8 launches per round per party.  Here a round is
// the tail's three kernels: every job's cross terms are computed inside round 0 (no cross
// product tensor, no concatenation) and the new shares are written straight to each job's
// output rows (no slicing, no stacking).  Element i of the concatenation of the jobs' rows
// uses the same keystream chunk as element i of the concatenated tensor in the generic
// path, so the shares are bitwise those of cross + concat + k_dot_tail_r0/r1/r2.
//
// A job (row length L shared by all jobs of a call):
//   value[r, e] = cb * (x0 y0 + x0 y1 + x1 y0)  +  ca * a[r, e]  +  ca2 * a2[r, e]
// with x_k[r, e] = x_k[r * sx + e] (sx = 0: one row broadcast), y likewise, a / a2 with
// strides sa / sa2 (null: no term; additive shares, e.g. a party's first share component),
// cb = 0: no cross term.  Outputs o0 / o1 are dense [rows, L].
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "moosex.h"
#include "party_batch.h"
#include "prf_dev.h"
#include "ring_common.h"
#include "rss_fused.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

namespace {

constexpr int kMaxJobs = MX_MAX_JOBS;

struct JobD {
  const void* x0;
  const void* x1;
  const void* y0;
  const void* y1;
  const void* a;
  const void* a2;
  void* o0;
  void* o1;
  int64_t rows, sx, sy, sa, sa2, start;
  int64_t ca, ca2, cb;
};

// The previous level's round-2 sums, still pending (parallel/party.py jobs_tail, defer):
// region k of this party's output rows o[k][0, len[k]) is a[k] + b[k] (its w and the
// received w).  Round 0 of the next level reads its operands through them and also writes
// them (so later readers find the rows materialised): one launch instead of two.
struct Pend {
  const void* o[kMaxJobs];
  const void* a[kMaxJobs];
  const void* b[kMaxJobs];
  int64_t len[kMaxJobs];
  int64_t total;
  int n;
};

struct Jobs {
  JobD j[kMaxJobs];
  int n;
  int64_t L;
  Pend pend;
};

// operand element p[idx], or its pending sum when it lies in a pending region
template <class T>
__device__ __forceinline__ T ld(const Jobs& js, const void* p, int64_t idx) {
  const T* q = (const T*)p + idx;
  for (int k = 0; k < js.pend.n; ++k) {
    const T* o = (const T*)js.pend.o[k];
    if (q >= o && q < o + js.pend.len[k]) {
      const int64_t off = q - o;
      return ((const T*)js.pend.a[k])[off] + ((const T*)js.pend.b[k])[off];
    }
  }
  return *q;
}

// the pending regions' sums, written (grid-stride over all their elements)
template <class T>
__device__ __forceinline__ void fill_pending(const Jobs& js, int first = 0) {
  // threads [first, blockDim.x) of every block; the others are not delayed by it
  const int64_t per = blockDim.x - first;
  for (int64_t g = blockIdx.x * per + (threadIdx.x - first); g < js.pend.total;
       g += (int64_t)gridDim.x * per) {
    int64_t i = g;
    int k = 0;
    while (k < js.pend.n - 1 && i >= js.pend.len[k]) i -= js.pend.len[k++];
    ((T*)js.pend.o[k])[i] = ((const T*)js.pend.a[k])[i] + ((const T*)js.pend.b[k])[i];
  }
}

template <class T>
struct Loc {
  int q;
  int64_t r, e;
};

template <class T>
__device__ __forceinline__ Loc<T> locate(const Jobs& js, int64_t i) {
  int q = js.n - 1;
  while (q > 0 && i < js.j[q].start) --q;
  const int64_t k = i - js.j[q].start;
  return {q, k / js.L, k % js.L};
}

template <class T>
__device__ __forceinline__ T job_value(const Jobs& js, const Loc<T>& l) {
  const JobD& J = js.j[l.q];
  T v = 0;
  if (J.cb != 0) {
    const int64_t ix = l.r * J.sx + l.e, iy = l.r * J.sy + l.e;
    const T x0 = ld<T>(js, J.x0, ix), x1 = ld<T>(js, J.x1, ix);
    const T y0 = ld<T>(js, J.y0, iy), y1 = ld<T>(js, J.y1, iy);
    v = (T)J.cb * (x0 * y0 + x0 * y1 + x1 * y0);
  }
  if (J.a != nullptr) v += (T)J.ca * ld<T>(js, J.a, l.r * J.sa + l.e);
  if (J.a2 != nullptr) v += (T)J.ca2 * ld<T>(js, J.a2, l.r * J.sa2 + l.e);
  return v;
}

template <class T>
__device__ __forceinline__ T* job_out(const Jobs& js, const Loc<T>& l, int which) {
  const JobD& J = js.j[l.q];
  return (T*)(which == 0 ? J.o0 : J.o1) + l.r * js.L + l.e;
}

// Round 0 (rss_party.hip k_dot_tail_r0 for one component of role ``role``): P0 m0, P1 m1, P2
// z2 of the jobs' values (main != 0), and the dealer P2's rt1 / rm1 and its new shares
// (dealer != 0; independent of the values, so it may run before they exist).
template <class T>
__device__ __forceinline__ void
    d_jobs_r0(const Jobs& js, int64_t n, int m, int role, int main, int dealer, T* __restrict__ msg,
              T* __restrict__ msg_rt, u64* __restrict__ msg_rm, const mxd::KeySrc& keys,
              uint64_t n_a, uint64_t n_r0, uint64_t n_r1, uint64_t n_t, uint64_t n_m,
              uint64_t n_z0, uint64_t n_z2) {
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2);
  fill_pending<T>(js);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const uint32_t* own = rks[0];
  const uint32_t* nxt = rks[1];
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)nb);
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nblk;
       g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t B = (uint64_t)g;
    if (main) {
      uint32_t wa[16], wb[16], wr[16];
      if (role != 1) mx::chacha_block(own, n_a, B, wa);
      if (role != 0) mx::chacha_block(nxt, n_a, B, wb);
      if (role == 0) mx::chacha_block(own, n_r0, B, wr);
      if (role == 1) mx::chacha_block(nxt, n_r1, B, wr);
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const int64_t b = (int64_t)mx::ks_chunk(B, part);
        if (b >= nb) break;
        uint64_t al = 0, ah = 0, bl = 0, bh = 0, rl = 0, rh = 0;
        if (role != 1) mx::part_u64(wa, part, &al, &ah);
        if (role != 0) mx::part_u64(wb, part, &bl, &bh);
        if (role != 2) mx::part_u64(wr, part, &rl, &rh);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t i = b * P + j;
          if (i >= n) break;
          const Loc<T> l = locate<T>(js, i);
          const T z = job_value<T>(js, l) + mxd::pick<T>(al, ah, j) - mxd::pick<T>(bl, bh, j);
          if (role == 0)
            msg[i] = mxf::trunc_mask0<T>(z, (T)0, mxd::pick<T>(rl, rh, j));
          else if (role == 1)
            msg[i] = z + mxd::pick<T>(rl, rh, j);
          else
            msg[i] = z;
        }
      }
    }
    if (role == 2 && dealer) {
      uint32_t w[6][16];
      mx::chacha_block(nxt, n_r0, B, w[0]);
      mx::chacha_block(own, n_r1, B, w[1]);
      mx::chacha_block(nxt, n_t, B, w[2]);
      mx::chacha_block(nxt, n_m, B, w[3]);
      mx::chacha_block(nxt, n_z0, B, w[4]);
      mx::chacha_block(own, n_z2, B, w[5]);
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const int64_t b = (int64_t)mx::ks_chunk(B, part);
        if (b >= nb) break;
        uint64_t lo[6], hi[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) mx::part_u64(w[q], part, &lo[q], &hi[q]);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t i = b * P + j;
          if (i >= n) break;
          T rt1;
          u64 rm1;
          mxf::trunc_dealer<T>(mxd::pick<T>(lo[0], hi[0], j), mxd::pick<T>(lo[1], hi[1], j),
                               mxd::pick<T>(lo[2], hi[2], j), mxd::pick<T>(lo[3], hi[3], j), m,
                               &rt1, &rm1);
          msg_rt[i] = rt1;
          msg_rm[i] = rm1;
          const Loc<T> l = locate<T>(js, i);
          *job_out<T>(js, l, 0) = mxd::pick<T>(lo[5], hi[5], j);
          *job_out<T>(js, l, 1) = mxd::pick<T>(lo[4], hi[4], j);
        }
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256)
    k_jobs_r0(Jobs js, int64_t n, int m, int role, int main, int dealer, T* __restrict__ msg,
              T* __restrict__ msg_rt, u64* __restrict__ msg_rm, mxd::KeySrc keys,
              uint64_t n_a, uint64_t n_r0, uint64_t n_r1, uint64_t n_t, uint64_t n_m,
              uint64_t n_z0, uint64_t n_z2) {
  d_jobs_r0<T>(js, n, m, role, main, dealer, msg, msg_rt, msg_rm, keys, n_a, n_r0, n_r1, n_t,
               n_m, n_z0, n_z2);
}

// Round 1 (k_dot_tail_r1, one component): P0 / P1 open c, w = y - z; P0's o0 = z0, P1's
// o1 = z2 at the jobs' output rows.
template <class T>
__device__ __forceinline__ void
    d_jobs_r1(const Jobs& js, int64_t n, int m, int role, const T* __restrict__ mine,
              const T* __restrict__ other, const T* __restrict__ z2m, const T* __restrict__ rt,
              const u64* __restrict__ rm, T* __restrict__ wo, const mxd::KeySrc& keys, uint64_t n_t,
              uint64_t n_m, uint64_t n_z0, uint64_t n_z2) {
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2);
  if (role != 0 && role != 1) return;
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)nb);
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nblk;
       g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t B = (uint64_t)g;
    uint32_t wt[16], wm[16], wz[16];
    if (role == 0) {
      mx::chacha_block(rks[0], n_t, B, wt);
      mx::chacha_block(rks[0], n_m, B, wm);
      mx::chacha_block(rks[0], n_z0, B, wz);
    } else {
      mx::chacha_block(rks[1], n_z2, B, wz);
    }
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int64_t b = (int64_t)mx::ks_chunk(B, part);
      if (b >= nb) break;
      uint64_t tl = 0, th = 0, ml = 0, mh = 0, zl, zh;
      if (role == 0) {
        mx::part_u64(wt, part, &tl, &th);
        mx::part_u64(wm, part, &ml, &mh);
      }
      mx::part_u64(wz, part, &zl, &zh);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = b * P + j;
        if (i >= n) break;
        T cc = mine[i] + other[i];
        if (z2m != nullptr) cc += z2m[i];
        const T z = mxd::pick<T>(zl, zh, j);
        const T y = role == 0 ? mxf::trunc_y<T>(cc, mxd::pick<T>(tl, th, j),
                                                mxd::pick<T>(ml, mh, j), m, true)
                              : mxf::trunc_y<T>(cc, rt[i], (T)rm[i], m, false);
        wo[i] = y - z;
        *job_out<T>(js, locate<T>(js, i), role == 0 ? 0 : 1) = z;
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256)
    k_jobs_r1(Jobs js, int64_t n, int m, int role, const T* __restrict__ mine,
              const T* __restrict__ other, const T* __restrict__ z2m, const T* __restrict__ rt,
              const u64* __restrict__ rm, T* __restrict__ wo, mxd::KeySrc keys, uint64_t n_t,
              uint64_t n_m, uint64_t n_z0, uint64_t n_z2) {
  d_jobs_r1<T>(js, n, m, role, mine, other, z2m, rt, rm, wo, keys, n_t, n_m, n_z0, n_z2);
}

// Round 2 (k_dot_tail_r2, one component): P0's o1 / P1's o0 = w0 + w1.
template <class T>
__device__ __forceinline__ void
    d_jobs_r2(const Jobs& js, int64_t n, int role, const T* __restrict__ a,
              const T* __restrict__ b) {
  if (role != 0 && role != 1) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    *job_out<T>(js, locate<T>(js, i), role == 0 ? 1 : 0) = a[i] + b[i];
}

template <class T>
__global__ void __launch_bounds__(256)
    k_jobs_r2(Jobs js, int64_t n, int role, const T* __restrict__ a, const T* __restrict__ b) {
  d_jobs_r2<T>(js, n, role, a, b);
}


// ---- latency forms (small launches: the per-party LR inference's 128-element tails) ----
// The keystream chunks of a block's EPB chunk positions, for every stream the role draws,
// are computed one per thread into LDS (one ChaCha block per thread on the critical path
// instead of up to eight in sequence); then EPB threads finish the elements.  Same
// streams, same chunks, same values as the walking kernels above.
constexpr int kLatEpb = 32;

struct Streams {
  int n;
  int key[8];  // 0 = own (k_p), 1 = next (k_{p+1})
  uint64_t nonce[8];
};

template <class T>
__device__ __forceinline__ void
    d_jobs_r0_lat(const Jobs& js, int64_t n, int m, int role, int main, int dealer,
                  T* __restrict__ msg, T* __restrict__ msg_rt, u64* __restrict__ msg_rm,
                  const mxd::KeySrc& keys, const Streams& ss) {
  // streams: main 0..1 (P0: a, r; P1: b, r; P2: a, b), dealer 2..7 (P2: r0, r1, t, m, z0, z2)
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  __shared__ uint64_t kl[8][kLatEpb], kh[8][kLatEpb];
  mxd::stage_keys(rks, keys, 2);
  // the pending sums by the waves that draw no keystream chunk (P0 / P1 draw 2 streams:
  // waves 1-3), beside the finishing wave 0 instead of before it
  const int fill_from = ss.n * kLatEpb < (int)blockDim.x ? ss.n * kLatEpb : 0;
  if ((int)threadIdx.x >= fill_from) fill_pending<T>(js, fill_from);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / kLatEpb, lb = tid % kLatEpb;
  for (int64_t b0 = (int64_t)blockIdx.x * kLatEpb; b0 < nb; b0 += (int64_t)gridDim.x * kLatEpb) {
    const bool fin = tid < kLatEpb && b0 + tid < nb;
    T val[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t i = (b0 + tid) * P + j;
      val[j] = (fin && main && i < n) ? job_value<T>(js, locate<T>(js, i)) : (T)0;
    }
    if (s < ss.n && b0 + lb < nb) {
      uint64_t lo, hi;
      mxd::prf_chunk(rks[ss.key[s]], ss.nonce[s], (uint64_t)(b0 + lb), &lo, &hi);
      kl[s][lb] = lo;
      kh[s][lb] = hi;
    }
    __syncthreads();
    if (fin) {
      const int64_t b = b0 + tid;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = b * P + j;
        if (i >= n) break;
        if (main) {
          const T k0 = mxd::pick<T>(kl[0][tid], kh[0][tid], j);
          const T k1 = mxd::pick<T>(kl[1][tid], kh[1][tid], j);
          if (role == 0)
            msg[i] = mxf::trunc_mask0<T>(val[j] + k0, (T)0, k1);
          else if (role == 1)
            msg[i] = val[j] - k0 + k1;
          else
            msg[i] = val[j] + k0 - k1;
        }
        if (role == 2 && dealer) {
          T rt1;
          u64 rm1;
          mxf::trunc_dealer<T>(mxd::pick<T>(kl[2][tid], kh[2][tid], j),
                               mxd::pick<T>(kl[3][tid], kh[3][tid], j),
                               mxd::pick<T>(kl[4][tid], kh[4][tid], j),
                               mxd::pick<T>(kl[5][tid], kh[5][tid], j), m, &rt1, &rm1);
          msg_rt[i] = rt1;
          msg_rm[i] = rm1;
          const Loc<T> l = locate<T>(js, i);
          *job_out<T>(js, l, 0) = mxd::pick<T>(kl[7][tid], kh[7][tid], j);
          *job_out<T>(js, l, 1) = mxd::pick<T>(kl[6][tid], kh[6][tid], j);
        }
      }
    }
    __syncthreads();
  }
}

template <class T>
__global__ void __launch_bounds__(256)
    k_jobs_r0_lat(Jobs js, int64_t n, int m, int role, int main, int dealer, T* __restrict__ msg,
                  T* __restrict__ msg_rt, u64* __restrict__ msg_rm, mxd::KeySrc keys,
                  Streams ss) {
  d_jobs_r0_lat<T>(js, n, m, role, main, dealer, msg, msg_rt, msg_rm, keys, ss);
}

template <class T>
__device__ __forceinline__ void
    d_jobs_r1_lat(const Jobs& js, int64_t n, int m, int role, const T* __restrict__ mine,
                  const T* __restrict__ other, const T* __restrict__ z2m,
                  const T* __restrict__ rt, const u64* __restrict__ rm, T* __restrict__ wo,
                  const mxd::KeySrc& keys, const Streams& ss) {
  // streams: P0 t, m, z0 (own); P1 z2 (next) -- at index 2
  __shared__ uint32_t rks[2][mxd::kKeyWords];
  __shared__ uint64_t kl[3][kLatEpb], kh[3][kLatEpb];
  mxd::stage_keys(rks, keys, 2);
  if (role != 0 && role != 1) return;
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  const int tid = threadIdx.x, s = tid / kLatEpb, lb = tid % kLatEpb;
  for (int64_t b0 = (int64_t)blockIdx.x * kLatEpb; b0 < nb; b0 += (int64_t)gridDim.x * kLatEpb) {
    const bool fin = tid < kLatEpb && b0 + tid < nb;
    T cc[P], r1t[P], r1m[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int64_t i = (b0 + tid) * P + j;
      const bool ok = fin && i < n;
      cc[j] = ok ? (T)(mine[i] + other[i] + (z2m != nullptr ? z2m[i] : (T)0)) : (T)0;
      r1t[j] = ok && role == 1 ? rt[i] : (T)0;
      r1m[j] = ok && role == 1 ? (T)rm[i] : (T)0;
    }
    const int slot = role == 0 ? s : 2;  // P1 draws z2 only, kept in slot 2
    if (s < ss.n && b0 + lb < nb) {
      uint64_t lo, hi;
      mxd::prf_chunk(rks[ss.key[s]], ss.nonce[s], (uint64_t)(b0 + lb), &lo, &hi);
      kl[slot][lb] = lo;
      kh[slot][lb] = hi;
    }
    __syncthreads();
    if (fin) {
      const int64_t b = b0 + tid;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = b * P + j;
        if (i >= n) break;
        const T z = mxd::pick<T>(kl[2][tid], kh[2][tid], j);
        const T y = role == 0 ? mxf::trunc_y<T>(cc[j], mxd::pick<T>(kl[0][tid], kh[0][tid], j),
                                                mxd::pick<T>(kl[1][tid], kh[1][tid], j), m, true)
                              : mxf::trunc_y<T>(cc[j], r1t[j], r1m[j], m, false);
        wo[i] = y - z;
        *job_out<T>(js, locate<T>(js, i), role == 0 ? 0 : 1) = z;
      }
    }
    __syncthreads();
  }
}

template <class T>
__global__ void __launch_bounds__(256)
    k_jobs_r1_lat(Jobs js, int64_t n, int m, int role, const T* __restrict__ mine,
                  const T* __restrict__ other, const T* __restrict__ z2m,
                  const T* __restrict__ rt, const u64* __restrict__ rm, T* __restrict__ wo,
                  mxd::KeySrc keys, Streams ss) {
  d_jobs_r1_lat<T>(js, n, m, role, mine, other, z2m, rt, rm, wo, keys, ss);
}

// party-batched twins for the composed one-GPU replay (party_batch.h)
MX_X3_GS(k_jobs_r0<u128>, d_jobs_r0<u128>);
MX_X3_GS(k_jobs_r1<u64>, d_jobs_r1<u64>);
MX_X3_GS(k_jobs_r1<u128>, d_jobs_r1<u128>);
MX_X3_GS(k_jobs_r2<u64>, d_jobs_r2<u64>);
MX_X3_GS(k_jobs_r2<u128>, d_jobs_r2<u128>);
MX_X3_GS(k_jobs_r0_lat<u64>, d_jobs_r0_lat<u64>);
MX_X3_GS(k_jobs_r0_lat<u128>, d_jobs_r0_lat<u128>);
MX_X3_GS(k_jobs_r1_lat<u64>, d_jobs_r1_lat<u64>);
MX_X3_GS(k_jobs_r1_lat<u128>, d_jobs_r1_lat<u128>);

// the latency forms run while the launch has at most this many chunk positions
constexpr int64_t kLatMaxChunks = 1 << 14;

bool lat_on() {  // MOOSEX_JOBS_LAT=0: the walking kernels at every size (A/B comparisons)
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_JOBS_LAT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// host: the flat (ptrs[8 q .. 8 q + 7], dims[8 q .. 8 q + 7]) job description
int make_jobs(int njobs, const void* const* ptrs, const int64_t* dims, int64_t L, Jobs* js,
              int64_t* n) {
  if (njobs < 1 || njobs > kMaxJobs || L < 1) return -3;
  js->n = njobs;
  js->L = L;
  js->pend = Pend{};
  int64_t at = 0;
  for (int q = 0; q < kMaxJobs; ++q) {
    JobD& J = js->j[q];
    if (q >= njobs) {
      J = JobD{};
      J.start = INT64_MAX;
      continue;
    }
    const void* const* pq = ptrs + 8 * q;
    const int64_t* dq = dims + 8 * q;
    J.x0 = pq[0];
    J.x1 = pq[1];
    J.y0 = pq[2];
    J.y1 = pq[3];
    J.a = pq[4];
    J.a2 = pq[5];
    J.o0 = const_cast<void*>(pq[6]);
    J.o1 = const_cast<void*>(pq[7]);
    J.rows = dq[0];
    J.sx = dq[1];
    J.sy = dq[2];
    J.sa = dq[3];
    J.sa2 = dq[4];
    J.ca = dq[5];
    J.ca2 = dq[6];
    J.cb = dq[7];
    J.start = at;
    at += J.rows * L;
  }
  *n = at;
  return 0;
}

}  // namespace

extern "C" {

int mxh_jobs_r0p(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                 int m, int role, int main, int dealer, void* msg, void* msg_rt, void* msg_rm,
                 const uint32_t* const* slots, const uint64_t* nn, int npend,
                 const void* const* pend, const int64_t* pend_len, void* stream) {
  Jobs js;
  int64_t n = 0;
  int rc = make_jobs(njobs, ptrs, dims, L, &js, &n);
  if (rc) return rc;
  if (npend < 0 || npend > kMaxJobs) return -3;
  js.pend.n = npend;
  for (int k = 0; k < npend; ++k) {
    js.pend.o[k] = pend[3 * k];
    js.pend.a[k] = pend[3 * k + 1];
    js.pend.b[k] = pend[3 * k + 2];
    js.pend.len[k] = pend_len[k];
    js.pend.total += pend_len[k];
  }
  if (n == 0) return 0;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2);
  hipStream_t st = (hipStream_t)stream;
  const int64_t nchunks = words == 1 ? (n + 1) / 2 : n;
  if (nchunks <= kLatMaxChunks && lat_on()) {
    Streams ss{};
    // main: P0 a (own), r0 (own); P1 b (next), r1 (next); P2 a (own), b (next)
    const int mk[3][2] = {{0, 0}, {1, 1}, {0, 1}};
    const uint64_t mn[3][2] = {{nn[0], nn[1]}, {nn[0], nn[2]}, {nn[0], nn[0]}};
    ss.n = 2;
    for (int q = 0; q < 2; ++q) {
      ss.key[q] = mk[role][q];
      ss.nonce[q] = mn[role][q];
    }
    if (role == 2 && dealer) {  // r0 (next), r1 (own), t, m, z0 (next), z2 (own)
      const int dk[6] = {1, 0, 1, 1, 1, 0};
      for (int q = 0; q < 6; ++q) {
        ss.key[2 + q] = dk[q];
        ss.nonce[2 + q] = nn[1 + q];
      }
      ss.n = 8;
    }
    const dim3 grid((unsigned)((nchunks + kLatEpb - 1) / kLatEpb));
    if (words == 1)
      hipLaunchKernelGGL(k_jobs_r0_lat<u64>, grid, dim3(256), 0, st, js, n, m, role, main, dealer,
                         (u64*)msg, (u64*)msg_rt, (u64*)msg_rm, k, ss);
    else if (words == 2)
      hipLaunchKernelGGL(k_jobs_r0_lat<u128>, grid, dim3(256), 0, st, js, n, m, role, main,
                         dealer, (u128*)msg, (u128*)msg_rt, (u64*)msg_rm, k, ss);
    else
      return -2;
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -100 - (int)e;
  }
  if (words == 1)
    hipLaunchKernelGGL(k_jobs_r0<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2)), dim3(256), 0, st,
                       js, n, m, role, main, dealer, (u64*)msg, (u64*)msg_rt, (u64*)msg_rm, k,
                       nn[0], nn[1], nn[2], nn[3], nn[4], nn[5], nn[6]);
  else if (words == 2)
    hipLaunchKernelGGL(k_jobs_r0<u128>, dim3(mxd::grid_for_chunks(n)), dim3(256), 0, st, js, n, m,
                       role, main, dealer, (u128*)msg, (u128*)msg_rt, (u64*)msg_rm, k, nn[0],
                       nn[1], nn[2], nn[3], nn[4], nn[5], nn[6]);
  else
    return -2;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_jobs_r0(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                int m, int role, int main, int dealer, void* msg, void* msg_rt, void* msg_rm,
                const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  return mxh_jobs_r0p(words, njobs, ptrs, dims, L, m, role, main, dealer, msg, msg_rt, msg_rm,
                      slots, nn, 0, nullptr, nullptr, stream);
}

int mxh_jobs_r1(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                int m, int role, const void* msg, const void* rmk, const void* rz,
                const void* rrt, const void* rrm, void* w, const uint32_t* const* slots,
                const uint64_t* nn, void* stream) {
  Jobs js;
  int64_t n = 0;
  int rc = make_jobs(njobs, ptrs, dims, L, &js, &n);
  if (rc) return rc;
  if (n == 0) return 0;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2);
  hipStream_t st = (hipStream_t)stream;
  if (role != 0 && role != 1) return 0;
  const int64_t nchunks = words == 1 ? (n + 1) / 2 : n;
  if (nchunks <= kLatMaxChunks && lat_on()) {
    Streams ss{};
    if (role == 0) {  // t, m, z0 under own
      ss.n = 3;
      for (int q = 0; q < 3; ++q) {
        ss.key[q] = 0;
        ss.nonce[q] = nn[3 + q];
      }
    } else {  // z2 under next
      ss.n = 1;
      ss.key[0] = 1;
      ss.nonce[0] = nn[6];
    }
    const dim3 grid((unsigned)((nchunks + kLatEpb - 1) / kLatEpb));
    if (words == 1)
      hipLaunchKernelGGL(k_jobs_r1_lat<u64>, grid, dim3(256), 0, st, js, n, m, role,
                         (const u64*)msg, (const u64*)rmk, (const u64*)rz, (const u64*)rrt,
                         (const u64*)rrm, (u64*)w, k, ss);
    else if (words == 2)
      hipLaunchKernelGGL(k_jobs_r1_lat<u128>, grid, dim3(256), 0, st, js, n, m, role,
                         (const u128*)msg, (const u128*)rmk, (const u128*)rz, (const u128*)rrt,
                         (const u64*)rrm, (u128*)w, k, ss);
    else
      return -2;
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -100 - (int)e;
  }
  if (words == 1)
    hipLaunchKernelGGL(k_jobs_r1<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2)), dim3(256), 0, st,
                       js, n, m, role, (const u64*)msg, (const u64*)rmk, (const u64*)rz,
                       (const u64*)rrt, (const u64*)rrm, (u64*)w, k, nn[3], nn[4], nn[5], nn[6]);
  else if (words == 2)
    hipLaunchKernelGGL(k_jobs_r1<u128>, dim3(mxd::grid_for_chunks(n)), dim3(256), 0, st, js, n, m,
                       role, (const u128*)msg, (const u128*)rmk, (const u128*)rz,
                       (const u128*)rrt, (const u64*)rrm, (u128*)w, k, nn[3], nn[4], nn[5],
                       nn[6]);
  else
    return -2;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_jobs_r2(int words, int njobs, const void* const* ptrs, const int64_t* dims, int64_t L,
                int role, const void* a, const void* b, void* stream) {
  Jobs js;
  int64_t n = 0;
  int rc = make_jobs(njobs, ptrs, dims, L, &js, &n);
  if (rc) return rc;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int grid = mxd::grid_for(n);
  if (words == 1)
    hipLaunchKernelGGL(k_jobs_r2<u64>, dim3(grid), dim3(256), 0, st, js, n, role,
                       (const u64*)a, (const u64*)b);
  else if (words == 2)
    hipLaunchKernelGGL(k_jobs_r2<u128>, dim3(grid), dim3(256), 0, st, js, n, role,
                       (const u128*)a, (const u128*)b);
  else
    return -2;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

}  // extern "C"
