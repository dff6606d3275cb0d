// Per-party protocol kernels for layouts where the three parties of a session sit on
// DIFFERENT GPUs (moose_amd/parallel/cyclic.py): a GPU stacks one party of each of up to
// three sessions, component c playing role roles[c].  Each kernel does every stacked
// role's local work of one protocol round in one pass; the messages between rounds go
// over RCCL.  Same PRF keys / nonces / counters as the generic protocol code, so the shares
// are bitwise equal to it (and to the single-GPU fused kernels of rss_fused.hip).
//
// TruncPr (dealer P2, reference additive/trunc.rs:114-170), rounds:
//   r0: P0 mk0 = x0 + x1 + 2^(k-2) + r0          -> P1
//       P1 mk1 = x2 + r1                          -> P0
//       P2 rt1, rm1 (dealer shares for P1)        -> P1;  P2's new shares (z2, z0)
//   r1: P0 c = mk0 + mk1, y0, w0 = y0 - z0        -> P1;  P0's s0 = z0
//       P1 c = mk1 + mk0, y1, w1 = y1 - z2        -> P0;  P1's s1 = z2
//   r2: z1 = w0 + w1 (elementwise, host side)
// Share by member j: one kernel computing every role's two slots (the owner's masked
// x_j is then sent to P_{j+2}).
// Key slots: component c passes (own k_p, next k_{p+1}[, k_all]) of its session.
#include <hip/hip_runtime.h>

#include "prf_dev.h"
#include "moosex.h"
#include "party_batch.h"
#include "ring_common.h"
#include "rss_fused.h"

using u64 = uint64_t;
using u128 = unsigned __int128;

namespace {

struct Roles {
  int r[3];
};

// Each thread walks ChaCha blocks (prf_dev.h) of one component: g = c * nblk + B, and the
// body runs for the block's chunks b = ks_chunk(B, part).
#define MX_PARTY_WALK(NB, NCOMP)                                                    \
  const int64_t nblk = (int64_t)mx::ks_blocks_for((uint64_t)(NB));               \
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nblk * (NCOMP); \
       g += (int64_t)gridDim.x * blockDim.x)

template <class T>
__device__ __forceinline__ void d_trunc_party_r0(int64_t n, int m, const Roles& roles,
                                                 const T* __restrict__ s0, const T* __restrict__ s1,
                                                 T* __restrict__ msg, u64* __restrict__ msg_rm,
                                                 T* __restrict__ out0, T* __restrict__ out1,
                                                 const mxd::KeySrc& keys, uint64_t n_r0,
                                                 uint64_t n_r1, uint64_t n_t, uint64_t n_m,
                                                 uint64_t n_z0, uint64_t n_z2, int ncomp) {
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2 * ncomp);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  MX_PARTY_WALK(nb, ncomp) {
    const int c = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - c * nblk);
    const int role = roles.r[c];
    const uint32_t* own = rks[2 * c];
    const uint32_t* nxt = rks[2 * c + 1];
    const int64_t base = (int64_t)c * n;
    if (role == 0) {  // k0 = own
      uint32_t wa[16];
      mx::chacha_block(own, n_r0, B, wa);
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const int64_t b = (int64_t)mx::ks_chunk(B, part);
        if (b >= nb) break;
        uint64_t al, ah;
        mx::part_u64(wa, part, &al, &ah);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t i = b * P + j;
          if (i >= n) break;
          msg[base + i] = mxf::trunc_mask0<T>(s0[base + i], s1[base + i], mxd::pick<T>(al, ah, j));
        }
      }
    } else if (role == 1) {  // k2 = next
      uint32_t wa[16];
      mx::chacha_block(nxt, n_r1, B, wa);
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const int64_t b = (int64_t)mx::ks_chunk(B, part);
        if (b >= nb) break;
        uint64_t al, ah;
        mx::part_u64(wa, part, &al, &ah);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t i = b * P + j;
          if (i >= n) break;
          msg[base + i] = s1[base + i] + mxd::pick<T>(al, ah, j);
        }
      }
    } else if (role == 2) {  // k2 = own, k0 = next
      // streams r0, r1, t, m, z0, z2
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
          msg[base + i] = rt1;
          msg_rm[base + i] = rm1;
          out0[base + i] = mxd::pick<T>(lo[5], hi[5], j);
          out1[base + i] = mxd::pick<T>(lo[4], hi[4], j);
        }
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_trunc_party_r0(int64_t n, int m, Roles roles,
                                                        const T* __restrict__ s0,
                                                        const T* __restrict__ s1,
                                                        T* __restrict__ msg,
                                                        u64* __restrict__ msg_rm,
                                                        T* __restrict__ out0, T* __restrict__ out1,
                                                        mxd::KeySrc keys, uint64_t n_r0,
                                                        uint64_t n_r1, uint64_t n_t, uint64_t n_m,
                                                        uint64_t n_z0, uint64_t n_z2, int ncomp) {
  d_trunc_party_r0<T>(n, m, roles, s0, s1, msg, msg_rm, out0, out1, keys, n_r0, n_r1, n_t, n_m,
                      n_z0, n_z2, ncomp);
}

template <class T>
__device__ __forceinline__ void d_trunc_party_r1(int64_t n, int m, const Roles& roles,
                                                 const T* __restrict__ msg,
                                                 const T* __restrict__ rmk,
                                                 const T* __restrict__ rrt,
                                                 const u64* __restrict__ rrm, T* __restrict__ w,
                                                 T* __restrict__ out0, T* __restrict__ out1,
                                                 const mxd::KeySrc& keys, uint64_t n_t,
                                                 uint64_t n_m, uint64_t n_z0, uint64_t n_z2,
                                                 int ncomp) {
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2 * ncomp);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  MX_PARTY_WALK(nb, ncomp) {
    const int c = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - c * nblk);
    const int role = roles.r[c];
    const int64_t base = (int64_t)c * n;
    if (role == 0) {
      const uint32_t* k0 = rks[2 * c];
      uint32_t wt[16], wm[16], wz[16];
      mx::chacha_block(k0, n_t, B, wt);
      mx::chacha_block(k0, n_m, B, wm);
      mx::chacha_block(k0, n_z0, B, wz);
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const int64_t b = (int64_t)mx::ks_chunk(B, part);
        if (b >= nb) break;
        uint64_t tl, th, ml, mh, zl, zh;
        mx::part_u64(wt, part, &tl, &th);
        mx::part_u64(wm, part, &ml, &mh);
        mx::part_u64(wz, part, &zl, &zh);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t i = b * P + j;
          if (i >= n) break;
          const T cc = msg[base + i] + rmk[base + i];
          const T z0 = mxd::pick<T>(zl, zh, j);
          const T y0 = mxf::trunc_y<T>(cc, mxd::pick<T>(tl, th, j), mxd::pick<T>(ml, mh, j), m, true);
          w[base + i] = y0 - z0;
          out0[base + i] = z0;
        }
      }
    } else if (role == 1) {
      const uint32_t* k2 = rks[2 * c + 1];
      uint32_t wz[16];
      mx::chacha_block(k2, n_z2, B, wz);
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const int64_t b = (int64_t)mx::ks_chunk(B, part);
        if (b >= nb) break;
        uint64_t zl, zh;
        mx::part_u64(wz, part, &zl, &zh);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int64_t i = b * P + j;
          if (i >= n) break;
          const T cc = msg[base + i] + rmk[base + i];
          const T z2 = mxd::pick<T>(zl, zh, j);
          const T y1 = mxf::trunc_y<T>(cc, rrt[base + i], (T)rrm[base + i], m, false);
          w[base + i] = y1 - z2;
          out1[base + i] = z2;
        }
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_trunc_party_r1(int64_t n, int m, Roles roles,
                                                        const T* __restrict__ msg,
                                                        const T* __restrict__ rmk,
                                                        const T* __restrict__ rrt,
                                                        const u64* __restrict__ rrm,
                                                        T* __restrict__ w, T* __restrict__ out0,
                                                        T* __restrict__ out1, mxd::KeySrc keys,
                                                        uint64_t n_t, uint64_t n_m, uint64_t n_z0,
                                                        uint64_t n_z2, int ncomp) {
  d_trunc_party_r1<T>(n, m, roles, msg, rmk, rrt, rrm, w, out0, out1, keys, n_t, n_m, n_z0, n_z2,
                      ncomp);
}

template <class T>
__device__ __forceinline__ void d_share_party(int kind, int64_t n, const Roles& rel,
                                              const void* __restrict__ xv, T* __restrict__ out0,
                                              T* __restrict__ out1, const mxd::KeySrc& keys,
                                              uint64_t n1, uint64_t na, int ncomp) {
  const bool mir = kind & MX_SHARE_MIRROR;
  kind &= ~MX_SHARE_MIRROR;
  const T* x = (const T*)xv;
  const double* xf = (const double*)xv;  // kind MX_SHARE_F64: encode in the kernel
  const double scale = kind == MX_SHARE_F64 ? ldexp(1.0, (int)na) : 0.0;
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  // keys: 2 per component, the first used: k_j of the owner j (rel 0: own, rel 2: next).
  // As the reference (replicated/convert.rs:74-90): slot j = PRF(k_j), slot j+1 = x - slot j
  // (sent to P_{j+1}), slot j+2 = 0, so rel 1 draws nothing.  Mirrored (MX_SHARE_MIRROR):
  // slot j+1 = PRF(k_{j+1}) (rel 0: next, rel 1: own), slot j = x - slot j+1 (sent to
  // P_{j+2}), slot j+2 = 0, so rel 2 draws nothing
  mxd::stage_keys(rks, keys, 2 * ncomp);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  MX_PARTY_WALK(nb, ncomp) {
    const int c = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - c * nblk);
    // rel code: the role relative to the owner (0..2) + 4 * (1 + the component of the
    // recipient P_{j+1}, mirrored P_{j+2}) when the owner's masked share stays on this device
    // (written straight into its s0, mirrored its s1)
    const int code = rel.r[c];
    if (code < 0) continue;
    const int r = code & 3, fwd = (code >> 2) - 1;
    const int64_t base = (int64_t)c * n;
    if (r > 2) continue;
    const bool draws = mir ? r != 2 : r != 1;
    uint32_t wa[16];
    if (draws) mx::chacha_block(rks[2 * c], n1, B, wa);
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int64_t b = (int64_t)mx::ks_chunk(B, part);
      if (b >= nb) break;
      uint64_t al = 0, ah = 0;
      if (draws) mx::part_u64(wa, part, &al, &ah);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int64_t i = b * P + j;
        if (i >= n) break;
        const T rr = mxd::pick<T>(al, ah, j);
        if (r == 0) {  // owner: (PRF(k_j), x - PRF(k_j)); mirrored (x - PRF(k_{j+1}), PRF)
          const T xi = kind == MX_SHARE_F64 ? (T)mxr::f64_to_i128(xf[i] * scale) : x[i];
          const T v = kind == MX_CROSS_BOOL ? (T)(xi ^ rr) : (T)(xi - rr);
          out0[base + i] = mir ? v : rr;
          out1[base + i] = mir ? rr : v;
          if (fwd >= 0) (mir ? out1 : out0)[(int64_t)fwd * n + i] = v;
        } else if (r == 1) {  // P_{j+1}: (received, 0); mirrored (PRF(k_{j+1}), 0)
          if (mir) out0[base + i] = rr;
          out1[base + i] = 0;
        } else {  // P_{j+2}: (0, PRF(k_j)); mirrored (0, received)
          out0[base + i] = 0;
          if (!mir) out1[base + i] = rr;
        }
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_share_party(int kind, int64_t n, Roles rel,
                                                     const void* __restrict__ xv,
                                                     T* __restrict__ out0, T* __restrict__ out1,
                                                     mxd::KeySrc keys, uint64_t n1, uint64_t na,
                                                     int ncomp) {
  d_share_party<T>(kind, n, rel, xv, out0, out1, keys, n1, na, ncomp);
}

inline Roles roles_of(const int* r, int ncomp) {
  Roles o;
  for (int c = 0; c < 3; ++c) o.r[c] = c < ncomp ? r[c] : -1;
  return o;
}


// ---------------------------------------------------------------------------------------
// Fixed-point dot tail (rep.dot_trunc) for parties on different GPUs.  Input: each party's
// local cross products (the RSS dot's GEMM output).  The reshare of rep.dot is folded into
// TruncPr's first round: P_p's product masked by the zero share is z_p (3-out-of-3
// additive), and the opening c = x + r + 2^(k-2) of TruncPr is assembled from
//   P0: m0 = z0 + 2^(k-2) + r0   -> P1
//   P1: m1 = z1 + r1              -> P0
//   P2: z2                        -> P0 and P1        (+ the dealer's rt1, rm1 -> P1)
// so both P0 and P1 get c = m0 + m1 + z2 in ONE round (the generic path needs the
// reshare round plus the P0 <-> P1 round).  c is the same value, and every output share
// depends on the input only through c, so the shares are bitwise equal to reshare +
// TruncPr (and to the stacked fused kernel).  Round 1 is k_trunc_party_r1's with the
// three-term c; round 2 adds the exchanged w's.  Every array argument is a per-component
// pointer triple (component slots need not be adjacent: rows of a larger stack, buffers
// received from other GPUs, or -- one party per process at N = 1 -- the sender's buffer).
// ---------------------------------------------------------------------------------------
struct CP3 {
  const void* p[3];
};
struct WP3 {
  void* p[3];
};

template <class T>
__device__ __forceinline__ const T* cp(const CP3& a, int c) {
  return (const T*)a.p[c];
}
template <class T>
__device__ __forceinline__ T* wp(const WP3& a, int c) {
  return (T*)a.p[c];
}

template <class T>
__device__ __forceinline__ void d_dot_tail_r0(int64_t n, int m, const Roles& roles,
                                              const CP3& cross, const WP3& msg, const WP3& msg_rt,
                                              const WP3& msg_rm, const WP3& out0, const WP3& out1,
                                              const mxd::KeySrc& keys, uint64_t n_a, uint64_t n_r0,
                                              uint64_t n_r1, uint64_t n_t, uint64_t n_m,
                                              uint64_t n_z0, uint64_t n_z2, int ncomp) {
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2 * ncomp);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  MX_PARTY_WALK(nb, ncomp) {
    const int c = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - c * nblk);
    const int role = roles.r[c];
    if (role < 0 || role > 2) continue;
    const uint32_t* own = rks[2 * c];
    const uint32_t* nxt = rks[2 * c + 1];
    const T* x = cp<T>(cross, c);
    T* mo = wp<T>(msg, c);
    // no cross (null): the dealer part only, launched before the product exists, so P2's
    // rt1 / rm1 travel while the GEMM runs; no msg_rt (null): no dealer part
    if (x != nullptr) {
      // zero share alpha: P0 f(k0), P1 -f(k2), P2 f(k2) - f(k0) (f = PRF at nonce n_a; sums
      // to zero).  z2 (sent to P0 and P1) is masked by f(k2) against P0 and f(k0) against
      // P1, m0 / m1 by the opening masks r0 / r1: every view is as with the textbook
      // alpha_p = f(k_p) - f(k_{p+1}), with one PRF stream less at P0 and at P1
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
          const T z = x[i] + mxd::pick<T>(al, ah, j) - mxd::pick<T>(bl, bh, j);
          if (role == 0)
            mo[i] = mxf::trunc_mask0<T>(z, (T)0, mxd::pick<T>(rl, rh, j));
          else if (role == 1)
            mo[i] = z + mxd::pick<T>(rl, rh, j);
          else
            mo[i] = z;
        }
      }
    }
    if (role == 2 && msg_rt.p[c] != nullptr) {  // dealer (as k_trunc_party_r0): r0, r1, t, m, z0, z2
      uint32_t w[6][16];
      mx::chacha_block(nxt, n_r0, B, w[0]);
      mx::chacha_block(own, n_r1, B, w[1]);
      mx::chacha_block(nxt, n_t, B, w[2]);
      mx::chacha_block(nxt, n_m, B, w[3]);
      mx::chacha_block(nxt, n_z0, B, w[4]);
      mx::chacha_block(own, n_z2, B, w[5]);
      T* rt = wp<T>(msg_rt, c);
      u64* rm = wp<u64>(msg_rm, c);
      T* o0 = wp<T>(out0, c);
      T* o1 = wp<T>(out1, c);
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
          rt[i] = rt1;
          rm[i] = rm1;
          o0[i] = mxd::pick<T>(lo[5], hi[5], j);
          o1[i] = mxd::pick<T>(lo[4], hi[4], j);
        }
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_dot_tail_r0(int64_t n, int m, Roles roles, CP3 cross,
                                                     WP3 msg, WP3 msg_rt, WP3 msg_rm, WP3 out0,
                                                     WP3 out1, mxd::KeySrc keys, uint64_t n_a,
                                                     uint64_t n_r0, uint64_t n_r1, uint64_t n_t,
                                                     uint64_t n_m, uint64_t n_z0, uint64_t n_z2,
                                                     int ncomp) {
  d_dot_tail_r0<T>(n, m, roles, cross, msg, msg_rt, msg_rm, out0, out1, keys, n_a, n_r0, n_r1, n_t,
                   n_m, n_z0, n_z2, ncomp);
}

// P0 / P1: c = own message + the other's + z2 (rz may be null: the two-term opening of
// k_trunc_party_r0's protocol), then y, w = y - z and the PRF share of the new sharing.
template <class T>
__device__ __forceinline__ void d_dot_tail_r1(int64_t n, int m, const Roles& roles, const CP3& msg,
                                              const CP3& rmk, const CP3& rz, const CP3& rrt,
                                              const CP3& rrm, const WP3& w, const WP3& out0,
                                              const WP3& out1, const mxd::KeySrc& keys,
                                              uint64_t n_t, uint64_t n_m, uint64_t n_z0,
                                              uint64_t n_z2, int ncomp) {
  __shared__ uint32_t rks[mxd::kMaxKeySlots][mxd::kKeyWords];
  mxd::stage_keys(rks, keys, 2 * ncomp);
  constexpr int P = mxd::Lane<T>::kPer;
  const int64_t nb = (n + P - 1) / P;
  MX_PARTY_WALK(nb, ncomp) {
    const int c = (int)(g / nblk);
    const uint64_t B = (uint64_t)(g - c * nblk);
    const int role = roles.r[c];
    if (role != 0 && role != 1) continue;
    const T* mine = cp<T>(msg, c);
    const T* other = cp<T>(rmk, c);
    const T* z2m = cp<T>(rz, c);
    T* wo = wp<T>(w, c);
    uint32_t wt[16], wm[16], wz[16];
    if (role == 0) {
      const uint32_t* k0 = rks[2 * c];
      mx::chacha_block(k0, n_t, B, wt);
      mx::chacha_block(k0, n_m, B, wm);
      mx::chacha_block(k0, n_z0, B, wz);
    } else {
      mx::chacha_block(rks[2 * c + 1], n_z2, B, wz);
    }
    const T* rt = cp<T>(rrt, c);
    const u64* rm = cp<u64>(rrm, c);
    T* o = role == 0 ? wp<T>(out0, c) : wp<T>(out1, c);
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
        const T y = role == 0
                        ? mxf::trunc_y<T>(cc, mxd::pick<T>(tl, th, j), mxd::pick<T>(ml, mh, j), m,
                                          true)
                        : mxf::trunc_y<T>(cc, rt[i], (T)rm[i], m, false);
        wo[i] = y - z;
        o[i] = z;
      }
    }
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_dot_tail_r1(int64_t n, int m, Roles roles, CP3 msg,
                                                     CP3 rmk, CP3 rz, CP3 rrt, CP3 rrm, WP3 w,
                                                     WP3 out0, WP3 out1, mxd::KeySrc keys,
                                                     uint64_t n_t, uint64_t n_m, uint64_t n_z0,
                                                     uint64_t n_z2, int ncomp) {
  d_dot_tail_r1<T>(n, m, roles, msg, rmk, rz, rrt, rrm, w, out0, out1, keys, n_t, n_m, n_z0, n_z2,
                   ncomp);
}

// out[c] = a[c] + b[c] for the components in role 0 or 1 (P0's s1, P1's s0 = w0 + w1)
template <class T>
__device__ __forceinline__ void d_dot_tail_r2(int64_t n, const Roles& roles, const CP3& a,
                                              const CP3& b, const WP3& out, int ncomp) {
  const int64_t total = n * ncomp;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(g / n);
    const int64_t i = g - (int64_t)c * n;
    const int role = roles.r[c];
    if (role != 0 && role != 1) continue;
    wp<T>(out, c)[i] = cp<T>(a, c)[i] + cp<T>(b, c)[i];
  }
}

template <class T>
__global__ void __launch_bounds__(256) k_dot_tail_r2(int64_t n, Roles roles, CP3 a, CP3 b, WP3 out,
                                                     int ncomp) {
  d_dot_tail_r2<T>(n, roles, a, b, out, ncomp);
}

// party-batched twins for the composed one-GPU replay (party_batch.h)
MX_X3(k_trunc_party_r0<u64>, d_trunc_party_r0<u64>);
MX_X3(k_trunc_party_r0<u128>, d_trunc_party_r0<u128>);
MX_X3(k_trunc_party_r1<u64>, d_trunc_party_r1<u64>);
MX_X3(k_trunc_party_r1<u128>, d_trunc_party_r1<u128>);
MX_X3(k_share_party<u64>, d_share_party<u64>);
MX_X3(k_share_party<u128>, d_share_party<u128>);
MX_X3(k_dot_tail_r0<u64>, d_dot_tail_r0<u64>);
MX_X3(k_dot_tail_r0<u128>, d_dot_tail_r0<u128>);
MX_X3(k_dot_tail_r1<u64>, d_dot_tail_r1<u64>);
MX_X3(k_dot_tail_r1<u128>, d_dot_tail_r1<u128>);
MX_X3(k_dot_tail_r2<u64>, d_dot_tail_r2<u64>);
MX_X3(k_dot_tail_r2<u128>, d_dot_tail_r2<u128>);

inline CP3 cp3(const void* const* a, int ncomp) {
  CP3 o{{nullptr, nullptr, nullptr}};
  if (a)
    for (int c = 0; c < ncomp; ++c) o.p[c] = a[c];
  return o;
}
inline WP3 wp3(void* const* a, int ncomp) {
  WP3 o{{nullptr, nullptr, nullptr}};
  if (a)
    for (int c = 0; c < ncomp; ++c) o.p[c] = a[c];
  return o;
}

}  // namespace

extern "C" {

int mxh_trunc_party_r0(int words, int64_t n, int m, int ncomp, const int* roles,
                       const void* s0, const void* s1, void* msg, void* msg_rm, void* out0,
                       void* out1, const uint32_t* const* slots, const uint64_t* nn,
                       void* stream) {
  if (n == 0) return 0;
  if (ncomp < 1 || ncomp > 3) return -3;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2 * ncomp);
  const Roles rr = roles_of(roles, ncomp);
  hipStream_t st = (hipStream_t)stream;
  if (words == 1) {
    hipLaunchKernelGGL(k_trunc_party_r0<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2) * ncomp),
                       dim3(256), 0, st, n, m, rr, (const u64*)s0, (const u64*)s1, (u64*)msg,
                       (u64*)msg_rm, (u64*)out0, (u64*)out1, k, nn[0], nn[1], nn[2], nn[3],
                       nn[4], nn[5], ncomp);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_trunc_party_r0<u128>, dim3(mxd::grid_for_chunks(n) * ncomp), dim3(256), 0, st,
                       n, m, rr, (const u128*)s0, (const u128*)s1, (u128*)msg, (u64*)msg_rm,
                       (u128*)out0, (u128*)out1, k, nn[0], nn[1], nn[2], nn[3], nn[4], nn[5],
                       ncomp);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_trunc_party_r1(int words, int64_t n, int m, int ncomp, const int* roles,
                       const void* msg, const void* rmk, const void* rrt, const void* rrm,
                       void* w, void* out0, void* out1, const uint32_t* const* slots,
                       const uint64_t* nn, void* stream) {
  if (n == 0) return 0;
  if (ncomp < 1 || ncomp > 3) return -3;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2 * ncomp);
  const Roles rr = roles_of(roles, ncomp);
  hipStream_t st = (hipStream_t)stream;
  if (words == 1) {
    hipLaunchKernelGGL(k_trunc_party_r1<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2) * ncomp),
                       dim3(256), 0, st, n, m, rr, (const u64*)msg, (const u64*)rmk,
                       (const u64*)rrt, (const u64*)rrm, (u64*)w, (u64*)out0, (u64*)out1, k,
                       nn[2], nn[3], nn[4], nn[5], ncomp);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_trunc_party_r1<u128>, dim3(mxd::grid_for_chunks(n) * ncomp), dim3(256), 0, st,
                       n, m, rr, (const u128*)msg, (const u128*)rmk, (const u128*)rrt,
                       (const u64*)rrm, (u128*)w, (u128*)out0, (u128*)out1, k, nn[2], nn[3],
                       nn[4], nn[5], ncomp);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_share_party(int kind, int words, int64_t n, int ncomp, const int* rel, const void* x,
                    void* out0, void* out1, const uint32_t* const* slots, uint64_t n1,
                    uint64_t na, void* stream) {
  if (n == 0) return 0;
  if (ncomp < 1 || ncomp > 3) return -3;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2 * ncomp);
  const Roles rr = roles_of(rel, ncomp);
  hipStream_t st = (hipStream_t)stream;
  switch (words) {
    case 0:
      hipLaunchKernelGGL(k_share_party<uint8_t>, dim3(mxd::grid_for_chunks((n + 15) / 16) * ncomp),
                         dim3(256), 0, st, kind, n, rr, (const uint8_t*)x, (uint8_t*)out0,
                         (uint8_t*)out1, k, n1, na, ncomp);
      break;
    case 1:
      hipLaunchKernelGGL(k_share_party<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2) * ncomp), dim3(256),
                         0, st, kind, n, rr, (const u64*)x, (u64*)out0, (u64*)out1, k, n1, na,
                         ncomp);
      break;
    case 2:
      hipLaunchKernelGGL(k_share_party<u128>, dim3(mxd::grid_for_chunks(n) * ncomp), dim3(256), 0, st,
                         kind, n, rr, (const u128*)x, (u128*)out0, (u128*)out1, k, n1, na, ncomp);
      break;
    default:
      return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}


int mxh_dot_tail_r0(int words, int64_t n, int m, int ncomp, const int* roles,
                    const void* const* cross, void* const* msg, void* const* msg_rt,
                    void* const* msg_rm, void* const* out0, void* const* out1,
                    const uint32_t* const* slots, const uint64_t* nn, void* stream) {
  if (n == 0) return 0;
  if (ncomp < 1 || ncomp > 3) return -3;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2 * ncomp);
  const Roles rr = roles_of(roles, ncomp);
  hipStream_t st = (hipStream_t)stream;
  const CP3 x = cp3(cross, ncomp);
  const WP3 mo = wp3(msg, ncomp), rt = wp3(msg_rt, ncomp), rm = wp3(msg_rm, ncomp),
            o0 = wp3(out0, ncomp), o1 = wp3(out1, ncomp);
  if (words == 1) {
    hipLaunchKernelGGL(k_dot_tail_r0<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2) * ncomp),
                       dim3(256), 0, st, n, m, rr, x, mo, rt, rm, o0, o1, k, nn[0], nn[1],
                       nn[2], nn[3], nn[4], nn[5], nn[6], ncomp);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_dot_tail_r0<u128>, dim3(mxd::grid_for_chunks(n) * ncomp), dim3(256), 0,
                       st, n, m, rr, x, mo, rt, rm, o0, o1, k, nn[0], nn[1], nn[2], nn[3], nn[4],
                       nn[5], nn[6], ncomp);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_dot_tail_r1(int words, int64_t n, int m, int ncomp, const int* roles,
                    const void* const* msg, const void* const* rmk, const void* const* rz,
                    const void* const* rrt, const void* const* rrm, void* const* w,
                    void* const* out0, void* const* out1, const uint32_t* const* slots,
                    const uint64_t* nn, void* stream) {
  if (n == 0) return 0;
  if (ncomp < 1 || ncomp > 3) return -3;
  const mxd::KeySrc k = mxd::keysrc_slots(slots, 2 * ncomp);
  const Roles rr = roles_of(roles, ncomp);
  hipStream_t st = (hipStream_t)stream;
  const CP3 a = cp3(msg, ncomp), b = cp3(rmk, ncomp), z = cp3(rz, ncomp), t = cp3(rrt, ncomp),
            r = cp3(rrm, ncomp);
  const WP3 wo = wp3(w, ncomp), o0 = wp3(out0, ncomp), o1 = wp3(out1, ncomp);
  if (words == 1) {
    hipLaunchKernelGGL(k_dot_tail_r1<u64>, dim3(mxd::grid_for_chunks((n + 1) / 2) * ncomp),
                       dim3(256), 0, st, n, m, rr, a, b, z, t, r, wo, o0, o1, k, nn[3], nn[4],
                       nn[5], nn[6], ncomp);
  } else if (words == 2) {
    hipLaunchKernelGGL(k_dot_tail_r1<u128>, dim3(mxd::grid_for_chunks(n) * ncomp), dim3(256), 0,
                       st, n, m, rr, a, b, z, t, r, wo, o0, o1, k, nn[3], nn[4], nn[5], nn[6],
                       ncomp);
  } else {
    return -2;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

int mxh_dot_tail_r2(int words, int64_t n, int ncomp, const int* roles, const void* const* a,
                    const void* const* b, void* const* out, void* stream) {
  if (n == 0) return 0;
  if (ncomp < 1 || ncomp > 3) return -3;
  const Roles rr = roles_of(roles, ncomp);
  hipStream_t st = (hipStream_t)stream;
  const CP3 x = cp3(a, ncomp), y = cp3(b, ncomp);
  const WP3 o = wp3(out, ncomp);
  const int grid = mxd::grid_for(n * ncomp);
  if (words == 1)
    hipLaunchKernelGGL(k_dot_tail_r2<u64>, dim3(grid), dim3(256), 0, st, n, rr, x, y, o, ncomp);
  else if (words == 2)
    hipLaunchKernelGGL(k_dot_tail_r2<u128>, dim3(grid), dim3(256), 0, st, n, rr, x, y, o, ncomp);
  else
    return -2;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -100 - (int)e;
}

}  // extern "C"
