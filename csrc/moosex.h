// moosex native core: C ABI shared by the CPU (ring_cpu.cpp) and the gfx950 HIP
// (ring_hip.hip, gemm_mfma.hip) implementations.
//
// Ring tensors: Z_2^64 elements are uint64 words; Z_2^128 elements are two little-endian
// uint64 words (lo, hi) == the in-memory layout of unsigned __int128 on x86-64 and
// AMDGPU.  "words" below is 1 (Z_2^64), 2 (Z_2^128) or 0 (one byte per element, used for
// bit tensors holding 0/1).
//
// Every entry point returns 0 on success, a negative error code otherwise; `dev` is
// 0 for host memory and 1 for device memory (then `stream` is a hipStream_t).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mx_binop { MX_ADD = 0, MX_SUB = 1, MX_MUL = 2, MX_AND = 3, MX_OR = 4, MX_XOR = 5 };
enum mx_unop { MX_NEG = 0, MX_NOT = 1, MX_SHL = 2, MX_SHR = 3, MX_SAR = 4 };
enum mx_cmpop { MX_LT = 0, MX_GT = 1, MX_EQ = 2, MX_MSB = 3 };
// RSS cross-term kinds: arithmetic (x0*y0 + x0*y1 + x1*y0 + a - b) or boolean (& and ^)
enum mx_cross { MX_CROSS_ARITH = 0, MX_CROSS_BOOL = 1 };
// share kernels (mx_share3*, mx_share_party): kind MX_SHARE_F64 = an arithmetic sharing of a
// float64 input, fixed-point encoded in the kernel (x * 2^na, truncated as RingFixedpointEncode);
// the nonce argument na carries the fractional bits (the zero slot draws no randomness)
// kind | MX_SHARE_MIRROR: the masked slot goes to P_{j+2} instead of P_{j+1} (slot j =
// x - PRF(k_{j+1}), slot j+1 = PRF(k_{j+1}), slot j+2 = 0; the key argument is k_{j+1})
enum mx_share_src { MX_SHARE_F64 = 2, MX_SHARE_MIRROR = 8 };

// AES-128 key schedule: 11 round keys of 4 big-endian-packed words (FIPS-197 layout)
typedef struct {
  uint32_t rk[44];
} mx_aes_key;

int mx_version(void);
int mx_device_count(void);

// out[i] = a[i] op b[i]; na, nb in {n, 1} (scalar broadcast)
int mx_ew_binary(int dev, int op, int words, const void* a, int64_t na, const void* b,
                 int64_t nb, void* out, int64_t n, void* stream);
// Stacked party vectors a[nparties, m]: out[p, i] = p == which ? a[p, i] op b[i % nb]
// : a[p, i] (a public operand applied to one party's share slot, in one pass); nb divides m
// (b repeats with period nb: scalars, full slots, trailing-axis vectors)
int mx_ew_binary_slot(int dev, int op, int words, const void* a, const void* b, int64_t nb,
                      void* out, int64_t m, int nparties, int which, void* stream);
// Zero share from precomputed keystreams + reshare, three stacked parties (arith):
// out0[p, i] = v[p, i] + r[p, i] - r[p+1, i] ; out1[p, i] = out0[p+1, i]
int mx_add_zs3(int dev, int words, const void* v, const void* r, void* out0, void* out1,
               int64_t n, void* stream);
// out[i] = op(a[i], param)
int mx_ew_unary(int dev, int op, int words, const void* a, void* out, int64_t n,
                int64_t param, void* stream);
// Share-pair forms (both replicated share vectors of a share-wise op, one launch):
// out0 = a0 op b0, out1 = a1 op b1 (same na / nb / n for both)
int mx_ew_binary2(int dev, int op, int words, const void* a0, const void* b0, void* out0,
                  const void* a1, const void* b1, void* out1, int64_t na, int64_t nb, int64_t n,
                  void* stream);
// o_y = a_y * f + (add_y ? c[0] : 0), y = 0, 1 (one party's two share components)
int mx_mul_add2(int dev, int words, const void* a0, const void* a1, const void* f,
                const void* c, int add0, int add1, void* out0, void* out1, int64_t n,
                void* stream);
int mx_ew_unary2(int dev, int op, int words, const void* a0, void* out0, const void* a1,
                 void* out1, int64_t n, int64_t param, void* stream);
// out_y = a_y^T, y = 0, 1 ([rows, cols] ring matrices -> [cols, rows])
int mx_transpose2(int dev, int words, const void* a0, void* out0, const void* a1, void* out1,
                  int64_t rows, int64_t cols, void* stream);
// mx_ew_binary_slot on a0 (slot which0) and a1 (slot which1) with one public b
int mx_ew_binary_slot2(int dev, int op, int words, const void* a0, const void* a1,
                       const void* b, int64_t nb, void* out0, void* out1, int64_t m,
                       int nparties, int which0, int which1, void* stream);
// Fixed-point product of three stacked parties in one launch (device, latency-bound sizes):
// rss_mul3 (zero share from slots k0, k1, k2 at nmul) followed by trunc_pr3 (slots k0 / k2,
// nonces r0 r1 t m z0 z2) on the product, outputs at party stride ostride.  views: operand
// {party stride[4], period[4]} or null.  Returns 1 when the size is not latency-bound (the
// caller then runs the two kernels), 0 on success.
int mx_mul_trunc3_kv(int dev, int words, const void* x0, const void* x1, const void* y0,
                     const void* y1, void* out0, void* out1, int64_t n, int64_t ostride,
                     const uint32_t* slots, uint64_t nmul, int m, const uint64_t* nonces,
                     const int64_t* views, void* stream);
// out = a + b + c elementwise (mod 2^w)
int mx_ew_add3(int dev, int words, const void* a, const void* b, const void* c, void* out,
               int64_t n, void* stream);
// Share-wise linear combination of nin <= 3 stacked replicated values [nparties, m], both
// share vectors in one launch: out_y = sum_t coef[t] * ins[2t + y] (mod 2^w), plus the public
// b (period nb, null = none) at party slot which_y.
int mx_lincomb2(int dev, int words, int nin, const void* const* ins, const int64_t* coef,
                const void* b, int64_t nb, void* out0, void* out1, int64_t m, int nparties,
                int which0, int which1, void* stream);
// Sum of k stacked share vectors that are views of one buffer at a constant element step
// is_y (party stride ps_y, each party's slot dense, m elements): out_y[p, e] =
// sum_t base_y[t * is_y + p * ps_y + e], both share vectors (y = 0, 1) in one launch.
int mx_sum_views2(int dev, int words, const void* base0, const void* base1, int64_t is0,
                  int64_t is1, int64_t ps0, int64_t ps1, int k, void* out0, void* out1, int64_t m,
                  int nparties, void* stream);
// Two trivial sharings in the stacked layout [nparties, m], one launch:
// out0[q, i] = q == which0 ? x0[i] : 0 ; out1[q, i] = q == which1 ? x1[i] : 0
int mx_slot_place2(int dev, int words, const void* x0, const void* x1, void* out0, void* out1,
                   int64_t m, int nparties, int which0, int which1, void* stream);
// out[i] = (a[i] cmp b[i]) as 0/1 bytes, signed two's-complement comparison
int mx_ew_compare(int dev, int op, int words, const void* a, int64_t na, const void* b,
                  int64_t nb, uint8_t* out, int64_t n, void* stream);
// out[i] = (a[i] >> bit) & 1
int mx_bit_extract(int dev, int words, const void* a, uint8_t* out, int64_t n, int bit,
                   void* stream);
// out[i] = (ring) bits[i] << bit
int mx_ring_inject(int dev, int words, const uint8_t* bits, void* out, int64_t n, int bit,
                   void* stream);
// out[i] = round(x[i] * 2^frac) mod 2^(64*words)
int mx_encode(int dev, int words, const double* x, void* out, int64_t n, int frac,
              void* stream);
// out[i] = signed(x[i]) / 2^frac
// decode(a + b + c [+ d]): a reveal's shares summed and decoded in one pass (d may be null)
int mx_addn_decode(int dev, int words, const void* a, const void* b, const void* c,
                   const void* d, double* out, int64_t n, int frac, void* stream);
int mx_decode(int dev, int words, const void* x, double* out, int64_t n, int frac,
              void* stream);
// out[i] = value (lo word, hi word for Z_2^128; low byte for bits)
int mx_fill(int dev, int words, void* out, int64_t n, uint64_t lo, uint64_t hi, void* stream);
// out[o, j, i] = bit (start + j) of a[o, i] (0/1 bytes)
int mx_bit_planes(int dev, int words, const void* a, uint8_t* out, int64_t outer, int64_t inner,
                  int start, int count, void* stream);
// out[o, i] = sum_j w[j] * a[o, j, i] (w: k ring elements in the memory named by dev)
int mx_weighted_sum(int dev, int words, const void* a, const void* w, void* out, int64_t outer,
                    int64_t k, int64_t inner, void* stream);
// out[o, i] = sum_r a[o, r, i]
int mx_sum_axis(int dev, int words, const void* a, void* out, int64_t outer, int64_t red,
                int64_t inner, void* stream);
// AES-128 in counter mode: block c (c = ctr0, ctr0+1, ...) = AES_k(nonce_le64 || c_le64);
// writes nbytes bytes of the keystream
int mx_prg(int dev, const uint8_t* key16, uint64_t nonce, uint64_t ctr0, void* out,
           int64_t nbytes, void* stream);
// AES-128 encryption of single 16-byte blocks (ECB) on the host; used for seed derivation
// DeriveSeed: 16-byte seed = first 16 bytes of PRF block(key; sync key as counter||nonce)
int mx_derive_seed(const uint8_t* key16, const uint8_t* sync16, uint8_t* out16);
int mx_aes_encrypt_blocks(const uint8_t* key16, const uint8_t* in, uint8_t* out,
                          int64_t nblocks);
// RSS local step for `nparties` stacked parties of n elements each:
//   party p, element i: out = x0*y0 + x0*y1 + x1*y0 + PRF(key[p])_i - PRF(key[p+1])_i
// (boolean flavour: & and ^).  keys has nparties+1 entries.  x1 or y1 may be null
// (then those terms are dropped: used for local products with public values).  y0 == null
// means out = x0 + zero share.  keys may be null (no zero share).
int mx_rss_cross(int dev, int kind, int words, const void* x0, const void* x1,
                 const void* y0, const void* y1, void* out, int64_t n, int nparties,
                 const uint8_t* keys16, uint64_t nonce, void* stream);
// zero share only: out[p, i] = PRF(key[p])_i - PRF(key[p+1])_i (xor for kind BOOL)
int mx_zero_share(int dev, int kind, int words, void* out, int64_t n, int nparties,
                  const uint8_t* keys16, uint64_t nonce, void* stream);
// PRF expansion of several keys: out[p, i] = PRF(key[p])_i (words 0 -> bytes & 1)
int mx_prf_expand(int dev, int words, void* out, int64_t n, int nkeys,
                  const uint8_t* keys16, uint64_t nonce, void* stream);
// Batched ring GEMM.  mode 0: C = A0 . B0.  mode 1 (RSS cross): C = A0.(B0+B1) + A1.B0.
// A* are [batch, M, K] row-major, B* are [batch, K, N] row-major, C is [batch, M, N].
// accumulate != 0 -> C += result.
int mx_gemm(int dev, int words, int64_t batch, int64_t M, int64_t N, int64_t K,
            const void* A0, const void* A1, const void* B0, const void* B1, int mode,
            void* C, int accumulate, void* stream);
// Scratch for the MFMA GEMM (device only): bytes needed for the given problem
int64_t mx_gemm_workspace_bytes(int words, int64_t batch, int64_t M, int64_t N,
                                int64_t K, int mode);
// Size (bytes) of the last GEMM workspace allocation that failed (the -4 return of the
// GEMM entry points), 0 if none since the last call; reading it resets it.  Held
// workspace bytes on the calling device (every stream's grow-only scratch).
int64_t mx_workspace_failed_bytes(void);
int64_t mx_workspace_held_bytes(void);
int64_t mx_workspace_shared_count(void);
// GEMM variant using caller-provided device workspace (graph-capture friendly)
int mx_gemm_ws(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
               const void* A1, const void* B0, const void* B1, int mode, void* C,
               int accumulate, void* workspace, int64_t ws_bytes, void* stream);
// Prepared-B GEMM (device only): B' limb planes built once, reused for several A row
// blocks; A given with a batch stride (elements).  mx_gemm_b_bytes returns 0 when K is
// above the exact single-chunk limit (then use mx_gemm).
int64_t mx_gemm_b_bytes(int words, int64_t batch, int64_t N, int64_t K, int mode);
int mx_gemm_prep_b(int words, int64_t batch, int64_t K, int64_t N, const void* B0,
                   const void* B1, int mode, void* lb, void* stream);
int mx_gemm_with_b(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                   const void* A1, int64_t a_bstride, int mode, const void* lb, void* C,
                   int accumulate, void* stream);
// Device GEMM with explicit batch strides (elements) for the A and B operands; a stride of 0
// broadcasts one operand over the batch (no copy of an expanded stack).
int mx_crt_tables4(int words, int n, uint32_t* wd_out, uint32_t* rd_out);
int mx_gemm_roll(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                 int64_t a_bstride, int64_t roll, const void* B0, const void* B1, const void* lb,
                 void* C, int accumulate, void* stream);
int mx_gemm_strided(int words, int64_t batch, int64_t M, int64_t N, int64_t K, const void* A0,
                    const void* A1, int64_t a_bstride, const void* B0, const void* B1,
                    int64_t b_bstride, int mode, void* C, int accumulate, void* stream);
// select the GEMM kernel: 0 = auto, 1 = force VALU reference kernel, 2 = force MFMA
void mx_set_gemm_impl(int impl);
// multi-modular (CRT) int8 GEMM for large products: 0 = auto, 1 = force, 2 = off
void mx_set_gemm_crt(int mode);
// moduli for an inner dimension K' (K, or 2K in mode 1); host copy of the CRT tables
int mx_crt_moduli(int words, int64_t kprime);
int mx_crt_tables(int words, int n, int32_t* p, uint8_t* wa, uint8_t* wb, int32_t* nega,
                  int32_t* negb, uint16_t* W, uint16_t* Mw);

// Fused stacked-session protocols (rss_fused.h).  s0/out0/out1 are [3, n] slot
// vectors (party p holds out0[p] = z_p and out1[p] = z_{p+1}).
// trunc_pr3 nonces: r0, r1, r_top, r_msb, z0, z2 (dealer keys k0, k2).
int mx_trunc_pr3(int dev, int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                 const uint8_t* k0, const uint8_t* k2, const uint64_t* nonces, void* stream);
// share3: owner party j; slot_j = PRF(k_j, n1) (k_j: held by P_j and P_{j+2}), slot_{j+1} =
// x - slot_j (sent to P_{j+1}), slot_{j+2} = 0 (reference replicated/convert.rs:74-90).
// The key argument is k_j; k_all / na are not read (kept for the ABI).
int mx_share3(int dev, int kind, int words, const void* x, void* out0, void* out1, int64_t n,
              int j, const uint8_t* k_next, const uint8_t* k_all, uint64_t n1, uint64_t na,
              void* stream);

// ---- PRF keys held in key slots (graph-capture friendly) -----------------------------
// A key slot is MX_KEY_SLOT_WORDS uint32 words: the raw 16-byte key (words 0..3) followed
// by its expanded AES-128 schedule (words 4..47).  Slots live in the memory named by
// `dev`; kernels read them at run time, so the keys are not baked into launch parameters.
#define MX_KEY_SLOT_WORDS 48
// host: fill n consecutive slots from n raw keys
void mx_key_slots(const uint8_t* keys16, int n, uint32_t* out);
// mx_rss_cross with keys from slots: party p uses slot p % nslots and (p + 1) % nslots
// (nslots == nparties: the ring of an RSS zero share; nslots == nparties + 1: explicit)
int mx_rss_cross_k(int dev, int kind, int words, const void* x0, const void* x1,
                   const void* y0, const void* y1, void* out, int64_t n, int nparties,
                   const uint32_t* slots, int nslots, uint64_t nonce, void* stream);
// mx_rss_cross with an explicit key PAIR per party: party p uses the key slots at
// slot_ptrs[2p] and slot_ptrs[2p+1] (a host array of 2 * nparties slot addresses).  Used
// when the stacked parties belong to different sessions (cyclic multi-GPU layout).
int mx_rss_cross_kp(int dev, int kind, int words, const void* x0, const void* x1,
                    const void* y0, const void* y1, void* out, int64_t n, int nparties,
                    const uint32_t* const* slot_ptrs, uint64_t nonce, void* stream);
// Stacked 3-party RSS product with the reshare fused in: out0[p] = z_p (cross terms +
// zero share from slots p, p+1 mod 3) and out1[p] = z_{p+1}, i.e. both shares of every
// party after the one-round reshare (x*/y*/out* are [3, n] slot vectors)
// mx_rss_mul3_k (device only) with operand views: views[0..3] party strides, views[4..7]
// periods (elements) of x0, x1, y0, y1 -- element e of party p is op[p * ps + e % per]
int mx_rss_mul3_kv(int dev, int kind, int words, const void* x0, const void* x1, const void* y0,
                   const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                   uint64_t nonce, const int64_t* views, void* stream);
int mx_rss_mul3_k(int dev, int kind, int words, const void* x0, const void* x1, const void* y0,
                  const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                  uint64_t nonce, void* stream);
// One Kogge-Stone level of the packed boolean adder for three stacked parties, reshare
// fused (x*, out* are [3, n] slot vectors of packed words):
//   t = pk AND (g << d)                     (RSS AND: cross terms ^ zero share)
//   g' = g ^ t ;  pk' = pk AND (pk << d) if both
// zero shares: party p xors PRF(k_p) ^ PRF(k_{p+1}) at element e (t) and n + e (pk') of
// ONE nonce -- the same values as the generic path's stacked [2, n] AND.
// rep.binary_adder's whole carry chain (nlev Kogge-Stone levels, level l at nonces[l]) for
// three stacked parties in one launch; returns the final g shares (device only)
int mx_ks_adder3_k(int dev, int words, const void* g0, const void* g1, const void* p0,
                   const void* p1, void* og0, void* og1, int64_t n, int nlev,
                   const uint32_t* slots, const uint64_t* nonces, void* stream);
int mx_ks_level3_k(int dev, int words, const void* g0, const void* g1, const void* p0,
                   const void* p1, void* og0, void* og1, void* op0, void* op1, int64_t n,
                   int d, int both, const uint32_t* slots, uint64_t nonce, void* stream);
// One party's share of a Kogge-Stone level (SPMD: one process per party), before the
// reshare: z[e] = pk AND (g << d) cross terms ^ PRF(k0)[e] ^ PRF(k1)[e]; if both, also
// z[n + e] for pk AND (pk << d).  keys16 = (k_p, k_{p+1}); z has (both ? 2n : n) words.
int mx_ks_cross1(int dev, int words, const void* g0, const void* g1, const void* p0,
                 const void* p1, void* z, int64_t n, int d, int both, const uint8_t* keys16,
                 uint64_t nonce, void* stream);
// mx_ks_cross1 with the two keys read from key slots (slots[0] = k_p, slots[1] = k_{p+1})
int mx_ks_cross1_s(int dev, int words, const void* g0, const void* g1, const void* p0,
                   const void* p1, void* z, int64_t n, int d, int both,
                   const uint32_t* const* slots, uint64_t nonce, void* stream);
// mx_ks_cross1_s with the previous level's xor folded in: the level's g is g ^ t (t = the
// previous level's reshared AND, both share components), written to go0 / go1 and used for
// the cross terms (t0 == null: plain mx_ks_cross1_s, go unused)
int mx_ks_cross1x_s(int dev, int words, const void* g0, const void* g1, const void* t0,
                    const void* t1, void* go0, void* go1, const void* p0, const void* p1,
                    void* z, int64_t n, int d, int both, const uint32_t* const* slots,
                    uint64_t nonce, void* stream);
// The adder's sum after the last level, both share components: o = p ^ ((g ^ t) << 1)
int mx_ks_sum2(int dev, int words, const void* p0, const void* p1, const void* g0,
               const void* g1, const void* t0, const void* t1, void* o0, void* o1, int64_t n,
               void* stream);
// mx_prf_expand with nkeys consecutive key slots
int mx_prf_expand_k(int dev, int words, void* out, int64_t n, int nkeys, const uint32_t* slots,
                    uint64_t nonce, void* stream);
int mx_trunc_pr3_k(int dev, int words, const void* s0, void* out0, void* out1, int64_t n, int m,
                   const uint32_t* slot_k0, const uint32_t* slot_k2, const uint64_t* nonces,
                   void* stream);
int mx_trunc_pr3_ko(int dev, int words, const void* s0, void* out0, void* out1, int64_t n,
                    int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                    const uint64_t* nonces, int64_t ostride, void* stream);
int mx_trunc_pr3_kmo(int dev, int words, const void* s0, void* out0, void* out1, int64_t n,
                     int m, const uint32_t* slot_k0, const uint32_t* slot_k2,
                     const uint64_t* nonces, int64_t ostride, const uint64_t* cm, void* stream);
int mx_share3_k(int dev, int kind, int words, const void* x, void* out0, void* out1, int64_t n,
                int j, const uint32_t* slot_next, const uint32_t* slot_all, uint64_t n1,
                uint64_t na, void* stream);

// Per-party protocol rounds for layouts with the parties of a session on different GPUs
// (rss_party.hip): ncomp stacked components [ncomp, n], component c in role roles[c]
// (-1 = idle), key slots (own k_p, next k_{p+1}) per component.  nonces: r0, r1, t, m, z0,
// z2 of the TruncPr.  Round 0 writes the outgoing messages (P0: mk0, P1: mk1, P2: rt1 in
// msg; P2: rm1 in msg_rm as u64) and P2's new shares; round 1 takes the received mask
// share (rmk) and dealer shares (rrt, rrm) and writes w (P0: y0 - z0, P1: y1 - z2) and
// P0's s0 / P1's s1.
int mx_trunc_party_r0(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                      const void* s0, const void* s1, void* msg, void* msg_rm, void* out0,
                      void* out1, const uint32_t* const* slots, const uint64_t* nonces,
                      void* stream);
int mx_trunc_party_r1(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                      const void* msg, const void* rmk, const void* rrt, const void* rrm,
                      void* w, void* out0, void* out1, const uint32_t* const* slots,
                      const uint64_t* nonces, void* stream);
// Share by member j, per component: rel[c] = (role - j) mod 3; key slots per component:
// rel 0 (next, all), rel 1 (own, all), rel 2 (all, all).  The owner's out0 (its masked
// x_j) is then sent to P_{j+2}, whose out1 it becomes.
int mx_share_party(int dev, int kind, int words, int64_t n, int ncomp, const int* rel,
                   const void* x, void* out0, void* out1, const uint32_t* const* slots,
                   uint64_t n1, uint64_t na, void* stream);
// Fixed-point dot tail (rep.dot_trunc) with the parties on different GPUs: the reshare of
// the dot is folded into TruncPr's first round (rss_party.hip).  Every array argument is
// an array of ncomp per-component pointers (entries a role does not use may be null).
// nonces: zero share, r0, r1, t, m, z0, z2.  r0: messages (P0 m0, P1 m1, P2 z2) in msg, the
// dealer's rt1 / rm1 (u64) in msg_rt / msg_rm, P2's new shares; r1: rmk = the other
// party's message, rz = z2, rrt / rrm = dealer shares (P1) -> w, P0's s0 / P1's s1;
// r2: out = a + b (P0's s1, P1's s0).
int mx_dot_tail_r0(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                   const void* const* cross, void* const* msg, void* const* msg_rt,
                   void* const* msg_rm, void* const* out0, void* const* out1,
                   const uint32_t* const* slots, const uint64_t* nonces, void* stream);
int mx_dot_tail_r1(int dev, int words, int64_t n, int m, int ncomp, const int* roles,
                   const void* const* msg, const void* const* rmk, const void* const* rz,
                   const void* const* rrt, const void* const* rrm, void* const* w,
                   void* const* out0, void* const* out1, const uint32_t* const* slots,
                   const uint64_t* nonces, void* stream);
int mx_dot_tail_r2(int dev, int words, int64_t n, int ncomp, const int* roles,
                   const void* const* a, const void* const* b, void* const* out, void* stream);

// The same tail for ONE party over up to MX_MAX_JOBS products ("jobs", rss_jobs.hip): job q
// is ptrs[8q..8q+7] = (x0, x1, y0, y1, a, a2, o0, o1) and dims[8q..8q+7] = (rows, sx, sy, sa,
// sa2, ca, ca2, cb): value[r, e] = cb (x0 y0 + x0 y1 + x1 y0) + ca a + ca2 a2 (row r of x at
// x + r sx, ...), for rows of length L; the new shares go to o0 / o1 (dense [rows, L]).
// Messages are dense over the concatenation of the jobs' rows.  main: the values' messages;
// dealer: P2's part.
#define MX_MAX_JOBS 4
int mx_jobs_r0(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
               int64_t L, int m, int role, int main, int dealer, void* msg, void* msg_rt,
               void* msg_rm, const uint32_t* const* slots, const uint64_t* nonces,
               void* stream);
// mx_jobs_r0 with the previous level's round-2 sums pending: region k = (o, a, b) =
// pend[3k .. 3k+2] of pend_len[k] elements, o = a + b; operands read through them, and the
// regions written too (one launch instead of the previous round 2 plus this round 0)
int mx_jobs_r0p(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
                int64_t L, int m, int role, int main, int dealer, void* msg, void* msg_rt,
                void* msg_rm, const uint32_t* const* slots, const uint64_t* nonces, int npend,
                const void* const* pend, const int64_t* pend_len, void* stream);
int mx_jobs_r1(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
               int64_t L, int m, int role, const void* msg, const void* rmk, const void* rz,
               const void* rrt, const void* rrm, void* w, const uint32_t* const* slots,
               const uint64_t* nonces, void* stream);
int mx_jobs_r2(int dev, int words, int njobs, const void* const* ptrs, const int64_t* dims,
               int64_t L, int role, const void* a, const void* b, void* stream);

// Per-party bit decomposition front and B2A (bits_party.h, rss_bits_party.hip): nonces
// nn = (n1 of the sharing, n_g of the product).  front: this party's p pair and zero-shared
// AND term z (P0 also the share message a1; P1 runs after receiving a1 in arecv).  b2a:
// phase 0 (P0, P2) / 1 (P1, arecv = A1): message (P0's A1), z, base pair of bit planes
// start.. start + count - 1 of src = (s0, s1, g0, g1, t0, t1) -- sum words (g0 = null) or
// the adder's last (p, g, t); phase 2: out = base - 2 (z, zr).  Elements [count, S].
int mx_bits_front(int dev, int words, int role, int64_t n, const void* xa, const void* xb,
                  const void* arecv, void* msg, void* z, void* p0, void* p1,
                  const uint32_t* const* slots, const uint64_t* nonces, void* stream);
// Per-party fused weighted sums over both share components (wsum_pair.h): ring values as
// ``words`` little-endian int64 each (w: nrows of them, cb: nblk).
int mx_wsum_pair(int dev, int words, int nrows, int nblk, int has2, int pub0, int pub1,
                 int64_t L, int64_t rs, const int64_t* w, const int64_t* wx, const int64_t* m2,
                 const int64_t* c2, const int64_t* cb, const void* r0, const void* r1,
                 const void* x0, const void* x1, void* o0, void* o1, void* q0, void* q1,
                 void* stream);
int mx_bits_b2a(int dev, int words, int phase, int role, int64_t S, int start, int count,
                int xbit, int blocks, const void* const* src, const void* arecv, void* msg, void* z, void* base0,
                void* base1, const void* zr, void* out0, void* out1,
                const uint32_t* const* slots, const uint64_t* nonces, void* stream);

#ifdef __cplusplus
}
#endif
