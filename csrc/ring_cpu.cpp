// Host (CPU) implementation of the moosex ring kernels.
//
// These are the correctness oracles for the gfx950 kernels (bit-exact ring arithmetic)
// and the execution path of the CPU-only LocalMooseRuntime.  Z_2^128 uses the compiler's
// unsigned __int128; AES uses AES-NI.  Work is split over a small pool of std::threads.
#include <immintrin.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "aes_core.h"
#include "prf_core.h"
#include "moosex.h"
#include "ring_common.h"

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;
using i128 = __int128;

int num_threads() {
  static int n = [] {
    const char* e = getenv("MOOSEX_CPU_THREADS");
    int v = e ? atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(v, 32));
  }();
  return n;
}

template <class F>
void parallel_for(int64_t n, int64_t grain, F f) {
  int nt = num_threads();
  if (n <= grain || nt == 1) {
    if (n > 0) f(0, n);
    return;
  }
  int64_t chunks = std::min<int64_t>(nt, (n + grain - 1) / grain);
  int64_t per = (n + chunks - 1) / chunks;
  std::vector<std::thread> ts;
  ts.reserve(chunks - 1);
  for (int64_t c = 1; c < chunks; ++c) {
    int64_t b = c * per, e = std::min(n, b + per);
    if (b < e) ts.emplace_back([=] { f(b, e); });
  }
  f(0, std::min(n, per));
  for (auto& t : ts) t.join();
}

// ---------------------------------------------------------------------------
// AES-NI block encryption (the AES dialect; the PRF is ChaCha, prf_core.h)
// ---------------------------------------------------------------------------
struct NiKey {
  __m128i rk[11];
};

__attribute__((target("aes,sse4.1"))) void ni_expand(const uint8_t* key, NiKey* k) {
  uint32_t w[44];
  mx::expand_key(key, w);
  for (int r = 0; r < 11; ++r) {
    uint8_t b[16];
    for (int i = 0; i < 4; ++i) {
      uint32_t x = w[4 * r + i];
      b[4 * i] = x >> 24;
      b[4 * i + 1] = x >> 16;
      b[4 * i + 2] = x >> 8;
      b[4 * i + 3] = x;
    }
    k->rk[r] = _mm_loadu_si128((const __m128i*)b);
  }
}

__attribute__((target("aes,sse4.1"))) inline __m128i ni_encrypt(const NiKey& k, __m128i b) {
  b = _mm_xor_si128(b, k.rk[0]);
  for (int r = 1; r < 10; ++r) b = _mm_aesenc_si128(b, k.rk[r]);
  return _mm_aesenclast_si128(b, k.rk[10]);
}

__attribute__((target("aes,sse4.1"))) void aesni_blocks(const NiKey& k, const uint8_t* in,
                                                        uint8_t* out, int64_t nblocks) {
  for (int64_t b = 0; b < nblocks; ++b)
    _mm_storeu_si128((__m128i*)(out + 16 * b),
                     ni_encrypt(k, _mm_loadu_si128((const __m128i*)(in + 16 * b))));
}

bool have_aesni() {
  static bool v = __builtin_cpu_supports("aes");
  return v;
}

uint32_t g_T0[256];
struct TInit {
  TInit() {
    for (int i = 0; i < 256; ++i) g_T0[i] = mx::t0_entry(mx::kSbox[i]);
  }
} g_tinit;

// The PRF keystream (prf_core.h): chunk c is part (c >> 6) & 3 of ChaCha12 block
// ((c >> 8) << 6) | (c & 63), so a 256-chunk group is exactly 64 blocks.
struct Prf {
  uint32_t k[4];
  explicit Prf(const uint8_t* key) { mx::key_words(key, k); }
  // chunks [ctr, ctr + n) into out (16 bytes each)
  void blocks(uint64_t nonce, uint64_t ctr, uint8_t* out, int64_t n) const {
    int64_t done = 0;
    uint32_t w[64][16];
    while (done < n) {
      const uint64_t c = ctr + (uint64_t)done;
      const uint64_t grp = c >> 8;
      const int off = (int)(c & 255);
      const int take = (int)std::min<int64_t>(256 - off, n - done);
      uint64_t have = 0;  // bit b: block b of the group computed
      for (int j = 0; j < take; ++j) {
        const int idx = off + j, b = idx & 63, part = idx >> 6;
        if (!((have >> b) & 1)) {
          mx::chacha_block(k, nonce, (grp << 6) | (uint64_t)b, w[b]);
          have |= 1ull << b;
        }
        memcpy(out + 16 * (done + j), &w[b][4 * part], 16);
      }
      done += take;
    }
  }
};

// keystream bytes [byte0, byte0 + nbytes) into out
void keystream_range(const Prf& p, uint64_t nonce, int64_t byte0, int64_t nbytes, uint8_t* out) {
  int64_t b0 = byte0 / 16, b1 = (byte0 + nbytes + 15) / 16;
  uint8_t tmp[16 * 256];
  int64_t pos = 0;
  for (int64_t b = b0; b < b1;) {
    // up to the end of b's 256-chunk group (whole ChaCha blocks per call)
    const int64_t nb = std::min<int64_t>(256 - (b & 255), b1 - b);
    p.blocks(nonce, (uint64_t)b, tmp, nb);
    int64_t start = (b == b0) ? byte0 - b0 * 16 : 0;
    int64_t avail = nb * 16 - start;
    int64_t take = std::min(avail, nbytes - pos);
    memcpy(out + pos, tmp + start, take);
    pos += take;
    b += nb;
  }
}

// PRF element i of a ring with `words` words (0 -> 1 byte masked to a bit)
template <class T>
void prf_elements(const Prf& p, uint64_t nonce, int64_t i0, int64_t n, T* out) {
  if constexpr (sizeof(T) == 1) {
    keystream_range(p, nonce, i0, n, (uint8_t*)out);
    for (int64_t i = 0; i < n; ++i) out[i] &= 1;
  } else {
    keystream_range(p, nonce, i0 * (int64_t)sizeof(T), n * (int64_t)sizeof(T), (uint8_t*)out);
  }
}

// ---------------------------------------------------------------------------
// generic elementwise templates
// ---------------------------------------------------------------------------
template <class T>
int binary_t(int op, const T* a, int64_t na, const T* b, int64_t nb, T* out, int64_t n) {
  parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      T x = a[na == 1 ? 0 : i], y = b[nb == 1 ? 0 : i];
      out[i] = mxr::binop<T>(op, x, y);
    }
  });
  return 0;
}

template <class T>
int unary_t(int op, const T* a, T* out, int64_t n, int64_t param) {
  parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) out[i] = mxr::unop<T>(op, a[i], (int)param);
  });
  return 0;
}

template <class T>
int compare_t(int op, const T* a, int64_t na, const T* b, int64_t nb, uint8_t* out, int64_t n) {
  parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i)
      out[i] = mxr::cmpop<T>(op, a[na == 1 ? 0 : i], b ? b[nb == 1 ? 0 : i] : (T)0);
  });
  return 0;
}

template <class T>
int rss_cross_t(int kind, const T* x0, const T* x1, const T* y0, const T* y1, T* out, int64_t n,
                int nparties, const uint8_t* keys, uint64_t nonce) {
  for (int p = 0; p < nparties; ++p) {
    const int64_t off = (int64_t)p * n;
    Prf* ka = keys ? new Prf(keys + 16 * p) : nullptr;
    Prf* kb = keys ? new Prf(keys + 16 * (p + 1)) : nullptr;
    parallel_for(n, 1 << 14, [&](int64_t s, int64_t e) {
      const int64_t CH = 1024;
      T ra[CH], rb[CH];
      for (int64_t c = s; c < e; c += CH) {
        int64_t m = std::min(CH, e - c);
        if (ka) {
          prf_elements<T>(*ka, nonce, c, m, ra);
          prf_elements<T>(*kb, nonce, c, m, rb);
        }
        for (int64_t j = 0; j < m; ++j) {
          int64_t i = off + c + j;
          T v;
          if (x0 && y0) {
            v = mxr::cross<T>(kind, x0[i], x1 ? x1[i] : (T)0, y0[i], y1 ? y1[i] : (T)0,
                              x1 != nullptr, y1 != nullptr);
          } else if (x0) {
            v = x0[i];  // add-zero-share mode
          } else {
            v = 0;
          }
          if (ka) v = mxr::zs_combine<T>(kind, v, ra[j], rb[j]);
          out[i] = v;
        }
      }
    });
    delete ka;
    delete kb;
  }
  return 0;
}

template <class T>
int prf_expand_t(T* out, int64_t n, int nkeys, const uint8_t* keys, uint64_t nonce) {
  for (int p = 0; p < nkeys; ++p) {
    Prf k(keys + 16 * p);
    parallel_for(n, 1 << 14, [&](int64_t s, int64_t e) {
      prf_elements<T>(k, nonce, s, e - s, out + (int64_t)p * n + s);
    });
  }
  return 0;
}

template <class T>
int sum_axis_t(const T* a, T* out, int64_t outer, int64_t red, int64_t inner) {
  parallel_for(outer * inner, 1 << 14, [&](int64_t s, int64_t e) {
    for (int64_t oi = s; oi < e; ++oi) {
      int64_t o = oi / inner, i = oi % inner;
      T acc = 0;
      const T* p = a + o * red * inner + i;
      for (int64_t r = 0; r < red; ++r) acc += p[r * inner];
      out[oi] = acc;
    }
  });
  return 0;
}

template <class T>
void gemm_plain(const T* A, const T* B, T* C, int64_t M, int64_t N, int64_t K, bool acc) {
  parallel_for(M, 4, [&](int64_t s, int64_t e) {
    std::vector<T> row(N);
    for (int64_t i = s; i < e; ++i) {
      std::fill(row.begin(), row.end(), (T)0);
      const T* a = A + i * K;
      for (int64_t k = 0; k < K; ++k) {
        T av = a[k];
        const T* b = B + k * N;
        for (int64_t j = 0; j < N; ++j) row[j] += av * b[j];
      }
      T* c = C + i * N;
      if (acc)
        for (int64_t j = 0; j < N; ++j) c[j] += row[j];
      else
        for (int64_t j = 0; j < N; ++j) c[j] = row[j];
    }
  });
}

template <class T>
int gemm_t(int64_t batch, int64_t M, int64_t N, int64_t K, const T* A0, const T* A1,
           const T* B0, const T* B1, int mode, T* C, int accumulate) {
  for (int64_t b = 0; b < batch; ++b) {
    const T* a0 = A0 + b * M * K;
    const T* b0 = B0 + b * K * N;
    T* c = C + b * M * N;
    if (mode == 0) {
      gemm_plain(a0, b0, c, M, N, K, accumulate != 0);
    } else {
      const T* a1 = A1 + b * M * K;
      const T* b1 = B1 + b * K * N;
      std::vector<T> bs(K * N);
      for (int64_t i = 0; i < K * N; ++i) bs[i] = b0[i] + b1[i];
      gemm_plain(a0, bs.data(), c, M, N, K, accumulate != 0);
      gemm_plain(a1, b0, c, M, N, K, true);
    }
  }
  return 0;
}

}  // namespace

// host PRF expansion used by the fused host kernels (rss_fused_cpu.cpp)
void mx_cpu_prf_range(const uint8_t* key, uint64_t nonce, int words, int64_t i0, int64_t n,
                      void* out) {
  Prf p(key);
  if (words == 0) prf_elements<uint8_t>(p, nonce, i0, n, (uint8_t*)out);
  if (words == 1) prf_elements<u64>(p, nonce, i0, n, (u64*)out);
  if (words == 2) prf_elements<u128>(p, nonce, i0, n, (u128*)out);
}

void mx_cpu_parallel_for(int64_t n, int64_t grain,
                         const std::function<void(int64_t, int64_t)>& f) {
  parallel_for(n, grain, f);
}

// ---------------------------------------------------------------------------
// C ABI (host side); device variants live in ring_hip.hip and are reached through
// the mxh_* symbols declared in ring_common.h
// ---------------------------------------------------------------------------
#define DISPATCH_WORDS(words, T, ...)                 \
  switch (words) {                                    \
    case 0: { using T = uint8_t; __VA_ARGS__; }        \
    case 1: { using T = u64; __VA_ARGS__; }            \
    case 2: { using T = u128; __VA_ARGS__; }           \
    default: return -2;                               \
  }

extern "C" {

int mx_version(void) { return 3; }

int mx_ew_binary(int dev, int op, int words, const void* a, int64_t na, const void* b,
                 int64_t nb, void* out, int64_t n, void* stream) {
  if (dev) return mxh_ew_binary(op, words, a, na, b, nb, out, n, stream);
  DISPATCH_WORDS(words, T,
                 return binary_t<T>(op, (const T*)a, na, (const T*)b, nb, (T*)out, n));
}

int mx_add_zs3(int dev, int words, const void* v, const void* r, void* out0, void* out1,
               int64_t n, void* stream) {
  if (dev) return mxh_add_zs3(words, v, r, out0, out1, n, stream);
  DISPATCH_WORDS(words, T, {
    const T *V = (const T*)v, *Rr = (const T*)r;
    T *O0 = (T*)out0, *O1 = (T*)out1;
    parallel_for(n, 1 << 14, [&](int64_t lo, int64_t hi) {
      for (int64_t e = lo; e < hi; ++e) {
        const T z0 = V[e] + Rr[e] - Rr[n + e], z1 = V[n + e] + Rr[n + e] - Rr[2 * n + e],
                z2 = V[2 * n + e] + Rr[2 * n + e] - Rr[e];
        O0[e] = z0; O0[n + e] = z1; O0[2 * n + e] = z2;
        O1[e] = z1; O1[n + e] = z2; O1[2 * n + e] = z0;
      }
    });
    return 0;
  });
}

int mx_ew_binary_slot(int dev, int op, int words, const void* a, const void* b, int64_t nb,
                      void* out, int64_t m, int nparties, int which, void* stream) {
  if (dev) return mxh_ew_binary_slot(op, words, a, b, nb, out, m, nparties, which, stream);
  DISPATCH_WORDS(words, T, {
    const T *A = (const T*)a, *B = (const T*)b;
    T* O = (T*)out;
    for (int p = 0; p < nparties; ++p) {
      if (p == which) {
        if (nb == 1 || nb == m) {
          binary_t<T>(op, A + p * m, m, B, nb, O + p * m, m);
        } else {  // b repeats with period nb (a trailing-axis public operand)
          for (int64_t r = 0; r < m; r += nb) binary_t<T>(op, A + p * m + r, nb, B, nb, O + p * m + r, nb);
        }
      } else if (O != A) {
        std::memcpy(O + p * m, A + p * m, sizeof(T) * m);
      }
    }
    return 0;
  });
}

int mx_ew_unary(int dev, int op, int words, const void* a, void* out, int64_t n,
                int64_t param, void* stream) {
  if (dev) return mxh_ew_unary(op, words, a, out, n, param, stream);
  DISPATCH_WORDS(words, T, return unary_t<T>(op, (const T*)a, (T*)out, n, param));
}

int mx_ew_binary2(int dev, int op, int words, const void* a0, const void* b0, void* out0,
                  const void* a1, const void* b1, void* out1, int64_t na, int64_t nb, int64_t n,
                  void* stream) {
  if (dev) return mxh_ew_binary2(op, words, a0, b0, out0, a1, b1, out1, na, nb, n, stream);
  int rc = mx_ew_binary(0, op, words, a0, na, b0, nb, out0, n, stream);
  return rc ? rc : mx_ew_binary(0, op, words, a1, na, b1, nb, out1, n, stream);
}

int mx_mul_add2(int dev, int words, const void* a0, const void* a1, const void* f,
                const void* c, int add0, int add1, void* out0, void* out1, int64_t n,
                void* stream) {
  if (dev) return mxh_mul_add2(words, a0, a1, f, c, add0, add1, out0, out1, n, stream);
  DISPATCH_WORDS(words, T, {
    const T* fs = (const T*)f;
    const T cv = *(const T*)c;
    for (int y = 0; y < 2; ++y) {
      const T* a = (const T*)(y ? a1 : a0);
      T* o = (T*)(y ? out1 : out0);
      const T add = (y ? add1 : add0) ? cv : (T)0;
      for (int64_t i = 0; i < n; ++i) o[i] = a[i] * fs[i] + add;
    }
    return 0;
  });
}

int mx_transpose2(int dev, int words, const void* a0, void* out0, const void* a1, void* out1,
                  int64_t rows, int64_t cols, void* stream) {
  if (dev) return mxh_transpose2(words, a0, out0, a1, out1, rows, cols, stream);
  DISPATCH_WORDS(words, T, {
    for (int y = 0; y < 2; ++y) {
      const T* a = (const T*)(y ? a1 : a0);
      T* o = (T*)(y ? out1 : out0);
      for (int64_t i = 0; i < rows; ++i)
        for (int64_t j = 0; j < cols; ++j) o[j * rows + i] = a[i * cols + j];
    }
    return 0;
  });
}

int mx_ew_unary2(int dev, int op, int words, const void* a0, void* out0, const void* a1,
                 void* out1, int64_t n, int64_t param, void* stream) {
  if (dev) return mxh_ew_unary2(op, words, a0, out0, a1, out1, n, param, stream);
  int rc = mx_ew_unary(0, op, words, a0, out0, n, param, stream);
  return rc ? rc : mx_ew_unary(0, op, words, a1, out1, n, param, stream);
}

int mx_ew_binary_slot2(int dev, int op, int words, const void* a0, const void* a1,
                       const void* b, int64_t nb, void* out0, void* out1, int64_t m,
                       int nparties, int which0, int which1, void* stream) {
  if (dev)
    return mxh_ew_binary_slot2(op, words, a0, a1, b, nb, out0, out1, m, nparties, which0,
                               which1, stream);
  int rc = mx_ew_binary_slot(0, op, words, a0, b, nb, out0, m, nparties, which0, stream);
  return rc ? rc
            : mx_ew_binary_slot(0, op, words, a1, b, nb, out1, m, nparties, which1, stream);
}

int mx_mul_trunc3_kv(int dev, int words, const void* x0, const void* x1, const void* y0,
                     const void* y1, void* out0, void* out1, int64_t n, int64_t ostride,
                     const uint32_t* slots, uint64_t nmul, int m, const uint64_t* nonces,
                     const int64_t* views, void* stream) {
  if (dev)
    return mxh_mul_trunc3_kv(words, x0, x1, y0, y1, out0, out1, n, ostride, slots, nmul, m,
                             nonces, views, stream);
  return 1;  // host: the caller composes mx_rss_mul3 and mx_trunc_pr3
}

int mx_ew_add3(int dev, int words, const void* a, const void* b, const void* c, void* out,
               int64_t n, void* stream) {
  if (dev) return mxh_ew_add3(words, a, b, c, out, n, stream);
  DISPATCH_WORDS(words, T, {
    const T *A = (const T*)a, *B = (const T*)b, *C = (const T*)c;
    T* O = (T*)out;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) O[i] = A[i] + B[i] + C[i];
    });
    return 0;
  });
}

int mx_lincomb2(int dev, int words, int nin, const void* const* ins, const int64_t* coef,
                const void* b, int64_t nb, void* out0, void* out1, int64_t m, int nparties,
                int which0, int which1, void* stream) {
  if (dev)
    return mxh_lincomb2(words, nin, ins, coef, b, nb, out0, out1, m, nparties, which0, which1,
                        stream);
  if (nin < 1 || nin > 3) return -3;
  DISPATCH_WORDS(words, T, {
    T* O[2] = {(T*)out0, (T*)out1};
    const int W[2] = {which0, which1};
    const T* B = (const T*)b;
    const int64_t n = m * nparties;
    for (int y = 0; y < 2; ++y) {
      parallel_for(n, 1 << 14, [&](int64_t lo, int64_t hi) {
        for (int64_t g = lo; g < hi; ++g) {
          T v = 0;
          for (int t = 0; t < nin; ++t) v += (T)(int64_t)coef[t] * ((const T*)ins[2 * t + y])[g];
          if (B != nullptr && g / m == W[y]) v += B[nb == 1 ? 0 : (g % m) % nb];
          O[y][g] = v;
        }
      });
    }
    return 0;
  });
}

int mx_sum_views2(int dev, int words, const void* base0, const void* base1, int64_t is0,
                  int64_t is1, int64_t ps0, int64_t ps1, int k, void* out0, void* out1, int64_t m,
                  int nparties, void* stream) {
  if (dev)
    return mxh_sum_views2(words, base0, base1, is0, is1, ps0, ps1, k, out0, out1, m, nparties,
                          stream);
  DISPATCH_WORDS(words, T, {
    const T* B[2] = {(const T*)base0, (const T*)base1};
    T* O[2] = {(T*)out0, (T*)out1};
    const int64_t IS[2] = {is0, is1}, PS[2] = {ps0, ps1};
    for (int y = 0; y < 2; ++y)
      for (int q = 0; q < nparties; ++q)
        for (int64_t e = 0; e < m; ++e) {
          T acc = 0;
          for (int t = 0; t < k; ++t) acc += B[y][t * IS[y] + q * PS[y] + e];
          O[y][q * m + e] = acc;
        }
    return 0;
  });
}

int mx_slot_place2(int dev, int words, const void* x0, const void* x1, void* out0, void* out1,
                   int64_t m, int nparties, int which0, int which1, void* stream) {
  if (dev)
    return mxh_slot_place2(words, x0, x1, out0, out1, m, nparties, which0, which1, stream);
  DISPATCH_WORDS(words, T, {
    const T* X[2] = {(const T*)x0, (const T*)x1};
    T* O[2] = {(T*)out0, (T*)out1};
    const int W[2] = {which0, which1};
    for (int y = 0; y < 2; ++y)
      for (int q = 0; q < nparties; ++q) {
        if (q == W[y])
          std::memcpy(O[y] + q * m, X[y], sizeof(T) * m);
        else
          std::memset((void*)(O[y] + q * m), 0, sizeof(T) * m);
      }
    return 0;
  });
}

int mx_ew_compare(int dev, int op, int words, const void* a, int64_t na, const void* b,
                  int64_t nb, uint8_t* out, int64_t n, void* stream) {
  if (dev) return mxh_ew_compare(op, words, a, na, b, nb, out, n, stream);
  DISPATCH_WORDS(words, T,
                 return compare_t<T>(op, (const T*)a, na, (const T*)b, nb, out, n));
}

int mx_bit_extract(int dev, int words, const void* a, uint8_t* out, int64_t n, int bit,
                   void* stream) {
  if (dev) return mxh_bit_extract(words, a, out, n, bit, stream);
  DISPATCH_WORDS(words, T, {
    const T* x = (const T*)a;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) out[i] = (uint8_t)((x[i] >> bit) & 1);
    });
    return 0;
  });
}

int mx_ring_inject(int dev, int words, const uint8_t* bits, void* out, int64_t n, int bit,
                   void* stream) {
  if (dev) return mxh_ring_inject(words, bits, out, n, bit, stream);
  DISPATCH_WORDS(words, T, {
    T* o = (T*)out;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) o[i] = ((T)(bits[i] & 1)) << bit;
    });
    return 0;
  });
}

int mx_encode(int dev, int words, const double* x, void* out, int64_t n, int frac,
              void* stream) {
  if (dev) return mxh_encode(words, x, out, n, frac, stream);
  if (words == 1) {
    u64* o = (u64*)out;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) o[i] = (u64)mxr::f64_to_i128(x[i] * std::ldexp(1.0, frac));
    });
    return 0;
  }
  if (words == 2) {
    u128* o = (u128*)out;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) o[i] = (u128)mxr::f64_to_i128(x[i] * std::ldexp(1.0, frac));
    });
    return 0;
  }
  return -2;
}

int mx_addn_decode(int dev, int words, const void* a, const void* b, const void* c,
                   const void* d, double* out, int64_t n, int frac, void* stream) {
  if (dev) return mxh_addn_decode(words, a, b, c, d, out, n, frac, stream);
  const double scale = std::ldexp(1.0, -frac);
  if (words == 1) {
    const u64 *x = (const u64*)a, *y = (const u64*)b, *z = (const u64*)c, *w = (const u64*)d;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i)
        out[i] = (double)(int64_t)(x[i] + y[i] + z[i] + (w ? w[i] : 0)) * scale;
    });
    return 0;
  }
  if (words == 2) {
    const u128 *x = (const u128*)a, *y = (const u128*)b, *z = (const u128*)c,
               *w = (const u128*)d;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i)
        out[i] = mxr::i128_to_f64(x[i] + y[i] + z[i] + (w ? w[i] : (u128)0)) * scale;
    });
    return 0;
  }
  return -2;
}

int mx_decode(int dev, int words, const void* x, double* out, int64_t n, int frac,
              void* stream) {
  if (dev) return mxh_decode(words, x, out, n, frac, stream);
  double scale = std::ldexp(1.0, -frac);
  if (words == 1) {
    const u64* a = (const u64*)x;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) out[i] = (double)(int64_t)a[i] * scale;
    });
    return 0;
  }
  if (words == 2) {
    const u128* a = (const u128*)x;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) out[i] = mxr::i128_to_f64(a[i]) * scale;
    });
    return 0;
  }
  return -2;
}

int mx_fill(int dev, int words, void* out, int64_t n, uint64_t lo, uint64_t hi, void* stream) {
  if (dev) return mxh_fill(words, out, n, lo, hi, stream);
  DISPATCH_WORDS(words, T, {
    T v;
    if constexpr (sizeof(T) == 16) {
      v = ((T)hi << 64) | (T)lo;
    } else {
      v = (T)lo;
    }
    T* o = (T*)out;
    parallel_for(n, 1 << 16, [&](int64_t s, int64_t e) {
      for (int64_t i = s; i < e; ++i) o[i] = v;
    });
    return 0;
  });
}

int mx_bit_planes(int dev, int words, const void* a, uint8_t* out, int64_t outer, int64_t inner,
                  int start, int count, void* stream) {
  if (dev) return mxh_bit_planes(words, a, out, outer, inner, start, count, stream);
  DISPATCH_WORDS(words, T, {
    const T* x = (const T*)a;
    parallel_for(outer * inner, 1 << 12, [&](int64_t s, int64_t e) {
      for (int64_t g = s; g < e; ++g) {
        const int64_t o = g / inner, i = g - o * inner;
        const T v = x[g];
        uint8_t* dst = out + o * count * inner + i;
        for (int j = 0; j < count; ++j) dst[(int64_t)j * inner] = (uint8_t)((v >> (start + j)) & 1);
      }
    });
    return 0;
  });
}

int mx_weighted_sum(int dev, int words, const void* a, const void* w, void* out, int64_t outer,
                    int64_t k, int64_t inner, void* stream) {
  if (dev) return mxh_weighted_sum(words, a, w, out, outer, k, inner, stream);
  DISPATCH_WORDS(words, T, {
    const T* x = (const T*)a;
    const T* ww = (const T*)w;
    T* o_ = (T*)out;
    parallel_for(outer * inner, 1 << 12, [&](int64_t s, int64_t e) {
      for (int64_t g = s; g < e; ++g) {
        const int64_t o = g / inner, i = g - o * inner;
        const T* src = x + o * k * inner + i;
        T acc = 0;
        for (int64_t j = 0; j < k; ++j) acc += ww[j] * src[j * inner];
        o_[g] = acc;
      }
    });
    return 0;
  });
}

int mx_sum_axis(int dev, int words, const void* a, void* out, int64_t outer, int64_t red,
                int64_t inner, void* stream) {
  if (dev) return mxh_sum_axis(words, a, out, outer, red, inner, stream);
  DISPATCH_WORDS(words, T, return sum_axis_t<T>((const T*)a, (T*)out, outer, red, inner));
}

int mx_prg(int dev, const uint8_t* key16, uint64_t nonce, uint64_t ctr0, void* out,
           int64_t nbytes, void* stream) {
  if (dev) return mxh_prg(key16, nonce, ctr0, out, nbytes, stream);
  Prf p(key16);
  parallel_for((nbytes + 15) / 16, 1 << 12, [&](int64_t s, int64_t e) {
    int64_t b0 = s * 16, b1 = std::min(nbytes, e * 16);
    keystream_range(p, nonce, (int64_t)ctr0 * 16 + b0, b1 - b0, (uint8_t*)out + b0);
  });
  return 0;
}

// HostSeed derivation (DeriveSeed): the first 16 bytes of PRF block (key; counter =
// sync[0..8), nonce = sync[8..16)) -- a PRF of the full 128-bit sync key.
int mx_derive_seed(const uint8_t* key16, const uint8_t* sync16, uint8_t* out16) {
  uint32_t k[4], w[16];
  mx::key_words(key16, k);
  uint64_t blk, nonce;
  memcpy(&blk, sync16, 8);
  memcpy(&nonce, sync16 + 8, 8);
  mx::chacha_block(k, nonce, blk, w);
  memcpy(out16, w, 16);
  return 0;
}

int mx_aes_encrypt_blocks(const uint8_t* key16, const uint8_t* in, uint8_t* out,
                          int64_t nblocks) {
  if (have_aesni()) {  // AES-NI (the AES dialect and the AES tests); table code otherwise
    NiKey k;
    ni_expand(key16, &k);
    aesni_blocks(k, in, out, nblocks);
    return 0;
  }
  uint32_t rk[44];
  mx::expand_key(key16, rk);
  for (int64_t b = 0; b < nblocks; ++b) {
    const uint8_t* p = in + 16 * b;
    uint32_t w[4], o[4];
    for (int i = 0; i < 4; ++i)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
             ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    mx::encrypt_block_tt(rk, g_T0, mx::kSbox, w[0], w[1], w[2], w[3], o);
    for (int i = 0; i < 4; ++i) {
      out[16 * b + 4 * i] = o[i] >> 24;
      out[16 * b + 4 * i + 1] = o[i] >> 16;
      out[16 * b + 4 * i + 2] = o[i] >> 8;
      out[16 * b + 4 * i + 3] = o[i];
    }
  }
  return 0;
}

int mx_rss_cross(int dev, int kind, int words, const void* x0, const void* x1,
                 const void* y0, const void* y1, void* out, int64_t n, int nparties,
                 const uint8_t* keys16, uint64_t nonce, void* stream) {
  if (dev)
    return mxh_rss_cross(kind, words, x0, x1, y0, y1, out, n, nparties, keys16, nonce, stream);
  DISPATCH_WORDS(words, T,
                 return rss_cross_t<T>(kind, (const T*)x0, (const T*)x1, (const T*)y0,
                                       (const T*)y1, (T*)out, n, nparties, keys16, nonce));
}

int mx_zero_share(int dev, int kind, int words, void* out, int64_t n, int nparties,
                  const uint8_t* keys16, uint64_t nonce, void* stream) {
  return mx_rss_cross(dev, kind, words, nullptr, nullptr, nullptr, nullptr, out, n, nparties,
                      keys16, nonce, stream);
}

int mx_prf_expand(int dev, int words, void* out, int64_t n, int nkeys, const uint8_t* keys16,
                  uint64_t nonce, void* stream) {
  if (dev) return mxh_prf_expand(words, out, n, nkeys, keys16, nonce, stream);
  DISPATCH_WORDS(words, T, return prf_expand_t<T>((T*)out, n, nkeys, keys16, nonce));
}

int mx_gemm(int dev, int words, int64_t batch, int64_t M, int64_t N, int64_t K,
            const void* A0, const void* A1, const void* B0, const void* B1, int mode, void* C,
            int accumulate, void* stream) {
  if (dev) return mxh_gemm(words, batch, M, N, K, A0, A1, B0, B1, mode, C, accumulate, stream);
  if (words == 1)
    return gemm_t<u64>(batch, M, N, K, (const u64*)A0, (const u64*)A1, (const u64*)B0,
                       (const u64*)B1, mode, (u64*)C, accumulate);
  if (words == 2)
    return gemm_t<u128>(batch, M, N, K, (const u128*)A0, (const u128*)A1, (const u128*)B0,
                        (const u128*)B1, mode, (u128*)C, accumulate);
  return -2;
}

// ---- key slots ---------------------------------------------------------------------
void mx_key_slots(const uint8_t* keys16, int n, uint32_t* out) {
  for (int i = 0; i < n; ++i) {
    uint32_t* slot = out + (int64_t)MX_KEY_SLOT_WORDS * i;
    memcpy(slot, keys16 + 16 * i, 16);
    mx::expand_key(keys16 + 16 * i, slot + 4);
  }
}

int mx_rss_cross_k(int dev, int kind, int words, const void* x0, const void* x1,
                   const void* y0, const void* y1, void* out, int64_t n, int nparties,
                   const uint32_t* slots, int nslots, uint64_t nonce, void* stream) {
  if (nslots < 1 || nparties < 1 || nparties > 3) return -3;
  if (dev)
    return mxh_rss_cross_k(kind, words, x0, x1, y0, y1, out, n, nparties, slots, nslots, nonce,
                           stream);
  uint8_t keys[16 * 4];  // host slots: the raw keys lead each slot
  for (int i = 0; i <= nparties; ++i)
    memcpy(keys + 16 * i, slots + MX_KEY_SLOT_WORDS * (i % nslots), 16);
  DISPATCH_WORDS(words, T,
                 return rss_cross_t<T>(kind, (const T*)x0, (const T*)x1, (const T*)y0,
                                       (const T*)y1, (T*)out, n, nparties, keys, nonce));
}

int mx_rss_cross_kp(int dev, int kind, int words, const void* x0, const void* x1,
                    const void* y0, const void* y1, void* out, int64_t n, int nparties,
                    const uint32_t* const* slot_ptrs, uint64_t nonce, void* stream) {
  if (nparties < 1 || nparties > 3) return -3;
  if (dev)
    return mxh_rss_cross_kp(kind, words, x0, x1, y0, y1, out, n, nparties, slot_ptrs, nonce,
                            stream);
  const int64_t es = words == 0 ? 1 : 8 * words;
  auto at = [&](const void* b, int p) -> const void* {
    return b ? (const uint8_t*)b + (int64_t)p * n * es : nullptr;
  };
  for (int p = 0; p < nparties; ++p) {
    uint8_t keys[32];
    memcpy(keys, slot_ptrs[2 * p], 16);
    memcpy(keys + 16, slot_ptrs[2 * p + 1], 16);
    void* o = (uint8_t*)out + (int64_t)p * n * es;
    int rc = -2;
    if (words == 0)
      rc = rss_cross_t<uint8_t>(kind, (const uint8_t*)at(x0, p), (const uint8_t*)at(x1, p),
                                (const uint8_t*)at(y0, p), (const uint8_t*)at(y1, p),
                                (uint8_t*)o, n, 1, keys, nonce);
    else if (words == 1)
      rc = rss_cross_t<u64>(kind, (const u64*)at(x0, p), (const u64*)at(x1, p),
                            (const u64*)at(y0, p), (const u64*)at(y1, p), (u64*)o, n, 1, keys,
                            nonce);
    else if (words == 2)
      rc = rss_cross_t<u128>(kind, (const u128*)at(x0, p), (const u128*)at(x1, p),
                             (const u128*)at(y0, p), (const u128*)at(y1, p), (u128*)o, n, 1,
                             keys, nonce);
    if (rc) return rc;
  }
  return 0;
}

int mx_rss_mul3_k(int dev, int kind, int words, const void* x0, const void* x1, const void* y0,
                  const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                  uint64_t nonce, void* stream) {
  if (dev)
    return mxh_rss_mul3_k(kind, words, x0, x1, y0, y1, out0, out1, n, slots, nonce, stream);
  int rc = mx_rss_cross_k(0, kind, words, x0, x1, y0, y1, out0, n, 3, slots, 3, nonce, stream);
  if (rc) return rc;
  const int64_t bytes = n * (words == 0 ? 1 : 8 * words);
  for (int p = 0; p < 3; ++p)  // out1[p] = out0[p + 1]
    memcpy((uint8_t*)out1 + p * bytes, (const uint8_t*)out0 + ((p + 1) % 3) * bytes, bytes);
  return 0;
}

int mx_rss_mul3_kv(int dev, int kind, int words, const void* x0, const void* x1, const void* y0,
                   const void* y1, void* out0, void* out1, int64_t n, const uint32_t* slots,
                   uint64_t nonce, const int64_t* views, void* stream) {
  if (!dev) return -2;  // device only: host callers pass contiguous operands
  return mxh_rss_mul3_kv(kind, words, x0, x1, y0, y1, out0, out1, n, slots, nonce, views, stream);
}

int mx_ks_cross1(int dev, int words, const void* g0, const void* g1, const void* p0,
                 const void* p1, void* z, int64_t n, int d, int both, const uint8_t* keys16,
                 uint64_t nonce, void* stream) {
  if (dev) return mxh_ks_cross1(words, g0, g1, p0, p1, z, n, d, both, keys16, nonce, stream);
  if (words != 1 && words != 2) return -2;
  DISPATCH_WORDS(words, T, {
    const int64_t m = both ? 2 * n : n;
    std::vector<T> r0(m), r1(m);
    mx_cpu_prf_range(keys16, nonce, words, 0, m, r0.data());
    mx_cpu_prf_range(keys16 + 16, nonce, words, 0, m, r1.data());
    const T *G0 = (const T*)g0, *G1 = (const T*)g1, *A0 = (const T*)p0, *A1 = (const T*)p1;
    T* Z = (T*)z;
    parallel_for(n, 4096, [&](int64_t lo, int64_t hi) {
      for (int64_t e = lo; e < hi; ++e) {
        const T s0 = G0[e] << d, s1 = G1[e] << d;
        Z[e] = (A0[e] & s0) ^ (A0[e] & s1) ^ (A1[e] & s0) ^ r0[e] ^ r1[e];
        if (both) {
          const T u0 = A0[e] << d, u1 = A1[e] << d;
          Z[n + e] = (A0[e] & u0) ^ (A0[e] & u1) ^ (A1[e] & u0) ^ r0[n + e] ^ r1[n + e];
        }
      }
    });
    return 0;
  });
}

int mx_ks_cross1_s(int dev, int words, const void* g0, const void* g1, const void* p0,
                   const void* p1, void* z, int64_t n, int d, int both,
                   const uint32_t* const* slots, uint64_t nonce, void* stream) {
  if (dev) return mxh_ks_cross1_s(words, g0, g1, p0, p1, z, n, d, both, slots, nonce, stream);
  uint8_t keys16[32];  // host slots: the raw key is the slot's first 16 bytes
  memcpy(keys16, slots[0], 16);
  memcpy(keys16 + 16, slots[1], 16);
  return mx_ks_cross1(0, words, g0, g1, p0, p1, z, n, d, both, keys16, nonce, stream);
}

int mx_ks_cross1x_s(int dev, int words, const void* g0, const void* g1, const void* t0,
                    const void* t1, void* go0, void* go1, const void* p0, const void* p1,
                    void* z, int64_t n, int d, int both, const uint32_t* const* slots,
                    uint64_t nonce, void* stream) {
  if (dev)
    return mxh_ks_cross1x_s(words, g0, g1, t0, t1, go0, go1, p0, p1, z, n, d, both, slots,
                            nonce, stream);
  if (t0 != nullptr) {  // g ^ t first, then the plain level on it
    if (words != 1 && words != 2) return -2;
    DISPATCH_WORDS(words, T, {
      const T *G0 = (const T*)g0, *G1 = (const T*)g1, *A = (const T*)t0, *B = (const T*)t1;
      T *O0 = (T*)go0, *O1 = (T*)go1;
      for (int64_t e = 0; e < n; ++e) {
        O0[e] = G0[e] ^ A[e];
        O1[e] = G1[e] ^ B[e];
      }
      return mx_ks_cross1_s(0, words, go0, go1, p0, p1, z, n, d, both, slots, nonce, stream);
    });
  }
  return mx_ks_cross1_s(0, words, g0, g1, p0, p1, z, n, d, both, slots, nonce, stream);
}

int mx_ks_sum2(int dev, int words, const void* p0, const void* p1, const void* g0,
               const void* g1, const void* t0, const void* t1, void* o0, void* o1, int64_t n,
               void* stream) {
  if (dev) return mxh_ks_sum2(words, p0, p1, g0, g1, t0, t1, o0, o1, n, stream);
  if (words != 1 && words != 2) return -2;
  DISPATCH_WORDS(words, T, {
    const T* P[2] = {(const T*)p0, (const T*)p1};
    const T* G[2] = {(const T*)g0, (const T*)g1};
    const T* X[2] = {(const T*)t0, (const T*)t1};
    T* O[2] = {(T*)o0, (T*)o1};
    for (int s = 0; s < 2; ++s)
      for (int64_t e = 0; e < n; ++e) O[s][e] = P[s][e] ^ (T)((G[s][e] ^ X[s][e]) << 1);
    return 0;
  });
}

int mx_ks_adder3_k(int dev, int words, const void* g0, const void* g1, const void* p0,
                   const void* p1, void* og0, void* og1, int64_t n, int nlev,
                   const uint32_t* slots, const uint64_t* nonces, void* stream) {
  if (dev)
    return mxh_ks_adder3_k(words, g0, g1, p0, p1, og0, og1, n, nlev, slots, nonces, stream);
  // host: the per-level chain (mx_ks_level3_k), ping-ponging through temporaries
  if (words != 1 && words != 2) return -2;
  const size_t es = 8 * (size_t)words, sz = 3 * (size_t)n * es;
  std::vector<uint8_t> G0(sz), G1(sz), A0(sz), A1(sz), NG0(sz), NG1(sz), NA0(sz), NA1(sz);
  memcpy(G0.data(), g0, sz);
  memcpy(G1.data(), g1, sz);
  memcpy(A0.data(), p0, sz);
  memcpy(A1.data(), p1, sz);
  int d = 1;
  for (int l = 0; l < nlev; ++l, d *= 2) {
    const int both = 2 * d < 64 * words;
    const int rc = mx_ks_level3_k(0, words, G0.data(), G1.data(), A0.data(), A1.data(),
                                  NG0.data(), NG1.data(), NA0.data(), NA1.data(), n, d, both,
                                  slots, nonces[l], stream);
    if (rc) return rc;
    G0.swap(NG0);
    G1.swap(NG1);
    if (both) {
      A0.swap(NA0);
      A1.swap(NA1);
    }
  }
  memcpy(og0, G0.data(), sz);
  memcpy(og1, G1.data(), sz);
  return 0;
}

int mx_ks_level3_k(int dev, int words, const void* g0, const void* g1, const void* p0,
                   const void* p1, void* og0, void* og1, void* op0, void* op1, int64_t n,
                   int d, int both, const uint32_t* slots, uint64_t nonce, void* stream) {
  if (dev)
    return mxh_ks_level3_k(words, g0, g1, p0, p1, og0, og1, op0, op1, n, d, both, slots, nonce,
                           stream);
  if (words != 1 && words != 2) return -2;
  DISPATCH_WORDS(words, T, {
    const int64_t m = both ? 2 * n : n;
    std::vector<T> r[3];
    for (int k = 0; k < 3; ++k) {
      r[k].resize(m);
      mx_cpu_prf_range((const uint8_t*)(slots + MX_KEY_SLOT_WORDS * k), nonce, words, 0, m,
                       r[k].data());
    }
    const T *G0 = (const T*)g0, *G1 = (const T*)g1, *A0 = (const T*)p0, *A1 = (const T*)p1;
    T *OG0 = (T*)og0, *OG1 = (T*)og1, *OP0 = (T*)op0, *OP1 = (T*)op1;
    parallel_for(n, 4096, [&](int64_t lo, int64_t hi) {
      for (int64_t e = lo; e < hi; ++e) {
        T t[3], q[3];
        for (int p = 0; p < 3; ++p) {
          const int64_t i = p * n + e;
          const int pn = (p + 1) % 3;
          const T s0 = G0[i] << d, s1 = G1[i] << d;
          t[p] = (A0[i] & s0) ^ (A0[i] & s1) ^ (A1[i] & s0) ^ r[p][e] ^ r[pn][e];
          if (both) {
            const T u0 = A0[i] << d, u1 = A1[i] << d;
            q[p] = (A0[i] & u0) ^ (A0[i] & u1) ^ (A1[i] & u0) ^ r[p][n + e] ^ r[pn][n + e];
          }
        }
        for (int p = 0; p < 3; ++p) {
          const int64_t i = p * n + e;
          const int pn = (p + 1) % 3;
          OG0[i] = G0[i] ^ t[p];
          OG1[i] = G1[i] ^ t[pn];
          if (both) {
            OP0[i] = q[p];
            OP1[i] = q[pn];
          }
        }
      }
    });
    return 0;
  });
}

int mx_prf_expand_k(int dev, int words, void* out, int64_t n, int nkeys, const uint32_t* slots,
                    uint64_t nonce, void* stream) {
  if (nkeys < 1 || nkeys > 4) return -3;
  if (dev) return mxh_prf_expand_k(words, out, n, nkeys, slots, nonce, stream);
  uint8_t keys[16 * 4];
  for (int i = 0; i < nkeys; ++i) memcpy(keys + 16 * i, slots + MX_KEY_SLOT_WORDS * i, 16);
  DISPATCH_WORDS(words, T, return prf_expand_t<T>((T*)out, n, nkeys, keys, nonce));
}

}  // extern "C"
