// Device-side pieces of replayed multi-party evaluations (moose_amd/parallel/threads.py,
// parallel/spmd_graphs.py): fresh PRF keys drawn on the device, and batched message copies.
//
// * mx_key_refresh: every replay of a taped evaluation needs fresh, independent PRF keys in
//   its key table (runtime/keys.py).  Drawing them on the host costs a urandom call, the
//   AES-128 key schedules and a pinned host->device copy per table and replay (~0.3 ms per
//   party, on the critical path before the graph launch).  Here ONE tiny kernel derives them
//   on the device: slot s of replay e gets the first 16 bytes of ChaCha12(master, nonce = e,
//   block = s) -- the PRF of prf_core.h under a per-table master key drawn once from the OS
//   -- followed by its AES-128 schedule (FIPS-197 key expansion, as the host's
//   mx_key_slots).  The replay counter e lives in device memory and the kernel advances it,
//   so a captured launch refreshes the keys too.  Keys of different replays are outputs of
//   a PRF at distinct inputs: pseudo-random and independent under the master key.
// * mx_copy_many: the messages of one round of all parties (a composed one-GPU replay) as ONE
//   kernel instead of one copy node each: a table of (dst, src, bytes) in device memory,
//   grid.y = the message, grid.x = 4 KiB pieces of it.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "aes_core.h"
#include "moosex.h"
#include "party_batch.h"
#include "prf_core.h"

namespace {

__constant__ uint8_t kSboxDev[256] = MX_SBOX_INIT;

__device__ void expand_key_dev(const uint32_t key_le[4], uint32_t* rk) {
  // rk[i] big-endian words of the key bytes (as mx::expand_key on the host)
  const uint8_t* kb = (const uint8_t*)key_le;
  for (int i = 0; i < 4; ++i)
    rk[i] = ((uint32_t)kb[4 * i] << 24) | ((uint32_t)kb[4 * i + 1] << 16) |
            ((uint32_t)kb[4 * i + 2] << 8) | (uint32_t)kb[4 * i + 3];
  const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = (t << 8) | (t >> 24);
      t = ((uint32_t)kSboxDev[t >> 24] << 24) | ((uint32_t)kSboxDev[(t >> 16) & 255] << 16) |
          ((uint32_t)kSboxDev[(t >> 8) & 255] << 8) | (uint32_t)kSboxDev[t & 255];
      t ^= (uint32_t)rcon[i / 4 - 1] << 24;
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

// one workgroup: every thread derives slots tid, tid + 256, ...; then the counter advances
__device__ __forceinline__ void d_key_refresh(uint32_t* __restrict__ slots, int n,
                                              const uint32_t* __restrict__ master,
                                              uint64_t* __restrict__ epoch) {
  const uint64_t e = *epoch;
  uint32_t mk[4] = {master[0], master[1], master[2], master[3]};
  for (int s = threadIdx.x; s < n; s += blockDim.x) {
    uint32_t w[16];
    mx::chacha_block(mk, e, (uint64_t)s, w);
    uint32_t* slot = slots + (int64_t)s * MX_KEY_SLOT_WORDS;
    for (int i = 0; i < 4; ++i) slot[i] = w[i];
    uint32_t rk[44];
    expand_key_dev(w, rk);
    for (int i = 0; i < 44; ++i) slot[4 + i] = rk[i];
  }
  __syncthreads();  // every thread has read e before it changes
  if (threadIdx.x == 0) *epoch = e + 1;
}

__global__ void __launch_bounds__(256) k_key_refresh(uint32_t* __restrict__ slots, int n,
                                                     const uint32_t* __restrict__ master,
                                                     uint64_t* __restrict__ epoch) {
  d_key_refresh(slots, n, master, epoch);
}

// the parties' refreshes at the head of a composed replay: one party-batched node
MX_X3(k_key_refresh, d_key_refresh);

struct CopyDesc {
  const uint8_t* src;
  uint8_t* dst;
  int64_t bytes;
};

constexpr int64_t kPiece = 4096;

__global__ void __launch_bounds__(256) k_copy_many(const CopyDesc* __restrict__ d, int n) {
  const int m = blockIdx.y;
  if (m >= n) return;
  const CopyDesc c = d[m];
  const int64_t lo = (int64_t)blockIdx.x * kPiece;
  if (lo >= c.bytes) return;
  const int64_t hi = lo + kPiece < c.bytes ? lo + kPiece : c.bytes;
  const bool vec = ((((uintptr_t)c.src) | ((uintptr_t)c.dst)) & 15) == 0;
  if (vec) {
    const int64_t v0 = lo / 16, v1 = hi / 16;
    const uint4* s = (const uint4*)c.src;
    uint4* t = (uint4*)c.dst;
    for (int64_t i = v0 + threadIdx.x; i < v1; i += blockDim.x) t[i] = s[i];
    for (int64_t i = v1 * 16 + threadIdx.x; i < hi; i += blockDim.x) c.dst[i] = c.src[i];
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) c.dst[i] = c.src[i];
  }
}

// ---- per-party graphs on separate streams / devices: device-side message signalling ----
// A party's replay is ONE graph on its own stream (or GPU); a message is pushed by the
// SENDER's graph into the receiver's landing buffer, then a flag is raised; the receiver's
// graph waits for the flag before the segment that reads the buffer.  The flags carry the
// replay number (each graph's first node advances its party's counter; all counters move
// in lock step), so no flag needs resetting and no graph waits on another's launch order.
struct PushDesc {
  const uint8_t* src;
  uint8_t* dst;
  int64_t bytes;
  uint32_t* flag;     // the receiver's flag of this message (its memory)
  uint32_t* pieces;   // blocks of this message done (reset by the last one)
};

__global__ void __launch_bounds__(64) k_epoch_step(uint64_t* __restrict__ epoch) {
  if (threadIdx.x == 0) *epoch = *epoch + 1;
}

// grid (pieces, messages): copy, then the message's last block raises the flag
__global__ void __launch_bounds__(256)
    k_push(const PushDesc* __restrict__ d, int n, const uint64_t* __restrict__ epoch) {
  const int m = blockIdx.y;
  if (m >= n) return;
  const PushDesc c = d[m];
  const int64_t lo = (int64_t)blockIdx.x * kPiece;
  const int64_t hi = lo + kPiece < c.bytes ? lo + kPiece : c.bytes;
  if (lo < c.bytes) {
    const bool vec = ((((uintptr_t)c.src) | ((uintptr_t)c.dst)) & 15) == 0;
    if (vec) {
      const int64_t v0 = lo / 16, v1 = hi / 16;
      for (int64_t i = v0 + threadIdx.x; i < v1; i += blockDim.x)
        ((uint4*)c.dst)[i] = ((const uint4*)c.src)[i];
      for (int64_t i = v1 * 16 + threadIdx.x; i < hi; i += blockDim.x) c.dst[i] = c.src[i];
    } else {
      for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) c.dst[i] = c.src[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();  // this block's bytes before the count / the flag
    const uint32_t npieces = (uint32_t)gridDim.x;
    const uint32_t done = atomicAdd(c.pieces, 1u) + 1u;
    if (done == npieces) {
      __hip_atomic_store(c.pieces, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(c.flag, (uint32_t)*epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// one workgroup: thread i < n waits for flag i to reach this replay's number; bounded --
// after ~kMaxPolls polls it records the flag index in err (read by the host) and returns, so
// a lost message ends the replay instead of holding the GPU
constexpr uint32_t kMaxPolls = 1u << 22;

__global__ void __launch_bounds__(256)
    k_wait(const uint32_t* __restrict__ flags, int n, const uint64_t* __restrict__ epoch,
           uint32_t* __restrict__ err) {
  const uint32_t want = (uint32_t)*epoch;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t polls = 0;
    while (__hip_atomic_load(flags + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
      if (++polls >= kMaxPolls) {
        __hip_atomic_store(err, 1u + (uint32_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

}  // namespace

extern "C" {

void* mx_party_kernel_fn(int which) {
  switch (which) {
    case 0:
      return (void*)k_epoch_step;
    case 1:
      return (void*)k_push;
    case 2:
      return (void*)k_wait;
    default:
      return nullptr;
  }
}

// Uncached device memory for what another GPU writes while this GPU reads it (the per-party
// graphs' message flags and landing buffers): the owner's L2 never holds a line of it, so a
// peer's xGMI write followed by its system-scope release (k_push) is what the owner's next
// load sees -- coarse-grained memory only guarantees that at kernel / queue boundaries
// (RCCL allocates its cross-GPU flags the same way).  Zero-filled.
int mx_alloc_uncached(int dev, int64_t bytes, void** out) {
  *out = nullptr;
  if (bytes <= 0) bytes = 1;
  int cur = 0;
  hipGetDevice(&cur);
  hipSetDevice(dev);
  hipError_t e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(*out, 0, (size_t)bytes);
  hipSetDevice(cur);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    if (*out) hipFree(*out);
    *out = nullptr;
    return -(int)e;
  }
  return 0;
}

int mx_free_uncached(int dev, void* p) {
  if (!p) return 0;
  int cur = 0;
  hipGetDevice(&cur);
  hipSetDevice(dev);
  hipError_t e = hipFree(p);
  hipSetDevice(cur);
  return e == hipSuccess ? 0 : -(int)e;
}

// Peer access from device dev to device peer's memory (the push kernels' writes into another
// GPU's landing buffers and flags); already enabled is fine.
int mx_enable_peer(int dev, int peer) {
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, peer) != hipSuccess || !can) return -1;
  int cur = 0;
  hipGetDevice(&cur);
  hipSetDevice(dev);
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  hipSetDevice(cur);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return 0;
  }
  return e == hipSuccess ? 0 : -2;
}

// An asynchronous copy on ``stream`` (a replay's argument upload from pinned host memory:
// one call instead of a framework copy op)
int mx_copy_async(void* dst, const void* src, int64_t bytes, void* stream) {
  if (bytes <= 0) return 0;
  return hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, (hipStream_t)stream) ==
                 hipSuccess
             ? 0
             : -1;
}

int mx_key_refresh(void* slots, int n, const void* master, void* epoch, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_key_refresh, dim3(1), dim3(256), 0, (hipStream_t)stream,
                     (uint32_t*)slots, n, (const uint32_t*)master, (uint64_t*)epoch);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Host reference of one refreshed slot (tests): the same derivation on the CPU.
void mx_key_refresh_host(const uint32_t* master, uint64_t epoch, int slot, uint32_t* out) {
  uint32_t w[16];
  mx::chacha_block(master, epoch, (uint64_t)slot, w);
  for (int i = 0; i < 4; ++i) out[i] = w[i];
  mx::expand_key((const uint8_t*)w, out + 4);
}

// Kernel-node parameters of a batched copy over the descriptor table ``desc`` (n entries,
// the largest ``max_bytes``): the launch geometry and the function, for the graph composer.
void* mx_copy_many_fn(void) { return (void*)k_copy_many; }

int mx_copy_many_grid(int n, int64_t max_bytes, int* gx, int* gy) {
  *gx = (int)((max_bytes + kPiece - 1) / kPiece);
  if (*gx < 1) *gx = 1;
  *gy = n;
  return 0;
}

int mx_copy_many(const void* desc, int n, int64_t max_bytes, void* stream) {
  if (n <= 0) return 0;
  int gx, gy;
  mx_copy_many_grid(n, max_bytes, &gx, &gy);
  hipLaunchKernelGGL(k_copy_many, dim3(gx, gy), dim3(256), 0, (hipStream_t)stream,
                     (const CopyDesc*)desc, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
