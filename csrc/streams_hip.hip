// Stream-placement probes (scripts/coresidency.py): a copy kernel with a fixed, small number
// of workgroups -- the shape of an RCCL point-to-point channel kernel (a few persistent
// workgroups moving a message) -- and streams restricted to a subset of the CUs
// (hipExtStreamCreateWithCUMask).  They answer whether a communication kernel issued on a
// second stream gets CUs while the CRT GEMM (one 8-wave workgroup per CU, 242 VGPRs,
// 96 KB LDS) occupies the device, and what leaving k CUs free costs the GEMM.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>

namespace {

__global__ void __launch_bounds__(256) k_copy_channels(uint4* __restrict__ dst,
                                                        const uint4* __restrict__ src,
                                                        int64_t n16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

}  // namespace

extern "C" {

// Copy ``bytes`` (a multiple of 16) with exactly ``nblocks`` workgroups of 256 threads.
int mx_copy_channels(void* dst, const void* src, int64_t bytes, int nblocks, void* stream) {
  if (bytes % 16 || nblocks < 1) return -2;
  hipLaunchKernelGGL(k_copy_channels, dim3(nblocks), dim3(256), 0, (hipStream_t)stream,
                     (uint4*)dst, (const uint4*)src, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A stream on the current device whose kernels run only on the CUs of ``mask`` (``words``
// 32-bit words, bit i = CU i in the runtime's numbering).
int mx_stream_cumask(const uint32_t* mask, int words, void** out) {
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return -1;
  *out = (void*)s;
  return 0;
}

int mx_stream_destroy(void* s) { return hipStreamDestroy((hipStream_t)s) == hipSuccess ? 0 : -1; }

}  // extern "C"
