// Per-device, thread-safe kernel attribute setup for the GEMM launchers.
//
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is a per-device setting: a process that
// launches the same kernel on several GPUs (one thread per device, or a device switch) must
// set it on each device before the first launch there.  ensure_lds_attr() keys the "done"
// set by (device of the launch stream, kernel) under a mutex.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

inline void ensure_lds_attr(const void* fn, int bytes, hipStream_t st) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  if (hipStreamGetDevice(st, &dev) != hipSuccess) (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  if (done.insert({dev, fn}).second) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (cur != dev) (void)hipSetDevice(cur);
  }
}
