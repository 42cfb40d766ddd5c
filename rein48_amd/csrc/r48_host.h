// r48_host.h -- host-side helpers shared by the C-ABI entry points (defined in r48_env.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace r48 {
void set_last_error(const std::string &msg);
// Device the stream's work runs on (the null stream: the calling thread's current device).
int stream_device(hipStream_t stream);
// Compute-unit count of `device` (queried once per device; 256 if the query fails).
int device_cus(int device);
// hipFuncAttributeMaxDynamicSharedMemorySize = bytes for `kernel` on `device`, set once per
// (kernel, device) pair; thread-safe (a mutex around a small set), the caller's current device kept.
// false (and r48_last_error set) when the opt-in fails; only a success is remembered.
bool ensure_dynamic_lds(const void *kernel, int bytes, int device);
}  // namespace r48
