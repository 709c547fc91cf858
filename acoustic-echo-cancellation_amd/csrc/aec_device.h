// aec_device.h — scoped HIP device selection for the C ABI entry points.
//
// Every entry point runs on its handle's device but must leave the caller's
// current device as it found it: a torchrun rank bound to cuda:k that calls
// into the library must still be on cuda:k afterwards (its RCCL collectives
// run on the current device).
#pragma once
#include <hip/hip_runtime.h>

namespace aec {

struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace aec
