// device_guard.h — scoped current-device switch for the C-ABI entry points (libadrp).
#pragma once

#include <hip/hip_runtime.h>

// Runs a C-ABI call on the handle's device and gives the calling thread its current device back:
// hipGetDevice is a thread-local read, hipSetDevice happens only when the devices differ (so the
// per-step path costs nothing when the caller already works on the handle's device, and a
// multi-GPU caller's current device is never changed behind its back).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};
