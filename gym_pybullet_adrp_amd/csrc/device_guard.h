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
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// The same for the handle-free entry points (adrp_gae, adrp_compact_rows, adrp_memcpy_async,
// adrp_stream_synchronize): a non-null stream names its device, and the work runs there whatever the
// calling thread's current device is.  A null stream is the current device's null stream, so the
// caller makes the env's device current (vec_env.py / rollout.py do).
struct StreamDeviceGuard {
    int prev = -1;
    explicit StreamDeviceGuard(hipStream_t s) {
        int dev = -1, cur = -1;
        if (s == nullptr || hipStreamGetDevice(s, &dev) != hipSuccess) return;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~StreamDeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    StreamDeviceGuard(const StreamDeviceGuard&) = delete;
    StreamDeviceGuard& operator=(const StreamDeviceGuard&) = delete;
};
