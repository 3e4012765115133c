// hip_guard.hpp — the caller's current HIP device survives every entry point of the C ABI.
//
// hipSetDevice is per-thread state. The engine switches to its own device to enqueue work, and a
// multi-GPU caller (or torch in the same process, which keeps its own notion of the current
// device) must find the device it had set when the call returns. Every NEB_API entry point that
// touches HIP holds a DeviceGuard for its whole body: it records the caller's device on entry and
// restores it on exit, whatever the body switched to in between.
#pragma once
#include <hip/hip_runtime.h>

struct DeviceGuard {
    int prev = -1;
    DeviceGuard() {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
    }
    explicit DeviceGuard(int dev) : DeviceGuard() {
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};
