// ldpc_internal.h -- shared helpers of libldpc_hip.so (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/ldpc_hip.h"

// Records a thread-local message for ldpc_last_error() and returns `code`.
int ldpc_fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// Makes `dev` the calling thread's current device for the guard's scope and
// restores the caller's device on exit (every ABI entry that touches a device).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};
