// common.h -- shared host/device helpers of libnngp_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/nngp.h"

namespace nngp {

// thread-local last error, returned by nngp_last_error()
void set_error(const char *fmt, ...);

#define NNGP_HIP_CHECK(expr)                                                                 \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) {                                                              \
            ::nngp::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),         \
                              __FILE__, __LINE__);                                           \
            return NNGP_E_HIP;                                                               \
        }                                                                                    \
    } while (0)

#define NNGP_REQUIRE(cond, ...)                                                              \
    do {                                                                                     \
        if (!(cond)) {                                                                       \
            ::nngp::set_error(__VA_ARGS__);                                                  \
            return NNGP_E_ARG;                                                               \
        }                                                                                    \
    } while (0)

// launch-error check right after a <<<>>> launch
#define NNGP_LAUNCH_CHECK()                                                                  \
    do {                                                                                     \
        hipError_t _e = hipGetLastError();                                                   \
        if (_e != hipSuccess) {                                                              \
            ::nngp::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e),     \
                              __FILE__, __LINE__);                                           \
            return NNGP_E_HIP;                                                               \
        }                                                                                    \
    } while (0)

// Grow-only device scratch owned by the library (one per device), so that steady-state
// calls never allocate.  Not thread-safe across host threads sharing a device.
void *workspace(size_t bytes, int *err);

}  // namespace nngp
