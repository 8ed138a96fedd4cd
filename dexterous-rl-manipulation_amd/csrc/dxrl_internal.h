// dxrl_internal.h -- handle struct, error plumbing and launch helpers shared
// by the translation units of libdxrl.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "dxrl_device.h"

struct dxrl_env {
    dxrl_env_config cfg;
    dxrl_env_layout layout;
    int32_t device;
    char* base;
    dxrl::EnvSoA soa;
    dxrl_curriculum* curricula;  // device table
    int32_t n_curricula;
};

namespace dxrl {

void set_error(const char* fmt, ...);

inline int hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return DXRL_E_HIP;
    }
    return DXRL_OK;
}
inline int launch_check(const char* what) { return hip_check(hipGetLastError(), what); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline Weights weights_of(const dxrl_env_config& c) {
    return Weights{c.distance_weight, c.contact_weight, c.closure_weight, c.stability_weight};
}

// RAII device guard: make `dev` current for the call, restore afterwards.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

constexpr int kBlock = 256;

}  // namespace dxrl

#define DXRL_REQUIRE(cond, ...)          \
    do {                                  \
        if (!(cond)) {                    \
            dxrl::set_error(__VA_ARGS__); \
            return DXRL_E_INVALID;        \
        }                                 \
    } while (0)
