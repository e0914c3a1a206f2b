// Shared helpers for the knightvision_amd HIP library (libkv.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/kv.h"

namespace kv {

void set_error(const char* fmt, ...);

}  // namespace kv

#define KV_HIP(call)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) {                                                                       \
            kv::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_));        \
            return KV_EHIP;                                                                           \
        }                                                                                             \
    } while (0)

#define KV_REQUIRE(cond, code, ...)         \
    do {                                    \
        if (!(cond)) {                      \
            kv::set_error(__VA_ARGS__);     \
            return (code);                  \
        }                                   \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
