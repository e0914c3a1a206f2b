// Shared helpers for the knightvision_amd HIP library (libkv.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/kv.h"

namespace kv {

void set_error(const char* fmt, ...);

// a device buffer freed with its scope (the device-test entry points)
template <class T>
struct DevBuf {
    T* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, n * sizeof(T) + 16); }
};

// a HIP event destroyed on every return path
struct DevEvent {
    hipEvent_t e = nullptr;
    ~DevEvent() {
        if (e) (void)hipEventDestroy(e);
    }
    hipError_t create() { return hipEventCreate(&e); }
};

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
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// fp32 -> bf16 bits, round to nearest even (finite inputs)
__device__ inline unsigned bf16_rne(float x) {
    const unsigned u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
