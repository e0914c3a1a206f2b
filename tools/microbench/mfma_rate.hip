// MFMA issue-rate probe: back-to-back MFMAs on register operands (4 independent
// accumulators per wave), every CU busy; prints ops/s per instruction form.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));

template <int FORM>
__global__ __launch_bounds__(256) void k(int iters, int seed, int* out) {
    i32x4 a = {seed, seed + 1, seed + 2, (int)threadIdx.x}, b = {seed * 3, 7, 9, (int)threadIdx.x};
    i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    i32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    for (int i = 0; i < iters; ++i) {
        if constexpr (FORM == 0) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
        } else {
            d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d1, 0, 0, 0);
            d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d2, 0, 0, 0);
            d3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d3, 0, 0, 0);
        }
    }
    int s = 0;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    for (int r = 0; r < 4; ++r) s += d0[r] + d1[r] + d2[r] + d3[r];
    if (s == 0x12345) out[0] = s;
}

template <int FORM>
static void run(const char* name, double ops_per_inst) {
    int* out;
    hipMalloc(&out, 4);
    const int iters = 20000, blocks = 256 * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<FORM>, dim3(blocks), dim3(256), 0, 0, 100, 1, out);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<FORM>, dim3(blocks), dim3(256), 0, 0, iters, 1, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double insts = (double)blocks * 4 * iters * 4;  // waves x iters x 4 MFMAs
    printf("%s: %.3f ms, %.1f TOPS (%.1f cycles/inst/SIMD at 2.4 GHz)\n", name, ms,
           insts * ops_per_inst / (ms * 1e-3) / 1e12, (ms * 1e-3 * 2.4e9) / (insts / 1024.0));
    hipFree(out);
}

int main() {
    run<0>("v_mfma_i32_32x32x32_i8", 32.0 * 32 * 32 * 2);
    run<1>("v_mfma_i32_16x16x64_i8", 16.0 * 16 * 64 * 2);
    return 0;
}
