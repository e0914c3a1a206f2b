// fp64 ChessNet forward (direct convolutions, activations in fp64 end to end)
// on the device: the yardstick of the load-time calibration that picks the
// fp32 AUTO path (kv_nn.hip, kv_net_calibration). It runs once per weight load
// on 64 calibration boards (about 110 GFLOP of fp64), so it is written for
// clarity, not speed. Same math as ai/model.py:51-77 with BN folded into the
// packed fp32 scale / shift (the folding every product path reads too, so the
// comparison measures the arithmetic of the candidate towers only).
#pragma once
#include <hip/hip_runtime.h>

#include "kv_common.h"

namespace kv {

// encode_board (ai/ai.py:17-30) as fp64 NHWC [board][64][16] (channels 12-15 zero)
__global__ void ref64_encode_kernel(const int8_t* __restrict__ boards, int nb, double* __restrict__ x) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // board*64 + square
    if (i >= nb * 64) return;
    const int code = boards[i];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[(size_t)i * 16 + c] = (code - 1 == c) ? 1.0 : 0.0;
}

// y = relu(conv3x3(x, w) * scale + shift (+ resid)), fp64. x: [nb][64][CIN],
// w: packed fp32 [cout][9][CIN]. Block = (board, 64 output channels): thread
// (pixel p = tid & 63, quarter q = tid >> 6) accumulates 16 channels; input
// halo and weights of each 16-channel chunk staged in LDS.
template <int CIN>
__global__ __launch_bounds__(256) void ref64_conv_kernel(const double* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const double* resid, double* y, int cout) {  // resid may alias y (in place)
    constexpr int CH = 16;  // 50 KB of LDS: 3 blocks per CU
    static_assert(CIN % CH == 0, "channel chunks");
    __shared__ double xs[100][CH];       // zero-padded 10x10 halo of the chunk
    __shared__ float ws[64][9][CH];      // this block's 64 output channels
    const int b = blockIdx.y, co0 = blockIdx.x * 64;
    const int tid = threadIdx.x, p = tid & 63, q = tid >> 6;
    const int py = p >> 3, px = p & 7;
    double acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0;
    for (int c0 = 0; c0 < CIN; c0 += CH) {
        for (int i = tid; i < 100 * CH; i += 256) {
            const int hp = i / CH, c = i % CH, hy = hp / 10 - 1, hx = hp % 10 - 1;
            xs[hp][c] = (hy >= 0 && hy < 8 && hx >= 0 && hx < 8) ? x[((size_t)b * 64 + hy * 8 + hx) * CIN + c0 + c]
                                                                 : 0.0;
        }
        for (int i = tid; i < 64 * 9 * CH; i += 256) {
            const int o = i / (9 * CH), t = (i / CH) % 9, c = i % CH;
            ws[o][t][c] = w[((size_t)(co0 + o) * 9 + t) * CIN + c0 + c];
        }
        __syncthreads();
        for (int t = 0; t < 9; ++t) {
            const int hp = (py + t / 3) * 10 + px + t % 3;
            for (int c = 0; c < CH; ++c) {
                const double xv = xs[hp][c];
#pragma unroll
                for (int j = 0; j < 16; ++j) acc[j] = __builtin_fma(xv, (double)ws[q * 16 + j][t][c], acc[j]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int co = co0 + q * 16 + j;
        const size_t o = ((size_t)b * 64 + p) * cout + co;
        double v = acc[j] * (double)scale[co] + (double)shift[co];
        if (resid) v += resid[o];
        y[o] = v > 0.0 ? v : 0.0;
    }
}

// heads (ai/model.py:64-73) in fp64 from X [nb][64][512]: policy [nb][4096], value [nb]
__global__ __launch_bounds__(256) void ref64_heads_kernel(const double* __restrict__ X, const float* __restrict__ hw,
                                                          const float* __restrict__ hs, const float* __restrict__ hb,
                                                          const float* __restrict__ pfw, const float* __restrict__ pfb,
                                                          const float* __restrict__ v1w, const float* __restrict__ v1b,
                                                          const float* __restrict__ v2w, const float* __restrict__ v2b,
                                                          double* __restrict__ policy, double* __restrict__ value) {
    __shared__ double pf[128], vf[64], hid[512], red[4];
    const int b = blockIdx.x, t = threadIdx.x;
    if (t < 192) {  // (head channel k, pixel p): k 0-1 policy, 2 value
        const int k = t / 64, p = t % 64;
        double a = 0.0;
        for (int c = 0; c < 512; ++c) a = __builtin_fma(X[((size_t)b * 64 + p) * 512 + c], (double)hw[k * 512 + c], a);
        const double v = a * (double)hs[k] + (double)hb[k];
        const double r = v > 0.0 ? v : 0.0;
        if (k < 2)
            pf[k * 64 + p] = r;  // NCHW flatten: c * 64 + square
        else
            vf[p] = r;
    }
    __syncthreads();
    for (int n = t; n < 4096; n += 256) {
        double a = (double)pfb[n];
        for (int k = 0; k < 128; ++k) a = __builtin_fma(pf[k], (double)pfw[(size_t)n * 128 + k], a);
        policy[(size_t)b * 4096 + n] = a;
    }
    for (int o = t; o < 512; o += 256) {
        double a = (double)v1b[o];
        for (int k = 0; k < 64; ++k) a = __builtin_fma(vf[k], (double)v1w[o * 64 + k], a);
        hid[o] = a > 0.0 ? a : 0.0;
    }
    __syncthreads();
    double part = (double)v2w[t] * hid[t] + (double)v2w[t + 256] * hid[t + 256];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m);
    if ((t & 63) == 0) red[t >> 6] = part;
    __syncthreads();
    if (t == 0) value[b] = tanh(red[0] + red[1] + red[2] + red[3] + (double)v2b[0]);
}

// max |a[i] - r[i]| over n (fp32 candidate vs fp64 reference) into *out as the
// bits of a non-negative double (which order like unsigned integers)
__global__ void ref64_maxdiff_kernel(const float* __restrict__ a, const double* __restrict__ r, size_t n,
                                     unsigned long long* out) {
    double m = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double d = fabs((double)a[i] - r[i]);
        m = (d > m || d != d) ? (d != d ? INFINITY : d) : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double v = __shfl_xor(m, o, 64);
        m = v > m ? v : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

}  // namespace kv
