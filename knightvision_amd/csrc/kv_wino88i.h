// F(8x8) Winograd GEMMs on the int8 matrix cores with exact integer
// accumulation (KV_PATH_WINO88_I8): the fp64 Winograd domain of kv_wino88d.h
// (U, V, M and both transforms in fp64) with the GEMM's products taken from
// int8 digits instead of v_mfma_f64.
//
// Every row of V (point xi, board) and of U (xi, output channel) -- K input
// channels -- is scaled by a power of two 2^-e to |a| < 1 (e from the row's
// largest magnitude) and split into 5 signed int8 digits,
//     a * 2^-e = sum_i d_i * 2^(-7(i+1)) + rest,  |d_i| <= 127,  |rest| <= 2^-35,
// d_i = rint(t_i), t_{i+1} = 128 (t_i - d_i), t_0 = 128 a 2^-e (each step exact
// in fp64). The product keeps the digit pairs with i + j <= S - 1, S = 5:
//     M = 2^(e_v + e_u - 14) * sum_{l < S} 2^(-7l) * sum_{i+j=l} (D_i . E_j)
// where each D_i . E_j is one v_mfma_i32_32x32x32_i8 chain over K (exact in
// int32: |level l| <= 5 * 512 * 127^2 < 2^31), and the five level sums are
// combined in fp64 exactly (at most 51 significant bits). The result is the
// exact dot product of the digit-truncated rows: no rounding anywhere in the
// GEMM, so it is independent of k order, tile shape and batch by construction.
// 15 int8 products at 32x the fp32 MFMA rate (the int8 rate is 2x bf16's)
// against v_mfma_f64 at half the fp32 rate: a ~4x higher ceiling than the fp64
// GEMM it replaces, at the same accuracy (host emulation on the stress weights:
// max |dlogit| 2.4e-6 against fp64's 2.9e-6, profiles/r04_ozaki_emulation.log).
//
// Layouts: digits [slab xi][row][K / 32][5][32] int8 (one 160-B chunk per 32 k:
// the five digits' 32 bytes each), exponents [xi][row] int32.
#pragma once
#include <hip/hip_runtime.h>

#include "kv_common.h"
#include "kv_wino88d.h"  // f64x2

namespace kv {

constexpr int kI8Digits = 5;                  // digits stored per value
constexpr int kI8Chunk = kI8Digits * 32;      // bytes of one row's 32-k chunk
constexpr int kI8Levels = 5;                  // S: the GEMM keeps digit pairs i + j < S

typedef int i8x16_t __attribute__((ext_vector_type(4)));   // 16 int8 in 4 dwords (MFMA A / B)
typedef int i32x16_t __attribute__((ext_vector_type(16)));  // 32x32 int32 accumulator block

// The digits and exponent of `nslab` slabs of n rows of K fp64 values: row r of
// slab x is src[(x * slab_rows + r) * K ...]; digits go to dst at the same row
// index (K * 5 bytes per row), the exponent to ex[x * slab_rows + r]. One wave
// per row; lane l holds channels [l * K/64, (l + 1) * K/64).
template <int K>
__global__ __launch_bounds__(256) void wino88i_slice_kernel(const double* __restrict__ src, int n, int slab_rows,
                                                            int nslab, int8_t* __restrict__ dst,
                                                            int* __restrict__ ex) {
    static_assert(K == 256 || K == 512, "rows of 256 or 512 channels");
    constexpr int CPL = K / 64;  // 4 or 8 channels per lane
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= n * nslab) return;  // whole waves
    const size_t row = (size_t)(gw / n) * slab_rows + gw % n;
    const double* s = src + row * K + lane * CPL;
    double v[CPL];
#pragma unroll
    for (int i = 0; i < CPL; i += 2) {
        const f64x2 p = *(const f64x2*)(s + i);
        v[i] = p[0];
        v[i + 1] = p[1];
    }
    // the high words of |v| order like |v|: their max carries the row's largest biased exponent E,
    // and every |v| < 2^(E - 1022)
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        const unsigned hw = (unsigned)(__double_as_longlong(v[i]) >> 32) & 0x7fffffffu;
        m = hw > m ? hw : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned t = (unsigned)__shfl_xor((int)m, o, 64);
        m = t > m ? t : m;
    }
    const int e = m ? (int)(m >> 20) - 1022 : 0;  // an all-zero row: digits 0
    if (lane == 0) ex[row] = e;
    unsigned long long pk[kI8Digits] = {};
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        double t = ldexp(v[i], -e);  // |t| < 1, exact
#pragma unroll
        for (int d = 0; d < kI8Digits; ++d) {
            t *= 128.0;
            double q = rint(t);
            q = q > 127.0 ? 127.0 : (q < -127.0 ? -127.0 : q);  // a clamped digit carries into the next
            t -= q;
            pk[d] |= (unsigned long long)(unsigned char)(signed char)(int)q << (8 * i);
        }
    }
    const int c = lane * CPL;
    int8_t* o = dst + row * (size_t)(K / 32) * kI8Chunk + (c / 32) * kI8Chunk + (c % 32);
#pragma unroll
    for (int d = 0; d < kI8Digits; ++d) {
        if constexpr (CPL == 8)
            *(unsigned long long*)(o + d * 32) = pk[d];
        else
            *(unsigned*)(o + d * 32) = (unsigned)pk[d];
    }
}

// Workgroup tile: WM rows x WN output channels of one point, WR x WC waves of
// (MT x 32) x (NT x 32). Each 32-k stage stages S digits' 32 bytes per row in
// LDS rows of S * 32 + 16 bytes (the pad makes the 16 rows of a ds_read_b128
// lane group hit 16 distinct 4-bank groups), double-buffered.
template <int S, int WR, int WC, int MT, int NT>
struct Wino88iTile {
    static constexpr int THREADS = WR * WC * 64;
    static constexpr int WM = WR * MT * 32, WN = WC * NT * 32;
    static constexpr int RB = S * 32, RS = RB + 16;
    static constexpr size_t STAGE = (size_t)(WM + WN) * RS;
    static constexpr size_t BYTES = 2 * STAGE;
};

// M[xi] (fp64 [xi][stride rows][cout]) = V[xi] x U[xi]^T from the digits (see the header comment).
// XCD-aware tile order as kv_wino.h's wino_gemm_kernel.
template <int K, int S, int WR, int WC, int MT, int NT>
__global__ __launch_bounds__(WR * WC * 64) void wino88i_gemm_kernel(const int8_t* __restrict__ V8,
                                                                      const int* __restrict__ ev,
                                                                      const int8_t* __restrict__ U8,
                                                                      const int* __restrict__ eu,
                                                                      double* __restrict__ M, int rows, int cout,
                                                                      int stride) {
    using T = Wino88iTile<S, WR, WC, MT, NT>;
    constexpr int WM = T::WM, WN = T::WN, TH = T::THREADS, RS = T::RS;
    constexpr int NK = K / 32;
    constexpr int CH = T::RB / 16;                 // 16-byte pieces per row and stage
    constexpr int TOT = (WM + WN) * CH;
    constexpr int NQ = (TOT + TH - 1) / TH;
    constexpr size_t ROWB = (size_t)(K / 32) * kI8Chunk;  // bytes of one digit row
    static_assert(S >= 1 && S <= kI8Digits, "digit levels");

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8[];
    char* const L0 = (char*)lds_i8;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WC, wn = wave % WC;
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x;  // a multiple of 8
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx / (CT * RT);
    const int n_base = (idx % CT) * WN;
    const int r_base = ((idx / CT) % RT) * WM;
    const int8_t* Va = V8 + ((size_t)xi * stride + r_base) * ROWB;
    const int8_t* Ub = U8 + ((size_t)xi * cout + n_base) * ROWB;

    i8x16_t rg[NQ];
    auto load = [&](int kt) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + q * TH;
            if (TOT % TH == 0 || i < TOT) {
                const int r = i / CH, c = i % CH;
                const int8_t* p = (r < WM ? Va + (size_t)r * ROWB : Ub + (size_t)(r - WM) * ROWB) + kt * kI8Chunk;
                rg[q] = *(const i8x16_t*)(p + c * 16);
            }
        }
    };
    auto store = [&](char* buf) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + q * TH;
            if (TOT % TH == 0 || i < TOT) *(i8x16_t*)(buf + (i / CH) * RS + (i % CH) * 16) = rg[q];
        }
    };

    // A: lane l holds A[row l & 31][k = 16 (l >> 5) + j], B: B[k = 16 (l >> 5) + j][col l & 31]
    const int lr = lane & 31, lh = lane >> 5;
    int aoff[MT], boff[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) aoff[mt] = (wm * MT * 32 + mt * 32 + lr) * RS + lh * 16;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) boff[nt] = (WM + wn * NT * 32 + nt * 32 + lr) * RS + lh * 16;

    i32x16_t acc[S][MT][NT];
#pragma unroll
    for (int l = 0; l < S; ++l)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[l][i][j] = i32x16_t{};

    load(0);
    for (int kt = 0; kt < NK; ++kt) {
        char* buf = L0 + (kt & 1) * T::STAGE;
        store(buf);
        if (kt + 1 < NK) load(kt + 1);
        __syncthreads();
        i8x16_t a[S][MT], b[S][NT];
#pragma unroll
        for (int d = 0; d < S; ++d) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) a[d][mt] = *(const i8x16_t*)(buf + aoff[mt] + d * 32);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) b[d][nt] = *(const i8x16_t*)(buf + boff[nt] + d * 32);
        }
#pragma unroll
        for (int l = 0; l < S; ++l)
#pragma unroll
            for (int i = 0; i <= l; ++i)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[l][mt][nt] =
                            __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i][mt], b[l - i][nt], acc[l][mt][nt], 0, 0, 0);
    }

    // D: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) inside the 32 x 32 block
    const int* evx = ev + (size_t)xi * stride + r_base + wm * MT * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = n_base + wn * NT * 32 + nt * 32 + lr;
        const int ec = eu[(size_t)xi * cout + col] - 14;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                double m = (double)acc[S - 1][mt][nt][r];
#pragma unroll
                for (int l = S - 2; l >= 0; --l) m = __builtin_fma(m, 0.0078125, (double)acc[l][mt][nt][r]);  // exact
                M[((size_t)xi * stride + r_base + wm * MT * 32 + row) * cout + col] = ldexp(m, evx[row] + ec);
            }
        }
    }
}

}  // namespace kv
