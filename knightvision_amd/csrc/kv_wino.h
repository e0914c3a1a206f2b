// Winograd F(4x4, 3x3) for the 3x3 convs with Cin 256 / 512 (ai/model.py
// conv2 and the ten ResidualBlock convs, :36, :11-14).
//
// An 8x8 board is 2x2 output tiles of 4x4; each tile reads a 6x6 input patch
// (zero padded). Per layer:
//   U[xi][cout][cin] = (G g G^T)[xi]       once at load time (fp64 -> fp32)
//   V[xi][tile][cin] = (B^T d B)[xi]       input transform
//   M[xi][tile][cout] = sum_cin V[xi][tile][cin] * U[xi][cout][cin]
//                                          36 independent GEMMs on the f32 MFMA
//   Y = A^T M A, then folded BN scale/shift (+ residual) + ReLU, and straight
//   into the next layer's V                output transform
// The GEMMs do 36*4 = 144 MACs per (board, cin, cout) instead of 64*9 = 576:
// 4x fewer MFMA FLOPs than the direct implicit GEMM. fp32 throughout; the
// transform constants are the standard Lavin-Gray points (0, +-1, +-2, inf),
// measured on the host at 1.2-4x the direct conv's rounding error.
//
// Layouts (fp32): V and M are [36][rows = board*4 + tile][C] (C contiguous),
// U is [36][Cout][Cin]. tile = ty*2 + tx.
#pragma once
#include <hip/hip_runtime.h>

#include "kv_common.h"

namespace kv {

constexpr int WN_XI = 36;

// B^T (6x6) applied to one 6-vector
__device__ inline void wino_bt(const float* d, float* o) {
    o[0] = 4.f * d[0] - 5.f * d[2] + d[4];
    o[1] = -4.f * d[1] - 4.f * d[2] + d[3] + d[4];
    o[2] = 4.f * d[1] - 4.f * d[2] - d[3] + d[4];
    o[3] = -2.f * d[1] - d[2] + 2.f * d[3] + d[4];
    o[4] = 2.f * d[1] - d[2] - 2.f * d[3] + d[4];
    o[5] = 4.f * d[1] - 5.f * d[3] + d[5];
}

// A^T (4x6) applied to one 6-vector
__device__ inline void wino_at(const float* m, float* o) {
    o[0] = m[0] + m[1] + m[2] + m[3] + m[4];
    o[1] = m[1] - m[2] + 2.f * m[3] - 2.f * m[4];
    o[2] = m[1] + m[2] + 4.f * m[3] + 4.f * m[4];
    o[3] = m[1] - m[2] + 8.f * m[3] - 8.f * m[4] + m[5];
}

// V of one tile (t = ty*2 + tx) of one channel from its 6x6 input patch d
// (row-major, zero padded) -> V[xi][row][c] at stride xi_stride
__device__ inline void wino_input_tile(const float (&d)[36], float* V, size_t off, size_t xi_stride) {
    float tmp[6][6];  // B^T d (columns)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        float col[6], o[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = d[i * 6 + j];
        wino_bt(col, o);
#pragma unroll
        for (int i = 0; i < 6; ++i) tmp[i][j] = o[i];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        float o[6];
        wino_bt(tmp[i], o);
#pragma unroll
        for (int j = 0; j < 6; ++j) V[(size_t)(i * 6 + j) * xi_stride + off] = o[j];
    }
}

// U = G g G^T for every (cout, cin) of one conv, in fp64, rounded once to fp32.
// w: packed [Cout][9][Cin]; U: [36][Cout][Cin].
__global__ void wino_weights_kernel(const float* __restrict__ w, int cout, int cin, float* __restrict__ U) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)cout * cin) return;
    const int co = (int)(i / cin), ci = (int)(i % cin);
    double g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = (double)w[((size_t)co * 9 + t) * cin + ci];
    const double G[6][3] = {{0.25, 0, 0},
                            {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                            {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                            {1.0 / 24, 1.0 / 12, 1.0 / 6},
                            {1.0 / 24, -1.0 / 12, 1.0 / 6},
                            {0, 0, 1}};
    double tg[6][3];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int k = 0; k < 3; ++k) tg[a][k] = G[a][0] * g[0][k] + G[a][1] * g[1][k] + G[a][2] * g[2][k];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            const double u = tg[a][0] * G[b][0] + tg[a][1] * G[b][1] + tg[a][2] * G[b][2];
            U[((size_t)(a * 6 + b) * cout + co) * cin + ci] = (float)u;
        }
}

// input transform of an NHWC activation [boards][64][C] (the stem output).
// Block: 4 waves = the 4 tiles of one board, lane = channel (64 per block).
template <int C>
__global__ __launch_bounds__(256) void wino_in_kernel(const float* __restrict__ X, int rows, float* __restrict__ V) {
    const int t = threadIdx.x >> 6, c = blockIdx.x * 64 + (threadIdx.x & 63), b = blockIdx.y;
    const int y0 = (t >> 1) * 4 - 1, x0 = (t & 1) * 4 - 1;
    float d[36];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int yy = y0 + i, xx = x0 + j;
            d[i * 6 + j] = (yy >= 0 && yy < 8 && xx >= 0 && xx < 8) ? X[((size_t)b * 64 + yy * 8 + xx) * C + c] : 0.f;
        }
    wino_input_tile(d, V, ((size_t)b * 4 + t) * C + c, (size_t)rows * C);
}

// output transform of layer l + folded BN (+ residual) + ReLU -> Y (NHWC,
// optional) and the next layer's V (optional). M: [36][rows][512].
// Block: 4 waves = the 4 tiles of one board, lane = channel (64 per block);
// the activated 8x8 planes are exchanged through LDS ([pixel][channel],
// conflict-free) for the next layer's overlapping 6x6 patches.
template <bool RESID, bool WRITE_Y, bool NEXT_V>
__global__ __launch_bounds__(256) void wino_out_kernel(const float* __restrict__ M, int rows,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       const float* resid, float* Y, float* __restrict__ Vn) {
    constexpr int C = 512;
    __shared__ float plane[64][64];  // [pixel][channel]
    const int t = threadIdx.x >> 6, cl = threadIdx.x & 63;
    const int c = blockIdx.x * 64 + cl, b = blockIdx.y;
    const size_t xs = (size_t)rows * C;
    const size_t base = ((size_t)b * 4 + t) * C + c;
    const float sc = scale[c], sh = shift[c];
    float tmp[4][6];  // A^T m (columns)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        float col[6], o[4];
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = M[(size_t)(i * 6 + j) * xs + base];
        wino_at(col, o);
#pragma unroll
        for (int i = 0; i < 4; ++i) tmp[i][j] = o[i];
    }
    const int y0 = (t >> 1) * 4, x0 = (t & 1) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float o[4];
        wino_at(tmp[i], o);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = (y0 + i) * 8 + x0 + j;
            const size_t idx = ((size_t)b * 64 + p) * C + c;
            float v = o[j] * sc + sh;
            if (RESID) v += resid[idx];
            v = v > 0.f ? v : 0.f;
            if (WRITE_Y) Y[idx] = v;
            if (NEXT_V) plane[p][cl] = v;
        }
    }
    if (!NEXT_V) return;
    __syncthreads();
    float d[36];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int yy = y0 - 1 + i, xx = x0 - 1 + j;
            d[i * 6 + j] = (yy >= 0 && yy < 8 && xx >= 0 && xx < 8) ? plane[yy * 8 + xx][cl] : 0.f;
        }
    wino_input_tile(d, Vn, base, xs);
}

// The 36 GEMMs M[xi] = V[xi] x U[xi]^T on v_mfma_f32_32x32x2_f32, over `rows`
// rows of V / M whose xi slabs are `stride` rows apart (a batch slice).
// Workgroup: WM x WN outputs of one xi; 8 waves in a WR x (8/WR) grid, each
// (MT*32) x (NT*32). K (= Cin) streams through LDS in k-tiles of 32
// (double-buffered A [WM][32] and B [WN][32], row stride 36 floats:
// conflict-free ds_read_b128), one barrier per k-tile, the next k-tile's
// global loads issued before the current tile's MFMAs.
template <int WR, int WC, int MT, int NT>
struct WinoTile {
    static constexpr int THREADS = WR * WC * 64;
    static constexpr int WM = WR * MT * 32, WN = WC * NT * 32;
    static constexpr size_t BYTES = (size_t)(2 * WM * 36 + 2 * WN * 36) * 4;
};

template <int K, int WR, int WC, int MT, int NT>
__global__ __launch_bounds__(WR * WC * 64) void wino_gemm_kernel(const float* __restrict__ V,
                                                                   const float* __restrict__ U,
                                                                   float* __restrict__ M, int rows, int cout,
                                                                   int stride) {
    using T = WinoTile<WR, WC, MT, NT>;
    constexpr int WM = T::WM, WN = T::WN, TH = T::THREADS;
    constexpr int CK = 32, PS = 36;
    constexpr int NK = K / CK;
    constexpr int KQ = CK / 4;
    constexpr int A_F4 = (WM * KQ) / TH;
    constexpr int B_F4 = (WN * KQ) / TH;
    constexpr int ABUF = WM * PS, BBUF = WN * PS;
    static_assert(A_F4 >= 1 && B_F4 >= 1 && (WM * KQ) % TH == 0 && (WN * KQ) % TH == 0, "tile shape");

    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* const A0 = smem;
    float* const A1 = smem + ABUF;
    float* const B0 = smem + 2 * ABUF;
    float* const B1 = B0 + BBUF;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WC, wn = wave % WC;
    // XCD-aware tile order: blocks b and b+8 share an XCD (round-robin
    // dealing), so each group of 8 gets a contiguous run of the xi-major tile
    // order -- the 4 column tiles of a row panel and the row panels of one xi
    // run on one XCD and re-read V / U from its L2 instead of HBM.
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = WN_XI * RT * CT;  // a multiple of 8 (36 * 4 * RT)
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx / (CT * RT);
    const int n_base = (idx % CT) * WN;
    const int r_base = ((idx / CT) % RT) * WM;
    const float* Va = V + ((size_t)xi * stride + r_base) * K;
    const float* Ub = U + ((size_t)xi * cout + n_base) * K;

    f32x4 ra[A_F4];
    f32x4 rb[B_F4];
    auto loadA = [&](int kt) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + q * TH;
            ra[q] = *(const f32x4*)(Va + (size_t)(idx / KQ) * K + kt * CK + (idx % KQ) * 4);
        }
    };
    auto storeA = [&](float* Ab) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + q * TH;
            *(f32x4*)(Ab + (idx / KQ) * PS + (idx % KQ) * 4) = ra[q];
        }
    };
    auto loadB = [&](int kt) {
#pragma unroll
        for (int q = 0; q < B_F4; ++q) {
            const int idx = tid + q * TH;
            rb[q] = *(const f32x4*)(Ub + (size_t)(idx / KQ) * K + kt * CK + (idx % KQ) * 4);
        }
    };
    auto storeB = [&](float* Bb) {
#pragma unroll
        for (int q = 0; q < B_F4; ++q) {
            const int idx = tid + q * TH;
            *(f32x4*)(Bb + (idx / KQ) * PS + (idx % KQ) * 4) = rb[q];
        }
    };

    const int h = lane >> 5, li = lane & 31;
    int aoff[MT], boff[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) aoff[mt] = (wm * MT * 32 + mt * 32 + li) * PS + 4 * h;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) boff[nt] = (wn * NT * 32 + nt * 32 + li) * PS + 4 * h;

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    loadA(0);
    loadB(0);
    for (int kt = 0; kt < NK; ++kt) {
        float* Ab = (kt & 1) ? A1 : A0;
        float* Bb = (kt & 1) ? B1 : B0;
        storeA(Ab);
        storeB(Bb);
        if (kt + 1 < NK) {
            loadA(kt + 1);
            loadB(kt + 1);
        }
        __syncthreads();
        // fragments for step s+1 are read from LDS while step s's MFMAs run
        f32x4 a[2][MT], b[2][NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[0][mt] = *(const f32x4*)(Ab + aoff[mt]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b[0][nt] = *(const f32x4*)(Bb + boff[nt]);
#pragma unroll
        for (int s = 0; s < CK / 8; ++s) {
            const int cb = s & 1, nb = cb ^ 1;
            if (s + 1 < CK / 8) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) a[nb][mt] = *(const f32x4*)(Ab + aoff[mt] + 8 * (s + 1));
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) b[nb][nt] = *(const f32x4*)(Bb + boff[nt] + 8 * (s + 1));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] =
                            __builtin_amdgcn_mfma_f32_32x32x2f32(a[cb][mt][j], b[cb][nt][j], acc[mt][nt], 0, 0, 0);
        }
    }

    // D[row][col]: row = (r&3) + 8*(r>>2) + 4*h inside the 32-row tile, col = li
    float* Mo = M + ((size_t)xi * stride + r_base + wm * MT * 32) * cout + n_base + wn * NT * 32 + li;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                Mo[(size_t)row * cout + nt * 32] = acc[mt][nt][r];
            }
}

}  // namespace kv
