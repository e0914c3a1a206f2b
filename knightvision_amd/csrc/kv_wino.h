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

// B^T (6x6) applied to one 6-vector. The only inexact product is the -5
// term: it is an explicit fma so that its rounding does not depend on how the
// compiler contracts a given call site (stem_kernel's inlined zero padding vs
// wino_in_kernel's loads) -- every caller gives the same bits.
__device__ inline void wino_bt(const float* d, float* o) {
    o[0] = __builtin_fmaf(-5.f, d[2], 4.f * d[0]) + d[4];
    o[1] = -4.f * d[1] - 4.f * d[2] + d[3] + d[4];
    o[2] = 4.f * d[1] - 4.f * d[2] - d[3] + d[4];
    o[3] = -2.f * d[1] - d[2] + 2.f * d[3] + d[4];
    o[4] = 2.f * d[1] - d[2] - 2.f * d[3] + d[4];
    o[5] = __builtin_fmaf(-5.f, d[3], 4.f * d[1]) + d[5];
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
template <int WR, int WC, int MT, int NT, int CK = 32>
struct WinoTile {
    static constexpr int THREADS = WR * WC * 64;
    static constexpr int WM = WR * MT * 32, WN = WC * NT * 32;
    static constexpr int PS = CK + 4;  // LDS row stride (floats): 36 / 20, conflict-free ds_read_b128
    static constexpr size_t BYTES = (size_t)(2 * WM * PS + 2 * WN * PS) * 4;
};

template <int K, int WR, int WC, int MT, int NT, int CK = 32>
__global__ __launch_bounds__(WR * WC * 64) void wino_gemm_kernel(const float* __restrict__ V,
                                                                   const float* __restrict__ U,
                                                                   float* __restrict__ M, int rows, int cout,
                                                                   int stride) {
    using T = WinoTile<WR, WC, MT, NT, CK>;
    constexpr int WM = T::WM, WN = T::WN, TH = T::THREADS;
    constexpr int PS = T::PS;
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

// ------------------------------------------------ bf16x6 (fp32-accurate) --
// x == h + m + l exactly for normal fp32 x: h = bf16(x), m = bf16(x - h),
// l = bf16(x - h - m) (each difference is exact in fp32, the last one has at
// most 8 significant bits). A product x*y is the sum of the 9 piece products;
// the GEMM keeps the six with weight >= 2^-16 (hh, hm, mh, hl, lh, mm) -- the
// dropped three are ~2^-24 of the product, the size of fp32's own rounding --
// each an exact bf16 x bf16 product accumulated in fp32 on
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate: 6 products = 2.67x).
// Measured on the peaked weight set: max |dlogit| 4.9e-6 (fp32 direct 4.4e-6).
__device__ inline void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
    h = bf16_rne(x);
    const float r1 = x - __uint_as_float(h << 16);
    m = bf16_rne(r1);
    const float r2 = r1 - __uint_as_float(m << 16);
    l = bf16_rne(r2);
}

__global__ void split3_kernel(const float* __restrict__ w, size_t n, uint16_t* __restrict__ h,
                              uint16_t* __restrict__ m, uint16_t* __restrict__ l) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned a, b, c;
    split3(w[i], a, b, c);
    h[i] = (uint16_t)a;
    m[i] = (uint16_t)b;
    l[i] = (uint16_t)c;
}

// M[xi] = V[xi] x U[xi]^T with both operands in three bf16 pieces. V stays
// fp32 in HBM and is split while it is staged into LDS; U is split once at
// load time. Workgroup: 128 rows x 128 channels of one xi, 4 waves of 64x64
// (2x2 tiles), k-tiles of 16 (one MFMA k-step), double-buffered: A and B
// piece rows at a 48-byte stride (conflict-free ds_read_b128), 72 KB of LDS
// -> 2 workgroups per CU. Tile order as in wino_gemm_kernel (XCD groups).
struct WinoBf6 {
    static constexpr int WM = 128, WN = 128, CK = 16, SR = 48;  // SR: bytes per piece row
    static constexpr int PIECE = 128 * SR;                       // one piece of A or B
    static constexpr int BUF = 6 * PIECE;                        // A h/m/l + B h/m/l
    static constexpr size_t BYTES = 2 * BUF;
};

template <int K>
__global__ __launch_bounds__(256) void wino_gemm_bf6_kernel(const float* __restrict__ V,
                                                            const uint16_t* __restrict__ Uh,
                                                            const uint16_t* __restrict__ Um,
                                                            const uint16_t* __restrict__ Ul, float* __restrict__ M,
                                                            int rows, int cout, int stride) {
    using T = WinoBf6;
    constexpr int CK = T::CK, SR = T::SR, PIECE = T::PIECE, BUF = T::BUF, NK = K / CK;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int CT = cout / T::WN, RT = rows / T::WM;
    const int nwg = WN_XI * RT * CT;
    const int idx0 = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx0 / (CT * RT);
    const int n_base = (idx0 % CT) * T::WN;
    const int r_base = ((idx0 / CT) % RT) * T::WM;
    const float* Va = V + ((size_t)xi * stride + r_base) * K;
    const size_t ub = ((size_t)xi * cout + n_base) * K;

    f32x4 ra[2];
    u32x4 rb[3];
    auto loadA = [&](int kt) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int i = tid + q * 256;  // 512 float4: 128 rows x 4
            ra[q] = *(const f32x4*)(Va + (size_t)(i >> 2) * K + kt * CK + (i & 3) * 4);
        }
    };
    auto storeA = [&](unsigned char* buf) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int i = tid + q * 256;
            const int off = (i >> 2) * SR + (i & 3) * 8;
            unsigned h[4], m[4], l[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) split3(ra[q][e], h[e], m[e], l[e]);
            *(u32x2*)(buf + off) = u32x2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
            *(u32x2*)(buf + PIECE + off) = u32x2{m[0] | (m[1] << 16), m[2] | (m[3] << 16)};
            *(u32x2*)(buf + 2 * PIECE + off) = u32x2{l[0] | (l[1] << 16), l[2] | (l[3] << 16)};
        }
    };
    auto loadB = [&](int kt) {  // 128 channels x 16 k x 3 pieces: one 16-byte chunk per thread per piece
        const size_t o = ub + (size_t)(tid >> 1) * K + kt * CK + (tid & 1) * 8;
        rb[0] = *(const u32x4*)(Uh + o);
        rb[1] = *(const u32x4*)(Um + o);
        rb[2] = *(const u32x4*)(Ul + o);
    };
    auto storeB = [&](unsigned char* buf) {
        const int off = 3 * PIECE + (tid >> 1) * SR + (tid & 1) * 16;
#pragma unroll
        for (int p = 0; p < 3; ++p) *(u32x4*)(buf + off + p * PIECE) = rb[p];
    };

    const int h = lane >> 5, li = lane & 31;
    int aoff[2], boff[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        aoff[t] = (wm * 64 + t * 32 + li) * SR + 16 * h;
        boff[t] = 3 * PIECE + (wn * 64 + t * 32 + li) * SR + 16 * h;
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    loadA(0);
    loadB(0);
    for (int kt = 0; kt < NK; ++kt) {
        unsigned char* buf = lds + (kt & 1) * BUF;
        storeA(buf);
        storeB(buf);
        if (kt + 1 < NK) {
            loadA(kt + 1);
            loadB(kt + 1);
        }
        __syncthreads();
        bf16x8 a[3][2], b[3][2];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                a[p][t] = *(const bf16x8*)(buf + aoff[t] + p * PIECE);
                b[p][t] = *(const bf16x8*)(buf + boff[t] + p * PIECE);
            }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {  // small terms first
                f32x16 c = acc[mt][nt];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mt], b[2][nt], c, 0, 0, 0);  // h*l
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][mt], b[0][nt], c, 0, 0, 0);  // l*h
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mt], b[1][nt], c, 0, 0, 0);  // m*m
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mt], b[1][nt], c, 0, 0, 0);  // h*m
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mt], b[0][nt], c, 0, 0, 0);  // m*h
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mt], b[0][nt], c, 0, 0, 0);  // h*h
                acc[mt][nt] = c;
            }
    }

    float* Mo = M + ((size_t)xi * stride + r_base + wm * 64) * cout + n_base + wn * 64 + li;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                Mo[(size_t)row * cout + nt * 32] = acc[mt][nt][r];
            }
}

}  // namespace kv
