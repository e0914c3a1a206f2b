// The point-batched GEMM of the fp32 F(8x8) tower (kv_wino88.h, KV_ALGO_WINOGRAD88): M[xi] = V[xi] x U[xi]^T on
// the f32 MFMA.
//
// Layouts (fp32): V and M are [xi][rows][C] (C contiguous), U is
// [xi][Cout][Cin]. (The 2-D F(4x4) tower, its bf16x6 GEMM and the bf16x3
// direct conv were retired in round 4; the F(4x8) tower and its f16x3 GEMM in round 6: no configuration used
// them.)
#pragma once
#include <hip/hip_runtime.h>

#include "kv_common.h"

namespace kv {

// The XI GEMMs M[xi] = V[xi] x U[xi]^T on v_mfma_f32_32x32x2_f32, over `rows`
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

template <int K, int WR, int WC, int MT, int NT, int CK, int XI>
__global__ __launch_bounds__(WR * WC * 64) void wino_gemm_kernel(const float* __restrict__ V,
                                                                   const float* __restrict__ U,
                                                                   float* __restrict__ M, int rows, int cout,
                                                                   int stride, int xi0 = 0) {
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
    // run on one XCD and re-read V / U from its L2 instead of HBM. A launch
    // covers the points [xi0, xi0 + gridDim.x / (RT * CT)) (F(8x8) splits its
    // 100 points over two tile shapes so that no round of tiles is left half full).
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x;  // a multiple of 8 (points x 4 column tiles x RT)
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = xi0 + idx / (CT * RT);
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
