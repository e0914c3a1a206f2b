// Winograd building blocks shared by the fp32 towers (kv_wino48.h F(4x8),
// kv_wino88.h F(8x8)): the 1-D F(4,3) transforms with the Lavin-Gray points
// (0, +-1, +-2, inf) that F(4x8) applies along the board's rows, the
// point-batched GEMM M[xi] = V[xi] x U[xi]^T on the f32 MFMA, and the f16x3
// (KV_PREC_F16X3) form of that GEMM.
//
// Layouts (fp32): V and M are [xi][rows][C] (C contiguous), U is
// [xi][Cout][Cin]. (The 2-D F(4x4) tower, its bf16x6 GEMM and the bf16x3
// direct conv were retired in round 4: no configuration used them.)
#pragma once
#include <hip/hip_runtime.h>

#include "kv_common.h"

namespace kv {

// B^T (6x6) applied to one 6-vector. The only inexact product is the -5
// term: it is an explicit fma so that its rounding does not depend on how the
// compiler contracts a given call site (stem_kernel's inlined zero padding vs
// wino48_in_kernel's loads) -- every caller gives the same bits.
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

// KV_PREC_F16X3 operand scaling. The GEMM splits every V element of board b
// into fp16 pieces after scaling by 2^s_b, s_b = 14 - exponent(max_b |V|), so
// the board's largest element lands in [2^14, 2^15): no fp16 overflow and the
// low piece stays normal for everything within 2^-17 of the maximum. The scale
// depends on the board alone (batch invariance) and is a power of two (exact).
// vmax holds max_b |V| as float bits (non-negative floats order as unsigned).
__device__ inline int h3_exp(unsigned mx) {
    if (mx == 0u) return 0;
    const int e = (int)((mx >> 23) & 0xFFu) - 127;
    const int s = 14 - e;
    return s < -100 ? -100 : (s > 100 ? 100 : s);
}

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

// ------------------------------------------------------------ f16x3 --
// KV_PREC_F16X3: M[xi] = V[xi] x U[xi]^T with both operands split into two
// fp16 pieces, x*2^s = h + l (h = fp16(x*2^s), l = fp16(x*2^s - h): 22
// significant bits), and the three products of weight >= 2^-22 -- h*l, l*h,
// h*h -- on v_mfma_f32_32x32x16_f16 with fp32 accumulation. Host emulation of
// the whole tower: 2x the error of rounding the operands to fp32, well under
// the direct fp32 conv's accumulation error. U is split once at load time
// with a per-layer scale 2^ut; V is split while it is staged into LDS with the
// per-board scale of h3_exp; the consumer (wino48_out_kernel) multiplies M by
// 2^-(s_b + ut). 3 MFMAs of 32 cycles per 32x32x16 block instead of the fp32
// kernel's 8 of 64: the f16 rate is 5.3x the fp32 MFMA rate per product.
//
// Workgroup: 64 rows x 128 channels of one xi (the fp32 kernel's 64x128 tile:
// exactly 3 rounds at 1,024 rows with LDS padded for 3 workgroups per CU),
// 4 waves of 32x64 (1x2 MFMA tiles), k-tiles of 16, double-buffered; piece
// rows at a 48-byte stride (conflict-free ds_read_b128).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Workgroup tile: WM = 64 * TM rows x 128 channels of one xi, 4 waves in a
// 2 x 2 grid of (32 TM) x 64 (TM x 2 MFMA tiles each). LDS stage (two
// stages): A h / l [WM rows][64 B], B h / l [128 rows][64 B] = 32 k. The four
// 16-byte chunks of a row are XOR-swizzled by (row / 4) % 4, which spreads
// every ds_read_b128 lane group (16 lanes = 16 rows) over all 64 banks with no
// padding -- so the B image can be filled by lane-linear global_load_lds
// straight from a Uf laid out as that image.
template <int TM>
struct WinoH3 {
    static constexpr int WM = 64 * TM, WN = 128, CK = 32, SR = 64;
    static constexpr int PA = WM * SR, PB = WN * SR;  // one piece of A / B
    static constexpr int STAGE = 2 * PA + 2 * PB;     // 24 / 32 KB
    static constexpr size_t BYTES = 2 * STAGE;
};
__host__ __device__ inline int h3_off(int row, int c) { return row * 64 + ((c ^ ((row >> 2) & 3)) << 4); }

// Uf (KV_PREC_F16X3): per (xi, 128-channel block, 32-k tile, piece) one 8 KB
// block holding the B image of that tile.
__host__ __device__ inline size_t h3_uidx(int xi, int co, int ci, int cout, int K) {
    const size_t blk = ((size_t)xi * (cout >> 7) + (co >> 7)) * (K >> 5) + (ci >> 5);
    return blk * 4096 + (h3_off(co & 127, (ci & 31) >> 3) >> 1) + (ci & 7);
}

// One barrier per k-tile. Iteration kt: B(kt+1) global_load_lds into the
// other stage; MFMAs on stage kt; A(kt+1) (in registers since iteration kt-2)
// split and written to the other stage; A(kt+3) loads issued; barrier. A
// (V, streamed from HBM / the Infinity Cache) has two k-tiles of latency
// cover, B (U, L2-resident) one compute phase.
// XI transform points; RSH: log2 of the V rows per board (2 for F(4x4), 1 for F(4x8))
template <int K, int TM, int XI, int RSH>
__global__ __launch_bounds__(256) void wino_gemm_h3_kernel(const float* __restrict__ V, const uint16_t* __restrict__ Uh,
                                                           const uint16_t* __restrict__ Ul,
                                                           const unsigned* __restrict__ vmax, float* __restrict__ M,
                                                           int rows, int cout, int stride) {
    using T = WinoH3<TM>;
    constexpr int CK = T::CK, PA = T::PA, PB = T::PB, STAGE = T::STAGE, NK = K / CK;
    static_assert(NK % 2 == 0 && NK >= 4, "k-tiles");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int CT = cout / T::WN, RT = rows / T::WM;
    const int nwg = XI * RT * CT;
    const int idx0 = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx0 / (CT * RT);
    const int nb_ = idx0 % CT;
    const int r_base = ((idx0 / CT) % RT) * T::WM;
    const float* Va = V + ((size_t)xi * stride + r_base) * K;
    const size_t ub = ((size_t)xi * CT + nb_) * NK * 4096;  // this workgroup's Uf blocks (halves)

    // A: thread = rows tid/4 + 64 i, 8 consecutive k each; the rows' board scales are fixed for the K loop
    const int ar = tid >> 2, ac = tid & 3;
    float asc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) asc[i] = ldexpf(1.f, h3_exp(vmax[(r_base + ar + 64 * i) >> RSH]));
    const float* asrc = Va + (size_t)ar * K + ac * 8;
    f32x4 ra[2][TM][2];
    auto loadA = [&](int kt, f32x4 (&a)[TM][2]) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            a[i][0] = *(const f32x4*)(asrc + (size_t)64 * i * K + kt * CK);
            a[i][1] = *(const f32x4*)(asrc + (size_t)64 * i * K + kt * CK + 4);
        }
    };
    auto writeA = [&](unsigned char* st, const f32x4 (&a)[TM][2]) {
        // split in pairs: v_pk_mul_f32, v_cvt_pk_f16_f32 (RNE), two v_cvt_f32_f16, v_pk_fma, v_cvt_pk_f16_f32
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            h16x2 hp[4], lp[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const f32x2 x = f32x2{a[i][e >> 1][(e & 1) * 2], a[i][e >> 1][(e & 1) * 2 + 1]} * asc[i];
                hp[e] = __builtin_convertvector(x, h16x2);
                lp[e] = __builtin_convertvector(x - __builtin_convertvector(hp[e], f32x2), h16x2);
            }
            const int w = h3_off(ar + 64 * i, ac);
            *(u32x4*)(st + w) = __builtin_bit_cast(u32x4, hp);
            *(u32x4*)(st + PA + w) = __builtin_bit_cast(u32x4, lp);
        }
    };
    // B: 2 x 8 KB per stage, lane-linear: chunk q*256 + tid of each piece image
    auto loadB = [&](int kt, unsigned char* st) {
        const size_t o = ub + (size_t)kt * 4096;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int ch = q * 256 + wave * 64;  // this wave's first 16-byte chunk
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(Uh + o + (q * 256 + tid) * 8),
                                             (__attribute__((address_space(3))) void*)(st + 2 * PA + ch * 16), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(Ul + o + (q * 256 + tid) * 8),
                                             (__attribute__((address_space(3))) void*)(st + 2 * PA + PB + ch * 16), 16, 0,
                                             0);
        }
    };

    const int h = lane >> 5, li = lane & 31;
    f32x16 acc[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto compute = [&](const unsigned char* st) {
#pragma unroll
        for (int kk = 0; kk < CK / 16; ++kk) {
            f16x8 ah[TM], al[TM], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int ao = h3_off(wm * 32 * TM + i * 32 + li, kk * 2 + h);
                ah[i] = *(const f16x8*)(st + ao);
                al[i] = *(const f16x8*)(st + PA + ao);
            }
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int bo = 2 * PA + h3_off(wn * 64 + nt * 32 + li, kk * 2 + h);
                bh[nt] = *(const f16x8*)(st + bo);
                bl[nt] = *(const f16x8*)(st + bo + PB);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {  // small terms first
                    f32x16 c = acc[i][nt];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[nt], c, 0, 0, 0);  // h*l
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[nt], c, 0, 0, 0);  // l*h
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[nt], c, 0, 0, 0);  // h*h
                    acc[i][nt] = c;
                }
        }
    };

    // prologue: stage 0 = A(0) + B(0); A(1), A(2) in flight
    loadA(0, ra[0]);
    loadB(0, lds);
    writeA(lds, ra[0]);
    loadA(1, ra[1]);
    loadA(2, ra[0]);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt0 = 0; kt0 < NK; kt0 += 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // j = kt & 1: this stage; A(kt + 1) is in register slot 1 - j
            const int kt = kt0 + j;
            unsigned char* cur = lds + j * STAGE;
            unsigned char* nxt = lds + (1 - j) * STAGE;
            if (kt + 1 < NK) loadB(kt + 1, nxt);
            compute(cur);
            if (kt + 1 < NK) {
                writeA(nxt, ra[1 - j]);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // B(kt+1) landed (and A(kt+2))
                if (kt + 3 < NK) loadA(kt + 3, ra[1 - j]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
    }

#pragma unroll
    for (int i = 0; i < TM; ++i) {
        float* Mo = M + ((size_t)xi * stride + r_base + wm * 32 * TM + i * 32) * cout + nb_ * 128 + wn * 64 + li;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                Mo[(size_t)row * cout + nt * 32] = acc[i][nt][r];
            }
    }
}

// max |x| over n floats into *out (as float bits); grid-stride, one atomic per wave
__global__ void absmax_kernel(const float* __restrict__ x, size_t n, unsigned* out) {
    float m = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(x[i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// U [nxi][cout][cin] (one layer) -> fp16 pieces of U * 2^ut in the Uf layout (h3_uidx)
__global__ void split_f16_kernel(const float* __restrict__ u, int cout, int cin, int ut, uint16_t* __restrict__ h,
                                 uint16_t* __restrict__ l, int nxi) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)nxi * cout * cin) return;
    const int ci = (int)(i % cin), co = (int)((i / cin) % cout), xi = (int)(i / ((size_t)cin * cout));
    const float a = ldexpf(u[i], ut);
    const _Float16 hh = (_Float16)a;
    const size_t o = h3_uidx(xi, co, ci, cout, cin);
    h[o] = __builtin_bit_cast(uint16_t, hh);
    l[o] = __builtin_bit_cast(uint16_t, (_Float16)(a - (float)hh));
}

}  // namespace kv
