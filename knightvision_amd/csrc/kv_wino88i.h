// F(8x8) Winograd GEMMs on the int8 matrix cores with exact integer
// accumulation (KV_PATH_WINO88_I8): the fp64 Winograd domain of kv_wino88d.h
// (U, V, M and both transforms in fp64) with the GEMM's products taken from
// int8 digits instead of v_mfma_f64.
//
// Every row of V (point xi, board) and of U (xi, output channel) -- K input
// channels -- is scaled by a power of two 2^-e to |a| < 255/256 (e from the
// row's largest magnitude, i8_row_exponent) and split into 5 signed int8 digits,
//     a * 2^-e = sum_i d_i * 2^(-7(i+1)) + rest,  |d_0| <= 127, |d_i| <= 64,
//     |rest| <= 2^-36,
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
// max |dlogit| 3.0e-6 against the fp64 path's 2.9e-6, profiles/r04_ozaki_emulation.log).
//
// Layouts: digit planes [slab xi][K / 32][digit 5][row][32] int8 (plane (xi, kc,
// d): digit d of channels 32 kc .. 32 kc + 31 of every row), exponents
// [xi][row] int32.
#pragma once
#include <hip/hip_runtime.h>

#include "kv_common.h"
#include "kv_wino88d.h"  // f64x2

namespace kv {

constexpr int kI8Digits = 5;    // digits per value in the fp64 domain (KV_PATH_WINO88_I8); the GEMM keeps
                                // the digit pairs i + j < digits
constexpr int kI8DigitsF32 = 4; // in the fp32 domain (KV_PATH_WINO88_I8F32): 28 bits, an fp32 value exactly
                                // when it is within 2^-4 of its row's max

typedef int i8x16_t __attribute__((ext_vector_type(4)));   // 16 int8 in 4 dwords (MFMA A / B)
typedef int i32x16_t __attribute__((ext_vector_type(16)));  // 32x32 int32 accumulator block

// Row exponent from the high word m of the row's largest |value| (biased exponent E in bits 20-30):
// 2^(e-1) <= max < 2^e, e = E - 1022, plus one when the max's top 7 fraction bits are all ones (max >=
// 255/256 * 2^e): then every t = a 2^-e < 255/256, so the first digit rint(128 t) <= 127 and every later
// remainder is within 1/2 -- no digit needs a clamp (35 bits kept on all but ~0.8 % of rows, 34 on
// those). An all-zero row gets e = 0 (digits 0).
__device__ inline int i8_row_exponent(unsigned m) {
    if (!m) return 0;
    return (int)(m >> 20) - 1022 + ((m & 0xFE000u) == 0xFE000u ? 1 : 0);
}

// fp32 form: m = the bits of the row's largest |float| (exponent in bits 23-30, top 7 fraction bits 16-22)
__device__ inline int i8_row_exponent_f32(unsigned m) {
    if (!m) return 0;
    return (int)(m >> 23) - 126 + ((m & 0x7F0000u) == 0x7F0000u ? 1 : 0);
}

// D digits of v under exponent e: t = 128 v 2^-e, d = rint(t), t = 128 (t - d), each step exact (in fp32
// too: t never has more significant bits than v)
template <int D, class T>
__device__ inline void i8_digits(T v, int e, int (&d)[D]) {
    T t = ldexp(v, 7 - e);
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const T q = rint(t);
        d[i] = (int)q;
        t = (t - q) * (T)128;
    }
}

// The digits and exponent of `nslab` slabs of n rows of K fp64 values: row r of
// slab x is src[(x * slab_rows + r) * K ...]; digit d of its channels
// [32 kc, 32 kc + 32) goes to plane (x, kc, d) of dst -- 32 bytes at
// (((x * K/32 + kc) * 5 + d) * slab_rows + r) * 32 -- and the exponent to
// ex[x * slab_rows + r]. One wave per row; lane l holds channels
// [l * K/64, (l + 1) * K/64). RL (row lines, 4 digits only): digit d of the
// 32 channels goes to (((x * K/32 + kc) * slab_rows + r) * 4 + d) * 32 instead
// -- the 4 digits of one row's chunk are one 128-byte line.
template <int K, class T, int D, bool RL = false>
__global__ __launch_bounds__(256) void wino88i_slice_kernel(const T* __restrict__ src, int n, int slab_rows,
                                                            int nslab, int8_t* __restrict__ dst,
                                                            int* __restrict__ ex) {
    static_assert(K == 256 || K == 512, "rows of 256 or 512 channels");
    static_assert(!RL || D == 4, "row lines hold 4 digits");
    constexpr int CPL = K / 64;  // 4 or 8 channels per lane
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= n * nslab) return;  // whole waves
    const int x = gw / n, r = gw % n;
    const size_t row = (size_t)x * slab_rows + r;
    const T* s = src + row * K + lane * CPL;
    T v[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) v[i] = s[i];
    // the (high) words of |v| order like |v|: their max carries the row's largest exponent
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        unsigned hw;
        if constexpr (sizeof(T) == 8)
            hw = (unsigned)(__double_as_longlong(v[i]) >> 32) & 0x7fffffffu;
        else
            hw = __float_as_uint(v[i]) & 0x7fffffffu;
        m = hw > m ? hw : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned t = (unsigned)__shfl_xor((int)m, o, 64);
        m = t > m ? t : m;
    }
    const int e = sizeof(T) == 8 ? i8_row_exponent(m) : i8_row_exponent_f32(m);
    if (lane == 0) ex[row] = e;
    unsigned long long pk[D] = {};
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        int dg[D];
        i8_digits<D>(v[i], e, dg);
#pragma unroll
        for (int d = 0; d < D; ++d) pk[d] |= (unsigned long long)(unsigned char)(signed char)dg[d] << (8 * i);
    }
    const int c = lane * CPL, kc = c / 32;
    int8_t* o = RL ? dst + (((size_t)x * (K / 32) + kc) * slab_rows + r) * (D * 32) + (c % 32)
                   : dst + ((((size_t)x * (K / 32) + kc) * D) * slab_rows + r) * 32 + (c % 32);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        int8_t* od = o + (size_t)d * (RL ? 32 : slab_rows * 32);
        if constexpr (CPL == 8)
            *(unsigned long long*)od = pk[d];
        else
            *(unsigned*)od = (unsigned)pk[d];
    }
}

// The GEMM: a workgroup computes 128 rows x 128 output channels of one point
// with 8 waves of 32 x 64 (1 x 2 accumulator blocks per digit level). K
// streams in 32-k stages; a stage is the 5 digit planes of the tile's rows
// (5 x 128 x 32 B of V, the same of U), copied global -> LDS by
// global_load_lds (1 KiB = 32 rows per wave-instruction, 5 per wave per
// stage) into a ring of 3 LDS buffers: the copies of stage kt + 2 run during
// stage kt's MFMAs, retired by a counted s_waitcnt vmcnt and a raw barrier.
// The LDS image is linear; the two 16-byte halves of a row are swapped when
// bit 3 of the row is set (on the global source address), so each ds_read_b128
// lane group reads 16 distinct 4-bank groups.
template <int D>
struct Wino88iTile {
    static constexpr int WR = 4, WC = 2, MT = 1, NT = 2;
    static constexpr int THREADS = WR * WC * 64;
    static constexpr int WM = WR * MT * 32, WN = WC * NT * 32;  // 128 x 128
    static constexpr int PLANE = 128 * 32;                      // bytes of one digit plane of a tile
    static constexpr int STAGE = 2 * D * PLANE;                 // A planes then B planes: 8 D KiB
    static constexpr int NBUF = 3;
    static constexpr size_t BYTES = (size_t)NBUF * STAGE;
    static constexpr int GL = STAGE / 1024 / (THREADS / 64);    // global_load_lds per wave and stage (= D)
};

__device__ inline int i8_lds_half(int row, int h) { return 16 * (h ^ ((row >> 3) & 1)); }

// RL layout in LDS: row r of an operand is its 128-byte line (16-byte chunk c = 2 d + half of digit d),
// chunk c at position c ^ ((r >> 1) & 7): a ds_read_b128 lane group (rows {0-3, 12-15, 20-27} or {4-11,
// 16-19, 28-31} of a 32-row block, one chunk) hits 16 distinct 16-byte bank groups -- even rows in the
// first 128 bytes of the 256-byte bank window, odd rows in the second, 8 distinct positions each. (A
// chunk-major image with one base + 256 d per digit needs lanes 128 bytes apart in the copy: the GEMM
// ran 551 us against 523, profiles/r04_i8f32_rowlines_ab.log.)
__device__ inline int i8_rl_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ ((row >> 1) & 7)); }

// M[xi] (fp64 [xi][stride rows][cout]) = V[xi] x U[xi]^T from the digits (see the header comment).
// V8: planes [xi][K/32][5][stride][32], U8: [xi][K/32][5][cout][32]. XCD-aware tile order as kv_wino.h's
// wino_gemm_kernel. RL (4 digits): row lines [xi][K/32][stride][4][32] and [xi][K/32][cout][4][32] -- a
// stage of a tile is one contiguous 16 KiB block per operand, and one workgroup of the fused output
// kernel (one board) writes whole lines.
template <int K, int S, bool SPREAD = true, class OutT = double, bool RL = false>
__global__ __launch_bounds__(512) void wino88i_gemm_kernel(const int8_t* __restrict__ V8,
                                                            const int* __restrict__ ev,
                                                            const int8_t* __restrict__ U8,
                                                            const int* __restrict__ eu,
                                                            OutT* __restrict__ M, int rows, int cout,
                                                            int stride) {
    constexpr int kI8Digits = S;  // digit planes per chunk = the levels kept
    using T = Wino88iTile<S>;
    constexpr int MT = T::MT, NT = T::NT, WM = T::WM, WN = T::WN, GL = T::GL;
    constexpr int NK = K / 32;
    static_assert(GL == S && GL * (T::THREADS / 64) * 1024 == T::STAGE, "stage split");
    static_assert(!RL || S == 4, "row lines hold 4 digits");

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8[];
    char* const L0 = (char*)lds_i8;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / T::WC, wn = wave % T::WC;
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x;  // a multiple of 8
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx / (CT * RT);
    const int n_base = (idx % CT) * WN;
    const int r_base = ((idx / CT) % RT) * WM;

    // the GL pieces per stage of this wave: piece q = wave * GL + g covers operand q / 4S (V, U: the
    // same for all of a wave's pieces), digit (q % 4S) / 4, rows 32 (q % 4) .. +31 of the tile; lane l
    // fills LDS row 32 (q % 4) + l / 2, half l & 1 (bit 3 of that row is bit 4 of l). Everything but the
    // lane's offset is wave-uniform.
    const int op = (wave * GL) / (4 * S);
    const size_t rstride = op ? (size_t)cout : (size_t)stride;
    const size_t tbase = RL ? (op ? (size_t)n_base : (size_t)r_base) * 4 : (op ? n_base : r_base);  // RL: 128 B rows
    const int8_t* gbase = op ? U8 + (((size_t)xi * NK) * kI8Digits * cout + tbase) * 32
                             : V8 + (((size_t)xi * NK) * kI8Digits * stride + tbase) * 32;
    const size_t sstep = (size_t)kI8Digits * rstride * 32;  // the next 32-k chunk
    const int lane_off = (lane >> 1) * 32 + 16 * ((lane & 1) ^ ((lane >> 4) & 1));
    // RL: piece q covers operand q / 16, rows 8 (q % 16) .. +7 (1 KiB contiguous in both places); lane l
    // fills position l & 7 of LDS row 8 (q % 16) + l / 8 from source chunk (l & 7) ^ (row >> 1 & 7)
    const int rl_off0 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4));
    const int rl_off1 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4) ^ 4);
    auto issue1 = [&](int g, int kt, int buf) {  // this wave's piece g of stage kt
        const int q = wave * GL + g, d = (q % (4 * S)) / 4, rg = q % 4;
        if constexpr (RL) {
            const int rg8 = q % 16;
            __builtin_amdgcn_global_load_lds(
                (const void*)(gbase + kt * sstep + (size_t)rg8 * 1024 + ((rg8 & 1) ? rl_off1 : rl_off0)),
                (__attribute__((address_space(3))) void*)(L0 + buf * T::STAGE + op * kI8Digits * T::PLANE +
                                                          rg8 * 1024),
                16, 0, 0);
            return;
        }
        __builtin_amdgcn_global_load_lds(
            (const void*)(gbase + kt * sstep + ((size_t)d * rstride + rg * 32) * 32 + lane_off),
            (__attribute__((address_space(3))) void*)(L0 + buf * T::STAGE + op * kI8Digits * T::PLANE +
                                                      d * T::PLANE + rg * 1024),
            16, 0, 0);
    };
    auto issue = [&](int kt, int buf) {
#pragma unroll
        for (int g = 0; g < GL; ++g) issue1(g, kt, buf);
    };

    // fragments: A digit d of row r: plane d, row wm * 32 + (lane & 31), half lane >> 5 (swapped as stored)
    const int lr = lane & 31, lh = lane >> 5;
    const int arow = wm * 32 + lr;
    const int aoff = arow * 32 + i8_lds_half(arow, lh);
    int boff[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int bcol = wn * NT * 32 + nt * 32 + lr;
        boff[nt] = kI8Digits * T::PLANE + bcol * 32 + i8_lds_half(bcol, lh);
    }
    // RL: the fragment of digit i is chunk 2 i + half of the row's line
    int aoffr[S], boffr[NT][S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        aoffr[i] = i8_rl_off(arow, 2 * i + lh);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
            boffr[nt][i] = kI8Digits * T::PLANE + i8_rl_off(wn * NT * 32 + nt * 32 + lr, 2 * i + lh);
    }

    i32x16_t acc[S][MT][NT];
#pragma unroll
    for (int l = 0; l < S; ++l)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[l][0][nt] = i32x16_t{};

    issue(0, 0);
    issue(1, 1);
    for (int kt = 0; kt < NK; ++kt) {
        // this wave's copies of stage kt have landed (stage kt + 1's may still be in flight), then
        // every wave's have, and every wave is done reading the buffer stage kt + 2 goes into
        if (kt + 1 < NK)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* buf = L0 + (kt % 3) * T::STAGE;
        // the A digits (one 32-row block) stay live; B digit j (two 32-column blocks) dies after its
        // S - j products, pairs i + j < S. Stage kt + 2's copies go out one per B digit, between the
        // MFMA groups (issued back to back after the barrier they delayed every wave's first MFMA:
        // profiles/r04_i8_glds_spread_ab.log)
        i8x16_t a[S];
#pragma unroll
        for (int i = 0; i < S; ++i) a[i] = *(const i8x16_t*)(buf + (RL ? aoffr[i] : aoff + i * T::PLANE));
#pragma unroll
        for (int j = 0; j < S; ++j) {
            i8x16_t b[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                b[nt] = *(const i8x16_t*)(buf + (RL ? boffr[nt][j] : boff[nt] + j * T::PLANE));
#pragma unroll
            for (int i = 0; i + j < S; ++i)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[i + j][0][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[nt], acc[i + j][0][nt], 0, 0, 0);
            if (SPREAD && kt + 2 < NK) {
#pragma unroll
                for (int g = j * GL / S; g < (j + 1) * GL / S; ++g) issue1(g, kt + 2, (kt + 2) % 3);
            }
        }
        if (!SPREAD && kt + 2 < NK) issue(kt + 2, (kt + 2) % 3);
    }

    // D: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) inside the 32 x 32 block
    const int* evx = ev + (size_t)xi * stride + r_base + wm * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = n_base + wn * NT * 32 + nt * 32 + lr;
        const int ec = eu[(size_t)xi * cout + col] - 14;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            double m = (double)acc[S - 1][0][nt][r];
#pragma unroll
            for (int l = S - 2; l >= 0; --l) m = __builtin_fma(m, 0.0078125, (double)acc[l][0][nt][r]);  // exact
            M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col] = (OutT)ldexp(m, evx[row] + ec);
        }
    }
}

// The next conv's digits come from two kernels, each at the occupancy of the
// fp64 out kernel (one workgroup = 128 channels of one board): the exponent of
// a V row needs the largest magnitude over all 512 channels, i.e. over 4
// workgroups. (One 1,024-thread workgroup per board computing both in one
// kernel was measured and dropped: 540-665 us per layer at 2,048 boards, its
// two passes serialised at one workgroup per CU, against 300-420 us for the
// fp64 out kernel; profiles/r04_i8_fused_out.log.)
//   wino88i_outmax_kernel: output transform + BN (+ residual) + ReLU -> fp32 Y
//     (as wino88d_out_half_kernel), the next V64 rows computed and reduced to
//     each point's max |V| over the workgroup's channels, folded into
//     evmax[xi][board] (high words of the doubles, atomicMax; zeroed before);
//   wino88i_in_kernel: the input transform of Y again (the same fma chains on
//     the same fp32 inputs: the same bits) and its 5 digits under the row
//     exponents -- what wino88i_slice_kernel makes of that V64.

// max over the 32 lanes of this half of v[0..9] (16 shuffles): lanes with (lane & 16) == 0 and
// (lane & 15) < 10 return the max of index lane & 15
__device__ inline unsigned i8_half_max10(const double (&o)[10], int lane) {
    unsigned v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = j < 10 ? (unsigned)(__double_as_longlong(o[j]) >> 32) & 0x7fffffffu : 0u;
#pragma unroll
    for (int st = 0; st < 4; ++st) {  // halving over offsets 8, 4, 2, 1: lane keeps index lane & 15
        const int off = 8 >> st;
        const bool up = (lane & off) != 0;
#pragma unroll
        for (int i = 0; i < off; ++i) {
            const unsigned mine = up ? v[off + i] : v[i];
            const unsigned other = (unsigned)__shfl_xor((int)(up ? v[i] : v[off + i]), off, 64);
            v[i] = mine > other ? mine : other;
        }
    }
    const unsigned o16 = (unsigned)__shfl_xor((int)v[0], 16, 64);
    return v[0] > o16 ? v[0] : o16;
}

template <bool RESID>
__global__ __launch_bounds__(256) void wino88i_outmax_kernel(const double* __restrict__ M, int rows,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, const float* resid,
                                                             float* Y, unsigned* __restrict__ evmax) {
    __shared__ unsigned red[4][2][5][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int c = blockIdx.x * 128 + w * 32 + (lane & 31), b = blockIdx.y;
    double t2[10][4];
    {
        float x2[4][8];
        wino88d_out_plane<RESID, true>(M, rows, b, c, h, (double)scale[c], (double)shift[c], resid, Y, x2);
        wino88d_input_cols(x2, h, t2);
    }
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        double o[10];
        wino88d_input_row(t2, h, aa, o);
        const unsigned m = i8_half_max10(o, lane);
        if ((lane & 16) == 0 && (lane & 15) < 10) red[w][h][aa][lane & 15] = m;
    }
    __syncthreads();
    if (threadIdx.x < 100) {
        const int xi = threadIdx.x, a = xi / 10, bb = xi % 10, hh = a / 5, aa = a % 5;
        unsigned m = 0;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) m = red[ww][hh][aa][bb] > m ? red[ww][hh][aa][bb] : m;
        if (m) atomicMax(evmax + (size_t)xi * rows + b, m);
    }
}

// grid (512 / 32, boards / 4) x 256: wave w = board 4 blockIdx.y + w, lanes = the 32 channels of chunk
// kc = blockIdx.x (plane split over lanes l, l ^ 32), so the 4 waves write 4 consecutive rows -- one
// whole 128-byte line -- of each digit plane (xi, kc, d): 32-byte pieces from different workgroups made
// the plane writes 2.8x slower (421 us per layer at 2,048 boards, profiles/r04_i8_fused_out.log).
// X the fp32 activation [board][64][512]; writes the row exponents ex[xi][board] (from evmax) too.
__global__ __launch_bounds__(256) void wino88i_in_kernel(const float* __restrict__ X, int rows,
                                                         const unsigned* __restrict__ evmax,
                                                         int8_t* __restrict__ V8n, int* __restrict__ ex) {
    constexpr int C = 512;
    __shared__ int exs[4][100];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int kc = blockIdx.x, c = kc * 32 + (lane & 31), b = blockIdx.y * 4 + w;
    for (int i = threadIdx.x; i < 400; i += 256) {
        const int bw = i / 100, xi = i % 100, bb = blockIdx.y * 4 + bw;
        const int e = i8_row_exponent(evmax[(size_t)xi * rows + bb]);
        exs[bw][xi] = e;
        if (kc == 0) ex[(size_t)xi * rows + bb] = e;
    }
    float x2[4][8];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < 8; ++j) x2[ii][j] = X[((size_t)b * 64 + (4 * h + ii) * 8 + j) * C + c];
    double t2[10][4];
    wino88d_input_cols(x2, h, t2);
    __syncthreads();
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        double o[10];
        wino88d_input_row(t2, h, aa, o);
        const int a = 5 * h + aa;
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) {
            const int xi = a * 10 + bb;
            int dg[kI8Digits];
            i8_digits<kI8Digits>(o[bb], exs[w][xi], dg);
            int8_t* dst = V8n + ((((size_t)xi * (C / 32) + kc) * kI8Digits) * rows + b) * 32 + (lane & 31);
#pragma unroll
            for (int d = 0; d < kI8Digits; ++d) dst[(size_t)d * rows * 32] = (int8_t)dg[d];
        }
    }
}

// ---- the fp32 Winograd domain with int8-digit GEMMs (KV_PATH_WINO88_I8F32) ----
// The fp32 F(8x8) tower's arithmetic (kv_wino88.h: fp32 transforms, V, M and activations; U as
// 4 digits of the fp64 U) with each GEMM taken from 4 int8 digits per value: the product of the
// 28-bit truncated rows is exact (int32 levels, fp64 combine) and rounded to fp32 once, where the
// fp32 MFMA GEMM rounds after every product. 10 int8 MFMAs per point product against one fp32 one at
// 1/32 the rate.

// The fp32 tower's own fused output / input transform kernels (kv_wino88.h) write the next fp32 V, and
// wino88i_slice_kernel<K, float, 4, true> turns it into row-line digits (one wave per row: whole lines).
// Dropped forms (profiles/r04_i8f32_outmax_form.log, profiles/r04_i8f32_fused_out.log): an output kernel
// computing only the row maxima plus a second input-transform pass writing the digits (294-356 + 220 us
// per layer at 2,048 boards), and one 512-thread workgroup per board keeping V in registers and reducing
// the row maxima in the workgroup (436-511 us: at 246 VGPRs one workgroup per CU, its load, transform
// and store phases serialised), against 142-238 + 165 us for the out kernel + slice.

}  // namespace kv
