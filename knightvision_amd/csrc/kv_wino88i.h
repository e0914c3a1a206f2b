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
// combined in fp64 exactly (at most 51 significant bits). What it computes:
// per-row 35-bit block fixed point (each value cut to the multiples of
// 2^(e-36) of its row's exponent), the 15 digit pairs i + j <= 4 of the 25
// (the 10 dropped pairs weigh < 2^-42 of the row maxima's product each), exact
// int32 levels, one exact fp64 combine. Nothing in the GEMM rounds, so M is
// independent of k order, tile shape and batch by construction. Its distance
// from the fp64 product of the unsplit rows is bounded per element by the
// truncation (|rest| <= 2^-36 per value) plus the dropped pairs:
// tests/test_wino_i8_gpu.py::test_i8_gemm_within_derived_bound_of_fp64_product.
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
#include "kv_wino88.h"   // w88_bt, wino88_out_plane
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

// Radix-256 form (KV_PATH_WINO88_I8R: 4 digits of 8 bits): e with max < 127/128 2^e (one more than the
// plain rule when the max's top 7 fraction bits are >= 126), so every N = rint(v 2^(31-e)) has |N| < 127/128
// 2^31 and its balanced base-256 digits d_0 (most significant) .. d_3, N = sum_i d_i 2^(8 (3 - i)), are all
// in [-128, 127] with |d_0| <= 127: v ~ 2^(e-7) sum_i d_i 2^(-8 i), 31-bit block fixed point.
__device__ inline int i8_row_exponent_r8(unsigned m) {
    if (!m) return 0;
    return (int)(m >> 20) - 1022 + ((m & 0xFE000u) >= 0xFC000u ? 1 : 0);
}

// fp32 form of the radix-256 rule (KV_PATH_WINO88_I8F32R3): m = the bits of the row's largest |float|; one more
// when its top 6 fraction bits are all ones (max >= 127/128 2^e)
__device__ inline int i8_row_exponent_f32r(unsigned m) {
    if (!m) return 0;
    return (int)(m >> 23) - 126 + ((m & 0x7E0000u) == 0x7E0000u ? 1 : 0);
}

// The 3 radix-256 digits of v under e (KV_PATH_WINO88_I8F32R3: the fp32 tower's 24-bit block fixed point), in
// the row lines' 4 digit slots: N = rint(v 2^(23-e)) by an fp64 magic-number add (ties to even; exact for
// |N| < 2^31 -- the fp32 magic add would round at |t| >= 2^22), |N| < 127/128 2^23 under the radix-256 rule, so
// the balanced digits d_0 (most significant) .. d_2, N = d_0 2^16 + d_1 2^8 + d_2, are the bytes of
// N + 0x808080 with their top bits flipped; packed byte d = d_d (slot 3 zero): v ~ 2^(e-7) sum_d d_d 2^(-8 d).
__device__ inline unsigned i8_digits_r3(double v, int e) {
#pragma clang fp contract(off)
    constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
    const unsigned n = (unsigned)__double_as_longlong(ldexp(v, 23 - e) + kMagic);
    return __builtin_amdgcn_perm(0u, (n + 0x808080u) ^ 0x808080u, 0x0c000102u);
}

// the 4 radix-256 digits of v under e, packed: byte k = d_(3-k) (two's complement). N by a magic-number add
// (rint, ties to even; the low word of t + 1.5 2^52 is N's two's complement for |t| < 2^31); then the balanced
// digits are the bytes of N + 0x80808080 (each d + 128 in [0, 255], no carry out) with their top bits flipped.
__device__ inline unsigned i8_digits_r8(double v, int e) {
#pragma clang fp contract(off)
    constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
    const unsigned n = (unsigned)__double_as_longlong(ldexp(v, 31 - e) + kMagic);
    return (n + 0x80808080u) ^ 0x80808080u;
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

// max over the 32 lanes of each half-wave of v, by DPP-modified max operations (no selects, no LDS-pipe
// shuffle): xor 1 and xor 2 within quads, the half-row and row mirrors (every lane then holds its 16-lane
// row's max), then row_bcast:15 into rows 1 and 3 -- lanes 16-31 end with the max of lanes 0-31, lanes
// 48-63 with the max of lanes 32-63.
__device__ inline unsigned i8_half_max_dpp(unsigned v) {
    // old = 0 (the identity of an unsigned max) so the compiler folds each DPP move into its max
    unsigned t = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);  // quad_perm 1,0,3,2
    v = v > t ? v : t;
    t = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true);  // quad_perm 2,3,0,1
    v = v > t ? v : t;
    t = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, true);  // row_half_mirror
    v = v > t ? v : t;
    t = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, true);  // row_mirror
    v = v > t ? v : t;
    t = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    return v > t ? v : t;
}

// i8_digits<D> of an fp64 v with each rint(t) as t + 1.5 * 2^52 (|t| <= 128: the add rounds to the integer,
// ties to even, as rint) -- q[i]'s low byte is digit i's two's complement; q - 1.5 * 2^52 is rint(t) exactly, so
// the remainders are i8_digits's: the same digits with full-rate fp64 adds instead of v_rndne_f64 +
// v_cvt_i32_f64
template <int D>
__device__ inline void i8_digits_magic(double v, int e, unsigned (&q)[D]) {
#pragma clang fp contract(off)
    constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
    double t = ldexp(v, 7 - e);
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const double qf = t + kMagic;
        q[i] = (unsigned)__double_as_longlong(qf);
        if (i + 1 < D) t = (t - (qf - kMagic)) * 128.0;
    }
}

// The 4 digits of an fp32 v under exponent e (i8_digits<4>) packed into one dword, digit d in byte d: each
// rint(t) as t + 1.5 * 2^23 (|t| <= 128: the add rounds to the integer, ties to even, as rintf) whose low byte
// is the digit's two's complement; q - 1.5 * 2^23 is rint(t) exactly, so t - rint(t) and the x128 are the
// same operations as i8_digits's -- the same digits, without the float -> int conversions.
__device__ inline unsigned i8_digits4_packed(float v, int e) {
#pragma clang fp contract(off)
    constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23
    float t = ldexpf(v, 7 - e);
    unsigned q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float qf = t + kMagic;
        q[i] = __float_as_uint(qf);
        if (i < 3) t = (t - (qf - kMagic)) * 128.0f;
    }
    const unsigned lo = __builtin_amdgcn_perm(q[1], q[0], 0x0c0c0400u);  // [q0.b0, q1.b0, 0, 0]
    const unsigned hi = __builtin_amdgcn_perm(q[3], q[2], 0x0c0c0400u);
    return lo | hi << 16;
}

// lane quad q = lane & 3 holds P = digits 0..3 of its channel (byte d = digit d); returns digit q of the
// quad's 4 channels (byte j = channel 4 (lane / 4) + j)
__device__ inline unsigned i8_quad_transpose(unsigned P, int lane) {
    const unsigned q1 = (unsigned)__builtin_amdgcn_mov_dpp((int)P, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    // even lane: [P.0 q1.0 P.2 q1.2], odd: [q1.1 P.1 q1.3 P.3]
    const unsigned R = __builtin_amdgcn_perm(q1, P, (lane & 1) ? 0x03070105u : 0x06020400u);
    const unsigned r2 = (unsigned)__builtin_amdgcn_mov_dpp((int)R, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    // lanes 0, 1 of the quad: [R.0 R.1 r2.0 r2.1], lanes 2, 3: [r2.2 r2.3 R.2 R.3]
    return __builtin_amdgcn_perm(r2, R, (lane & 2) ? 0x03020706u : 0x05040100u);
}

// CW channels per workgroup (2 CW threads: a plane split over lanes l, l ^ 32): 512 -- the row's exponent
// over all its channels, one workgroup per board -- or 256 -- one exponent per 256-channel segment
// (ex[(xi * 2 + seg) * rows + b]), two workgroups per board, so a CU holds two of them and one's loads
// overlap the other's transforms and reductions.
// The digits and exponent of `nslab` slabs of n rows of K fp64 values: row r of
// slab x is src[(x * slab_rows + r) * K ...]; digit d of its channels
// [32 kc, 32 kc + 32) goes to plane (x, kc, d) of dst -- 32 bytes at
// (((x * K/32 + kc) * 5 + d) * slab_rows + r) * 32 -- and the exponent to
// ex[x * slab_rows + r]. One wave per row; lane l holds channels
// [l * K/64, (l + 1) * K/64). RL (row lines, 4 digits only): digit d of the
// 32 channels goes to (((x * K/32 + kc) * slab_rows + r) * 4 + d) * 32 instead
// -- the 4 digits of one row's chunk are one 128-byte line. NSEG = 2 (K = 512 only): one exponent per
// 256-channel segment instead of per row (lanes 0-31 hold segment 0), at ex[(x * 2 + seg) * slab_rows + r].
// R3 (KV_PATH_WINO88_I8F32R3; row lines): 3 radix-256 digits (i8_digits_r3) under the radix-256 exponent rule of
// the fp32 or fp64 rows, in 96-byte lines (((x * K/32 + kc) * slab_rows + r) * 3 + d) * 32
template <int K, class T, int D, bool RL = false, int NSEG = 1, bool R8 = false, bool R3 = false>
__global__ __launch_bounds__(256) void wino88i_slice_kernel(const T* __restrict__ src, int n, int slab_rows,
                                                            int nslab, int8_t* __restrict__ dst,
                                                            int* __restrict__ ex) {
    static_assert(K == 256 || K == 512, "rows of 256 or 512 channels");
    static_assert(!RL || D == 4, "row lines hold 4 digits");
    static_assert(NSEG == 1 || (NSEG == 2 && K == 512), "segments of 256 channels");
    static_assert(!R8 || (D == 4 && sizeof(T) == 8 && NSEG == 1), "radix 256: 4 digits of fp64 rows");
    static_assert(!R3 || (D == 4 && RL && NSEG == 1 && !R8), "3 radix-256 digits in 96-byte row lines");
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
    for (int o = 64 / (2 * NSEG); o > 0; o >>= 1) {
        const unsigned t = (unsigned)__shfl_xor((int)m, o, 64);
        m = t > m ? t : m;
    }
    const int e = (R8 || (R3 && sizeof(T) == 8)) ? i8_row_exponent_r8(m)
                  : R3                              ? i8_row_exponent_f32r(m)
                  : sizeof(T) == 8                  ? i8_row_exponent(m)
                                                    : i8_row_exponent_f32(m);
    if (NSEG == 1 && lane == 0) ex[row] = e;
    if (NSEG == 2 && (lane & 31) == 0) ex[((size_t)x * 2 + (lane >> 5)) * slab_rows + r] = e;
    unsigned long long pk[D] = {};
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        int dg[D];
        if constexpr (R8) {
            const unsigned P = i8_digits_r8((double)v[i], e);
#pragma unroll
            for (int d = 0; d < D; ++d) dg[d] = (int)(signed char)(P >> (8 * (D - 1 - d)));
        } else if constexpr (R3) {
            const unsigned P = i8_digits_r3((double)v[i], e);  // byte d = digit d, slot 3 zero
#pragma unroll
            for (int d = 0; d < D; ++d) dg[d] = (int)(signed char)(P >> (8 * d));
        } else {
            i8_digits<D>(v[i], e, dg);
        }
#pragma unroll
        for (int d = 0; d < D; ++d) pk[d] |= (unsigned long long)(unsigned char)(signed char)dg[d] << (8 * i);
    }
    const int c = lane * CPL, kc = c / 32;
    constexpr int LW = R3 ? 3 * 32 : D * 32;  // row-line bytes (R3: the 3 digits only)
    int8_t* o = RL ? dst + (((size_t)x * (K / 32) + kc) * slab_rows + r) * LW + (c % 32)
                   : dst + ((((size_t)x * (K / 32) + kc) * D) * slab_rows + r) * 32 + (c % 32);
#pragma unroll
    for (int d = 0; d < (R3 ? 3 : D); ++d) {
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

// wino88i_gemm_kernel<K, 4, ., float, true> with the stage barrier moved to the middle of the stage
// (MID): a stage's MFMAs run in two halves (B digits 0-1: 14 of its 20 MFMAs per wave; 2-3: 6), and between
// them the waves wait for the NEXT stage's copies, pass one barrier, and read that stage's A digits and first
// B digit -- so those LDS reads run under the second half's MFMAs instead of after a barrier with both waves
// of a SIMD idle. The ring has 4 buffers: stage kt + 3's copies go out after the barrier in the middle of
// stage kt (all waves are then past stage kt - 1, whose buffer they refill), two per B digit of the second
// half. Same products, same k order, same bits.
template <int K>
__global__ __launch_bounds__(512) void wino88i32_gemm_mid_kernel(const int8_t* __restrict__ V8,
                                                                 const int* __restrict__ ev,
                                                                 const int8_t* __restrict__ U8,
                                                                 const int* __restrict__ eu, float* __restrict__ M,
                                                                 int rows, int cout, int stride) {
    constexpr int S = 4, NBUF = 4;
    using T = Wino88iTile<S>;
    constexpr int NT = T::NT, WM = T::WM, WN = T::WN, GL = T::GL;
    constexpr int NK = K / 32;
    static_assert(GL == 4 && NK >= 4, "4 pieces per wave and stage");

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8m[];
    char* const L0 = (char*)lds_i8m;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / T::WC, wn = wave % T::WC;
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x;  // a multiple of 8
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx / (CT * RT);
    const int n_base = (idx % CT) * WN;
    const int r_base = ((idx / CT) % RT) * WM;

    // copy pieces as wino88i_gemm_kernel's row-line path: piece q = wave * 4 + g covers operand q / 16,
    // rows 8 (q % 16) .. +7
    const int op = (wave * GL) / (4 * S);
    const size_t rstride = op ? (size_t)cout : (size_t)stride;
    const int8_t* gbase = op ? U8 + (((size_t)xi * NK) * cout + (size_t)n_base) * 128
                             : V8 + (((size_t)xi * NK) * stride + (size_t)r_base) * 128;
    const size_t sstep = rstride * 128;
    const int rl_off0 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4));
    const int rl_off1 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4) ^ 4);
    auto issue1 = [&](int g, int kt) {
        const int q = wave * GL + g, rg8 = q % 16;
        __builtin_amdgcn_global_load_lds(
            (const void*)(gbase + kt * sstep + (size_t)rg8 * 1024 + ((rg8 & 1) ? rl_off1 : rl_off0)),
            (__attribute__((address_space(3))) void*)(L0 + (kt % NBUF) * T::STAGE + op * S * T::PLANE + rg8 * 1024),
            16, 0, 0);
    };

    const int lr = lane & 31, lh = lane >> 5;
    const int arow = wm * 32 + lr;
    int aoffr[S], boffr[NT][S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        aoffr[i] = i8_rl_off(arow, 2 * i + lh);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) boffr[nt][i] = S * T::PLANE + i8_rl_off(wn * NT * 32 + nt * 32 + lr, 2 * i + lh);
    }

    i32x16_t acc[S][NT];
#pragma unroll
    for (int l = 0; l < S; ++l)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[l][nt] = i32x16_t{};

    // prologue: stages 0-2 in flight, stage 0 landed (this wave's copies, then every wave's), its A digits
    // and first B digit read
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int g = 0; g < GL; ++g) issue1(g, k);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    i8x16_t a[S], b0[NT];
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = *(const i8x16_t*)(L0 + aoffr[i]);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) b0[nt] = *(const i8x16_t*)(L0 + boffr[nt][0]);

    for (int kt = 0; kt < NK; ++kt) {
        const char* buf = L0 + (kt % NBUF) * T::STAGE;
        i8x16_t b1[NT], b2[NT], b3[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b1[nt] = *(const i8x16_t*)(buf + boffr[nt][1]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                acc[i][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b0[nt], acc[i][nt], 0, 0, 0);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b2[nt] = *(const i8x16_t*)(buf + boffr[nt][2]);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                acc[i + 1][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b1[nt], acc[i + 1][nt], 0, 0, 0);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b3[nt] = *(const i8x16_t*)(buf + boffr[nt][3]);
        // the A digits of stage kt that the second half still needs (i = 0, 1), before they are replaced
        const i8x16_t a0 = a[0], a1 = a[1];
        // middle: stage kt + 1 landed (only stage kt + 2's copies may still be in flight), then every wave
        // is past stage kt - 1, whose buffer stage kt + 3's copies refill
        if (kt + 1 < NK) {
            if (kt + 2 < NK)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 1 < NK) {
            const char* nb = L0 + ((kt + 1) % NBUF) * T::STAGE;
#pragma unroll
            for (int i = 0; i < S; ++i) a[i] = *(const i8x16_t*)(nb + aoffr[i]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                acc[i + 2][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(i ? a1 : a0, b2[nt], acc[i + 2][nt], 0, 0, 0);
        if (kt + 3 < NK) {
            issue1(0, kt + 3);
            issue1(1, kt + 3);
        }
        if (kt + 1 < NK) {
            const char* nb = L0 + ((kt + 1) % NBUF) * T::STAGE;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) b0[nt] = *(const i8x16_t*)(nb + boffr[nt][0]);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
            acc[3][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b3[nt], acc[3][nt], 0, 0, 0);
        if (kt + 3 < NK) {
            issue1(2, kt + 3);
            issue1(3, kt + 3);
        }
    }

    // epilogue (as wino88i_gemm_kernel's): D col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int* evx = ev + (size_t)xi * stride + r_base + wm * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = n_base + wn * NT * 32 + nt * 32 + lr;
        const int ec = eu[(size_t)xi * cout + col] - 14;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            double m = (double)acc[S - 1][nt][r];
#pragma unroll
            for (int l = S - 2; l >= 0; --l) m = __builtin_fma(m, 0.0078125, (double)acc[l][nt][r]);  // exact
            M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col] = (float)ldexp(m, evx[row] + ec);
        }
    }
}

// The same GEMM as one loop over stage barriers in which a wave's MFMAs for stage k are split in two
// halves: h1(k) = B digits 0-1 (14 of 20 MFMAs per wave), h2(k) = B digits 2-3 (6). Two programs:
//   LAG ("mid"): after barrier k it reads stage k's A digits and first B digit while it runs h2(k - 1)
//     from registers (the A digits 0-1 and B digits 2-3 of stage k - 1, kept), then h1(k);
//   plain: after barrier k it reads stage k's digits and runs h1(k) and h2(k).
// Either way every LDS read of stage k happens between barriers k and k + 1, so stage k + 2's copies go into
// stage k - 1's buffer right after barrier k (3 buffers, two stages in flight). STAG: waves 0-3 lag, waves
// 4-7 do not -- the two waves of a SIMD then reach each barrier at different points of their MFMA streams
// (one finishing a stage, one mid-stage), so one issues MFMAs while the other waits on its LDS reads; else
// every wave lags. Same products, same bits.
#ifndef KV_LAG_OPAQUE
// 1: the lagging operands redefined opaquely after the pre-barrier lgkmcnt(0) (so the compiler's waitcnt pass
// cannot make the first lagging MFMA wait for the new stage's LDS reads). Bit-identical either way; measured
// (profiles/r06_gemm_opaque_lj_ab.log) neutral on the 4-digit tower and 0.6-1.5 % slower forward on R3: off.
#define KV_LAG_OPAQUE 0
#endif
template <int K, bool STAG, int LJ = 2>
__global__ __launch_bounds__(512) void wino88i32_gemm_lag_kernel(const int8_t* __restrict__ V8,
                                                                 const int* __restrict__ ev,
                                                                 const int8_t* __restrict__ U8,
                                                                 const int* __restrict__ eu, float* __restrict__ M,
                                                                 int rows, int cout, int stride) {
    constexpr int S = 4, NBUF = 3;
    using T = Wino88iTile<S>;
    constexpr int NT = T::NT, WM = T::WM, WN = T::WN, GL = T::GL;
    constexpr int NK = K / 32;
    constexpr int NA = S - LJ;  // A digits the lagging half uses (0 .. S - LJ - 1)
    static_assert(GL == 4 && NK >= 3 && LJ >= 1 && LJ <= 3, "4 pieces per wave and stage; B digits LJ.. lag");

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8l[];
    char* const L0 = (char*)lds_i8l;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const bool lag = !STAG || wave < 4;  // wave-uniform
    const int wm = wave / T::WC, wn = wave % T::WC;
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x;  // a multiple of 8
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx / (CT * RT);
    const int n_base = (idx % CT) * WN;
    const int r_base = ((idx / CT) % RT) * WM;

    const int op = (wave * GL) / (4 * S);
    const size_t rstride = op ? (size_t)cout : (size_t)stride;
    const int8_t* gbase = op ? U8 + (((size_t)xi * NK) * cout + (size_t)n_base) * 128
                             : V8 + (((size_t)xi * NK) * stride + (size_t)r_base) * 128;
    const size_t sstep = rstride * 128;
    const int rl_off0 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4));
    const int rl_off1 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4) ^ 4);
    auto issue1 = [&](int g, int kt) {
        const int q = wave * GL + g, rg8 = q % 16;
        __builtin_amdgcn_global_load_lds(
            (const void*)(gbase + kt * sstep + (size_t)rg8 * 1024 + ((rg8 & 1) ? rl_off1 : rl_off0)),
            (__attribute__((address_space(3))) void*)(L0 + (kt % NBUF) * T::STAGE + op * S * T::PLANE + rg8 * 1024),
            16, 0, 0);
    };

    const int lr = lane & 31, lh = lane >> 5;
    const int arow = wm * 32 + lr;
    int aoffr[S], boffr[NT][S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        aoffr[i] = i8_rl_off(arow, 2 * i + lh);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) boffr[nt][i] = S * T::PLANE + i8_rl_off(wn * NT * 32 + nt * 32 + lr, 2 * i + lh);
    }

    i32x16_t acc[S][NT];
#pragma unroll
    for (int l = 0; l < S; ++l)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[l][nt] = i32x16_t{};
    // h2 of a stage: B digits j >= LJ with the A digits i < S - j
    i8x16_t pa[NA] = {}, pb[S - LJ][NT] = {};
    auto h2 = [&](const i8x16_t (&x)[NA], const i8x16_t (&y)[S - LJ][NT]) {
#pragma unroll
        for (int j = LJ; j < S; ++j)
#pragma unroll
            for (int i = 0; i + j < S; ++i)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[i + j][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(x[i], y[j - LJ][nt], acc[i + j][nt], 0, 0, 0);
    };

    issue1(0, 0); issue1(1, 0); issue1(2, 0); issue1(3, 0);
    issue1(0, 1); issue1(1, 1); issue1(2, 1); issue1(3, 1);
    for (int kt = 0; kt < NK; ++kt) {
        // stage kt landed: only stage kt + 1's copies may still be in flight; lgkmcnt(0): the lagging B digits
        // of stage kt - 1 were read from the buffer stage kt + 2's copies overwrite once every wave passes this
        // barrier, and their reads are only waited for at the MFMAs after it (a formal WAR race)
        if (kt + 1 < NK)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#if KV_LAG_OPAQUE  // the lagging operands are in registers (wino88i32_gemm_lagt_kernel)
#pragma unroll
        for (int i = 0; i < NA; ++i) asm volatile("" : "+v"(pa[i]));
#pragma unroll
        for (int jb = 0; jb < S - LJ; ++jb)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(pb[jb][nt]));
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* buf = L0 + (kt % NBUF) * T::STAGE;
        i8x16_t a[S], b[S][NT];
#pragma unroll
        for (int i = 0; i < S; ++i) a[i] = *(const i8x16_t*)(buf + aoffr[i]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b[0][nt] = *(const i8x16_t*)(buf + boffr[nt][0]);
        if (lag && kt > 0) h2(pa, pb);  // under the reads above
        // stage kt + 2 into stage kt - 1's buffer, two pieces at the start, two after the first B digit
        if (kt + 2 < NK) {
            issue1(0, kt + 2);
            issue1(1, kt + 2);
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {
            if (j + 1 < S) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) b[j + 1][nt] = *(const i8x16_t*)(buf + boffr[nt][j + 1]);
            }
            if (j < LJ) {
#pragma unroll
                for (int i = 0; i + j < S; ++i)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[i + j][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j][nt], acc[i + j][nt], 0, 0, 0);
            }
            if (j == 0 && kt + 2 < NK) {
                issue1(2, kt + 2);
                issue1(3, kt + 2);
            }
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) pa[i] = a[i];
#pragma unroll
        for (int j = LJ; j < S; ++j)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) pb[j - LJ][nt] = b[j][nt];
        if (!lag) h2(pa, pb);  // h2(kt) now
    }
    if (lag) h2(pa, pb);

    // epilogue (as wino88i_gemm_kernel's): D col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int* evx = ev + (size_t)xi * stride + r_base + wm * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = n_base + wn * NT * 32 + nt * 32 + lr;
        const int ec = eu[(size_t)xi * cout + col] - 14;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            double m = (double)acc[S - 1][nt][r];
#pragma unroll
            for (int l = S - 2; l >= 0; --l) m = __builtin_fma(m, 0.0078125, (double)acc[l][nt][r]);  // exact
            M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col] = (float)ldexp(m, evx[row] + ec);
        }
    }
}

// wino88i32_gemm_lag_kernel with TPW tiles per workgroup: the copy ring runs across the tile boundaries (a tile's
// first two stages go out during the previous tile's last two), so every tile after a workgroup's first starts
// with its operands in LDS. kv_nn.hip picks TPW so the workgroups fill whole rounds in no more tile-times than
// single tiles: C3's 6,400 tiles as 5 rounds of 5-tile workgroups (497 vs 511 us), C2's 800 as one round of
// 4-tile workgroups (72 vs 76 us; profiles/r05_i8gemm_lagt_ab.log, r05_i8gemm_tpw5_ab.log). The tile loop is
// unrolled (a runtime count recomputing tile coordinates per copy ran 13 % slower,
// profiles/r05_i8gemm_tpw_runtime_ab.log). Tile j of workgroup w is virtual
// block w + j * gridDim in the XCD-aware order (the same XCD). At the first stage of a later tile a wave waits
// for that stage's pieces with the previous tile's 32 M stores still allowed in flight. Same products, same bits.
#ifndef KV_I8F32_LJ
#define KV_I8F32_LJ 2
#endif
// STAMP (a diagnostic build, never the product's): wave 0 of each workgroup records the shader clock
// (s_memtime) and the 100 MHz constant clock (s_memrealtime) at its start and end into stamps[4 * block] -- a
// buffer of its own that no other code reads; kv_dev_gemm_clock turns them into the clock the chip held.
// ND: digit levels (4; round 6's ND = 3 form for KV_PATH_WINO88_I8F32R3 retired with R3's 128-byte lines: R3 runs
// wino88i32_gemm_r3k64_kernel on 96-byte lines).
// KV_COPY_SADDR (1): the ring's copies address a wave-uniform 64-bit base plus an unsigned 32-bit lane offset,
// so they issue in the scalar-base form (one address VGPR per lane); 0: a 64-bit VGPR address pair per lane.
#ifndef KV_COPY_SADDR
#define KV_COPY_SADDR 1
#endif
// NB: buffers of the copy ring (NB x 32 KiB of LDS), so NB - 1 stages are in flight past the one being read: the
// copies of stage k + NB - 1 go into stage k - 1's buffer right after barrier k.
template <int N>
__device__ __forceinline__ void vm_lgkm_wait() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
template <int K, int TPW, int LJ = KV_I8F32_LJ, bool STAMP = false, int ND = 4, int NB = 3>
__global__ __launch_bounds__(512) void wino88i32_gemm_lagt_kernel(const int8_t* __restrict__ V8,
                                                                  const int* __restrict__ ev,
                                                                  const int8_t* __restrict__ U8,
                                                                  const int* __restrict__ eu, float* __restrict__ M,
                                                                  int rows, int cout, int stride,
                                                                  unsigned long long* __restrict__ stamps) {
    unsigned long long t0 = 0, r0 = 0;
    if constexpr (STAMP) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    constexpr int S = 4, NBUF = NB, PD = NB - 1;  // PD: prefetch distance in stages
    using T = Wino88iTile<S>;
    constexpr int NT = T::NT, WM = T::WM, WN = T::WN, GL = T::GL;
    constexpr int NK = K / 32, NS = TPW * NK;
    constexpr int NA = ND - LJ;
    static_assert(GL == 4 && NK >= 3 && LJ >= 1 && LJ < ND && ND == 4, "4 pieces per wave and stage, 4 digits");
    static_assert(NB >= 3 && NB <= 5 && PD < NK, "ring of 3-5 stage buffers (at most 160 KiB)");
    constexpr double kStep = ND == 4 ? 0.0078125 : 0.00390625;  // level weight: radix 128 / 256

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8t[];
    char* const L0 = (char*)lds_i8t;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / T::WC, wn = wave % T::WC;
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x, nv = nwg * TPW;  // nwg a multiple of 8
    int xis[TPW], nbs[TPW], rbs[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        const int vb = (int)blockIdx.x + j * nwg;
        const int idx = (vb & 7) * (nv >> 3) + (vb >> 3);
        xis[j] = idx / (CT * RT);
        nbs[j] = (idx % CT) * WN;
        rbs[j] = ((idx / CT) % RT) * WM;
    }

    const int wu = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar tile bases
    const int op = (wu * GL) / (4 * S);
    const size_t sstep = (op ? (size_t)cout : (size_t)stride) * 128;
    const int8_t* gb[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
        gb[j] = op ? U8 + (((size_t)xis[j] * NK) * cout + (size_t)nbs[j]) * 128
                   : V8 + (((size_t)xis[j] * NK) * stride + (size_t)rbs[j]) * 128;
    const int rl_off0 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4));
    const int rl_off1 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4) ^ 4);
    auto issue1 = [&](int g, int s) {  // piece g of global stage s (tile s / NK, stage s % NK)
        const int q = wu * GL + g, rg8 = q % 16;
        const int j = s / NK, kt = s - j * NK;
        const int8_t* base = gb[0];
#pragma unroll
        for (int jj = 1; jj < TPW; ++jj) base = j == jj ? gb[jj] : base;
        const int8_t* const sb = base + kt * sstep + (size_t)rg8 * 1024;  // wave-uniform
#if KV_COPY_SADDR
        const void* src = (const void*)(sb + (unsigned)((rg8 & 1) ? rl_off1 : rl_off0));
#else
        const void* src = (const void*)(sb + (size_t)((rg8 & 1) ? rl_off1 : rl_off0));
#endif
        __builtin_amdgcn_global_load_lds(
            src, (__attribute__((address_space(3))) void*)(L0 + (s % NBUF) * T::STAGE + op * S * T::PLANE + rg8 * 1024),
            16, 0, 0);
    };

    const int lr = lane & 31, lh = lane >> 5;
    const int arow = wm * 32 + lr;
    int aoffr[ND], boffr[NT][ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        aoffr[i] = i8_rl_off(arow, 2 * i + lh);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) boffr[nt][i] = S * T::PLANE + i8_rl_off(wn * NT * 32 + nt * 32 + lr, 2 * i + lh);
    }

#pragma unroll
    for (int p = 0; p < PD; ++p) {
        issue1(0, p); issue1(1, p); issue1(2, p); issue1(3, p);
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        i32x16_t acc[ND][NT];
#pragma unroll
        for (int l = 0; l < ND; ++l)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[l][nt] = i32x16_t{};
        i8x16_t pa[NA] = {}, pb[ND - LJ][NT] = {};
        auto h2 = [&]() {
#pragma unroll
            for (int jb = LJ; jb < ND; ++jb)
#pragma unroll
                for (int i = 0; i + jb < ND; ++i)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[i + jb][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(pa[i], pb[jb - LJ][nt], acc[i + jb][nt], 0, 0, 0);
        };
        for (int kt = 0; kt < NK; ++kt) {
            const int s = j * NK + kt;
            // stage s's pieces landed: vmcnt counts in issue order, so what may stay outstanding is the m later
            // stages already issued and, for a tile's first PD stages, the previous tile's 32 M stores (issued
            // after them). For NB = 3 and kt = 1 this is one wait less strict than round 5's vmcnt(GL)
            const int m = NS - 1 - s < PD - 1 ? NS - 1 - s : PD - 1;
            if (j > 0 && kt < PD) {
                if (m == 0) vm_lgkm_wait<32>();
                else if (m == 1) vm_lgkm_wait<GL + 32>();
                else if (m == 2) vm_lgkm_wait<2 * GL + 32>();
                else vm_lgkm_wait<3 * GL + 32>();
            } else {
                if (m == 0) vm_lgkm_wait<0>();
                else if (m == 1) vm_lgkm_wait<GL>();
                else if (m == 2) vm_lgkm_wait<2 * GL>();
                else vm_lgkm_wait<3 * GL>();
            }
            // the lagging operands are in registers now (lgkmcnt(0) above); KV_LAG_OPAQUE tells the compiler
            // so by an opaque redefinition (measured: no gain, see its definition)
#if KV_LAG_OPAQUE
#pragma unroll
            for (int i = 0; i < NA; ++i) asm volatile("" : "+v"(pa[i]));
#pragma unroll
            for (int jb = 0; jb < ND - LJ; ++jb)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(pb[jb][nt]));
#endif
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const char* buf = L0 + (s % NBUF) * T::STAGE;
            i8x16_t a[ND], b[ND][NT];
#pragma unroll
            for (int i = 0; i < ND; ++i) a[i] = *(const i8x16_t*)(buf + aoffr[i]);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) b[0][nt] = *(const i8x16_t*)(buf + boffr[nt][0]);
            // the stage's reads issue before the lagging MFMAs (hipcc otherwise hoists those MFMAs above the reads,
            // so the reads start ~14 MFMA issues after the barrier): forward -2.3 % at 2,048 boards, -3.4 % at 256,
            // bit-identical; with the same barrier after each B digit's reads below, -5 % / -6 %
            // (profiles/r05_reads_first_ab.log; the 13-pair fp64-domain GEMM and the one-tile lag kernel came out
            // 1-2 % slower with it, so only here)
            __builtin_amdgcn_sched_barrier(0);
            if (kt > 0) h2();
            if (s + PD < NS) {
                issue1(0, s + PD);
                issue1(1, s + PD);
            }
#pragma unroll
            for (int jb = 0; jb < ND; ++jb) {
                if (jb + 1 < ND) {
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) b[jb + 1][nt] = *(const i8x16_t*)(buf + boffr[nt][jb + 1]);
                }
                __builtin_amdgcn_sched_barrier(0);  // likewise each next B digit's reads before this one's MFMAs
                if (jb < LJ) {
#pragma unroll
                    for (int i = 0; i + jb < ND; ++i)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[i + jb][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[jb][nt], acc[i + jb][nt], 0, 0, 0);
                }
                if (jb == 0 && s + PD < NS) {
                    issue1(2, s + PD);
                    issue1(3, s + PD);
                }
            }
#pragma unroll
            for (int i = 0; i < NA; ++i) pa[i] = a[i];
#pragma unroll
            for (int jb = LJ; jb < ND; ++jb)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) pb[jb - LJ][nt] = b[jb][nt];
        }
        h2();
        const int xi = xis[j], n_base = nbs[j], r_base = rbs[j];
        const int* evx = ev + (size_t)xi * stride + r_base + wm * 32;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int col = n_base + wn * NT * 32 + nt * 32 + lr;
            const int ec = eu[(size_t)xi * cout + col] - 14;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
                double m = (double)acc[ND - 1][nt][r];
#pragma unroll
                for (int l = ND - 2; l >= 0; --l) m = __builtin_fma(m, kStep, (double)acc[l][nt][r]);  // exact
                M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col] = (float)ldexp(m, evx[row] + ec);
            }
        }
    }
    if constexpr (STAMP) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x < 4) {  // one vector store per value, lanes 0-3
            const unsigned long long v = threadIdx.x == 0 ? t0 : threadIdx.x == 1 ? t1 : threadIdx.x == 2 ? r0 : r1;
            stamps[(size_t)blockIdx.x * 4 + threadIdx.x] = v;
        }
    }
}

template <int ABL>
__device__ __forceinline__ i32x16_t r3mfma(i8x16_t a, i8x16_t b, i32x16_t c) {
    if constexpr ((ABL & 2) != 0) {  // ablation: the fragments are consumed, no MFMA issues
        asm volatile("" ::"v"(a), "v"(b));
        return c;
    } else {
        return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    }
}
// R3's GEMM (KV_PATH_WINO88_I8F32R3) with 64-k stages: the 32-k lagt kernel gives a wave 12 MFMAs per stage
// barrier at 3 digits (20 at 4), and its time did not move with 3, 4 or 5 ring buffers (370.6 / 371.3 / 371.6
// us, profiles/r06_ring_depth_ab.log): the barrier's fixed cost, not the copies' latency, sets it. Here a stage is
// two 32-channel chunks (24 MFMAs per wave per barrier) of R3's 96-byte row lines [xi][K/32][row][3][32] (3
// digits, no zero slot), so a stage is 48 KiB and the ring keeps 3 buffers (144 KiB) with two stages in flight.
// LDS image per operand and chunk: 128 rows of 96 bytes (a contiguous 12 KiB block of the global lines), 16-byte
// piece c = 2 d + half at position c ^ ((row >> 4) & 1) -- every ds_read_b128 lane group conflict-free
// (rows 16-31 of a 32-row block land on the odd 16-byte bank groups, rows 0-15 on the even ones). Copies: wave
// w fills 6 KiB pieces of plane (operand w >> 2, chunk (w >> 1) & 1), pieces 6 (w & 1) .. + 5; lane l of piece
// pp carries unit u = 64 pp + l = (row u / 6, slot u % 6). Per stage a wave runs chunk 0's 12 MFMAs, chunk 1's
// B digit 0 (6), and chunk 1's B digits 1-2 (6) after the next barrier under that stage's first reads. Same
// products, same exact int32 levels, same bits as the 32-k lagt form it replaced (measured bit-identical,
// profiles/r06_r3k64_ab.log; that form read 128-byte lines with a zero 4th slot and was retired with them).
// ABL (timing ablations, outputs invalid; never the product's): 1 no copies after the prologue, 2 no MFMAs (the
// fragments still read), 4 no M stores, 8 no exponent loads in the epilogue. KV_R3_M_NT (1): M stored non-temporally -- the GEMM 339 -> 325 us, the
// output kernels that read it +2 %, forward -1.5 % at 2,048 boards, neutral at 256 (profiles/r06_mnt_ab.log).
#ifndef KV_R3_M_NT
#define KV_R3_M_NT 1
#endif
template <int K, int TPW, bool STAMP = false, int ABL = 0>
__global__ __launch_bounds__(512) void wino88i32_gemm_r3k64_kernel(const int8_t* __restrict__ V8,
                                                                   const int* __restrict__ ev,
                                                                   const int8_t* __restrict__ U8,
                                                                   const int* __restrict__ eu, float* __restrict__ M,
                                                                   int rows, int cout, int stride,
                                                                   unsigned long long* __restrict__ stamps) {
    unsigned long long t0 = 0, r0 = 0;
    if constexpr (STAMP) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    constexpr int ND = 3, NB = 3, PD = NB - 1, GL = 6;
    constexpr int NT = 2, WM = 128, WN = 128, WC = 2;
    constexpr int NK = K / 32, NU = NK / 2, NSG = TPW * NU;  // stages per group of TPW tiles
    constexpr int PLANE = 128 * 96, STAGE = 4 * PLANE;  // [operand][chunk] planes: 48 KiB
    static_assert(NK % 2 == 0 && NU > PD && 8 * GL * 1024 == STAGE, "64-k stages, 6 pieces per wave");
    constexpr double kStep = 0.00390625;  // level weight: radix 256

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8k64[];
    char* const L0 = (char*)lds_i8k64;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WC, wn = wave % WC;
    const int CT = cout / WN, RT = rows / WM;
    // nwg a multiple of 8; a workgroup runs ng groups of TPW tiles (the host makes nv = nwg TPW ng exact): one group
    // per workgroup in rounds, or, when the groups fill whole rounds of the CUs, ng of them per workgroup in one
    // round, the copy ring running across the group boundaries too
    const int nwg = (int)gridDim.x, nv = kv::W88_XI * RT * CT, ng = nv / (nwg * TPW), NST = ng * NSG;
    auto coords = [&](int T, int& xi, int& nb, int& rb) {  // tile T of this workgroup (XCD-aware order)
        const int vb = (int)blockIdx.x + T * nwg;
        const int idx = (vb & 7) * (nv >> 3) + (vb >> 3);
        xi = idx / (CT * RT);
        nb = (idx % CT) * WN;
        rb = ((idx / CT) % RT) * WM;
    };
    int xis[TPW], nbs[TPW], rbs[TPW];

    const int wu = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: the plane this wave copies
    const int op = wu >> 2, chunk = (wu >> 1) & 1, pp0 = 6 * (wu & 1);
    const size_t sstep = (op ? (size_t)cout : (size_t)stride) * 96;  // one 32-channel chunk of 96-byte row lines
    auto tile_base = [&](int xi, int nb, int rb) {
        return (op ? U8 + (((size_t)xi * NK) * cout + (size_t)nb) * 96 : V8 + (((size_t)xi * NK) * stride + (size_t)rb) * 96) +
               (size_t)chunk * sstep;
    };
    const int8_t* gb[TPW + 1];  // the group's tiles, then the next group's first
    // this lane's source byte in a chunk's row-line block, per piece: unsigned 32-bit, so the copy takes the
    // scalar-base + 32-bit-offset address form (one address VGPR per lane instead of a 64-bit pair)
    unsigned goff[GL];
#pragma unroll
    for (int g = 0; g < GL; ++g) {
        const int u = (pp0 + g) * 64 + lane, row = u / 6, slot = u - 6 * (u / 6);
        goff[g] = (unsigned)(row * 96 + 16 * (slot ^ ((row >> 4) & 1)));
    }
    const int ldst = (op * 2 + chunk) * PLANE + pp0 * 1024;
    auto issue1 = [&](int g, int s, int sg) {  // piece g of the group's stage s (tile s / NU), ring stage sg
        if constexpr ((ABL & 1) != 0)
            if (sg >= PD) return;
        const int j = s / NU, ku = s - j * NU;
        const int8_t* base = gb[0];
#pragma unroll
        for (int jj = 1; jj <= TPW; ++jj) base = j == jj ? gb[jj] : base;
        const int8_t* const sb = base + (size_t)(2 * ku) * sstep;  // wave-uniform
#if KV_COPY_SADDR
        const void* src = (const void*)(sb + goff[g]);
#else
        const void* src = (const void*)(sb + (size_t)(int)goff[g]);
#endif
        __builtin_amdgcn_global_load_lds(src,
                                         (__attribute__((address_space(3))) void*)(L0 + (sg % NB) * STAGE + ldst +
                                                                                   g * 1024),
                                         16, 0, 0);
    };

    const int lr = lane & 31, lh = lane >> 5;
    const int arow = wm * 32 + lr;
    int aoff[2][ND], boff[2][NT][ND];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            aoff[h][d] = h * PLANE + arow * 96 + 16 * ((2 * d + lh) ^ ((arow >> 4) & 1));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int brow = wn * NT * 32 + nt * 32 + lr;
                boff[h][nt][d] = (2 + h) * PLANE + brow * 96 + 16 * ((2 * d + lh) ^ ((brow >> 4) & 1));
            }
        }

    // each group's row / column exponents staged in LDS beside the ring (2 x TPW x 1 KiB, by group parity): loaded
    // into registers at the group's start and stored after its first two stages, so the epilogue reads LDS instead
    // of waiting on global loads at each tile's end (timing ablation without the loads: 339 -> 323 us,
    // profiles/r06_r3k64_ablations_final.log)
    constexpr int NEX = (TPW * 256 + 511) / 512;
    int* const exl = (int*)(L0 + NB * STAGE);  // [2][TPW][256]: ev rows 0-127, eu columns 128-255
    for (int gi = 0; gi < ng; ++gi) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        coords(gi * TPW + j, xis[j], nbs[j], rbs[j]);
        gb[j] = tile_base(xis[j], nbs[j], rbs[j]);
    }
    {
        int xn, nn, rn;
        coords(gi + 1 < ng ? (gi + 1) * TPW : gi * TPW, xn, nn, rn);
        gb[TPW] = tile_base(xn, nn, rn);
    }
    int exv[NEX];
#pragma unroll
    for (int q = 0; q < NEX; ++q) {
        const int t = tid + q * 512;
        exv[q] = 0;
        if (t < TPW * 256) {
            const int jj = t >> 8, k = t & 255;
            exv[q] = k < 128 ? ev[(size_t)xis[jj] * stride + rbs[jj] + k] : eu[(size_t)xis[jj] * cout + nbs[jj] + k - 128];
        }
    }
    int* const exg = exl + (gi & 1) * TPW * 256;
    if (gi == 0) {
#pragma unroll
        for (int p = 0; p < PD; ++p)
#pragma unroll
            for (int g = 0; g < GL; ++g) issue1(g, p, p);
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        i32x16_t acc[ND][NT];
#pragma unroll
        for (int l = 0; l < ND; ++l)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[l][nt] = i32x16_t{};
        i8x16_t pa[2] = {}, pb[2][NT] = {};  // chunk 1's A digits 0-1 and B digits 1-2, lagging
        auto h2 = [&]() {
#pragma unroll
            for (int jb = 1; jb < ND; ++jb)
#pragma unroll
                for (int i = 0; i + jb < ND; ++i)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[i + jb][nt] = r3mfma<ABL>(pa[i], pb[jb - 1][nt], acc[i + jb][nt]);
        };
        for (int ku = 0; ku < NU; ++ku) {
            const int s = j * NU + ku, sg = gi * NSG + s;
            // stage sg's pieces landed (vmcnt counts in issue order): what may stay outstanding is the m later
            // stages already issued and, for a tile's first PD stages, the previous tile's 32 M stores
            const int m = NST - 1 - sg < PD - 1 ? NST - 1 - sg : PD - 1;
            if ((gi > 0 || j > 0) && ku < PD) {
                if (m == 0) vm_lgkm_wait<32>();
                else vm_lgkm_wait<GL + 32>();
            } else {
                if (m == 0) vm_lgkm_wait<0>();
                else vm_lgkm_wait<GL>();
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const char* buf = L0 + (sg % NB) * STAGE;
            i8x16_t a0[ND], b0[ND][NT], a1[ND], b1[ND][NT];
#pragma unroll
            for (int d = 0; d < ND; ++d) a0[d] = *(const i8x16_t*)(buf + aoff[0][d]);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) b0[0][nt] = *(const i8x16_t*)(buf + boff[0][nt][0]);
            __builtin_amdgcn_sched_barrier(0);
            if (ku > 0) h2();
            if (sg + PD < NST) {
                issue1(0, s + PD, sg + PD);
                issue1(1, s + PD, sg + PD);
                issue1(2, s + PD, sg + PD);
            }
            // chunk 0: all 6 pairs
#pragma unroll
            for (int jb = 0; jb < ND; ++jb) {
                if (jb + 1 < ND) {
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) b0[jb + 1][nt] = *(const i8x16_t*)(buf + boff[0][nt][jb + 1]);
                } else {
#pragma unroll
                    for (int d = 0; d < ND; ++d) a1[d] = *(const i8x16_t*)(buf + aoff[1][d]);
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) b1[0][nt] = *(const i8x16_t*)(buf + boff[1][nt][0]);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i + jb < ND; ++i)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[i + jb][nt] = r3mfma<ABL>(a0[i], b0[jb][nt], acc[i + jb][nt]);
                if (jb == 0 && sg + PD < NST) {
                    issue1(3, s + PD, sg + PD);
                    issue1(4, s + PD, sg + PD);
                    issue1(5, s + PD, sg + PD);
                }
            }
            // chunk 1: B digit 0 now, digits 1-2 after the next barrier
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                b1[1][nt] = *(const i8x16_t*)(buf + boff[1][nt][1]);
                b1[2][nt] = *(const i8x16_t*)(buf + boff[1][nt][2]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < ND; ++i)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[i][nt] = r3mfma<ABL>(a1[i], b1[0][nt], acc[i][nt]);
            pa[0] = a1[0];
            pa[1] = a1[1];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                pb[0][nt] = b1[1][nt];
                pb[1][nt] = b1[2][nt];
            }
            if (j == 0 && ku == 1) {  // the group's exponents (read back after the next barrier)
#pragma unroll
                for (int q = 0; q < NEX; ++q)
                    if (tid + q * 512 < TPW * 256) exg[tid + q * 512] = exv[q];
            }
        }
        h2();
        const int xi = xis[j], n_base = nbs[j], r_base = rbs[j];
        const int* evx = exg + j * 256 + wm * 32;  // LDS (staged above)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int col = n_base + wn * NT * 32 + nt * 32 + lr;
            const int ec = (ABL & 8) ? -14 : exg[j * 256 + 128 + wn * NT * 32 + nt * 32 + lr] - 14;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
                double mm = (double)acc[ND - 1][nt][r];
#pragma unroll
                for (int l = ND - 2; l >= 0; --l) mm = __builtin_fma(mm, kStep, (double)acc[l][nt][r]);  // exact
                const float o = (float)ldexp(mm, ((ABL & 8) ? 0 : evx[row]) + ec);
                if constexpr ((ABL & 4) != 0)
                    asm volatile("" ::"v"(o));
                else if constexpr (KV_R3_M_NT)
                    __builtin_nontemporal_store(o, &M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col]);
                else
                    M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col] = o;
            }
        }
    }
    }  // groups
    if constexpr (STAMP) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x < 4) {  // one vector store per value, lanes 0-3
            const unsigned long long v = threadIdx.x == 0 ? t0 : threadIdx.x == 1 ? t1 : threadIdx.x == 2 ? r0 : r1;
            stamps[(size_t)blockIdx.x * 4 + threadIdx.x] = v;
        }
    }
}

// KV_PREC_I8X5's GEMM (5 digits, digit planes, fp64 M) with wino88i32_gemm_lag_kernel's schedule: the
// B digits j >= LJ of a stage (their pairs i + j <= 4) run after the next barrier, under that stage's first
// LDS reads; stage k + 2's copies (5 pieces per wave) go into stage k - 1's buffer right after barrier k.
// Same products, same bits as wino88i_gemm_kernel<K, 5, ., double>.
// S = 4, RB = 8 (KV_PATH_WINO88_I8R): 4 radix-256 digit planes per operand (4 pieces per wave and stage), the
// 13 pairs i + j <= 4 of 16 -- the same 5 levels, weighted 2^-8l -- combined in fp64 (the last two fma steps
// may round: |level| <= 4 K 2^14 = 2^25, so the value has up to 57 significant bits; one fp64 rounding each).
// RL (S = 4): the operands in row lines [xi][K/32][row][4][32] (the fp32 tower's layout and LDS image: a
// stage of a tile is one contiguous 16 KiB block per operand), so the fused output kernel of one board writes
// whole 128-byte lines.
template <int K, int LJ = 3, int S = 5, int RB = 7, bool RL = false>
__global__ __launch_bounds__(512) void wino88i_gemm_lag5_kernel(const int8_t* __restrict__ V8,
                                                                const int* __restrict__ ev,
                                                                const int8_t* __restrict__ U8,
                                                                const int* __restrict__ eu, double* __restrict__ M,
                                                                int rows, int cout, int stride) {
    constexpr int LEV = 5, NBUF = 3;  // levels: pairs i + j < LEV
    using T = Wino88iTile<S>;
    constexpr int NT = T::NT, WM = T::WM, WN = T::WN, GL = T::GL;
    constexpr int NK = K / 32;
    constexpr int NA = S < LEV - LJ ? S : LEV - LJ;  // A digits the lagging half uses
    static_assert(GL == S && NK >= 3 && LJ >= 1 && LJ < S && (S == 5 || (S == 4 && RB == 8)) && (!RL || S == 4),
                  "S pieces per wave and stage; row lines hold 4 digits");

    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8l5[];
    char* const L0 = (char*)lds_i8l5;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / T::WC, wn = wave % T::WC;
    const int CT = cout / WN, RT = rows / WM;
    const int nwg = (int)gridDim.x;  // a multiple of 8
    const int idx = (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3);
    const int xi = idx / (CT * RT);
    const int n_base = (idx % CT) * WN;
    const int r_base = ((idx / CT) % RT) * WM;

    // copy pieces as wino88i_gemm_kernel's planes path: piece q = wave * S + g covers operand q / 4S, digit
    // (q % 4S) / 4, rows 32 (q % 4) .. +31; lane l fills LDS row 32 (q % 4) + l / 2, half l & 1 (swapped on
    // bit 3 of the row)
    const int op = (__builtin_amdgcn_readfirstlane(wave) * GL) / (4 * S);  // wave-uniform
    const size_t rstride = op ? (size_t)cout : (size_t)stride;
    // (a tile's rows start at row * 32 in a plane, row * 128 in row lines; a stage is S * 32 B per row in both)
    const int8_t* gbase = op ? U8 + ((size_t)xi * NK) * S * cout * 32 + (size_t)n_base * (RL ? 128 : 32)
                             : V8 + ((size_t)xi * NK) * S * stride * 32 + (size_t)r_base * (RL ? 128 : 32);
    const size_t sstep = (size_t)S * rstride * 32;
    const int lane_off = (lane >> 1) * 32 + 16 * ((lane & 1) ^ ((lane >> 4) & 1));
    // RL: piece q = wave * 4 + g is 8 row lines (1 KiB) of operand q / 16, rows 8 (q % 16) .. +7, copied as
    // wino88i32_gemm_lag_kernel's (the 16-byte chunks swizzled by i8_rl_off on the global side)
    const int rl_off0 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4));
    const int rl_off1 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4) ^ 4);
    auto issue1 = [&](int g, int kt) {
        const int q = wave * GL + g;
        if constexpr (RL) {
            const int rg8 = __builtin_amdgcn_readfirstlane(q) % 16;  // wave-uniform: the scalar-base form
            const int8_t* const sb = gbase + kt * sstep + (size_t)rg8 * 1024;
#if KV_COPY_SADDR
            const void* src = (const void*)(sb + (unsigned)((rg8 & 1) ? rl_off1 : rl_off0));
#else
            const void* src = (const void*)(sb + (size_t)((rg8 & 1) ? rl_off1 : rl_off0));
#endif
            __builtin_amdgcn_global_load_lds(
                src, (__attribute__((address_space(3))) void*)(L0 + (kt % NBUF) * T::STAGE + op * S * T::PLANE + rg8 * 1024),
                16, 0, 0);
        } else {
            const int d = (q % (4 * S)) / 4, rg = q % 4;
            __builtin_amdgcn_global_load_lds(
                (const void*)(gbase + kt * sstep + ((size_t)d * rstride + rg * 32) * 32 + lane_off),
                (__attribute__((address_space(3))) void*)(L0 + (kt % NBUF) * T::STAGE + op * S * T::PLANE +
                                                          d * T::PLANE + rg * 1024),
                16, 0, 0);
        }
    };

    const int lr = lane & 31, lh = lane >> 5;
    const int arow = wm * 32 + lr;
    // LDS offsets of digit d's fragments: planes (d * PLANE + a fixed offset) or row lines (i8_rl_off per digit)
    int aoffd[S], boffd[NT][S];
#pragma unroll
    for (int d = 0; d < S; ++d) {
        aoffd[d] = RL ? i8_rl_off(arow, 2 * d + lh) : d * T::PLANE + arow * 32 + i8_lds_half(arow, lh);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int bcol = wn * NT * 32 + nt * 32 + lr;
            boffd[nt][d] = S * T::PLANE + (RL ? i8_rl_off(bcol, 2 * d + lh) : d * T::PLANE + bcol * 32 +
                                                                               i8_lds_half(bcol, lh));
        }
    }

    i32x16_t acc[LEV][NT];
#pragma unroll
    for (int l = 0; l < LEV; ++l)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[l][nt] = i32x16_t{};
    i8x16_t pa[NA] = {}, pb[S - LJ][NT] = {};
    auto h2 = [&]() {
#pragma unroll
        for (int j = LJ; j < S; ++j)
#pragma unroll
            for (int i = 0; i < S && i + j < LEV; ++i)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[i + j][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(pa[i], pb[j - LJ][nt], acc[i + j][nt], 0, 0, 0);
    };

#pragma unroll
    for (int g = 0; g < GL; ++g) issue1(g, 0);
#pragma unroll
    for (int g = 0; g < GL; ++g) issue1(g, 1);
    for (int kt = 0; kt < NK; ++kt) {
        if (kt + 1 < NK)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#if KV_LAG_OPAQUE  // the lagging operands are in registers (wino88i32_gemm_lagt_kernel)
#pragma unroll
        for (int i = 0; i < NA; ++i) asm volatile("" : "+v"(pa[i]));
#pragma unroll
        for (int jb = 0; jb < S - LJ; ++jb)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(pb[jb][nt]));
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* buf = L0 + (kt % NBUF) * T::STAGE;
        i8x16_t a[S], b[NT];
#pragma unroll
        for (int i = 0; i < S; ++i) a[i] = *(const i8x16_t*)(buf + aoffd[i]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b[nt] = *(const i8x16_t*)(buf + boffd[nt][0]);
        if (kt > 0) h2();  // the previous stage's lagging half, under the reads above
        if (kt + 2 < NK) {
            issue1(0, kt + 2);
            issue1(1, kt + 2);
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {
            if (j > 0) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) b[nt] = *(const i8x16_t*)(buf + boffd[nt][j]);
            }
            if (j < LJ) {
#pragma unroll
                for (int i = 0; i < S && i + j < LEV; ++i)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[i + j][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[nt], acc[i + j][nt], 0, 0, 0);
            } else {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) pb[j - LJ][nt] = b[nt];
            }
            if (j == 0 && kt + 2 < NK) {
#pragma unroll
                for (int g = 2; g < GL; ++g) issue1(g, kt + 2);
            }
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) pa[i] = a[i];
    }
    h2();

    // epilogue (as wino88i_gemm_kernel's): D col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int* evx = ev + (size_t)xi * stride + r_base + wm * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = n_base + wn * NT * 32 + nt * 32 + lr;
        const int ec = eu[(size_t)xi * cout + col] - 14;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            constexpr double w = RB == 8 ? 0.00390625 : 0.0078125;  // 2^-RB (radix 128: every step exact)
            double m = (double)acc[LEV - 1][nt][r];
#pragma unroll
            for (int l = LEV - 2; l >= 0; --l) m = __builtin_fma(m, w, (double)acc[l][nt][r]);
            M[((size_t)xi * stride + r_base + wm * 32 + row) * cout + col] = ldexp(m, evx[row] + ec);
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

template <bool RESID>
__global__ __launch_bounds__(256) void wino88i_outmax_kernel(const double* __restrict__ M, int rows,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, const float* resid,
                                                             float* Y, unsigned* __restrict__ evmax) {
    __shared__ __attribute__((aligned(16))) unsigned red[4][2][5][16];
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
        unsigned m[10];
#pragma unroll
        for (int bb = 0; bb < 10; ++bb)
            m[bb] = i8_half_max_dpp((unsigned)(__double_as_longlong(o[bb]) >> 32) & 0x7fffffffu);
        if ((lane & 31) == 16) {  // this half's 10 maxima (high words), written by one lane
            uint4* rr = (uint4*)&red[w][h][aa][0];
            rr[0] = make_uint4(m[0], m[1], m[2], m[3]);
            rr[1] = make_uint4(m[4], m[5], m[6], m[7]);
            *(uint2*)&red[w][h][aa][8] = make_uint2(m[8], m[9]);
        }
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
// R8 (KV_PATH_WINO88_I8R): 4 radix-256 digit planes (i8_digits_r8) instead of 5 radix-128 ones.
template <bool R8 = false>
__global__ __launch_bounds__(256) void wino88i_in_kernel(const float* __restrict__ X, int rows,
                                                         const unsigned* __restrict__ evmax,
                                                         int8_t* __restrict__ V8n, int* __restrict__ ex) {
    constexpr int C = 512, D = R8 ? 4 : kI8Digits;
    __shared__ int exs[4][100];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int kc = blockIdx.x, c = kc * 32 + (lane & 31), b = blockIdx.y * 4 + w;
    for (int i = threadIdx.x; i < 400; i += 256) {
        const int bw = i / 100, xi = i % 100, bb = blockIdx.y * 4 + bw;
        const unsigned m = evmax[(size_t)xi * rows + bb];
        const int e = R8 ? i8_row_exponent_r8(m) : i8_row_exponent(m);
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
    // 32-bit byte offsets (the digit planes of 100 x rows x 512 values, 5 digits: < 2^32 bytes): one base
    // register + a 32-bit offset per store
    const unsigned off0 = ((unsigned)kc * D * rows + b) * 32 + (lane & 31);
    const unsigned dstride = (unsigned)rows * 32, xstride = (C / 32) * D * dstride;
    // (one byte store per digit: a lane-quad transpose into dword stores measured 3 % slower here,
    // profiles/r05_i8x5_ab.log -- the kernel is bound by its fp64 transform and digit arithmetic; the digits
    // by magic-number adds: profiles/r05_i8x5_magic_ab.log; non-temporal byte stores -- 32-byte pieces of
    // lines -- made the forward 28 % slower: profiles/r05_i8x5_nt_ab.log)
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        double o[10];
        wino88d_input_row(t2, h, aa, o);
        const int a = 5 * h + aa;
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) {
            const int xi = a * 10 + bb;
            unsigned dg[D];
            if constexpr (R8) {
                const unsigned P = i8_digits_r8(o[bb], exs[w][xi]);
#pragma unroll
                for (int d = 0; d < D; ++d) dg[d] = P >> (8 * (D - 1 - d));
            } else {
                i8_digits_magic<D>(o[bb], exs[w][xi], dg);
            }
#pragma unroll
            for (int d = 0; d < D; ++d) V8n[off0 + (unsigned)xi * xstride + (unsigned)d * dstride] = (int8_t)dg[d];
        }
    }
}

// ---- the fp32 tower's GEMM on 4 int8 digits, round 5 (wino88i32_gemm_kernel) ----
// The same products as wino88i_gemm_kernel<K, 4, ., float, true> -- exact int32 levels, one rounding to fp32 --
// with four changes, none of which changes a bit of M:
//  * operands swapped: A = U (32 output channels per wave), B = V (2 x 32 boards), so the accumulator's 4
//    consecutive registers are 4 consecutive output channels of one board and the epilogue writes M with
//    16-byte stores (8 per wave instead of 32 dword stores);
//  * the level combine in integers first: H = 128 L0 + L1 and L = 128 L2 + L3 are exact in int32 (|L0| <=
//    K 127^2 < 2^23, |L1| <= 2 K 127 64, |L2| <= K (2 127 64 + 64^2), |L3| <= K (2 127 64 + 2 64^2), all at
//    K = 512), then m = 2^14 H + L in fp64 (< 2^46: exact) -- the same value as the fp64 chain
//    L0 + L1/128 + L2/128^2 + L3/128^3 times 2^21, so the same fp32 after ldexp and the one rounding;
//  * persistent workgroups: one per CU, each walking a contiguous run of its XCD's share of the tile order
//    (the XCD-aware order of wino88i_gemm_kernel), with the copy ring running across tiles -- the next tile's
//    first stages are in flight during this tile's last stages and its epilogue;
//  * the row exponents of a tile (128 of V, 128 of U) come into LDS by one more global_load_lds piece with
//    the tile's first stage and are read into registers after that stage's barrier (an ordinary load's
//    first use, or an LDS read in the epilogue, makes hipcc wait vmcnt(0) on the ring).
// KS: k per stage (32 or 64: one barrier per KS), NBUF: ring buffers (prefetch distance NBUF - 1).
template <int KS, int NBUF>
struct I8G32 {
    static constexpr int THREADS = 512, WM = 128, WN = 128;  // WM output channels x WN boards
    static constexpr int NCH = KS / 32;                      // 32-k chunks per stage
    static constexpr int CHB = 128 * 128;                    // one operand's chunk: 128 rows x 128-B lines
    static constexpr int STAGE = 2 * NCH * CHB;              // [op U, V][chunk][row][128 B]
    static constexpr int GL = STAGE / 1024 / (THREADS / 64); // global_load_lds pieces per wave and stage
    static constexpr int EXP = NBUF * STAGE;                 // 2 x 2 KiB of exponents (tile parity)
    static constexpr size_t BYTES = (size_t)NBUF * STAGE + 4096;
    static constexpr int NS = 8;                             // epilogue stores per wave
};

// NSEG: V's exponents per 256-channel segment (K / 256 of them, ev[(xi * NSEG + seg)][row]: the output
// kernel that writes V sees 256 channels of a board) instead of per row (1). Each segment's levels are
// combined exactly (2^14 H + L, fp64) and scaled by its exponent; the segments' scaled values add in fp64 in
// segment order (one fp64 rounding, 2^-53: deterministic, so still batch-invariant), then the one rounding to
// fp32. NSEG = 1 is bit-identical to wino88i_gemm_kernel.
// ABL (timing ablations of kv_dev_i8gemm_bench only; M is wrong): 1 no M stores (the values kept live),
// 2 no operand copies (the waits and barriers stay; LDS holds whatever it held).
// DEFER: a tile's 8 M stores per wave wait in registers until the next tile's first stage has issued its
// copies, so no vmcnt wait of the next tile's first PD + 1 stages has to retire them (the stores are older
// than every copy such a wait needs otherwise; vmcnt counts in issue order).
template <int K, int KS, int NBUF, int NSEG = 1, int ABL = 0, bool DEFER = false>
__global__ __launch_bounds__(512) void wino88i32_gemm_kernel(const int8_t* __restrict__ V8,
                                                             const int* __restrict__ ev,
                                                             const int8_t* __restrict__ U8,
                                                             const int* __restrict__ eu, float* __restrict__ M,
                                                             int rows, int stride) {
    using T = I8G32<KS, NBUF>;
    constexpr int NK = K / KS, NCH = T::NCH, GL = T::GL, PD = NBUF - 1;
    static_assert(GL * 8 * 1024 == T::STAGE && GL % 4 == 0, "stage split");
    static_assert(NSEG == 1 || (NSEG == 2 && K == 512 && NK % 2 == 0), "256-channel segments");
    constexpr int NEP = NSEG == 1 ? 1 : 2;  // exponent pieces per tile (items of 128 ints: ev segs, eu)
    extern __shared__ __attribute__((aligned(16))) i8x16_t lds_i8g[];
    char* const L0 = (char*)lds_i8g;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;  // 32 output channels, 64 boards
    const int RT = rows / T::WN, CT = 512 / T::WM;
    const int ntiles = kv::W88_XI * RT * CT;
    // this workgroup's tiles: XCD group x = blockIdx % 8 owns [x T8, (x + 1) T8) of the tile order; its P
    // workgroups take every P-th tile of that run (gridDim = ntiles: one tile each, the plain XCD order)
    const int T8 = ntiles >> 3, P = (int)gridDim.x >> 3;
    const int tfirst = (int)(blockIdx.x & 7) * T8 + (int)(blockIdx.x >> 3);
    const int tend = (int)(blockIdx.x & 7) * T8 + T8;
    const int ntile_wg = tfirst < tend ? (tend - tfirst + P - 1) / P : 0;
    const int nstage = ntile_wg * NK;

    // piece q = wave * GL + g: operand q / (16 NCH) (U: waves 0-3, V: waves 4-7), chunk (q / 16) % NCH,
    // rows 8 (q % 16) .. +7; lane l fills position l & 7 of LDS row 8 (q % 16) + l / 8 from source chunk
    // (l & 7) ^ (row >> 1 & 7) (the row-line image of wino88i_gemm_kernel)
    const int op = wave >> 2;
    const int rl_off0 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4));
    const int rl_off1 = (lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 4) ^ 4);
    const size_t cstride = (size_t)(op ? stride : 512) * 128;  // the next 32-k chunk of an operand
    auto tile_of = [&](int n, int& xi, int& n_base, int& r_base) {  // n-th tile of this workgroup
        const int idx = tfirst + n * P;
        xi = idx / (CT * RT);
        n_base = (idx % CT) * T::WM;
        r_base = ((idx / CT) % RT) * T::WN;
    };
    // a tile's operand base (this wave's operand) and exponent-piece sources: item i of the exponent slot
    // (128 ints at byte 512 i) is ev of segment i for i < NSEG, then eu (repeated to fill the last piece);
    // piece p carries items 2p (lanes 0-31) and 2p + 1 (lanes 32-63)
    auto tile_base = [&](int n, const int8_t*& gb, const int* (&es)[NEP]) {
        int xi, n_base, r_base;
        tile_of(n, xi, n_base, r_base);
        gb = op ? V8 + (((size_t)xi * (K / 32)) * stride + r_base) * 128
                : U8 + (((size_t)xi * (K / 32)) * 512 + n_base) * 128;
#pragma unroll
        for (int p = 0; p < NEP; ++p) {
            const int item = 2 * p + (lane >> 5);
            const bool isv = item < NSEG;
            es[p] = (isv ? ev : eu) + (isv ? ((size_t)xi * NSEG + item) * stride + r_base
                                           : (size_t)xi * 512 + n_base) + 4 * (lane & 31);
        }
    };
    // pieces g0 .. g1 - 1 of stage kt of the tile at gb (exponents first when ex != nullptr), into buffer buf
    auto issue = [&](const int8_t* gb, int kt, int buf, int g0, int g1) {
        if (ABL == 2) return;
        const int8_t* gk = gb + (size_t)(kt * NCH) * cstride;
#pragma unroll
        for (int g = g0; g < g1; ++g) {
            const int q = wave * GL + g, rg8 = q % 16, ch = (q / 16) % NCH;
            __builtin_amdgcn_global_load_lds(
                (const void*)(gk + (size_t)ch * cstride + (size_t)rg8 * 1024 + ((rg8 & 1) ? rl_off1 : rl_off0)),
                (__attribute__((address_space(3))) void*)(L0 + buf * T::STAGE + (op * NCH + ch) * T::CHB +
                                                          rg8 * 1024),
                16, 0, 0);
        }
    };
    auto issue_exp = [&](const int* const* es, int n) {
#pragma unroll
        for (int p = 0; p < NEP; ++p)
            __builtin_amdgcn_global_load_lds(
                (const void*)es[p], (__attribute__((address_space(3))) void*)(L0 + T::EXP + (n & 1) * 2048 + p * 1024),
                16, 0, 0);
    };

    // fragments: A = U digit i of channel row wm * 32 + (lane & 31), B = V digit j of board row
    // wn * 64 + nt * 32 + (lane & 31); the 16-byte chunk 2 i + (lane >> 5) of the row's line
    const int lr = lane & 31, lh = lane >> 5;
    int aoff[4], boff[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        aoff[i] = i8_rl_off(wm * 32 + lr, 2 * i + lh);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) boff[nt][i] = NCH * T::CHB + i8_rl_off(wn * 64 + nt * 32 + lr, 2 * i + lh);
    }

    const int8_t *gb_cur = nullptr, *gb_nxt = nullptr;
    const int *es_cur[NEP] = {}, *es_nxt[NEP] = {};
    if (ntile_wg > 0) {
        tile_base(0, gb_cur, es_cur);
        if (wave == 0) issue_exp(es_cur, 0);
        for (int k = 0; k < PD && k < NK; ++k) issue(gb_cur, k, k % NBUF, 0, GL);
    }
    int s = 0, bcur = 0, bpre = PD % NBUF;  // ring buffers of stage s and of stage s + PD
    float4 pend[2][4];  // DEFER: the previous tile's M rows
    float* prow[2] = {nullptr, nullptr};
    auto store_pend = [&]() {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int k = 0; k < 4; ++k) *(float4*)(prow[nt] + 8 * k) = pend[nt][k];
    };
    for (int n = 0; n < ntile_wg; ++n) {
        if (n + 1 < ntile_wg) tile_base(n + 1, gb_nxt, es_nxt);
        i32x16_t acc[4][2];
#pragma unroll
        for (int l = 0; l < 4; ++l)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[l][nt] = i32x16_t{};
        int evr[NSEG][2];  // ev - 35 of the wave's two 32-board blocks (this lane's board), per segment
        int euv[4][4];     // eu of this lane's 16 output channels
        double sacc[NSEG == 2 ? 2 : 1][NSEG == 2 ? 16 : 1];  // segment 0, scaled (NSEG 2)
        for (int kt = 0; kt < NK; ++kt, ++s, bcur = bcur + 1 == NBUF ? 0 : bcur + 1,
                                     bpre = bpre + 1 == NBUF ? 0 : bpre + 1) {
            // stage s has landed once only the batches issued after it may be outstanding: the next PD - 1
            // stages' (those that exist) and, in a tile's first PD stages after an epilogue, its NS stores
            const int ahead = nstage - 1 - s < PD - 1 ? nstage - 1 - s : PD - 1;
            const bool st = DEFER ? (n > 0 && kt >= 1 && kt <= PD) : (n > 0 && kt < PD);
            if (PD == 2) {
                if (ahead == 1) {
                    if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL + T::NS) : "memory");
                    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
                } else {
                    if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::NS) : "memory");
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            } else {  // PD == 3
                if (ahead == 2) {
                    if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL + T::NS) : "memory");
                    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL) : "memory");
                } else if (ahead == 1) {
                    if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL + T::NS) : "memory");
                    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
                } else {
                    if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::NS) : "memory");
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (kt == 0) {  // the tile's exponents landed with its first stage: ev of the 2 boards, eu of 16 channels
                const int* ex = (const int*)(L0 + T::EXP + (n & 1) * 2048);
#pragma unroll
                for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt) evr[sg][nt] = ex[sg * 128 + wn * 64 + nt * 32 + lr] - 35;
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) euv[k][jj] = ex[NSEG * 128 + wm * 32 + 8 * k + 4 * lh + jj];
            }
            const char* buf = L0 + bcur * T::STAGE;
            const bool more = s + PD < nstage;
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                const char* cb = buf + ch * T::CHB;
                i8x16_t a[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = *(const i8x16_t*)(cb + aoff[i]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    i8x16_t b[2];
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt) b[nt] = *(const i8x16_t*)(cb + boff[nt][j]);
#pragma unroll
                    for (int i = 0; i + j < 4; ++i)
#pragma unroll
                        for (int nt = 0; nt < 2; ++nt)
                            acc[i + j][nt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[nt], acc[i + j][nt], 0, 0, 0);
                    // stage s + PD's copies (this tile's or the next one's), one group per (chunk, B digit)
                    // between the MFMA groups; the next tile's exponents ahead of its first stage
                    if (more) {
                        constexpr int PER = GL / (4 * NCH);
                        const int g0 = (ch * 4 + j) * PER;
                        const bool nx = kt + PD >= NK;
                        if (nx && kt + PD == NK && g0 == 0 && wave == 0) issue_exp(es_nxt, n + 1);
                        issue(nx ? gb_nxt : gb_cur, nx ? kt + PD - NK : kt + PD, bpre, g0, g0 + PER);
                    }
                }
            }
            if (DEFER && kt == 0 && n > 0) store_pend();  // after this stage's copies (stage s + PD's)
            if constexpr (NSEG == 2) {
              if (kt == NK / 2 - 1) {  // segment 0 done: its exact value, scaled, then restart
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    const double sc = ldexp(1.0, evr[0][nt]);
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int hi = acc[0][nt][r] * 128 + acc[1][nt][r];
                        const int lo = acc[2][nt][r] * 128 + acc[3][nt][r];
                        sacc[nt][r] = __builtin_fma((double)hi, 16384.0, (double)lo) * sc;  // exact
                    }
#pragma unroll
                    for (int l = 0; l < 4; ++l) acc[l][nt] = i32x16_t{};
                }
              }
            }
        }
        // epilogue (registers only; the ring keeps loading the next tile)
        int xi, n_base, r_base;
        tile_of(n, xi, n_base, r_base);
        gb_cur = gb_nxt;
#pragma unroll
        for (int p = 0; p < NEP; ++p) es_cur[p] = es_nxt[p];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int bl = wn * 64 + nt * 32 + lr;
            const int eb = evr[NSEG - 1][nt];
            const double sc1 = ldexp(1.0, eb);
            float* mrow = M + ((size_t)xi * stride + r_base + bl) * 512 + n_base + wm * 32 + 4 * lh;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float o[4];
                const int* ec = euv[k];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int r = 4 * k + jj;
                    const int hi = acc[0][nt][r] * 128 + acc[1][nt][r];
                    const int lo = acc[2][nt][r] * 128 + acc[3][nt][r];
                    const double m = __builtin_fma((double)hi, 16384.0, (double)lo);  // exact
                    if constexpr (NSEG == 2)  // segment 1 scaled (exact) plus segment 0: one fp64 rounding
                        o[jj] = (float)ldexp(__builtin_fma(m, sc1, sacc[nt][r]), ec[jj]);
                    else
                        o[jj] = (float)ldexp(m, eb + ec[jj]);
                }
                if (ABL == 1)
                    asm volatile("" ::"v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]));
                else if (DEFER)
                    pend[nt][k] = make_float4(o[0], o[1], o[2], o[3]);
                else
                    *(float4*)(mrow + 8 * k) = make_float4(o[0], o[1], o[2], o[3]);
            }
            if (DEFER) prow[nt] = mrow;
        }
    }
    if (DEFER && ntile_wg > 0) store_pend();
}

// ---- the fp32 Winograd domain with int8-digit GEMMs (KV_PATH_WINO88_I8F32) ----
// The fp32 F(8x8) tower's arithmetic (kv_wino88.h: fp32 transforms, V, M and activations; U as
// 4 digits of the fp64 U) with each GEMM taken from 4 int8 digits per value: per-row 28-bit block
// fixed point (each value cut to the multiples of 2^(e-29) of its row's exponent e), the 10 digit pairs
// i + j <= 3 of the 16, exact int32 levels, combined exactly and rounded to fp32 once -- where the fp32
// MFMA GEMM rounds after every product. An fp32 value within 2^-4 of its row's max keeps all its bits; one
// 2^-k below keeps 28 - k (the bound test: tests/test_wino_i8_gpu.py). 10 int8 MFMAs per point product against one fp32 one at
// 1/32 the rate.

// wino88i32_out_kernel: the fp32 tower's output transform + BN (+ residual) + ReLU -> Y (optional), then
// the next conv's V as row-line digits under each row's exponent -- what wino88_out_kernel's fp32 V
// followed by wino88i_slice_kernel<512, float, 4, true> gives, bit for bit, without V's HBM round trip.
// One 512-thread workgroup per board, thread = channel, so the 512 channels of a row (the exponent's
// domain) are in one workgroup. Each (board, channel) plane is split over lanes l and l ^ 32 (the
// transforms' half exchanges are v_permlane32_swap), so a lane keeps its 50 V values in registers across
// the exponent barrier: the row maxima (DPP max per half-wave, then LDS over the waves), the exponents, then
// the digits of the kept values -- the same fmaf chains on the same inputs as wino88_out_kernel + the slice
// kernel, so the same bits. A thread's 4 digits of a point go through a 4x4 byte transpose within its lane
// quad (two DPP exchanges + v_perm), so every lane stores one dword and each half-wave writes one whole
// 128-byte line.
// (Round 4 dropped a form that kept all 100 V values in registers for the reduction: 246 VGPRs, one
// workgroup per CU, 436-511 us per layer against 142-238 + 165 us for the out kernel + slice,
// profiles/r04_i8f32_fused_out.log; and an output kernel computing only the row maxima plus a second
// input-transform pass, 294-356 + 220 us, profiles/r04_i8f32_outmax_form.log.)

// fp32 transform row 5h + aa of a plane split over lanes l, l ^ 32 (half h), from the half's 4 columns after the
// half exchange (xc[kk][i] = pixel (i, 4h + kk)): the fmaf chains of wino88_input_cols + wino88_input_row on the
// same inputs -- each column's w88_bt taken for rows aa and 5 + aa only -- so the same bits, and no 10x4
// intermediate is live. The asm makes xc opaque per row: otherwise the compiler merges the two passes of
// wino88i32_out2_kernel (the same chains on the same values) and keeps the 50 results across the barrier.
__device__ inline void wino88_input_row_of_cols(float (&xc)[4][8], int aa, float (&o)[10]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(xc[kk][i]));
    float row[10];
    row[0] = 0.f;
    row[9] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        float col[10], t[10];
        col[0] = 0.f;
        col[9] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) col[1 + i] = xc[kk][i];
        w88_bt(col, t);
        float lo = t[aa], hi = t[5 + aa];
        half_swap(lo, hi);
        row[1 + kk] = lo;
        row[5 + kk] = hi;
    }
    w88_bt(row, o);
}

// Row-line width: 4 digit slots (128 bytes) per 32-channel chunk, or R3's 3 (96 bytes: no zero slot in memory)
template <bool R3>
constexpr unsigned kI8LineBytes = R3 ? 96u : 128u;
// The board an output workgroup handles. R3's 96-byte lines of boards 4g .. 4g+3 share 128-byte lines (4 x 96 =
// 3 x 128), so those 4 boards go to one XCD (workgroups are dealt to the 8 XCDs round-robin: id mod 8), whose L2
// merges their partial lines; dealt board by board, each shared line took partial writes from two XCDs. A
// bijection on [0, nb) for nb a multiple of 32.
template <bool R3>
__device__ inline int out_board(int id) {
    if constexpr (!R3) return id;
    const int x = id & 7, s = id >> 3;
    return 4 * (x + 8 * (s >> 2)) + (s & 3);
}

// R3 (KV_PATH_WINO88_I8F32R3): the next V's 3 radix-256 digits (i8_digits_r3 under i8_row_exponent_f32r) in
// the same lines, slot 3 zero
template <bool R3>
__device__ inline int i8f32_row_exponent(unsigned m) {
    return R3 ? i8_row_exponent_f32r(m) : i8_row_exponent_f32(m);
}
template <bool R3>
__device__ inline unsigned i8f32_digits(float v, int e) {
    if constexpr (R3)
        return i8_digits_r3((double)v, e);
    else
        return i8_digits4_packed(v, e);
}

// Phase stagger of the one-board-per-workgroup output kernels: every board runs load M -> transforms -> store
// digits, and boards that start together on every CU put the whole chip in the same phase (HBM saturated in the
// load and store phases, idle in the transforms). The first-round workgroups of half the CUs (first: the
// resident workgroup count; (b >> 3) & 1 picks half the workgroups of each XCD) wait `stag` x 8,128 cycles
// before starting, and the slots they occupy keep that offset for the rest of the grid. Timing only: no
// output depends on it.
__device__ inline void out_stagger(int b, int stag, int first) {
    if (b < first && ((b >> 3) & 1))
        for (int i = 0; i < stag; ++i) __builtin_amdgcn_s_sleep(127);
}

// wino88i32_out2_kernel: wino88i32_out_kernel<RESID, WRITE_Y, 512>'s result, bit for bit, in a register budget
// that lets two boards (two 1,024-thread workgroups) share a CU, so one board's digit stores drain under the
// other's transforms: a lane keeps its 32 fp32 activations (xc) across the exponent barrier instead of 50 V
// values and runs the input transform twice -- once for the row maxima, once for the digits. The transform is
// partitioned by row, not repeated within a pass (each pass computes each V value once), so the VALU work is
// twice the held form's input transform; at 8 waves per SIMD that is ~20 us of issue over 2,048 boards.
template <bool RESID, bool WRITE_Y, bool R3 = false>
__global__ __launch_bounds__(1024, 8) void wino88i32_out2_kernel(const float* __restrict__ M, int rows,
                                                                 const float* __restrict__ scale,
                                                                 const float* __restrict__ shift, const float* resid,
                                                                 float* Y, int8_t* __restrict__ V8,
                                                                 int* __restrict__ ex, int stag, int first) {
#pragma clang fp contract(off)
    constexpr int NK = 512 / 32, NW = 16;
    __shared__ __attribute__((aligned(16))) unsigned red[NW][2][5][16];
    __shared__ int exs[100];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int c = w * 32 + (lane & 31), b = out_board<R3>((int)blockIdx.y);
    out_stagger(b, stag, first);
    float xc[4][8];  // the half's columns 4h .. 4h+3, all 8 rows (after the half exchange)
    {
        float x2[4][8];
        wino88_out_plane_half<RESID, WRITE_Y, true>(M, rows, b, c, h, scale[c], shift[c], resid, Y, x2);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) {
                float lo = x2[ii][kk], hi = x2[ii][4 + kk];
                half_swap(lo, hi);
                xc[kk][ii] = lo;
                xc[kk][4 + ii] = hi;
            }
    }
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        float o[10];
        wino88_input_row_of_cols(xc, aa, o);
        unsigned m[10];
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) m[bb] = i8_half_max_dpp(__float_as_uint(o[bb]) & 0x7fffffffu);
        if ((lane & 31) == 16) {  // this half's 10 maxima, written by one lane
            uint4* rr = (uint4*)&red[w][h][aa][0];
            rr[0] = make_uint4(m[0], m[1], m[2], m[3]);
            rr[1] = make_uint4(m[4], m[5], m[6], m[7]);
            *(uint2*)&red[w][h][aa][8] = make_uint2(m[8], m[9]);
        }
    }
    __syncthreads();
    if (threadIdx.x < 100) {
        const int xi = threadIdx.x, a = xi / 10, bb = xi % 10, hh = a / 5, aa = a % 5;
        unsigned m = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) m = red[ww][hh][aa][bb] > m ? red[ww][hh][aa][bb] : m;
        const int e = i8f32_row_exponent<R3>(m);
        exs[xi] = e;
        ex[(size_t)xi * rows + b] = e;
    }
    __syncthreads();
    const int q = lane & 3;
    const unsigned off0 = ((unsigned)(c >> 5) * rows + b) * kI8LineBytes<R3> + q * 32 + (c & 28),
                   xstride = NK * rows * kI8LineBytes<R3>;
    unsigned* const dst = (unsigned*)V8;
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        float o[10];
        wino88_input_row_of_cols(xc, aa, o);
        const int a = 5 * h + aa;
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) {
            const int xi = a * 10 + bb;
            const unsigned P = i8f32_digits<R3>(o[bb], exs[xi]);
            {
                const unsigned T4 = i8_quad_transpose(P, lane);  // lane q of the quad: digit q's 4 channels
                if constexpr (!R3)
                    __builtin_nontemporal_store(T4, &dst[(off0 + (unsigned)xi * xstride) >> 2]);
                else if (q < 3)  // R3's 96-byte lines share 128-byte lines: ordinary stores, merged in L2
                    dst[(off0 + (unsigned)xi * xstride) >> 2] = T4;
            }
        }
    }
}

// STAMP (a diagnostic build, never the product's; kv_dev_out_phases): waves 0 and 15 record the shader clock at the
// kernel's phase boundaries into kOutStamps[board][wave 0/15][8] -- a buffer no other code reads: start, V ready
// (M loaded, both transforms done), after the maxima barrier, after the exponent barrier, digit stores issued,
// stores drained.
constexpr int kOutStampBoards = 4096;
__device__ unsigned long long kOutStamps[kOutStampBoards][2][8];

template <bool RESID, bool WRITE_Y, int CW, bool R3 = false, bool STAMP = false, int ABL = 0, bool YNT = false>
__global__ __launch_bounds__(2 * CW) void wino88i32_out_kernel(const float* __restrict__ M, int rows,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, const float* resid,
                                                               float* Y, int8_t* __restrict__ V8,
                                                               int* __restrict__ ex, int stag, int first) {
#pragma clang fp contract(off)
    static_assert(CW == 512 || CW == 256, "a row or a 256-channel segment per workgroup");
    constexpr int NK = 512 / 32, NW = CW / 32, NSEG = 512 / CW;
    __shared__ __attribute__((aligned(16))) unsigned red[NW][2][5][16];
    __shared__ int exs[100];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int seg = blockIdx.x, c = seg * CW + w * 32 + (lane & 31), b = out_board<R3>((int)blockIdx.y);
    out_stagger(b, stag, first);
    unsigned long long st[6] = {};
    const bool stamper = STAMP && (w == 0 || w == NW - 1) && lane == 0 && b < kOutStampBoards;
    if constexpr (STAMP) st[0] = __builtin_amdgcn_s_memtime();
    float vk[5][10];  // this half's 50 V values (rows 5h .. 5h+4), kept across the exponent barrier
    {
        float t2[10][4];  // B10^T of the plane's columns 4h .. 4h+3
        {
            float x2[4][8];
            wino88_out_plane_half<RESID, WRITE_Y, false, ABL, YNT>(M, rows, b, c, h, scale[c], shift[c], resid, Y, x2);
            wino88_input_cols(x2, h, t2);
        }
#pragma unroll
        for (int aa = 0; aa < 5; ++aa) wino88_input_row(t2, h, aa, vk[aa]);
    }
    if constexpr (STAMP) {  // V ready: the transforms' results are consumed by an opaque use first
#pragma unroll
        for (int aa = 0; aa < 5; ++aa)
#pragma unroll
            for (int bb = 0; bb < 10; ++bb) asm volatile("" ::"v"(vk[aa][bb]));
        st[1] = __builtin_amdgcn_s_memtime();
    }
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        const float (&o)[10] = vk[aa];
        unsigned m[10];
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) m[bb] = i8_half_max_dpp(__float_as_uint(o[bb]) & 0x7fffffffu);
        if ((lane & 31) == 16) {  // this half's 10 maxima, written by one lane
            uint4* rr = (uint4*)&red[w][h][aa][0];
            rr[0] = make_uint4(m[0], m[1], m[2], m[3]);
            rr[1] = make_uint4(m[4], m[5], m[6], m[7]);
            *(uint2*)&red[w][h][aa][8] = make_uint2(m[8], m[9]);
        }
    }
    __syncthreads();
    if constexpr (STAMP) st[2] = __builtin_amdgcn_s_memtime();
    if (threadIdx.x < 100) {
        const int xi = threadIdx.x, a = xi / 10, bb = xi % 10, hh = a / 5, aa = a % 5;
        unsigned m = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) m = red[ww][hh][aa][bb] > m ? red[ww][hh][aa][bb] : m;
        const int e = i8f32_row_exponent<R3>(m);
        exs[xi] = e;
        ex[((size_t)xi * NSEG + seg) * rows + b] = e;
    }
    __syncthreads();
    if constexpr (STAMP) st[3] = __builtin_amdgcn_s_memtime();
    // row line (xi, kc = c / 32, b): 128 bytes, digit d of channel 32 kc + i at byte 32 d + i
    const int q = lane & 3;
    // 32-bit byte offsets (the digits of 100 x rows x 512 values < 2^32 bytes)
    const unsigned off0 = ((unsigned)(c >> 5) * rows + b) * kI8LineBytes<R3> + q * 32 + (c & 28),
                   xstride = NK * rows * kI8LineBytes<R3>;
    unsigned* const dst = (unsigned*)V8;
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        const int a = 5 * h + aa;
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) {
            const int xi = a * 10 + bb;
            const unsigned P = i8f32_digits<R3>(vk[aa][bb], exs[xi]);
            // non-temporal: the digits are read once, by the next GEMM (forward -1.2 % at 2,048 boards against
            // plain stores, bit-identical; the GEMM's M stored non-temporal instead slowed the output kernel that
            // reads it: profiles/r05_out_nt_ab.log)
            {
                const unsigned T4 = i8_quad_transpose(P, lane);  // lane q of the quad: digit q's 4 channels
                if constexpr (!R3)
                    __builtin_nontemporal_store(T4, &dst[(off0 + (unsigned)xi * xstride) >> 2]);
                else if (q < 3)  // R3's 96-byte lines share 128-byte lines: ordinary stores, merged in L2
                    dst[(off0 + (unsigned)xi * xstride) >> 2] = T4;
            }
        }
    }
    if constexpr (STAMP) {
        st[4] = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st[5] = __builtin_amdgcn_s_memtime();
        if (stamper) {
            unsigned long long* o = kOutStamps[b][w == 0 ? 0 : 1];
#pragma unroll
            for (int k = 0; k < 6; ++k) o[k] = st[k];
        }
    }
}

// wino88i32_outp_kernel: wino88i32_out_kernel<RESID, WRITE_Y, 512, R3>'s result, bit for bit, as a persistent
// kernel that streams M through LDS by DMA. One 1,024-thread workgroup per CU loops over its boards (blockIdx.x,
// + gridDim.x, ...); a board's output transform runs in 5 column steps, step jj reading M's points i*10 + jj and
// i*10 + 5 + jj (the two plane halves' columns, 20 points x 512 channels = 40 KiB: a "slot"). Slots are copied
// global -> LDS by global_load_lds_dwordx4 (1 KiB per wave-instruction, 40 per slot, dealt over the 16 waves)
// into a ring of 3 LDS buffers, two steps ahead -- across the board boundary, so the next board's first two
// slots land while this board reduces its row maxima and stores its digits. The M loads then hold no VGPRs (the
// held kernel keeps 50 loads per lane in flight at the board's start, the 64-register one only 10), and a board's
// load latency hides under its predecessor's back half. Same fmaf chains on the same values as the held kernel.
// Waits: before step t the wave waits for its own pieces of slot t (vmcnt = its pieces of slot t + 1, the only
// VMEM issued since) and lgkmcnt(0) (its reads of slot t - 1, whose buffer slot t + 2's copies overwrite once
// every wave passes this barrier); the first two slots of a later board were drained by the vmcnt(0) before the
// previous board's digit stores.
template <bool RESID, bool WRITE_Y, bool R3 = false>
__global__ __launch_bounds__(1024) void wino88i32_outp_kernel(const float* __restrict__ M, int rows,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, const float* resid,
                                                              float* Y, int8_t* __restrict__ V8,
                                                              int* __restrict__ ex) {
#pragma clang fp contract(off)
    constexpr int NK = 512 / 32, NW = 16, NSLOT = 3, SLOT = 20 * 2048;
    extern __shared__ __attribute__((aligned(16))) char lds_outp[];  // NSLOT slots, then red, exs
    unsigned(*red)[2][5][16] = (unsigned(*)[2][5][16])(lds_outp + NSLOT * SLOT);
    int* exs = (int*)(lds_outp + NSLOT * SLOT + NW * 2 * 5 * 16 * 4);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int c = w * 32 + (lane & 31);
    const int G = (int)gridDim.x;
    const int nbw = ((int)rows - (int)blockIdx.x + G - 1) / G;  // boards of this workgroup
    const int nsteps = 5 * nbw;
    const int npieces = wu < 8 ? 3 : 2;  // this wave's pieces of a slot (40 = 16 + 16 + 8)
    const float sc = scale[c], sh = shift[c];
    const unsigned xs = (unsigned)rows * 512;
    // slot of step t: board blockIdx.x + (t / 5) G, column step t % 5; LDS row r = hh * 10 + i holds point
    // i * 10 + 5 hh + jj; piece q = row q / 2, channels 256 (q & 1) ..
    auto issue = [&](int t) {
        if (t >= nsteps) return;
        const int b = (int)blockIdx.x + (t / 5) * G, jj = t % 5;
        char* dst = lds_outp + (t % NSLOT) * SLOT;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int q = wu + 16 * k;
            if (q < 40) {
                const int r = q >> 1, hh = r / 10, i = r - 10 * hh;
                const float* src = M + (unsigned)(i * 10 + 5 * hh + jj) * xs + (unsigned)b * 512 + (q & 1) * 256 +
                                   lane * 4;
                __builtin_amdgcn_global_load_lds((const void*)src,
                                                 (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, 0, 0);
            }
        }
    };
    issue(0);
    issue(1);
    int t = 0;
    for (int k = 0; k < nbw; ++k) {
        const int b = (int)blockIdx.x + k * G;
        float tt[8][5];  // A8^T m of this half's columns 5h + jj
#pragma unroll
        for (int jj = 0; jj < 5; ++jj, ++t) {
            if (k > 0 && jj < 2) {  // drained before the previous board's digit stores
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else {
                const int younger = t + 1 < nsteps ? npieces : 0;  // slot t + 1's pieces, issued after slot t's
                if (younger == 3)
                    asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
                else if (younger == 2)
                    asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            issue(t + 2);  // into slot t - 1's buffer: every wave has read it (lgkmcnt(0) before this barrier)
            const float* sl = (const float*)(lds_outp + (t % NSLOT) * SLOT) + h * 10 * 512 + c;
            float col[10], o[8];
#pragma unroll
            for (int i = 0; i < 10; ++i) col[i] = sl[i * 512];
            w88_at(col, o);
#pragma unroll
            for (int i = 0; i < 8; ++i) tt[i][jj] = o[i];
        }
        // the row pass, BN (+ residual) + ReLU (+ Y) -- wino88_out_plane_half's
        float x2[4][8];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            float row[10];
#pragma unroll
            for (int jj = 0; jj < 5; ++jj) {
                float lo = tt[ii][jj], hi = tt[4 + ii][jj];
                half_swap(lo, hi);
                row[jj] = lo;
                row[5 + jj] = hi;
            }
            float o[8];
            w88_at(row, o);
            const int i = 4 * h + ii;
            float res[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) res[j] = RESID ? resid[((unsigned)b * 64 + i * 8 + j) * 512 + c] : 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = o[j] * sc + sh;
                if (RESID) v += res[j];
                v = v > 0.f ? v : 0.f;
                if (WRITE_Y) Y[((unsigned)b * 64 + i * 8 + j) * 512 + c] = v;
                x2[ii][j] = v;
            }
        }
        // the next V (held: 50 values per lane), its row maxima, exponents, digits -- wino88i32_out_kernel's
        float vk[5][10];
        {
            float t2[10][4];
            wino88_input_cols(x2, h, t2);
#pragma unroll
            for (int aa = 0; aa < 5; ++aa) wino88_input_row(t2, h, aa, vk[aa]);
        }
#pragma unroll
        for (int aa = 0; aa < 5; ++aa) {
            unsigned m[10];
#pragma unroll
            for (int bb = 0; bb < 10; ++bb) m[bb] = i8_half_max_dpp(__float_as_uint(vk[aa][bb]) & 0x7fffffffu);
            if ((lane & 31) == 16) {
                uint4* rr = (uint4*)&red[w][h][aa][0];
                rr[0] = make_uint4(m[0], m[1], m[2], m[3]);
                rr[1] = make_uint4(m[4], m[5], m[6], m[7]);
                *(uint2*)&red[w][h][aa][8] = make_uint2(m[8], m[9]);
            }
        }
        __syncthreads();
        if (threadIdx.x < 100) {
            const int xi = threadIdx.x, a = xi / 10, bb = xi % 10, hh = a / 5, aa = a % 5;
            unsigned m = 0;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) m = red[ww][hh][aa][bb] > m ? red[ww][hh][aa][bb] : m;
            const int e = i8f32_row_exponent<R3>(m);
            exs[xi] = e;
            ex[(size_t)xi * rows + b] = e;
        }
        __syncthreads();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next board's first two slots (and Y) landed
        const int q = lane & 3;
        const unsigned off0 = ((unsigned)(c >> 5) * rows + b) * kI8LineBytes<R3> + q * 32 + (c & 28),
                   xstride = NK * rows * kI8LineBytes<R3>;
        unsigned* const dst = (unsigned*)V8;
#pragma unroll
        for (int aa = 0; aa < 5; ++aa) {
            const int a = 5 * h + aa;
#pragma unroll
            for (int bb = 0; bb < 10; ++bb) {
                const int xi = a * 10 + bb;
                const unsigned P = i8f32_digits<R3>(vk[aa][bb], exs[xi]);
                {
                const unsigned T4 = i8_quad_transpose(P, lane);  // lane q of the quad: digit q's 4 channels
                if constexpr (!R3)
                    __builtin_nontemporal_store(T4, &dst[(off0 + (unsigned)xi * xstride) >> 2]);
                else if (q < 3)  // R3's 96-byte lines share 128-byte lines: ordinary stores, merged in L2
                    dst[(off0 + (unsigned)xi * xstride) >> 2] = T4;
            }
            }
        }
    }
}

constexpr int kOutpLds = 3 * 20 * 2048 + 16 * 2 * 5 * 16 * 4 + 100 * 4;  // wino88i32_outp_kernel's dynamic LDS

// ---- the fp32 tower with fp64 input transforms (KV_PATH_WINO88_I8F32V) ----
// The same tower as KV_PATH_WINO88_I8F32 (fp32 M, output transform and activations, the 4-digit GEMM)
// except that every conv's V is the fp64 input transform of its fp32 input, cut to 4 digits from fp64:
// on learn-loop weights the fp32 input transform is what sets the fp32 tower's value error
// (profiles/r05_learn_stage_emulate.log).

// Transform rows of the two halves at step aa: one +-p row pair of w88d_bt's even / odd form, (1, 2), (3, 4),
// (5, 6), (7, 8), or (0, 9) at aa = 0 -- half 0 takes the first, half 1 the second.
__device__ inline int w88v_row(int h, int aa) { return aa == 0 ? 9 * h : 2 * aa - 1 + h; }

// fp64 transform row w88v_row(h, aa) of a plane split over lanes l, l ^ 32, from the half's 4 columns after
// the half exchange (xc[kk][i] = pixel (i, 4h + kk)): the fma chains of wino88d_input_cols +
// wino88d_input_row on the same inputs -- so the same bits as wino88d_input_plane -- one transform row pair
// at a time (each column's w88d_bt is taken for that pair only, which shares its even / odd halves), so no
// 10x4 fp64 intermediate is live.
__device__ inline void wino88d_input_row_of_cols(float (&xc)[4][8], int aa, double (&o)[10]) {
    // opaque to the compiler per row: otherwise it keeps the 32 widened values (64 VGPRs) live across the
    // rows and both passes instead of widening them again, and spills
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(xc[kk][i]));
    double row[10];
    row[0] = 0.0;
    row[9] = 0.0;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        double col[10], t[10];
        col[0] = 0.0;
        col[9] = 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i) col[1 + i] = (double)xc[kk][i];
        w88d_bt(col, t);
        double lo = t[w88v_row(0, aa)], hi = t[w88v_row(1, aa)];
        half_swap(lo, hi);
        row[1 + kk] = lo;
        row[5 + kk] = hi;
    }
    w88d_bt(row, o);
}

// wino88i32v_out_kernel: wino88i32_out_kernel<RESID, WRITE_Y, 512> with the next conv's V taken as the fp64
// input transform of the fp32 activation (what wino88d_in_kernel + wino88i_slice_kernel<512, double, 4,
// true> give, bit for bit). 50 fp64 V values per lane do not fit beside the rest at 1,024 threads, so the
// lane keeps its 32 fp32 activations across the exponent barrier instead and transforms them twice: once
// for the row maxima (the high words of |V|), once for the digits (magic-number fp64 rint).
// wino88i64r_out_kernel (KV_PATH_WINO88_I8R): the same from an fp64 M with the fp64 output transform
// (wino88d_out_plane, as wino88d_out_half_kernel) and the 4 radix-256 digits (i8_digits_r8 under
// i8_row_exponent_r8) -- what wino88d_out_half_kernel's Y + wino88d_in_kernel + the radix-256 slice kernel
// give, bit for bit -- replacing the outmax + in kernel pair of the planes layout.
template <bool RESID, bool WRITE_Y, class MT>
__device__ inline void wino88v_out_body(const MT* __restrict__ M, int rows, const float* __restrict__ scale,
                                        const float* __restrict__ shift, const float* resid, float* Y,
                                        int8_t* __restrict__ V8, int* __restrict__ ex, int stag, int first) {
    constexpr bool R8 = sizeof(MT) == 8;
    constexpr int NK = 512 / 32, NW = 16;
    __shared__ __attribute__((aligned(16))) unsigned red[NW][2][5][16];
    __shared__ int exs[100];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const int c = w * 32 + (lane & 31), b = blockIdx.y;
    out_stagger(b, stag, first);
    float xc[4][8];  // the half's columns 4h .. 4h+3, all 8 rows (after the half exchange)
    {
        float x2[4][8];
        if constexpr (R8)
            wino88d_out_plane<RESID, WRITE_Y>(M, rows, b, c, h, (double)scale[c], (double)shift[c], resid, Y, x2);
        else
            wino88_out_plane_half<RESID, WRITE_Y>(M, rows, b, c, h, scale[c], shift[c], resid, Y, x2);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) {
                float lo = x2[ii][kk], hi = x2[ii][4 + kk];
                half_swap(lo, hi);
                xc[kk][ii] = lo;
                xc[kk][4 + ii] = hi;
            }
    }
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        double o[10];
        wino88d_input_row_of_cols(xc, aa, o);
        unsigned m[10];
#pragma unroll
        for (int bb = 0; bb < 10; ++bb)
            m[bb] = i8_half_max_dpp((unsigned)(__double_as_longlong(o[bb]) >> 32) & 0x7fffffffu);
        if ((lane & 31) == 16) {
            uint4* rr = (uint4*)&red[w][h][aa][0];
            rr[0] = make_uint4(m[0], m[1], m[2], m[3]);
            rr[1] = make_uint4(m[4], m[5], m[6], m[7]);
            *(uint2*)&red[w][h][aa][8] = make_uint2(m[8], m[9]);
        }
    }
    __syncthreads();
    if (threadIdx.x < 100) {  // point row a came from half hh at step aa (w88v_row)
        const int xi = threadIdx.x, a = xi / 10, bb = xi % 10;
        const int hh = a == 9 ? 1 : (a == 0 ? 0 : (a - 1) & 1), aa = (a == 0 || a == 9) ? 0 : (a + 1) >> 1;
        unsigned m = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) m = red[ww][hh][aa][bb] > m ? red[ww][hh][aa][bb] : m;
        const int e = R8 ? i8_row_exponent_r8(m) : i8_row_exponent(m);
        exs[xi] = e;
        ex[(size_t)xi * rows + b] = e;
    }
    __syncthreads();
    const int q = lane & 3;
    const unsigned off0 = ((unsigned)(c >> 5) * rows + b) * 128 + q * 32 + (c & 28), xstride = NK * rows * 128;
    unsigned* const dst = (unsigned*)V8;
#pragma unroll
    for (int aa = 0; aa < 5; ++aa) {
        double o[10];
        wino88d_input_row_of_cols(xc, aa, o);
        const int a = w88v_row(h, aa);
#pragma unroll
        for (int bb = 0; bb < 10; ++bb) {
            const int xi = a * 10 + bb;
            unsigned P;  // byte d = digit d (the most significant first)
            if constexpr (R8) {
                P = __builtin_bswap32(i8_digits_r8(o[bb], exs[xi]));
            } else {
                unsigned dq[4];
                i8_digits_magic<4>(o[bb], exs[xi], dq);
                P = __builtin_amdgcn_perm(dq[1], dq[0], 0x0c0c0400u) | __builtin_amdgcn_perm(dq[3], dq[2], 0x0c0c0400u) << 16;
            }
            __builtin_nontemporal_store(i8_quad_transpose(P, lane), &dst[(off0 + (unsigned)xi * xstride) >> 2]);
        }
    }
}

template <bool RESID, bool WRITE_Y>
__global__ __launch_bounds__(1024) void wino88i32v_out_kernel(const float* __restrict__ M, int rows,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, const float* resid,
                                                              float* Y, int8_t* __restrict__ V8, int* __restrict__ ex,
                                                              int stag, int first) {
    wino88v_out_body<RESID, WRITE_Y>(M, rows, scale, shift, resid, Y, V8, ex, stag, first);
}

template <bool RESID, bool WRITE_Y>
__global__ __launch_bounds__(1024) void wino88i64r_out_kernel(const double* __restrict__ M, int rows,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, const float* resid,
                                                              float* Y, int8_t* __restrict__ V8, int* __restrict__ ex,
                                                              int stag, int first) {
    wino88v_out_body<RESID, WRITE_Y>(M, rows, scale, shift, resid, Y, V8, ex, stag, first);
}

}  // namespace kv
