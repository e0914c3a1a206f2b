// Update-step kernels: the reference trains ChessNet
// under torch.cuda.amp.autocast (scripts/train.py:161-184), so every 3x3
// convolution of the tower runs with fp16 operands and fp32 accumulation, the
// BatchNorms in training mode (batch statistics in fp32, fp16 output), and the
// backward pass in the same precisions. These kernels restate that on MI355X
// for the convolutions and BatchNorm(+residual)(+ReLU) units of the tower
// (ai/model.py:8-25, :58-62), in NHWC fp16 ([board][64 squares][channels]),
// replacing the MIOpen convolutions (and their NCHW<->NHWC transposes) of the
// PyTorch-ROCm path. The heads stay PyTorch ops (a few MFLOP per board).
//
//   conv3x3_f16_kernel : implicit GEMM on v_mfma_f32_32x32x16_f16.
//       y[n][p][co] = bias[co] + sum_{t<9, ci} x[n][p + off(t)][ci] * w[co][t][ci]
//       (zero padding outside the 8x8 board). The data gradient is the same
//       kernel on dy with the weights flipped and transposed
//       (w'[ci][8 - t][co] = w[co][t][ci]).
//   conv3x3_wgrad_f16_kernel : dw[co][t][ci] = sum_{n,p} dy[n][p][co] x[n][p + off(t)][ci],
//       12 waves (channel halves x a row of 3 taps), split over boards (fp32 partials, reduced in a fixed
//       order: deterministic), both operands read transposed from LDS with
//       ds_read_b64_tr_b16.
//   bn_* : per-channel sums in fp32 per row block, combined in fp64 in block
//       order; the affine + residual + ReLU epilogue in the reference's
//       rounding order (BN output rounded to fp16, the residual added in fp32
//       and rounded again, as fp16 tensors add on the GPU).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kv_common.h"

#pragma clang fp contract(off)

namespace kv {
namespace tr {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

// ------------------------------------------------------------------ conv --
// Workgroup: 8 boards x 128 output channels, 8 waves; wave w takes board w and
// all 128 channels as 4 x 2 MFMA tiles with M = output channel, N = square (a
// lane's accumulators are 4 consecutive channels of one square: 8-byte
// stores; 0.75 LDS fragment reads per MFMA). K = 9 taps x input channels, in
// stages of 16 input channels, double-buffered in LDS:
//   W image : [128 co][9 taps][16 ci] f16, co stride 304 B (19 slots: the 32
//             rows an A read touches land on distinct 16-B bank slots);
//   X image : per board the 64 squares at 48 B (32 B data + 16 B pad, row of 8
//             squares = 24 slots); a tap that leaves the board reads a 16-B
//             zero slot instead (same address in every such lane: broadcast).
// Squares are dealt to the lanes of an N tile so that every ds_read_b128 lane
// group reads tile rows {0, 1} or {2, 3}: 16 distinct bank slots for every
// tap whose squares stay on the board. Global -> LDS through registers with
// prefetch distance 2, one barrier per stage; each tap's fragments are read
// while the previous tap's 8 MFMAs issue.
namespace cv {
constexpr int WCO = 128, NB = 8, CK = 16;
constexpr int WROW = 9 * 32 + 16;          // 304 B per output channel
constexpr int XSQ = 48;                    // B per square
constexpr int XBOARD = 64 * XSQ;           // 3,072 B
constexpr int WIMG = WCO * WROW;           // 38,912 B
constexpr int STAGE = WIMG + NB * XBOARD;  // 63,488 B
constexpr int ZERO = 2 * STAGE;            // the zero slot, after both stages
constexpr int LDS = 2 * STAGE + 16;        // 126,992 B
constexpr int THREADS = 512;
constexpr int W_CHUNKS = WCO * 9 * 2;      // 16-B pieces of a stage's W image (2,304)
}  // namespace cv

// square of an N tile handled by lane li (0..31): lane group {0-3,12-15,20-27}
// takes tile rows 0 and 1, {4-11,16-19,28-31} rows 2 and 3
__device__ inline int conv_lane_square(int li) {
    const bool g0 = li < 4 || (li >= 12 && li < 16) || (li >= 20 && li < 28);
    // rank of li inside its group (0..15): group 0 = 0-3, 12-15, 20-27; group 1 = 4-11, 16-19, 28-31
    const int j = li < 4 ? li : li < 12 ? li - 4 : li < 20 ? li - 8 : li < 28 ? li - 12 : li - 16;
    return ((j >> 3) + (g0 ? 0 : 2)) * 8 + (j & 7);
}

__global__ __launch_bounds__(cv::THREADS) void conv3x3_f16_kernel(const _Float16* __restrict__ x, int n, int ci,
                                                                  const _Float16* __restrict__ w,
                                                                  const float* __restrict__ bias, int co,
                                                                  const _Float16* __restrict__ add,
                                                                  _Float16* __restrict__ y) {
    using namespace cv;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, h = lane >> 5;
    // XCD-aware order (block b runs on XCD b % 8): every XCD keeps ONE output-channel block, so its
    // weights (1.2 MB for 512 input channels) stay in that XCD's L2 for all its board blocks; the
    // 8 / cblocks XCDs of a channel block interleave the board blocks
    const int cblocks = co / WCO, nblocks = (n + NB - 1) / NB;
    const int xcd = (int)(blockIdx.x & 7), per_c = 8 / cblocks;
    const int cb = xcd % cblocks, bb = (int)(blockIdx.x >> 3) * per_c + xcd / cblocks;
    if (bb >= nblocks) return;
    const int co0 = cb * WCO, n0 = bb * NB;

    if (tid == 0) *(u32x4*)(lds + ZERO) = u32x4{0, 0, 0, 0};

    // this thread's global -> LDS pieces: W chunks tid + 512 i (i < 4, and i = 4 for tid < 256), X chunks tid, tid + 512
    u32x4 rw[5], rx[2];
    auto load = [&](int s) {
        const int c0 = s * CK;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int c = tid + i * THREADS;
            if (i < 4 || c < W_CHUNKS) {
                const int o = c / 18, r = c % 18;
                rw[i] = *(const u32x4*)(w + ((size_t)(co0 + o) * 9 + (r >> 1)) * ci + c0 + (r & 1) * 8);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + i * THREADS, b = c >> 7, sq = (c >> 1) & 63;
            rx[i] = n0 + b < n ? *(const u32x4*)(x + ((size_t)(n0 + b) * 64 + sq) * ci + c0 + (c & 1) * 8)
                               : u32x4{0, 0, 0, 0};
        }
    };
    auto store = [&](unsigned char* st) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int c = tid + i * THREADS;
            if (i < 4 || c < W_CHUNKS) {
                const int o = c / 18, r = c % 18;
                *(u32x4*)(st + o * WROW + (r >> 1) * 32 + (r & 1) * 16) = rw[i];
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + i * THREADS, b = c >> 7, sq = (c >> 1) & 63;
            *(u32x4*)(st + WIMG + b * XBOARD + sq * XSQ + (c & 1) * 16) = rx[i];
        }
    };

    int abase[4], bbase[2];
    bool up[2], down[2], left[2], right[2];
#pragma unroll
    for (int m = 0; m < 4; ++m) abase[m] = (m * 32 + li) * WROW + 16 * h;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int sq = q * 32 + conv_lane_square(li), sy = sq >> 3, sx = sq & 7;
        bbase[q] = WIMG + wave * XBOARD + sq * XSQ + 16 * h;
        up[q] = sy > 0;
        down[q] = sy < 7;
        left[q] = sx > 0;
        right[q] = sx < 7;
    }
    f32x16 acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][q][r] = 0.f;

    // prefetch distance 2: at the top of iteration s the registers hold stage s+1 (loaded during
    // stage s-1's MFMAs) and go to the free LDS buffer, then stage s+2's global loads are issued
    const int ns = ci / CK;
    load(0);
    store(lds);
    if (ns > 1) load(1);
    __syncthreads();
    for (int s = 0; s < ns; ++s) {
        const unsigned char* cur = lds + (s & 1) * STAGE;
        if (s + 1 < ns) {
            store(lds + ((s + 1) & 1) * STAGE);
            if (s + 2 < ns) load(s + 2);
        }
        h8 fa[2][4], fb[2][2];
        auto frag = [&](int tp, int k) {
            const int dr = tp / 3 - 1, dc = tp % 3 - 1;
#pragma unroll
            for (int m = 0; m < 4; ++m) fa[k][m] = *(const h8*)(cur + abase[m] + tp * 32);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const bool ok = (dr < 0 ? up[q] : dr > 0 ? down[q] : true) && (dc < 0 ? left[q] : dc > 0 ? right[q] : true);
                fb[k][q] = *(const h8*)(ok ? cur + bbase[q] + (dr * 8 + dc) * XSQ : lds + ZERO);
            }
        };
        frag(0, 0);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
            if (tp + 1 < 9) frag(tp + 1, (tp + 1) & 1);
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[tp & 1][m], fb[tp & 1][q], acc[m][q], 0, 0, 0);
        }
        __syncthreads();
    }

    if (n0 + wave >= n) return;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int sq = q * 32 + conv_lane_square(li);
        const size_t o = ((size_t)(n0 + wave) * 64 + sq) * co + co0;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = m * 32 + 8 * g + 4 * h;  // 4 consecutive channels in registers 4g .. 4g+3
                f32x4 v = {acc[m][q][4 * g], acc[m][q][4 * g + 1], acc[m][q][4 * g + 2], acc[m][q][4 * g + 3]};
                if (bias) {
                    const f32x4 bv = *(const f32x4*)(bias + co0 + c);
                    v = v + bv;
                }
                h4 hv = __builtin_convertvector(v, h4);
                if (add) {  // autograd's gradient accumulation: fp16(float(dx) + float(other))
                    const h4 av = *(const h4*)(add + o + c);
                    hv = __builtin_convertvector(__builtin_convertvector(hv, f32x4) + __builtin_convertvector(av, f32x4),
                                                 h4);
                }
                *(h4*)(y + o + c) = hv;
            }
    }
}

// fp32 PyTorch weight [co][ci_real][3][3] -> fp16 forward image [co][9][ci]
// (ci >= ci_real, zero-filled) and flipped data-gradient image [ci][9][co]
__global__ void conv_weights_f16_kernel(const float* __restrict__ w, int co, int ci_real, int ci,
                                        _Float16* __restrict__ wf, _Float16* __restrict__ wt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= co * 9 * ci) return;
    const int c = i % ci, t = (i / ci) % 9, o = i / (9 * ci);
    const _Float16 v = c < ci_real ? (_Float16)w[((size_t)o * ci_real + c) * 9 + t] : (_Float16)0.f;
    wf[i] = v;
    if (wt) wt[((size_t)c * 9 + (8 - t)) * co + o] = v;
}

// ----------------------------------------------------------------- wgrad --
// Workgroup: 64 output x 64 input channels, all 9 taps (12 waves: output half x
// input half x a kernel row of 3 taps, the dY fragment shared by the row), boards
// [b0, b1) of this split, 2 boards per LDS stage (double-buffered). Images
// (rows 192 B = 64 channels + 64 B pad: the 4 rows x 64 B of a transposed
// read's 32-lane half land on 4 distinct quarter bank rows):
//   dY : [64 squares][64 co] per board,
//   X  : [10 x 12 halo squares][64 ci] per board (border zeroed once).
// K = squares: k-step s of a board covers board rows 2s, 2s+1 (16 squares).
namespace wg {
constexpr int TC = 64, RB = 192, BPS = 2;
constexpr int DYB = 64 * RB;                // 12,288 B per board
constexpr int XB = 10 * 12 * RB;            // 23,040 B per board
constexpr int STAGE = BPS * (DYB + XB);     // 70,656 B
constexpr int LDS = 2 * STAGE;              // 141,312 B
constexpr int THREADS = 12 * 64;          // 3 waves per SIMD
constexpr int CHUNKS = BPS * 2 * 64 * 8;    // 16-B pieces per stage (dY + X interiors): 2,048
}  // namespace wg

__global__ __launch_bounds__(wg::THREADS) void conv3x3_wgrad_f16_kernel(const _Float16* __restrict__ dy,
                                                                        const _Float16* __restrict__ x, int n,
                                                                        int ci, int co, int splits,
                                                                        float* __restrict__ part) {
    using namespace wg;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // wave w: output-channel half m, input-channel half jn, taps 3 gt .. 3 gt + 2 (kernel row dr = gt - 1,
    // columns dc = -1, 0, 1): one 32 x 32 MFMA block per tap, the dY fragment shared by the three taps.
    // 12 waves = 3 per SIMD (9 waves, one per tap, left one SIMD a third wave: 3/2/2/2)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m = wave & 1, jn = (wave >> 1) & 1, gt = wave >> 2;
    const int dr = gt - 1;
    // XCD-aware order (block b runs on XCD b % 8): the tiles of one board split run side by side on
    // the same XCD(s), so each board's dY / X pass through HBM once per XCD and the tiles share them in L2
    const int ct = co / TC, it = ci / TC, tiles = ct * it;
    const int xcd = (int)(blockIdx.x & 7), k = (int)(blockIdx.x >> 3);
    int split, tile;
    if (splits >= 8) {  // splits spread over the XCDs
        split = (k / tiles) * 8 + xcd;
        tile = k % tiles;
    } else {  // 8 / splits XCDs per split, its tiles dealt over them
        const int xs = 8 / splits;
        split = xcd / xs;
        tile = k * xs + xcd % xs;
    }
    if (split >= splits || tile >= tiles) return;
    const int co0 = (tile % ct) * TC, ci0 = (tile / ct) * TC;
    const int per = (n + splits - 1) / splits;
    const int b0 = split * per, b1 = min(n, b0 + per);

    for (int o = tid * 16; o < BPS * XB; o += THREADS * 16) {  // both stages' X halos
        *(u32x4*)(lds + BPS * DYB + o) = u32x4{0, 0, 0, 0};
        *(u32x4*)(lds + STAGE + BPS * DYB + o) = u32x4{0, 0, 0, 0};
    }

    constexpr int PER = (CHUNKS + THREADS - 1) / THREADS;
    u32x4 reg[PER];
    auto load = [&](int bb) {  // boards bb, bb+1
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = tid + i * THREADS;
            if (c < CHUNKS) {
                const int isx = c >= CHUNKS / 2, cc = c & (CHUNKS / 2 - 1);
                const int b = cc >> 9, sq = (cc >> 3) & 63, part8 = cc & 7;
                const int board = bb + b;
                const _Float16* src = isx ? x + ((size_t)board * 64 + sq) * ci + ci0 + part8 * 8
                                          : dy + ((size_t)board * 64 + sq) * co + co0 + part8 * 8;
                reg[i] = board < b1 ? *(const u32x4*)src : u32x4{0, 0, 0, 0};
            }
        }
    };
    auto store = [&](unsigned char* st) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = tid + i * THREADS;
            if (c < CHUNKS) {
                const int isx = c >= CHUNKS / 2, cc = c & (CHUNKS / 2 - 1);
                const int b = cc >> 9, sq = (cc >> 3) & 63, part8 = cc & 7;
                const int off = isx ? BPS * DYB + b * XB + (((sq >> 3) + 1) * 12 + (sq & 7) + 1) * RB
                                    : b * DYB + sq * RB;
                *(u32x4*)(st + off + part8 * 16) = reg[i];
            }
        }
    };

    // transposed-read addresses: lane l, group g = l / 16, i = l % 16, q = i / 4, p = i % 4;
    // rows 8h + q (+4 for elements 4..7), columns 16 (g & 1) + 4p (+32 per tile). Square k =
    // 16 ks + 8h + q + 4e sits at board row 2 ks + h, column q + 4e, so every read is a per-lane
    // base plus a compile-time offset (ks, e, tile, board)
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, h = lane >> 5;
    const int col = (16 * (g & 1) + 4 * p) * 2;
    const int dy_lane = (8 * h + q) * RB + col + m * 64;                              // + (16 ks + 4 e) RB
    const int x_lane = BPS * DYB + ((h + 1 + dr) * 12 + q + 1) * RB + col + jn * 64;   // + (24 ks + 4 e + dc) RB
    f32x16 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    // prefetch distance 2, as in conv3x3_f16_kernel
    const int nst = (b1 - b0 + BPS - 1) / BPS;
    if (nst > 0) load(b0);
    __syncthreads();
    if (nst > 0) store(lds);
    if (nst > 1) load(b0 + BPS);
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
        const unsigned char* cur = lds + (s & 1) * STAGE;
        if (s + 1 < nst) {
            store(lds + ((s + 1) & 1) * STAGE);
            if (s + 2 < nst) load(b0 + (s + 2) * BPS);
        }
        const unsigned char* dyl = cur + dy_lane;
        const unsigned char* xl = cur + x_lane;
#pragma unroll
        for (int b = 0; b < BPS; ++b) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                s4 av4[2], bv4[3][2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    av4[e] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(dyl + b * DYB + (16 * ks + 4 * e) * RB));
#pragma unroll
                    for (int t = 0; t < 3; ++t)
                        bv4[t][e] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s4*)(xl + b * XB + (24 * ks + 4 * e + t - 1) * RB));
                }
                // elements 0-3 from the first read, 4-7 from the second
                const h8 a = __builtin_bit_cast(h8, __builtin_shufflevector(av4[0], av4[1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const h8 bv = __builtin_bit_cast(h8, __builtin_shufflevector(bv4[t][0], bv4[t][1], 0, 1, 2, 3, 4, 5, 6, 7));
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bv, acc[t], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // D[row = co][col = ci]: lane li holds ci = 32 jn + li, rows (r&3) + 8 (r>>2) + 4h of half m
    const int li = lane & 31;
    float* po = part + (size_t)split * co * 9 * ci;
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = co0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            po[((size_t)o * 9 + 3 * gt + t) * ci + ci0 + jn * 32 + li] = acc[t][r];
        }
}

// sum of the split partials in split order -> fp16 rounding (the gradient of
// an autocast fp16 convolution is fp16) -> fp32 PyTorch layout [co][ci_real][3][3]
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int co, int ci, int ci_real,
                                    float* __restrict__ dw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= co * ci_real * 9) return;
    const int t = i % 9, c = (i / 9) % ci_real, o = i / (9 * ci_real);
    const size_t src = ((size_t)o * 9 + t) * ci + c, stride = (size_t)co * 9 * ci;
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += part[src + k * stride];
    dw[i] = (float)(_Float16)s;
}

// -------------------------------------------------------------- BatchNorm --
// rows x C fp16 (C a multiple of 64, <= 512). Partial sums: a block of 256
// threads takes BN_ROWS rows; a thread takes 8 channels (one 16-B load per
// row) of every (256 / (C/8))-th row, then the block adds its row lanes in a
// fixed order through LDS and writes fp32 partials [block][C] of two sums:
//   mode 0 (forward statistics): x - k and (x - k)^2, k = row 0's value
//          (no cancellation when |mean| >> std);
//   mode 1 (backward): g = dy * (y > 0 if relu) and g * (x - mean) * invstd;
//   mode 2: x (the channel sums of dy: the gradient of a conv bias).
// The finalize kernel adds the block partials in fp64 in a fixed order.
constexpr int BN_ROWS = 256;
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

__device__ inline void h8_to_f(const u32x4 v, float* f) {
    const h8 hv = __builtin_bit_cast(h8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (float)hv[e];
}

// MODE is a template argument so the row loop can keep U rows' loads in flight
// (U 16-B loads per operand issued before the first is consumed); the sums
// still take the rows in the same order.
template <int MODE>
__global__ __launch_bounds__(256) void bn_partial_kernel(const _Float16* __restrict__ x, const _Float16* __restrict__ dy,
                                                         const _Float16* __restrict__ yout, int rows, int C, int relu,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, float* __restrict__ p0,
                                                         float* __restrict__ p1) {
    constexpr int U = MODE == 1 ? 4 : 8;
    __shared__ float red[2][256 * 8];
    const int cg = C / 8, rl = 256 / cg;  // channel groups, row lanes
    const int tid = threadIdx.x, g = tid % cg, lr = tid / cg;
    const int c = g * 8;
    // threads past rl * cg (C / 8 not a divisor of 256) take no rows
    const int r0 = blockIdx.x * BN_ROWS, r1 = lr < rl ? min(rows, r0 + BN_ROWS) : r0;
    float k[8], m[8], iv[8], s0[8], s1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        s0[e] = 0.f;
        s1[e] = 0.f;
        k[e] = 0.f;
        m[e] = 0.f;
        iv[e] = 0.f;
    }
    if (MODE == 0) h8_to_f(*(const u32x4*)(x + c), k);
    if (MODE == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            m[e] = mean[c + e];
            iv[e] = invstd[c + e];
        }
    }
    for (int r = r0 + lr; r < r1; r += U * rl) {
        u32x4 xa[U], ga[U], ya[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int rr = r + u * rl;
            if (rr < r1) {
                xa[u] = *(const u32x4*)(x + (size_t)rr * C + c);
                if (MODE == 1) {
                    ga[u] = *(const u32x4*)(dy + (size_t)rr * C + c);
                    if (relu) ya[u] = *(const u32x4*)(yout + (size_t)rr * C + c);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r + u * rl >= r1) break;
            float xv[8];
            h8_to_f(xa[u], xv);
            if (MODE == 0) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float d = xv[e] - k[e];
                    s0[e] += d;
                    s1[e] += d * d;
                }
            } else if (MODE == 2) {
#pragma unroll
                for (int e = 0; e < 8; ++e) s0[e] += xv[e];
            } else {
                float gv[8], yv[8];
                h8_to_f(ga[u], gv);
                if (relu) h8_to_f(ya[u], yv);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float gg = (relu && !(yv[e] > 0.f)) ? 0.f : gv[e];
                    s0[e] += gg;
                    s1[e] += gg * ((xv[e] - m[e]) * iv[e]);
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        red[0][tid * 8 + e] = s0[e];
        red[1][tid * 8 + e] = s1[e];
    }
    __syncthreads();
    // thread t < C: channel t, row lanes added in order
    for (int ch = tid; ch < C; ch += 256) {
        const int gg = ch / 8, e = ch % 8;
        float a = 0.f, b2 = 0.f;
        for (int l = 0; l < rl; ++l) {
            a += red[0][(l * cg + gg) * 8 + e];
            b2 += red[1][(l * cg + gg) * 8 + e];
        }
        p0[(size_t)blockIdx.x * C + ch] = a;
        if (MODE != 2) p1[(size_t)blockIdx.x * C + ch] = b2;
    }
}

// block partials -> per-channel results (fp64; block = 16 channels x 64
// groups, thread (channel, group j) adds blocks j, j+64, ... then the 64 groups
// are added in order):
//   mode 0: mean, biased var, invstd = 1/sqrt(var + eps) (out0, out1, out2)
//   mode 1: sum g, sum g*xhat (out0, out1 if given); p1 is not read without out1
constexpr int BNF_CH = 16, BNF_GROUPS = 64;

__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                           int blocks, int C, int rows, int mode, float eps,
                                                           const _Float16* __restrict__ shift, float* __restrict__ out0,
                                                           float* __restrict__ out1, float* __restrict__ out2) {
    __shared__ double ra[BNF_GROUPS][BNF_CH], rb[BNF_GROUPS][BNF_CH];
    const int cl = threadIdx.x % BNF_CH, j = threadIdx.x / BNF_CH;
    const int c = blockIdx.x * BNF_CH + cl;
    const bool two = mode == 0 || out1 != nullptr;
    double a = 0.0, b = 0.0;
    if (c < C) {
#pragma unroll 4
        for (int k = j; k < blocks; k += BNF_GROUPS) {
            a += (double)p0[(size_t)k * C + c];
            if (two) b += (double)p1[(size_t)k * C + c];
        }
    }
    ra[j][cl] = a;
    rb[j][cl] = b;
    __syncthreads();
    if (j != 0 || c >= C) return;
    a = 0.0;
    b = 0.0;
    for (int q = 0; q < BNF_GROUPS; ++q) {
        a += ra[q][cl];
        b += rb[q][cl];
    }
    if (mode == 0) {  // a, b: sums of (x - k) and (x - k)^2, k = the first row's value
        const double d = a / rows;
        double v = b / rows - d * d;
        if (v < 0.0) v = 0.0;
        const double m = (double)(float)shift[c] + d;
        out0[c] = (float)m;
        out1[c] = (float)v;
        out2[c] = (float)(1.0 / sqrt(v + (double)eps));
    } else {
        out0[c] = (float)a;
        if (out1) out1[c] = (float)b;
    }
}

// y = fp16((x - mean) * invstd * gamma + beta); + residual: fp16(float(y) + float(res)); ReLU.
// Thread = 8 channels (16-B accesses, its channels' parameters in registers) of
// every (256 / (C/8))-th row of the block's BN_EW_ROWS rows.
constexpr int BN_EW_ROWS = 64;

__global__ __launch_bounds__(256) void bn_apply_kernel(const _Float16* __restrict__ x, int rows, int C,
                                                       const float* __restrict__ mean, const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       const _Float16* __restrict__ res, int relu,
                                                       _Float16* __restrict__ y) {
    const int cg = C / 8, rl = 256 / cg;
    const int g = threadIdx.x % cg, lr = threadIdx.x / cg, c = g * 8;
    float m[8], iv[8], ga[8], be[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        m[e] = mean[c + e];
        iv[e] = invstd[c + e];
        ga[e] = gamma[c + e];
        be[e] = beta[c + e];
    }
    const int r0 = blockIdx.x * BN_EW_ROWS, r1 = lr < rl ? min(rows, r0 + BN_EW_ROWS) : r0;
    for (int r = r0 + lr; r < r1; r += rl) {
        const size_t i = (size_t)r * C + c;
        float xv[8], rv[8];
        h8_to_f(*(const u32x4*)(x + i), xv);
        if (res) h8_to_f(*(const u32x4*)(res + i), rv);
        h8 out;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float v = (xv[e] - m[e]) * iv[e] * ga[e] + be[e];
            _Float16 hv = (_Float16)v;
            if (res) hv = (_Float16)((float)hv + rv[e]);
            if (relu && !((float)hv > 0.f)) hv = (_Float16)0.f;
            out[e] = hv;
        }
        *(h8*)(y + i) = out;
    }
}

// dx = fp16(gamma * invstd * (g - sum_g / M - xhat * sum_gx / M)), g = dy * (y > 0 if relu);
// dres (if given) = g. Same thread layout as bn_apply_kernel.
__global__ __launch_bounds__(256) void bn_backward_kernel(const _Float16* __restrict__ x, const _Float16* __restrict__ dy,
                                                          const _Float16* __restrict__ yout, int rows, int C, int relu,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma, const float* __restrict__ sg,
                                                          const float* __restrict__ sgx, _Float16* __restrict__ dx,
                                                          _Float16* __restrict__ dres, float* __restrict__ dsp) {
    __shared__ float red[256 * 8];
    const int cg = C / 8, rl = 256 / cg;
    const int g = threadIdx.x % cg, lr = threadIdx.x / cg, c = g * 8;
    const float inv_m = 1.0f / (float)rows;
    float m[8], iv[8], mg[8], mgx[8], sc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        m[e] = mean[c + e];
        iv[e] = invstd[c + e];
        mg[e] = sg[c + e] * inv_m;
        mgx[e] = sgx[c + e] * inv_m;
        sc[e] = gamma[c + e] * iv[e];
    }
    float ds[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int r0 = blockIdx.x * BN_EW_ROWS, r1 = lr < rl ? min(rows, r0 + BN_EW_ROWS) : r0;
    for (int r = r0 + lr; r < r1; r += rl) {
        const size_t i = (size_t)r * C + c;
        float xv[8], gv[8], yv[8];
        h8_to_f(*(const u32x4*)(x + i), xv);
        h8_to_f(*(const u32x4*)(dy + i), gv);
        if (relu) h8_to_f(*(const u32x4*)(yout + i), yv);
        h8 o, rr;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float gg = (relu && !(yv[e] > 0.f)) ? 0.f : gv[e];
            const float xh = (xv[e] - m[e]) * iv[e];
            o[e] = (_Float16)((gg - mg[e] - xh * mgx[e]) * sc[e]);
            rr[e] = (_Float16)gg;
            ds[e] += (float)o[e];
        }
        *(h8*)(dx + i) = o;
        if (dres) *(h8*)(dres + i) = rr;
    }
    if (!dsp) return;
    // the channel sums of dx (the producing conv's bias gradient): block partials [block][C], row lanes in order
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = ds[e];
    __syncthreads();
    for (int ch = threadIdx.x; ch < C; ch += 256) {
        float a = 0.f;
        for (int l = 0; l < rl; ++l) a += red[(l * cg + ch / 8) * 8 + ch % 8];
        dsp[(size_t)blockIdx.x * C + ch] = a;
    }
}

// ----------------------------------------------------------- head 1x1s --
// The policy (512 -> 2) and value (512 -> 1) 1x1 convolutions of the heads
// (ai/model.py:42-49, :64-73) as autocast fp16 ops over rows = boards x 64
// squares of the tower output h [rows][512]: out[r][j] = fp16(b[j] + sum_c
// h[r][c] w[j][c]) for j < 3 (out row stride 4). One wave per row, lane = 8
// channels, rows grid-strided over the waves.
__global__ __launch_bounds__(256) void head1x1_fwd_kernel(const _Float16* __restrict__ h, int rows,
                                                          const _Float16* __restrict__ w, const float* __restrict__ b,
                                                          _Float16* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    float wv[3][8];
#pragma unroll
    for (int j = 0; j < 3; ++j) h8_to_f(*(const u32x4*)(w + j * 512 + lane * 8), wv[j]);
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    for (int r = wave; r < rows; r += nw) {
        float xv[8];
        h8_to_f(*(const u32x4*)(h + (size_t)r * 512 + lane * 8), xv);
        float a[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float t = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) t += xv[e] * wv[j][e];
            a[j] = t;
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
            for (int j = 0; j < 3; ++j) a[j] += __shfl_xor(a[j], m);
        if (lane < 3) {
            const float v = lane == 0 ? a[0] : lane == 1 ? a[1] : a[2];
            out[(size_t)r * 4 + lane] = (_Float16)(v + b[lane]);
        }
    }
}

// backward: dh[r][c] = fp16(sum_j dout[r][j] w[j][c]); partial sums per block of
// dw[j][c] = sum_r dout[r][j] h[r][c] and db[j] = sum_r dout[r][j] (fp32,
// [block][4][512], the row lanes added in a fixed order)
constexpr int H1_ROWS = 256;
__global__ __launch_bounds__(256) void head1x1_bwd_kernel(const _Float16* __restrict__ h,
                                                          const _Float16* __restrict__ dout, int rows,
                                                          const _Float16* __restrict__ w, _Float16* __restrict__ dh,
                                                          float* __restrict__ part) {
    __shared__ float red[4][4][512];
    const int tid = threadIdx.x, g = tid & 63, lr = tid >> 6, c = g * 8;
    float wv[3][8], acc[3][8], db[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        h8_to_f(*(const u32x4*)(w + j * 512 + c), wv[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
    }
    const int r0 = blockIdx.x * H1_ROWS, r1 = min(rows, r0 + H1_ROWS);
    for (int r = r0 + lr; r < r1; r += 4) {
        float xv[8];
        h8_to_f(*(const u32x4*)(h + (size_t)r * 512 + c), xv);
        const h4 dv = *(const h4*)(dout + (size_t)r * 4);
        const float d[3] = {(float)dv[0], (float)dv[1], (float)dv[2]};
        h8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            o[e] = (_Float16)(d[0] * wv[0][e] + d[1] * wv[1][e] + d[2] * wv[2][e]);
#pragma unroll
            for (int j = 0; j < 3; ++j) acc[j][e] += d[j] * xv[e];
        }
        *(h8*)(dh + (size_t)r * 512 + c) = o;
#pragma unroll
        for (int j = 0; j < 3; ++j) db[j] += d[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lr][j][c + e] = acc[j][e];
    if (g == 0)
#pragma unroll
        for (int j = 0; j < 3; ++j) red[lr][3][j] = db[j];
    __syncthreads();
    for (int i = tid; i < 4 * 512; i += 256) {
        const int j = i / 512, ch = i % 512;
        if (j == 3 && ch >= 3) {
            part[(size_t)blockIdx.x * 2048 + i] = 0.f;
            continue;
        }
        part[(size_t)blockIdx.x * 2048 + i] = ((red[0][j][ch] + red[1][j][ch]) + red[2][j][ch]) + red[3][j][ch];
    }
}

// block partials [blocks][4][512] -> dw fp32 [3][512] (fp16-rounded) and db fp32 [3] (fp16-rounded);
// thread (entry, group q) adds blocks q, q+4, ..., then the 4 groups in order (fp64)
__global__ __launch_bounds__(256) void head1x1_reduce_kernel(const float* __restrict__ part, int blocks,
                                                             float* __restrict__ dw, float* __restrict__ db) {
    __shared__ double red[4][64];
    const int el = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + el;  // entry of [4][512]
    double a = 0.0;
    for (int k = q; k < blocks; k += 4) a += (double)part[(size_t)k * 2048 + i];
    red[q][el] = a;
    __syncthreads();
    if (q != 0) return;
    const double t = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
    const int j = i / 512, ch = i % 512;
    if (j < 3) dw[j * 512 + ch] = (float)(_Float16)(float)t;
    else if (ch < 3) db[ch] = (float)(_Float16)(float)t;
}

// planes fp32 [n][12][8][8] (encode_board) -> NHWC fp16 [n][64][cpad], channels >= 12 zero
__global__ void planes_to_nhwc_kernel(const float* __restrict__ planes, int n, int cpad, _Float16* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)n * 64 * cpad) return;
    const int c = (int)(i % cpad), sq = (int)((i / cpad) % 64);
    const size_t b = i / ((size_t)cpad * 64);
    out[i] = c < 12 ? (_Float16)planes[(b * 12 + c) * 64 + sq] : (_Float16)0.f;
}

}  // namespace tr
}  // namespace kv

using namespace kv::tr;

// The large-LDS opt-in of a kernel is per device: done once per (kernel, device)
// and recorded in a per-kernel bitset of devices (atomic, so concurrent host
// threads at worst set the attribute twice, which is harmless).
#include <atomic>
static std::atomic<unsigned long long> g_lds_opted[2];
static hipError_t lds_opt_in(const void* fn, int bytes, int which) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (g_lds_opted[which].load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) g_lds_opted[which].fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

extern "C" {

int kv_tr_conv3x3_f16(const void* x_dev, int n, int ci, const void* w_dev, const float* bias_dev, int co,
                      void* y_dev, void* stream) {
    return kv_tr_conv3x3_add_f16(x_dev, n, ci, w_dev, bias_dev, co, nullptr, y_dev, stream);
}

int kv_tr_conv3x3_add_f16(const void* x_dev, int n, int ci, const void* w_dev, const float* bias_dev, int co,
                          const void* add_dev, void* y_dev, void* stream) {
    KV_REQUIRE(x_dev && w_dev && y_dev && n > 0 && add_dev != y_dev, KV_EINVAL, "kv_tr_conv3x3_f16: bad arguments");
    KV_REQUIRE(ci > 0 && ci % cv::CK == 0 && co > 0 && co % cv::WCO == 0, KV_EINVAL,
               "kv_tr_conv3x3_f16: ci %d must be a multiple of %d, co %d of %d", ci, cv::CK, co, cv::WCO);
    KV_HIP(lds_opt_in((const void*)conv3x3_f16_kernel, cv::LDS, 0));
    const int cblocks = co / cv::WCO, nblocks = (n + cv::NB - 1) / cv::NB;
    KV_REQUIRE(8 % cblocks == 0, KV_EINVAL, "kv_tr_conv3x3_f16: co %d: at most 1024 output channels, a power of two "
               "number of 128-channel blocks", co);
    const int grid = (nblocks + 8 / cblocks - 1) / (8 / cblocks) * 8;
    hipLaunchKernelGGL(conv3x3_f16_kernel, dim3(grid), dim3(cv::THREADS), cv::LDS, (hipStream_t)stream,
                       (const _Float16*)x_dev, n, ci, (const _Float16*)w_dev, bias_dev, co, (const _Float16*)add_dev,
                       (_Float16*)y_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int kv_tr_conv_weights_f16(const float* w_dev, int co, int ci_real, int ci, void* wf_dev, void* wt_dev, void* stream) {
    KV_REQUIRE(w_dev && wf_dev && co > 0 && ci_real > 0 && ci >= ci_real, KV_EINVAL,
               "kv_tr_conv_weights_f16: bad arguments");
    const int total = co * 9 * ci;
    hipLaunchKernelGGL(conv_weights_f16_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, w_dev,
                       co, ci_real, ci, (_Float16*)wf_dev, (_Float16*)wt_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

size_t kv_tr_wgrad_workspace(int n, int ci, int co, int* splits) {
    const int tiles = (co / wg::TC) * (ci / wg::TC);
    int s = (256 + tiles - 1) / tiles;  // about one workgroup per CU
    if (s > (n + 1) / 2) s = (n + 1) / 2;
    if (s < 1) s = 1;
    // a power of two up to 8 (8 / splits XCDs per split), else a multiple of 8 (splits spread over the XCDs)
    if (s < 8) {
        int p = 1;
        while (p * 2 <= s) p *= 2;
        s = p;
    } else {
        s = s / 8 * 8;
    }
    if (splits) *splits = s;
    return (size_t)s * co * 9 * ci * sizeof(float);
}

int kv_tr_conv3x3_wgrad_f16(const void* dy_dev, const void* x_dev, int n, int ci, int ci_real, int co, float* dw_dev,
                            void* ws_dev, size_t ws_bytes, void* stream) {
    KV_REQUIRE(dy_dev && x_dev && dw_dev && ws_dev && n > 0, KV_EINVAL, "kv_tr_conv3x3_wgrad_f16: bad arguments");
    KV_REQUIRE(ci % wg::TC == 0 && co % wg::TC == 0 && ci_real <= ci, KV_EINVAL,
               "kv_tr_conv3x3_wgrad_f16: ci %d / co %d must be multiples of %d", ci, co, wg::TC);
    int splits = 0;
    const size_t need = kv_tr_wgrad_workspace(n, ci, co, &splits);
    KV_REQUIRE(ws_bytes >= need, KV_EINVAL, "kv_tr_conv3x3_wgrad_f16: workspace %zu < %zu B", ws_bytes, need);
    KV_HIP(lds_opt_in((const void*)conv3x3_wgrad_f16_kernel, wg::LDS, 1));
    const int tiles = (co / wg::TC) * (ci / wg::TC);
    int grid;
    if (splits >= 8) {
        grid = splits * tiles;  // splits % 8 == 0
    } else {
        const int xs = 8 / splits;
        grid = (tiles + xs - 1) / xs * 8;
    }
    hipLaunchKernelGGL(conv3x3_wgrad_f16_kernel, dim3(grid), dim3(wg::THREADS), wg::LDS, (hipStream_t)stream,
                       (const _Float16*)dy_dev, (const _Float16*)x_dev, n, ci, co, splits, (float*)ws_dev);
    KV_HIP(hipGetLastError());
    const int total = co * ci_real * 9;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const float*)ws_dev, splits, co, ci, ci_real, dw_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

size_t kv_tr_bn_workspace(int rows, int C) {
    // two partial sums per BN_ROWS block, or (backward) the dx sums per BN_EW_ROWS block after them
    const size_t a = 2 * (size_t)((rows + BN_ROWS - 1) / BN_ROWS), b = (size_t)((rows + BN_EW_ROWS - 1) / BN_EW_ROWS);
    return std::max(a, b) * C * sizeof(float);
}

int kv_tr_bn_stats_f16(const void* x_dev, int rows, int C, float eps, float* mean_dev, float* var_dev,
                       float* invstd_dev, void* ws_dev, size_t ws_bytes, void* stream) {
    KV_REQUIRE(x_dev && mean_dev && var_dev && invstd_dev && ws_dev && rows > 0 && C > 0 && C % 64 == 0 && C <= 512,
               KV_EINVAL, "kv_tr_bn_stats_f16: bad arguments");
    KV_REQUIRE(ws_bytes >= kv_tr_bn_workspace(rows, C), KV_EINVAL, "kv_tr_bn_stats_f16: workspace too small");
    const int blocks = (rows + BN_ROWS - 1) / BN_ROWS;
    float* p0 = (float*)ws_dev;
    float* p1 = p0 + (size_t)blocks * C;
    hipLaunchKernelGGL(bn_partial_kernel<0>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const _Float16*)x_dev,
                       (const _Float16*)nullptr, (const _Float16*)nullptr, rows, C, 0, (const float*)nullptr,
                       (const float*)nullptr, p0, p1);
    KV_HIP(hipGetLastError());
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + BNF_CH - 1) / BNF_CH), dim3(1024), 0, (hipStream_t)stream, p0, p1, blocks, C,
                       rows, 0, eps, (const _Float16*)x_dev, mean_dev, var_dev, invstd_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int kv_tr_bn_apply_f16(const void* x_dev, int rows, int C, const float* mean_dev, const float* invstd_dev,
                       const float* gamma_dev, const float* beta_dev, const void* res_dev, int relu, void* y_dev,
                       void* stream) {
    KV_REQUIRE(x_dev && mean_dev && invstd_dev && gamma_dev && beta_dev && y_dev && rows > 0 && C % 64 == 0 && C <= 512,
               KV_EINVAL, "kv_tr_bn_apply_f16: bad arguments");
    hipLaunchKernelGGL(bn_apply_kernel, dim3((rows + BN_EW_ROWS - 1) / BN_EW_ROWS), dim3(256), 0, (hipStream_t)stream,
                       (const _Float16*)x_dev, rows, C, mean_dev, invstd_dev, gamma_dev, beta_dev,
                       (const _Float16*)res_dev, relu, (_Float16*)y_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int kv_tr_bn_backward_f16(const void* x_dev, const void* dy_dev, const void* y_dev, int rows, int C, int relu,
                          const float* mean_dev, const float* invstd_dev, const float* gamma_dev, float* dgamma_dev,
                          float* dbeta_dev, void* dx_dev, void* dres_dev, float* dxsum_dev, void* ws_dev,
                          size_t ws_bytes, void* stream) {
    KV_REQUIRE(x_dev && dy_dev && (y_dev || !relu) && mean_dev && invstd_dev && gamma_dev && dgamma_dev && dbeta_dev &&
                   dx_dev && ws_dev && rows > 0 && C % 64 == 0 && C <= 512,
               KV_EINVAL, "kv_tr_bn_backward_f16: bad arguments");
    KV_REQUIRE(ws_bytes >= kv_tr_bn_workspace(rows, C), KV_EINVAL, "kv_tr_bn_backward_f16: workspace too small");
    const int blocks = (rows + BN_ROWS - 1) / BN_ROWS;
    float* p0 = (float*)ws_dev;
    float* p1 = p0 + (size_t)blocks * C;
    hipLaunchKernelGGL(bn_partial_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const _Float16*)x_dev,
                       (const _Float16*)dy_dev, (const _Float16*)y_dev, rows, C, relu, mean_dev, invstd_dev, p0, p1);
    KV_HIP(hipGetLastError());
    // sum g -> dbeta, sum g * xhat -> dgamma
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + BNF_CH - 1) / BNF_CH), dim3(1024), 0, (hipStream_t)stream, p0, p1, blocks, C,
                       rows, 1, 0.f, (const _Float16*)nullptr, dbeta_dev, dgamma_dev, (float*)nullptr);
    KV_HIP(hipGetLastError());
    hipLaunchKernelGGL(bn_backward_kernel, dim3((rows + BN_EW_ROWS - 1) / BN_EW_ROWS), dim3(256), 0, (hipStream_t)stream,
                       (const _Float16*)x_dev, (const _Float16*)dy_dev, (const _Float16*)y_dev, rows, C, relu,
                       mean_dev, invstd_dev, gamma_dev, dbeta_dev, dgamma_dev, (_Float16*)dx_dev, (_Float16*)dres_dev,
                       dxsum_dev ? p0 : nullptr);  // p0 / p1 are consumed: the dx partials reuse the workspace
    KV_HIP(hipGetLastError());
    if (dxsum_dev) {
        hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + BNF_CH - 1) / BNF_CH), dim3(1024), 0, (hipStream_t)stream, p0,
                           p0, (rows + BN_EW_ROWS - 1) / BN_EW_ROWS, C, rows, 1, 0.f, (const _Float16*)nullptr,
                           dxsum_dev, (float*)nullptr, (float*)nullptr);
        KV_HIP(hipGetLastError());
    }
    return KV_OK;
}

int kv_tr_channel_sum_f16(const void* x_dev, int rows, int C, float* sum_dev, void* ws_dev, size_t ws_bytes,
                          void* stream) {
    KV_REQUIRE(x_dev && sum_dev && ws_dev && rows > 0 && C % 64 == 0 && C <= 512, KV_EINVAL,
               "kv_tr_channel_sum_f16: bad arguments");
    KV_REQUIRE(ws_bytes >= kv_tr_bn_workspace(rows, C), KV_EINVAL, "kv_tr_channel_sum_f16: workspace too small");
    const int blocks = (rows + BN_ROWS - 1) / BN_ROWS;
    float* p0 = (float*)ws_dev;
    float* p1 = p0 + (size_t)blocks * C;
    hipLaunchKernelGGL(bn_partial_kernel<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const _Float16*)x_dev,
                       (const _Float16*)nullptr, (const _Float16*)nullptr, rows, C, 0, (const float*)nullptr,
                       (const float*)nullptr, p0, p1);
    KV_HIP(hipGetLastError());
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + BNF_CH - 1) / BNF_CH), dim3(1024), 0, (hipStream_t)stream, p0, p1, blocks, C,
                       rows, 1, 0.f, (const _Float16*)nullptr, sum_dev, (float*)nullptr, (float*)nullptr);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int kv_tr_head1x1_f16(const void* h_dev, int rows, const void* w_dev, const float* b_dev, void* out_dev,
                      void* stream) {
    KV_REQUIRE(h_dev && w_dev && b_dev && out_dev && rows > 0, KV_EINVAL, "kv_tr_head1x1_f16: bad arguments");
    const int grid = std::min(2048, (rows + 3) / 4);
    hipLaunchKernelGGL(head1x1_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const _Float16*)h_dev, rows,
                       (const _Float16*)w_dev, b_dev, (_Float16*)out_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

size_t kv_tr_head1x1_workspace(int rows) { return (size_t)((rows + H1_ROWS - 1) / H1_ROWS) * 2048 * sizeof(float); }

int kv_tr_head1x1_backward_f16(const void* h_dev, const void* dout_dev, int rows, const void* w_dev, void* dh_dev,
                               float* dw_dev, float* db_dev, void* ws_dev, size_t ws_bytes, void* stream) {
    KV_REQUIRE(h_dev && dout_dev && w_dev && dh_dev && dw_dev && db_dev && ws_dev && rows > 0, KV_EINVAL,
               "kv_tr_head1x1_backward_f16: bad arguments");
    KV_REQUIRE(ws_bytes >= kv_tr_head1x1_workspace(rows), KV_EINVAL, "kv_tr_head1x1_backward_f16: workspace too small");
    const int blocks = (rows + H1_ROWS - 1) / H1_ROWS;
    hipLaunchKernelGGL(head1x1_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const _Float16*)h_dev,
                       (const _Float16*)dout_dev, rows, (const _Float16*)w_dev, (_Float16*)dh_dev, (float*)ws_dev);
    KV_HIP(hipGetLastError());
    hipLaunchKernelGGL(head1x1_reduce_kernel, dim3(2048 / 64), dim3(256), 0, (hipStream_t)stream,
                       (const float*)ws_dev, blocks, dw_dev, db_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int kv_tr_planes_to_nhwc(const float* planes_dev, int n, int cpad, void* out_dev, void* stream) {
    KV_REQUIRE(planes_dev && out_dev && n > 0 && cpad >= 12, KV_EINVAL, "kv_tr_planes_to_nhwc: bad arguments");
    const size_t total = (size_t)n * 64 * cpad;
    hipLaunchKernelGGL(planes_to_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       planes_dev, n, cpad, (_Float16*)out_dev);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

}  // extern "C"
