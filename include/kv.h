/*
 * kv.h -- C ABI of libkv.so, the MI355X-native self-play engine that drops in
 * under the reference's self-play data-generation path.
 *
 * The reference has no native boundary: its callers bind Python names
 * (SURVEY.md 8b). Each entry point below replaces one of those names; the
 * Python mirror in knightvision_amd/ (same names, argument meaning and error
 * behaviour) binds them with ctypes, see INTEGRATION.md.
 *
 * Conventions: every call returns int status (0 ok, negative KV_E*); the text
 * of the last error is kv_last_error(). Pointers named *_dev are HIP device
 * pointers, everything else is host memory owned by the caller. `stream` is a
 * hipStream_t passed as void* (NULL = the default stream). An engine or net
 * is not re-entrant: one host thread per object / GPU.
 */
#ifndef KV_H
#define KV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KV_OK 0
#define KV_EINVAL -1
#define KV_ENOMEM -2
#define KV_EHIP -3
#define KV_EOVERFLOW -4

const char* kv_last_error(void);
int kv_version(void);

/* ------------------------------------------------------------------ NN ---
 * ChessNet forward (replaces ai/model.py:51-77 ChessNet.forward).
 * Packed weights: BN folded into per-channel scale/shift; layout produced by
 * knightvision_amd/weights.py:pack_weights and re-derived by kv_net_packed_size
 * (each tensor padded to a multiple of 16 floats):
 *   12 convs, each: w[Cout][9][CinPad], scale[Cout], shift[Cout]
 *     (conv1 12->256 CinPad 16, conv2 256->512, 10 residual convs 512->512)
 *   head.w[3][512] head.scale[3] head.shift[3]   (policy_conv x2, value_conv)
 *   pfc.w[4096][128] pfc.b[4096] vfc1.w[512][64] vfc1.b[512] vfc2.w[512] vfc2.b[1]
 */
typedef struct kv_net kv_net;

size_t kv_net_packed_size(void);
int kv_net_create(int device, kv_net** out);
int kv_net_load(kv_net* net, const float* packed, size_t n_floats);
/* planes_dev: [B][12][8][8] fp32 (encode_board layout, ai/ai.py:17-30);
 * policy_dev: [B][4096] logits; value_dev: [B] tanh value. Any B >= 1: a batch of more than 16,384
 * boards (the tower's 32-bit workspace offsets) runs as equal slices of at most 16,384, each in the same
 * size class (> 16 boards) as the whole batch, so every output is the one a single pass would give. The same
 * holds for the two board-code forwards below. */
int kv_net_forward(kv_net* net, const float* planes_dev, int B, float* policy_dev, float* value_dev, void* stream);
/* boards_dev: [B][64] int8 piece codes (0 empty, 1..6 wK wQ wR wB wN wp,
 * 7..12 bK bQ bR bB bN bp; square r*8+c, row 0 = rank 8). */
int kv_net_forward_boards(kv_net* net, const int8_t* boards_dev, int B, float* policy_dev, float* value_dev,
                          void* stream);
/* The same forward with only the listed moves' logits (the MCTS leaves' legal
 * moves): moves_dev [B][maxm] move words (from | to << 6, as kv_dev_valid_moves),
 * n_moves_dev [B] (0: no logits for that board; values above maxm are read as
 * maxm -- a row holds maxm moves); legal_dev [B][maxm] receives
 * policy logit (from*64 + to) of each listed move, bit-identical to the
 * corresponding entry of kv_net_forward_boards; value_dev [B]. */
int kv_net_forward_boards_legal(kv_net* net, const int8_t* boards_dev, int B, const uint16_t* moves_dev,
                                const int* n_moves_dev, int maxm, float* legal_dev, float* value_dev, void* stream);
/* per-launch timing of the last forward (HIP events on `stream`): ms of the
 * residual conv launches summed, and count of those launches. */
int kv_net_last_timing(kv_net* net, float* conv_ms, int* n_conv);
/* Arithmetic of the 3x3 convs with Cin 256/512 (the stem conv, the heads and
 * the activations between layers are fp32 in every mode):
 * KV_PREC_FP32   fp32 (default; the parity mode). Under KV_ALGO_AUTO the net
 *                picks its conv path per weight load by measuring the
 *                candidates against an fp64 forward (kv_net_calibration).
 * KV_PREC_F64W   Winograd F(8x8) with every Winograd-domain quantity (U, V, M,
 *                transforms) in fp64, on v_mfma_f64_16x16x4_f64, at every batch
 *                size: logits within ~3e-6 of an fp64 forward on every weight set
 *                measured.
 * KV_PREC_I8X5   the same fp64 Winograd domain with the GEMMs on the int8
 *                matrix cores: every V / U row scaled by a power of two and
 *                split into 5 int8 digits, the 15 digit products of weight
 *                >= 2^-28 accumulated exactly in int32 and combined in fp64
 *                (per-row 35-bit block fixed point, 15 of 25 digit pairs: within
 *                ~2^-36 of the fp64 product per element); logits
 *                as close to fp64 as KV_PREC_F64W's, at every batch size (the
 *                fp32 AUTO fallback for trained weights before F64W).
 * KV_PREC_I8R4   the same fp64 domain with 4 radix-256 digits per value
 *                (31-bit block fixed point: N = rint(a 2^(31-e)) split into
 *                balanced bytes) and the 13 digit pairs i + j <= 4 of 16:
 *                13 int8 GEMMs instead of 15 over 4 digit planes instead of
 *                5 (AUTO's candidate before KV_PREC_I8X5).
 * Values 1 and 2 (bf16x3 / bf16x6) were retired in round 4, 3 (f16x3: F(4x8) GEMMs on fp16 MFMA with both
 * operands split in two fp16 pieces) in round 6 -- no configuration chose them: KV_EINVAL. */
#define KV_PREC_FP32 0
#define KV_PREC_F64W 4
#define KV_PREC_I8X5 5
#define KV_PREC_I8R4 6
int kv_net_set_precision(kv_net* net, int precision);
/* Algorithm of the fp32 3x3 convs with Cin 256/512:
 * KV_ALGO_AUTO      per weight load, the fastest path whose logits / values are
 *                   within 4e-5 / 4e-6 of an fp64 forward on 64 calibration
 *                   boards (the initial position, 16 positions of reference
 *                   self-play, 47 seeded random ones): > 16 boards F(8x8) fp32
 *                   on 3 radix-256 int8 digits (KV_ALGO_WINOGRAD88_I8R3),
 *                   else on 4 radix-128 ones (KV_ALGO_WINOGRAD88_I8), else the
 *                   same with fp64 input transforms (KV_ALGO_WINOGRAD88_I8V),
 *                   else the fp64 Winograd domain on 4 radix-256 int8
 *                   digits (KV_PREC_I8R4), else on fp64 MFMA; <= 16 boards
 *                   direct (split-K), else F(8x8)
 *                   fp64 (kv_net_calibration reports it)
 * KV_ALGO_DIRECT    implicit GEMM over the 9 taps (exact fp32 products)
 * KV_ALGO_WINOGRAD88 F(8x8,3x3): 100 GEMMs of 1 tile x Cin x Cout per board,
 *                   5.76x fewer FLOPs than direct (fp32 MFMA)
 * KV_ALGO_WINOGRAD88_I8 the F(8x8) fp32 tower (fp32 U, V, M, transforms) with
 *                   each GEMM on 4 int8 digits per value: per-row 28-bit
 *                   block fixed point, the 10 digit pairs i + j <= 3, exact
 *                   int32 levels, one rounding to fp32, on
 *                   v_mfma_i32_32x32x32_i8
 * KV_ALGO_WINOGRAD88_I8V the same tower with each conv's V the fp64 input
 *                   transform of its fp32 input, cut to 4 digits from fp64
 *                   (M, the output transform and the activations stay fp32)
 * KV_ALGO_WINOGRAD88_I8R3 the fp32 tower of KV_ALGO_WINOGRAD88_I8 with each
 *                   GEMM on 3 radix-256 int8 digits per value: per-row 24-bit
 *                   block fixed point (N = rint(a 2^(23-e)) as balanced
 *                   bytes), the 6 digit pairs i + j <= 2 of 9, exact int32
 *                   levels, one rounding to fp32 -- 6 int8 GEMMs per point
 *                   instead of 10 (AUTO's first candidate)
 * Values 2 (F(4x4)) and 3 (F(4x8)) were retired in rounds 4 and 6: KV_EINVAL. Setting the precision or
 * the algorithm of a loaded net re-prepares it (synchronous).
 * Results are batch-invariant inside a class (<= 16 boards, > 16 boards). */
#define KV_ALGO_AUTO 0
#define KV_ALGO_DIRECT 1
#define KV_ALGO_WINOGRAD88 4
#define KV_ALGO_WINOGRAD88_I8 5
#define KV_ALGO_WINOGRAD88_I8V 6
#define KV_ALGO_WINOGRAD88_I8R3 7
int kv_net_set_algo(kv_net* net, int algo);
/* conv paths (what a forward runs) */
#define KV_PATH_DIRECT 0
#define KV_PATH_WINO88 2
#define KV_PATH_WINO88_F64 3
#define KV_PATH_WINO88_I8 5     /* (1 and 4, the retired F(4x8) towers, stay unused indices) */
#define KV_PATH_WINO88_I8F32 6
#define KV_PATH_WINO88_I8F32V 7
#define KV_PATH_WINO88_I8R 8
#define KV_PATH_WINO88_I8F32R3 9
#define KV_NPATH 10
typedef struct {
    int calibrated;      /* 1: the last load / setting ran the fp32 AUTO calibration */
    int path_large;      /* KV_PATH_* of batches > 16 boards (also without calibration) */
    int path_small;      /* KV_PATH_* of batches <= 16 boards */
    int n_boards;        /* calibration boards */
    double tol_logit;    /* budget: max |logit - fp64| */
    double tol_value;    /* budget: max |value - fp64| */
    double err_logit[KV_NPATH]; /* > 16-board candidates measured, per path (-1: not run) */
    double err_value[KV_NPATH];
    double err_small_logit;     /* the <= 16-board direct path on 16 of the boards */
    double err_small_value;
    double ms;                  /* wall time of the calibration */
} kv_calib;
int kv_net_calibration(kv_net* net, kv_calib* out);
int kv_net_set_timing(kv_net* net, int enable);
void kv_net_destroy(kv_net* net);

/* ------------------------------------------------------------- engine ---
 * Self-play engine (replaces scripts/self_play.py self_play :258-291 /
 * _run_single_game :111-255 / _init_worker :52-85 state).
 */
#define KV_SEED_PER_GAME 0   /* game g seeded SEED+g in both streams, no carried eval */
#define KV_SEED_SEQUENTIAL 1 /* one numpy + one CPython stream seeded SEED, games in order */

#define KV_EVAL_FAITHFUL 0 /* every board evaluated once, as the reference does */
#define KV_EVAL_LAZY 1     /* the network runs only on the rows the schedule consumes (reference move
                              selection): <= 16 slots, all slots' rows on the steps where one is
                              consumed (the sequential drop-in path); above, the consumed rows as one
                              compact batch. Identical outputs, ~1/SELFPLAY_BATCH_SIZE of the network
                              work -- the reference evaluates every board and reads one row in 16 */
#define KV_EVAL_HASH 2     /* TEST ONLY: uniform logits + hash value instead of the network */

typedef struct {
    int device;
    int slots;            /* concurrent games on this GPU */
    int64_t n_games;      /* games to play (global ids game_id_base + k*game_id_stride) */
    int64_t game_id_base; /* first global game id on this rank */
    int64_t game_id_stride;
    uint64_t seed;        /* SEED (self_play.py:24) */
    int seed_mode;        /* KV_SEED_* */
    int max_moves;        /* <= 0: None */
    int batch;            /* SELFPLAY_BATCH_SIZE (self_play.py:34) */
    double eps;           /* DIR_NOISE_EPS */
    double alpha;         /* DIR_NOISE_ALPHA, a normal double in (0,1) (numpy's legacy gamma shape < 1
                             branch, restated exactly down to subnormal / zero draws; a ply whose 4096
                             draws are all 0 fails kv_run with KV_EINVAL, as the reference's
                             random.choices raises ValueError on the NaN weights) */
    int sims;             /* 0: reference move selection; 1..KV_MAX_SIMS: PUCT MCTS sims/move */
    float c_puct;
    int eval_mode;        /* KV_EVAL_* */
    int64_t record_cap;   /* record buffer capacity (records, one per committed ply; <= 0: 2^20); a run that
                             fills it fails with KV_EOVERFLOW ("record buffer full"), never a silent drop */
    int recycle;          /* 1: a finished slot starts the next game id */
    int precision;        /* KV_PREC_* of the network convs */
    int algo;             /* KV_ALGO_* of the network convs */
    int tree_edge_cap;    /* MCTS edges per slot; <= 0: KV_MAXM x (sims + 1), which cannot overflow. An
                             expansion that does not fit raises KV_EOVERFLOW (kv_stats.tree_overflows) */
    int keep_root_visits; /* 1: keep each MCTS move's root visit counts (pi) for kv_root_visits[_device] */
} kv_config;

#define KV_MAXM 320 /* move-list capacity per position */
#define KV_MAX_SIMS 65000 /* MCTS edges keep 16-bit visit counts and child node ids */

typedef struct {
    int64_t game_id;
    int32_t ply;
    uint16_t move;       /* encode_move index (ai/ai.py:51-57) */
    uint16_t pad;
    int8_t board[64];    /* position before the move (encode_board input) */
} kv_record;             /* 80 bytes */

typedef struct {
    int64_t game_id;
    int32_t plies;
    int32_t outcome;     /* +1 white win, 0 draw, -1 black win (self_play.py:211-238) */
    float reward;        /* 1.0 / 0.2 / -1.0 (self_play.py:245-250) */
    int32_t reason;      /* 0 max_moves 1 resign 2 mate 3 stalemate 4 draw 5 material */
    int32_t n_evals;     /* network rows consumed by this game's schedule */
    int32_t pad;
} kv_game;               /* 32 bytes */

typedef struct {
    int64_t steps;        /* ply-steps executed */
    int64_t plies;        /* moves committed */
    int64_t games_done;
    int64_t nn_rows;      /* boards evaluated by the network */
    int64_t sims;         /* MCTS backups completed */
    int64_t records;
    double res_conv_ms;   /* device time of the measured dominant-kernel launches (HIP events):
                             direct: the 10 residual convs of each forward; Winograd: one
                             residual GEMM launch per forward */
    int64_t res_conv_launches;
    double step_ms;       /* wall time inside kv_run */
    double dom_flop;      /* MFMA FLOPs of one measured launch (padded rows included) */
    int64_t dom_algo;     /* KV_ALGO_DIRECT or _WINOGRAD88 for those launches */
    int64_t tree_overflows; /* MCTS expansions dropped for a full edge pool (each also fails kv_run) */
    int64_t nn_rows_lazy;   /* KV_EVAL_LAZY above 16 slots: rows the compact batches sent through the
                               network (nn_rows counts the rows the reference's schedule evaluates) */
    int64_t dom_path;       /* KV_PATH_* of those launches (F(8x8) fp32 or fp64 for KV_ALGO_WINOGRAD88) */
    int64_t dom_split;      /* fp32 F(8x8): points of the GEMM layer run as 128x128 tiles in its first launch
                               (the rest as 64x128 tiles in a second one; 100: one launch); 0 otherwise */
    char dom_kernel[96];    /* the name of the kernel those launches ran, as the library chose it (template
                               arguments included, e.g. "wino88i32_gemm_lagt_kernel<512,5>") */
} kv_stats;

typedef struct kv_engine kv_engine;

int kv_create(const kv_config* cfg, kv_engine** out);
/* Loads the network weights; under fp32 + KV_ALGO_AUTO this runs the conv-path
 * calibration (kv_net_calibration), reported by kv_engine_calibration. */
int kv_load_weights(kv_engine* e, const float* packed, size_t n_floats);
int kv_engine_calibration(kv_engine* e, kv_calib* out);
/* Run ply-steps until every game is finished, or max_steps steps (>= 0), or
 * stop_after_games games have finished in total (>= 0), whichever is first. */
int kv_run(kv_engine* e, int64_t max_steps, int64_t stop_after_games);
/* max_moves for games from now on (_run_single_game's max_moves argument) */
int kv_set_max_moves(kv_engine* e, int max_moves);
int kv_records(kv_engine* e, kv_record* out, size_t cap, size_t* n);
/* The same records, unsorted (allocation order), copied device-to-device into
 * out_dev (a device buffer of cap records on the engine's GPU) on `stream`:
 * the experience stays in HBM for the RCCL gather. out_dev
 * NULL: only *n. The engine's next kv_run / kv_reset_records waits for the
 * copy on its own stream (an event recorded on `stream`), and kv_destroy
 * waits for it before freeing the buffer. */
int kv_records_device(kv_engine* e, kv_record* out_dev, size_t cap, size_t* n, void* stream);
/* finished games (the last 2^20 at most), ordered by game id */
int kv_games(kv_engine* e, kv_game* out, size_t cap, size_t* n);
/* drop the records collected so far (between kv_run calls) */
int kv_reset_records(kv_engine* e);
int kv_stats_get(kv_engine* e, kv_stats* out);
/* MCTS root visit counts of every committed move (keep_root_visits = 1):
 * out [n][KV_MAXM] in root move-list order, -1 padded, rows in kv_records'
 * order. No reference counterpart (the reference has no search); used by the
 * parity tests against the oracle's PUCT restatement. */
int kv_root_visits(kv_engine* e, int32_t* out, size_t cap, size_t* n);
/* the same visit counts (pi of the (s, pi, z) training triple, BASELINE config C4) device to device, uint16
 * [n][KV_MAXM] in the engine's record order -- row k belongs to record k of kv_records_device (0xffff past the
 * position's move list); stream as in kv_records_device */
int kv_root_visits_device(kv_engine* e, uint16_t* out_dev, size_t cap, size_t* n, void* stream);
int kv_sync(kv_engine* e);
void kv_destroy(kv_engine* e);

/* ------------------------------------------------- device test entry points ---
 * Run one device kernel over host-provided inputs (copies in and out). They
 * exist so parity tests can call the product kernels through the C ABI. */

/* getValidMoves (core/chessEngine.py:277-321) for n states (80-byte vectors,
 * see oracle/kv_oracle.c); moves_out [n][cap] as uint16 from|to<<6|flags<<12
 * (flags bit0 ep, bit1 castle, bit2 promotion); n_moves [n]; states_after
 * [n][80] (the reference may mutate the board); in_check [n]. */
int kv_dev_valid_moves(int device, const int8_t* states, int n, uint16_t* moves_out, int cap, int* n_moves,
                       int8_t* states_after, uint8_t* in_check);
/* squareUnderAttack (chessEngine.py:400-415) for all 64 squares: bit r*8+c of
 * attacked[i] is set when an opponent pseudo-move of state i ends on (r, c);
 * inCheck (:388-394) is the bit of the mover's stored king location. */
int kv_dev_attacks(int device, const int8_t* states, int n, uint64_t* attacked);
/* makeMove (chessEngine.py:127-197) of move index[i] of each state's list. */
int kv_dev_make_move(int device, int8_t* states, const int* index, int n);
/* numpy RandomState(seed[i]).dirichlet([alpha]*k) `draws` times per stream:
 * out [n][draws][k] fp64, attempts [n][draws] gamma attempts consumed,
 * tail [n] = the stream's next random_sample() after the draws. */
int kv_dev_dirichlet(int device, const uint64_t* seeds, int n, double alpha, int k, int draws, double* out,
                     int64_t* attempts, double* tail);
/* The device's restatement of glibc log (op 0: out = log(x)) / pow (op 1:
 * out = pow(x, y)) (csrc/kv_libm.h, used by the Dirichlet draw), run on the
 * host CPU: the same source compiled for the host, so tests can pin it against
 * libm itself without a GPU. */
int kv_host_libm(int op, const double* x, const double* y, int n, double* out);
/* CPython random.Random(seed[i]): count random() values -> out [n][count]. */
int kv_dev_py_random(int device, const uint64_t* seeds, int n, int count, double* out);
/* The int8-digit Winograd GEMM of one conv layer (csrc/kv_wino88i.h): V [100][rows][K]
 * and U [100][512][K] fp64 (K 256 or 512, rows a multiple of 128) are split into
 * `digits` int8 digits by the product's slice kernel and multiplied by its GEMM
 * kernel: M [100][rows][512] (digits 5: KV_PREC_I8X5's fp64 M; 4: the fp32
 * domain's (KV_ALGO_WINOGRAD88_I8) fp32 M, widened); v_digits (5 digits: planes
 * [100][K/32][5][rows][32]; 4 digits: row lines [100][K/32][rows][4][32]) and
 * v_exp [100][rows] (either may be NULL) return V's digits and row exponents. seg 1 (4 digits, K 512):
 * V's exponents per 256-channel segment (v_exp [100][2][rows]), the fp32 tower's A/B form. seg 2 (4 digits):
 * KV_PREC_I8R4's 4 radix-256 digits in row lines [100][K/32][rows][4][32], its GEMM and fp64 M. seg 3
 * (4 digits): KV_ALGO_WINOGRAD88_I8R3's 3 radix-256 digits in 96-byte row lines [100][K/32][rows][3][32] (the
 * first 3/4 of v_digits, the rest zero), the product's 6-pair GEMM and fp32 M. */
int kv_dev_wino88i(int device, const double* V, int rows, const double* U, int K, int digits, int seg, double* M,
                   int8_t* v_digits, int* v_exp);
/* The fp32 tower's residual output kernel on int8 digits (KV_ALGO_WINOGRAD88_I8): M [100][rows][512] fp32
 * (rows a multiple of 128), folded BN scale / shift [512], resid [rows][64][512] or NULL -> Y
 * [rows][64][512] (= ReLU(A^T M A * scale + shift (+ resid))) and the next conv's V as row-line digits
 * [100][16][rows][4][32] with row exponents [100][rows]. fused bit 0 set: the product's one-kernel form
 * (KV_I8F32_OUT's choice; with bit 3 also set the 64-register wino88i32_out2_kernel, with bit 5 the
 * persistent LDS-DMA wino88i32_outp_kernel; bit 4: 3 radix-256 digits, KV_ALGO_WINOGRAD88_I8R3's, in 96-byte
 * lines [100][16][rows][3][32] in the first 3/4 of v_digits, the rest zero), clear:
 * wino88_out_kernel's fp32 V then the slice kernel (bit-identical); bit 1:
 * exponents per 256-channel segment ([100][2][rows]) instead of per row; bit 2 (KV_ALGO_WINOGRAD88_I8V's V,
 * per row): with bit 0 the one-kernel wino88i32v_out_kernel, without it wino88_out_kernel's Y, then
 * wino88d_in_kernel's fp64 V and the slice kernel (bit-identical). */
int kv_dev_wino88i32_out(int device, const float* M, int rows, const float* scale, const float* shift,
                         const float* resid, int fused, float* Y, int8_t* v_digits, int* v_exp);
/* KV_PREC_I8R4's output step: M [100][rows][512] fp64 (rows a multiple of 128), folded BN scale / shift,
 * resid or NULL -> Y [rows][64][512] and the next conv's V as 4 radix-256 digits in row lines
 * [100][16][rows][4][32] with row exponents [100][rows]. fused 1: the product's wino88i64r_out_kernel; 0:
 * wino88d_out_half_kernel's Y, wino88d_in_kernel's fp64 V, the radix-256 slice kernel (bit-identical). */
int kv_dev_wino88r_out(int device, const double* M, int rows, const float* scale, const float* shift,
                       const float* resid, int fused, float* Y, int8_t* v_digits, int* v_exp);
/* Timing / A-B harness of the fp32 tower's int8-digit GEMM on seeded random digits (rows boards, K 256 or
 * 512): variant 0 the round-4 kernel, 1.. round-5 forms (persistent / per-tile, k per stage, ring depth);
 * avg_us = mean HIP-event time of `iters` launches; M_out [100][rows][512] (optional) for a bit-for-bit
 * comparison of the variants. */
int kv_dev_i8gemm_bench(int device, int rows, int K, int variant, int iters, float* avg_us, float* M_out);
/* The clock the chip holds under the headline GEMM (a diagnostic; MI355X_MICROARCH.md "DVFS give-back" item 6):
 * the product's fp32-tower GEMM (K 512, `rows` boards, `digits` 4 or 3 (KV_ALGO_WINOGRAD88_I8R3), seeded random
 * digits) back to back for `seconds`, then
 * one launch of its stamped build: out[0] = median over workgroups of (s_memtime delta / s_memrealtime delta)
 * x 100 MHz, out[1] = the back-to-back launches' mean time (us), out[2] = their count, out[3] = tiles per
 * workgroup of the stamped kernel. */
int kv_dev_gemm_clock(int device, int rows, int digits, double seconds, double* out);
/* Phase timing of the fp32 tower's output kernel (a diagnostic build of wino88i32_out_kernel with shader-clock
 * stamps) at `rows` boards on seeded M (resid: the residual + Y variant; r3: 3 radix-256 digits): stamps
 * [min(rows, 4096)][2][6] = s_memtime of waves 0 and 15 of each board's workgroup at start, V ready, after the
 * maxima barrier, after the exponent barrier, digit stores issued, stores drained; us = that launch's time. */
int kv_dev_out_phases(int device, int rows, int resid, int r3, unsigned long long* stamps, float* us);

/* ------------------------------------------------------- data pipeline ---
 * Full-rules chess (python-chess 1.999 semantics, csrc/kv_chess.cpp) for the
 * reference's PGN -> JSONL ingestion and its JSONL datasets. Host code: no
 * GPU is touched. Squares here are python-chess's (a1 = 0, h8 = 63).
 *
 * kv_pgn_extract replaces data_utils/parser_pgn.py:81-118
 * extract_data_from_pgn's loop (chess.pgn.read_game + board.fen() /
 * board.san(move) / board.push(move) per mainline move): one record per
 * mainline move of every game in `text`, in file order. Stops before a game
 * whose records would not fit in `cap` and reports in *consumed the bytes of
 * `text` processed (whole games), so callers loop over large inputs;
 * KV_EOVERFLOW if a single game does not fit (*n_out = its move count). */
#define KV_PGN_OUTCOME_NONE (-128) /* Result "*" or unknown: the reference's `outcome = None` */
typedef struct kv_pgn_record {
    char fen[100];   /* board.fen() before the move, NUL-terminated */
    char san[12];    /* board.san(move) */
    int32_t outcome; /* 1 ("1-0"), -1 ("0-1"), 0 ("1/2-1/2"), KV_PGN_OUTCOME_NONE */
    int32_t game;    /* index of the game within this call */
} kv_pgn_record;
int kv_pgn_extract(const char* text, size_t len, kv_pgn_record* out, size_t cap, size_t* n_out, size_t* consumed,
                   int64_t* n_games);
/* fen_to_tensor's piece scan (data_utils/dataset.py:59-68, scripts/train.py:531-545):
 * n FENs, `stride` bytes apart (NUL-terminated) -> codes[n][64] int8, 0 empty,
 * 1..12 = P N B R Q K p n b r q k (the PGN plane order + 1), index row*8+col
 * with row 0 = rank 8. */
int kv_fen_codes(const char* fens, size_t stride, int n, int8_t* codes);
/* ChessPGNDataset.default_move_encoder (scripts/train.py:553-558):
 * board.parse_san(san) -> from_square*64 + to_square. */
int kv_san_move_index(const char* fens, size_t fen_stride, const char* sans, size_t san_stride, int n,
                      int32_t* out);
/* test / tooling entry points: perft node count, SAN round trip (parse_san ->
 * san, fen after push), Board(fen).fen() */
int kv_chess_perft(const char* fen, int depth, uint64_t* nodes);
int kv_chess_san(const char* fen, const char* san_in, char* san_out, size_t san_cap, char* fen_after, size_t fen_cap);
int kv_chess_fen(const char* fen_in, char* fen_out, size_t cap);

/* --------------------------------------------------------------- train ---
 * Update-step kernels of the learn loop. The reference
 * trains ChessNet under torch.cuda.amp.autocast (scripts/train.py:161-184):
 * its 3x3 convolutions (ai/model.py:34-40, :8-25) run on fp16 operands with
 * fp32 accumulation and fp16 outputs, its BatchNorms in training mode (fp32
 * batch statistics, fp16 output). These entry points restate those units for
 * the tower (conv1, conv2, the 5 residual blocks), replacing the MIOpen
 * convolutions / BatchNorms torch calls there (knightvision_amd/train_ops.py
 * wraps them as autograd functions). Activations are NHWC fp16 device arrays
 * [n boards][64 squares][C]; weights fp16 [co][9][ci] (tap = 3 * row + col of
 * the 3x3 kernel); every call is asynchronous on `stream`.
 */
/* y = bias + conv3x3(x, w), pad 1 on the 8x8 board; ci % 16 == 0, co % 128 == 0;
 * bias_dev fp32 [co] or NULL. Also the data gradient: x = dy, w = the flipped
 * image of kv_tr_conv_weights_f16, co = the conv's input channels. */
int kv_tr_conv3x3_f16(const void* x_dev, int n, int ci, const void* w_dev, const float* bias_dev, int co,
                      void* y_dev, void* stream);
/* the same with a fused fp16 addend: y = fp16(float(fp16(bias + conv3x3(x, w))) + float(add)) -- the data
 * gradient of a residual block's first conv plus the residual branch's gradient, rounded as autograd's
 * fp16 gradient accumulation rounds it; add_dev [n][64][co] (not y_dev) or NULL */
int kv_tr_conv3x3_add_f16(const void* x_dev, int n, int ci, const void* w_dev, const float* bias_dev, int co,
                          const void* add_dev, void* y_dev, void* stream);
/* fp32 torch weight [co][ci_real][3][3] -> fp16 forward image [co][9][ci] (channels >= ci_real zero) and,
 * if wt_dev != NULL, the data-gradient image [ci][9][co] (taps flipped) */
int kv_tr_conv_weights_f16(const float* w_dev, int co, int ci_real, int ci, void* wf_dev, void* wt_dev, void* stream);
/* bytes of workspace kv_tr_conv3x3_wgrad_f16 needs (and the board splits it uses) */
size_t kv_tr_wgrad_workspace(int n, int ci, int co, int* splits);
/* dw fp32 [co][ci_real][3][3] = fp16-rounded sum over boards and squares of dy (x) shifted x;
 * ci % 64 == 0, co % 64 == 0; deterministic (fixed split order) */
int kv_tr_conv3x3_wgrad_f16(const void* dy_dev, const void* x_dev, int n, int ci, int ci_real, int co, float* dw_dev,
                            void* ws_dev, size_t ws_bytes, void* stream);
/* bytes of workspace the BatchNorm / channel-sum calls need for rows x C */
size_t kv_tr_bn_workspace(int rows, int C);
/* training BatchNorm statistics over rows (= boards x 64) of fp16 x: mean, biased var, 1/sqrt(var + eps) */
int kv_tr_bn_stats_f16(const void* x_dev, int rows, int C, float eps, float* mean_dev, float* var_dev,
                       float* invstd_dev, void* ws_dev, size_t ws_bytes, void* stream);
/* y = fp16((x - mean) * invstd * gamma + beta); res_dev != NULL: y = fp16(y + res); relu: max(y, 0) */
int kv_tr_bn_apply_f16(const void* x_dev, int rows, int C, const float* mean_dev, const float* invstd_dev,
                       const float* gamma_dev, const float* beta_dev, const void* res_dev, int relu, void* y_dev,
                       void* stream);
/* backward of kv_tr_bn_apply_f16 (y_dev = its output, for the ReLU mask): dgamma, dbeta fp32 [C], dx fp16 and,
 * if dres_dev != NULL, the residual's gradient (the masked dy); if dxsum_dev != NULL, the channel sums of dx
 * fp32 [C] (the bias gradient of the conv that produced x, without a second pass over dx) */
int kv_tr_bn_backward_f16(const void* x_dev, const void* dy_dev, const void* y_dev, int rows, int C, int relu,
                          const float* mean_dev, const float* invstd_dev, const float* gamma_dev, float* dgamma_dev,
                          float* dbeta_dev, void* dx_dev, void* dres_dev, float* dxsum_dev, void* ws_dev,
                          size_t ws_bytes, void* stream);
/* per-channel sum of fp16 rows x C (a conv bias gradient) */
int kv_tr_channel_sum_f16(const void* x_dev, int rows, int C, float* sum_dev, void* ws_dev, size_t ws_bytes,
                          void* stream);
/* the heads' 1x1 convolutions (policy 512 -> 2, value 512 -> 1; ai/model.py:42-49) over rows = boards x 64 of
 * the tower output h fp16 [rows][512]: w fp16 [3][512] (policy rows 0-1, value row 2), b fp32 [3] (fp16 values);
 * out fp16 [rows][4] (column 3 unused) */
int kv_tr_head1x1_f16(const void* h_dev, int rows, const void* w_dev, const float* b_dev, void* out_dev,
                      void* stream);
size_t kv_tr_head1x1_workspace(int rows);
/* its backward from dout fp16 [rows][4]: dh fp16 [rows][512], dw fp32 [3][512], db fp32 [3] (fp16-rounded) */
int kv_tr_head1x1_backward_f16(const void* h_dev, const void* dout_dev, int rows, const void* w_dev, void* dh_dev,
                               float* dw_dev, float* db_dev, void* ws_dev, size_t ws_bytes, void* stream);
/* encode_board planes fp32 [n][12][8][8] (ai/ai.py:17-30) -> NHWC fp16 [n][64][cpad], channels >= 12 zero */
int kv_tr_planes_to_nhwc(const float* planes_dev, int n, int cpad, void* out_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KV_H */
