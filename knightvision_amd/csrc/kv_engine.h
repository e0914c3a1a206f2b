// Shared device state of the self-play engine (kv_engine.hip: reference
// move selection; kv_mcts.hip: PUCT search).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kv_common.h"
#include "kv_movegen.h"
#include "kv_rng.h"

#pragma clang fp contract(off)

namespace kv {

int net_forward_boards_internal(kv_net* net, const int8_t* boards_dev, int B, float* policy, float* value,
                                hipStream_t st);
int net_forward_boards_legal_internal(kv_net* net, const int8_t* boards_dev, int B, const uint16_t* moves,
                                      const int* n_moves, int maxm, float* legal, float* value, hipStream_t st);
int net_set_res_events(kv_net* net, hipEvent_t a, hipEvent_t b);
void net_dom_info(const kv_net* net, int* algo, int* launches, double* flop, int* path, int* split,
                  const char** kernel);

enum : int { ST_IDLE = 0, ST_ACTIVE = 1, ST_FINISHED = 2 };
enum : int { END_NONE = 0, END_NOMOVES = 1, END_DRAW = 2, END_RESIGN = 3, END_MAXED = 4 };

struct Slot {
    long long game_id;
    int status;
    int ply;
    int wtm, wkr, wkc, bkr, bkc, flags, ep;
    int nmoves;
    int buf;
    int has_last;
    float last_value;
    int consumed;
    int need_flush;
    int n_evals;
    int end_kind;
    int outcome;
    int reason;
    int rows_total;   // network rows this slot has appended (all its games; k_count sums them)
    int plies_total;  // moves this slot has committed (all its games)
    int movegen_clean;  // k_movegen's getValidMoves left the position as it found it
    int pad[8];
};
static_assert(sizeof(Slot) == 128, "slot is one cache line");

struct Ctr {
    unsigned long long rec_count;
    unsigned long long games_count;
    unsigned long long next_game;
    unsigned long long plies;
    unsigned long long nn_rows;
    unsigned long long sims;
    unsigned long long nn_rows_slots;  // k_count: sum of Slot::rows_total (nn_rows adds the MCTS leaf rows)
    unsigned long long tree_overflows;  // MCTS expansions that did not fit the slot's pools (error flag 4)
    int active;
    int error;
    int need_eval;  // KV_EVAL_LAZY: some slot consumes a network row this step
    int comp_rows;  // KV_EVAL_LAZY above 16 slots: network rows of this step's compact batch
};

struct DevCfg {
    int slots;
    long long n_games;
    long long id_base, id_stride;
    unsigned long long seed;
    int seed_mode;
    int max_moves;
    int batch;
    double eps, alpha;
    long long record_cap;
    int recycle;
    int rows;  // NN rows per step (slots, or 2*slots with flush rows)
    long long games_cap;  // game-record ring capacity
    int sims;             // 0: reference move selection; >0: PUCT search
    int eval_mode;        // KV_EVAL_*
};

__device__ inline Pos slot_pos(const Slot& s, const int8_t* board) {
    Pos p;
    pos_from_board(p, board, s.wtm, s.wkr, s.wkc, s.bkr, s.bkc, s.flags, s.ep);
    return p;
}

__device__ inline void slot_store_pos(Slot& s, int8_t* board, const Pos& p) {
    pos_to_board(p, board);
    s.wtm = p.wtm;
    s.wkr = p.wkr; s.wkc = p.wkc; s.bkr = p.bkr; s.bkc = p.bkc;
    s.flags = p.flags;
    s.ep = p.ep;
}


struct MctsSlot {  // per-slot search scratch (kv_mcts.hip)
    int node_count;
    int edge_count;
    int path_len;
    int leaf_edge;
    int leaf_pending;  // 1: the leaf row is in this step's network batch
    int leaf_n;
    int leaf_wtm;
    float leaf_value;  // terminal value (white perspective) when !leaf_pending
    float root_value;
    int root_wtm;
    int overflow;      // expansions skipped because the slot's edge / node pool was full (an error)
    int pad[5];
};

constexpr uint16_t NO_CHILD = 0xffff;  // e_child of an unexpanded edge

struct __attribute__((aligned(16))) NodeRec {
    int first, cnt, N, pad;
};

struct Tree {  // per-slot SoA edge pools + node records, slot i at i*ecap / i*ncap
    uint16_t* e_move;
    float* e_P;
    uint16_t* e_N;      // visit count (<= sims <= KV_MAX_SIMS)
    float* e_W;
    uint16_t* e_child;  // child node id (< ncap) or NO_CHILD
    NodeRec* node;    // [slot][ncap]: first edge, edge count, visit count (one 16-B load per tree level)
    int* path;        // [slot][ncap]
    uint16_t* leaf_moves;  // [slot][MAXM]
    int* leaf_cnt;         // [slot]: moves of the leaf in this step's network batch (0: none)
    float* leaf_logits;    // [slot][MAXM]: their policy logits (kv_net_forward_boards_legal)
    MctsSlot* ms;
    const float* sqrt_tab;  // (float)sqrt((double)n), n < ncap + 2
    uint16_t* root_visits;  // optional [record_cap][MAXM]: root visit counts (pi) of each committed move, 0xffff padded
    int ecap, ncap;
    float c_puct;
    int sims;
};

__device__ inline float wave_max(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
    return v;
}
__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}

// torch.softmax over 4096 fp32 logits (self_play.py:150): max, exp(x-max),
// sum, x * (1/sum)
__device__ void wave_softmax_4096(const float* lg, float* out, int lane) {
    float v[64];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        v[j] = lg[j * 64 + lane];
        m = fmaxf(m, v[j]);
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        v[j] = expf(v[j] - m);
        s += v[j];
    }
    s = wave_sum(s);
    const float inv = 1.0f / s;
#pragma unroll
    for (int j = 0; j < 64; ++j) out[j * 64 + lane] = v[j] * inv;
}

// exp(x) for the MCTS priors (build-defined; no reference counterpart),
// made of IEEE double basic operations only -- Cody-Waite reduction by ln 2,
// degree-11 Taylor polynomial, exact power-of-two scaling, one rounding to
// float -- so that oracle/kv_oracle.c det_expf reproduces it bit for bit
// (ocml's expf and glibc's expf differ in the last bit). Results below
// e^-87 (float subnormals) are 0.
__device__ inline float det_expf(float x) {
    if (!(x >= -87.0f)) return 0.0f;
    const double xd = (double)x;
    const double kd = rint(xd * 1.4426950408889634);
    const double r = (xd - kd * 6.93147180369123816490e-01) - kd * 1.90821492927058770002e-10;
    double p = 2.5052108385441720e-08;  // 1/11!
    p = p * r + 2.7557319223985893e-07;
    p = p * r + 2.7557319223985888e-06;
    p = p * r + 2.4801587301587302e-05;
    p = p * r + 1.9841269841269841e-04;
    p = p * r + 1.3888888888888889e-03;
    p = p * r + 8.3333333333333332e-03;
    p = p * r + 4.1666666666666664e-02;
    p = p * r + 1.6666666666666666e-01;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    const double scale = __longlong_as_double((long long)((int)kd + 1023) << 52);
    return (float)(p * scale);
}

// softmax over 4096 logits with det_expf (MCTS root): max, e = det_expf(x -
// max), each lane sums its 64 entries j*64+lane in j order, xor-butterfly
// over the wave (offsets 32..1), x * (1/sum)
__device__ void wave_softmax_4096_det(const float* lg, float* out, int lane) {
    float v[64];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        v[j] = lg[j * 64 + lane];
        m = fmaxf(m, v[j]);
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        v[j] = det_expf(v[j] - m);
        s += v[j];
    }
    s = wave_sum(s);
    const float inv = 1.0f / s;
#pragma unroll
    for (int j = 0; j < 64; ++j) out[j * 64 + lane] = v[j] * inv;
}

// mixed legal weights of the reference (self_play.py:147-160) for a slot's
// move list: (1-eps)*softmax [fp32] + eps*dirichlet [fp64], in list order.
// Consumes the slot's numpy stream exactly as np.random.dirichlet does. All
// 256 threads of the slot's workgroup; gam is 4096 doubles of LDS.
__device__ inline void mixed_legal_weights(const DevCfg& cfg, const float* lp, const uint16_t* ml, int n,
                                           double* gam, uint32_t* np_state, uint32_t* mt_ring, int* scratch,
                                           double* vals, int tid) {
    BlockMT w;
    bmt_load(w, np_state, mt_ring, tid);
    long long att;
    const double acc = block_dirichlet_gamma(w, cfg.alpha, 4096, gam, &att, scratch, tid);
    bmt_store(w, np_state, tid);
    const double invacc = 1 / acc;
    const float keep = (float)(1.0 - cfg.eps);
    for (int j = tid; j < n; j += RNG_THREADS) {
        const int mv = ml[j];
        const int idx = (mv & 63) * 64 + ((mv >> 6) & 63);
        const float p32 = keep * lp[idx];
        const double noise = gam[idx] * invacc;
        vals[j] = (double)p32 + cfg.eps * noise;
    }
    __syncthreads();
}

// random.choices(population, weights) / random.choice when the total is 0
// (self_play.py:162-167, CPython random.py:506-541). Lane 0 only.
// the pick of random.choices for a non-zero total with r = random() already
// drawn (cum_weights by serial accumulation, bisect_right on r * total)
__device__ inline int choose_from(const double* vals, double* cum, int n, double total, double r) {
    double c = 0.0;
    for (int j = 0; j < n; ++j) {
        c = c + vals[j] / total;
        cum[j] = c;
    }
    const double tot = cum[n - 1] + 0.0;
    const double x = r * tot;
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (x < cum[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

__device__ inline int choose_weighted(const double* vals, double* cum, int n, uint32_t* py) {
    double total = 0.0;
    for (int j = 0; j < n; ++j) total = total + vals[j];
    if (total == 0.0) return mt_randbelow_serial(py, n);
    return choose_from(vals, cum, n, total, mt_random_serial(py));
}

// record the position + move, makeMove, then the reference's termination
// checks in order: isDraw (:180), resign (:185, `value` is the row the move
// was chosen with), max_moves (:196). All lanes of the slot's wave.
__device__ inline unsigned long long commit_move(const DevCfg& cfg, Slot& s, int i, int mv, int8_t* boards,
                                                 kv_record* rec, int8_t* last_board, Ctr* ctr, int lane) {
    // lane = thread index of the slot's workgroup; lanes 0..63 (wave 0) carry
    // the 64 squares, every thread reaches the barriers
    int8_t* board = boards + (size_t)i * 64;
    const bool sqlane = lane < 64;
    const unsigned long long r = lane == 0 ? atomicAdd(&ctr->rec_count, 1ull) : 0ull;
    const unsigned long long ridx = __shfl(r, 0);
    const int8_t sq = sqlane ? board[lane] : 0;
    if (sqlane) last_board[(size_t)i * 64 + lane] = sq;
    if ((long long)ridx < cfg.record_cap) {
        if (sqlane) rec[ridx].board[lane] = sq;
        if (lane == 0) {
            rec[ridx].game_id = s.game_id;
            rec[ridx].ply = s.ply;
            rec[ridx].move = (uint16_t)((mv & 63) * 64 + ((mv >> 6) & 63));
            rec[ridx].pad = 0;
        }
    } else if (lane == 0) {
        atomicOr(&ctr->error, 2);
    }
    __syncthreads();
    if (lane == 0) {
        make_move_board(board, s.wtm, s.wkr, s.wkc, s.bkr, s.bkc, s.flags, s.ep, mv);
        s.ply += 1;
        s.plies_total += 1;
    }
    __syncthreads();
    const int8_t b2 = sqlane ? board[lane] : 0;
    const bool non_king = b2 != 0 && b2 != 1 && b2 != 7;
    const bool draw = __ballot(non_king) == 0ull;
    if (lane == 0) {
        if (draw) {
            s.end_kind = END_DRAW;
        } else if (s.ply > 15 && (double)s.last_value < -0.7) {
            s.end_kind = END_RESIGN;
            s.outcome = s.wtm ? -1 : 1;
            s.reason = 1;
        } else if (cfg.max_moves > 0 && s.ply >= cfg.max_moves) {
            s.end_kind = END_MAXED;
        }
        if (s.end_kind != END_NONE) s.status = ST_FINISHED;
        s.consumed = 0;
    }
    return ridx;  // the record's index
}

// MCTS launches (kv_mcts.hip), all on `st`
int mcts_root(const DevCfg& cfg, const Tree& t, Slot* slots, const uint16_t* moves, const float* logits,
              const float* values, float* probs_scratch, uint32_t* np_mt, Ctr* ctr, hipStream_t st);
// select / backup for slots [slot0, slot0 + count)
int mcts_select(const DevCfg& cfg, const Tree& t, const Slot* slots, const int8_t* boards, int8_t* nn_boards,
                Ctr* ctr, hipStream_t st, int slot0, int count);
int mcts_backup(const DevCfg& cfg, const Tree& t, const Slot* slots, const float* logits, const float* values,
                float* probs, Ctr* ctr, hipStream_t st, int slot0, int count);
// backup of one sim-step fused with the next sim-step's select
int mcts_backup_select(const DevCfg& cfg, const Tree& t, const Slot* slots, const int8_t* boards, const float* logits,
                       const float* values, float* probs, int8_t* nn_boards, Ctr* ctr, hipStream_t st, int slot0,
                       int count);
int mcts_choose(const DevCfg& cfg, const Tree& t, Slot* slots, int8_t* boards, uint32_t* py_mt, kv_record* rec,
                int8_t* last_board, Ctr* ctr, hipStream_t st);
int hash_eval(const int8_t* boards, int rows, float* logits, float* values, hipStream_t st);
int hash_legal(const Tree& t, int rows, hipStream_t st);

}  // namespace kv
