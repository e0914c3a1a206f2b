// Self-play engine on MI355X: replaces scripts/self_play.py _run_single_game
// :111-255 / self_play :258-291 for `slots` concurrent games per GPU.
//
// One ply-step of every live game slot is four launches on one stream:
//   k_movegen  one wave per slot, lane = square: reference-exact legal list
//              (kv_movegen.h wave_valid_moves), game-over detection, SELFPLAY_BATCH_SIZE schedule bookkeeping
//   NN         ChessNet over the slots' boards (kv_nn.hip) -- every board is
//              evaluated once, as the reference does (faithful), or only the
//              rows the schedule consumes (lazy)
//   k_sample   one wave per slot: softmax of the consumed row, numpy-legacy
//              Dirichlet noise on the slot's own MT19937 (wave-parallel),
//              0.75/0.25 mix in the reference's fp32/fp64 order, CPython
//              random.choices on the slot's second stream, makeMove, record,
//              termination (draw / resign / max_moves)
//   k_finish   one wave per finished slot: outcome + reward exactly as :210-250, game
//              record, then the slot starts the next game id (recycling)
// The host only launches and, every few steps, reads one counter.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "kv_common.h"
#include "kv_movegen.h"
#include "kv_rng.h"
#include "kv_engine.h"

#pragma clang fp contract(off)

namespace kv {

__constant__ const int8_t kStart[64] = {9, 11, 10, 8, 7, 10, 11, 9, 12, 12, 12, 12, 12, 12, 12, 12,
                                        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                        6, 6, 6, 6, 6, 6, 6, 6, 3, 5, 4, 2, 1, 4, 5, 3};

// GameState() :34-84: the slot fields of a new game (board and streams set by the caller)
__device__ void start_game_fields(const DevCfg& cfg, Slot& s, long long gid) {
    s.game_id = gid;
    s.status = ST_ACTIVE;
    s.ply = 0;
    s.wtm = 1; s.wkr = 7; s.wkc = 4; s.bkr = 0; s.bkc = 4; s.flags = 0; s.ep = -1;
    s.nmoves = 0;
    s.buf = 0;
    s.consumed = 0;
    s.n_evals = 0;
    s.end_kind = END_NONE;
    s.outcome = 0;
    s.reason = -1;
    if (cfg.seed_mode == KV_SEED_PER_GAME) {
        s.has_last = 0;
        s.need_flush = 0;
    }
}

// GameState() + per-game seeding (_init_worker :81-85 with SEED+g), one thread
__device__ void start_game(const DevCfg& cfg, Slot& s, int8_t* board, uint32_t* np_mt, uint32_t* py_mt,
                           long long k) {
    const long long gid = cfg.id_base + k * cfg.id_stride;
    for (int i = 0; i < 64; ++i) board[i] = kStart[i];
    start_game_fields(cfg, s, gid);
    if (cfg.seed_mode == KV_SEED_PER_GAME) {
        const unsigned long long sd = cfg.seed + (unsigned long long)gid;
        mt_seed_genrand(np_mt, (uint32_t)sd);
        mt_seed_python(py_mt, sd);
    }
}

__global__ void k_init(DevCfg cfg, Slot* slots, int8_t* boards, uint32_t* np_mt, uint32_t* py_mt, Ctr* ctr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cfg.slots) return;
    Slot s;
    memset(&s, 0, sizeof(s));
    s.status = ST_IDLE;
    s.has_last = 0;
    s.need_flush = 0;
    if (cfg.seed_mode == KV_SEED_SEQUENTIAL) {  // one pair of streams seeded SEED (self_play.py:270)
        mt_seed_genrand(np_mt + (size_t)i * MT_WORDS, (uint32_t)cfg.seed);
        mt_seed_python(py_mt + (size_t)i * MT_WORDS, cfg.seed);
    }
    if ((long long)i < cfg.n_games) {
        start_game(cfg, s, boards + (size_t)i * 64, np_mt + (size_t)i * MT_WORDS, py_mt + (size_t)i * MT_WORDS, i);
        atomicAdd(&ctr->active, 1);
    }
    slots[i] = s;
}

// ------------------------------------------------------------- counts ----
// the per-ply counters from the slots themselves, one workgroup: active slots,
// and the running sums of the slots' committed plies and appended network rows
// (per-slot fields instead of one device-scope atomic per slot and kernel on a
// shared counter, which serialised across the XCDs at ~0.1 us each)
__global__ __launch_bounds__(256) void k_count(DevCfg cfg, const Slot* slots, Ctr* ctr) {
    __shared__ unsigned long long red[3][4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long a = 0, rows = 0, pl = 0;
    for (int j = tid; j < cfg.slots; j += 256) {
        a += slots[j].status == ST_ACTIVE;
        rows += (unsigned long long)slots[j].rows_total;
        pl += (unsigned long long)slots[j].plies_total;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        a += __shfl_xor(a, m);
        rows += __shfl_xor(rows, m);
        pl += __shfl_xor(pl, m);
    }
    if (lane == 0) {
        red[0][wave] = a;
        red[1][wave] = rows;
        red[2][wave] = pl;
    }
    __syncthreads();
    if (tid == 0) {
        ctr->active = (int)(red[0][0] + red[0][1] + red[0][2] + red[0][3]);
        ctr->nn_rows_slots = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        ctr->plies = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    }
}

// ------------------------------------------------------------ movegen ----
__global__ __launch_bounds__(64) void k_movegen(DevCfg cfg, Slot* slots, int8_t* boards, uint16_t* moves,
                                                Ctr* ctr) {
    const int i = blockIdx.x, lane = threadIdx.x;
    Slot s = slots[i];
    if (s.status != ST_ACTIVE) return;
    int8_t* board = boards + (size_t)i * 64;
    const int8_t before = board[lane];
    Pos p = wave_pos(before, s.wtm, s.wkr, s.wkc, s.bkr, s.bkc, s.flags, s.ep);
    const int n = wave_valid_moves(p, moves + (size_t)i * MAXM, MAXM, lane);
    const int8_t after = (int8_t)pos_at(p, lane);
    board[lane] = after;  // the reference may mutate the board (stale king, double check)
    const bool board_same = __ballot(after != before) == 0ull;
    if (lane != 0) return;
    if (n > MAXM) atomicOr(&ctr->error, 1);
    s.movegen_clean = board_same && p.wtm == s.wtm && p.wkr == s.wkr && p.wkc == s.wkc && p.bkr == s.bkr &&
                      p.bkc == s.bkc && p.flags == s.flags && p.ep == s.ep;
    s.wtm = p.wtm;
    s.wkr = p.wkr; s.wkc = p.wkc; s.bkr = p.bkr; s.bkc = p.bkc;
    s.flags = p.flags;
    s.ep = p.ep;
    s.nmoves = n < MAXM ? n : MAXM;
    if (n == 0) {
        s.end_kind = END_NOMOVES;
        s.status = ST_FINISHED;
        s.consumed = 0;
    } else {
        // buffer.append(board); eval when len >= BATCH_SIZE or nothing evaluated yet (:129-145)
        s.buf += 1;
        const bool has = s.has_last || s.need_flush;
        s.consumed = (s.buf >= cfg.batch) || !has;
        s.rows_total += 1;
    }
    if (s.consumed || s.need_flush) ctr->need_eval = 1;  // read by the host in KV_EVAL_LAZY
    slots[i] = s;
}

// ------------------------------------------------------------- sample ----
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_sample(DevCfg cfg, Slot* slots, int8_t* boards, const uint16_t* moves,
                                                const float* logits, const float* values, float* last_probs,
                                                uint32_t* np_mt, uint32_t* py_mt, kv_record* rec, int8_t* last_board,
                                                Ctr* ctr, const int* row_of) {
    __shared__ uint32_t mt3[MT_RW];
    __shared__ double gam[4096];
    __shared__ double vals[MAXM];
    __shared__ double cum[MAXM];
    __shared__ int scratch[RNG_SCRATCH];
    __shared__ int s_pick;
    const int i = blockIdx.x, lane = threadIdx.x;
    Slot s = slots[i];
    if (s.status != ST_ACTIVE) return;
    float* lp = last_probs + (size_t)i * 4096;
    if (s.need_flush) {  // previous game's final flush row (sequential mode)
        if (lane < 64) wave_softmax_4096(logits + (size_t)(cfg.slots + i) * 4096, lp, lane);
        s.last_value = values[cfg.slots + i];
        s.has_last = 1;
        s.need_flush = 0;
    }
    if (s.consumed) {  // policy/value = _last_outputs[...][-1] (:147-150)
        __syncthreads();
        const int row = row_of ? row_of[i] : i;  // the compact lazy batch's row of this slot
        if (lane < 64) wave_softmax_4096(logits + (size_t)row * 4096, lp, lane);
        s.last_value = values[row];
        s.has_last = 1;
        s.buf = 0;
        s.n_evals += 1;
    }
    __syncthreads();
    const int n = s.nmoves;
    const uint16_t* ml = moves + (size_t)i * MAXM;
    mixed_legal_weights(cfg, lp, ml, n, gam, np_mt + (size_t)i * MT_WORDS, mt3, scratch, vals, lane);
    // random.choices (:162-167): the total, then random() drawn by the whole
    // workgroup (a twist of the CPython state, every 312 plies of a game, runs
    // block-parallel in LDS -- one slot's serial twist would stretch the launch)
    __shared__ double s_total;
    if (lane == 0) {
        double total = 0.0;
        for (int j = 0; j < n; ++j) total = total + vals[j];
        s_total = total;
    }
    __syncthreads();
    uint32_t* py = py_mt + (size_t)i * MT_WORDS;
    if (!isfinite(s_total)) {
        // every gamma draw of the ply was 0 (only a tiny alpha can do this):
        // noise = 0 * (1/0) = NaN, and the reference's random.choices raises
        // ValueError('Total of weights must be finite') -- an error, not a move
        if (lane == 0) atomicOr(&ctr->error, 8);
        return;
    }
    if (s_total == 0.0) {
        if (lane == 0) s_pick = mt_randbelow_serial(py, n);  // random.choice
    } else {
        const double r = block_mt_random(py, mt3, lane);
        if (lane == 0) s_pick = choose_from(vals, cum, n, s_total, r);
    }
    __syncthreads();
    commit_move(cfg, s, i, ml[s_pick], boards, rec, last_board, ctr, lane);
    if (lane == 0) slots[i] = s;
}

// ------------------------------------------------------------- finish ----
// two waves per slot: wave 1 takes the slot's next game and seeds its CPython
// stream (the longer chain) while wave 0 scores the finished game, then sets up
// the next one and seeds its numpy stream
__global__ __launch_bounds__(128) void k_finish(DevCfg cfg, Slot* slots, int8_t* boards, uint16_t* moves,
                                                uint32_t* np_mt, uint32_t* py_mt, kv_game* games, Ctr* ctr) {
    const int i = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    Slot s = slots[i];
    if (s.status != ST_FINISHED) return;
    int8_t* board = boards + (size_t)i * 64;
    // the slot's next game first, so that wave 1 seeds its CPython stream (the
    // longer chain) while wave 0 scores the finished game
    __shared__ long long s_next;
    if (tid == 64) {
        long long next = -1;
        if (cfg.recycle) {
            const unsigned long long k = atomicAdd(&ctr->next_game, 1ull);
            if ((long long)k < cfg.n_games) next = (long long)k;
        }
        s_next = next;
    }
    __syncthreads();
    const long long k = s_next;
    const long long gid = cfg.id_base + k * cfg.id_stride;
    const unsigned long long sd = cfg.seed + (unsigned long long)gid;
    if (wave == 1) {
        if (k >= 0 && cfg.seed_mode == KV_SEED_PER_GAME) wave_seed_python(py_mt + (size_t)i * MT_WORDS, sd, lane);
        return;
    }
    // outcome (:210-238)
    if (s.end_kind == END_MAXED) {
        s.outcome = 0;
        s.reason = 0;
    } else if (s.end_kind == END_NOMOVES && s.movegen_clean) {
        // k_movegen's getValidMoves on this very position found no moves and
        // rewrote nothing, so both getValidMoves calls of the chain below would
        // return none on it: inCheck alone decides mate / stalemate
        const Pos p = wave_pos(board[lane], s.wtm, s.wkr, s.wkc, s.bkr, s.bkc, s.flags, s.ep);
        const bool chk = in_check(p);
        s.outcome = chk ? (p.wtm ? -1 : 1) : 0;
        s.reason = chk ? 2 : 3;
    } else if (s.end_kind != END_RESIGN) {
        Pos p = wave_pos(board[lane], s.wtm, s.wkr, s.wkc, s.bkr, s.bkc, s.flags, s.ep);
        uint16_t* ml = moves + (size_t)i * MAXM;
        const bool chk = in_check(p);
        int n1 = -1;
        if (chk) n1 = wave_valid_moves(p, ml, MAXM, lane);
        if (chk && n1 == 0) {
            s.outcome = p.wtm ? -1 : 1;
            s.reason = 2;
        } else if (wave_valid_moves(p, ml, MAXM, lane) == 0) {
            s.outcome = 0;
            s.reason = 3;
        } else {
            const bool kings_only = (p.w | p.b) == p.K;
            s.outcome = 0;
            s.reason = kings_only ? 4 : 5;  // material branch: always 0 (see oracle/kv_oracle.c)
        }
        board[lane] = (int8_t)pos_at(p, lane);
        s.wtm = p.wtm;
        s.wkr = p.wkr; s.wkc = p.wkc; s.bkr = p.bkr; s.bkc = p.bkc;
        s.flags = p.flags;
        s.ep = p.ep;
    }
    if (tid == 0) {
        // flush of a non-empty buffer (:202-208): one more forward call
        if (cfg.sims == 0 && s.buf > 0) {
            s.n_evals += 1;
            if (cfg.seed_mode == KV_SEED_SEQUENTIAL) s.need_flush = 1;
        }
        const unsigned long long gi = atomicAdd(&ctr->games_count, 1ull);
        kv_game gm;
        gm.game_id = s.game_id;
        gm.plies = s.ply;
        gm.outcome = s.outcome;
        gm.reward = s.outcome == 1 ? 1.0f : (s.outcome == 0 ? 0.2f : -1.0f);
        gm.reason = s.reason;
        gm.n_evals = s.n_evals;
        gm.pad = 0;
        games[gi % (unsigned long long)cfg.games_cap] = gm;
        s.status = ST_IDLE;
    }
    if (k >= 0) {  // the slot starts game k: board + numpy stream by wave 0, fields by thread 0
        board[lane] = kStart[lane];
        if (cfg.seed_mode == KV_SEED_PER_GAME) wave_seed_genrand(np_mt + (size_t)i * MT_WORDS, (uint32_t)sd, lane);
        if (tid == 0) start_game_fields(cfg, s, gid);
    }
    if (tid == 0) slots[i] = s;
}

// KV_EVAL_LAZY above 16 slots: the boards of the slots whose network row the
// schedule consumes this step (the only rows self_play.py reads: :147-150),
// gathered in slot order into a compact batch; row_of[i] = the slot's row or
// -1. A batch of 1-16 rows is padded to 17 with copies of its first board: the
// network is batch-invariant bit for bit inside its > 16-board class (the
// class of the all-slots batch of faithful mode), so every consumed row equals
// the faithful row and the games are identical (tests/test_engine_gpu.py).
__global__ __launch_bounds__(1024) void k_compact(DevCfg cfg, const Slot* slots, const int8_t* boards,
                                                  int8_t* comp_boards, int* row_of, Ctr* ctr) {
    __shared__ int wsum[16];
    __shared__ int base;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < cfg.slots; c0 += 1024) {
        const int i = c0 + tid;
        const bool need = i < cfg.slots && slots[i].status == ST_ACTIVE && slots[i].consumed;
        const unsigned long long bal = __ballot(need);
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int k = 0; k < w; ++k) off += wsum[k];
        const int row = off + __popcll(bal & ((1ull << lane) - 1));
        if (i < cfg.slots) row_of[i] = need ? row : -1;
        if (need)
            for (int q = 0; q < 4; ++q)
                ((u32x4*)(comp_boards + (size_t)row * 64))[q] = ((const u32x4*)(boards + (size_t)i * 64))[q];
        __syncthreads();
        if (tid == 0)
            for (int k = 0; k < 16; ++k) base += wsum[k];
        __syncthreads();
    }
    const int cnt = base, padded = cnt > 0 && cnt < 17 ? 17 : cnt;
    for (int r = cnt + tid / 4; r < padded; r += 256)  // 4 threads per padding row
        ((u32x4*)(comp_boards + (size_t)r * 64))[tid & 3] = ((const u32x4*)comp_boards)[tid & 3];
    if (tid == 0) ctr->comp_rows = padded;
}

// MCTS with fewer active slots than slots (a finite run whose game queue has
// run dry: its last games, a test's tail): the leaf batches carry only the
// active slots' rows. slot_of[r] = the r-th active slot in slot order, rows
// past the count (padding up to the > 16-board class) repeat row 0; row_of[i]
// = the slot's row or -1. The network is batch-invariant bit for bit inside a
// class, so every active slot's leaf row equals its row in the full batch and
// the searches are unchanged (tests/test_mcts_gpu.py).
__global__ __launch_bounds__(1024) void k_compact_active(DevCfg cfg, const Slot* slots, int rows, int* slot_of,
                                                         int* row_of, Ctr* ctr) {
    __shared__ int wsum[16];
    __shared__ int base;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < cfg.slots; c0 += 1024) {
        const int i = c0 + tid;
        const bool act = i < cfg.slots && slots[i].status == ST_ACTIVE;
        const unsigned long long bal = __ballot(act);
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int k = 0; k < w; ++k) off += wsum[k];
        const int row = off + __popcll(bal & ((1ull << lane) - 1));
        if (i < cfg.slots) row_of[i] = act && row < rows ? row : -1;
        if (act && row < rows) slot_of[row] = i;
        __syncthreads();
        if (tid == 0)
            for (int k = 0; k < 16; ++k) base += wsum[k];
        __syncthreads();
    }
    const int cnt = base < rows ? base : rows;
    // more active slots than the host sized the batch for: some slot would search on stale leaf rows
    if (tid == 0 && base > rows) atomicOr(&ctr->error, 16);
    __syncthreads();
    const int first = cnt > 0 ? slot_of[0] : 0;
    for (int r = cnt + tid; r < rows; r += 1024) slot_of[r] = first;  // padding rows
}

// this sim-step's leaves of the active slots -> the compact batch (one wave per row)
__global__ __launch_bounds__(64) void k_gather_leaves(const int* slot_of, const int8_t* nn_boards,
                                                      const uint16_t* leaf_moves, const int* leaf_cnt, int8_t* cb,
                                                      uint16_t* cm, int* cc) {
    const int r = blockIdx.x, lane = threadIdx.x;
    const int s = slot_of[r];
    cb[(size_t)r * 64 + lane] = nn_boards[(size_t)s * 64 + lane];
    const int n = min(leaf_cnt[s], MAXM);
    if (lane == 0) cc[r] = n;
    for (int j = lane; j < n; j += 64) cm[(size_t)r * MAXM + j] = leaf_moves[(size_t)s * MAXM + j];
}

// the compact batch's outputs back to the slots' rows (padding rows dropped)
__global__ __launch_bounds__(64) void k_scatter_leaves(const int* slot_of, const int* row_of, const float* cl,
                                                       const float* cv, const int* cc, float* leaf_logits,
                                                       float* values) {
    const int r = blockIdx.x, lane = threadIdx.x;
    const int s = slot_of[r];
    if (row_of[s] != r) return;
    if (lane == 0) values[s] = cv[r];
    const int n = cc[r];
    for (int j = lane; j < n; j += 64) leaf_logits[(size_t)s * MAXM + j] = cl[(size_t)r * MAXM + j];
}

// the flush rows of sequential mode: boards [slots, 2*slots) = last appended board
__global__ void k_flush_rows(DevCfg cfg, const Slot* slots, const int8_t* last_board, int8_t* nn_boards) {
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= cfg.slots) return;
    nn_boards[(size_t)(cfg.slots + i) * 64 + lane] = slots[i].need_flush ? last_board[(size_t)i * 64 + lane] : 0;
}

}  // namespace kv

// ---------------------------------------------------------------- host --
struct kv_engine {
    kv_config cfg;
    kv::DevCfg dc;
    kv_net* net = nullptr;
    hipStream_t st = nullptr;
    kv::Slot* slots = nullptr;
    int8_t* boards = nullptr;  // [rows][64]: slot boards, then flush rows
    uint16_t* moves = nullptr;
    float* logits = nullptr;
    float* values = nullptr;
    float* last_probs = nullptr;
    int8_t* comp_boards = nullptr;  // KV_EVAL_LAZY above 16 slots: this step's compact batch
    int* row_of = nullptr;
    long long lazy_rows = 0;        // rows sent through the network by the compact batches
    uint32_t* np_mt = nullptr;
    uint32_t* py_mt = nullptr;
    kv_record* rec = nullptr;
    kv_game* games = nullptr;
    int8_t* last_board = nullptr;
    kv::Ctr* ctr = nullptr;
    kv::Ctr* ctr_host = nullptr;  // pinned
    long long steps = 0;
    double wall_ms = 0;
    std::vector<hipEvent_t> ev;  // residual-conv section start/end per forward
    int n_ev_used = 0;
    double nn_res_ms = 0;
    long long nn_res_launches = 0;
    int dom_algo = KV_ALGO_DIRECT, dom_launches = 10;  // what each event pair brackets
    int dom_path = KV_PATH_DIRECT, dom_split = 0;
    double dom_flop = 0;
    const char* dom_kernel = "";
    bool loaded = false;
    // MCTS (sims > 0)
    kv::Tree tree;
    kv::MctsSlot* ms = nullptr;
    int8_t* nn_boards = nullptr;
    float* probs = nullptr;
    float* sqrt_tab = nullptr;
    // MCTS leaf batches of the active slots only (k_compact_active)
    int* mc_slot_of = nullptr;
    int* mc_row_of = nullptr;
    int8_t* mc_boards = nullptr;
    uint16_t* mc_moves = nullptr;
    int* mc_cnt = nullptr;
    float* mc_logits = nullptr;
    float* mc_values = nullptr;
    long long mc_rows = 0;  // leaf rows the compact batches sent through the network
    // kv_records_device / kv_root_visits_device copy out of e->rec / root_visits on the caller's
    // stream; the next write to those buffers (kv_run, kv_reset_records) or their release
    // (kv_destroy) waits for that copy on e->st
    hipEvent_t copy_done = nullptr;
    bool copy_pending = false;
};

// order e->st after an outstanding device-to-device copy of the engine's buffers on a caller stream
static int eng_wait_copies(kv_engine* e) {
    if (!e->copy_pending) return KV_OK;
    KV_HIP(hipStreamWaitEvent(e->st, e->copy_done, 0));
    e->copy_pending = false;
    return KV_OK;
}

// The engine stream waits for the copy right away (whatever stream the caller used), so two copies on
// two caller streams are both ordered before the next write to e->rec / root_visits; the event is
// kept for kv_destroy, which waits for the last copy before freeing the buffers.
static int eng_note_copy(kv_engine* e, hipStream_t caller) {
    if (!e->copy_done) KV_HIP(hipEventCreateWithFlags(&e->copy_done, hipEventDisableTiming));
    KV_HIP(hipEventRecord(e->copy_done, caller));
    KV_HIP(hipStreamWaitEvent(e->st, e->copy_done, 0));
    e->copy_pending = true;
    return KV_OK;
}

static int eng_counters(kv_engine* e, bool check_error = true) {
    // active slots / plies / rows are summed from the slots only when the host reads them
    hipLaunchKernelGGL(kv::k_count, dim3(1), dim3(256), 0, e->st, e->dc, e->slots, e->ctr);
    KV_HIP(hipGetLastError());
    KV_HIP(hipMemcpyAsync(e->ctr_host, e->ctr, sizeof(kv::Ctr), hipMemcpyDeviceToHost, e->st));
    KV_HIP(hipStreamSynchronize(e->st));
    if (check_error && e->ctr_host->error) {
        kv::set_error("engine device error flags 0x%x (1: move list overflow, 2: record buffer full, "
                      "4: MCTS tree pool full, %llu expansions dropped -- raise kv_config.tree_edge_cap; "
                      "8: move weights not finite -- every Dirichlet gamma draw of a ply was 0, where the "
                      "reference's random.choices raises ValueError; 16: more active MCTS slots than the compact "
                      "leaf batch holds -- a host / device count mismatch)",
                      e->ctr_host->error, (unsigned long long)e->ctr_host->tree_overflows);
        return (e->ctr_host->error & (8 | 16)) ? KV_EINVAL : KV_EOVERFLOW;
    }
    return KV_OK;
}

static int eng_collect_timing(kv_engine* e) {
    for (int k = 0; k + 1 < e->n_ev_used; k += 2) {
        float ms = 0.f;
        KV_HIP(hipEventSynchronize(e->ev[k + 1]));
        KV_HIP(hipEventElapsedTime(&ms, e->ev[k], e->ev[k + 1]));
        e->nn_res_ms += ms;
        e->nn_res_launches += e->dom_launches;
    }
    e->n_ev_used = 0;
    return KV_OK;
}

extern "C" {

int kv_create(const kv_config* cfg, kv_engine** out) {
    KV_REQUIRE(cfg && out, KV_EINVAL, "kv_create: NULL argument");
    KV_REQUIRE(cfg->slots > 0 && cfg->n_games >= 0, KV_EINVAL, "kv_create: slots must be > 0");
    // numpy's legacy gamma for shape < 1 (the branch restated on the device); a
    // normal double keeps 1/alpha finite, and kv_libm.h's pow is exact over the
    // whole range, subnormal / zero gamma draws of a small alpha included
    KV_REQUIRE(cfg->alpha >= 2.2250738585072014e-308 && cfg->alpha < 1.0, KV_EINVAL,
               "kv_create: DIR_NOISE_ALPHA must be a normal double in (0,1) (legacy gamma shape<1 branch), got %g",
               cfg->alpha);
    KV_REQUIRE(cfg->batch >= 1, KV_EINVAL, "kv_create: SELFPLAY_BATCH_SIZE must be >= 1");
    KV_REQUIRE(cfg->seed_mode == KV_SEED_PER_GAME || cfg->seed_mode == KV_SEED_SEQUENTIAL, KV_EINVAL,
               "kv_create: bad seed_mode");
    KV_REQUIRE(cfg->seed_mode != KV_SEED_SEQUENTIAL || cfg->slots == 1, KV_EINVAL,
               "kv_create: sequential seeding plays games in order on one slot");
    KV_REQUIRE(cfg->sims >= 0 && cfg->sims <= KV_MAX_SIMS, KV_EINVAL,
               "kv_create: sims %d out of range [0, %d] (16-bit edge visit counts and child ids)", cfg->sims,
               KV_MAX_SIMS);
    KV_REQUIRE(cfg->tree_edge_cap <= 0 || cfg->tree_edge_cap >= kv::MAXM, KV_EINVAL,
               "kv_create: tree_edge_cap %d must be 0 (auto) or >= KV_MAXM (the root's list)", cfg->tree_edge_cap);
    KV_REQUIRE(cfg->sims == 0 || cfg->seed_mode == KV_SEED_PER_GAME, KV_EINVAL,
               "kv_create: MCTS mode uses per-game seeding");
    KV_REQUIRE(cfg->eval_mode == KV_EVAL_FAITHFUL || cfg->eval_mode == KV_EVAL_HASH ||
                   (cfg->eval_mode == KV_EVAL_LAZY && cfg->sims == 0),
               KV_EINVAL, "kv_create: eval_mode %d not available (lazy: reference move selection only)",
               cfg->eval_mode);
    KV_HIP(hipSetDevice(cfg->device));
    kv_engine* e = new kv_engine();
    e->cfg = *cfg;
    if (e->cfg.game_id_stride <= 0) e->cfg.game_id_stride = 1;
    if (e->cfg.record_cap <= 0) e->cfg.record_cap = 1 << 20;
    kv::DevCfg& d = e->dc;
    d.slots = cfg->slots;
    d.n_games = cfg->n_games;
    d.id_base = cfg->game_id_base;
    d.id_stride = e->cfg.game_id_stride;
    d.seed = cfg->seed;
    d.seed_mode = cfg->seed_mode;
    d.max_moves = cfg->max_moves;
    d.batch = cfg->batch;
    d.eps = cfg->eps;
    d.alpha = cfg->alpha;
    d.record_cap = e->cfg.record_cap;
    d.recycle = cfg->recycle;
    d.rows = cfg->seed_mode == KV_SEED_SEQUENTIAL ? 2 * cfg->slots : cfg->slots;
    d.games_cap = std::max<long long>(1, std::min<long long>(cfg->n_games, 1 << 20));
    d.sims = cfg->sims;
    d.eval_mode = cfg->eval_mode;
    const size_t S = (size_t)cfg->slots, R = (size_t)d.rows;
    int rc = KV_OK;
#define ALLOC(ptr, bytes)                                   \
    do {                                                    \
        hipError_t er_ = hipMalloc(&(ptr), (bytes));        \
        if (er_ != hipSuccess) {                            \
            kv::set_error("kv_create: hipMalloc %s (%zu B): %s", #ptr, (size_t)(bytes), hipGetErrorString(er_)); \
            kv_destroy(e);                                  \
            return KV_ENOMEM;                               \
        }                                                   \
    } while (0)
    ALLOC(e->slots, S * sizeof(kv::Slot));
    ALLOC(e->boards, R * 64);
    ALLOC(e->moves, S * kv::MAXM * sizeof(uint16_t));
    ALLOC(e->logits, R * 4096 * sizeof(float));
    ALLOC(e->values, R * sizeof(float));
    ALLOC(e->last_probs, S * 4096 * sizeof(float));
    if (cfg->eval_mode == KV_EVAL_LAZY && S > 16) {
        ALLOC(e->comp_boards, (S + 17) * 64);
        ALLOC(e->row_of, S * sizeof(int));
    }
    ALLOC(e->np_mt, S * kv::MT_WORDS * sizeof(uint32_t));
    ALLOC(e->py_mt, S * kv::MT_WORDS * sizeof(uint32_t));
    ALLOC(e->rec, (size_t)e->cfg.record_cap * sizeof(kv_record));
    ALLOC(e->games, (size_t)d.games_cap * sizeof(kv_game));
    ALLOC(e->last_board, S * 64);
    ALLOC(e->ctr, sizeof(kv::Ctr));
    if (cfg->sims > 0) {
        kv::Tree& t = e->tree;
        t.ncap = cfg->sims + 2;
        // every expansion adds <= MAXM edges: (sims + 1) x MAXM edges can never
        // overflow (C3: 2,048 slots x 801 x 320 x 14 B = 7.3 GB of the 288 GB);
        // a smaller cap is honoured and an overflow raises KV_EOVERFLOW
        const long long full = (long long)kv::MAXM * (cfg->sims + 1);
        // node edge blocks start on 16-edge boundaries (kv_mcts.hip), so a
        // caller's cap is rounded down to a multiple of 16 (MAXM is one) and
        // every expansion still takes at most MAXM edges
        t.ecap = (int)(cfg->tree_edge_cap > 0 ? std::min<long long>(cfg->tree_edge_cap & ~15, full) : full);
        t.c_puct = cfg->c_puct > 0.f ? cfg->c_puct : 1.5f;
        t.sims = cfg->sims;
        const size_t E = S * (size_t)t.ecap, N = S * (size_t)t.ncap;
        ALLOC(t.e_move, E * sizeof(uint16_t));
        ALLOC(t.e_P, E * sizeof(float));
        ALLOC(t.e_N, E * sizeof(uint16_t));
        ALLOC(t.e_W, E * sizeof(float));
        ALLOC(t.e_child, E * sizeof(uint16_t));
        ALLOC(t.node, N * sizeof(kv::NodeRec));
        ALLOC(t.path, N * sizeof(int));
        ALLOC(t.leaf_moves, S * kv::MAXM * sizeof(uint16_t));
        ALLOC(t.leaf_cnt, S * sizeof(int));
        ALLOC(t.leaf_logits, S * kv::MAXM * sizeof(float));
        (void)hipMemset(t.leaf_cnt, 0, S * sizeof(int));
        ALLOC(e->ms, S * sizeof(kv::MctsSlot));
        ALLOC(e->nn_boards, S * 64);
        ALLOC(e->probs, S * 4096 * sizeof(float));
        ALLOC(e->sqrt_tab, (size_t)(t.ncap + 2) * sizeof(float));
        if (cfg->keep_root_visits) ALLOC(t.root_visits, (size_t)e->cfg.record_cap * kv::MAXM * sizeof(uint16_t));
        const char* mc_env = getenv("KV_MCTS_COMPACT");  // "0": always the full-slot leaf batch (A/B timing)
        if (cfg->eval_mode != KV_EVAL_HASH && S > 1 && !(mc_env && mc_env[0] == '0')) {
            ALLOC(e->mc_slot_of, S * sizeof(int));
            ALLOC(e->mc_row_of, S * sizeof(int));
            ALLOC(e->mc_boards, S * 64);
            ALLOC(e->mc_moves, S * kv::MAXM * sizeof(uint16_t));
            ALLOC(e->mc_cnt, S * sizeof(int));
            ALLOC(e->mc_logits, S * kv::MAXM * sizeof(float));
            ALLOC(e->mc_values, S * sizeof(float));
        }
        t.ms = e->ms;
        std::vector<float> sq(t.ncap + 2);
        for (int k = 0; k < t.ncap + 2; ++k) sq[k] = (float)sqrt((double)k);
        if (hipMemcpy(e->sqrt_tab, sq.data(), sq.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
            kv_destroy(e);
            kv::set_error("kv_create: sqrt table copy");
            return KV_EHIP;
        }
        t.sqrt_tab = e->sqrt_tab;
        (void)hipMemset(e->ms, 0, S * sizeof(kv::MctsSlot));
    }
#undef ALLOC
    if (hipHostMalloc(&e->ctr_host, sizeof(kv::Ctr)) != hipSuccess) {
        kv_destroy(e);
        kv::set_error("kv_create: hipHostMalloc failed");
        return KV_ENOMEM;
    }
    if ((rc = kv_net_create(cfg->device, &e->net)) || (rc = kv_net_set_precision(e->net, cfg->precision)) ||
        (rc = kv_net_set_algo(e->net, cfg->algo))) {
        kv_destroy(e);
        return rc;
    }
    if (hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) != hipSuccess) {
        kv_destroy(e);
        kv::set_error("kv_create: stream");
        return KV_EHIP;
    }
    (void)hipMemsetAsync(e->boards, 0, R * 64, e->st);
    (void)hipMemsetAsync(e->ctr, 0, sizeof(kv::Ctr), e->st);
    (void)hipMemsetAsync(e->last_probs, 0, S * 4096 * sizeof(float), e->st);
    kv::Ctr c0;
    memset(&c0, 0, sizeof(c0));
    c0.next_game = (unsigned long long)std::min<long long>(cfg->n_games, cfg->slots);
    (void)hipMemcpyAsync(e->ctr, &c0, sizeof(c0), hipMemcpyHostToDevice, e->st);
    hipLaunchKernelGGL(kv::k_init, dim3((cfg->slots + 63) / 64), dim3(64), 0, e->st, d, e->slots, e->boards,
                       e->np_mt, e->py_mt, e->ctr);
    KV_HIP(hipGetLastError());
    KV_HIP(hipStreamSynchronize(e->st));
    *out = e;
    return KV_OK;
}

int kv_load_weights(kv_engine* e, const float* packed, size_t n_floats) {
    KV_REQUIRE(e, KV_EINVAL, "kv_load_weights: NULL engine");
    KV_HIP(hipStreamSynchronize(e->st));  // the load (and its calibration) runs on the null stream
    int rc = kv_net_load(e->net, packed, n_floats);
    if (rc == KV_OK) e->loaded = true;
    return rc;
}

int kv_engine_calibration(kv_engine* e, kv_calib* out) {
    KV_REQUIRE(e && out, KV_EINVAL, "kv_engine_calibration: NULL argument");
    return kv_net_calibration(e->net, out);
}

int kv_set_max_moves(kv_engine* e, int max_moves) {
    KV_REQUIRE(e, KV_EINVAL, "kv_set_max_moves: NULL");
    e->cfg.max_moves = max_moves;
    e->dc.max_moves = max_moves;
    return KV_OK;
}

// one network pass over `rows` boards (or the hash test evaluator), with the
// residual-tower section bracketed by HIP events for the roofline; `leaf`:
// the MCTS leaf batch, whose policy is only the leaves' legal moves
// (kv_net_forward_boards_legal into tree.leaf_logits)
// `comp`: the leaf batch is the compact active-slot batch (e->mc_*) instead of the slots' rows
static int eng_eval(kv_engine* e, const int8_t* boards, int rows, bool leaf = false, bool comp = false) {
    kv_net* net = e->net;
    hipStream_t st = e->st;
    float* logits = e->logits;
    float* values = comp ? e->mc_values : e->values;
    if (e->dc.eval_mode == KV_EVAL_HASH) {
        int rc = kv::hash_eval(boards, rows, logits, values, st);
        if (rc || !leaf) return rc;
        return kv::hash_legal(e->tree, rows, st);  // its logits (all 0) in the compact layout
    }
    if ((size_t)e->n_ev_used + 2 > e->ev.size()) {
        for (int k = 0; k < 2; ++k) {
            hipEvent_t x;
            KV_HIP(hipEventCreate(&x));
            e->ev.push_back(x);
        }
    }
    kv::net_set_res_events(net, e->ev[e->n_ev_used], e->ev[e->n_ev_used + 1]);
    e->n_ev_used += 2;
    const int rc = leaf ? kv::net_forward_boards_legal_internal(net, boards, rows,
                                                                comp ? e->mc_moves : e->tree.leaf_moves,
                                                                comp ? e->mc_cnt : e->tree.leaf_cnt, kv::MAXM,
                                                                comp ? e->mc_logits : e->tree.leaf_logits,
                                                                values, st)
                        : kv::net_forward_boards_internal(net, boards, rows, logits, values, st);
    kv::net_set_res_events(net, nullptr, nullptr);
    kv::net_dom_info(net, &e->dom_algo, &e->dom_launches, &e->dom_flop, &e->dom_path, &e->dom_split,
                     &e->dom_kernel);
    return rc;
}

int kv_run(kv_engine* e, int64_t max_steps, int64_t stop_after_games) {
    KV_REQUIRE(e && e->loaded, KV_EINVAL, "kv_run: engine has no weights");
    KV_HIP(hipSetDevice(e->cfg.device));
    const auto t0 = std::chrono::steady_clock::now();
    const int S = e->cfg.slots;
    const bool mcts = e->dc.sims > 0;
    const int check_every = (S >= 64 && stop_after_games < 0 && !mcts) ? 4 : 1;
    int rc = eng_wait_copies(e);
    if (rc) return rc;
    rc = eng_counters(e);
    if (rc) return rc;
    long long done = 0;
    while ((max_steps < 0 || done < max_steps) && e->ctr_host->active > 0 &&
           (stop_after_games < 0 || (int64_t)e->ctr_host->games_count < stop_after_games)) {
        const bool lazy = e->dc.eval_mode == KV_EVAL_LAZY;
        const bool compact = lazy && e->comp_boards != nullptr;  // above 16 slots
        if (lazy && !compact) KV_HIP(hipMemsetAsync(&e->ctr->need_eval, 0, sizeof(int), e->st));
        hipLaunchKernelGGL(kv::k_movegen, dim3(S), dim3(64), 0, e->st, e->dc, e->slots, e->boards,
                           e->moves, e->ctr);
        KV_HIP(hipGetLastError());
        if (e->dc.rows > S)
            hipLaunchKernelGGL(kv::k_flush_rows, dim3(S), dim3(64), 0, e->st, e->dc, e->slots, e->last_board,
                               e->boards);
        bool eval_now = true;
        if (compact) {  // only the consumed rows, as one compact batch (identical outputs)
            hipLaunchKernelGGL(kv::k_compact, dim3(1), dim3(1024), 0, e->st, e->dc, e->slots, e->boards,
                               e->comp_boards, e->row_of, e->ctr);
            KV_HIP(hipGetLastError());
            KV_HIP(hipMemcpyAsync(&e->ctr_host->comp_rows, &e->ctr->comp_rows, sizeof(int), hipMemcpyDeviceToHost,
                                  e->st));
            KV_HIP(hipStreamSynchronize(e->st));
            const int rows = e->ctr_host->comp_rows;
            if (rows > 0 && (rc = eng_eval(e, e->comp_boards, rows))) return rc;
            e->lazy_rows += rows;
            eval_now = false;
        } else if (lazy) {  // evaluate only on the steps whose row the schedule consumes (identical outputs)
            KV_HIP(hipMemcpyAsync(&e->ctr_host->need_eval, &e->ctr->need_eval, sizeof(int), hipMemcpyDeviceToHost,
                                  e->st));
            KV_HIP(hipStreamSynchronize(e->st));
            eval_now = e->ctr_host->need_eval != 0;
        }
        if (eval_now && (rc = eng_eval(e, e->boards, e->dc.rows))) return rc;
        if (!mcts) {
            hipLaunchKernelGGL(kv::k_sample, dim3(S), dim3(256), 0, e->st, e->dc, e->slots, e->boards, e->moves,
                               e->logits, e->values, e->last_probs, e->np_mt, e->py_mt, e->rec, e->last_board,
                               e->ctr, compact ? (const int*)e->row_of : (const int*)nullptr);
            KV_HIP(hipGetLastError());
        } else {
            const kv::Tree& t = e->tree;
            // fewer active slots than slots (no game left to start): compact leaf batches of the active
            // slots, padded to the network class of the full batch (> 16 boards: at least 17 rows)
            const int act = e->ctr_host->active;
            const bool comp = e->mc_slot_of != nullptr && act < S;
            const int R = comp ? (S > 16 ? std::max(act, 17) : act) : S;
            if (comp) {
                hipLaunchKernelGGL(kv::k_compact_active, dim3(1), dim3(1024), 0, e->st, e->dc, e->slots, R,
                                   e->mc_slot_of, e->mc_row_of, e->ctr);
                KV_HIP(hipGetLastError());
            }
            if ((rc = kv::mcts_root(e->dc, t, e->slots, e->moves, e->logits, e->values, e->probs, e->np_mt, e->ctr, e->st)))
                return rc;
            if ((rc = kv::mcts_select(e->dc, t, e->slots, e->boards, e->nn_boards, e->ctr, e->st, 0, S))) return rc;
            for (int k = 0; k < e->dc.sims; ++k) {
                if (comp) {
                    hipLaunchKernelGGL(kv::k_gather_leaves, dim3(R), dim3(64), 0, e->st, e->mc_slot_of, e->nn_boards,
                                       t.leaf_moves, t.leaf_cnt, e->mc_boards, e->mc_moves, e->mc_cnt);
                    KV_HIP(hipGetLastError());
                    if ((rc = eng_eval(e, e->mc_boards, R, true, true))) return rc;
                    hipLaunchKernelGGL(kv::k_scatter_leaves, dim3(R), dim3(64), 0, e->st, e->mc_slot_of,
                                       e->mc_row_of, e->mc_logits, e->mc_values, e->mc_cnt, t.leaf_logits,
                                       e->values);
                    KV_HIP(hipGetLastError());
                    e->mc_rows += R;
                } else if ((rc = eng_eval(e, e->nn_boards, S, true))) {
                    return rc;
                }
                rc = k + 1 < e->dc.sims
                         ? kv::mcts_backup_select(e->dc, t, e->slots, e->boards, e->logits, e->values, e->probs,
                                                  e->nn_boards, e->ctr, e->st, 0, S)
                         : kv::mcts_backup(e->dc, t, e->slots, e->logits, e->values, e->probs, e->ctr, e->st, 0, S);
                if (rc) return rc;
            }
            if ((rc = kv::mcts_choose(e->dc, t, e->slots, e->boards, e->py_mt, e->rec, e->last_board, e->ctr,
                                      e->st)))
                return rc;
        }
        hipLaunchKernelGGL(kv::k_finish, dim3(S), dim3(128), 0, e->st, e->dc, e->slots, e->boards,
                           e->moves, e->np_mt, e->py_mt, e->games, e->ctr);
        KV_HIP(hipGetLastError());
        ++done;
        ++e->steps;
        if (done % check_every == 0 || (max_steps >= 0 && done >= max_steps)) {
            if ((rc = eng_counters(e))) return rc;
            if ((rc = eng_collect_timing(e))) return rc;
        }
    }
    if ((rc = eng_counters(e))) return rc;
    if ((rc = eng_collect_timing(e))) return rc;
    e->wall_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return KV_OK;
}

int kv_reset_records(kv_engine* e) {
    KV_REQUIRE(e, KV_EINVAL, "kv_reset_records: NULL");
    const int rc = eng_wait_copies(e);
    if (rc) return rc;
    KV_HIP(hipMemsetAsync(&e->ctr->rec_count, 0, sizeof(unsigned long long), e->st));
    KV_HIP(hipStreamSynchronize(e->st));
    return KV_OK;
}

int kv_sync(kv_engine* e) {
    KV_REQUIRE(e, KV_EINVAL, "kv_sync: NULL");
    KV_HIP(hipStreamSynchronize(e->st));
    return KV_OK;
}

int kv_records(kv_engine* e, kv_record* out, size_t cap, size_t* n) {
    KV_REQUIRE(e && n, KV_EINVAL, "kv_records: NULL argument");
    int rc = eng_counters(e);
    if (rc) return rc;
    size_t cnt = (size_t)std::min<unsigned long long>(e->ctr_host->rec_count, (unsigned long long)e->cfg.record_cap);
    *n = cnt;
    if (!out) return KV_OK;
    KV_REQUIRE(cap >= cnt, KV_EINVAL, "kv_records: buffer holds %zu, need %zu", cap, cnt);
    KV_HIP(hipMemcpy(out, e->rec, cnt * sizeof(kv_record), hipMemcpyDeviceToHost));
    std::stable_sort(out, out + cnt, [](const kv_record& a, const kv_record& b) {
        return a.game_id != b.game_id ? a.game_id < b.game_id : a.ply < b.ply;
    });
    return KV_OK;
}

int kv_records_device(kv_engine* e, kv_record* out_dev, size_t cap, size_t* n, void* stream) {
    KV_REQUIRE(e && n, KV_EINVAL, "kv_records_device: NULL argument");
    int rc = eng_counters(e);
    if (rc) return rc;
    const size_t cnt =
        (size_t)std::min<unsigned long long>(e->ctr_host->rec_count, (unsigned long long)e->cfg.record_cap);
    *n = cnt;
    if (!out_dev) return KV_OK;
    KV_REQUIRE(cap >= cnt, KV_EINVAL, "kv_records_device: buffer holds %zu, need %zu", cap, cnt);
    // the engine stream is idle after eng_counters; the copy runs on the caller's stream, and the
    // engine's next write to e->rec waits for it (eng_wait_copies)
    KV_HIP(hipMemcpyAsync(out_dev, e->rec, cnt * sizeof(kv_record), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return eng_note_copy(e, (hipStream_t)stream);
}

int kv_games(kv_engine* e, kv_game* out, size_t cap, size_t* n) {
    KV_REQUIRE(e && n, KV_EINVAL, "kv_games: NULL argument");
    int rc = eng_counters(e);
    if (rc) return rc;
    size_t cnt = (size_t)std::min<unsigned long long>(e->ctr_host->games_count, (unsigned long long)e->dc.games_cap);
    *n = cnt;
    if (!out) return KV_OK;
    KV_REQUIRE(cap >= cnt, KV_EINVAL, "kv_games: buffer holds %zu, need %zu", cap, cnt);
    KV_HIP(hipMemcpy(out, e->games, cnt * sizeof(kv_game), hipMemcpyDeviceToHost));
    std::sort(out, out + cnt, [](const kv_game& a, const kv_game& b) { return a.game_id < b.game_id; });
    return KV_OK;
}

int kv_stats_get(kv_engine* e, kv_stats* out) {
    KV_REQUIRE(e && out, KV_EINVAL, "kv_stats_get: NULL argument");
    int rc = eng_counters(e, false);  // readable after an error too (tree_overflows)
    if (rc) return rc;
    out->steps = e->steps;
    out->plies = (int64_t)e->ctr_host->plies;
    out->games_done = (int64_t)e->ctr_host->games_count;
    out->nn_rows = (int64_t)(e->ctr_host->nn_rows + e->ctr_host->nn_rows_slots);
    out->sims = (int64_t)e->ctr_host->sims;
    out->records = (int64_t)e->ctr_host->rec_count;
    out->res_conv_ms = e->nn_res_ms;
    out->res_conv_launches = e->nn_res_launches;
    out->step_ms = e->wall_ms;
    out->dom_flop = e->dom_flop;
    out->dom_algo = e->dom_algo;
    out->dom_path = e->dom_path;
    out->dom_split = e->dom_split;
    snprintf(out->dom_kernel, sizeof(out->dom_kernel), "%s", e->dom_kernel ? e->dom_kernel : "");
    out->tree_overflows = (int64_t)e->ctr_host->tree_overflows;
    out->nn_rows_lazy = e->lazy_rows;
    return KV_OK;
}

int kv_root_visits(kv_engine* e, int32_t* out, size_t cap, size_t* n) {
    KV_REQUIRE(e && n, KV_EINVAL, "kv_root_visits: NULL argument");
    KV_REQUIRE(e->tree.root_visits, KV_EINVAL, "kv_root_visits: engine was created without keep_root_visits");
    int rc = eng_counters(e);
    if (rc) return rc;
    const size_t cnt = (size_t)std::min<unsigned long long>(e->ctr_host->rec_count, (unsigned long long)e->cfg.record_cap);
    *n = cnt;
    if (!out) return KV_OK;
    KV_REQUIRE(cap >= cnt, KV_EINVAL, "kv_root_visits: buffer holds %zu records, need %zu", cap, cnt);
    std::vector<kv_record> rec(cnt);
    std::vector<uint16_t> vis(cnt * kv::MAXM);
    KV_HIP(hipMemcpy(rec.data(), e->rec, cnt * sizeof(kv_record), hipMemcpyDeviceToHost));
    KV_HIP(hipMemcpy(vis.data(), e->tree.root_visits, vis.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
    std::vector<size_t> ord(cnt);
    for (size_t k = 0; k < cnt; ++k) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {  // kv_records' order
        return rec[a].game_id != rec[b].game_id ? rec[a].game_id < rec[b].game_id : rec[a].ply < rec[b].ply;
    });
    for (size_t k = 0; k < cnt; ++k)
        for (int j = 0; j < kv::MAXM; ++j) {
            const uint16_t v = vis[ord[k] * kv::MAXM + j];
            out[k * kv::MAXM + j] = v == 0xffff ? -1 : (int32_t)v;
        }
    return KV_OK;
}

int kv_root_visits_device(kv_engine* e, uint16_t* out_dev, size_t cap, size_t* n, void* stream) {
    KV_REQUIRE(e && n, KV_EINVAL, "kv_root_visits_device: NULL argument");
    KV_REQUIRE(e->tree.root_visits, KV_EINVAL, "kv_root_visits_device: engine was created without keep_root_visits");
    int rc = eng_counters(e);
    if (rc) return rc;
    const size_t cnt = (size_t)std::min<unsigned long long>(e->ctr_host->rec_count, (unsigned long long)e->cfg.record_cap);
    *n = cnt;
    if (!out_dev) return KV_OK;
    KV_REQUIRE(cap >= cnt, KV_EINVAL, "kv_root_visits_device: buffer holds %zu records, need %zu", cap, cnt);
    KV_HIP(hipMemcpyAsync(out_dev, e->tree.root_visits, cnt * kv::MAXM * sizeof(uint16_t), hipMemcpyDeviceToDevice,
                          (hipStream_t)stream));
    return eng_note_copy(e, (hipStream_t)stream);
}

void kv_destroy(kv_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->cfg.device);
    if (e->copy_pending) (void)hipEventSynchronize(e->copy_done);  // a caller-stream copy out of e->rec
    if (e->st) (void)hipStreamSynchronize(e->st);
    kv::Tree& t = e->tree;
    void* bufs[] = {e->slots, e->boards, e->moves, e->logits, e->values, e->last_probs, e->comp_boards, e->row_of,
                    e->np_mt, e->py_mt, e->rec, e->games, e->last_board, e->ctr,
                    t.e_move, t.e_P, t.e_N, t.e_W, t.e_child, t.node, t.path,
                    t.leaf_moves, e->ms, e->nn_boards, e->probs, e->sqrt_tab, t.root_visits, t.leaf_cnt,
                    t.leaf_logits, e->mc_slot_of, e->mc_row_of, e->mc_boards, e->mc_moves, e->mc_cnt,
                    e->mc_logits, e->mc_values};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (e->ctr_host) (void)hipHostFree(e->ctr_host);
    for (auto x : e->ev) (void)hipEventDestroy(x);
    if (e->copy_done) (void)hipEventDestroy(e->copy_done);
    if (e->net) kv_net_destroy(e->net);
    if (e->st) (void)hipStreamDestroy(e->st);
    delete e;
}

}  // extern "C"
