// PUCT Monte-Carlo tree search on MI355X (no reference counterpart: the
// reference samples moves from the network policy, self_play.py:150-167; the
// semantics below are build-defined and restated on the CPU in
// oracle/kv_oracle.c kvo_mcts_*). One wavefront per concurrent game.
//
// Per move of each game slot:
//   root   : network row of the position; priors = the reference's own mixed
//            move distribution (softmax x (1-eps) + Dirichlet x eps over the
//            legal list, normalised; self_play.py:147-166), so the numpy
//            stream is consumed exactly as in the reference; node 0 created.
//   sims x : select (PUCT from the root: Q + c_puct * P * sqrt(N_parent) /
//            (1 + N_child), Q = W/N or 0, first maximum in move-list order) ->
//            apply the path's moves to the slot's board -> leaf = first edge
//            with no child: isDraw => value 0; no legal moves => mate (-1 for
//            the side to move) or stalemate 0; else the leaf board joins this
//            step's network batch (one row per slot) -> backup: priors =
//            softmax over the legal moves' logits only, node created, N += 1
//            and W += value from the mover's side along the path (the value
//            head is white-perspective, self_play.py:253).
//            Softmaxes use det_expf (kv_engine.h) with a fixed summation
//            order, so the CPU restatement reproduces every prior bit for bit.
//            An expansion that does not fit the slot's edge pool (sized
//            MAXM x (sims + 1) by default, so it cannot happen unless the
//            caller shrinks it) raises KV_EOVERFLOW.
//   choose : random.choices over the root visit counts on the CPython stream
//            (tau = 1), then makeMove / record / termination as the reference.
// Tree: structure-of-arrays edge pools per slot in HBM (move u16, P f32, N u16,
// W f32, child u16 per edge: 14 B; a node's edges start on a 16-edge boundary)
// and one 16-byte record per node (first edge, edge count; N for the root only:
// a non-root node's visit count is its parent edge's N).
#include <hip/hip_runtime.h>
#include <math.h>

#include "kv_engine.h"

#pragma clang fp contract(off)

namespace kv {

__device__ inline void wave_argmax_first(float& best, int& idx) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const float ob = __shfl_xor(best, m);
        const int oi = __shfl_xor(idx, m);
        if (ob > best || (ob == best && oi < idx)) {
            best = ob;
            idx = oi;
        }
    }
}

// PUCT score; identical op order in kvo_mcts (oracle), no contraction
__device__ inline float puct(float c_puct, float P, float sq, int N, float W) {
    const float u = c_puct * P * sq / (float)(1 + N);
    const float q = N > 0 ? W / (float)N : 0.0f;
    return q + u;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_mcts_root(DevCfg cfg, Tree t, Slot* slots, const uint16_t* moves,
                                                   const float* logits, const float* values, float* probs,
                                                   uint32_t* np_mt, Ctr* ctr) {
    __shared__ uint32_t mt3[MT_RW];
    __shared__ double gam[4096];
    __shared__ double vals[MAXM];
    __shared__ int scratch[RNG_SCRATCH];
    const int i = blockIdx.x, lane = threadIdx.x;
    Slot s = slots[i];
    if (s.status != ST_ACTIVE) return;
    float* lp = probs + (size_t)i * 4096;
    if (lane < 64) wave_softmax_4096_det(logits + (size_t)i * 4096, lp, lane);
    __syncthreads();
    const int n = s.nmoves;
    const uint16_t* ml = moves + (size_t)i * MAXM;
    mixed_legal_weights(cfg, lp, ml, n, gam, np_mt + (size_t)i * MT_WORDS, mt3, scratch, vals, lane);
    __shared__ double s_total;
    if (lane == 0) {
        double total = 0.0;
        for (int j = 0; j < n; ++j) total = total + vals[j];
        s_total = total;
    }
    __syncthreads();
    const double total = s_total;
    if (!isfinite(total)) {  // all-zero gamma draws: NaN weights (k_sample's error 8)
        if (lane == 0) atomicOr(&ctr->error, 8);
        return;
    }
    const size_t eb = (size_t)i * t.ecap, nb = (size_t)i * t.ncap;
    for (int j = lane; j < n; j += 256) {
        t.e_move[eb + j] = ml[j];
        t.e_P[eb + j] = total == 0.0 ? 1.0f / (float)n : (float)(vals[j] / total);
        t.e_N[eb + j] = 0;
        t.e_W[eb + j] = 0.f;
        t.e_child[eb + j] = NO_CHILD;
    }
    if (lane == 0) {
        t.node[nb] = NodeRec{0, n, 1, 0};
        MctsSlot m = t.ms[i];
        m.node_count = 1;
        m.edge_count = n;
        m.root_value = values[i];
        m.root_wtm = s.wtm;
        m.path_len = 0;
        m.leaf_pending = 0;
        m.pad[0] = 1;  // network rows consumed this move
        m.pad[1] = 0;  // leaf rows sent to the network this move (Ctr::nn_rows at the choice)
        t.ms[i] = m;
        slots[i].last_value = values[i];
    }
}

// one slot's select, by the 64 threads of its workgroup
__device__ inline void mcts_select_slot(const DevCfg& cfg, const Tree& t, const Slot* slots, const int8_t* boards,
                                        int8_t* nn_boards, Ctr* ctr, int i) {
    __shared__ int8_t bd[64];
    __shared__ int s_meta[8];  // wtm wkr wkc bkr bkc flags ep
    const int lane = threadIdx.x;
    const Slot s = slots[i];
    if (s.status != ST_ACTIVE) {
        if (lane == 0) t.leaf_cnt[i] = 0;  // no logits for this row of the batch
        return;
    }
    bd[lane] = boards[(size_t)i * 64 + lane];
    if (lane == 0) {
        s_meta[0] = s.wtm; s_meta[1] = s.wkr; s_meta[2] = s.wkc; s_meta[3] = s.bkr; s_meta[4] = s.bkc;
        s_meta[5] = s.flags; s_meta[6] = s.ep;
    }
    __syncthreads();
    const size_t eb = (size_t)i * t.ecap, nb = (size_t)i * t.ncap;
    int* path = t.path + nb;
    int node = 0, depth = 0, leaf = -1, parent_n = 0;
    for (;;) {
        const NodeRec nd = t.node[nb + node];
        const int first = nd.first, cnt = nd.cnt;
        // a non-root node's visit count is its parent edge's (both rise in
        // the same backups), so only the root keeps one in its record
        const float sq = t.sqrt_tab[node == 0 ? nd.N : parent_n];
        float best = -INFINITY;
        int bi = 0x7fffffff;
        for (int j = lane; j < cnt; j += 64) {
            const size_t e = eb + first + j;
            const float sc = puct(t.c_puct, t.e_P[e], sq, t.e_N[e], t.e_W[e]);
            if (sc > best) {  // lanes see their edges in increasing j: strict > keeps the first
                best = sc;
                bi = j;
            }
        }
        wave_argmax_first(best, bi);
        const int e = first + bi;
        if (lane == 0) {
            path[depth] = e;
            make_move_board(bd, s_meta[0], s_meta[1], s_meta[2], s_meta[3], s_meta[4], s_meta[5], s_meta[6],
                            t.e_move[eb + e]);
        }
        ++depth;
        __syncthreads();
        const int child = t.e_child[eb + e];
        if (child == NO_CHILD || depth >= t.ncap) {
            leaf = e;
            break;
        }
        parent_n = t.e_N[eb + e];
        node = child;
    }
    MctsSlot m = t.ms[i];
    m.path_len = depth;
    m.leaf_edge = leaf;
    m.leaf_pending = 0;
    m.leaf_n = 0;
    m.leaf_value = 0.f;
    const int8_t code = bd[lane];
    if (__ballot(code != 0 && code != 1 && code != 7) == 0ull) {
        // GameState.isDraw after the move ends the game (self_play.py:180)
        m.leaf_value = 0.f;
    } else {
        Pos p = wave_pos(code, s_meta[0], s_meta[1], s_meta[2], s_meta[3], s_meta[4], s_meta[5], s_meta[6]);
        const int n = wave_valid_moves(p, t.leaf_moves + (size_t)i * MAXM, MAXM, lane);
        if (n > MAXM && lane == 0) atomicOr(&ctr->error, 1);
        m.leaf_wtm = p.wtm;
        if (n == 0) {
            m.leaf_value = in_check(p) ? (p.wtm ? -1.f : 1.f) : 0.f;  // mate / stalemate
        } else {
            bd[lane] = (int8_t)pos_at(p, lane);  // the board the reference would encode (after getValidMoves)
            m.leaf_pending = 1;
            m.leaf_n = n < MAXM ? n : MAXM;
            m.pad[1] += 1;
        }
    }
    if (lane == 0) {
        t.ms[i] = m;
        t.leaf_cnt[i] = m.leaf_pending ? m.leaf_n : 0;  // the logits the network computes for this slot
    }
    __syncthreads();
    nn_boards[(size_t)i * 64 + lane] = bd[lane];
}

// one slot's backup, by the 64 threads of its workgroup
__device__ inline void mcts_backup_slot(const DevCfg& cfg, const Tree& t, const Slot* slots, const float* logits,
                                        const float* values, float* probs, Ctr* ctr, int i) {
    __shared__ float pri[MAXM];
    const int lane = threadIdx.x;
    const Slot s = slots[i];
    if (s.status != ST_ACTIVE) return;
    MctsSlot m = t.ms[i];
    const size_t eb = (size_t)i * t.ecap, nb = (size_t)i * t.ncap;
    float v = m.leaf_value;
    if (m.leaf_pending) {
        v = values[i];
        // priors = softmax over the legal moves' logits only, which the network
        // wrote compactly in list order (kv_net_forward_boards_legal):
        // max, e_j = det_expf(l_j - max) kept in LDS, lane partial sums over
        // j = lane, lane+64, ... in order, xor butterfly
        const float* lg = t.leaf_logits + (size_t)i * MAXM;
        const uint16_t* lm = t.leaf_moves + (size_t)i * MAXM;
        const int n = m.leaf_n;
        float mx = -INFINITY;
        for (int j = lane; j < n; j += 64) {
            const float l = lg[j];
            pri[j] = l;
            mx = fmaxf(mx, l);
        }
        mx = wave_max(mx);
        float part = 0.f;
        for (int j = lane; j < n; j += 64) {
            const float e = det_expf(pri[j] - mx);
            pri[j] = e;
            part += e;
        }
        const float sum = wave_sum(part);
        // a node's edges start on a 16-edge boundary, so the descent's P / W
        // (and N / child / move) reads of one node touch the fewest HBM lines
        const int first = (m.edge_count + 15) & ~15;
        const bool fits = first + n <= t.ecap && m.node_count < t.ncap;
        if (fits) {
            for (int j = lane; j < n; j += 64) {
                const size_t e = eb + first + j;
                t.e_move[e] = lm[j];
                t.e_P[e] = sum > 0.f ? pri[j] / sum : 1.0f / (float)n;  // sum >= 1 for finite logits
                t.e_N[e] = 0;
                t.e_W[e] = 0.f;
                t.e_child[e] = NO_CHILD;
            }
        }
        if (lane == 0) {
            if (fits) {
                const int id = m.node_count;
                t.node[nb + id] = NodeRec{first, n, 0, 0};
                t.e_child[eb + m.leaf_edge] = (uint16_t)id;
                m.node_count += 1;
                m.edge_count = first + n;
            } else {
                // the expansion does not fit the slot's pools: counted and
                // raised as an error (kv_run -> KV_EOVERFLOW), never silent
                m.overflow += 1;
                atomicAdd(&ctr->tree_overflows, 1ull);
                atomicOr(&ctr->error, 4);
            }
            m.pad[0] += 1;
        }
    }
    if (lane == 0) {
        // backup along the path: the mover at depth d is the root side flipped d times
        // (a non-root node's visit count is its parent edge's N: only the
        // root's record is updated)
        const int* path = t.path + nb;
        t.node[nb].N += 1;
        for (int d = 0; d < m.path_len; ++d) {
            const size_t e = eb + path[d];
            const bool white_moved = ((m.root_wtm != 0) ^ (d & 1)) != 0;
            t.e_N[e] += 1;
            t.e_W[e] = t.e_W[e] + (white_moved ? v : -v);
        }
        t.ms[i] = m;
    }
}

__global__ __launch_bounds__(64) void k_mcts_select(DevCfg cfg, Tree t, const Slot* slots, const int8_t* boards,
                                                    int8_t* nn_boards, Ctr* ctr, int slot0) {
    mcts_select_slot(cfg, t, slots, boards, nn_boards, ctr, slot0 + blockIdx.x);
}

__global__ __launch_bounds__(64) void k_mcts_backup(DevCfg cfg, Tree t, const Slot* slots, const float* logits,
                                                    const float* values, float* probs, Ctr* ctr, int slot0) {
    mcts_backup_slot(cfg, t, slots, logits, values, probs, ctr, slot0 + blockIdx.x);
}

// backup of sim-step k and select of sim-step k+1 for the same slot in one
// launch (a slot's next descent depends only on its own tree): one kernel
// boundary less per sim-step. The barrier orders thread 0's tree writes
// before the descent reads them (workgroup scope).
__global__ __launch_bounds__(64) void k_mcts_backup_select(DevCfg cfg, Tree t, const Slot* slots,
                                                           const int8_t* boards, const float* logits,
                                                           const float* values, float* probs, int8_t* nn_boards,
                                                           Ctr* ctr, int slot0) {
    const int i = slot0 + blockIdx.x;
    mcts_backup_slot(cfg, t, slots, logits, values, probs, ctr, i);
    __syncthreads();
    mcts_select_slot(cfg, t, slots, boards, nn_boards, ctr, i);
}

__global__ __launch_bounds__(64) void k_mcts_choose(DevCfg cfg, Tree t, Slot* slots, int8_t* boards,
                                                    uint32_t* py_mt, kv_record* rec, int8_t* last_board, Ctr* ctr) {
    __shared__ double vals[MAXM];
    __shared__ double cum[MAXM];
    __shared__ int s_pick;
    const int i = blockIdx.x, lane = threadIdx.x;
    Slot s = slots[i];
    if (s.status != ST_ACTIVE) return;
    const MctsSlot m = t.ms[i];
    const size_t eb = (size_t)i * t.ecap, nb = (size_t)i * t.ncap;
    const int n = t.node[nb].cnt;
    for (int j = lane; j < n; j += 64) vals[j] = (double)t.e_N[eb + j];
    __syncthreads();
    if (lane == 0) s_pick = choose_weighted(vals, cum, n, py_mt + (size_t)i * MT_WORDS);
    __syncthreads();
    // the move's counters in one update per slot (one device-scope atomic per
    // slot and sim-step on a shared counter cost ~3.5 us per select / backup)
    if (lane == 0) {
        atomicAdd(&ctr->sims, (unsigned long long)cfg.sims);
        atomicAdd(&ctr->nn_rows, (unsigned long long)m.pad[1]);
    }
    s.last_value = m.root_value;  // resign test on the root's network value (:185)
    s.n_evals += m.pad[0];
    const unsigned long long ridx = commit_move(cfg, s, i, t.e_move[eb + s_pick], boards, rec, last_board, ctr, lane);
    if (t.root_visits && (long long)ridx < cfg.record_cap) {
        uint16_t* rv = t.root_visits + (size_t)ridx * MAXM;
        for (int j = lane; j < MAXM; j += 64) rv[j] = j < n ? t.e_N[eb + j] : (uint16_t)0xffff;
    }
    if (lane == 0) slots[i] = s;
}

// Test evaluator (KV_EVAL_HASH): all logits 0 (uniform priors, exact in
// float), value = dyadic hash of the 64 board codes. Lets the CPU restatement
// reproduce every PUCT score bit for bit.
__global__ void k_hash_eval(const int8_t* boards, int rows, float* logits, float* values) {
    const int r = blockIdx.x, lane = threadIdx.x;
    if (r >= rows) return;
    for (int j = lane; j < 4096; j += 64) logits[(size_t)r * 4096 + j] = 0.f;
    if (lane == 0) {
        uint32_t h = 2166136261u;
        for (int q = 0; q < 64; ++q) {
            h ^= (uint8_t)boards[(size_t)r * 64 + q];
            h *= 16777619u;
        }
        values[r] = (float)((int)(h % 129u) - 64) / 64.0f;
    }
}

// the hash evaluator's leaf logits (all 0) in kv_net_forward_boards_legal's layout
__global__ void k_hash_legal(int* cnt, float* out) {
    const int r = blockIdx.x, lane = threadIdx.x;
    for (int j = lane; j < cnt[r]; j += 64) out[(size_t)r * MAXM + j] = 0.f;
}

int hash_legal(const Tree& t, int rows, hipStream_t st) {
    hipLaunchKernelGGL(k_hash_legal, dim3(rows), dim3(64), 0, st, t.leaf_cnt, t.leaf_logits);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int mcts_root(const DevCfg& cfg, const Tree& t, Slot* slots, const uint16_t* moves, const float* logits,
              const float* values, float* probs, uint32_t* np_mt, Ctr* ctr, hipStream_t st) {
    hipLaunchKernelGGL(k_mcts_root, dim3(cfg.slots), dim3(256), 0, st, cfg, t, slots, moves, logits, values, probs,
                       np_mt, ctr);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int mcts_select(const DevCfg& cfg, const Tree& t, const Slot* slots, const int8_t* boards, int8_t* nn_boards,
                Ctr* ctr, hipStream_t st, int slot0, int count) {
    hipLaunchKernelGGL(k_mcts_select, dim3(count), dim3(64), 0, st, cfg, t, slots, boards, nn_boards, ctr, slot0);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int mcts_backup(const DevCfg& cfg, const Tree& t, const Slot* slots, const float* logits, const float* values,
                float* probs, Ctr* ctr, hipStream_t st, int slot0, int count) {
    hipLaunchKernelGGL(k_mcts_backup, dim3(count), dim3(64), 0, st, cfg, t, slots, logits, values, probs, ctr,
                       slot0);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int mcts_backup_select(const DevCfg& cfg, const Tree& t, const Slot* slots, const int8_t* boards, const float* logits,
                       const float* values, float* probs, int8_t* nn_boards, Ctr* ctr, hipStream_t st, int slot0,
                       int count) {
    hipLaunchKernelGGL(k_mcts_backup_select, dim3(count), dim3(64), 0, st, cfg, t, slots, boards, logits, values, probs,
                       nn_boards, ctr, slot0);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int mcts_choose(const DevCfg& cfg, const Tree& t, Slot* slots, int8_t* boards, uint32_t* py_mt, kv_record* rec,
                int8_t* last_board, Ctr* ctr, hipStream_t st) {
    hipLaunchKernelGGL(k_mcts_choose, dim3(cfg.slots), dim3(64), 0, st, cfg, t, slots, boards, py_mt, rec,
                       last_board, ctr);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

int hash_eval(const int8_t* boards, int rows, float* logits, float* values, hipStream_t st) {
    hipLaunchKernelGGL(k_hash_eval, dim3(rows), dim3(64), 0, st, boards, rows, logits, values);
    KV_HIP(hipGetLastError());
    return KV_OK;
}

}  // namespace kv
