// Device MT19937 streams, bit-compatible with the two generators the
// reference's move selection reads (self_play.py:153 and :162-167):
//   * numpy legacy RandomState (init_genrand seeding, random_double = res53,
//     legacy_standard_gamma for shape < 1, dirichlet with a serial fp64 sum
//     and x * (1/acc));
//   * CPython random (init_by_array seeding, random() = res53, choices,
//     _randbelow_with_getrandbits).
// A stream lives in HBM as 624 state words + the output index (625 u32).
//
// The Dirichlet draw is workgroup-parallel: each gamma attempt consumes exactly
// four u32 (U = res53, V = -log(1 - res53)), so attempt a reads words
// 4a..4a+3 and 256 threads run 1,024 consecutive attempts at once; accepted
// attempts are ranked in order (ballots + prefix popcounts) and the draw stops
// at the exact attempt that yields element k-1 so the stream position matches
// the sequential generator word for word. The twist runs on the workgroup as
// the word recurrence, 227 words per barrier-separated step (BlockMT).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kv_libm.h"

// numpy/CPython evaluate these expressions without FMA contraction
#pragma clang fp contract(off)

namespace kv {

constexpr int MT_N = 624, MT_M = 397;
constexpr int MT_WORDS = 625;  // state + index

__host__ __device__ inline uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

__host__ __device__ inline uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000U) | (b & 0x7fffffffU);
    return m ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
}

// ------------------------------------------------- single-thread forms ----
__host__ __device__ inline void mt_seed_genrand(uint32_t* mt, uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < MT_N; ++i) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    mt[MT_N] = MT_N;
}

__host__ __device__ inline void mt_seed_by_array(uint32_t* mt, const uint32_t* key, int len) {
    mt_seed_genrand(mt, 19650218U);
    int i = 1, j = 0;
    int k = MT_N > len ? MT_N : len;
    for (; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
        ++i; ++j;
        if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
        if (j >= len) j = 0;
    }
    for (k = MT_N - 1; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
        ++i;
        if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
    }
    mt[0] = 0x80000000U;
    mt[MT_N] = MT_N;
}

// CPython random.seed(int n): |n| split into 32-bit little-endian words
__host__ __device__ inline void mt_seed_python(uint32_t* mt, uint64_t seed) {
    uint32_t key[2];
    int n = 0;
    key[n++] = (uint32_t)seed;
    if (seed >> 32) key[n++] = (uint32_t)(seed >> 32);
    mt_seed_by_array(mt, key, n);
}

// Wave-level seeding (one 64-lane wave, every lane calls): the same words as
// mt_seed_genrand / mt_seed_python. The recurrences are serial, so the chain
// runs on wave-uniform values (scalar ALU) and each word is parked with
// v_writelane in lane (i & 63) of register i >> 6; the state is then written
// to global memory with coalesced stores. No memory round trip sits on the
// chain: k_finish (which seeds every recycled slot) went from 115 to 55 us
// per step at 256 slots (rocprofv3, reference move selection).
constexpr int MT_REGS = (MT_N + 63) / 64;  // 10

// v_writelane: word x into lane l of r (x wave-uniform)
__device__ inline uint32_t put_lane(uint32_t r, uint32_t x, int l) { return (int)__lane_id() == l ? x : r; }

__device__ inline void wave_mt_store(const uint32_t (&r)[MT_REGS], uint32_t* g, int lane) {
#pragma unroll
    for (int m = 0; m < MT_REGS; ++m)
        if (m * 64 + lane < MT_N) g[m * 64 + lane] = r[m];
    if (lane == 0) g[MT_N] = MT_N;
}

__device__ inline void wave_seed_genrand(uint32_t* g, uint32_t s, int lane) {
    uint32_t r[MT_REGS] = {};
    uint32_t x = __builtin_amdgcn_readfirstlane(s);
    (void)lane;
#pragma unroll
    for (int m = 0; m < MT_REGS; ++m) {
        const int lend = m == MT_REGS - 1 ? MT_N - 64 * m : 64;
        for (int l = 0; l < lend; ++l) {
            const int i = m * 64 + l;
            if (i > 0) x = 1812433253U * (x ^ (x >> 30)) + (uint32_t)i;
            r[m] = put_lane(r[m], x, l);
        }
    }
    wave_mt_store(r, g, lane);
}

// init_genrand(19650218): the words init_by_array starts from, the same for every seed
struct MtInit19650218 {
    uint32_t v[MT_N];
    constexpr MtInit19650218() : v() {
        v[0] = 19650218U;
        for (int i = 1; i < MT_N; ++i) v[i] = 1812433253U * (v[i - 1] ^ (v[i - 1] >> 30)) + (uint32_t)i;
    }
};
__constant__ constexpr MtInit19650218 kMtInitPy{};

__device__ inline void wave_seed_python(uint32_t* g, uint64_t seed, int lane) {
    const uint32_t k0 = __builtin_amdgcn_readfirstlane((uint32_t)seed);
    const uint32_t k1 = __builtin_amdgcn_readfirstlane((uint32_t)(seed >> 32));
    const int len = k1 ? 2 : 1;
    uint32_t r[MT_REGS] = {};
    // init_by_array pass 1 (mt_seed_by_array's first loop, i = 1..623), fused with
    // the init_genrand(19650218) words it reads
    uint32_t prev = 19650218U;
    int j = 0;
#pragma unroll
    for (int m = 0; m < MT_REGS; ++m) {
        const int lend = m == MT_REGS - 1 ? MT_N - 64 * m : 64;
        for (int l = (m == 0 ? 1 : 0); l < lend; ++l) {
            const int i = m * 64 + l;
            const uint32_t gi = kMtInitPy.v[i];
            const uint32_t cur = (gi ^ ((prev ^ (prev >> 30)) * 1664525U)) + (j ? k1 : k0) + (uint32_t)j;
            r[m] = put_lane(r[m], cur, l);
            prev = cur;
            if (++j >= len) j = 0;
        }
    }
    // the 624th iteration after the wrap: mt[0] = mt[623], i = 1
    uint32_t cur = (__builtin_amdgcn_readlane(r[0], 1) ^ ((prev ^ (prev >> 30)) * 1664525U)) + (j ? k1 : k0) +
                   (uint32_t)j;
    r[0] = put_lane(r[0], cur, 1);
    prev = cur;
    // pass 2: i = 2..623, then the wrap and i = 1
#pragma unroll
    for (int m = 0; m < MT_REGS; ++m) {
        const int lend = m == MT_REGS - 1 ? MT_N - 64 * m : 64;
        for (int l = (m == 0 ? 2 : 0); l < lend; ++l) {
            const int i = m * 64 + l;
            cur = (__builtin_amdgcn_readlane(r[m], l) ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)i;
            r[m] = put_lane(r[m], cur, l);
            prev = cur;
        }
    }
    cur = (__builtin_amdgcn_readlane(r[0], 1) ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;
    r[0] = put_lane(r[0], cur, 1);
    r[0] = put_lane(r[0], 0x80000000U, 0);
    wave_mt_store(r, g, lane);
}

__host__ __device__ inline void mt_twist_serial(uint32_t* mt) {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + MT_M]);
    for (; kk < MT_N - 1; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + (MT_M - MT_N)]);
    mt[MT_N - 1] = mt_mix(mt[MT_N - 1], mt[0], mt[MT_M - 1]);
}

__host__ __device__ inline uint32_t mt_next_serial(uint32_t* mt) {
    if (mt[MT_N] >= (uint32_t)MT_N) {
        mt_twist_serial(mt);
        mt[MT_N] = 0;
    }
    return mt_temper(mt[mt[MT_N]++]);
}

__host__ __device__ inline double res53(uint32_t a, uint32_t b) {
    return ((a >> 5) * 67108864.0 + (b >> 6)) / 9007199254740992.0;
}

__host__ __device__ inline double mt_random_serial(uint32_t* mt) {
    const uint32_t a = mt_next_serial(mt);
    const uint32_t b = mt_next_serial(mt);
    return res53(a, b);
}

// _randbelow_with_getrandbits(n), CPython 3.10 random.py:239-249
__host__ __device__ inline int mt_randbelow_serial(uint32_t* mt, int n) {
    int k = 0;
    while ((n >> k) != 0) ++k;
    uint32_t r = mt_next_serial(mt) >> (32 - k);
    while ((int)r >= n) r = mt_next_serial(mt) >> (32 - k);
    return (int)r;
}

// ------------------------------------------------------ block forms ----
// Called by every thread of ONE 256-thread workgroup (4 waves).
constexpr int RNG_THREADS = 256;

// in-place twist of an LDS state: three dependency-free phases
// ([0,227) reads old words only; [227,454) and [454,623) read words the
// previous phase produced), then the last word
__device__ inline void mt_twist_block(uint32_t* mt, int tid) {
    constexpr int P = MT_N - MT_M;  // 227
#pragma unroll
    for (int ph = 0; ph < 3; ++ph) {
        const int lo = ph * P, hi = ph < 2 ? lo + P : MT_N - 1;
        const int kk = lo + tid;
        uint32_t v = 0;
        if (kk < hi) v = mt_mix(mt[kk], mt[kk + 1], ph == 0 ? mt[kk + MT_M] : mt[kk + (MT_M - MT_N)]);
        __syncthreads();
        if (kk < hi) mt[kk] = v;
        __syncthreads();
    }
    if (tid == 0) mt[MT_N - 1] = mt_mix(mt[MT_N - 1], mt[0], mt[MT_M - 1]);
    __syncthreads();
}

// A block-local view of a stream as the word sequence x_m of MT19937: the
// twist is the recurrence x_{m+624} = mix(x_m, x_{m+1}, x_{m+397}), so any 227
// consecutive new words depend only on older ones and one barrier-separated
// step of the workgroup extends the sequence by 227 words. The words live in
// an LDS ring of MT_RW (stream index m at ring[m & (MT_RW - 1)]); m counts from
// word 0 of the state loaded from HBM. rd = next word to consume, wr = words
// generated so far.
constexpr int MT_RW = 8192;
constexpr int MT_STEP = MT_N - MT_M;  // 227
struct BlockMT {
    uint32_t* ring;  // MT_RW words of LDS
    int rd;
    int wr;
};

__device__ inline void bmt_load(BlockMT& w, const uint32_t* g, uint32_t* lds_ring, int tid) {
    for (int i = tid; i < MT_N; i += RNG_THREADS) lds_ring[i] = g[i];
    w.ring = lds_ring;
    w.rd = (int)g[MT_N];  // 624: the state is spent, the next word needs the twist
    w.wr = MT_N;
    __syncthreads();
}

// extend the sequence by MT_STEP words (every thread of the workgroup)
__device__ inline void bmt_step(BlockMT& w, int tid) {
    constexpr int K = MT_RW - 1;
    const int m = w.wr + tid;
    if (tid < MT_STEP) w.ring[m & K] = mt_mix(w.ring[(m - MT_N) & K], w.ring[(m - MT_N + 1) & K], w.ring[(m - MT_STEP) & K]);
    w.wr += MT_STEP;
    __syncthreads();
}

// make words [rd, rd + need) addressable (need + 624 + 227 <= MT_RW)
__device__ inline void bmt_ensure(BlockMT& w, int need, int tid) {
    while (w.rd + need > w.wr) bmt_step(w, tid);
}

__device__ inline uint32_t bmt_word(const BlockMT& w, int j) {  // j relative to rd
    return mt_temper(w.ring[(w.rd + j) & (MT_RW - 1)]);
}

__device__ inline void bmt_advance(BlockMT& w, int n) { w.rd += n; }

// back to HBM as (state, index): the state holding word rd (a spent state with
// index 624 when rd sits on a state boundary), completed first if needed
__device__ inline void bmt_store(BlockMT& w, uint32_t* g, int tid) {
    int S = w.rd / MT_N, pos = w.rd - S * MT_N;
    if (pos == 0 && S > 0) {
        --S;
        pos = MT_N;
    }
    while (w.wr < MT_N * (S + 1)) bmt_step(w, tid);
    for (int i = tid; i < MT_N; i += RNG_THREADS) g[i] = w.ring[(MT_N * S + i) & (MT_RW - 1)];
    if (tid == 0) g[MT_N] = (uint32_t)pos;
}

// random() (two words as res53) from a stream in HBM, for every thread of the
// workgroup. When the draw crosses the end of the state the stream goes
// through LDS (`lds`, 624 words) and twists block-parallel instead of one
// lane walking 624 global read-modify-writes; same words as mt_random_serial.
__device__ inline double block_mt_random(uint32_t* g, uint32_t* lds, int tid) {
    __shared__ double s_r;
    const int idx = (int)g[MT_N];
    __syncthreads();  // every thread has the index before it is rewritten
    if (idx + 2 <= MT_N) {
        if (tid == 0) {
            s_r = res53(mt_temper(g[idx]), mt_temper(g[idx + 1]));
            g[MT_N] = (uint32_t)(idx + 2);
        }
        __syncthreads();
        return s_r;
    }
    for (int i = tid; i < MT_N; i += RNG_THREADS) lds[i] = g[i];
    __syncthreads();
    int p = idx;
    uint32_t wd[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (p >= MT_N) {
            mt_twist_block(lds, tid);
            p = 0;
        }
        wd[j] = mt_temper(lds[p]);
        ++p;
    }
    for (int i = tid; i < MT_N; i += RNG_THREADS) g[i] = lds[i];
    if (tid == 0) g[MT_N] = (uint32_t)p;
    __syncthreads();
    return res53(wd[0], wd[1]);
}

// numpy RandomState.dirichlet([alpha]*k) (legacy) without the final scaling:
// gamma values go to gam[0..k) (LDS or global), the serial left-to-right fp64
// sum is returned to every thread, *attempts gets the attempt count. Each
// attempt consumes exactly four u32 (U = res53, V = -log(1 - res53)), so a
// round runs DIR_AP x 256 consecutive attempts at once (attempt j*256 + tid of
// the round on thread tid: DIR_AP independent log/pow chains per thread for the
// scheduler to interleave); accepted attempts are ranked in attempt order
// (wave ballots + a prefix over the DIR_AP x 4 wave counts) and the draw stops
// at the exact attempt that yields element k-1, leaving the stream where the
// sequential generator leaves it. `scratch` is RNG_SCRATCH ints of LDS.
constexpr int DIR_AP = 4;
constexpr int RNG_SCRATCH = 4 * DIR_AP + 1;
__device__ inline double block_dirichlet_gamma(BlockMT& w, double alpha, int k, double* gam, long long* attempts,
                                               int* scratch, int tid) {
    constexpr int RA = DIR_AP * RNG_THREADS;  // attempts per round
    static_assert(4 * RA + MT_N + MT_STEP <= MT_RW, "MT ring too small for a round");
    const int lane = tid & 63, wave = tid >> 6;
    const double one_m = 1.0 - alpha, inv_a = 1. / alpha;
    int base = 0;
    long long att = 0;
    while (base < k) {
        bmt_ensure(w, 4 * RA, tid);
        double X[DIR_AP];
        bool ok[DIR_AP];
#pragma unroll
        for (int j = 0; j < DIR_AP; ++j) {
            const int a = j * RNG_THREADS + tid;
            const uint32_t w0 = bmt_word(w, 4 * a), w1 = bmt_word(w, 4 * a + 1);
            const uint32_t w2 = bmt_word(w, 4 * a + 2), w3 = bmt_word(w, 4 * a + 3);
            // legacy_standard_gamma (numpy legacy-distributions.c) with glibc's
            // log / pow restated bit for bit (kv_libm.h)
            const double U = res53(w0, w1);
            const double V = -glibc_log(1.0 - res53(w2, w3));
            if (U <= one_m) {
                X[j] = glibc_pow(U, inv_a);
                ok[j] = X[j] <= V;
            } else {
                const double Y = -glibc_log((1 - U) / alpha);
                X[j] = glibc_pow(one_m + alpha * Y, inv_a);
                ok[j] = X[j] <= (V + Y);
            }
        }
        unsigned long long mask[DIR_AP];
#pragma unroll
        for (int j = 0; j < DIR_AP; ++j) {
            mask[j] = __ballot(ok[j]);
            if (lane == 0) scratch[j * 4 + wave] = __popcll(mask[j]);
        }
        if (tid == 0) scratch[4 * DIR_AP] = RA;  // attempts used unless the draw completes here
        __syncthreads();
        const int rem = k - base;
        int before = 0, total = 0;  // accepted in (sub-round, wave) groups ahead of this thread's group
#pragma unroll
        for (int j = 0; j < DIR_AP; ++j) {
            int bj = before;
#pragma unroll
            for (int q = 0; q < 4; ++q) bj += q < wave ? scratch[j * 4 + q] : 0;
            const int rank = bj + __popcll(mask[j] & ((1ull << lane) - 1));
            if (ok[j] && rank == rem - 1) scratch[4 * DIR_AP] = j * RNG_THREADS + tid + 1;  // yields element k-1
            if (ok[j] && rank < rem) gam[base + rank] = X[j];
#pragma unroll
            for (int q = 0; q < 4; ++q) before += scratch[j * 4 + q];
        }
        total = before;
        __syncthreads();
        const int used = scratch[4 * DIR_AP];
        base += total < rem ? total : rem;
        att += used;
        bmt_advance(w, 4 * used);
        __syncthreads();  // scratch reused by the next round
    }
    __shared__ double s_acc;
    if (tid == 0) {
        double acc = 0.0;
        for (int i = 0; i < k; ++i) acc = acc + gam[i];
        s_acc = acc;
    }
    __syncthreads();
    *attempts = att;
    return s_acc;
}

// two consecutive u32 as res53 (numpy random_sample()); all threads get it
__device__ inline double block_random(BlockMT& w, int tid) {
    bmt_ensure(w, 2, tid);
    const double r = res53(bmt_word(w, 0), bmt_word(w, 1));
    bmt_advance(w, 2);
    return r;
}

}  // namespace kv
