// Device MT19937 streams, bit-compatible with the two generators the
// reference's move selection reads (self_play.py:153 and :162-167):
//   * numpy legacy RandomState (init_genrand seeding, random_double = res53,
//     legacy_standard_gamma for shape < 1, dirichlet with a serial fp64 sum
//     and x * (1/acc));
//   * CPython random (init_by_array seeding, random() = res53, choices,
//     _randbelow_with_getrandbits).
// A stream lives in HBM as 624 state words + the output index (625 u32).
//
// The Dirichlet draw is wave-parallel: each gamma attempt consumes exactly four
// u32 (U = res53, V = -log(1 - res53)), so attempt a reads words 4a..4a+3 and
// the 64 lanes of a wave run 64 consecutive attempts at once; accepted attempts
// are compacted in order with a ballot + prefix popcount, and the draw stops at
// the exact attempt that yields element k-1 so the stream position matches the
// sequential generator word for word. The twist is done by the wave in three
// dependency-free phases ([0,227), [227,454), [454,623) + the last word).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// ------------------------------------------------------- wave forms ----
// All of these are called by every lane of ONE 64-lane wave (blockDim 64).

// in-place twist of an LDS state
__device__ inline void mt_twist_wave(uint32_t* mt, int lane) {
    for (int base = 0; base < MT_N - MT_M; base += 64) {  // [0,227): reads old words only
        const int kk = base + lane;
        uint32_t v = 0;
        if (kk < MT_N - MT_M) v = mt_mix(mt[kk], mt[kk + 1], mt[kk + MT_M]);
        __syncthreads();
        if (kk < MT_N - MT_M) mt[kk] = v;
        __syncthreads();
    }
    for (int lo = MT_N - MT_M; lo < MT_N - 1; lo += MT_N - MT_M) {  // [227,454), [454,623)
        const int hi = lo + (MT_N - MT_M) < MT_N - 1 ? lo + (MT_N - MT_M) : MT_N - 1;
        for (int base = lo; base < hi; base += 64) {
            const int kk = base + lane;
            uint32_t v = 0;
            if (kk < hi) v = mt_mix(mt[kk], mt[kk + 1], mt[kk + (MT_M - MT_N)]);
            __syncthreads();
            if (kk < hi) mt[kk] = v;
            __syncthreads();
        }
    }
    if (lane == 0) mt[MT_N - 1] = mt_mix(mt[MT_N - 1], mt[0], mt[MT_M - 1]);
    __syncthreads();
}

// A wave-local view of a stream: `cur` holds the raw state whose tempered
// words are being consumed at index `pos`; `nxt` the state after one more
// twist (valid when have_nxt).
struct WaveMT {
    uint32_t* cur;
    uint32_t* nxt;
    int pos;
    int have_nxt;
};

__device__ inline void wmt_load(WaveMT& w, const uint32_t* g, uint32_t* lds_a, uint32_t* lds_b, int lane) {
    for (int i = lane; i < MT_N; i += 64) lds_a[i] = g[i];
    w.cur = lds_a;
    w.nxt = lds_b;
    w.pos = (int)g[MT_N];
    w.have_nxt = 0;
    __syncthreads();
    if (w.pos >= MT_N) {
        mt_twist_wave(w.cur, lane);
        w.pos = 0;
    }
}

__device__ inline void wmt_store(const WaveMT& w, uint32_t* g, int lane) {
    for (int i = lane; i < MT_N; i += 64) g[i] = w.cur[i];
    if (lane == 0) g[MT_N] = (uint32_t)w.pos;
}

// make words [pos, pos + need) addressable (need <= 624)
__device__ inline void wmt_ensure(WaveMT& w, int need, int lane) {
    if (w.pos + need > MT_N && !w.have_nxt) {
        for (int i = lane; i < MT_N; i += 64) w.nxt[i] = w.cur[i];
        __syncthreads();
        mt_twist_wave(w.nxt, lane);
        w.have_nxt = 1;
    }
}

__device__ inline uint32_t wmt_word(const WaveMT& w, int j) {  // j relative to pos
    const int i = w.pos + j;
    return mt_temper(i < MT_N ? w.cur[i] : w.nxt[i - MT_N]);
}

__device__ inline void wmt_advance(WaveMT& w, int n) {
    w.pos += n;
    if (w.pos >= MT_N && w.have_nxt) {  // pos == MT_N without nxt: cur exhausted, twist on demand
        uint32_t* t = w.cur;
        w.cur = w.nxt;
        w.nxt = t;
        w.pos -= MT_N;
        w.have_nxt = 0;
    }
}

__device__ inline double wave_bcast_d(double v, int src) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), src);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), src);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// numpy RandomState.dirichlet([alpha]*k) (legacy). gamma values go to `gam`
// (k doubles, global or LDS), the serial sum is returned to every lane;
// *attempts receives the attempt count. Caller multiplies by 1/acc when it
// needs normalised values (the reference computes val * invacc).
__device__ inline double wave_dirichlet_gamma(WaveMT& w, double alpha, int k, double* gam, long long* attempts,
                                              int lane) {
    const double one_m = 1.0 - alpha, inv_a = 1. / alpha;
    double acc = 0.0;
    int base = 0;
    long long att = 0;
    while (base < k) {
        wmt_ensure(w, 256, lane);
        const uint32_t w0 = wmt_word(w, 4 * lane), w1 = wmt_word(w, 4 * lane + 1);
        const uint32_t w2 = wmt_word(w, 4 * lane + 2), w3 = wmt_word(w, 4 * lane + 3);
        const double U = res53(w0, w1);
        const double V = -log(1.0 - res53(w2, w3));
        double X;
        bool ok;
        if (U <= one_m) {
            X = pow(U, inv_a);
            ok = X <= V;
        } else {
            const double Y = -log((1 - U) / alpha);
            X = pow(one_m + alpha * Y, inv_a);
            ok = X <= (V + Y);
        }
        const unsigned long long mask = __ballot(ok);
        const int cnt = __popcll(mask);
        const int rem = k - base;
        int used = 64;
        unsigned long long take = mask;
        if (cnt >= rem) {  // stop at the attempt that yields element k-1
            unsigned long long m = mask;
            for (int i = 0; i < rem - 1; ++i) m &= m - 1;
            const int last = __ffsll(m) - 1;
            used = last + 1;
            take = (last == 63) ? mask : (mask & ((2ull << last) - 1));
        }
        const unsigned long long below = lane == 0 ? 0ull : (take & ((1ull << lane) - 1));
        if ((take >> lane) & 1) gam[base + __popcll(below)] = X;
        // serial left-to-right accumulation in element order
        for (unsigned long long m = take; m; m &= m - 1) acc = acc + wave_bcast_d(X, __ffsll(m) - 1);
        base += __popcll(take);
        att += used;
        wmt_advance(w, 4 * used);
    }
    *attempts = att;
    return acc;
}

// two consecutive u32 as res53 (CPython random() / numpy random_sample())
__device__ inline double wave_random(WaveMT& w, int lane) {
    wmt_ensure(w, 2, lane);
    const double r = res53(wmt_word(w, 0), wmt_word(w, 1));
    wmt_advance(w, 2);
    return r;
}

__device__ inline int wave_randbelow(WaveMT& w, int n, int lane) {
    int k = 0;
    while ((n >> k) != 0) ++k;
    for (;;) {
        wmt_ensure(w, 1, lane);
        const uint32_t r = wmt_word(w, 0) >> (32 - k);
        wmt_advance(w, 1);
        if ((int)r < n) return (int)r;
    }
}

}  // namespace kv
