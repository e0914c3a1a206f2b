// Device test entry points (include/kv.h "device test entry points"): run the
// product's own device functions over host-provided inputs so the parity
// tests can reach them through the C ABI.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "kv_common.h"
#include "kv_movegen.h"
#include "kv_rng.h"
#include "kv_libm.h"

#pragma clang fp contract(off)

namespace kv {

__device__ inline void pos_to_vec(const Pos& p, int8_t* v) {
    pos_to_board(p, v);
    v[64] = (int8_t)p.wtm;
    v[65] = p.wkr; v[66] = p.wkc; v[67] = p.bkr; v[68] = p.bkc;
    v[69] = (p.flags & F_WKM) ? 1 : 0; v[70] = (p.flags & F_BKM) ? 1 : 0;
    v[71] = (p.flags & F_WRK) ? 1 : 0; v[72] = (p.flags & F_WRQ) ? 1 : 0;
    v[73] = (p.flags & F_BRK) ? 1 : 0; v[74] = (p.flags & F_BRQ) ? 1 : 0;
    v[75] = p.ep < 0 ? -1 : p.ep / 8;
    v[76] = p.ep < 0 ? -1 : p.ep % 8;
    v[77] = v[78] = v[79] = 0;
}

__device__ inline Pos wave_pos_from_vec(const int8_t* v, int lane) {
    return wave_pos(v[lane], v[64], v[65], v[66], v[67], v[68],
                    (v[69] ? F_WKM : 0) | (v[70] ? F_BKM : 0) | (v[71] ? F_WRK : 0) | (v[72] ? F_WRQ : 0) |
                        (v[73] ? F_BRK : 0) | (v[74] ? F_BRQ : 0),
                    v[75] < 0 ? -1 : v[75] * 8 + v[76]);
}

// one wave per position, exactly as the engine runs the generator
__global__ __launch_bounds__(64) void k_dev_valid(const int8_t* states, int n, uint16_t* moves, int cap,
                                                  int* nmoves, int8_t* after, uint8_t* chk) {
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= n) return;
    Pos p = wave_pos_from_vec(states + (size_t)i * 80, lane);
    const int m = wave_valid_moves(p, moves + (size_t)i * cap, cap, lane);
    const bool c = in_check(p);
    if (lane == 0) {
        nmoves[i] = m > cap ? -m : m;
        pos_to_vec(p, after + (size_t)i * 80);
        chk[i] = c ? 1 : 0;
    }
}

__global__ __launch_bounds__(64) void k_dev_make(int8_t* states, const int* index, int n, uint16_t* scratch,
                                                 int* status) {
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= n) return;
    int8_t* v = states + (size_t)i * 80;
    Pos p = wave_pos_from_vec(v, lane);
    uint16_t* ml = scratch + (size_t)i * MAXM;
    const int m = wave_valid_moves(p, ml, MAXM, lane);
    __syncthreads();
    if (lane != 0) return;
    if (index[i] < 0 || index[i] >= m || index[i] >= MAXM) {
        status[i] = -1;
        return;
    }
    pos_to_vec(p, v);
    int wtm = p.wtm, wkr = p.wkr, wkc = p.wkc, bkr = p.bkr, bkc = p.bkc, fl = p.flags, ep = p.ep;
    make_move_board(v, wtm, wkr, wkc, bkr, bkc, fl, ep, ml[index[i]]);
    Pos q;
    pos_from_board(q, v, wtm, wkr, wkc, bkr, bkc, fl, ep);
    pos_to_vec(q, v);
    status[i] = 0;
}

// squareUnderAttack's set for the side to move (chessEngine.py:400-415): end
// squares of every opponent pseudo-move, one bit per square
__global__ void k_dev_attacks(const int8_t* states, int n, unsigned long long* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int8_t* v = states + (size_t)i * 80;
    Pos p;
    pos_from_board(p, v, v[64], v[65], v[66], v[67], v[68],
                   (v[69] ? F_WKM : 0) | (v[70] ? F_BKM : 0) | (v[71] ? F_WRK : 0) | (v[72] ? F_WRQ : 0) |
                       (v[73] ? F_BRK : 0) | (v[74] ? F_BRQ : 0),
                   v[75] < 0 ? -1 : v[75] * 8 + v[76]);
    out[i] = targets(p, p.wtm ? 1 : 0);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_dev_dirichlet(const unsigned long long* seeds, double alpha, int k,
                                                       int draws, double* out, long long* attempts, double* tail,
                                                       uint32_t* state) {
    __shared__ uint32_t mt3[MT_RW];
    __shared__ int scratch[RNG_SCRATCH];
    const int i = blockIdx.x, tid = threadIdx.x;
    uint32_t* g = state + (size_t)i * MT_WORDS;
    if (tid == 0) mt_seed_genrand(g, (uint32_t)seeds[i]);
    __syncthreads();
    BlockMT w;
    bmt_load(w, g, mt3, tid);
    for (int d = 0; d < draws; ++d) {
        double* o = out + ((size_t)i * draws + d) * k;
        long long att;
        const double acc = block_dirichlet_gamma(w, alpha, k, o, &att, scratch, tid);
        const double inv = 1 / acc;
        for (int j = tid; j < k; j += RNG_THREADS) o[j] = o[j] * inv;
        if (tid == 0) attempts[(size_t)i * draws + d] = att;
        __syncthreads();
    }
    const double t = block_random(w, tid);
    if (tid == 0) tail[i] = t;
}

__global__ void k_dev_py_random(const unsigned long long* seeds, int n, int count, double* out, uint32_t* state) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* g = state + (size_t)i * MT_WORDS;
    mt_seed_python(g, seeds[i]);
    for (int j = 0; j < count; ++j) out[(size_t)i * count + j] = mt_random_serial(g);
}

}  // namespace kv

extern "C" {

int kv_dev_valid_moves(int device, const int8_t* states, int n, uint16_t* moves_out, int cap, int* n_moves,
                       int8_t* states_after, uint8_t* in_check) {
    KV_REQUIRE(n > 0 && cap > 0 && states && moves_out && n_moves && states_after && in_check, KV_EINVAL,
               "kv_dev_valid_moves: bad arguments");
    KV_HIP(hipSetDevice(device));
    kv::DevBuf<int8_t> s, a;
    kv::DevBuf<uint16_t> m;
    kv::DevBuf<int> nm;
    kv::DevBuf<uint8_t> c;
    KV_HIP(s.alloc((size_t)n * 80));
    KV_HIP(a.alloc((size_t)n * 80));
    KV_HIP(m.alloc((size_t)n * cap));
    KV_HIP(nm.alloc(n));
    KV_HIP(c.alloc(n));
    KV_HIP(hipMemcpy(s.p, states, (size_t)n * 80, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kv::k_dev_valid, dim3(n), dim3(64), 0, 0, s.p, n, m.p, cap, nm.p, a.p, c.p);
    KV_HIP(hipGetLastError());
    KV_HIP(hipDeviceSynchronize());
    KV_HIP(hipMemcpy(moves_out, m.p, (size_t)n * cap * sizeof(uint16_t), hipMemcpyDeviceToHost));
    KV_HIP(hipMemcpy(n_moves, nm.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
    KV_HIP(hipMemcpy(states_after, a.p, (size_t)n * 80, hipMemcpyDeviceToHost));
    KV_HIP(hipMemcpy(in_check, c.p, (size_t)n, hipMemcpyDeviceToHost));
    return KV_OK;
}

int kv_dev_attacks(int device, const int8_t* states, int n, uint64_t* attacked) {
    KV_REQUIRE(n > 0 && states && attacked, KV_EINVAL, "kv_dev_attacks: bad arguments");
    KV_HIP(hipSetDevice(device));
    kv::DevBuf<int8_t> s;
    kv::DevBuf<unsigned long long> o;
    KV_HIP(s.alloc((size_t)n * 80));
    KV_HIP(o.alloc(n));
    KV_HIP(hipMemcpy(s.p, states, (size_t)n * 80, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kv::k_dev_attacks, dim3((n + 63) / 64), dim3(64), 0, 0, s.p, n, o.p);
    KV_HIP(hipGetLastError());
    KV_HIP(hipDeviceSynchronize());
    KV_HIP(hipMemcpy(attacked, o.p, (size_t)n * 8, hipMemcpyDeviceToHost));
    return KV_OK;
}

int kv_dev_make_move(int device, int8_t* states, const int* index, int n) {
    KV_REQUIRE(n > 0 && states && index, KV_EINVAL, "kv_dev_make_move: bad arguments");
    KV_HIP(hipSetDevice(device));
    kv::DevBuf<int8_t> s;
    kv::DevBuf<int> ix, stt;
    kv::DevBuf<uint16_t> scr;
    KV_HIP(s.alloc((size_t)n * 80));
    KV_HIP(ix.alloc(n));
    KV_HIP(stt.alloc(n));
    KV_HIP(scr.alloc((size_t)n * kv::MAXM));
    KV_HIP(hipMemcpy(s.p, states, (size_t)n * 80, hipMemcpyHostToDevice));
    KV_HIP(hipMemcpy(ix.p, index, (size_t)n * sizeof(int), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kv::k_dev_make, dim3(n), dim3(64), 0, 0, s.p, ix.p, n, scr.p, stt.p);
    KV_HIP(hipGetLastError());
    KV_HIP(hipDeviceSynchronize());
    std::vector<int> st(n);
    KV_HIP(hipMemcpy(st.data(), stt.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) KV_REQUIRE(st[i] == 0, KV_EINVAL, "kv_dev_make_move: index out of range at %d", i);
    KV_HIP(hipMemcpy(states, s.p, (size_t)n * 80, hipMemcpyDeviceToHost));
    return KV_OK;
}

int kv_dev_dirichlet(int device, const uint64_t* seeds, int n, double alpha, int k, int draws, double* out,
                     int64_t* attempts, double* tail) {
    KV_REQUIRE(n > 0 && k > 0 && draws > 0 && seeds && out && attempts && tail, KV_EINVAL,
               "kv_dev_dirichlet: bad arguments");
    KV_REQUIRE(alpha >= 2.2250738585072014e-308 && alpha < 1.0, KV_EINVAL, "kv_dev_dirichlet: alpha must be a normal double in (0,1)");
    KV_HIP(hipSetDevice(device));
    kv::DevBuf<unsigned long long> sd;
    kv::DevBuf<double> o, t;
    kv::DevBuf<long long> at;
    kv::DevBuf<uint32_t> st;
    KV_HIP(sd.alloc(n));
    KV_HIP(o.alloc((size_t)n * draws * k));
    KV_HIP(t.alloc(n));
    KV_HIP(at.alloc((size_t)n * draws));
    KV_HIP(st.alloc((size_t)n * kv::MT_WORDS));
    KV_HIP(hipMemcpy(sd.p, seeds, (size_t)n * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kv::k_dev_dirichlet, dim3(n), dim3(256), 0, 0, sd.p, alpha, k, draws, o.p, at.p, t.p, st.p);
    KV_HIP(hipGetLastError());
    KV_HIP(hipDeviceSynchronize());
    KV_HIP(hipMemcpy(out, o.p, (size_t)n * draws * k * sizeof(double), hipMemcpyDeviceToHost));
    KV_HIP(hipMemcpy(attempts, at.p, (size_t)n * draws * sizeof(long long), hipMemcpyDeviceToHost));
    KV_HIP(hipMemcpy(tail, t.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
    return KV_OK;
}

int kv_host_libm(int op, const double* x, const double* y, int n, double* out) {
    KV_REQUIRE(x && out && n >= 0 && (op == 0 || (op == 1 && y)), KV_EINVAL, "kv_host_libm: bad arguments");
    for (int i = 0; i < n; ++i) out[i] = op == 0 ? kv::glibc_log(x[i]) : kv::glibc_pow(x[i], y[i]);
    return KV_OK;
}

int kv_dev_py_random(int device, const uint64_t* seeds, int n, int count, double* out) {
    KV_REQUIRE(n > 0 && count > 0 && seeds && out, KV_EINVAL, "kv_dev_py_random: bad arguments");
    KV_HIP(hipSetDevice(device));
    kv::DevBuf<unsigned long long> sd;
    kv::DevBuf<double> o;
    kv::DevBuf<uint32_t> st;
    KV_HIP(sd.alloc(n));
    KV_HIP(o.alloc((size_t)n * count));
    KV_HIP(st.alloc((size_t)n * kv::MT_WORDS));
    KV_HIP(hipMemcpy(sd.p, seeds, (size_t)n * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kv::k_dev_py_random, dim3((n + 63) / 64), dim3(64), 0, 0, sd.p, n, count, o.p, st.p);
    KV_HIP(hipGetLastError());
    KV_HIP(hipDeviceSynchronize());
    KV_HIP(hipMemcpy(out, o.p, (size_t)n * count * sizeof(double), hipMemcpyDeviceToHost));
    return KV_OK;
}

}  // extern "C"
