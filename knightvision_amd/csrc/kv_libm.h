// glibc's double-precision log() and pow() restated bit for bit, for the
// device Dirichlet (scripts/self_play.py:153 np.random.dirichlet -> numpy
// legacy_standard_gamma -> libm log / pow).
//
// glibc >= 2.28 computes both with ARM optimized-routines' table-driven
// algorithms (sysdeps/ieee754/dbl-64/e_log.c, e_pow.c). On an x86-64 host
// with FMA the IFUNC picks the -mfma build, where GCC contracted several
// a*b+c expressions into fused multiply-adds; the sequences below follow that
// machine code operation for operation (every fma() here is one vfmadd /
// vfmsub of the resolved target, every other operation is separately
// rounded), so the device returns the same bits as numpy's calls. Tables:
// kv_libm_tables.h (tools/gen_libm_tables.py). Pinned against libm on the
// host by tests/test_libm_cpu.py (kv_host_libm through the C ABI) and on the
// GPU by tests/test_engine_gpu.py (Dirichlet values identical to numpy).
//
// Domain: what legacy gamma with 0 < shape < 1 feeds them.
//  * log(x): x in [2^-53, 1] -- 1 - res53 and (1 - U) / shape with
//    U > 1 - shape, both >= 2^-53 -- and the tests' wider normal range; the
//    subnormal / zero / negative input branch of e_log.c is never reached and
//    is not restated.
//  * pow(x, y): x = 0 or x in [2^-53, 2^1024) normal, y = 1/shape > 1 (shape a
//    normal double, kv_create). Every result is restated, including the
//    underflowing ones a small shape produces (U^(1/shape) < 2^-1022 once
//    shape < 53/1022): exp_inline's specialcase() (scaled subnormal result with
//    the double-rounding fix, and the scaled overflow side), the total
//    underflow / overflow for |y log x| >= 1024, and pow's |y| >= 2^63 case.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kv_libm_tables.h"

#pragma clang fp contract(off)

namespace kv {

__host__ __device__ inline double libm_asdouble(uint64_t u) {
    union { uint64_t u; double d; } x;
    x.u = u;
    return x.d;
}
__host__ __device__ inline uint64_t libm_asuint64(double d) {
    union { uint64_t u; double d; } x;
    x.d = d;
    return x.u;
}

// log (e_log.c with __FP_FAST_FMA), glibc 2.35 __log_fma
__host__ __device__ inline double glibc_log(double x) {
    const double* H = kv_log_hdr;  // ln2hi ln2lo A[0..4] B[0..10]
    const uint64_t ix = libm_asuint64(x);
    const uint64_t LO = 0x3fee000000000000ull;  // asuint64(1.0 - 0x1p-4)
    if (ix - LO < 0x3090000000000ull) {         // HI - LO, HI = asuint64(1.0 + 0x1.09p-4)
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double* B = H + 7;
        const double r = x - 1.0;
        const double r2 = r * r;
        const double r3 = r * r2;
        double in = fma(r3, B[10], fma(r2, B[9], fma(r, B[8], B[7])));
        in = fma(in, r3, fma(r2, B[6], fma(r, B[5], B[4])));
        in = fma(in, r3, fma(r2, B[3], fma(r, B[2], B[1])));
        const double t = fma(r, 134217728.0, r);  // r + r * 0x1p27
        const double rhi = fma(-134217728.0, r, t);
        const double rlo = r - rhi;
        const double rr = rhi * rhi;
        const double hi = fma(rr, B[0], r);
        double lo = fma(rr, B[0], r - hi);
        lo = fma(B[0] * rlo, rhi + r, lo);
        const double y = fma(in, r3, lo);
        return hi + y;
    }
    const uint64_t tmp = ix - 0x3fe6000000000000ull;  // OFF
    const int i = (int)((tmp >> 45) & 127);
    const double kd = (double)((int64_t)tmp >> 52);
    const double z = libm_asdouble(ix - (tmp & 0xfff0000000000000ull));
    const double invc = kv_log_tab[2 * i], logc = kv_log_tab[2 * i + 1];
    const double* A = H + 2;
    const double r = fma(z, invc, -1.0);
    const double w = fma(kd, H[0], logc);
    const double hi = r + w;
    const double r2 = r * r;
    const double lo = fma(kd, H[1], (w - hi) + r);
    const double r3 = r * r2;
    const double q = fma(fma(r, A[4], A[3]), r2, fma(r, A[2], A[1]));
    return fma(r3, q, fma(r2, A[0], lo)) + hi;
}

// exp_inline's specialcase() (e_pow.c), for 512 <= |ehi| < 1024, where the
// table scale 2^(k/N) has left the normal range. As the resolved __pow_fma
// evaluates it (0x76b88..0x76cd9 and 0x76e08 in this image's libm): the
// overflow side contracts scale + scale*tmp into one fma; the underflow side
// keeps scale * tmp separately rounded and, for |y| < 1, re-rounds y to the
// precision of the subnormal result before the final scaling (no double
// rounding).
__host__ __device__ inline double glibc_exp_specialcase(double tmp, uint64_t sbits, uint64_t ki) {
    if ((ki & 0x80000000ull) == 0) {  // k > 0: the exponent of scale overflowed by <= 460
        const double scale = libm_asdouble(sbits - (1009ull << 52));
        return fma(scale, tmp, scale) * 0x1p1009;
    }
    sbits += 1022ull << 52;  // k < 0: scale 2^1022 too large, the result lands in the subnormal range
    const double scale = libm_asdouble(sbits);
    const double st = scale * tmp;
    double y = scale + st;
    if (fabs(y) < 1.0) {
        const double one = y < 0.0 ? -1.0 : 1.0;
        double lo = (scale - y) + st;
        const double hi = y + one;
        lo = ((one - hi) + y) + lo;
        y = (lo + hi) - one;
        if (y == 0.0) y = libm_asdouble(sbits & 0x8000000000000000ull);  // the sign of 0
    }
    return y * 0x1p-1022;
}

// pow (e_pow.c with __FP_FAST_FMA), glibc 2.35 __pow_fma: log_inline -> exp_inline
__host__ __device__ inline double glibc_pow(double x, double y) {
    if (x == 0.0) return 0.0;  // y > 0 (the special-case path's result for +0)
    // pow's special-y path (e_pow.c: |y| >= 2^63, y > 0 here): 1 at x == 1,
    // else __math_oflow(0) = +inf for x > 1 and __math_uflow(0) = +0 for x < 1
    if (((uint32_t)(libm_asuint64(y) >> 52) & 0x7ff) >= 0x43e)
        return x == 1.0 ? 1.0 : (x > 1.0 ? libm_asdouble(0x7ff0000000000000ull) : 0.0);
    const double* P = kv_pow_log_hdr;  // ln2hi ln2lo A[0..6]
    const double* A = P + 2;
    const uint64_t ix = libm_asuint64(x);
    const uint64_t tmp = ix - 0x3fe6955500000000ull;  // OFF
    const int i = (int)((tmp >> 45) & 127);
    const double kd = (double)((int64_t)tmp >> 52);
    const double z = libm_asdouble(ix - (tmp & 0xfff0000000000000ull));
    const double invc = kv_pow_log_tab[4 * i], logc = kv_pow_log_tab[4 * i + 2], logctail = kv_pow_log_tab[4 * i + 3];
    const double t1 = fma(kd, P[0], logc);
    const double r = fma(z, invc, -1.0);
    const double ar = r * A[0];
    const double lo1 = fma(kd, P[1], logctail);
    const double pa = fma(r, A[2], A[1]);
    const double pb = fma(r, A[4], A[3]);
    const double t2 = r + t1;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double lo3 = fma(ar, r, -ar2);
    const double lo2 = (t1 - t2) + r;
    const double pc = fma(r, A[6], A[5]);
    const double hi = t2 + ar2;
    const double lo4 = (t2 - hi) + ar2;
    const double q = fma(ar2, fma(pc, ar2, pb), pa);
    const double lo = fma(ar3, q, ((lo1 + lo2) + lo3) + lo4);
    const double lhi = hi + lo;
    const double ltail = (hi - lhi) + lo;
    // exp_inline(ehi, elo, 0)
    const double ehi = y * lhi;
    const double elo = fma(y, ltail, fma(lhi, y, -ehi));
    const uint32_t abstop = (uint32_t)(libm_asuint64(ehi) >> 52) & 0x7ff;
    bool special = false;
    if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {  // |ehi| < 2^-54 or |ehi| >= 512
        if (abstop < 0x3c9) return ehi + 1.0;  // |ehi| < 2^-54 (abstop - top12(0x1p-54) wraps)
        if (abstop > 0x408)                    // |ehi| >= 1024: __math_uflow(0) / __math_oflow(0)
            return (libm_asuint64(ehi) >> 63) ? 0.0 : libm_asdouble(0x7ff0000000000000ull);
        special = true;                        // 512 <= |ehi| < 1024: specialcase() below
    }
    const double* E = kv_exp_hdr;  // invln2N shift negln2hiN negln2loN C2..C5
    const double kz = fma(ehi, E[0], E[1]);
    const uint64_t ki = libm_asuint64(kz);
    const double kk = kz - E[1];
    const double rr = fma(kk, E[3], fma(kk, E[2], ehi));
    const double re = elo + rr;
    const uint64_t idx = 2 * (ki & 127);
    const uint64_t sbits = kv_exp_tab[idx + 1] + (ki << 45);
    const double tail = libm_asdouble(kv_exp_tab[idx]);
    const double c23 = fma(re, E[5], E[4]);
    const double tr = re + tail;
    const double re2 = re * re;
    const double c45 = fma(re, E[7], E[6]);
    const double tmpv = fma(c45, re2 * re2, fma(c23, re2, tr));
    if (special) return glibc_exp_specialcase(tmpv, sbits, ki);
    const double scale = libm_asdouble(sbits);
    return fma(tmpv, scale, scale);
}

}  // namespace kv
