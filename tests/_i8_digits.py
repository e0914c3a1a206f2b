"""numpy restatement of the int8-digit split and integer GEMMs
(knightvision_amd/csrc/kv_wino88i.h: KV_PREC_I8X5's 5 digits, the fp32 tower's 4, with per-row or
per-256-channel-segment exponents) for the tests: the same operations in the same order, so digits,
exponents and M compare bit for bit."""
import numpy as np

DIGITS = 5
LEVELS = 5


def row_exponents(a):
    """a [..., K] fp64 -> e [...] int (i8_row_exponent): the row max's biased exponent - 1022, plus one when
    its top 7 fraction bits are all ones; 0 for an all-zero row."""
    hi = (a.view(np.uint64) >> np.uint64(32)).astype(np.uint32) & np.uint32(0x7FFFFFFF)
    m = hi.max(axis=-1)
    bump = ((m & np.uint32(0xFE000)) == np.uint32(0xFE000)).astype(np.int64)
    return np.where(m > 0, (m >> np.uint32(20)).astype(np.int64) - 1022 + bump, 0)


def split(a, e, digits=DIGITS):
    """a [..., K], e [...] -> digits [digits][..., K] int8 (t = 128 a 2^-e; q = rint(t); t = 128 (t - q))."""
    t = np.ldexp(a, (7 - e[..., None]).astype(np.int32))
    out = []
    for _ in range(digits):
        q = np.rint(t)
        out.append(q.astype(np.int8))
        t = (t - q) * 128.0
    return np.stack(out)


def pack(d):
    """digits [DIGITS][X][R][K] -> the product's digit planes [X][K/32][DIGITS][R][32] int8."""
    D, X, R, K = d.shape
    return d.reshape(D, X, R, K // 32, 32).transpose(1, 3, 0, 2, 4).copy()


def gemm_seg(V, U):
    """The fp32 tower's GEMM with V's exponents per 256-channel segment (4 digits, K 512; wino88i32_gemm_kernel
    NSEG 2): each segment's levels combined exactly (2^14 H + L) and scaled by 2^(ev_s - 35), segment 1 added
    to segment 0 in fp64 (one rounding), times 2^eu, rounded to fp32. -> (M [X][R][C] widened, V digits
    [4][X][R][K], V exponents [X][2][R])."""
    X, R, K = V.shape
    assert K == 512
    eu = row_exponents(U)
    du = split(U, eu, 4).astype(np.float64)
    evs, dvs, total = [], [], None
    for sg in range(2):
        Vs = V[:, :, 256 * sg:256 * (sg + 1)]
        ev = row_exponents(Vs)
        dv = split(Vs, ev, 4)
        fv, fu = dv.astype(np.float64), du[:, :, :, 256 * sg:256 * (sg + 1)]
        lev = []
        for l in range(4):
            acc = np.zeros((X, R, U.shape[1]))
            for i in range(l + 1):
                acc += np.matmul(fv[i], np.swapaxes(fu[l - i], 1, 2))
            lev.append(acc)
        m = (lev[0] * 128 + lev[1]) * 16384.0 + (lev[2] * 128 + lev[3])  # exact: < 2^46
        part = np.ldexp(m, (ev[:, :, None] - 35).astype(np.int32))     # exact
        total = part if total is None else total + part                  # one fp64 rounding
        evs.append(ev)
        dvs.append(dv)
    M = np.ldexp(total, eu[:, None, :].astype(np.int32)).astype(np.float32).astype(np.float64)
    return M, np.concatenate(dvs, axis=-1), np.stack(evs, axis=1)


def gemm(V, U, digits=DIGITS):
    """V [X][R][K], U [X][C][K] fp64 -> (M [X][R][C], V digits [digits][X][R][K], V exponents [X][R]).
    digits 5: fp64 M (KV_PREC_I8X5); 4: M rounded to fp32 once (KV_ALGO_WINOGRAD88_I8), returned widened."""
    ev, eu = row_exponents(V), row_exponents(U)
    dv, du = split(V, ev, digits), split(U, eu, digits)
    fv, fu = dv.astype(np.float64), du.astype(np.float64)
    lev = []
    for l in range(digits):  # exact: every partial sum is an integer below 2^31
        acc = np.zeros((V.shape[0], V.shape[1], U.shape[1]))
        for i in range(l + 1):
            acc += np.matmul(fv[i], np.swapaxes(fu[l - i], 1, 2))
        lev.append(acc)
    m = lev[digits - 1]
    for l in range(digits - 2, -1, -1):
        m = m * 0.0078125 + lev[l]  # exact, as the kernel's fma
    M = np.ldexp(m, (ev[:, :, None] + eu[:, None, :] - 14).astype(np.int32))
    if digits == 4:
        M = M.astype(np.float32).astype(np.float64)
    return M, dv, ev


def row_exponents_r8(a):
    """KV_PREC_I8R4's rule (i8_row_exponent_r8): as row_exponents, plus one when the max's top 7 fraction bits
    are >= 126 (max >= 127/128 2^e), so every rint(a 2^(31 - e)) stays below 127/128 2^31."""
    hi = (a.view(np.uint64) >> np.uint64(32)).astype(np.uint32) & np.uint32(0x7FFFFFFF)
    m = hi.max(axis=-1)
    bump = ((m & np.uint32(0xFE000)) >= np.uint32(0xFC000)).astype(np.int64)
    return np.where(m > 0, (m >> np.uint32(20)).astype(np.int64) - 1022 + bump, 0)


def split_r8(a, e):
    """a [..., K], e [...] -> the 4 radix-256 digits [4][..., K] int8, d_0 most significant: N = rint(a
    2^(31 - e)), N = sum_i d_i 2^(8 (3 - i)) with every d_i in [-128, 127] (the bytes of N + 0x80808080, each
    minus 128)."""
    N = np.rint(np.ldexp(a, (31 - e[..., None]).astype(np.int32))).astype(np.int64)
    u = (N + 0x80808080) & 0xFFFFFFFF
    return np.stack([(((u >> (8 * (3 - i))) & 255) - 128).astype(np.int8) for i in range(4)])


def gemm_r8(V, U):
    """KV_PREC_I8R4's GEMM (wino88i_gemm_lag5_kernel<K, 2, 4, 8>): V [X][R][K], U [X][C][K] fp64 -> (M fp64,
    V digits [4][X][R][K], V exponents [X][R]); the 13 pairs i + j <= 4 as 5 exact integer levels, combined
    m = L4, m = m 2^-8 + L_l (each step one fp64 rounding, as the kernel's fma with an exact product), scaled
    by 2^(ev + eu - 14)."""
    ev, eu = row_exponents_r8(V), row_exponents_r8(U)
    dv, du = split_r8(V, ev), split_r8(U, eu)
    fv, fu = dv.astype(np.float64), du.astype(np.float64)
    lev = []
    for l in range(5):
        acc = np.zeros((V.shape[0], V.shape[1], U.shape[1]))
        for i in range(4):
            if 0 <= l - i < 4:
                acc += np.matmul(fv[i], np.swapaxes(fu[l - i], 1, 2))
        lev.append(acc)
    m = lev[4]
    for l in range(3, -1, -1):
        m = m * 0.00390625 + lev[l]
    return np.ldexp(m, (ev[:, :, None] + eu[:, None, :] - 14).astype(np.int32)), dv, ev


def row_exponents_r3(a):
    """KV_PATH_WINO88_I8F32R3's rule: the radix-256 one (row_exponents_r8) on fp64 rows; on fp32 rows (a is
    fp32-representable, widened) the same rule read from the fp32 bits (i8_row_exponent_f32r: biased exponent
    - 126, plus one when the top 6 fraction bits are all ones) -- both give the e with max < 127/128 2^e."""
    return row_exponents_r8(a)


def row_exponents_r3_f32(a):
    """i8_row_exponent_f32r on fp32 rows a [..., K] (float32)."""
    b = np.abs(a.astype(np.float32)).view(np.uint32)
    m = b.max(axis=-1)
    bump = ((m & np.uint32(0x7E0000)) == np.uint32(0x7E0000)).astype(np.int64)
    return np.where(m > 0, (m >> np.uint32(23)).astype(np.int64) - 126 + bump, 0)


def split_r3(a, e):
    """a [..., K], e [...] -> the 3 radix-256 digits [3][..., K] int8, d_0 most significant: N = rint(a 2^(23 - e))
    (ties to even), N = d_0 2^16 + d_1 2^8 + d_2 with every d_i in [-128, 127] (the bytes of N + 0x808080, each
    minus 128)."""
    N = np.rint(np.ldexp(np.asarray(a, dtype=np.float64), (23 - e[..., None]).astype(np.int32))).astype(np.int64)
    u = (N + 0x808080) & 0xFFFFFF
    return np.stack([(((u >> (8 * (2 - i))) & 255) - 128).astype(np.int8) for i in range(3)])


def gemm_r3(V, U, f32_rows=False):
    """KV_PATH_WINO88_I8F32R3's GEMM (wino88i32_gemm_r3k64_kernel<K, TPW>): V [X][R][K], U [X][C][K]
    -> (M [X][R][C] rounded to fp32 once, returned widened; V digits [3][X][R][K]; V exponents [X][R]). The 6 pairs i + j <= 2 as 3 exact integer levels, combined m = L2, m = m 2^-8 + L_l (exact), scaled
    by 2^(ev + eu - 14). f32_rows: V's exponents by the fp32-bit rule (the output kernel's and conv2's slice of
    fp32 V), U's always from fp64."""
    ev = row_exponents_r3_f32(V) if f32_rows else row_exponents_r3(V)
    eu = row_exponents_r3(U)
    dv, du = split_r3(V, ev), split_r3(U, eu)
    fv, fu = dv.astype(np.float64), du.astype(np.float64)
    lev = []
    for l in range(3):
        acc = np.zeros((V.shape[0], V.shape[1], U.shape[1]))
        for i in range(l + 1):
            acc += np.matmul(fv[i], np.swapaxes(fu[l - i], 1, 2))
        lev.append(acc)
    m = lev[2]
    for l in (1, 0):
        m = m * 0.00390625 + lev[l]  # exact, as the kernel's fma
    M = np.ldexp(m, (ev[:, :, None] + eu[:, None, :] - 14).astype(np.int32)).astype(np.float32).astype(np.float64)
    return M, dv, ev
