"""KV_PREC_I8X5's slice and GEMM kernels (csrc/kv_wino88i.h) through
kv_dev_wino88i, bit for bit against the numpy restatement (tests/_i8_digits.py):
the digits and row exponents of V, and M -- per-row block fixed point, the
digit pairs i + j < digits, exact int32 levels -- so any lane-mapping or
accumulation slip shows as a differing bit; and M against the fp64 product
of the unsplit operands within the bound the arithmetic implies. 4 digits (the fp32 domain) use the row-line layout
[xi][K/32][row][4][32]; 5 digits the planes [xi][K/32][5][row][32]."""
import ctypes as C

import numpy as np
import pytest

from tests import _i8_digits as D

pytestmark = pytest.mark.gpu


def _run(V, U, digits=D.DIGITS, seg=0):
    from knightvision_amd import _lib
    L = _lib.lib()
    X, R, K = V.shape
    M = np.zeros((X, R, 512))
    dg = np.zeros((X, K // 32, digits, R, 32), dtype=np.int8)
    ex = np.zeros((X, 2, R) if seg == 1 else (X, R), dtype=np.int32)
    P = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    _lib.check(L.kv_dev_wino88i(0, P(np.ascontiguousarray(V), C.c_double), R, P(np.ascontiguousarray(U), C.c_double),
                                K, digits, seg, P(M, C.c_double), P(dg, C.c_int8), P(ex, C.c_int32)), "kv_dev_wino88i")
    return M, dg, ex


@pytest.mark.parametrize("K,rows,digits", [(256, 128, 5), (512, 128, 5), (512, 256, 5), (256, 128, 4), (512, 128, 4)])
def test_i8_gemm_bit_exact(K, rows, digits):
    rng = np.random.default_rng(K + rows)
    V = rng.standard_normal((100, rows, K)) * np.exp2(rng.integers(-20, 20, size=(100, rows, 1)))
    V[0, 0] = 0.0                                 # all-zero row
    V[1, 1] = np.nextafter(np.exp2(3.0), 0.0)     # max just under a power of two: the exponent steps up
    V[2, 2, ::3] = 1e-310                         # subnormals beside normals
    V[3, 3] = np.where(rng.random(K) < 0.5, -1.0, 1.0) * np.exp2(-40.0)
    U = rng.standard_normal((100, 512, K)) * 0.05
    U[5, 7] = 0.0
    if digits == 4:  # the fp32 domain: fp32 operands
        V, U = V.astype(np.float32).astype(np.float64), U.astype(np.float32).astype(np.float64)
    M, dg, ex = _run(V, U, digits)
    Mr, dv, evr = D.gemm(V, U, digits)
    assert np.array_equal(ex, evr.astype(np.int32))
    want = D.pack(dv)
    if digits == 4:  # row lines
        want = want.transpose(0, 1, 3, 2, 4)
    assert np.array_equal(dg.reshape(want.shape), want)
    assert np.array_equal(M.view(np.uint64), Mr.view(np.uint64)), float(np.abs(M - Mr).max())


@pytest.mark.parametrize("K,rows", [(256, 128), (512, 128), (512, 256)])
def test_i8r_gemm_bit_exact(K, rows):
    """KV_PREC_I8R4: the radix-256 slice kernel (4 balanced byte digits of rint(a 2^(31 - e)), the exponent
    bumped at 127/128 of a power of two) and the 13-pair lag GEMM, bit for bit against tests/_i8_digits
    (split_r8, gemm_r8): digits, exponents, fp64 M. Rows at the exponent rule's edges: a max just under
    127/128 2^3 (no bump), exactly 127/128 2^3 (bump), an all-zero row, subnormals, +-2^-40."""
    rng = np.random.default_rng(K + rows + 3)
    V = rng.standard_normal((100, rows, K)) * np.exp2(rng.integers(-20, 20, size=(100, rows, 1)))
    V[0, 0] = 0.0
    V[1, 1] = np.nextafter(8.0 * 127 / 128, 0.0) * np.where(rng.random(K) < 0.5, -1.0, 1.0)
    V[1, 2] = 8.0 * 127 / 128
    V[1, 3] = -8.0 * 255 / 256
    V[2, 2, ::3] = 1e-310
    V[3, 3] = np.where(rng.random(K) < 0.5, -1.0, 1.0) * np.exp2(-40.0)
    U = rng.standard_normal((100, 512, K)) * 0.05
    U[5, 7] = 0.0
    M, dg, ex = _run(V, U, 4, seg=2)
    Mr, dv, evr = D.gemm_r8(V, U)
    assert np.array_equal(ex, evr.astype(np.int32))
    assert ex[1, 1] == 3 and ex[1, 2] == 4 and ex[1, 3] == 4
    assert np.array_equal(dg.reshape(100, K // 32, rows, 4, 32), D.pack(dv).transpose(0, 1, 3, 2, 4))  # row lines
    assert np.array_equal(M.view(np.uint64), Mr.view(np.uint64)), float(np.abs(M - Mr).max())


@pytest.mark.parametrize("K,rows", [(256, 128), (512, 128), (512, 256), (512, 2048)])
def test_i8r3_gemm_bit_exact(K, rows):
    """KV_PATH_WINO88_I8F32R3: the slice kernel's 3 radix-256 digits (balanced bytes of rint(a 2^(23 - e)), the
    exponent bumped at 127/128 of a power of two) in 96-byte row lines [100][K/32][rows][3][32], and the 6-pair
    GEMM (3 digit levels; wino88i32_gemm_r3k64_kernel: 64-k stages, at 2,048 rows C3's grid with 5 tiles per
    workgroup), bit for bit against tests/_i8_digits (split_r3, gemm_r3): digits, exponents, M rounded to fp32.
    Rows at the exponent rule's edges, an all-zero row, subnormals, +-2^-40."""
    rng = np.random.default_rng(K + rows + 5)
    V = rng.standard_normal((100, rows, K)) * np.exp2(rng.integers(-20, 20, size=(100, rows, 1)))
    V[0, 0] = 0.0
    V[1, 1] = np.nextafter(8.0 * 127 / 128, 0.0) * np.where(rng.random(K) < 0.5, -1.0, 1.0)
    V[1, 2] = 8.0 * 127 / 128
    V[1, 3] = -8.0 * 255 / 256
    V[2, 2, ::3] = 1e-310
    V[3, 3] = np.where(rng.random(K) < 0.5, -1.0, 1.0) * np.exp2(-40.0)
    U = rng.standard_normal((100, 512, K)) * 0.05
    U[5, 7] = 0.0
    M, dg, ex = _run(V, U, 4, seg=3)
    Mr, dv, evr = D.gemm_r3(V, U)
    assert np.array_equal(ex, evr.astype(np.int32))
    assert ex[1, 1] == 3 and ex[1, 2] == 4 and ex[1, 3] == 4
    nb = 100 * K * rows * 3  # 96-byte row lines fill the first 3/4 of the (4-digit-sized) buffer
    lines = dg.reshape(-1)[:nb].reshape(100, K // 32, rows, 3, 32)
    assert not dg.reshape(-1)[nb:].any()  # nothing written past them
    assert np.array_equal(lines, D.pack(dv).transpose(0, 1, 3, 2, 4))
    assert np.array_equal(M.view(np.uint64), Mr.view(np.uint64)), float(np.abs(M - Mr).max())


@pytest.mark.parametrize("rows,resid", [(128, False), (128, True), (256, True)])
def test_i8r_out_kernel_writes_the_two_kernel_forms_digits(rows, resid):
    """wino88i64r_out_kernel (KV_PREC_I8R4's output step: fp64 output transform + BN (+ residual) + ReLU, then
    the next V as the fp64 input transform of that activation, cut to 4 radix-256 digits in row lines, one
    workgroup per board) == wino88d_out_half_kernel's Y + wino88d_in_kernel's fp64 V + the radix-256 slice
    kernel, bit for bit; and its digits decode to numpy's fp64 transform of Y within half a unit of the 31-bit
    block (2^(e-32)) plus fp64 rounding, with the radix-256 exponent rule on numpy's row max."""
    from knightvision_amd import _lib
    from tests._wino_emul import input_transform_f64
    L = _lib.lib()
    rng = np.random.default_rng(rows + 17 * resid)
    M = rng.standard_normal((100, rows, 512)) * 0.3
    M[:, 5, :] = 0.0
    scale = (0.5 + rng.random(512)).astype(np.float32)
    scale[::7] *= np.float32(2.0 ** -12)
    shift = -np.abs(rng.standard_normal(512) * 0.1).astype(np.float32)
    R = (np.abs(rng.standard_normal((rows, 64, 512))) * 0.5).astype(np.float32) if resid else None
    if resid:
        R[5] = 0.0
    P = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    out = []
    for fused in (1, 0):
        Y = np.zeros((rows, 64, 512), dtype=np.float32)
        dg = np.zeros((100, 16, rows, 4, 32), dtype=np.int8)
        ex = np.zeros((100, rows), dtype=np.int32)
        rp = P(np.ascontiguousarray(R), C.c_float) if resid else None
        _lib.check(L.kv_dev_wino88r_out(0, P(np.ascontiguousarray(M), C.c_double), rows, P(scale, C.c_float),
                                        P(shift, C.c_float), rp, fused, P(Y, C.c_float), P(dg, C.c_int8),
                                        P(ex, C.c_int32)), "kv_dev_wino88r_out")
        out.append((Y, dg, ex))
    (Yf, df, ef), (Ys, ds, es) = out
    assert np.array_equal(Yf.view(np.uint32), Ys.view(np.uint32))
    assert np.array_equal(ef, es) and np.array_equal(df, ds)
    assert (ef[:, 5] == 0).all() and not df[:, :, 5].any()
    V = input_transform_f64(Yf.astype(np.float64))
    assert np.array_equal(ef, D.row_exponents_r8(V).astype(np.int32))
    dec = np.zeros_like(V)
    dgt = df.astype(np.float64).transpose(0, 2, 1, 4, 3)           # [100][rows][16][32][4]
    for d in range(4):
        dec += dgt[..., d].reshape(100, rows, 512) * 2.0 ** (-8 * d)
    dec = np.ldexp(dec, (ef - 7)[:, :, None])
    tol = np.ldexp(1.0, ef - 32)[:, :, None] + 1e-12 * np.abs(V).max(-1)[:, :, None]
    assert (np.abs(dec - V) <= tol).all(), float((np.abs(dec - V) / tol).max())


@pytest.mark.parametrize("rows", [128, 256])
def test_i8f32_segment_gemm_bit_exact(rows):
    """The fp32 tower's GEMM with V's exponents per 256-channel segment (KV_I8F32_SEG=1): digits, the two
    segment exponents of every row and M bit for bit against the numpy restatement (tests/_i8_digits.gemm_seg),
    including rows whose two halves sit 2^20 apart and a row with one all-zero half."""
    rng = np.random.default_rng(rows + 7)
    V = rng.standard_normal((100, rows, 512)) * np.exp2(rng.integers(-20, 20, size=(100, rows, 1)))
    V[:, 4, 256:] *= 2.0 ** -20
    V[:, 5, :256] = 0.0
    U = rng.standard_normal((100, 512, 512)) * 0.05
    V, U = V.astype(np.float32).astype(np.float64), U.astype(np.float32).astype(np.float64)
    M, dg, ex = _run(V, U, 4, seg=1)
    Mr, dv, evr = D.gemm_seg(V, U)
    assert np.array_equal(ex, evr.astype(np.int32))
    assert (ex[:, 1, 4] < ex[:, 0, 4]).all() and (ex[:, 0, 5] == 0).all()
    assert np.array_equal(dg.reshape(100, 16, rows, 4, 32), D.pack(dv).transpose(0, 1, 3, 2, 4))
    assert np.array_equal(M.view(np.uint64), Mr.view(np.uint64)), float(np.abs(M - Mr).max())


def _out(M, scale, shift, resid, flags):
    from knightvision_amd import _lib
    L = _lib.lib()
    R = M.shape[1]
    Y = np.zeros((R, 64, 512), dtype=np.float32)
    dg = np.zeros((100, 16, R, 4, 32), dtype=np.int8)
    ex = np.zeros((100, 2, R) if flags & 2 else (100, R), dtype=np.int32)
    P = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    rp = P(np.ascontiguousarray(resid), C.c_float) if resid is not None else None
    _lib.check(L.kv_dev_wino88i32_out(0, P(np.ascontiguousarray(M), C.c_float), R, P(scale, C.c_float),
                                      P(shift, C.c_float), rp, int(flags), P(Y, C.c_float), P(dg, C.c_int8),
                                      P(ex, C.c_int32)), "kv_dev_wino88i32_out")
    if flags & 16:  # R3: 96-byte row lines [100][16][R][3][32] in the first 3/4 of the buffer, nothing after
        nb = 100 * 16 * R * 96
        assert not dg.reshape(-1)[nb:].any()
        dg = dg.reshape(-1)[:nb].reshape(100, 16, R, 3, 32)
    return Y, dg, ex


@pytest.mark.parametrize("rows,resid,seg", [(128, False, 0), (128, True, 0), (256, True, 0), (128, True, 2),
                                            (256, False, 2), (128, False, 8), (256, True, 8), (128, False, 16),
                                            (256, True, 16), (128, True, 24), (128, False, 32), (384, True, 32),
                                            (256, True, 48)])
def test_i8f32_out_kernel_writes_the_slice_kernels_digits(rows, resid, seg):
    """The fused output kernel (output transform + BN (+ residual) + ReLU, then the next V's row-line digits in
    one kernel; the product's form, KV_I8F32_OUT) == wino88_out_kernel's fp32 V + wino88i_slice_kernel, bit for
    bit: Y, every digit and every exponent (per row, or per 256-channel segment: seg 2; seg 8: the 64-register
    form wino88i32_out2_kernel; seg 32: the persistent LDS-DMA form wino88i32_outp_kernel, 384 rows = 1.5 boards
    per CU, so workgroups loop over different board counts; seg 16: 3 radix-256 digits). Board 5 is all zero
    after the ReLU (its V rows: exponent 0, digits 0); every 7th channel sits 2^-12 below the others."""
    rng = np.random.default_rng(rows + resid + seg)
    M = (rng.standard_normal((100, rows, 512)) * 0.3).astype(np.float32)
    M[:, 5, :] = 0.0
    scale = (0.5 + rng.random(512)).astype(np.float32)
    scale[::7] *= np.float32(2.0 ** -12)  # channels far below the row max
    scale[256:] *= np.float32(2.0 ** -5)  # the two segments at different scales
    shift = (rng.standard_normal(512) * 0.1).astype(np.float32)
    shift = -np.abs(shift)  # M = 0 (and resid = 0) on board 5: ReLU(shift) = 0
    R = (np.abs(rng.standard_normal((rows, 64, 512))) * 0.5).astype(np.float32) if resid else None
    if resid:
        R[5] = 0.0
    Yf, df, ef = _out(M, scale, shift, R, 1 | seg)
    Ys, ds, es = _out(M, scale, shift, R, seg & 18)  # the slice-kernel form of the same exponents / digits
    assert np.array_equal(Yf.view(np.uint32), Ys.view(np.uint32))
    assert np.array_equal(ef, es)
    assert np.array_equal(df, ds)
    assert (ef[..., 5] == 0).all() and not df[:, :, 5].any()
    assert len(np.unique(ef)) > 3  # exponents actually vary across rows
    if seg & 16:  # 3 radix-256 digits (KV_PATH_WINO88_I8F32R3): 96-byte row lines
        assert df.shape == (100, 16, rows, 3, 32)


@pytest.mark.parametrize("rows,resid", [(128, False), (128, True), (256, True)])
def test_i8f32v_out_kernel_writes_the_fp64_transforms_digits(rows, resid):
    """wino88i32v_out_kernel (KV_ALGO_WINOGRAD88_I8V: output transform + BN (+ residual) + ReLU in fp32, then
    the next V as the fp64 input transform of that activation, cut to 4 row-line digits) == wino88_out_kernel's
    Y + wino88d_in_kernel's fp64 V + wino88i_slice_kernel, bit for bit: Y, every digit, every exponent. Then the
    digits against numpy's fp64 transform of the same Y: each value within half a unit of the 28-bit block
    (2^(e-29)) plus fp64 rounding, each exponent the rule's on numpy's row max."""
    from tests._wino_emul import input_transform_f64
    rng = np.random.default_rng(rows + 11 * resid)
    M = (rng.standard_normal((100, rows, 512)) * 0.3).astype(np.float32)
    M[:, 5, :] = 0.0
    scale = (0.5 + rng.random(512)).astype(np.float32)
    scale[::7] *= np.float32(2.0 ** -12)
    shift = -np.abs(rng.standard_normal(512) * 0.1).astype(np.float32)
    R = (np.abs(rng.standard_normal((rows, 64, 512))) * 0.5).astype(np.float32) if resid else None
    if resid:
        R[5] = 0.0
    Yf, df, ef = _out(M, scale, shift, R, 1 | 4)
    Ys, ds, es = _out(M, scale, shift, R, 4)
    assert np.array_equal(Yf.view(np.uint32), Ys.view(np.uint32))
    assert np.array_equal(ef, es)
    assert np.array_equal(df, ds)
    assert (ef[:, 5] == 0).all() and not df[:, :, 5].any()
    # the fp32 form's digits differ (the fp32 transform rounds): the fp64 transform is what ran
    _, d32, _ = _out(M, scale, shift, R, 1)
    assert not np.array_equal(df, d32)
    V = input_transform_f64(Yf.astype(np.float64))              # [100][rows][512]
    dec = np.zeros_like(V)
    dg = df.astype(np.float64).transpose(0, 2, 1, 4, 3)           # [100][rows][16][32][4]
    for d in range(4):
        dec += dg[..., d].reshape(100, rows, 512) * 2.0 ** (-7 * (d + 1))
    dec = np.ldexp(dec, ef[:, :, None])
    mx = np.abs(V).max(-1)
    e_np = np.where(mx > 0, np.frexp(mx)[1] + (np.frexp(mx)[0] * 2 >= 255 / 128), 0)
    assert np.array_equal(ef, e_np.astype(np.int32))
    tol = np.ldexp(1.0, ef - 29)[:, :, None] + 1e-12 * mx[:, :, None]
    assert (np.abs(dec - V) <= tol).all(), float((np.abs(dec - V) / tol).max())


def _error_bound(V, U, digits, M):
    """Per-element bound of |M - V U^T| for the kernel's arithmetic (V U^T in fp64 from the unsplit
    operands): each operand row is scaled by 2^-e (|a| 2^-e < 1) and cut to `digits` base-128 digits, so
    a 2^-e = sum_i d_i 2^-7(i+1) + rho, |rho| <= rho_max = 2^-(7 digits + 1); the GEMM keeps the digit pairs
    i + j < digits and drops the rest. Hence
        |M - V U^T| <= 2^(ev + eu) [rho_max (sum |a 2^-ev| + sum |b 2^-eu|) + 3 K rho_max^2
                                   + sum_{i + j >= digits} |d_i| . |e_j| 2^-7(i+j+2)]
                       + the one rounding of M (2^-24 |M| in fp32, 2^-53 in fp64)."""
    K = V.shape[-1]
    ev, eu = D.row_exponents(V), D.row_exponents(U)
    dv, du = np.abs(D.split(V, ev, digits).astype(np.float64)), np.abs(D.split(U, eu, digits).astype(np.float64))
    rho = 2.0 ** -(7 * digits + 1)
    an = np.abs(np.ldexp(V, (-ev[..., None]).astype(np.int32))).sum(-1)
    bn = np.abs(np.ldexp(U, (-eu[..., None]).astype(np.int32))).sum(-1)
    b = rho * (an[:, :, None] + bn[:, None, :]) + 3 * K * rho * rho
    for i in range(digits):
        for j in range(digits):
            if i + j >= digits:
                b = b + np.matmul(dv[i], np.swapaxes(du[j], 1, 2)) * 2.0 ** (-7 * (i + j + 2))
    b = np.ldexp(b, (ev[:, :, None] + eu[:, None, :]).astype(np.int32))
    return b + np.abs(M) * (2.0 ** -24 if digits == 4 else 2.0 ** -53)


def _error_bound_r8(V, U, M):
    """_error_bound for KV_PREC_I8R4: a 2^-e = 2^-7 sum_i d_i 2^-8i + rho, |rho| <= 2^-32 (half a unit of the
    31-bit block), the 13 pairs i + j <= 4 of the 4 radix-256 digits kept, the combine's fp64 roundings."""
    K = V.shape[-1]
    ev, eu = D.row_exponents_r8(V), D.row_exponents_r8(U)
    dv, du = np.abs(D.split_r8(V, ev).astype(np.float64)), np.abs(D.split_r8(U, eu).astype(np.float64))
    rho = 2.0 ** -32
    an = np.abs(np.ldexp(V, (-ev[..., None]).astype(np.int32))).sum(-1)
    bn = np.abs(np.ldexp(U, (-eu[..., None]).astype(np.int32))).sum(-1)
    b = rho * (an[:, :, None] + bn[:, None, :]) + K * rho * rho
    for i in range(4):
        for j in range(4):
            if i + j > 4:
                b = b + np.matmul(dv[i], np.swapaxes(du[j], 1, 2)) * 2.0 ** (-14 - 8 * (i + j))
    b = np.ldexp(b, (ev[:, :, None] + eu[:, None, :]).astype(np.int32))
    return b + np.abs(M) * 2.0 ** -51


@pytest.mark.parametrize("digits", [4, 5, "r8"])
def test_i8_gemm_within_derived_bound_of_fp64_product(digits):
    """M of the int8-digit GEMM against an fp64 matmul of the UNSPLIT operands, on adversarial rows:
    channels spread over 2^-30 .. 1 of their row's max (so most values keep far fewer than the block's 28 /
    35 bits), all-equal rows, rows with one large channel, and sign-alternating rows. Every element must be
    within the bound derived from the arithmetic (_error_bound): per-row block fixed point of 7 x digits
    bits, digit pairs i + j < digits, exact int32 levels, one rounding."""
    rng = np.random.default_rng(40 + (6 if digits == "r8" else digits))
    X, R, K = 100, 128, 512
    V = np.where(rng.random((X, R, K)) < 0.5, -1.0, 1.0) * np.exp2(-30.0 * rng.random((X, R, K)))
    V *= np.exp2(rng.integers(-12, 12, size=(X, R, 1)))
    V[:, 0] = 0.75                        # all-equal rows
    V[:, 1] = 1e-9
    V[:, 1, 7] = 3.0                      # one large channel, the rest 2^-31 below it
    V[:, 2] = np.where(np.arange(K) % 2 == 0, 1.0, -1.0) * (1 + 2.0 ** -20)
    U = rng.standard_normal((X, 512, K)) * np.exp2(-10.0 * rng.random((X, 512, K)))
    U[:, 3] = -0.3                        # an all-equal weight row
    if digits == 4:
        V, U = V.astype(np.float32).astype(np.float64), U.astype(np.float32).astype(np.float64)
    M, _, _ = _run(V, U, 4, seg=2) if digits == "r8" else _run(V, U, digits)
    M64 = np.matmul(V, np.swapaxes(U, 1, 2))
    bound = _error_bound_r8(V, U, M) if digits == "r8" else _error_bound(V, U, digits, M)
    err = np.abs(M - M64)
    ratio = err / np.maximum(bound, 1e-300)
    print(f"digits {digits}: max |M - VU^T| / bound = {ratio.max():.3f}, max |err| / |M| (|M| > 0) = "
          f"{(err / np.where(np.abs(M64) > 0, np.abs(M64), np.inf)).max():.2e}")
    assert (err <= bound).all(), float(ratio.max())
