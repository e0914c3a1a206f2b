"""KV_PREC_I8X5's slice and GEMM kernels (csrc/kv_wino88i.h) through
kv_dev_wino88i, bit for bit against the numpy restatement (tests/_i8_digits.py):
the digits and row exponents of V, and M -- the exact dot products of the
digit-truncated rows, so any lane-mapping or accumulation slip shows as a
differing bit. 4 digits (the fp32 domain) use the row-line layout
[xi][K/32][row][4][32]; 5 digits the planes [xi][K/32][5][row][32]."""
import ctypes as C

import numpy as np
import pytest

from tests import _i8_digits as D

pytestmark = pytest.mark.gpu


def _run(V, U, digits=D.DIGITS):
    from knightvision_amd import _lib
    L = _lib.lib()
    X, R, K = V.shape
    M = np.zeros((X, R, 512))
    dg = np.zeros((X, K // 32, digits, R, 32), dtype=np.int8)
    ex = np.zeros((X, R), dtype=np.int32)
    P = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    _lib.check(L.kv_dev_wino88i(0, P(np.ascontiguousarray(V), C.c_double), R, P(np.ascontiguousarray(U), C.c_double),
                                K, digits, P(M, C.c_double), P(dg, C.c_int8), P(ex, C.c_int32)), "kv_dev_wino88i")
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
