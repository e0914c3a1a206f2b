"""The int8-digit split of KV_PREC_I8X5 (csrc/kv_wino88i.h), restated in numpy
(tests/_i8_digits.py): its arithmetic claims, checked on the host. The GPU
kernels are compared with this restatement bit for bit in test_wino_i8_gpu.py."""
import numpy as np

from tests import _i8_digits as D


def _rows(rng, n, K):
    a = rng.standard_normal((n, K)) * np.exp2(rng.integers(-30, 30, size=(n, 1)))
    a[0] = 0.0                                   # an all-zero row
    a[1] = np.nextafter(np.exp2(5.0), 0.0)       # max just below 2^5: the exponent steps up (no clamp needed)
    a[2, ::2] = -a[2, ::2]
    a[3] = 5e-320                                # subnormals
    a[4, :] = 0.0
    a[4, 7] = -1.0                               # one exact power of two
    return a


def test_digits_reconstruct_to_2_pow_minus_35_of_row_max():
    rng = np.random.default_rng(1)
    for K in (256, 512):
        a = _rows(rng, 64, K)
        e = D.row_exponents(a)
        d = D.split(a, e)
        di = d.astype(int)
        assert d.dtype == np.int8 and np.abs(di[0]).max() <= 127 and np.abs(di[1:]).max() <= 64  # no clamp needed
        rec = sum(d[i].astype(np.float64) * 2.0 ** (-7 * (i + 1)) for i in range(D.DIGITS))
        err = np.abs(np.ldexp(rec, e[:, None].astype(np.int32)) - a)
        bound = np.ldexp(np.ones_like(e, dtype=np.float64), (e - 36).astype(np.int32))
        assert (err <= bound[:, None]).all()
        nz = np.abs(a).max(axis=1) > 1e-300  # max |row| < 255/256 2^e, and >= 2^(e-2) (rows of tiny subnormals: e = 0)
        mx = np.abs(a).max(axis=1)[nz]
        assert (mx < np.exp2(e[nz].astype(float)) * 255 / 256).all() and (mx >= np.exp2(e[nz] - 2.0)).all()
        assert (e[1] == 6)  # row 1: max = 2^5 - ulp, top fraction bits all ones -> bumped from 5 to 6


def test_level_sums_fit_int32_and_combine_exactly():
    # worst case (bound of any digit 127), K = 512: level l sums (l + 1) products of 512 terms
    worst = max((l + 1) * 512 * 127 * 127 for l in range(D.LEVELS))
    assert worst < 2 ** 31
    # combining the five levels spans <= 23 + 28 bits: exact in fp64
    rng = np.random.default_rng(2)
    lev = [rng.integers(-worst, worst, size=1000).astype(np.float64) for _ in range(D.LEVELS)]
    m = lev[-1]
    for l in range(D.LEVELS - 2, -1, -1):
        m = m * 0.0078125 + lev[l]
    exact = sum(int(x) * 2 ** (7 * (D.LEVELS - 1 - l)) for l, x in enumerate(np.array(lev)[:, 0]))
    assert m[0] * 2 ** (7 * (D.LEVELS - 1)) == exact


def test_gemm_matches_fp64_to_the_truncation():
    rng = np.random.default_rng(3)
    V = rng.standard_normal((3, 32, 512))
    U = rng.standard_normal((3, 64, 512)) * 0.01
    M, _, _ = D.gemm(V, U)
    ref = np.matmul(V, np.swapaxes(U, 1, 2))
    scale = np.abs(V).max(axis=2)[:, :, None] * np.abs(U).max(axis=2)[:, None, :] * 512
    assert (np.abs(M - ref) <= scale * 2.0 ** -33).all()


def test_f88_input_transform_restatement_matches_the_kernel_constants():
    """tests/_wino_emul.bt88 (B10^T derived exactly from the points) == the coefficients of
    csrc/kv_wino88d.h's w88d_bt fma chains, entry for entry -- the GPU test of wino88i32v_out_kernel checks its
    digits against numpy's fp64 transform with this matrix."""
    import os
    import re
    from tests._wino_emul import bt88
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "knightvision_amd", "csrc", "kv_wino88d.h")).read()
    body = src[src.index("void w88d_bt"):]
    body = body[:body.index("\n}")]
    M = np.zeros((10, 10))
    rows = re.findall(r"o\[(\d)\] = (.*);", body)
    assert len(rows) == 10
    for a, expr in rows:
        for c, i in re.findall(r"(-?[\d.]+(?:e-?\d+)?),? ?\*? ?d\[(\d)\]", expr):
            M[int(a), int(i)] = float(c)
    assert np.array_equal(M, bt88())
