"""The device Dirichlet's log / pow (csrc/kv_libm.h: glibc 2.35's table-driven
log and pow restated operation for operation, tables from
tools/gen_libm_tables.py) against the libm numpy's legacy gamma calls
(numpy/random/src/legacy/legacy-distributions.c -> log(), pow(); reached from
scripts/self_play.py:153). The restatement is compiled for the host inside
libkv.so (kv_host_libm), so this runs without a GPU; the device build of the
same source is checked end to end by tests/test_engine_gpu.py (Dirichlet
values bit-identical to numpy)."""
import ctypes as C

import numpy as np
import pytest

from knightvision_amd import _lib

libm = C.CDLL("libm.so.6")
libm.log.restype = C.c_double
libm.log.argtypes = [C.c_double]
libm.pow.restype = C.c_double
libm.pow.argtypes = [C.c_double, C.c_double]


def _host(op, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y if y is not None else x, dtype=np.float64)
    out = np.empty_like(x)
    P = C.POINTER(C.c_double)
    _lib.check(_lib.lib().kv_host_libm(op, x.ctypes.data_as(P), y.ctypes.data_as(P), len(x), out.ctypes.data_as(P)),
               "kv_host_libm")
    return out


def _res53(rng, n):
    a = rng.integers(0, 1 << 27, n, dtype=np.int64)
    b = rng.integers(0, 1 << 26, n, dtype=np.int64)
    return (a * 67108864.0 + b) / 9007199254740992.0


def _mismatch(got, want):
    return np.flatnonzero(got.view(np.int64) != want.view(np.int64))


@pytest.mark.parametrize("seed", range(4))
def test_log_bit_identical_to_libm(seed):
    rng = np.random.default_rng(seed)
    u = _res53(rng, 200_000)
    alpha = 0.3
    xs = np.concatenate([
        1.0 - u,                                   # legacy_standard_exponential: -log(1 - res53)
        (1.0 - (0.7 + 0.3 * u)) / alpha,           # -log((1 - U) / shape), U > 1 - shape
        1.0 + (u - 0.5) * 0.2,                     # around the near-1 branch edges
        np.exp(rng.uniform(-700, 700, 50_000)),    # wide normal range
        np.array([1.0, 0.9375, np.nextafter(0.9375, 1), 1.0 + float.fromhex("0x1.09p-4"), np.nextafter(1.0 + float.fromhex("0x1.09p-4"), 0),
                  2.0 ** -53, 1.0 - 2.0 ** -53, 0.5, 2.0, 1e300]),
    ])
    xs = xs[xs > 0]
    want = np.array([libm.log(float(x)) for x in xs])
    got = _host(0, xs)
    bad = _mismatch(got, want)
    assert bad.size == 0, f"{bad.size}/{xs.size} differ, e.g. x={xs[bad[:3]]} got {got[bad[:3]]} want {want[bad[:3]]}"


@pytest.mark.parametrize("seed", range(4))
def test_pow_bit_identical_to_libm(seed):
    rng = np.random.default_rng(100 + seed)
    u = _res53(rng, 200_000)
    alpha = 0.3
    inv = 1.0 / alpha
    y_ = -np.log((1.0 - (0.7 + 0.3 * u)) / alpha)
    xs = np.concatenate([u * 0.7, 0.7 + alpha * y_, np.array([0.0, 1.0, 2.0 ** -53, 0.7, 1e-300 ** 0.1])])
    ys = np.full(xs.size, inv)
    # other legacy shapes (DIR_NOISE_ALPHA is configurable in (0, 1))
    a2 = rng.uniform(0.01, 0.99, 50_000)
    x2 = _res53(rng, 50_000) * (1 - a2)
    xs, ys = np.concatenate([xs, x2]), np.concatenate([ys, 1.0 / a2])
    want = np.array([libm.pow(float(x), float(y)) for x, y in zip(xs, ys)])
    got = _host(1, xs, ys)
    bad = _mismatch(got, want)
    assert bad.size == 0, f"{bad.size}/{xs.size} differ, e.g. x={xs[bad[:3]]} y={ys[bad[:3]]}"


@pytest.mark.parametrize("alpha", [0.05, 0.03, 0.01, 0.003, 0.001])
def test_pow_underflow_bit_identical_to_libm(alpha):
    """Small DIR_NOISE_ALPHA (scripts/self_play.py:13): U^(1/alpha) with U down
    to 2^-53 falls below 2^-1022 (alpha < 53/1022) -- glibc pow's specialcase
    (scaled subnormal result, the re-rounding for |y| < 1, total underflow for
    y log x <= -1024) -- and the second branch's (1 - alpha + alpha Y)^(1/alpha)
    reaches large finite results (the overflow-side specialcase)."""
    rng = np.random.default_rng(int(alpha * 1e6))
    u = _res53(rng, 100_000)
    inv = 1.0 / alpha
    # first branch U <= 1 - alpha, log-uniform down to 2^-53 so that every
    # result range (normal, specialcase subnormal, total underflow) is hit
    lu = np.exp2(rng.uniform(-53, 0, 100_000)) * (1 - alpha)
    # edges of the subnormal range: x with x^(1/alpha) near 2^-1022 and 2^-1074
    edge = np.concatenate([2.0 ** (e * alpha) * (1 + rng.uniform(-1e-3, 1e-3, 5_000)) for e in (-1022, -1050, -1074, -1075)])
    y2 = -np.log((1.0 - (1 - alpha + alpha * u)) / alpha)
    xs = np.concatenate([u * (1 - alpha), lu, edge, 1 - alpha + alpha * y2,
                         np.array([2.0 ** -53, 0.0, 1.0 - alpha, np.nextafter(1.0, 0)])])
    xs = xs[(xs >= 0) & (xs < 2.0 ** 1000)]
    ys = np.full(xs.size, inv)
    want = np.array([libm.pow(float(x), float(y)) for x, y in zip(xs, ys)])
    got = _host(1, xs, ys)
    bad = _mismatch(got, want)
    n_sub = int(np.count_nonzero((want > 0) & (want < 2.2250738585072014e-308)))
    assert n_sub > 100, "the subnormal range was not exercised"
    assert bad.size == 0, f"{bad.size}/{xs.size} differ, e.g. x={xs[bad[:3]]} got {got[bad[:3]]} want {want[bad[:3]]}"


def test_pow_large_y_and_overflow_side_bit_identical_to_libm():
    """pow's |y| >= 2^63 path and exp_inline's k > 0 specialcase (results in
    [2^738, 2^1024)) and total overflow, for positive x and y."""
    rng = np.random.default_rng(7)
    xs = np.concatenate([1 + rng.uniform(0, 1, 20_000), rng.uniform(0, 1, 2_000), np.array([1.0, 0.5, 2.0, 0.0])])
    ys = np.concatenate([rng.uniform(738, 1500, 20_000) / np.log2(xs[:20_000]),
                         np.full(2_000, 2.0 ** 63), np.array([2.0 ** 63, 2.0 ** 64, 2.0 ** 64, 2.0 ** 70])])
    want = np.array([libm.pow(float(x), float(y)) for x, y in zip(xs, ys)])
    got = _host(1, xs, ys)
    bad = _mismatch(got, want)
    assert np.isinf(want).sum() > 100 and ((want > 2.0 ** 738) & np.isfinite(want)).sum() > 100
    assert bad.size == 0, f"{bad.size}/{xs.size} differ, e.g. x={xs[bad[:3]]} y={ys[bad[:3]]}"


def test_numpy_dirichlet_uses_this_libm():
    """The pin above is against the libm numpy's legacy gamma links: replay
    RandomState(42).dirichlet([0.3]*64) with libm log/pow in Python and
    compare with numpy bit for bit."""
    rs = np.random.RandomState(42)
    want = rs.dirichlet([0.3] * 64)
    st = np.random.RandomState(42)

    def gamma():
        while True:
            U = st.random_sample()
            V = -libm.log(1.0 - st.random_sample())
            if U <= 0.7:
                X = libm.pow(U, 1.0 / 0.3)
                if X <= V:
                    return X
            else:
                Y = -libm.log((1 - U) / 0.3)
                X = libm.pow(0.7 + 0.3 * Y, 1.0 / 0.3)
                if X <= V + Y:
                    return X

    g = [gamma() for _ in range(64)]
    acc = 0.0
    for v in g:
        acc = acc + v
    got = np.array(g) * (1 / acc)
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
