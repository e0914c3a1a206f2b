"""A/B of the fp32 tower's int8-digit GEMM forms (kv_dev_i8gemm_bench, seeded random digits): every
variant's M bit for bit against variant 0 (the round-4 kernel), then interleaved timing rounds in one
process (HIP events, mean of `iters` launches per round).

    python tools/i8gemm_ab.py [rows ...]   (default 2048 256)
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd import _lib  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("I8_VARIANTS", "0,14,16,17").split(",")]
SAME_M = {1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19}  # 6: segment exponents (another M); 7-9: timing ablations (no stores / no copies)
L = _lib.lib()
rows_list = [int(a) for a in sys.argv[1:]] or [2048, 256]
for K in (512,):
    for rows in rows_list:
        us = C.c_float()
        ref = np.zeros((100, rows, 512), dtype=np.float32)
        _lib.check(L.kv_dev_i8gemm_bench(0, rows, K, 0, 1, C.byref(us), ref.ctypes.data_as(C.POINTER(C.c_float))), "bench")
        for v in [v for v in VARIANTS if v in SAME_M]:
            m = np.zeros_like(ref)
            _lib.check(L.kv_dev_i8gemm_bench(0, rows, K, v, 1, C.byref(us), m.ctypes.data_as(C.POINTER(C.c_float))), "bench")
            same = np.array_equal(m.view(np.uint32), ref.view(np.uint32))
            print(f"K={K} rows={rows} variant {v}: M {'bit-identical' if same else 'DIFFERS'} to variant 0", flush=True)
        iters = 50 if rows >= 1024 else 200
        res = {v: [] for v in VARIANTS}
        for rnd in range(4):
            for v in VARIANTS:
                _lib.check(L.kv_dev_i8gemm_bench(0, rows, K, v, iters, C.byref(us), None), "bench")
                res[v].append(us.value)
        ops = 10 * 2.0 * rows * 512 * K * 100
        for v in VARIANTS:
            t = sorted(res[v])
            print(f"K={K} rows={rows} variant {v}: median {t[len(t)//2]:.1f} us  min {t[0]:.1f}  "
                  f"= {ops / t[0] / 1e6:.0f} int8 TOPS at min", flush=True)
