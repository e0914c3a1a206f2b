"""Phase timing of the fp32 tower's output kernel (kv_dev_out_phases: a diagnostic build with shader-clock stamps)
at 2,048 boards: per board, the cycles from the workgroup's start to V ready (M loaded + output and input
transforms), through the row-maxima barrier, the exponent barrier, the digit stores' issue and their drain; the
median / 10th / 90th percentile over boards for waves 0 and 15, the workgroups' start spread and the kernel span.

    python tools/out_phases.py [rows] [resid] [r3]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    resid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    r3 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    from knightvision_amd import _lib
    L = _lib.lib()
    nb = min(rows, 4096)
    st = np.zeros((nb, 2, 6), dtype=np.uint64)
    us = C.c_float()
    _lib.check(L.kv_dev_out_phases(0, rows, resid, r3, st.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(us)),
               "kv_dev_out_phases")
    s = st.astype(np.int64)
    t0 = s[:, :, 0].min()
    names = ["V ready (M + transforms)", "maxima barrier", "exponent barrier", "digit stores issued", "stores drained"]
    out = {"rows": rows, "resid": resid, "r3": r3, "launch_us": us.value, "phases": {}}
    for w, wn in ((0, "wave0"), (1, "wave15")):
        d = np.diff(s[:, w, :], axis=1)
        out["phases"][wn] = {n: [int(np.percentile(d[:, k], q)) for q in (10, 50, 90)] for k, n in enumerate(names)}
        out["phases"][wn]["lifetime"] = [int(np.percentile(s[:, w, 5] - s[:, w, 0], q)) for q in (10, 50, 90)]
    span = int(s[:, :, 5].max() - t0)
    out["kernel_span_cycles"] = span
    out["clock_mhz_implied"] = span / us.value if us.value > 0 else None
    starts = np.sort(s[:, 0, 0] - t0)
    out["start_quantiles_cycles"] = [int(np.percentile(starts, q)) for q in (0, 12.5, 25, 50, 75, 100)]
    out["first_round_start_spread"] = int(starts[min(255, nb - 1)] - starts[0])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
