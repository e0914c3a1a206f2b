#!/bin/bash
# round 5: the trained-weights path (KV_PREC=i8x5) with the in kernel's digits by magic-number fp64 adds and
# 32-bit store offsets, 32-bit offsets in the fp64 output plane (this build) against the previous build (knightvision_amd/libkv_head.so):
# forward time, outputs bit for bit, then a kernel trace of this build
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_i8x5_magic}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_PREC=i8x5
: > $O/ab.log
for rep in 1 2; do
    KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 200 python -u tools/ab_forward.py head 2048 256 >> $O/ab.log 2>&1
    timeout -k 10 200 python -u tools/ab_forward.py new 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for t in ("new",):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_head_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{t}_{B}_{k}.npy")
            print(B, t, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
for rep in 1; do
    KV_PREC=f64w KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 200 python -u tools/ab_forward.py fhead 2048 256 >> $O/ab.log 2>&1
    KV_PREC=f64w timeout -k 10 200 python -u tools/ab_forward.py fnew 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_fhead_{B}_{k}.npy"); b = np.load(f"/tmp/ab_fnew_{B}_{k}.npy")
        print("f64w", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nn_gpu.py \
    tests/test_wino_i8_gpu.py -k "i8 or f64" > $O/tests.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/ab_forward.py p 2048 > $O/prof.log 2>&1
echo i8x5-ab-done
