#!/bin/bash
# round 5: the fp32 output kernels with all 50 M loads of a lane issued before the first transform (KV_OUT_LOADS_FIRST,
# libkv_b.so) against the default; forward A/B on the headline tower, 3 alternating repeats, outputs bit for bit
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_loadsfirst}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
: > $O/ab.log
for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/ab_forward.py a 2048 256 >> $O/ab.log 2>&1
    KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py b 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for y in ("b",):
    for B in (2048, 256):
        for k in ("p", "v"):
            p = np.load(f"/tmp/ab_a_{B}_{k}.npy"); q = np.load(f"/tmp/ab_{y}_{B}_{k}.npy")
            print("a", y, B, k, "bit-identical" if np.array_equal(p.view(np.uint32), q.view(np.uint32)) else "DIFFER")
PY
echo ab-done
