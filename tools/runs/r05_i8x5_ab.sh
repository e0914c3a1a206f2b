#!/bin/bash
# round 5: the trained-weights path (KV_PREC=i8x5) with the in kernel's quad-transposed dword stores and the
# outmax kernel's DPP maxima (this build) against the previous build (knightvision_amd/libkv_head.so):
# forward time, outputs bit for bit, then a kernel trace of this build
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_i8x5_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_PREC=i8x5
: > $O/ab.log
for rep in 1 2; do
    KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 200 python -u tools/ab_forward.py head 2048 256 >> $O/ab.log 2>&1
    KV_I8X5_GEMM=r4 timeout -k 10 200 python -u tools/ab_forward.py newr4 2048 256 >> $O/ab.log 2>&1
    timeout -k 10 200 python -u tools/ab_forward.py new 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for t in ("newr4", "new"):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_head_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{t}_{B}_{k}.npy")
            print(B, t, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/ab_forward.py p 2048 > $O/prof.log 2>&1
echo i8x5-ab-done
