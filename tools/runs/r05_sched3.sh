#!/bin/bash
# round 5: (b) a sched_barrier after the lagt stage's first copies (KV_I8_COPY_BARRIER) on the headline tower; (c) the
# per-B-digit reads-first barrier in the 13-pair fp64-domain GEMM (KV_I8R_READS_FIRST2) on i8r4; forward A/B against the
# default build, 3 alternating repeats, outputs bit for bit
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_sched3}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
: > $O/ab.log
for rep in 1 2 3; do
    KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py a 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8 KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py b 2048 256 >> $O/ab.log 2>&1
    KV_PREC=i8r4 timeout -k 10 200 python -u tools/ab_forward.py ar 2048 256 >> $O/ab.log 2>&1
    KV_PREC=i8r4 KV_LIB_PATH=$R/knightvision_amd/libkv_c.so timeout -k 10 200 python -u tools/ab_forward.py cr 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for x, y in (("a", "b"), ("ar", "cr")):
    for B in (2048, 256):
        for k in ("p", "v"):
            p = np.load(f"/tmp/ab_{x}_{B}_{k}.npy"); q = np.load(f"/tmp/ab_{y}_{B}_{k}.npy")
            print(x, y, B, k, "bit-identical" if np.array_equal(p.view(np.uint32), q.view(np.uint32)) else "DIFFER")
PY
echo ab-done
