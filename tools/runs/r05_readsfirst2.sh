#!/bin/bash
# round 5: further sched_barriers in the fp32 tower's GEMMs: (b) also after each B-digit read inside the lagt
# kernel's stage (KV_I8_READS_FIRST2), (c) the reads-first barrier in the one-tile lag kernel (KV_I8_READS_FIRST_LAG,
# timed with KV_I8F32_TPW=1, which runs it); forward A/B against the default build, 3 alternating repeats
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_readsfirst2}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
: > $O/ab.log
for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/ab_forward.py a 2048 256 >> $O/ab.log 2>&1
    KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py b 2048 256 >> $O/ab.log 2>&1
    KV_I8F32_TPW=1 timeout -k 10 200 python -u tools/ab_forward.py a1 2048 256 >> $O/ab.log 2>&1
    KV_I8F32_TPW=1 KV_LIB_PATH=$R/knightvision_amd/libkv_c.so timeout -k 10 200 python -u tools/ab_forward.py c1 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for x, y in (("a", "b"), ("a1", "c1"), ("a", "a1")):
    for B in (2048, 256):
        for k in ("p", "v"):
            p = np.load(f"/tmp/ab_{x}_{B}_{k}.npy"); q = np.load(f"/tmp/ab_{y}_{B}_{k}.npy")
            print(x, y, B, k, "bit-identical" if np.array_equal(p.view(np.uint32), q.view(np.uint32)) else "DIFFER")
PY
echo ab-done
