#!/bin/bash
# round 5: a sched_barrier after each stage's LDS reads in the lagt / lag5 GEMMs (KV_I8_READS_FIRST, libkv_b.so) so
# the reads issue before the lagging MFMAs (the compiler hoists those MFMAs above the reads): forward A/B on the
# headline tower (winograd88i8) and the radix-256 fp64 domain (i8r4), 3 alternating repeats, outputs bit for bit
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_readsfirst}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
: > $O/ab.log
for rep in 1 2 3; do
    for m in "KV_ALGO=winograd88i8" "KV_PREC=i8r4"; do
        t=$(echo $m | cut -d= -f2)
        env $m timeout -k 10 200 python -u tools/ab_forward.py a_$t 2048 256 >> $O/ab.log 2>&1
        env $m KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py b_$t 2048 256 >> $O/ab.log 2>&1
    done
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for t in ("winograd88i8", "i8r4"):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_a_{t}_{B}_{k}.npy"); b = np.load(f"/tmp/ab_b_{t}_{B}_{k}.npy")
            print(t, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else "DIFFER")
PY
echo ab-done
