#!/bin/bash
# round 6: non-temporal Y / residual (YNT, 1,024+ boards) in the other output kernels -- the 4-digit tower's, the
# fp64-input-transform tower's (winograd88i8v) and the fp64 domain's (KV_PREC=i8r4: the trained-weights path) --
# against the previous commit (libkv_old.so); forward A/B with outputs compared
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_ynt2_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
OLD=$R/knightvision_amd/libkv_old.so
: > $O/ab.log
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u tools/ab_forward.py $tag 2048 256 >> $O/ab.log 2>&1
}
for rep in 1 2; do
    run i8 KV_ALGO=winograd88i8
    run i8o KV_ALGO=winograd88i8 KV_LIB_PATH=$OLD
    run i8v KV_ALGO=winograd88i8v
    run i8vo KV_ALGO=winograd88i8v KV_LIB_PATH=$OLD
    run i8r KV_PREC=i8r4
    run i8ro KV_PREC=i8r4 KV_LIB_PATH=$OLD
    run r3 KV_ALGO=auto
    run r3o KV_ALGO=auto KV_LIB_PATH=$OLD
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for a_, b_ in (("i8o", "i8"), ("i8vo", "i8v"), ("i8ro", "i8r"), ("r3o", "r3")):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_{a_}_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{b_}_{B}_{k}.npy")
            print(b_, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
PY
grep -v amdgpu $O/ab.log
