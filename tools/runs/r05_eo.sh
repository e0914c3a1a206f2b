#!/bin/bash
# round 5: fp64 transforms in even / odd form (w88d_bt / w88d_at, tools/gen_wino88.py): the kernel tests that
# pin the fp64 transforms, then forward A/B against the previous build (knightvision_amd/libkv_b.so) on the fp64
# domain (KV_PREC=i8x5), the fp64-input-transform tower (winograd88i8v) and f64w, 2 alternating repeats each
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_eo}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_wino_i8_gpu.py tests/test_nn_gpu.py -k "i8f32v or out_kernel or winograd88i8v or i8x5 or f64w" \
    -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests-done
: > $O/ab.log
for rep in 1 2; do
    for mode in "KV_PREC=i8x5" "KV_ALGO=winograd88i8v" "KV_PREC=f64w"; do
        t=$(echo $mode | tr -d '=' | tr 'A-Z' 'a-z')
        env $mode KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py old_$t 2048 256 >> $O/ab.log 2>&1
        env $mode timeout -k 10 200 python -u tools/ab_forward.py new_$t 2048 256 >> $O/ab.log 2>&1
    done
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for t in ("kv_preci8x5", "kv_algowinograd88i8v", "kv_precf64w"):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_old_{t}_{B}_{k}.npy"); b = np.load(f"/tmp/ab_new_{t}_{B}_{k}.npy")
            print(t, B, k, "max |new - old|", float(np.abs(a - b).max()))
PY
echo ab-done
cd /tmp
export TMPDIR=/tmp
KV_PREC=i8x5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_i8x5 -o run -- python3 $R/tools/ab_forward.py pi 2048 > $O/prof_i8x5.log 2>&1
KV_ALGO=winograd88i8v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_v -o run -- python3 $R/tools/ab_forward.py pv 2048 > $O/prof_v.log 2>&1
echo prof-done
