#!/bin/bash
# round 6: the lagt GEMM with its lagging operands made opaque after the pre-barrier lgkmcnt(0) (the compiler then
# issues the lagging MFMAs under the new stage's LDS reads instead of waiting for all of them; KV_LAG_OPAQUE=0:
# libkv_noopq.so) and the R3 lag depth (KV_I8R3_LJ 1 vs 2: libkv_lj2.so); bit-exact GEMM tests; forward A/B with
# outputs compared; kernel traces; then the output kernel's phase timing (tools/out_phases.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_gemm_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "gemm_bit_exact or derived_bound" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab.log
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u tools/ab_forward.py $tag 2048 256 >> $O/ab.log 2>&1
}
for rep in 1 2; do
    run r3 KV_ALGO=winograd88i8r3
    run r3noopq KV_ALGO=winograd88i8r3 KV_LIB_PATH=$R/knightvision_amd/libkv_noopq.so
    run r3lj2 KV_ALGO=winograd88i8r3 KV_LIB_PATH=$R/knightvision_amd/libkv_lj2.so
    run i8 KV_ALGO=winograd88i8
    run i8noopq KV_ALGO=winograd88i8 KV_LIB_PATH=$R/knightvision_amd/libkv_noopq.so
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for a_, b_ in (("r3", "r3noopq"), ("r3", "r3lj2"), ("i8", "i8noopq")):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_{a_}_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{b_}_{B}_{k}.npy")
            print(b_, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
PY
cd /tmp
export TMPDIR=/tmp
prof() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$tag -o run -- \
        python3 $R/tools/ab_forward.py p$tag 2048 > $O/prof_$tag.log 2>&1
    python3 $R/tools/rocpd_stats.py $O/prof_$tag/run_results.db $O/${tag}_kernel_stats.csv > $O/$tag.txt
    rm -rf $O/prof_$tag
}
prof r3 KV_ALGO=winograd88i8r3
prof i8 KV_ALGO=winograd88i8
cd $R
for a in "0 0" "1 0" "0 1"; do
    timeout -k 10 120 python -u tools/out_phases.py 2048 $a > $O/phases_$(echo $a | tr ' ' _).json 2>&1
done
echo gemm-ab-done
