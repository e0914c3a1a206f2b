#!/bin/bash
# round 6: R3's GEMM with 64-k stages and 96-byte row copies (KV_I8R3_K64=1: wino88i32_gemm_r3k64_kernel) against
# the 32-k lagt kernel: the R3 bit-exact GEMM tests under the new kernel, forward A/B with outputs compared,
# kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_k64_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "i8r3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab.log
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u tools/ab_forward.py $tag 2048 256 >> $O/ab.log 2>&1
}
for rep in 1 2 3; do
    run r3 KV_ALGO=winograd88i8r3
    run r3k64 KV_ALGO=winograd88i8r3 KV_I8R3_K64=1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for a_, b_ in (("r3", "r3k64"),):
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
        python3 $R/tools/ab_forward.py p$tag 2048 256 > $O/prof_$tag.log 2>&1
    python3 $R/tools/rocpd_stats.py $O/prof_$tag/run_results.db $O/${tag}_kernel_stats.csv > $O/$tag.txt
    rm -rf $O/prof_$tag
}
prof r3 KV_ALGO=winograd88i8r3
prof r3k64 KV_ALGO=winograd88i8r3 KV_I8R3_K64=1
echo k64-ab-done
