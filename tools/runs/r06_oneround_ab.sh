#!/bin/bash
# round 6: R3 GEMM in one round (256 workgroups, each running its 5 groups of 5 tiles back to back, the copy ring
# across the groups) against one group per workgroup in rounds (KV_R3_ONEROUND=0); R3 bit-exact tests (2,048 rows
# runs the one-round grid), back-to-back GEMM, forward A/B with outputs compared, kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_oneround_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "i8r3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/b2b.log
for rep in 1 2; do
    timeout -k 10 60 python -u tools/gemm_b2b.py oneround >> $O/b2b.log 2>&1
    KV_R3_ONEROUND=0 timeout -k 10 60 python -u tools/gemm_b2b.py rounds >> $O/b2b.log 2>&1
done
: > $O/ab.log
for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/ab_forward.py one 2048 256 >> $O/ab.log 2>&1
    KV_R3_ONEROUND=0 timeout -k 10 200 python -u tools/ab_forward.py rnd 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_rnd_{B}_{k}.npy"); b = np.load(f"/tmp/ab_one_{B}_{k}.npy")
        print("one", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
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
prof one KV_ALGO=auto
prof rnd KV_R3_ONEROUND=0
grep -v amdgpu $O/b2b.log | cut -c1-90
grep -v amdgpu $O/ab.log
head -3 $O/one.txt $O/rnd.txt
