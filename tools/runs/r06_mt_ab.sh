#!/bin/bash
# round 6: the output kernels read M with ordinary loads (KV_OUT_M_NT=0: libkv_mt.so) against the
# product build; forward A/B with outputs compared, kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_mt_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
V=$R/knightvision_amd/libkv_mt.so
: > $O/ab.log
for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/ab_forward.py base 2048 256 >> $O/ab.log 2>&1
    KV_LIB_PATH=$V timeout -k 10 200 python -u tools/ab_forward.py mt 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_base_{B}_{k}.npy"); b = np.load(f"/tmp/ab_mt_{B}_{k}.npy")
        print("mt", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
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
prof base KV_ALGO=auto
prof mt KV_LIB_PATH=$V
grep -v amdgpu $O/ab.log
head -6 $O/base.txt $O/mt.txt
