#!/bin/bash
# round 6: the fp64 domain's GEMM (wino88i_gemm_lag5_kernel: the trained-weights path, KV_PREC=i8r4; and the
# 5-digit form, KV_PREC=i8x5) storing its fp64 M non-temporally (KV_LAG5_M_NT=1: libkv_l5nt.so) against the product
# build; forward A/B with outputs compared, kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_l5nt_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
V=$R/knightvision_amd/libkv_l5nt.so
: > $O/ab.log
for rep in 1 2 3; do
    KV_PREC=i8r4 timeout -k 10 200 python -u tools/ab_forward.py base 2048 256 >> $O/ab.log 2>&1
    KV_PREC=i8r4 KV_LIB_PATH=$V timeout -k 10 200 python -u tools/ab_forward.py l5nt 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_base_{B}_{k}.npy"); b = np.load(f"/tmp/ab_l5nt_{B}_{k}.npy")
        print("l5nt", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
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
prof base KV_PREC=i8r4
prof l5nt KV_PREC=i8r4 KV_LIB_PATH=$V
grep -v amdgpu $O/ab.log
head -5 $O/base.txt $O/l5nt.txt
