#!/bin/bash
# round 6: timing probe (outputs invalid): the R3 GEMM writing and its output kernels reading M board-major
# [board][xi][512] (KV_R3_MBM=1: libkv_mbm.so) against the product's point-major [xi][board][512]; forward times and
# kernel traces only
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_mbm_probe}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
V=$R/knightvision_amd/libkv_mbm.so
: > $O/ab.log
for rep in 1 2; do
    KV_ALGO=winograd88i8r3 timeout -k 10 200 python -u tools/ab_forward.py base 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8r3 KV_LIB_PATH=$V timeout -k 10 200 python -u tools/ab_forward.py mbm 2048 256 >> $O/ab.log 2>&1
done
cd /tmp
export TMPDIR=/tmp
prof() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$tag -o run -- \
        python3 $R/tools/ab_forward.py p$tag 2048 > $O/prof_$tag.log 2>&1
    python3 $R/tools/rocpd_stats.py $O/prof_$tag/run_results.db $O/${tag}_kernel_stats.csv > $O/$tag.txt
    rm -rf $O/prof_$tag
}
prof base KV_ALGO=winograd88i8r3
prof mbm KV_ALGO=winograd88i8r3 KV_LIB_PATH=$V
grep -v amdgpu $O/ab.log
head -6 $O/base.txt $O/mbm.txt
