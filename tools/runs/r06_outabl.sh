#!/bin/bash
# round 6: is the output kernel's M-load phase bound by its 50 4-byte loads per lane? KV_OUT_ABL=1 reads the
# same bytes as 13 16-byte loads per lane (values misplaced: timing only); forward times and kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_outabl}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
: > $O/ab.log
for rep in 1 2; do
    KV_ALGO=winograd88i8r3 timeout -k 10 200 python -u tools/ab_forward.py r3 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8r3 KV_OUT_ABL=1 timeout -k 10 200 python -u tools/ab_forward.py r3x4 2048 256 >> $O/ab.log 2>&1
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
prof r3 KV_ALGO=winograd88i8r3
prof r3x4 KV_ALGO=winograd88i8r3 KV_OUT_ABL=1
grep -v amdgpu $O/ab.log
head -5 $O/r3.txt $O/r3x4.txt
