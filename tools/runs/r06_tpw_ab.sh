#!/bin/bash
# round 6: tiles per workgroup for R3's 64-k GEMM: the rule's choice (5 at 2,048 rows, 4 at 256) against single
# tiles (KV_I8F32_TPW=1), back to back, two rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_tpw_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
: > $O/b2b.log
for rep in 1 2; do
    for rows in 2048 256; do
        timeout -k 10 60 python -u tools/gemm_b2b.py rule $rows >> $O/b2b.log 2>&1
        KV_I8F32_TPW=1 timeout -k 10 60 python -u tools/gemm_b2b.py tpw1 $rows >> $O/b2b.log 2>&1
    done
done
grep -v amdgpu $O/b2b.log
