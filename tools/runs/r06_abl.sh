#!/bin/bash
# round 6: what bounds R3's 64-k-stage GEMM: back-to-back launch time of the full kernel and of timing ablations
# (KV_R3K64_ABL 1 no copies after the prologue, 2 no MFMAs, 3 neither, 4 no M stores, 7 none of the three),
# against the 32-k lagt kernel; two rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_abl}
mkdir -p $O
export PYTHONUNBUFFERED=1
: > $O/abl.log
for rep in 1 2; do
    timeout -k 10 60 python -u tools/gemm_b2b.py lagt32 >> $O/abl.log 2>&1
    for a in 0 1 2 3 4 7; do
        KV_I8R3_K64=1 KV_R3K64_ABL=$a timeout -k 10 60 python -u tools/gemm_b2b.py k64abl$a >> $O/abl.log 2>&1
    done
done
grep -v amdgpu $O/abl.log
