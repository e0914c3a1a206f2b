#!/bin/bash
# round 6, final R3 GEMM (96-byte lines, non-temporal M): back-to-back time of the full kernel and its timing
# ablations (KV_R3K64_ABL 1 no copies, 2 no MFMAs, 4 no M stores, 8 no exponent loads in the epilogue); two rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_abl2}
mkdir -p $O
export PYTHONUNBUFFERED=1
: > $O/abl.log
for rep in 1 2; do
    for a in 0 1 2 4 8; do
        KV_R3K64_ABL=$a timeout -k 10 60 python -u tools/gemm_b2b.py abl$a >> $O/abl.log 2>&1
    done
done
grep -v amdgpu $O/abl.log
