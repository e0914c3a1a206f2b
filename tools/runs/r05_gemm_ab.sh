#!/bin/bash
# round 5: the int8-digit GEMM forms (tools/i8gemm_ab.py), then the fused out kernel A/B (r05_fused_out.sh)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_gemm_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/i8gemm_ab.py 2048 256 > $O/gemm_ab.log 2>&1
bash tools/runs/r05_fused_out.sh ${1:-r05_gemm_ab}/fused
echo gemm-ab-done
