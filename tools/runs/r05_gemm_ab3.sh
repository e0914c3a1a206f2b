#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_gemm_ab3}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/i8gemm_ab.py 2048 256 > $O/gemm_ab.log 2>&1
echo gemm-ab3-done
