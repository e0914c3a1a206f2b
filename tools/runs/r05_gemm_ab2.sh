#!/bin/bash
# round 5: int8-digit GEMM forms A/B (tools/i8gemm_ab.py); the library layout under rocprofv3 --pmc for the
# round-3 SIGSEGV attribution (tools/runs/r05_maps.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_gemm_ab2}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/i8gemm_ab.py 2048 256 > $O/gemm_ab.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES -d $O/maps_prof -o m -- python3 $R/tools/runs/r05_maps.py $O/maps.txt > $O/maps.log 2>&1
echo gemm-ab-done
