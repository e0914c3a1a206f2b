#!/bin/bash
# round 5: the trained-weights path (fp64 Winograd domain on int8 digits, KV_PREC=i8x5) at 2,048 and 256 boards:
# forward time and a kernel trace
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_i8x5_prof}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_PREC=i8x5
timeout -k 10 200 python -u tools/ab_forward.py i8x5 2048 256 > $O/ab.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/ab_forward.py p 2048 > $O/prof.log 2>&1
echo i8x5-prof-done
