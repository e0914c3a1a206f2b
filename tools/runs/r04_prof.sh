#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of the forward: F(8x8) fp32 at 256 boards under the
# GEMM schedules KV_W88_SPLIT=1 / 2, and the fp64 Winograd domain (KV_PREC=f64w) at 2,048 / 256 boards.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp
export TMPDIR=/tmp KV_CALIBRATE=0
for m in 1 2; do
  KV_W88_SPLIT=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/w88_256_m$m -o t -- python3 $R/tools/nn_speed.py 256 > $O/w88_256_m$m.log 2>&1
done
KV_PREC=f64w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/f64w_2048 -o t -- python3 $R/tools/nn_speed.py 2048 > $O/f64w_2048.log 2>&1
KV_PREC=f64w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/f64w_256 -o t -- python3 $R/tools/nn_speed.py 256 > $O/f64w_256.log 2>&1
echo prof-done
