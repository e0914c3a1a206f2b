#!/bin/bash
# kernel trace of the C3 bench (2 timed moves) on the row-line layout: the GEMM average the bench's HIP
# events must match
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_rl_c3prof
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/c3 -o c3 -- python3 $R/bench.py --steps 2 --warmup 1 --alt-precision= --alt-algo= --ref-block 0 --no-cpu-baseline --trained-steps 0 > $O/c3_bench.log 2> $O/c3_bench.err
echo prof-done
