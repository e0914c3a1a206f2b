#!/bin/bash
# Network parity tests, then the C3 bench under rocprofv3 --kernel-trace --stats
# (1 warm-up + 2 timed moves) and the driver's own bench command. Every GPU
# step has its own time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03c3}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -x -v --timeout 120 --timeout-method thread > $O/nn_tests.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o c3 -- python3 $R/bench.py --steps 2 --warmup 1 --alt-precision= --alt-algo= --ref-block 0 --no-cpu-baseline > $O/c3_traced.log 2>&1
cd $R
timeout -k 10 780 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1
echo c3-done
