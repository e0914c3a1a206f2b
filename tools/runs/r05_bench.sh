#!/bin/bash
# round 5: the driver's bench command on the current code
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_bench}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1150 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err
echo bench-done
