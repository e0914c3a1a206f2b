#!/bin/bash
# round 6: the bench line with the driver's round-5 step counts (--steps 20 --warmup 5: plies 6-25)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_bench20}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err
tail -1 $O/bench.log | cut -c1-400
