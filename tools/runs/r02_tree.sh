#!/bin/bash
# Tree-kernel HBM bytes per simulation at C3's 2,048 slots (300 sims/move:
# rocprofv3 --pmc segfaults in its host library on the 800-sim run): one
# kernel-trace pass for durations, separate FETCH_SIZE / WRITE_SIZE passes.
# Run through gpurun from the repo root; the first failure ends it.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tree}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --sims 300 --alt-precision= --ref-block 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t -- python3 $R/bench.py $ARGS > $O/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_mcts" -f csv -d $O/pmc_fetch -o f -- python3 $R/bench.py $ARGS > $O/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_mcts" -f csv -d $O/pmc_write -o w -- python3 $R/bench.py $ARGS > $O/pmc_write.log 2>&1
echo tree-done
