#!/bin/bash
# Tree-kernel HBM bytes per simulation at C3 itself (2,048 slots x 800 sims/move):
# one kernel-trace pass for durations, then separate FETCH_SIZE / WRITE_SIZE
# passes restricted to k_mcts_backup_select (the kernel `tree_hbm` reports)
# and to its launches of one move (--kernel-iteration-range), so the counter
# collection covers the whole 800-sim move and nothing else. r02's --pmc runs
# over every k_mcts kernel of an 800-sim move segfaulted in the profiler's host
# library; each pass here has its own log and time limit, and the first
# failure ends the script. Run through gpurun from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tree}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --sims 800 --alt-precision= --ref-block 0 --no-cpu-baseline"
RANGE="[1-799]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t -- python3 $R/bench.py $ARGS > $O/trace.log 2>&1
echo trace-done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "$RANGE" -f csv -d $O/pmc_fetch -o f -- python3 $R/bench.py $ARGS > $O/pmc_fetch.log 2>&1
echo fetch-done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "$RANGE" -f csv -d $O/pmc_write -o w -- python3 $R/bench.py $ARGS > $O/pmc_write.log 2>&1
echo tree-done
