#!/bin/bash
# Tree-kernel HBM bytes per simulation at C3 itself (2,048 slots x 800 sims/move):
# one kernel-trace pass for durations, then separate FETCH_SIZE / WRITE_SIZE
# passes restricted to k_mcts_backup_select (the kernel `tree_hbm` reports)
# and to its launches of one move (--kernel-iteration-range), so the counter
# collection covers the whole 800-sim move and nothing else. r02's --pmc runs
# over every k_mcts kernel of an 800-sim move segfaulted in the profiler's host
# library. r03's first run of this script reproduced it with the narrow
# filter: SIGSEGV inside the launch of k_mcts_backup_select (kv_run ->
# kv::mcts_backup_select -> HIP launch -> profiler interception -> a copy that
# faults at a page-aligned address, 0x735a7bd00000, in the device-memory range,
# not in the kernel -- profiles/r03_pmc_tree_crash_stack.log). HIP places
# kernel arguments in device memory on this GPU by default
# (HIP_FORCE_DEV_KERNARG) and this kernel's arguments (DevCfg + Tree by value,
# ~300 B) are the largest of the run, so the PMC passes below put them in host
# memory (HIP_FORCE_DEV_KERNARG=0) -- the kernel's own HBM traffic, which the
# counters measure, is unchanged. Each pass has its own log and time limit;
# the first failure ends the script. Run through gpurun from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tree}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --sims 800 --alt-precision= --ref-block 0 --no-cpu-baseline ${EXTRA_ARGS:-}"
RANGE="${RANGE:-[1-799]}"
if [ "${SKIP_TRACE:-0}" != 1 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t -- python3 $R/bench.py $ARGS > $O/trace.log 2>&1
echo trace-done
fi
export HIP_FORCE_DEV_KERNARG=0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "$RANGE" -f csv -d $O/pmc_fetch -o f -- python3 $R/bench.py $ARGS > $O/pmc_fetch.log 2>&1
echo fetch-done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "$RANGE" -f csv -d $O/pmc_write -o w -- python3 $R/bench.py $ARGS > $O/pmc_write.log 2>&1
echo tree-done
