#!/bin/bash
# Tree-kernel HBM bytes per simulation at C3 itself (2,048 slots x 800 sims/move), measured directly:
# a kernel-trace pass for durations, then separate FETCH_SIZE / WRITE_SIZE passes over
# k_mcts_backup_select's 799 launches of one move (the profiler run that segfaulted in round 3,
# profiles/r03_pmc_tree_crash_stack.log, completes in round 4 at the default kernel-argument placement).
# Every pass runs bench.py through tools/crash_diag.py, whose SIGSEGV handler would name the faulting
# library (frames + mappings) if the crash came back. The last pass repeats the FETCH pass with round 3's
# HIP_FORCE_DEV_KERNARG=0 (kernel arguments in host memory). Run through gpurun from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tree}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --sims 800 --alt-precision= --alt-algo= --f64w-steps 0 --ref-block 0 --no-cpu-baseline"
D="python3 $R/tools/crash_diag.py $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t -- $D > $O/trace.log 2>&1
echo trace-done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "[1-799]" -f csv -d $O/pmc_fetch -o f -- $D > $O/pmc_fetch.log 2>&1
echo fetch-done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "[1-799]" -f csv -d $O/pmc_write -o w -- $D > $O/pmc_write.log 2>&1
echo write-done
HIP_FORCE_DEV_KERNARG=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_mcts_backup_select" --kernel-iteration-range "[1-799]" -f csv -d $O/pmc_fetch_hostkernarg -o f -- $D > $O/pmc_fetch_hostkernarg.log 2>&1
echo tree-done
