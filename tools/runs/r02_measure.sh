#!/bin/bash
# Round-2 measurement pass on the GPU box (run through gpurun from the repo
# root): C3 bench line, rocprofv3 kernel-trace summary at C3, GEMM HBM PMC at
# 2,048 boards, tree-kernel HBM PMC at C3. Every GPU step has its own time
# limit and the first failure ends the script (set -e).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r2m}
mkdir -p $O
cd $R
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
  tail -1 $O/bench.log > $O/bench.json
fi
cd /tmp
export TMPDIR=/tmp
SHORT="--steps 1 --warmup 1 --alt-precision= --ref-block 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o c3 -- python3 $R/bench.py $SHORT > $O/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wino_gemm" -f csv -d $O/pmc_gemm_fetch -o f -- python3 $R/tools/nn_speed.py 2048 > $O/pmc_gemm_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wino_gemm" -f csv -d $O/pmc_gemm_write -o w -- python3 $R/tools/nn_speed.py 2048 > $O/pmc_gemm_write.log 2>&1
# tree-kernel PMC at C3's 2,048 slots with 300 sims/move: rocprofv3 --pmc segfaults in its host
# library on the 800-sim run (tools/runs/r02_tree.sh)
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_mcts" -f csv -d $O/pmc_tree_fetch -o f -- python3 $R/bench.py $SHORT --warmup 0 --sims 300 > $O/pmc_tree_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_mcts" -f csv -d $O/pmc_tree_write -o w -- python3 $R/bench.py $SHORT --warmup 0 --sims 300 > $O/pmc_tree_write.log 2>&1
echo measure-done
