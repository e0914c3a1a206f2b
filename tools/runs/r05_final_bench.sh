#!/bin/bash
# round 5: the learn loop's path / sims-per-second per iteration, then the driver's bench command and the C2 line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_final}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u tools/learn_bench.py --iterations 20 --games 256 --max-moves 80 --sims 64 \
    > $O/learn20_mcts.log 2>&1
echo learn-done
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err
echo bench-done
timeout -k 10 200 python -u bench.py --slots 256 --sims 400 --steps 5 --warmup 2 > $O/bench_c2.log 2> $O/bench_c2.err
echo c2-done
