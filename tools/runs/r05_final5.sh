#!/bin/bash
# round 5, final code: the whole -m gpu suite, smoke(), the driver's bench command, the 20-iteration learn loop
# (path, calibration and sims/s per iteration) and the C2 line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_final5}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
echo suite-done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke-done
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err
echo bench-done
timeout -k 10 420 python -u tools/learn_bench.py --iterations 20 --games 256 --max-moves 80 --sims 64 \
    > $O/learn20_mcts.log 2>&1
echo learn-done
