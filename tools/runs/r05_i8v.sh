#!/bin/bash
# round 5: the fp32 tower with fp64 input transforms (KV_ALGO_WINOGRAD88_I8V): its kernel / forward tests, a
# forward A/B against the fp32-transform tower at 2,048 / 256 boards, the 20-iteration learn loop's path and
# sims/s per iteration, and a kernel trace of its forward
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_i8v}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino_i8_gpu.py tests/test_nn_gpu.py -k "i8f32v or out_kernel or winograd88i8v" \
    -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests-done
: > $O/ab.log
for rep in 1 2; do
    KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py i8f32 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8v timeout -k 10 200 python -u tools/ab_forward.py i8f32v 2048 256 >> $O/ab.log 2>&1
done
echo ab-done
timeout -k 10 420 python -u tools/learn_bench.py --iterations 20 --games 256 --max-moves 80 --sims 64 \
    > $O/learn20_mcts.log 2>&1
echo learn-done
cd /tmp
export TMPDIR=/tmp
KV_ALGO=winograd88i8v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/ab_forward.py pv 2048 > $O/prof.log 2>&1
echo prof-done
