#!/bin/bash
# round 5: the learn loop (20 iterations x 256 games, MCTS 64 sims) -- the calibrated conv path and rank 0's
# self-play sims/s per iteration -- then the trained-weights accuracy table on the loop's weights
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/learn_bench.py --iterations 20 --games 256 --max-moves 80 --sims 64 \
    > gpurun_out/r05_learn20_mcts_paths.log 2>&1
echo learn-done
