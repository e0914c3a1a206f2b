#!/bin/bash
# round-4 final: the learn loop's calibrated conv path per iteration and the trained-weights accuracy table
# (20 iterations x 256 games) with every conv path, on the final code
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/learn_bench.py --iterations 20 --games 256 --max-moves 80 \
    > gpurun_out/r04_learn20_nn_paths_final.log 2>&1
KV_TRAINED_ITERS=20 KV_TRAINED_GAMES=256 KV_TRAINED_MAX_MOVES=80 KV_TRAINED_BOARDS=512 timeout -k 10 400 \
    python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_nn_accuracy_gpu.py -k trained \
    > gpurun_out/r04_trained20_accuracy_final.log 2>&1
