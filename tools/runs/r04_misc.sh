#!/bin/bash
# round 4 extras: the learn loop's calibrated conv path per iteration (20 iterations x 256 games), the
# trained-weights accuracy table with the int8-digit path, and a 2-rank gloo rehearsal of the bench line
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/learn_bench.py --iterations 20 --games 256 --max-moves 80 \
    > gpurun_out/r04_learn20_paths.log 2>&1
KV_TRAINED_ITERS=20 KV_TRAINED_GAMES=256 KV_TRAINED_MAX_MOVES=80 KV_TRAINED_BOARDS=512 timeout -k 10 400 \
    python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_nn_accuracy_gpu.py -k trained \
    > gpurun_out/r04_trained20_accuracy_i8.log 2>&1
KV_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --slots 256 --sims 50 \
    --alt-precision= --alt-algo= --ref-block 0 --no-cpu-baseline --trained-steps 0 \
    > gpurun_out/r04_bench_gloo2_rehearsal.log 2> gpurun_out/r04_bench_gloo2_rehearsal.err
bash tools/runs/r04_i8out_pmc.sh r04_i8io_pmc
AB_ENVS="KV_I8_PRIO=0 KV_I8_PRIO=1 KV_I8_PRIO=0 KV_I8_PRIO=1" bash tools/runs/r04_i8_ab.sh
