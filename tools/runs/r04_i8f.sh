#!/bin/bash
# GPU checks of the fp32 F(8x8) tower on int8 digits (KV_ALGO_WINOGRAD88_I8): bit-exact GEMM test (4 and
# 5 digits), network tests, accuracy / calibration, forward timing beside the fp32 MFMA tower, a profile
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
T="--timeout 280 --timeout-method thread"
timeout -k 10 300 python -u -m pytest -x -q $T tests/test_wino_i8_gpu.py > gpurun_out/r04_i8f_exact.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v -s $T tests/test_nn_gpu.py -k "i8" > gpurun_out/r04_i8f_nn.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v -s $T tests/test_nn_accuracy_gpu.py -k "not trained" \
    > gpurun_out/r04_i8f_acc.log 2>&1
KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py i8f32 2048 256 128 > gpurun_out/r04_i8f_speed.log 2>&1
KV_ALGO=winograd88 timeout -k 10 200 python -u tools/ab_forward.py fp32_w88 2048 256 128 >> gpurun_out/r04_i8f_speed.log 2>&1
cd /tmp && export TMPDIR=/tmp KV_ALGO=winograd88i8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04_i8f_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/ab_forward.py" i8fprof 2048 > "$GRAFT_REPO_ROOT/gpurun_out/r04_i8f_prof.log" 2>&1
