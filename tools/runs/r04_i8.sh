#!/bin/bash
# GPU checks of KV_PREC_I8X5 (the fp64 Winograd domain on int8 digits): bit-exact kernel test, network
# parity / accuracy tests (and the f64w ones, whose kernels share code), forward timing beside KV_PREC_F64W,
# a kernel-trace profile.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
T="--timeout 280 --timeout-method thread"
timeout -k 10 300 python -u -m pytest -x -q $T tests/test_wino_i8_gpu.py > gpurun_out/r04_i8_exact.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v -s $T tests/test_nn_gpu.py -k "i8 or f64w" > gpurun_out/r04_i8_nn.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v -s $T tests/test_nn_accuracy_gpu.py -k "stress or calibration" \
    > gpurun_out/r04_i8_acc.log 2>&1
KV_PREC=i8x5 timeout -k 10 200 python -u tools/ab_forward.py i8 2048 256 128 > gpurun_out/r04_i8_speed.log 2>&1
KV_PREC=f64w timeout -k 10 200 python -u tools/ab_forward.py f64w 2048 256 128 >> gpurun_out/r04_i8_speed.log 2>&1
cd /tmp && export TMPDIR=/tmp KV_PREC=i8x5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04_i8_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/ab_forward.py" i8prof 2048 > "$GRAFT_REPO_ROOT/gpurun_out/r04_i8_prof.log" 2>&1
