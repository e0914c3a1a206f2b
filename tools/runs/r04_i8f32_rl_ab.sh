#!/bin/bash
# row-line digit layout A/B: the int8-digit GEMM tests, then the fp32 tower on int8 digits with the
# previous build (planes layout, knightvision_amd/libkv_head.so) against this one (row lines), alternating,
# then a kernel trace of each. $1: output directory name
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r04_i8f32_rl}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py -k "i8 or winograd88i8" > $O/tests.log 2>&1
: > $O/ab.log
for rep in 1 2 3; do
    KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 200 python -u tools/ab_forward.py planes 2048 256 128 >> $O/ab.log 2>&1
    timeout -k 10 200 python -u tools/ab_forward.py rowlines 2048 256 128 >> $O/ab.log 2>&1
done
cd /tmp
export TMPDIR=/tmp
KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_planes -o run -- \
    python3 $R/tools/ab_forward.py pp 2048 > $O/prof_planes.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rl -o run -- \
    python3 $R/tools/ab_forward.py pr 2048 > $O/prof_rl.log 2>&1
echo rl-done
