#!/bin/bash
# 3- vs 4-buffer LDS ring of the int8 GEMMs: bit-exact test with each, forward timing of both towers
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
KV_I8_NBUF=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_i8_gpu.py \
    > gpurun_out/r04_i8_nbuf_exact.log 2>&1
: > gpurun_out/r04_i8_nbuf_ab.log
for n in 3 4 3 4; do
    KV_I8_NBUF=$n KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py "f32_nbuf$n" 2048 256 >> gpurun_out/r04_i8_nbuf_ab.log 2>&1
    KV_I8_NBUF=$n KV_PREC=i8x5 timeout -k 10 200 python -u tools/ab_forward.py "f64_nbuf$n" 2048 256 >> gpurun_out/r04_i8_nbuf_ab.log 2>&1
done
