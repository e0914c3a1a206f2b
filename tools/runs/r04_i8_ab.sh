#!/bin/bash
# A/B of KV_PREC_I8X5 GEMM forms: bit-exact kernel test, then forward timing per setting of $AB_ENVS
# (space-separated VAR=VALUE, one forward timing each), then a kernel-trace profile of the default
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_i8_gpu.py \
    > gpurun_out/r04_i8_exact.log 2>&1
: > gpurun_out/r04_i8_ab.log
for e in $AB_ENVS; do
    env $e KV_PREC=${AB_PREC:-i8x5} KV_ALGO=${AB_ALGO:-auto} timeout -k 10 200 python -u tools/ab_forward.py "$e" 2048 256 128 >> gpurun_out/r04_i8_ab.log 2>&1
done
cd /tmp && export TMPDIR=/tmp KV_PREC=i8x5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04_i8_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/ab_forward.py" i8prof 2048 > "$GRAFT_REPO_ROOT/gpurun_out/r04_i8_prof.log" 2>&1
