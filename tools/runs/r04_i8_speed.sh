#!/bin/bash
# KV_PREC_I8X5: bit-exact kernel test, forward timing per GEMM variant (KV_I8_TILE) beside KV_PREC_F64W,
# and a kernel-trace profile of the default variant
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_i8_gpu.py \
    > gpurun_out/r04_i8_exact.log 2>&1
for t in ${I8_TILES:-0 1 2}; do
    KV_I8_TILE=$t KV_PREC=i8x5 timeout -k 10 200 python -u tools/ab_forward.py i8_tile$t 2048 256 64 \
        >> gpurun_out/r04_i8_speed.log 2>&1
done
cd /tmp && export TMPDIR=/tmp KV_PREC=i8x5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04_i8_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/ab_forward.py" i8prof 2048 > "$GRAFT_REPO_ROOT/gpurun_out/r04_i8_prof.log" 2>&1
