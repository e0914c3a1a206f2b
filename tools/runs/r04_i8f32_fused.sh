#!/bin/bash
# (historical: the fused kernel and KV_I8F32_FUSED were dropped after this measurement, profiles/r04_i8f32_fused_out.log)
# fp32 tower on int8 digits, fused output kernel (wino88i32_out_kernel, row-line digit layout): the
# bit-exact GEMM test, the fused-vs-slice bit-identity test and the tower's accuracy / invariance tests,
# then forward timing with KV_I8F32_FUSED=1 / 0 alternating, a kernel trace of the fused form, and the
# new GEMM's HBM bytes (separate FETCH_SIZE / WRITE_SIZE passes). Each GPU step has its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04_i8f32_fused
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py -k "i8 or winograd88i8 or fused" > $O/tests.log 2>&1
: > $O/ab.log
for rep in 1 2; do
    for f in 1 0; do
        KV_I8F32_FUSED=$f KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py "fused$f" 2048 256 128 >> $O/ab.log 2>&1
    done
done
cd /tmp
export TMPDIR=/tmp
KV_ALGO=winograd88i8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
    python3 $R/tools/ab_forward.py fprof 2048 > $O/prof.log 2>&1
KV_ALGO=winograd88i8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wino88i" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
KV_ALGO=winograd88i8 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wino88i" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
echo fused-done
