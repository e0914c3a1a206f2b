#!/bin/bash
# round 5: the lag GEMM as the default -- its bit-identity tests, a forward A/B against the round-4 GEMM, the
# C3 bench under rocprofv3 --kernel-trace --stats (2 timed moves), the GEMM's HBM bytes (FETCH_SIZE and
# WRITE_SIZE passes) and SQ counters at 2,048 boards
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_lag_final}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
KV_ALGO=winograd88i8 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py -k "i8 or winograd88i8" > $O/tests.log 2>&1
: > $O/ab.log
for rep in 1 2; do
    KV_ALGO=winograd88i8 KV_I8F32_GEMM=r4 timeout -k 10 200 python -u tools/ab_forward.py r4 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py lag 2048 256 >> $O/ab.log 2>&1
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
    --alt-precision= --alt-algo= --ref-block 0 --trained-steps 0 --no-cpu-baseline > $O/bench_under_rocprof.log 2>&1
RX="wino88i32_gemm_lag_kernel<512"
export KV_ALGO=winograd88i8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-include-regex "$RX" -f csv -d $O/wait -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/wait.log 2>&1
echo lag-final-done
