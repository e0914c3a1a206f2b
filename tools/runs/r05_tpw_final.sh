#!/bin/bash
# round 5: 5 / 4 tiles per workgroup as the fp32 tower's GEMM default (wino88i32_gemm_lagt_kernel) -- the int8 and
# network GPU tests, a forward A/B against one tile per workgroup (KV_I8F32_TPW=1, outputs bit for bit), the C3
# bench under rocprofv3 --kernel-trace --stats, the GEMM's HBM bytes (FETCH_SIZE and WRITE_SIZE passes) and SQ
# counters at 2,048 boards, then the driver's bench command
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_tpw_final}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py tests/test_mcts_gpu.py -k "i8 or winograd88i8 or invariance or c3" > $O/tests.log 2>&1
echo tests-done
: > $O/ab.log
for rep in 1 2; do
    KV_ALGO=winograd88i8 KV_I8F32_TPW=1 timeout -k 10 200 python -u tools/ab_forward.py t1 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py tn 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_t1_{B}_{k}.npy"); b = np.load(f"/tmp/ab_tn_{B}_{k}.npy")
        print(B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
echo ab-done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
    --alt-precision= --alt-algo= --ref-block 0 --trained-steps 0 --no-cpu-baseline > $O/bench_under_rocprof.log 2>&1
echo rocprof-done
RX="wino88i32_gemm_lagt_kernel<512"
export KV_ALGO=winograd88i8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
echo pmc-done
unset KV_ALGO
cd $R
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err
echo bench-done
