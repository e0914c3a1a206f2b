#!/bin/bash
# round 5, final code: HBM bytes (FETCH_SIZE / WRITE_SIZE passes) and SQ counters of the trained-weights path's GEMM
# (KV_PREC_I8R4, 2,048 boards), then the N>1 bench path rehearsed with 2 gloo ranks sharing the box at the full C3
# per-rank size (every rank's calibration in the line)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_final_multi}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp
export TMPDIR=/tmp
RX="wino88i_gemm_lag5_kernel<512"
export KV_PREC=i8r4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
echo pmc-done
unset KV_PREC
cd $R
export KV_BENCH_BACKEND=gloo
X="--alt-precision= --alt-algo= --ref-block 0 --trained-steps 0 --no-cpu-baseline"
timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 $X > $O/gloo2.log 2> $O/gloo2.err
echo multi-done
