#!/bin/bash
# round 5, final code (reads-first GEMM schedule): the whole -m gpu suite, smoke(), the fp32-tower GEMM's HBM bytes
# (FETCH_SIZE / WRITE_SIZE passes) and SQ counters at 2,048 boards, the C3 bench under rocprofv3 --kernel-trace
# --stats, the driver's bench command and the C2 line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_final7}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
echo suite-done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke-done
cd /tmp
export TMPDIR=/tmp
RX="wino88i32_gemm_lagt_kernel<512"
export KV_ALGO=winograd88i8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
echo pmc-done
unset KV_ALGO
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
    --alt-precision= --alt-algo= --ref-block 0 --trained-steps 0 --no-cpu-baseline > $O/bench_under_rocprof.log 2>&1
echo rocprof-done
cd $R
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err
echo bench-done
timeout -k 10 200 python -u bench.py --slots 256 --sims 400 --steps 5 --warmup 2 > $O/bench_c2.log 2> $O/bench_c2.err
echo c2-done
