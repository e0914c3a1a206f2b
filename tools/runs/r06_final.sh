#!/bin/bash
# round 6, final code (R3 headline, its GEMM with 64-k stages, F(4x8)/f16x3 retired, 5-digit fp64 out of AUTO): the whole -m gpu suite,
# smoke(), the R3 GEMM's HBM bytes (FETCH_SIZE / WRITE_SIZE passes) and SQ counters at 2,048 boards, the C3 bench
# under rocprofv3 --kernel-trace --stats, the driver's bench command (defaults) and the C2 line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_final}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest ${SUITE:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_suite.log 2>&1 \
    || { tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke-done
cd /tmp
export TMPDIR=/tmp
RX="${RX:-wino88i32_gemm_r3k64_kernel<512}"
export KV_ALGO=winograd88i8r3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
echo pmc-done
unset KV_ALGO
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
    --alt-precision= --alt-algo= --ref-block 0 --trained-steps 0 --no-cpu-baseline > $O/bench_under_rocprof.log 2>&1
echo rocprof-done
cd $R
timeout -k 10 700 python -u bench.py > $O/bench.log 2> $O/bench.err
tail -1 $O/bench.log
echo bench-done
timeout -k 10 200 python -u bench.py --slots 256 --sims 400 --steps 5 --warmup 2 > $O/bench_c2.log 2> $O/bench_c2.err
echo c2-done
