#!/bin/bash
# round-4 row-line layout, final checks: the GPU suite, smoke(), the row-line GEMM's HBM bytes at 2,048
# boards (separate FETCH_SIZE / WRITE_SIZE passes), the driver's default bench line. Each GPU step has its
# own time limit; the steps are chained by set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04_rl_final
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp
export TMPDIR=/tmp
KV_ALGO=winograd88i8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wino88i_gemm" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
KV_ALGO=winograd88i8 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wino88i_gemm" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
cd $R
timeout -k 10 900 python -u bench.py > $O/bench.log 2> $O/bench.err
echo final-done
