#!/bin/bash
# Standard measurement pass on the GPU box (run through gpurun from the repo
# root): default bench line, rocprofv3 kernel-trace summary of the same
# command, and PMC passes (HBM bytes, MFMA busy) for the dominant kernel at the
# bench's batch. Outputs under gpurun_out/round/. Every GPU step has its own
# time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log > $O/bench.json
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -- python3 $R/bench.py > $O/bench_traced.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wino_gemm|conv3x3" -f csv -d $O/pmc_fetch -o f -- python3 $R/tools/nn_speed.py 256 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wino_gemm|conv3x3" -f csv -d $O/pmc_write -o w -- python3 $R/tools/nn_speed.py 256 > $O/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "wino_gemm|conv3x3" -f csv -d $O/pmc_sq -o s -- python3 $R/tools/nn_speed.py 256 > $O/pmc_sq.log 2>&1

cd $R
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -q -s -k "golden" --timeout 200 --timeout-method thread > $O/nn_errors.log 2>&1
echo done
