#!/bin/bash
# Round-3 counter passes of the F(4x8) tower at 2,048 boards on the final code
# (tools/nn_speed.py 2048: 13 forwards, ~330 dispatches -- far under
# rocprofv3's ~8K-dispatch limit): HBM bytes of the residual GEMM and of the
# output/input transforms (separate FETCH_SIZE / WRITE_SIZE passes), then the
# GEMM's clock and MFMA-busy cycles. Each pass has its own time limit; the
# first failure ends the script. Run through gpurun from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03gemm}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
RX="wino_gemm|wino48_out"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/nn_speed.py 2048 > $O/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/nn_speed.py 2048 > $O/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --kernel-include-regex "wino_gemm" -f csv -d $O/sq -o s -- python3 $R/tools/nn_speed.py 2048 > $O/sq.log 2>&1
echo gemm-pmc-done
