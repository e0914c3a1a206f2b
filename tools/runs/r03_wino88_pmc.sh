#!/bin/bash
# Counter and kernel-trace passes of the fp32 F(8x8) tower (the fp32 default
# above 16 boards) at 2,048 boards (tools/nn_speed.py 2048: 13 forwards, ~400
# dispatches -- far under rocprofv3's ~8K-dispatch counter limit): per-kernel
# durations, HBM bytes of the GEMMs and the transforms (separate FETCH_SIZE /
# WRITE_SIZE passes), the GEMM's clock and MFMA-busy cycles. Each pass has its
# own time limit; the first failure ends the script. Run through gpurun from
# the repo root; summarise with tools/pmc_kernels.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03w88}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
RX="wino_gemm|wino88"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o t -- python3 $R/tools/nn_speed.py 2048 > $O/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/nn_speed.py 2048 > $O/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/nn_speed.py 2048 > $O/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --kernel-include-regex "wino_gemm" -f csv -d $O/sq -o s -- python3 $R/tools/nn_speed.py 2048 > $O/sq.log 2>&1
echo w88-pmc-done
