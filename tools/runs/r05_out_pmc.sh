#!/bin/bash
# round 5: SQ counters of the fp32 tower's output kernels (wino88i32_out_kernel) at 2,048 boards -- is the kernel
# VALU-issue bound or waiting on memory / its barrier?
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r05_out_pmc}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp PYTHONUNBUFFERED=1 KV_ALGO=winograd88i8
RX="wino88i32_out_kernel"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --kernel-include-regex "$RX" -f csv -d $O/sq2 -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq2.log 2>&1
echo out-pmc-done
