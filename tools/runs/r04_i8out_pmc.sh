#!/bin/bash
# counter passes of the fused int8 out kernel (wino88i_out_kernel) at 2,048 boards
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_i8out_pmc}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp KV_PREC=i8x5 AB_DIR=/tmp
RX="wino88i_outmax|wino88i_in_kernel|wino88d_out_half"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SALU --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d $O/write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/write.log 2>&1
echo pmc-done
