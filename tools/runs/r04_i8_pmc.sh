#!/bin/bash
# counter passes of the KV_PREC_I8X5 GEMM at 2,048 boards (tools/ab_forward.py: 13 forwards): clock and
# MFMA-busy cycles, LDS activity / bank conflicts, HBM bytes. Each pass has its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_i8_pmc}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp KV_PREC=i8x5 AB_DIR=/tmp
RX="wino88i_gemm"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES --kernel-include-regex "$RX" -f csv -d $O/sq -o s -- python3 $R/tools/ab_forward.py p 2048 > $O/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA --kernel-include-regex "$RX" -f csv -d $O/lds -o l -- python3 $R/tools/ab_forward.py p 2048 > $O/lds.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d $O/fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-include-regex "$RX" -f csv -d $O/wait -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/wait.log 2>&1
echo pmc-done
