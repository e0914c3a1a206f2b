#!/bin/bash
# round-4 profiles of the int8-digit towers: HBM bytes of the two GEMMs at 2,048 boards (separate FETCH_SIZE /
# WRITE_SIZE passes), then a kernel trace of the C3 bench (2 timed moves) whose GEMM average the bench's HIP
# events must match
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_i8prof
mkdir -p $O
cd /tmp
export TMPDIR=/tmp AB_DIR=/tmp
KV_ALGO=winograd88i8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wino88i_gemm" -f csv -d $O/f32fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/f32fetch.log 2>&1
KV_ALGO=winograd88i8 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wino88i_gemm" -f csv -d $O/f32write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/f32write.log 2>&1
KV_PREC=i8x5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wino88i_gemm" -f csv -d $O/f64fetch -o f -- python3 $R/tools/ab_forward.py p 2048 > $O/f64fetch.log 2>&1
KV_PREC=i8x5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wino88i_gemm" -f csv -d $O/f64write -o w -- python3 $R/tools/ab_forward.py p 2048 > $O/f64write.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/c3 -o c3 -- python3 $R/bench.py --steps 2 --warmup 1 --alt-precision= --alt-algo= --ref-block 0 --no-cpu-baseline --trained-steps 0 > $O/c3_bench.log 2> $O/c3_bench.err
echo prof-done
