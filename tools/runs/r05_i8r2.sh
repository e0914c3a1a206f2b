#!/bin/bash
# round 5: KV_PREC_I8R4 in row lines with its fused output kernel (wino88i64r_out_kernel): kernel tests, the
# forward tests, forward A/B against KV_PREC_I8X5 and against the GEMM with 1 lagging B digit
# (knightvision_amd/libkv_b.so, KV_I8R_LJ=3), a kernel trace
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_i8r2}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wino_i8_gpu.py -k "i8r or r8" -x -v --timeout 120 --timeout-method thread > $O/kernel_tests.log 2>&1
echo kernel-tests-done
timeout -k 10 500 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_accuracy_gpu.py -k "i8r4 or auto_within or calibration_choice" -x -v -s --timeout 200 --timeout-method thread > $O/nn_tests.log 2>&1
echo nn-tests-done
: > $O/ab.log
for rep in 1 2; do
    KV_PREC=i8x5 timeout -k 10 200 python -u tools/ab_forward.py i8x5 2048 256 >> $O/ab.log 2>&1
    KV_PREC=i8r4 timeout -k 10 200 python -u tools/ab_forward.py i8r4 2048 256 >> $O/ab.log 2>&1
    KV_PREC=i8r4 KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py i8r4lj3 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_i8r4_{B}_{k}.npy"); b = np.load(f"/tmp/ab_i8r4lj3_{B}_{k}.npy")
        print("LJ 2 vs 3", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else "DIFFER")
PY
echo ab-done
cd /tmp
export TMPDIR=/tmp
KV_PREC=i8r4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/ab_forward.py pr 2048 > $O/prof.log 2>&1
echo prof-done
