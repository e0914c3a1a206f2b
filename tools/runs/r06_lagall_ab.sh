#!/bin/bash
# round 6: R3 GEMM with all of a stage's chunk-1 MFMAs lagging to the next barrier (KV_R3_LAGALL=1:
# libkv_lagall.so) against the product (chunk 1's B digits 1-2 lag); bit-exact R3 GEMM test under the variant,
# back-to-back GEMM, forward A/B with outputs compared
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_lagall_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
V=$R/knightvision_amd/libkv_lagall.so
KV_LIB_PATH=$V timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_wino_i8_gpu.py -k "i8r3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/b2b.log
for rep in 1 2; do
    timeout -k 10 60 python -u tools/gemm_b2b.py base >> $O/b2b.log 2>&1
    KV_LIB_PATH=$V timeout -k 10 60 python -u tools/gemm_b2b.py lagall >> $O/b2b.log 2>&1
done
: > $O/ab.log
for rep in 1 2; do
    timeout -k 10 200 python -u tools/ab_forward.py base 2048 256 >> $O/ab.log 2>&1
    KV_LIB_PATH=$V timeout -k 10 200 python -u tools/ab_forward.py lagall 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_base_{B}_{k}.npy"); b = np.load(f"/tmp/ab_lagall_{B}_{k}.npy")
        print("lagall", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
PY
grep -v amdgpu $O/b2b.log | cut -c1-90
grep -v amdgpu $O/ab.log
