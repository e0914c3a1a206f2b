#!/bin/bash
# round 6: the fp32 tower on 3 radix-256 digits (KV_PATH_WINO88_I8F32R3) as AUTO's first candidate: the whole GPU
# suite (bit-exact GEMM / output kernels, network tolerances, golden games, MCTS parity on the AUTO path), then
# the R3 GEMM's lag depth (KV_I8R3_LJ 1, the default build, vs 2: knightvision_amd/libkv_lj2.so) at 2,048 / 256
# boards, outputs compared bit for bit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_r3val}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 800 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || \
    { echo suite-failed; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
: > $O/ab.log
for rep in 1 2; do
    KV_ALGO=winograd88i8r3 timeout -k 10 200 python -u tools/ab_forward.py lj1 2048 256 >> $O/ab.log 2>&1
    KV_LIB_PATH=$R/knightvision_amd/libkv_lj2.so KV_ALGO=winograd88i8r3 timeout -k 10 200 python -u tools/ab_forward.py lj2 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_lj1_{B}_{k}.npy"); b = np.load(f"/tmp/ab_lj2_{B}_{k}.npy")
        print("lj2", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
PY
echo r3val-done
