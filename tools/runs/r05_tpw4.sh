#!/bin/bash
# round 5: four tiles per workgroup for C2-size grids (wino88i32_gemm_lagt_kernel<.,4>, chosen at 256 boards):
# M bit-identity + timing, the int8 / network GPU tests, a forward A/B at 256 boards against one tile per
# workgroup (KV_I8F32_TPW=1) with outputs compared bit for bit, then the C2 bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_tpw4}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
I8_VARIANTS=0,14,18 timeout -k 10 300 python -u tools/i8gemm_ab.py 256 2048 > $O/gemm_ab.log 2>&1
echo gemm-ab-done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py -k "i8 or winograd88i8 or invariance" > $O/tests.log 2>&1
echo tests-done
: > $O/ab.log
for rep in 1 2 3; do
    KV_ALGO=winograd88i8 KV_I8F32_TPW=1 timeout -k 10 200 python -u tools/ab_forward.py t1 256 2048 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py t4 256 2048 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (256, 2048):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_t1_{B}_{k}.npy"); b = np.load(f"/tmp/ab_t4_{B}_{k}.npy")
        print(B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
timeout -k 10 200 python -u bench.py --slots 256 --sims 400 --steps 5 --warmup 2 > $O/bench_c2.log 2> $O/bench_c2.err
echo tpw4-done
