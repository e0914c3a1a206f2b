#!/bin/bash
# round 5: fp32 transforms w88_bt / w88_at in even / odd form (tools/gen_wino88.py KV_GEN_EO_F32): the fp32 kernels'
# tests (fused output kernels == two-kernel forms, golden logits, batch sizes, golden games on the explicit fp32
# towers), then a forward A/B against the previous build (libkv_b.so, plain chains) on the headline tower
# (winograd88i8), the fp32 MFMA tower (winograd88) and the fp64-input-transform tower (winograd88i8v)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_eo32}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_wino_i8_gpu.py tests/test_nn_gpu.py tests/test_engine_gpu.py \
    -k "out_kernel or golden or batch_sizes or invariance or games_match" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests-done
: > $O/ab.log
for rep in 1 2; do
    for a in winograd88i8 winograd88 winograd88i8v; do
        KV_ALGO=$a KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py old_$a 2048 256 >> $O/ab.log 2>&1
        KV_ALGO=$a timeout -k 10 200 python -u tools/ab_forward.py new_$a 2048 256 >> $O/ab.log 2>&1
    done
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for t in ("winograd88i8", "winograd88", "winograd88i8v"):
    for B in (2048, 256):
        a = np.load(f"/tmp/ab_old_{t}_{B}_p.npy"); b = np.load(f"/tmp/ab_new_{t}_{B}_p.npy")
        print(t, B, "max |new - old| logit", float(np.abs(a - b).max()))
PY
echo ab-done
