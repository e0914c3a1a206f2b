#!/bin/bash
# A/B of the 32-row F(8x8) GEMM tile's k-tile (new: 32 floats, 16 k-steps per
# tile; ck16: 16 floats) and the 64-padding of the previous commit (head), at the
# batches that use it; outputs compared bit for bit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
S="17 32 80 96 2048"
for i in 1 2; do
  KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 150 python tools/ab_forward.py head $S
  KV_LIB_PATH=$R/knightvision_amd/libkv_ck16.so timeout -k 10 150 python tools/ab_forward.py ck16 $S
  timeout -k 10 150 python tools/ab_forward.py new $S
done
python - <<PY
import numpy as np
for B in "$S".split():
    for tag in ("ck16", "new"):
        for t in ("p", "v"):
            a = np.load(f"/tmp/ab/ab_head_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_{tag}_{B}_{t}.npy")
            print(B, tag, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
