#!/bin/bash
# A/B of F(8x8) batches padded to 32 boards with a 32-row GEMM tile (new)
# against the padding to 64 (head = knightvision_amd/libkv_head.so, the
# previous commit), alternating on one box; outputs compared bit for bit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
S="17 24 32 48 64 80 96 128 160 192 256"
for i in 1 2; do
  KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 150 python tools/ab_forward.py head $S
  timeout -k 10 150 python tools/ab_forward.py new $S
done
python - <<PY
import numpy as np
for B in "$S".split():
    for t in ("p", "v"):
        a = np.load(f"/tmp/ab/ab_head_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_new_{B}_{t}.npy")
        print(B, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
