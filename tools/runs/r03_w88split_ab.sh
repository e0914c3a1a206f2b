#!/bin/bash
# A/B of two F(8x8) forward changes against the previous build, alternating on
# one box, outputs compared bit for bit: head = knightvision_amd/libkv_head.so
# (the previous commit); stem = the stem writing conv2's F(8x8) V itself
# (KV_W88_SPLIT=0); split = that + the GEMM's points split over two tile shapes
# so no round of tiles is left half full (KV_W88_SPLIT=1).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
for i in 1 2; do
  KV_LIB_PATH=$R/knightvision_amd/libkv_head.so timeout -k 10 120 python tools/ab_forward.py head 2048 1024 256
  KV_W88_SPLIT=0 timeout -k 10 120 python tools/ab_forward.py stem 2048 1024 256
  KV_W88_SPLIT=1 timeout -k 10 120 python tools/ab_forward.py split 2048 1024 256
done
python - <<'PY'
import numpy as np
for B in (2048, 1024, 256):
    for tag in ("stem", "split"):
        for t in ("p", "v"):
            a = np.load(f"/tmp/ab/ab_head_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_{tag}_{B}_{t}.npy")
            print(B, tag, t, "identical to head" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
