#!/bin/bash
# A/B of the F(8x8) output transform forms (KV_W88_OUT2=0: one lane per
# (board, channel) plane; 1: two lanes per plane), alternating on one box, from
# 17 to 2,048 boards; outputs compared bit for bit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
S="17 32 64 96 128 192 256 384 512 1024 2048"
for i in 1 2; do
  KV_W88_OUT2=0 timeout -k 10 150 python tools/ab_forward.py one $S
  KV_W88_OUT2=1 timeout -k 10 150 python tools/ab_forward.py two $S
  KV_LIB_PATH=$R/knightvision_amd/libkv_k16.so timeout -k 10 150 python tools/ab_forward.py k16 1024 2048
done
python - <<PY
import numpy as np
for B in "$S".split():
    for t in ("p", "v"):
        a = np.load(f"/tmp/ab/ab_one_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_two_{B}_{t}.npy")
        print(B, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
