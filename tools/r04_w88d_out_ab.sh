#!/bin/bash
# A/B of the fp64-domain output transform: one lane per (board, channel) plane (KV_W88D_OUT=1) against the
# lane-pair form (default), forward at 2048 / 256 boards, alternating; outputs compared bit for bit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab KV_PREC=f64w
for i in 1 2; do
  KV_W88D_OUT=1 timeout -k 10 120 python tools/ab_forward.py one 2048 256
  timeout -k 10 120 python tools/ab_forward.py pair 2048 256
done
python - <<'PY'
import numpy as np
for B in (2048, 256):
    for t in ("p", "v"):
        a = np.load(f"/tmp/ab/ab_one_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_pair_{B}_{t}.npy")
        print(B, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
