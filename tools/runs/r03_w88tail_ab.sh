#!/bin/bash
# A/B probe of the F(8x8) GEMM's last round at 2,048 boards (6,400 tiles on 512
# slots: the last 256 run one per CU): KV_W88_TAIL=0 one launch; 1 / 2 / 3: points
# 96-99 as 64x64 tiles (k-tile 32 / 16) or 128x64 tiles in a second launch.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
for i in 1 2; do
  for m in 0 1 2 3; do KV_W88_TAIL=$m timeout -k 10 150 python tools/ab_forward.py t$m 2048; done
done
python - <<PY
import numpy as np
for m in (1, 2, 3):
    for t in ("p", "v"):
        a = np.load(f"/tmp/ab/ab_t0_2048_{t}.npy"); b = np.load(f"/tmp/ab/ab_t{m}_2048_{t}.npy")
        print(m, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
