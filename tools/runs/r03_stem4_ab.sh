#!/bin/bash
# A/B of the F(8x8) stem: s3 = the plane exchanged through LDS (stem_kernel<3>,
# knightvision_amd/libkv_s3.so) vs s4 = lane-half split with lane swaps
# (stem_kernel<4>), alternating on one box; outputs compared bit for bit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
S="32 256 2048"
for i in 1 2; do
  KV_LIB_PATH=$R/knightvision_amd/libkv_s3.so timeout -k 10 150 python tools/ab_forward.py s3 $S
  timeout -k 10 150 python tools/ab_forward.py s4 $S
done
python - <<PY
import numpy as np
for B in "$S".split():
    for t in ("p", "v"):
        a = np.load(f"/tmp/ab/ab_s3_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_s4_{B}_{t}.npy")
        print(B, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/stem4 -o s -- python3 $R/tools/nn_speed.py 2048 > /dev/null 2>&1
echo stem-ab-done
