set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export AB_DIR=/tmp/ab
for i in 1 2; do
  timeout -k 10 120 python tools/ab_forward.py base 2048 1024
  KV_LIB_PATH=$R/knightvision_amd/libkv_k16.so timeout -k 10 120 python tools/ab_forward.py k16 2048 1024
done
python - <<'PY'
import numpy as np
for B in (2048, 1024):
    for t in ("p", "v"):
        a = np.load(f"/tmp/ab/ab_base_{B}_{t}.npy"); b = np.load(f"/tmp/ab/ab_k16_{B}_{t}.npy")
        print(B, t, "identical" if np.array_equal(a, b) else f"DIFFER max {np.abs(a-b).max()}")
PY
