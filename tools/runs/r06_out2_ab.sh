#!/bin/bash
# round 6: the fp32 tower's output kernel at a 64-register budget (wino88i32_out2_kernel: the 32 activations
# held across the exponent barrier, the input transform run twice, two boards per CU) against the held-V form
# (KV_I8F32_OUT=hold): the bit-identity test of both forms against the slice kernel, a forward A/B with the
# outputs compared bit for bit, and a kernel trace of each form at 2,048 boards.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_out2}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "i8f32_out_kernel" > $O/tests.log 2>&1
: > $O/ab.log
for rep in 1 2 3; do
    KV_I8F32_OUT=hold timeout -k 10 200 python -u tools/ab_forward.py hold 2048 256 >> $O/ab.log 2>&1
    timeout -k 10 200 python -u tools/ab_forward.py out2 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_hold_{B}_{k}.npy"); b = np.load(f"/tmp/ab_out2_{B}_{k}.npy")
        print(B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
cd /tmp
export TMPDIR=/tmp
KV_I8F32_OUT=hold timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_hold -o run -- \
    python3 $R/tools/ab_forward.py ph 2048 > $O/prof_hold.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_out2 -o run -- \
    python3 $R/tools/ab_forward.py po 2048 > $O/prof_out2.log 2>&1
echo out2-done
