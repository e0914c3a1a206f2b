#!/bin/bash
# round 5: the fp32 tower's output kernel writing the next V's int8 digits itself (wino88i32_out_kernel)
# against the round-4 form (out kernel + slice, KV_I8F32_SLICE=1): the kernel's bit-identity test, the
# int8 network tests, a forward A/B (outputs compared bit for bit), then a kernel trace of the new form.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_fused_out}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py -k "i8 or winograd88i8" > $O/tests.log 2>&1
: > $O/ab.log
for rep in 1 2 3; do
    KV_I8F32_SLICE=1 timeout -k 10 200 python -u tools/ab_forward.py slice 2048 256 128 >> $O/ab.log 2>&1
    timeout -k 10 200 python -u tools/ab_forward.py fused 2048 256 128 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256, 128):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_slice_{B}_{k}.npy"); b = np.load(f"/tmp/ab_fused_{B}_{k}.npy")
        print(B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
    python3 $R/tools/ab_forward.py pf 2048 > $O/prof.log 2>&1
echo fused-done
