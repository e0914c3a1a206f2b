#!/bin/bash
# round 6: (1) phase stagger of the fp32 tower's output kernels (KV_OUT_STAG = s_sleep-127 units for the
# first-round workgroups of half the CUs) on the held-V kernel (KV_I8F32_OUT=hold) and the 64-register one;
# (2) the fp32 tower on 3 radix-256 digits (KV_ALGO winograd88i8r3: 6 digit pairs per GEMM instead of 10).
# Forward A/B at 2,048 / 256 boards, outputs compared, kernel traces.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_ab1}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "i8f32_out_kernel or i8_gemm_bit_exact" > $O/tests.log 2>&1
: > $O/ab.log
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u tools/ab_forward.py $tag 2048 256 >> $O/ab.log 2>&1
}
for rep in 1 2; do
    run hold0 KV_ALGO=winograd88i8 KV_I8F32_OUT=hold KV_OUT_STAG=0
    run hold3 KV_ALGO=winograd88i8 KV_I8F32_OUT=hold KV_OUT_STAG=3
    run out20 KV_ALGO=winograd88i8 KV_OUT_STAG=0
    run out23 KV_ALGO=winograd88i8 KV_OUT_STAG=3
    run r3hold KV_ALGO=winograd88i8r3 KV_I8F32_OUT=hold
    run r3out2 KV_ALGO=winograd88i8r3
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for t in ("hold3", "out20", "out23", "r3hold", "r3out2"):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_hold0_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{t}_{B}_{k}.npy")
            print(t, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
PY
cd /tmp
export TMPDIR=/tmp
prof() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$tag -o run -- \
        python3 $R/tools/ab_forward.py p$tag 2048 > $O/prof_$tag.log 2>&1
    python3 $R/tools/rocpd_stats.py $O/prof_$tag/run_results.db $O/${tag}_kernel_stats.csv > $O/$tag.txt
    rm -rf $O/prof_$tag
}
prof hold3 KV_ALGO=winograd88i8 KV_I8F32_OUT=hold KV_OUT_STAG=3
prof out23 KV_ALGO=winograd88i8 KV_OUT_STAG=3
prof r3hold KV_ALGO=winograd88i8r3 KV_I8F32_OUT=hold
echo ab1-done
