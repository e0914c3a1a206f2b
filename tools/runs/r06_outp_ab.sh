#!/bin/bash
# round 6: the persistent LDS-DMA output kernel (KV_I8F32_OUT=p: wino88i32_outp_kernel) against the held-V kernel
# (the default): the output kernels' bit-identity tests (every form), a forward A/B on the 4-digit and the 3-digit
# (R3) towers with outputs compared bit for bit, kernel traces of the persistent form.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_outp}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "i8f32_out_kernel" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab.log
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u tools/ab_forward.py $tag 2048 256 >> $O/ab.log 2>&1
}
for rep in 1 2; do
    run i8hold KV_ALGO=winograd88i8
    run i8p KV_ALGO=winograd88i8 KV_I8F32_OUT=p
    run r3hold KV_ALGO=winograd88i8r3
    run r3p KV_ALGO=winograd88i8r3 KV_I8F32_OUT=p
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for a_, b_ in (("i8hold", "i8p"), ("r3hold", "r3p")):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_{a_}_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{b_}_{B}_{k}.npy")
            print(b_, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
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
prof r3p KV_ALGO=winograd88i8r3 KV_I8F32_OUT=p
echo outp-done
