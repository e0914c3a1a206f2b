#!/bin/bash
# round 6: the fused R3 stem (stem_r3_kernel: conv2's digits straight from the stem) against the stem + slice pair
# (KV_STEM_R3=0); R3 / NN tests, forward A/B with outputs compared (must be bit-identical), kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_stemr3_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nn_gpu.py \
    tests/test_wino_i8_gpu.py -k "r3 or slice_limit or golden or batch_invariance" > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab.log
for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/ab_forward.py fused 2048 256 128 >> $O/ab.log 2>&1
    KV_STEM_R3=0 timeout -k 10 200 python -u tools/ab_forward.py slice 2048 256 128 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256, 128):
    for k in ("p", "v"):
        a = np.load(f"/tmp/ab_slice_{B}_{k}.npy"); b = np.load(f"/tmp/ab_fused_{B}_{k}.npy")
        print("fused", B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
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
prof fused KV_ALGO=auto
prof slice KV_STEM_R3=0
grep -v amdgpu $O/ab.log
grep -i "stem\|slice" $O/fused.txt $O/slice.txt
