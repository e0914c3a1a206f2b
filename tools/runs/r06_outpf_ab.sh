#!/bin/bash
# round 6: the output kernel prefetching the next board's M into L2 (KV_OUT_PF = 25 / 50 loads per lane, by
# global_load_lds into a scratch LDS line) against none; forward A/B with outputs compared (must be bit-identical),
# kernel traces
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_outpf_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
: > $O/ab.log
for rep in 1 2 3; do
    timeout -k 10 200 python -u tools/ab_forward.py pf0 2048 1024 >> $O/ab.log 2>&1
    KV_OUT_PF=25 timeout -k 10 200 python -u tools/ab_forward.py pf25 2048 1024 >> $O/ab.log 2>&1
    KV_OUT_PF=50 timeout -k 10 200 python -u tools/ab_forward.py pf50 2048 1024 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 1024):
    for t in ("pf25", "pf50"):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_pf0_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{t}_{B}_{k}.npy")
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
prof pf0 KV_ALGO=auto
prof pf25 KV_OUT_PF=25
prof pf50 KV_OUT_PF=50
grep -v amdgpu $O/ab.log
grep -h "out_kernel" $O/pf0.txt $O/pf25.txt $O/pf50.txt | cut -c1-160
