#!/bin/bash
# round 6: phase stagger of the fp32 tower's output kernels (KV_OUT_STAG = s_sleep-127 units for the first-round
# workgroups of half the CUs) on the held-V kernel (KV_I8F32_OUT=hold, one board per CU) and the 64-register one
# (two per CU): forward A/B at 2,048 / 256 boards with outputs compared bit for bit, then kernel traces.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_stag}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
: > $O/ab.log
for rep in 1 2; do
  for st in 0 2 4; do
    KV_OUT_STAG=$st KV_I8F32_OUT=hold timeout -k 10 200 python -u tools/ab_forward.py hold$st 2048 256 >> $O/ab.log 2>&1
    KV_OUT_STAG=$st timeout -k 10 200 python -u tools/ab_forward.py out2$st 2048 256 >> $O/ab.log 2>&1
  done
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for t in ("hold2", "hold4", "out20", "out22", "out24"):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_hold0_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{t}_{B}_{k}.npy")
            print(t, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
cd /tmp
export TMPDIR=/tmp
for st in 2 4; do
KV_OUT_STAG=$st KV_I8F32_OUT=hold timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_hold$st -o run -- \
    python3 $R/tools/ab_forward.py ph 2048 > $O/prof_hold$st.log 2>&1
python3 $R/tools/rocpd_stats.py $O/prof_hold$st/run_results.db $O/hold${st}_kernel_stats.csv > $O/hold$st.txt
KV_OUT_STAG=$st timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_out2$st -o run -- \
    python3 $R/tools/ab_forward.py po 2048 > $O/prof_out2$st.log 2>&1
python3 $R/tools/rocpd_stats.py $O/prof_out2$st/run_results.db $O/out2${st}_kernel_stats.csv > $O/out2$st.txt
done
rm -rf $O/prof_*/
echo stag-done
