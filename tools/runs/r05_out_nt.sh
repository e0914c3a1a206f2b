#!/bin/bash
# round 5: non-temporal stores for the output kernel's digits (KV_I8F32_OUT_NT) and the GEMM's M (KV_I8F32_M_NT):
# forward A/B at 2,048 / 256 boards, outputs bit for bit, 4 alternating repeats, then kernel traces of both.
# The two switches were removed after this run (the digits are now always non-temporal, M plain), so rerunning
# this script measures the kept code three times; profiles/r05_out_nt_ab.log holds the A/B it recorded.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_out_nt2}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
: > $O/ab.log
for rep in 1 2 3 4; do
    timeout -k 10 200 python -u tools/ab_forward.py st 2048 256 >> $O/ab.log 2>&1
    KV_I8F32_OUT_NT=1 timeout -k 10 200 python -u tools/ab_forward.py nt 2048 256 >> $O/ab.log 2>&1
    KV_I8F32_OUT_NT=1 KV_I8F32_M_NT=1 timeout -k 10 200 python -u tools/ab_forward.py ntm 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for t in ("nt", "ntm"):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_st_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{t}_{B}_{k}.npy")
            print(t, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER {np.abs(a-b).max()}")
PY
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_st -o run -- python3 $R/tools/ab_forward.py pst 2048 > $O/prof_st.log 2>&1
KV_I8F32_OUT_NT=1 KV_I8F32_M_NT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ntm -o run -- python3 $R/tools/ab_forward.py pntm 2048 > $O/prof_ntm.log 2>&1
echo nt-done
