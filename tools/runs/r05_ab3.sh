#!/bin/bash
# round 5: the int8-digit GEMM forms (tools/i8gemm_ab.py), the int8 tests, the fp32-tower forms A/B
# (slice / fused per-row / fused per-segment: forward time, outputs compared), kernel traces of the two fused
# forms, the library layout under rocprofv3 --pmc (round-3 SIGSEGV attribution)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_ab3}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp KV_ALGO=winograd88i8
timeout -k 10 300 python -u tools/i8gemm_ab.py 2048 256 > $O/gemm_ab.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    tests/test_nn_gpu.py -k "i8 or winograd88i8" > $O/tests.log 2>&1
: > $O/ab.log
for rep in 1 2; do
    KV_I8F32_SLICE=1 KV_I8F32_GEMM=r4 timeout -k 10 200 python -u tools/ab_forward.py slice 2048 256 >> $O/ab.log 2>&1
    KV_I8F32_GEMM=r4 timeout -k 10 200 python -u tools/ab_forward.py rowr4 2048 256 >> $O/ab.log 2>&1
    timeout -k 10 200 python -u tools/ab_forward.py row 2048 256 >> $O/ab.log 2>&1
    KV_I8F32_SEG=1 timeout -k 10 200 python -u tools/ab_forward.py seg 2048 256 >> $O/ab.log 2>&1
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for B in (2048, 256):
    for t in ("rowr4", "row", "seg"):
        a = np.load(f"/tmp/ab_slice_{B}_p.npy"); b = np.load(f"/tmp/ab_{t}_{B}_p.npy")
        print(B, t, "logits bit-identical to slice form" if np.array_equal(a.view(np.uint32), b.view(np.uint32))
              else f"logits differ from slice form by {np.abs(a-b).max():.3e}")
PY
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_row -o run -- python3 $R/tools/ab_forward.py pr 2048 > $O/prof_row.log 2>&1
KV_I8F32_SEG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_seg -o run -- python3 $R/tools/ab_forward.py ps 2048 > $O/prof_seg.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES -d $O/maps_prof -o m -- python3 $R/tools/runs/r05_maps.py $O/maps.txt > $O/maps.log 2>&1
echo ab3-done
