#!/bin/bash
# round 5: the fp64 domain on 4 radix-256 digits (KV_PREC_I8R4): kernel bit-exact / bound tests, forward tests,
# the accuracy table on bn / peaked / stress (AUTO's choice), a forward A/B against KV_PREC_I8X5 and a kernel trace
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_i8r}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wino_i8_gpu.py -k "i8r or r8" -x -v --timeout 120 --timeout-method thread > $O/kernel_tests.log 2>&1
echo kernel-tests-done
timeout -k 10 500 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_accuracy_gpu.py -k "i8r4 or auto_within or calibration_choice" -x -v -s --timeout 200 --timeout-method thread > $O/nn_tests.log 2>&1
echo nn-tests-done
: > $O/ab.log
for rep in 1 2; do
    KV_PREC=i8x5 timeout -k 10 200 python -u tools/ab_forward.py i8x5 2048 256 >> $O/ab.log 2>&1
    KV_PREC=i8r4 timeout -k 10 200 python -u tools/ab_forward.py i8r4 2048 256 >> $O/ab.log 2>&1
done
echo ab-done
cd /tmp
export TMPDIR=/tmp
KV_PREC=i8r4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/ab_forward.py pr 2048 > $O/prof.log 2>&1
echo prof-done
