#!/bin/bash
# round 5: fp32 even / odd transforms, second A/B: the headline tower only, 4 alternating repeats, plus the accuracy
# table (AUTO's calibration errors on bn / peaked / stress) with the new chains
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r05_eo32b}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
: > $O/ab.log
for rep in 1 2 3 4; do
    KV_ALGO=winograd88i8 KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 200 python -u tools/ab_forward.py old 2048 256 >> $O/ab.log 2>&1
    KV_ALGO=winograd88i8 timeout -k 10 200 python -u tools/ab_forward.py new 2048 256 >> $O/ab.log 2>&1
done
echo ab-done
timeout -k 10 400 python -u -m pytest tests/test_nn_accuracy_gpu.py -k "auto_within" -x -v -s --timeout 200 --timeout-method thread > $O/acc_new.log 2>&1
KV_LIB_PATH=$R/knightvision_amd/libkv_b.so timeout -k 10 400 python -u -m pytest tests/test_nn_accuracy_gpu.py -k "auto_within" -x -v -s --timeout 200 --timeout-method thread > $O/acc_old.log 2>&1
echo acc-done
