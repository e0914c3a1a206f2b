#!/bin/bash
# round 6: the rest of the GPU suite after r06_r3val's stop (test_nn_gpu onward, R3 in the matrices), then the
# persistent output kernel A/B (tools/runs/r06_outp_ab.sh)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r06_suite2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_shard_gpu.py tests/test_train_gpu.py tests/test_train_ops_gpu.py tests/test_wino_i8_gpu.py \
    > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
bash tools/runs/r06_outp_ab.sh r06_outp
