#!/bin/bash
# round 6: phase timing of the fp32 tower's held-V output kernel (tools/out_phases.py) on 2,048 boards, plain and
# residual, 4- and 3-digit
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r06_phases
mkdir -p $O
export PYTHONUNBUFFERED=1
for a in "0 0" "1 0" "0 1"; do
    timeout -k 10 120 python -u tools/out_phases.py 2048 $a > $O/phases_$(echo $a | tr ' ' _).json 2>&1
done
cat $O/phases_0_0.json
