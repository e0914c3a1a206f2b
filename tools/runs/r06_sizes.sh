#!/bin/bash
# round 6: forward time per board of the R3 tower by batch size (is a C3 batch faster as slices that keep M in the
# 256 MiB Infinity Cache?), then the second game-length batch
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r06_sizes
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
for rep in 1 2; do
    KV_ALGO=winograd88i8r3 timeout -k 10 200 python -u tools/ab_forward.py sz 256 512 768 1024 1536 2048 >> $O/ab.log 2>&1
done
grep -v amdgpu $O/ab.log
bash tools/runs/r06_gamelen2.sh
