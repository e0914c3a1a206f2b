#!/bin/bash
# round 6: the N>1 bench path rehearsed on the final code (R3 path) with gloo ranks sharing the 1-GPU box (RCCL refuses
# two ranks on one device): 2 and 8 ranks, each the full C3 / C4 per-rank workload (2,048 slots x 800 sims),
# the R3 tower, the (s, pi, z) gather to rank 0 and every rank's calibration in the line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_multi}
mkdir -p $O
export PYTHONUNBUFFERED=1 KV_BENCH_BACKEND=gloo
X="--alt-precision= --alt-algo= --ref-block 0 --trained-steps 0 --no-cpu-baseline"
timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 $X > $O/gloo2.log 2> $O/gloo2.err
timeout -k 10 700 python -u bench.py --gpus 8 --steps 1 --warmup 1 $X > $O/gloo8.log 2> $O/gloo8.err
echo multi-done
