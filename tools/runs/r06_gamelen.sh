#!/bin/bash
# round 6: complete MCTS games at C3's settings on the path the headline runs (AUTO on random-init weights: the fp32
# tower on 3 radix-256 int8 digits), game ids 0..255 -- the steady-state games/hour sample bench.py reads
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r06_gamelen
export PYTHONUNBUFFERED=1
timeout -k 10 1130 python -u tools/mcts_game_length.py --games 256 --seconds 1080 \
    --out gpurun_out/r06_gamelen/r06_mcts_game_length_c3_i8f32r3.json > gpurun_out/r06_gamelen/run.log 2>&1
tail -c 600 gpurun_out/r06_gamelen/run.log
