#!/bin/bash
# round 6: the second batch of complete C3-settings MCTS games (game ids 256..383) on the headline's AUTO path;
# merged with ids 0..255 (profiles/r06_gamelen_batch_ids0-255.json) by tools/mcts_game_length.py --merge
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r06_gamelen
export PYTHONUNBUFFERED=1
timeout -k 10 1130 python -u tools/mcts_game_length.py --games 128 --first 256 --seconds 1080 \
    --out gpurun_out/r06_gamelen/r06_gamelen_batch_ids256-383.json > gpurun_out/r06_gamelen/run2.log 2>&1
tail -c 400 gpurun_out/r06_gamelen/run2.log
