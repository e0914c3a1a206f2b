#!/bin/bash
# The whole -m gpu suite, smoke(), then the C2 bench line (256 games x 400
# sims). Each step under its own time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03suite}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --slots 256 --sims 400 --steps 10 --warmup 3 --alt-precision= --alt-algo= --ref-block 0 --no-cpu-baseline > $O/c2.log 2>&1
echo suite-done
