#!/bin/bash
# The driver's GPU checks on this tree: the whole -m gpu suite, then smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${1:-suite}.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/${1:-suite}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${1:-suite}_smoke.log 2>&1
