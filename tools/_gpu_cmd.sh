cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 python -m pytest tests/test_nn_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/t.log 2>&1 && \
timeout -k 10 120 python tools/nn_speed.py 16 256 1024 > gpurun_out/speed.log 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/stemprof -o p -- python3 $GRAFT_REPO_ROOT/tools/nn_speed.py 256 > /dev/null 2>&1
