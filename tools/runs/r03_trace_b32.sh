set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tr32; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
KV_ALGO=auto timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/a -o a -- python3 $R/tools/nn_speed.py 32 > $O/a.log 2>&1
KV_ALGO=winograd48 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/b -o b -- python3 $R/tools/nn_speed.py 32 > $O/b.log 2>&1
echo ok
