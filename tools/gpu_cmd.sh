cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
PYTEST_ARGS='-x' bash tools/gpu_round.sh test || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --steps 100 --no-cpu-baseline --no-trainer-loop > $GRAFT_REPO_ROOT/$O/prof5.log 2>&1
