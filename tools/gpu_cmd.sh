set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/perprof -o run -- python3 tools/per_probe.py > $O/perprof.log 2>&1
