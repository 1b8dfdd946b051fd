cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-x -k "per"' bash tools/gpu_round.sh test
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --no-trainer-loop --steps 100 > $O/c3.json 2> $O/c3.err
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/perprof -o run -- python3 tools/per_probe.py > $O/perprof.log 2>&1
true
