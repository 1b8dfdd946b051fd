set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-x -k "dropin or select or act"' bash tools/gpu_round.sh test
timeout -k 10 200 python tools/act_probe.py > $O/act.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/tl.json 2> $O/tl.err
