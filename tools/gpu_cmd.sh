set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
bash tools/gpu_round.sh test
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 100 > $O/tl.json 2> $O/tl.err
