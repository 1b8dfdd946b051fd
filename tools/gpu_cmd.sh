cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-x' bash tools/gpu_round.sh test || exit 1
timeout -k 10 300 python3 bench.py --steps 100 --no-cpu-baseline --no-roofline > $O/v_z1.json 2>$O/v_z1.err || exit 1
