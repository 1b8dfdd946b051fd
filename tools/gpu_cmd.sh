cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-k "per"' bash tools/gpu_round.sh test || exit 1
timeout -k 10 200 python3 bench.py --config 3 --steps 100 --no-cpu-baseline --no-trainer-loop > $O/v_c3.json 2>$O/v_c3.err || exit 1
