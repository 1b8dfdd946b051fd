cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-k "sample or many_updates or ride or dp or golden"' bash tools/gpu_round.sh test || exit 1
timeout -k 10 200 python3 bench.py --config 5 --steps 200 --no-cpu-baseline --no-trainer-loop > $O/v_main.json 2>$O/v_main.err || exit 1
