cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python3 bench.py --config 5 > $O/b_c5.json 2> $O/b_c5.err || exit 1
