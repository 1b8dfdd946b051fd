cd $GRAFT_REPO_ROOT
PYTEST_ARGS='-k "rng_seed or graph_and_eager"' bash tools/gpu_round.sh test
