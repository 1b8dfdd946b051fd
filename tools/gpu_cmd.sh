cd $GRAFT_REPO_ROOT
PYTEST_ARGS='-k "many_updates"' bash tools/gpu_round.sh test
