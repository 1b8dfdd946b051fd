cd $GRAFT_REPO_ROOT
PYTEST_ARGS='-k "shadows"' bash tools/gpu_round.sh test
