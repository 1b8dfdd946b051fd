cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-k "b4096 or bf16"' bash tools/gpu_round.sh test
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --no-trainer-loop --steps 100 > $O/c3.json 2> $O/c3.err
true
