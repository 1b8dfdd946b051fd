cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
PYTEST_ARGS='-k "bf16"' bash tools/gpu_round.sh test || exit 1
for c in 2 3 5; do
  PMC_ARGS="--config $c --steps 100 --warmup 20 --fill 200000 --no-cpu-baseline --no-roofline --no-trainer-loop" bash tools/gpu_pmc.sh > $O/pmc_run_c$c.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O $O/pmc_c$c.json > $O/pmc_c$c.txt || exit 1
done
