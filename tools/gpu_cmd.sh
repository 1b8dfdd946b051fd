set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
bash tools/gpu_pmc.sh
python3 tools/pmc_summary.py $O $O/pmc_c2.json > $O/pmc_c2.txt
PMC_ARGS="--config 3 --steps 40 --warmup 10 --fill 200000 --no-cpu-baseline --no-roofline --no-trainer-loop" bash tools/gpu_pmc.sh
python3 tools/pmc_summary.py $O $O/pmc_c3.json > $O/pmc_c3.txt
