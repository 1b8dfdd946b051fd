cd $GRAFT_REPO_ROOT
O=gpurun_out
V=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi
PYTEST_ARGS='' bash tools/gpu_round.sh test || exit 1
for v in main ns; do
  if [ $v = main ]; then L=""; else L=$V/libsacmi_$v.so; fi
  SACMI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --config 5 --steps 200 --no-cpu-baseline --no-trainer-loop > $O/v_$v.json 2>$O/v_$v.err || exit 1
done
