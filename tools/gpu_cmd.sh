cd $GRAFT_REPO_ROOT
O=gpurun_out
PYTEST_ARGS='-k "act or dropin or select"' bash tools/gpu_round.sh test || exit 1
for z in 1 0; do
  SACMI_ACT_ZEROCOPY=$z timeout -k 10 300 python3 bench.py --steps 100 --no-cpu-baseline --no-roofline > $O/v_z$z.json 2>$O/v_z$z.err || exit 1
done
