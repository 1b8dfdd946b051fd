set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
for v in base t64 t65 t66; do
  if [ $v = base ]; then L=""; else L=$PWD/humanoid-walking-with-sac_amd/sacmi/libsacmi_$v.so; fi
  SACMI_LIB_PATH=$L timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --no-trainer-loop --steps 100 > $O/c3_$v.json 2> $O/c3_$v.err
done
