#!/bin/bash
# round 4: k_gemm scalar round trips (desc + level-wide epilogue scalars in the desc's trip)
# A/B against the previous pinning (libsacmi_pin0: -DSACMI_PIN_EPI=0); phase stamps.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
L=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi
A="--config ${CONFIG:-2} --no-trainer-loop --no-cpu-baseline --steps 40 --warmup 10"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/b_new$r.json 2> $O/b_new$r.err || exit 1
  SACMI_LIB_PATH=$L/libsacmi_${BASE:-pin0}.so timeout -k 10 200 python3 bench.py $A > $O/b_old$r.json 2> $O/b_old$r.err || exit 1
done
for f in $O/b_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
if [ -n "${PHASES:-1}" ]; then
  TAG=${TAG:-r4m} LIB=phases bash tools/gpu_phases.sh > /dev/null || exit 1
  grep -A14 "^site" $O/phases_c${CONFIG:-2}.txt
fi
