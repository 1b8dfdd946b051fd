#!/bin/bash
# round 4: SACMI_PIN_EPI 0/1 A/B on the current sources (libsacmi_pin0), config 3 / 5 lines
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4r}
mkdir -p $O
L=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi
A="--config 2 --no-trainer-loop --no-cpu-baseline --steps 40 --warmup 10"
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py $A > $O/b_pin1_$r.json 2> $O/b_pin1_$r.err || exit 1
  SACMI_LIB_PATH=$L/libsacmi_pin0.so timeout -k 10 200 python3 bench.py $A > $O/b_pin0_$r.json 2> $O/b_pin0_$r.err || exit 1
done
timeout -k 10 300 python3 bench.py --config 3 --no-trainer-loop --no-cpu-baseline > $O/b_c3.json 2> $O/b_c3.err || exit 1
timeout -k 10 300 python3 bench.py --config 5 --no-trainer-loop --no-cpu-baseline > $O/b_c5.json 2> $O/b_c5.err || exit 1
for f in $O/b_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
