#!/bin/bash
# round 4: operand-shape experiment for config 2 — delivery rates incl. the dword MN form;
# bench A/B of the contiguous-read timing build (SACMI_EXP_LINFETCH: wrong values, timing
# only) against the product build; phase stamps of both.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4l
mkdir -p $O
L=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi
timeout -k 10 60 tools/l2_rate_bench > $O/l2rate3.txt 2>&1 || exit 1
A="--config 2 --no-trainer-loop --no-cpu-baseline --steps 40 --warmup 10"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/b_base$r.json 2> $O/b_base$r.err || exit 1
  SACMI_LIB_PATH=$L/libsacmi_linfetch.so timeout -k 10 200 python3 bench.py $A > $O/b_lin$r.json 2> $O/b_lin$r.err || exit 1
done
TAG=r4l LIB=phases bash tools/gpu_phases.sh > /dev/null || exit 1
mv $O/phases_c2.txt $O/phases_base_c2.txt
TAG=r4l LIB=linfetch_ph bash tools/gpu_phases.sh > /dev/null || exit 1
mv $O/phases_c2.txt $O/phases_lin_c2.txt
for f in $O/b_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
