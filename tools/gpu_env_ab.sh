#!/bin/bash
# HIP runtime knobs A/B on the config-2 line: ENVS is a list of "NAME=VALUE" (or "default"),
# REPS rounds, alternating.  usage: ENVS="default HIP_FORCE_DEV_KERNARG=1" TAG=r6i bash tools/gpu_env_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envab}
mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for e in ${ENVS:-default}; do
    n=$(echo $e | tr '=' '_')
    if [ "$e" = default ]; then e=""; fi
    timeout -k 10 200 env $e python3 bench.py --no-trainer-loop --no-cpu-baseline --config ${CONFIG:-2} \
      > $O/${n}_$r.json 2> $O/${n}_$r.err || { tail $O/${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${n}_$r.json')); r=d.get('roofline') or {}
print('$n', d['value'], d['ms_per_step'], r.get('frac'))"
  done
done
