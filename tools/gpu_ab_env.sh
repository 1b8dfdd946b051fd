#!/bin/bash
# A/B of one environment switch on one box: bench lines alternating without / with it.
#   AB_ENV="SACMI_NO_DH16=1" BENCH_ARGS="--config 5 --no-trainer-loop --no-cpu-baseline" bash tools/gpu_ab_env.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 bench.py ${BENCH_ARGS} > $O/a$r.json 2> $O/a$r.err || exit 1
  timeout -k 10 300 env ${AB_ENV} python3 bench.py ${BENCH_ARGS} > $O/b$r.json 2> $O/b$r.err || exit 1
done
for f in $O/a1.json $O/b1.json $O/a2.json $O/b2.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['sites_us'] if d.get('roofline') else '')"
done
