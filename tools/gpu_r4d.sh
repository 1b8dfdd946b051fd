#!/bin/bash
# round 4: GPU tests with the staged core, config-2 A/B, config 3 / 5 lines, DP sequence at
# a simulated world of 8 (per-rank work minus collectives) in both optimizer forms
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4d}
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
SACMI_GRAD_TABLE=$PWD/$O/grad_table.jsonl SACMI_STAGED=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
B="timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline"
for i in 1 2; do
  SACMI_STAGED=1 $B > $O/b_stg$i.json 2> $O/b_stg$i.err || { tail $O/b_stg$i.err; exit 1; }
  SACMI_NO_STAGED=1 $B > $O/b_old$i.json 2> $O/b_old$i.err || { tail $O/b_old$i.err; exit 1; }
done
SACMI_STAGED=1 $B --config 3 > $O/b_c3.json 2> $O/b_c3.err || { tail $O/b_c3.err; exit 1; }
SACMI_STAGED=1 $B --config 5 > $O/b_c5.json 2> $O/b_c5.err || { tail $O/b_c5.err; exit 1; }
SACMI_STAGED=1 SACMI_DP_SHARD=1 SACMI_DP_LOOPBACK_ONE_RANK=1 $B --force-dp --dp-sim-world 8 --steps 20 > $O/dp8_shard.json 2> $O/dp8_shard.err || { tail $O/dp8_shard.err; exit 1; }
SACMI_STAGED=1 SACMI_DP_SHARD=0 $B --force-dp --dp-sim-world 8 --steps 20 > $O/dp8_ar.json 2> $O/dp8_ar.err || { tail $O/dp8_ar.err; exit 1; }
for f in $O/b_*.json $O/dp8_*.json; do echo $f; python3 -c "import json; d=json.load(open('$f')); r=d.get('roofline') or {}; print(d['value'], d['ms_per_step'], r.get('frac'), r.get('step_us_timeline'))"; done
