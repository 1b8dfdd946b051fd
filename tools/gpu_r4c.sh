#!/bin/bash
# staged-core check: GPU tests, then config-2 bench A/B (staged vs SACMI_NO_STAGED)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4c}
mkdir -p $O
SACMI_GRAD_TABLE=$PWD/$O/grad_table.jsonl SACMI_STAGED=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  SACMI_STAGED=1 timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline > $O/b_stg$i.json 2> $O/b_stg$i.err || { tail $O/b_stg$i.err; exit 1; }
  SACMI_NO_STAGED=1 timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline > $O/b_old$i.json 2> $O/b_old$i.err || { tail $O/b_old$i.err; exit 1; }
done
for f in $O/b_*.json; do echo $f; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"; done
