#!/bin/bash
# A/B pass on one GPU box: the GPU tests, then bench lines with and without an env setting
# (TOGGLE="NAME=value").
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-5}; do
  timeout -k 10 300 python3 bench.py --config $c --no-trainer-loop --no-cpu-baseline > $O/b_c${c}_new.json 2> $O/b_c${c}_new.err || { tail $O/b_c${c}_new.err; exit 1; }
  if [ -n "${TOGGLE:-}" ]; then
    env $TOGGLE timeout -k 10 300 python3 bench.py --config $c --no-trainer-loop --no-cpu-baseline > $O/b_c${c}_old.json 2> $O/b_c${c}_old.err || { tail $O/b_c${c}_old.err; exit 1; }
  fi
done
for f in $O/b_c*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"; done
