#!/bin/bash
# round-4 first look: config-2 bench (baseline and a variant library), cache PMC passes
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "drawn_ahead or many_updates" --timeout 120 --timeout-method thread > $O/pytest_pf.log 2>&1 || { tail -30 $O/pytest_pf.log; exit 1; }
tail -2 $O/pytest_pf.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline > $O/b_base$i.json 2> $O/b_base$i.err || { tail $O/b_base$i.err; exit 1; }
  SACMI_LIB_PATH=$PWD/humanoid-walking-with-sac_amd/sacmi/libsacmi_kcontig.so timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline > $O/b_kc$i.json 2> $O/b_kc$i.err || { tail $O/b_kc$i.err; exit 1; }
done
for f in $O/b_*.json; do echo $f; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"; done
bash tools/gpu_pmc_cache.sh c2 --steps 20 --warmup 5 --profile-only --no-cpu-baseline --no-trainer-loop || exit 1
timeout -k 10 120 tools/cohort_bench 200 > $O/cohort.txt 2>&1; rc=$?; cat $O/cohort.txt; exit $rc
