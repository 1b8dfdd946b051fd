#!/bin/bash
# round 4: the fused-Adam levels' scalar work at the level's start (adam_wg -2) — GPU tests,
# A/B against block 0 after its tile (SACMI_B0_LATE=1), phase stamps with the slowest WGs
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
A="--config ${CONFIG:-2} --no-trainer-loop --no-cpu-baseline --steps 40 --warmup 10"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/b_new$r.json 2> $O/b_new$r.err || exit 1
  SACMI_B0_LATE=1 timeout -k 10 200 python3 bench.py $A > $O/b_old$r.json 2> $O/b_old$r.err || exit 1
done
for f in $O/b_*.json; do python3 -c "
import json; d=json.load(open('$f')); s=d['roofline'].get('sites_us',{})
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], {k[:8]:round(v,2) for k,v in s.items() if 'L6' in k or 'L13' in k})"; done
TAG=${TAG:-r4q} SLOW=3 LIB=phases bash tools/gpu_phases.sh > /dev/null || exit 1
grep -A14 "^site" $O/phases_c${CONFIG:-2}.txt; grep "slow gemm_L6\|slow gemm_L13" $O/phases_c${CONFIG:-2}.txt
