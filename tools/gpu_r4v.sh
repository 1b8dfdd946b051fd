#!/bin/bash
# round 4 final verification on the last GPU-verified kernel sources (e70f1db; the heads
# fold of r4s is parked on branch heads-fold-wip after an illegal-address fault in that run):
# GPU tests, smoke, the driver's bench command (trainer loops + CPU baseline), configs 3 / 5
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4v}
mkdir -p $O
SACMI_GRAD_TABLE=$PWD/$O/grad_table.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_driver.json 2> $O/b_driver.err || { tail $O/b_driver.err; exit 1; }
cut -c1-400 $O/b_driver.json
timeout -k 10 400 python3 bench.py --config 3 --no-trainer-loop > $O/b_c3.json 2> $O/b_c3.err || { tail $O/b_c3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config 5 --no-trainer-loop > $O/b_c5.json 2> $O/b_c5.err || { tail $O/b_c5.err; exit 1; }
cut -c1-200 $O/b_c3.json $O/b_c5.json
