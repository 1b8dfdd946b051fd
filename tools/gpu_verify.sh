#!/bin/bash
# Verification pass on one GPU box: GPU tests, smoke, the driver's bench command and the
# config-3 / config-5 lines.  Every GPU step has its own time limit; the first failure ends it.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-v}
mkdir -p $O
eval "timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_driver.json 2> $O/b_driver.err || { tail $O/b_driver.err; exit 1; }
cat $O/b_driver.json | cut -c1-600
[ -n "${SKIP_CONFIGS:-}" ] && exit 0
timeout -k 10 400 python3 bench.py --config 3 --no-trainer-loop > $O/b_c3.json 2> $O/b_c3.err || { tail $O/b_c3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config 5 --no-trainer-loop > $O/b_c5.json 2> $O/b_c5.err || { tail $O/b_c5.err; exit 1; }
cut -c1-300 $O/b_c3.json $O/b_c5.json
