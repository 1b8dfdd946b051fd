#!/bin/bash
# one GPU session: tests, bench, kernel-trace profile.  Every GPU step is time-limited
# and chained: the script stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  eval "timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}" > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_rc=$rc" >> $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; cat $OUT/bench.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench.err; exit $rc; }
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py ${PROF_ARGS:-${BENCH_ARGS:-}} > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
  rc=$?; echo prof_rc=$rc; [ $rc -ne 0 ] && { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit $rc; }
  python3 $GRAFT_REPO_ROOT/tools/rocprof_kgemm.py $GRAFT_REPO_ROOT/$OUT/prof/run_kernel_stats.csv > $GRAFT_REPO_ROOT/$OUT/prof_summary.txt
  tail -3 $GRAFT_REPO_ROOT/$OUT/prof_summary.txt; tail -1 $GRAFT_REPO_ROOT/$OUT/prof.log | cut -c1-400
fi
