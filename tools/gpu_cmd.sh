cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
PYTEST_ARGS='' bash tools/gpu_round.sh test || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/b_c2.json 2> $O/b_c2.err || exit 1
timeout -k 10 400 python3 bench.py --config 3 > $O/b_c3.json 2> $O/b_c3.err || exit 1
timeout -k 10 400 python3 bench.py --config 5 > $O/b_c5.json 2> $O/b_c5.err || exit 1
timeout -k 10 400 python3 bench.py --networks model2 --no-cpu-baseline > $O/b_m2.json 2> $O/b_m2.err || exit 1
cd /tmp
for c in 2 3 5; do
  rm -rf $GRAFT_REPO_ROOT/$O/prof_c$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-trainer-loop > $GRAFT_REPO_ROOT/$O/prof_c$c.log 2>&1 || exit 1
done
