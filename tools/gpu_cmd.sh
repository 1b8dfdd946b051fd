set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
PYTEST_ARGS='-x' bash tools/gpu_round.sh test
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python bench.py --config 3 --cpu-seconds 15 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 400 python bench.py --config 5 --cpu-seconds 15 --steps 100 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 400 python bench.py --config 2 --networks model2 --no-cpu-baseline > $O/bench_m2.json 2> $O/bench_m2.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-trainer-loop > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/rocprof_kgemm.py $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv > $GRAFT_REPO_ROOT/$O/prof_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 100 --no-cpu-baseline --no-trainer-loop > $GRAFT_REPO_ROOT/$O/prof3.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/rocprof_kgemm.py $GRAFT_REPO_ROOT/$O/prof3/run_kernel_stats.csv > $GRAFT_REPO_ROOT/$O/prof3_summary.txt
