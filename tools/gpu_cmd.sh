set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python bench.py --config 5 --steps 100 --warmup 20 --cpu-seconds 10 > $O/c5_bf16.json 2> $O/c5.err
timeout -k 10 300 python bench.py --config 5 --dtype fp32 --steps 100 --warmup 20 --no-cpu-baseline > $O/c5_fp32.json 2>> $O/c5.err
timeout -k 10 300 python bench.py --config 2 --networks model2 --no-cpu-baseline > $O/c2_m2.json 2>> $O/c5.err
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.json 2>> $O/c5.err
timeout -k 10 300 python bench.py --config 2 --dtype bf16 --no-cpu-baseline > $O/c2_bf16.json 2>> $O/c5.err
