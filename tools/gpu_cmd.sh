set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python bench.py --force-dp > $O/dp_torch.json 2> $O/dp_torch.err
timeout -k 10 300 python bench.py --force-dp --dp-native > $O/dp_native.json 2> $O/dp_native.err
timeout -k 10 300 python bench.py --force-dp --dp-native --config 3 --steps 100 > $O/dp_native_c3.json 2> $O/dp_native_c3.err
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-trainer-loop --no-roofline > $O/single.json 2> $O/single.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --warmup 10 > $O/trun.json 2> $O/trun.err
