cd $GRAFT_REPO_ROOT
O=gpurun_out
L=$PWD/humanoid-walking-with-sac_amd/sacmi
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-trainer-loop --steps 100 > $O/c5_base.json 2> $O/c5.err
SACMI_LIB_PATH=$L/libsacmi_all64.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-trainer-loop --steps 100 > $O/c5_all64.json 2> $O/c5b.err
true
