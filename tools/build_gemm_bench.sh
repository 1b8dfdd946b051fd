#!/bin/bash
# GEMM microbenchmark: timing build and the diagnostic stamp build
set -e
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 --offload-arch=gfx950 -Ihumanoid-walking-with-sac_amd/csrc -Iinclude"
/opt/rocm/bin/hipcc $F tools/gemm_bench.hip -o tools/gemm_bench
/opt/rocm/bin/hipcc $F -DSACMI_DIAG_STAMPS tools/gemm_bench.hip -o tools/gemm_stamps
