#!/bin/bash
# k_actors occupancy A/B (configs 3, 4) over tools/micro/var2, then the GPU parity
# suite run against the variant library (CBEV_LIB) to check it bit-exact.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -20 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
BENCH_ARGS="--config 3" bash tools/micro/kernel_ab.sh tools/micro/var2/*.so || exit 1
BENCH_ARGS="--config 4" bash tools/micro/kernel_ab.sh tools/micro/var2/*.so || exit 1
CBEV_LIB=$PWD/tools/micro/var2/libcbev_awpe4.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_awpe4.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_awpe4.txt; exit $rc
