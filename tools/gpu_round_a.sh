#!/bin/bash
# GPU check after a kernel change: the parity tests named by PYTEST_K (all by
# default), quick bench lines for CFGS, then a rocprofv3 kernel trace of config
# ${PROF_CFG:-3} (summary copied to gpurun_out/k${PROF_CFG}_stats.csv).
set -u
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
CFGS="${CFGS:-2 3 4}" bash tools/configs_quick.sh || exit 1
c=${PROF_CFG:-3}
export TMPDIR=/tmp
rm -rf gpurun_out/prof_k$c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k$c -o run --output-format csv -- python bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-wire --fresh-workers 0 > gpurun_out/prof_k$c.txt 2>&1 || exit 1
cp "$(find gpurun_out/prof_k$c -name '*kernel_stats.csv' | head -1)" gpurun_out/k${c}_stats.csv
