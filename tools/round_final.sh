#!/bin/bash
# Milestone GPU pass: tools/round_check.sh (GPU tests, default bench line, rocprofv3
# passes), then the bench lines of configs 3-5 at N=1.
set -u
bash tools/round_check.sh || exit 1
for c in 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_config$c.json 2> gpurun_out/bench_config$c.err || { echo "config $c failed"; tail -5 gpurun_out/bench_config$c.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_config$c.json').read().strip().splitlines()[-1]); print($c, d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
