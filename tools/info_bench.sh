#!/bin/bash
# bench lines in info_mode none and full (config ${CFG:-2}), each under its own limit
set -u
mkdir -p gpurun_out
for m in none full; do
  timeout -k 10 300 python -u bench.py --config ${CFG:-2} --info-mode $m --no-cpu-baseline --no-wire > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || { echo "bench $m failed"; tail -5 gpurun_out/bench_$m.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/bench_$m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['kernel_ms'])
"
done
