#!/bin/bash
# the three step modes, twice each, interleaved (config ${CFG:-2})
set -u
mkdir -p gpurun_out
for rep in 1 2; do
for m in fused split; do
  CBEV_STEP_MODE=$m timeout -k 10 200 python bench.py --config ${CFG:-2} --steps 200 --warmup 20 --no-cpu-baseline --no-wire > gpurun_out/m.json 2> gpurun_out/m.err || { echo "$m failed"; tail -5 gpurun_out/m.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
done
