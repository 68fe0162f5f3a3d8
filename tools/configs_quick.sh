#!/bin/bash
# quick bench lines for configs ${CFGS:-3 4 5} (no CPU baseline, no wire pass)
set -u
mkdir -p gpurun_out
for c in ${CFGS:-3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-100} --no-cpu-baseline --no-wire ${EXTRA:-} > gpurun_out/cfg$c.json 2> gpurun_out/cfg$c.err || { echo "config $c failed"; tail -5 gpurun_out/cfg$c.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/cfg$c.json').read().strip().splitlines()[-1]); print('config $c', d['value'], d['ms_per_step'], d['kernel_ms'], d['raster_ms_per_launch'])
"
done
