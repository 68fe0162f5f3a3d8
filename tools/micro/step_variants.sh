#!/bin/bash
# bench prebuilt libcbev variants (tools/micro/so/*.so) on config ${CFG:-2}, then the phase stamps
set -u
mkdir -p gpurun_out
for so in tools/micro/so/*.so; do
  CBEV_LIB=$so timeout -k 10 200 python bench.py --config ${CFG:-2} --steps 100 --warmup 10 --no-cpu-baseline --no-wire > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$so failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/v.json').read().strip().splitlines()[-1]); print('$so', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
timeout -k 10 300 python tools/micro/step_phases.py --config ${CFG:-2} > gpurun_out/step_phases.txt 2>&1 && grep -v "xcd \|XCC" gpurun_out/step_phases.txt
