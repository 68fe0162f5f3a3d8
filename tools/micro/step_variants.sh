#!/bin/bash
# bench prebuilt libcbev variants (tools/micro/so/*.so) on configs ${CFGS:-2}, optionally phase stamps
set -u
mkdir -p gpurun_out
for cfg in ${CFGS:-2}; do
for so in tools/micro/so/*.so; do
  CBEV_LIB=$so timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline --no-wire > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$so failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/v.json').read().strip().splitlines()[-1]); print('cfg $cfg', '$so'.split('/')[-1], d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
done
if [ -n "${PHASES:-}" ]; then
timeout -k 10 300 python tools/micro/step_phases.py --config ${CFG:-2} > gpurun_out/step_phases.txt 2>&1 && grep -v "xcd \|XCC" gpurun_out/step_phases.txt
fi
