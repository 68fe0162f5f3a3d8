#!/bin/bash
# A/B pass: bench values by info mode (config ${INFO_CFG:-2}, skip with NO_INFO=1), then
# rocprofv3 kernel averages of libcbev variants per config: AB_<cfg>="so so ..."
set -u
mkdir -p gpurun_out/ab
CACHE=/tmp/cbev_scene_cache
if [ -z "${NO_INFO:-}" ]; then
  for mode in none full; do
    timeout -k 10 300 python -u bench.py --config ${INFO_CFG:-2} --no-cpu-baseline --no-wire --fresh-workers 0 --info-mode $mode --scene-cache $CACHE > gpurun_out/ab/info_$mode.json 2> gpurun_out/ab/info_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/ab/info_$mode.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab/info_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['ms_per_step_min_max'], d['kernel_ms'], d['host_enqueue_ms_per_step'])"
  done
fi
for c in 2 3 4 5; do
  v="AB_$c"; sos="${!v:-}"
  [ -z "$sos" ] && continue
  echo "== config $c"
  BENCH_ARGS="--config $c --scene-cache $CACHE" bash tools/micro/kernel_ab.sh $sos || exit 1
done
