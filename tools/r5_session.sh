#!/bin/bash
# Round-5 combined GPU session: raster A/B of library builds (configs in
# ${AB_CONFIGS:-5 2}), then bench A/B of env-var variants at config 2
# (${BENCH_VARIANTS}), then the -m gpu suite unless SKIP_TESTS is set.
# Every GPU step has its own limit; the first failure ends the call.
set -u
mkdir -p gpurun_out/r5s
export TMPDIR=/tmp
CACHE=/tmp/cbev_scene_cache
for c in ${AB_CONFIGS:-5 2}; do
  timeout -k 10 300 python -u tools/micro/raster_ab.py --config $c --libs ${AB_LIBS} > gpurun_out/r5s/ab_c$c.txt 2>&1 || { echo "ab $c failed"; tail -5 gpurun_out/r5s/ab_c$c.txt; exit 1; }
  tail -4 gpurun_out/r5s/ab_c$c.txt
done
for spec in ${BENCH_VARIANTS:-}; do
  name=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 300 env ${envs//,/ } python -u bench.py --config 2 --scene-cache $CACHE --no-cpu-baseline --fresh-workers 0 > gpurun_out/r5s/bench_$name.json 2> gpurun_out/r5s/bench_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/r5s/bench_$name.err; exit 1; }
  python - $name <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r5s/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], d["ms_per_step_min_max"], d["kernel_ms"], d["raster_ms_per_launch"])
PY
done
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r5s/pytest_gpu.txt 2>&1
  rc=$?
  tail -n 30 gpurun_out/r5s/pytest_gpu.txt
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
echo done
