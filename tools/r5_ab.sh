#!/bin/bash
# same-box A/B of bench variants: each "name|args" runs bench.py config ${CONFIG:-2}
# (scenes cached) and prints value / ms per step / kernel ms; then kernel stats
set -u
mkdir -p gpurun_out/ab
CACHE=/tmp/cbev_scene_cache
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python -u bench.py --config ${CONFIG:-2} --scene-cache $CACHE --no-cpu-baseline --fresh-workers 0 $args > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { echo "$name failed"; tail -5 gpurun_out/ab/$name.err; exit 1; }
  python - $name <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab/{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], d["ms_per_step_min_max"], d["kernel_ms"], d["raster_ms_per_launch"])
PY
done
