#!/bin/bash
# GPU pass (round 6): parity tests, then for each config in ${CONFIGS:-2 5} a bench
# line and a rocprofv3 kernel-stats pass (scenes cached in /tmp on the box).
# Every GPU step has its own limit; the first failure ends the call.
set -u
D=gpurun_out/${TAG:-r6}
mkdir -p $D
CACHE=/tmp/cbev_scene_cache
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-420} python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $D/pytest_gpu.txt 2>&1
  rc=$?
  tail -n 30 $D/pytest_gpu.txt
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
for c in ${CONFIGS:-2 5}; do
  timeout -k 10 ${BENCH_LIMIT:-300} python -u bench.py --config $c --scene-cache $CACHE ${BENCH_EXTRA:-} > $D/bench_c$c.json 2> $D/bench_c$c.err || { echo "bench $c failed"; tail -5 $D/bench_c$c.err; exit 1; }
  python - $D/bench_c$c.json $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["kernel_ms"], d["raster_ms_per_launch"], d["roofline"]["frac"],
      d["roofline"].get("write_floor_ratio"), d.get("info_mode"), d.get("bank_rows_handed_out"), d.get("resets_per_step"))
for k in ("surface_loop", "surface_loop_fresh"):
    if d.get(k):
        print(k, {x: d[k][x] for x in ("value", "ms_per_step", "resets_per_step", "scenes_built", "fresh_reset_frac")})
PY
  if [ -z "${SKIP_PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof$c -o run --output-format csv -- python bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-wire --fresh-workers 0 --surface-steps 0 --scene-cache $CACHE ${PROF_EXTRA:-} > $D/prof$c.log 2>&1 || { echo "prof $c failed"; tail -5 $D/prof$c.log; exit 1; }
    f=$(find $D/prof$c -name "*kernel_stats.csv" | head -1)
    cp "$f" $D/kstats_c$c.csv
    python - "$f" <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0].replace("void ", ""): r for r in csv.DictReader(open(sys.argv[1]))}
print("  ".join(f"{k} {float(r['AverageNs'])/1000:.2f}us x{r['Calls']}" for k, r in rows.items() if k.startswith("k_")))
PY
    rm -rf $D/prof$c
  fi
done
