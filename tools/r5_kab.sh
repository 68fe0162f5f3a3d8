#!/bin/bash
# same-box kernel A/B: for each library in ${LIBS}, a rocprofv3 kernel-stats pass
# of bench.py --config ${CONFIG:-2} (scenes cached), k_* averages printed
set -u
mkdir -p gpurun_out/kab
export TMPDIR=/tmp
CACHE=/tmp/cbev_scene_cache
i=0
for lib in ${LIBS}; do
  i=$((i+1))
  CBEV_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kab/p$i -o run --output-format csv -- python bench.py --config ${CONFIG:-2} --steps 50 --warmup 10 --no-cpu-baseline --no-wire --surface-steps 0 --fresh-workers 0 --scene-cache $CACHE > gpurun_out/kab/p$i.log 2>&1 || { echo "prof $lib failed"; tail -5 gpurun_out/kab/p$i.log; exit 1; }
  f=$(find gpurun_out/kab/p$i -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kab/kstats_$i.csv
  python - "$f" "$lib" <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0].replace("void ", ""): r for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], "  ".join(f"{k} {float(r['AverageNs'])/1000:.2f}us x{r['Calls']}" for k, r in rows.items() if k.startswith("k_")))
PY
  rm -rf gpurun_out/kab/p$i
done
