set -u
mkdir -p gpurun_out/pm
export TMPDIR=/tmp
ARGS="--steps 30 --warmup 3 --no-cpu-baseline --no-wire --fresh-workers 0"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pm/tcc -o tcc --output-format csv -- python bench.py $ARGS > gpurun_out/pm/tcc.log 2>&1 || { tail -5 gpurun_out/pm/tcc.log; exit 1; }
f=$(find gpurun_out/pm/tcc -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    h = sum(d["TCC_HIT_sum"]) / max(len(d["TCC_HIT_sum"]), 1); m = sum(d["TCC_MISS_sum"]) / max(len(d["TCC_MISS_sum"]), 1)
    print(f"{k:32s} hit {h:12.0f} miss {m:12.0f} hit% {100*h/max(h+m,1):5.1f}")
PY
rm -rf gpurun_out/pm/tcc
