# rocprofv3 kernel averages of the default bench run for each libcbev variant given
set -u
mkdir -p gpurun_out/kab
export TMPDIR=/tmp
for so in "$@"; do
  n=$(basename $so .so)
  CBEV_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kab/$n -o run --output-format csv -- python bench.py ${BENCH_ARGS:-} --steps 50 --warmup 10 --no-cpu-baseline --no-wire --fresh-workers 0 > gpurun_out/kab/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/kab/$n.log; exit 1; }
  f=$(find gpurun_out/kab/$n -name "*kernel_stats.csv" | head -1)
  python - "$f" "$n" <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0].replace("void ", ""): r for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], "  ".join(f"{k} {float(r['AverageNs'])/1000:.2f}us x{r['Calls']}" for k, r in rows.items() if k.startswith("k_")))
PY
  rm -rf gpurun_out/kab/$n
done
