set -u
mkdir -p gpurun_out/rr
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "reset or surface or bank" --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-2 5}; do for so in tools/micro/so/*.so; do
  n=$(basename $so .so)_$cfg
  CBEV_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rr/$n -o $n --output-format csv -- python bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline --no-wire > gpurun_out/rr/$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/rr/$n.log; exit 1; }
  python - "$n" <<'PY'
import csv, glob, sys, json
n = sys.argv[1]
f = glob.glob(f"gpurun_out/rr/{n}/**/*kernel_stats.csv", recursive=True)[0]
d = {r["Name"].split("(")[0].replace("void ", ""): round(float(r["AverageNs"]) / 1000, 2) for r in csv.DictReader(open(f)) if "k_" in r["Name"][:12]}
v = json.loads([l for l in open(f"gpurun_out/rr/{n}.log") if l.startswith("{\"metric")][-1])
print(n, v["value"], v["ms_per_step"], d)
PY
done; done
