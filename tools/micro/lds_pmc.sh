# LDS counters of k_raster for each tools/micro/so variant (config 2)
set -u
mkdir -p gpurun_out/lp
export TMPDIR=/tmp
for so in tools/micro/so/*.so; do
  n=$(basename $so .so)
  CBEV_LIB=$so timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU -d gpurun_out/lp/$n -o $n --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-wire > gpurun_out/lp/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/lp/$n.log; exit 1; }
  python - "$n" <<'PY'
import csv, glob, sys, collections
n = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/lp/{n}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void k_raster"):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(n, {k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
done
