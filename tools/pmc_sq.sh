set -u
mkdir -p gpurun_out/pm
export TMPDIR=/tmp
run() {
  n=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pm/$n -o $n --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-wire --fresh-workers 0 > gpurun_out/pm/$n.log 2>&1 || { tail -3 gpurun_out/pm/$n.log; exit 1; }
  f=$(find gpurun_out/pm/$n -name "*counter_collection.csv" | head -1)
  python - "$f" <<'PY' >> gpurun_out/pm/sq_summary.jsonl
import csv, sys, collections, json
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if k.startswith("k_"): agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}))
PY
  rm -rf gpurun_out/pm/$n
}
rm -f gpurun_out/pm/sq_summary.jsonl
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
run sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS
run tcc TCC_HIT_sum TCC_MISS_sum
cat gpurun_out/pm/sq_summary.jsonl | python -c "
import sys, json
m = {}
for l in sys.stdin: 
    for k, d in json.loads(l).items(): m.setdefault(k, {}).update(d)
json.dump(m, open('gpurun_out/pm/round3_config2_sq.json', 'w'), indent=1, sort_keys=True)
print(json.dumps({k: {c: round(v) for c, v in d.items()} for k, d in m.items() if k.startswith('k_raster') or k == 'k_ego'}))
"
