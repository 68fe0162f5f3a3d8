#!/bin/bash
# SQ / TCC counter passes over a short bench run of config ${CFG:-2}, one
# rocprofv3 --pmc pass per counter group (each under its own time limit);
# per-kernel means -> gpurun_out/pm/${TAG:-round4}_config${CFG}_sq.json.
set -u
CFG=${CFG:-2}
TAG=${TAG:-round4}
mkdir -p gpurun_out/pm
export TMPDIR=/tmp
CACHE=/tmp/cbev_scene_cache
run() {
  n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pm/$n -o $n --output-format csv -- python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-wire --fresh-workers 0 --surface-steps 0 --raster-reps 5 --scene-cache $CACHE > gpurun_out/pm/$n.log 2>&1 || { tail -3 gpurun_out/pm/$n.log; exit 1; }
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
python - "$TAG" "$CFG" <<'PY'
import sys, json
tag, cfg = sys.argv[1], sys.argv[2]
m = {}
for l in open("gpurun_out/pm/sq_summary.jsonl"):
    for k, d in json.loads(l).items():
        m.setdefault(k, {}).update(d)
json.dump(m, open(f"gpurun_out/pm/{tag}_config{cfg}_sq.json", "w"), indent=1, sort_keys=True)
print(json.dumps({k: {c: round(v) for c, v in d.items()} for k, d in m.items() if k.startswith("k_raster") or k == "k_ego"}))
PY
