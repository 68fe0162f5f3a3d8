"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats copy),
profiles/<tag>_pmc.json (per-kernel mean of every collected counter) and
profiles/pmc_raster_config<cfg>.json, the per-launch HBM traffic of k_raster
that bench.py reports as roofline.traffic: (2 * FETCH_SIZE + WRITE_SIZE) KiB,
FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B read
requests at 64 B).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("--src", default="gpurun_out/prof")
ap.add_argument("--tag", default="round1")
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--out", default="profiles")
a = ap.parse_args()

os.makedirs(a.out, exist_ok=True)
stats = os.path.join(a.src, "trace", "trace_kernel_stats.csv")
shutil.copy(stats, f"{a.out}/{a.tag}_kernel_stats.csv")
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.src, "pmc_*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        pmc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in pmc.items() if k.startswith("k_")}
dur = {}
for r in csv.DictReader(open(stats)):
    name = r["Name"].split("(")[0].replace("void ", "")
    if name.startswith("k_"):
        dur[name] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
json.dump({"kernel_trace": dur, "pmc_mean_per_dispatch": summary}, open(f"{a.out}/{a.tag}_pmc.json", "w"),
          indent=1, sort_keys=True)
rk = next(k for k in summary if k.startswith("k_raster"))
fetch_kb, write_kb = summary[rk]["FETCH_SIZE"], summary[rk]["WRITE_SIZE"]
out = {"kernel": rk, "config": a.config, "envs": a.envs, "fetch_kb": fetch_kb, "write_kb": write_kb,
       "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
       "avg_ns": dur.get(rk, {}).get("avg_ns"), "source": f"{a.tag} rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes"}
json.dump(out, open(f"{a.out}/pmc_raster_config{a.config}.json", "w"), indent=1)
print(json.dumps(out))
