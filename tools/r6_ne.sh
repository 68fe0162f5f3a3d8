#!/bin/bash
# k_ego envs per workgroup (CBEV_EGO_NE) against the default, bench lines per config
set -u
D=gpurun_out/r6ne
mkdir -p $D
export TMPDIR=/tmp
CACHE=/tmp/cbev_scene_cache
for c in ${CONFIGS:-2 3}; do
  for ne in default ${NES:-4 8 16}; do
    if [ $ne = default ]; then unset CBEV_EGO_NE; else export CBEV_EGO_NE=$ne; fi
    timeout -k 10 300 python -u bench.py --config $c --scene-cache $CACHE --no-cpu-baseline --no-wire --surface-steps 0 --fresh-workers 0 > $D/b_${c}_$ne.json 2> $D/b_${c}_$ne.err || { echo "bench $c $ne failed"; tail -5 $D/b_${c}_$ne.err; exit 1; }
    python - $D/b_${c}_$ne.json $c $ne <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ne", sys.argv[3], d["value"], d["ms_per_step"], d.get("ms_per_step_min_max"), d["kernel_ms"])
PY
  done
done
unset CBEV_EGO_NE
