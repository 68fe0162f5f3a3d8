#!/bin/bash
# One config's measurement set (config ${CFG}): bench line with the CPU baseline,
# then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes over a short run.
# Scenes are built once and cached in /tmp on the box.
set -u
: "${CFG:?set CFG}"
mkdir -p gpurun_out
CACHE=/tmp/cbev_scene_cache
timeout -k 10 600 python -u bench.py --config $CFG --scene-cache $CACHE ${BENCH_EXTRA:-} > gpurun_out/bench_cfg$CFG.json 2> gpurun_out/bench_cfg$CFG.err || { echo "bench failed"; tail -5 gpurun_out/bench_cfg$CFG.err; exit 1; }
tail -1 gpurun_out/bench_cfg$CFG.json
OUT=gpurun_out/prof$CFG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--config $CFG --steps 30 --warmup 3 --no-cpu-baseline --no-wire --fresh-workers 0 --surface-steps 0 --raster-reps 5 --scene-cache $CACHE"
run() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run trace --kernel-trace --stats
run pmc_fetch --kernel-trace --pmc FETCH_SIZE
run pmc_write --kernel-trace --pmc WRITE_SIZE
# summaries only (the raw traces exceed what gpurun copies back)
ENVS=$(python -c "import json; print(json.loads(open('gpurun_out/bench_cfg$CFG.json').read().strip().splitlines()[-1])['config']['envs_per_gpu'])")
python tools/summarize_profile.py --src $OUT --tag ${TAG:-round3}_config$CFG --config $CFG --envs $ENVS --out gpurun_out/psum || exit 1
rm -rf $OUT
exit 0
