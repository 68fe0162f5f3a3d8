#!/bin/bash
# fused vs split step: smoke, GPU parity tests, bench both modes (config 2)
set -u
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python __graft_entry__.py smoke
step bench_fused 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-wire
CBEV_STEP_MODE=split step bench_split 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-wire
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
exit 0
