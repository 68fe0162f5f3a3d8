#!/bin/bash
# One GPU session: smoke -> gpu parity tests -> short bench. Each step has its
# own time limit; a crash/abort/timeout (anything but pass/fail) ends the run.
set -u
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step smoke 400 python __graft_entry__.py smoke
step pytest_gpu 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-}
step bench 500 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10}
exit 0
