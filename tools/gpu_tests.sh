#!/bin/bash
# GPU parity tests (+ optional short bench): each step under its own limit; a
# crash, abort or timeout ends the call.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
tail -n 40 gpurun_out/pytest_gpu.txt
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 300 python -u bench.py $BENCH_ARGS > gpurun_out/bench.txt 2> gpurun_out/bench_err.txt
  rc=$?; tail -n 3 gpurun_out/bench_err.txt; tail -n 1 gpurun_out/bench.txt; exit $rc
fi
