#!/bin/bash
# One GPU pass at a milestone: GPU parity tests, the default bench line, then
# the rocprofv3 passes of tools/profile.sh (PROFILE=0 skips them).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
if [ "${PROFILE:-1}" = 1 ]; then
  bash tools/profile.sh || exit 1
fi
