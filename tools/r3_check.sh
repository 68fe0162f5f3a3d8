#!/bin/bash
# Round-3 milestone pass on one GPU: the -m gpu suite, smoke(), the default
# bench line, then k_ego / k_raster phase stamps (CBEV_TIMING build) at config 2.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.json
if [ "${PHASES:-1}" = 1 ]; then
  timeout -k 10 300 python -u tools/micro/step_phases.py --config 2 --reset > gpurun_out/phases2.log 2>&1 || { echo "phases failed"; tail -20 gpurun_out/phases2.log; exit 1; }
  cat gpurun_out/phases2.log | grep -v "^   xcd"
fi
