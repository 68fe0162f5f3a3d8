#!/bin/bash
# smoke, fused vs split step (config ${CFG:-2}), GPU tests, phase stamps
set -u
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/micro/step_modes2.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
if [ -n "${PHASES:-}" ]; then
timeout -k 10 300 python tools/micro/step_phases.py --config ${CFG:-2} > gpurun_out/step_phases.txt 2>&1 && grep -v "xcd \|XCC" gpurun_out/step_phases.txt
fi
