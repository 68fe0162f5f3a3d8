#!/bin/bash
# Round-3 re-entry pass: GPU parity tests + smoke + a default bench line, then a
# rocprofv3 A/B of the libcbev variants under tools/micro/var (if any).
set -u
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
BENCH_ARGS="--steps 100 --warmup 20" bash tools/gpu_tests.sh || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.txt 2>&1 || { tail -5 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
fi
if ls tools/micro/var/*.so > /dev/null 2>&1; then
  bash tools/micro/kernel_ab.sh tools/micro/var/*.so || exit 1
  BENCH_ARGS="--config 3" bash tools/micro/kernel_ab.sh tools/micro/var/*.so || exit 1
fi
