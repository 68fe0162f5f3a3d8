#!/bin/bash
# k_raster_pipe vs round 4's k_raster (CBEV_RASTER_TILE=1) side by side, then the
# pipe's in-kernel phase stamps, for each config in ${CONFIGS:-2 5}
set -u
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp
SO=carlabev_env_amd/libcbev.so
for c in ${CONFIGS:-2 5}; do
  timeout -k 10 240 python -u tools/micro/raster_ab.py --config $c --libs $SO $SO:CBEV_RASTER_TILE=1 ${AB_EXTRA:-} > gpurun_out/pipe/ab_c$c.txt 2>&1 || { echo "ab $c failed"; tail -5 gpurun_out/pipe/ab_c$c.txt; exit 1; }
  tail -4 gpurun_out/pipe/ab_c$c.txt
  if [ -z "${SKIP_PHASES:-}" ]; then
    timeout -k 10 240 python -u tools/micro/pipe_phases.py --config $c ${PH_EXTRA:-} > gpurun_out/pipe/ph_c$c.txt 2>&1 || { echo "phases $c failed"; tail -5 gpurun_out/pipe/ph_c$c.txt; exit 1; }
    tail -9 gpurun_out/pipe/ph_c$c.txt
  fi
done
