#!/bin/bash
# three rasters side by side (glds pipe, register-staged pipe, round 4's tile raster)
# and the register-staged pipe's phase stamps, for each config in ${CONFIGS:-2 5}
set -u
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp
SO=carlabev_env_amd/libcbev.so
REG=carlabev_env_amd/libcbev_pipereg.so
for c in ${CONFIGS:-2 5}; do
  timeout -k 10 240 python -u tools/micro/raster_ab.py --config $c --libs $SO $REG $SO:CBEV_RASTER_TILE=1 > gpurun_out/pipe/ab2_c$c.txt 2>&1 || { echo "ab $c failed"; tail -5 gpurun_out/pipe/ab2_c$c.txt; exit 1; }
  tail -5 gpurun_out/pipe/ab2_c$c.txt
  timeout -k 10 240 python -u tools/micro/pipe_phases.py --config $c --so carlabev_env_amd/libcbev_pipereg_t.so > gpurun_out/pipe/ph2_c$c.txt 2>&1 || { echo "phases $c failed"; tail -5 gpurun_out/pipe/ph2_c$c.txt; exit 1; }
  tail -9 gpurun_out/pipe/ph2_c$c.txt
done
