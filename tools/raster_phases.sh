#!/bin/bash
# Raster phase timing: build libcbev variants with CBEV_RASTER_PHASES (1 stage,
# 2 paint, 4 gather, 8 store) and time k_raster in bench.py for each.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/phases
mkdir -p $OUT
CFG=${CFG:-2}
for ph in ${PHASES:-15 14 11 7 1 13 9}; do
  so=$OUT/libcbev_p$ph.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math -Iinclude \
    -DCBEV_RASTER_PHASES=$ph ${EXTRA_DEFS:-} -o $so carlabev_env_amd/csrc/cbev.hip || exit 1
  CBEV_LIB=$so timeout -k 10 300 python bench.py --config $CFG --steps 100 --warmup 10 --no-cpu-baseline --no-wire \
    > $OUT/p$ph.json 2> $OUT/p$ph.err
  rc=$?
  echo "phases=$ph rc=$rc $(python -c "import json,sys; d=json.loads(open('$OUT/p$ph.json').read().strip().splitlines()[-1]); print(d['kernel_ms'])" 2>&1)"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$ph.err; exit $rc; fi
done
