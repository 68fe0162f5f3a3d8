#!/bin/bash
# k_raster phase costs for the nibble and byte LDS images (see tools/raster_phases.sh)
set -u
for bm in 64 128; do
  echo "== CBEV_RASTER_BYTES_MAX=$bm"
  EXTRA_DEFS="-DCBEV_RASTER_BYTES_MAX=$bm" PHASES="${PHASES:-63 62 59 55 51 49}" bash tools/raster_phases.sh || exit 1
done
