#!/bin/bash
# k_ego / k_raster phase stamps (timing build) with and without the folded reset,
# and a kernel-stats pass with the reset launched on its own (--no-defer-reset)
set -u
D=gpurun_out/${TAG:-r6p}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/micro/step_phases.py --config ${CFG:-2} --steps 30 --reset > $D/phases_reset.txt 2>&1 || { tail -5 $D/phases_reset.txt; exit 1; }
timeout -k 10 300 python -u tools/micro/step_phases.py --config ${CFG:-2} --steps 30 > $D/phases_noreset.txt 2>&1 || { tail -5 $D/phases_noreset.txt; exit 1; }
grep -E "k_ego|cycles since|p50" $D/phases_reset.txt | head -20
echo ----
grep -E "k_ego|cycles since|p50" $D/phases_noreset.txt | head -20
