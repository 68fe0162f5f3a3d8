#!/bin/bash
# round 6: the masked reset's scene-bytes copy -- its parity tests, then a
# same-box kernel A/B of k_reset_mask variants (tools/micro/ab) at configs 3, 4
set -u
mkdir -p gpurun_out/rab
export TMPDIR=/tmp
timeout -k 10 ${TEST_LIMIT:-400} python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "${PYTEST_K:-reset or config3_masked}" > gpurun_out/rab/pytest.txt 2>&1
rc=$?
tail -n 15 gpurun_out/rab/pytest.txt
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
for c in ${CONFIGS:-3 4}; do
  echo "config $c"
  CONFIG=$c LIBS="${LIBS}" ./tools/r5_kab.sh || exit 1
done
