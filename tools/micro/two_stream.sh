#!/bin/bash
# tools/micro/two_stream.py at configs 2 and 3
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-2 3}; do
  timeout -k 10 240 python -u tools/micro/two_stream.py --config $c > gpurun_out/two_stream_c$c.txt 2>&1
  rc=$?
  grep "config" gpurun_out/two_stream_c$c.txt
  [ $rc -ne 0 ] && { tail -5 gpurun_out/two_stream_c$c.txt; exit $rc; }
done
exit 0
