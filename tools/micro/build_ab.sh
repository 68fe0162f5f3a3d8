#!/bin/bash
# build libcbev variants into tools/micro/ab/: one "name:-Dflags" per argument
set -eu
mkdir -p tools/micro/ab
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc $(python -c "from carlabev_env_amd import build as B; print(' '.join(B.FLAGS))") \
    $flags -o tools/micro/ab/libcbev_$name.so carlabev_env_amd/csrc/cbev.hip &
done
wait
ls tools/micro/ab
