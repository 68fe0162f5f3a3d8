#!/bin/bash
# build libcbev variants into tools/micro/ab/: one "name:-Dflags" per argument
set -eu
mkdir -p tools/micro/ab
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math \
    -Wno-unused-function -Iinclude $flags -o tools/micro/ab/libcbev_$name.so carlabev_env_amd/csrc/cbev.hip &
done
wait
ls tools/micro/ab
