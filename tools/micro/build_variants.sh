#!/bin/bash
# build libcbev variants for tools/micro/step_variants.sh: one "name:-Dflags" per argument
set -eu
mkdir -p ${VARDIR:-tools/micro/so}
rm -f ${VARDIR:-tools/micro/so}/*.so
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math \
    -Wno-unused-function -mllvm -amdgpu-kernarg-preload-count=16 -Iinclude $flags -o ${VARDIR:-tools/micro/so}/libcbev_$name.so carlabev_env_amd/csrc/cbev.hip &
done
wait
ls ${VARDIR:-tools/micro/so}
