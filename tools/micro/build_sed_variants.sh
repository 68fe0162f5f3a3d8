#!/bin/bash
# Build libcbev variants for A/B timing (tools/micro/kernel_ab.sh) from edited
# copies of the product source, so no build switch lives in cbev.hip:
#   build_sed_variants.sh "name:sed-expression" ...
# -> tools/micro/ab/libcbev_<name>.so (name "base": the source as it is).
set -eu
mkdir -p tools/micro/ab
for v in "$@"; do
  name=${v%%:*}; expr=${v#*:}
  src=carlabev_env_amd/csrc/.variant_$name.hip
  if [ "$name" = base ]; then cp carlabev_env_amd/csrc/cbev.hip $src; else sed -e "$expr" carlabev_env_amd/csrc/cbev.hip > $src; fi
  if cmp -s $src carlabev_env_amd/csrc/cbev.hip && [ "$name" != base ]; then echo "variant $name: the edit matched nothing"; exit 1; fi
  ( /opt/rocm/bin/hipcc $(python -c "from carlabev_env_amd import build as B; print(' '.join(B.FLAGS))") \
      -o tools/micro/ab/libcbev_$name.so $src && rm -f $src ) &
done
wait
ls tools/micro/ab
