set -u
# envs per workgroup for the staged thread-per-env kernels (k_hero, k_collide)
for ne in 4 8 16 32; do
  CBEV_STAGED_NE=$ne timeout -k 10 300 python bench.py --no-cpu-baseline --no-wire > gpurun_out/bn.json 2> gpurun_out/bn.err || { echo "fail $ne"; tail -3 gpurun_out/bn.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/bn.json').read().strip().splitlines()[-1]); print('ne=$ne', d['value'], d['ms_per_step'], d['kernel_ms'])
"
done
