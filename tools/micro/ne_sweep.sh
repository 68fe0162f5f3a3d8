set -u
# envs per k_ego workgroup (CBEV_EGO_NE, read at cbev_create), config ${CFG:-2}
for ne in ${NES:-2 4 8 16 32}; do
  CBEV_EGO_NE=$ne timeout -k 10 300 python bench.py --config ${CFG:-2} --no-cpu-baseline --no-wire --fresh-workers 0 --scene-cache /tmp/cbev_scene_cache > gpurun_out/bn.json 2> gpurun_out/bn.err || { echo "fail $ne"; tail -3 gpurun_out/bn.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/bn.json').read().strip().splitlines()[-1]); print('ne=$ne', d['value'], d['ms_per_step'], d['kernel_ms'])
"
done
