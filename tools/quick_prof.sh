set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for ne in 16 8 4 16 8 4; do
CBEV_EGO_NE=$ne timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire --fresh-workers 0 > gpurun_out/bk.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bk.json').read().strip().splitlines()[-1]); print('ne $ne', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
