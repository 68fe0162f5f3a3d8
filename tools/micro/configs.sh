set -u
# configs 3-5 at N=1, short runs (parity of these configs: tests/test_gpu_parity.py)
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-wire > gpurun_out/bc$c.json 2> gpurun_out/bc$c.err || { echo "config $c failed"; tail -5 gpurun_out/bc$c.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/bc$c.json').read().strip().splitlines()[-1]); print($c, d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])
"
done
