set -u
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
for m in "CBEV_SERIAL_STEP=1" "CBEV_COLLIDE_CUS=8" "CBEV_COLLIDE_CUS=16" "CBEV_COLLIDE_CUS=32"; do
  env $m timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-wire > gpurun_out/bm.json 2> gpurun_out/bm.err || { echo "fail $m"; tail -5 gpurun_out/bm.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/bm.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['kernel_ms'])
"
done
