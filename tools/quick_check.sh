set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire --fresh-workers 0 > gpurun_out/bk.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bk.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['ms_per_step_min_max'], 'host', d['host_enqueue_ms_per_step'])"
done
