set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
CFGS="5" bash tools/micro/step_variants.sh || exit 1
for c in 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_config$c.json 2> gpurun_out/bench_config$c.err || { echo "config $c failed"; tail -5 gpurun_out/bench_config$c.err; exit 1; }
  tail -1 gpurun_out/bench_config$c.json | cut -c1-400
done
