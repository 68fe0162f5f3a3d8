set -u
mkdir -p gpurun_out
AB="tools/micro/ab"
timeout -k 10 300 python -u tools/micro/step_phases.py --config 2 > gpurun_out/phases.log 2>&1 || { tail -5 gpurun_out/phases.log; exit 1; }
grep -E "^k_raster|^k_ego|^collide" gpurun_out/phases.log | grep -v XCC
timeout -k 10 300 python -u tools/micro/raster_ab.py --config 2 --libs $AB/libcbev_base.so $AB/libcbev_ktouch.so > gpurun_out/ab10.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab10.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire --fresh-workers 0 > gpurun_out/bk.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bk.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['raster_ms_per_launch'])"
