set -u
mkdir -p gpurun_out
CBEV_LIB=tools/micro/so/libcbev_b_nt1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "config5 or profile_raster or 256" --timeout 120 --timeout-method thread > gpurun_out/pytest_nt.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_nt.log; exit 1; }
tail -1 gpurun_out/pytest_nt.log
CFGS="5" bash tools/micro/step_variants.sh
