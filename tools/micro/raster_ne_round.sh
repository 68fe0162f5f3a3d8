set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
CBEV_LIB=tools/micro/so/libcbev_ne2p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ne2p.log 2>&1 || { echo pytest ne2p failed; tail -30 gpurun_out/pytest_ne2p.log; exit 1; }
tail -1 gpurun_out/pytest_ne2p.log
CFGS="2 3" bash tools/micro/step_variants.sh
