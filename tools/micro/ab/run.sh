set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/micro/kernel_ab.sh tools/micro/ab/libcbev_cur.so tools/micro/ab/libcbev_s1.so tools/micro/ab/libcbev_cur.so tools/micro/ab/libcbev_s1.so
