set -u
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/raster_ceiling.bin > gpurun_out/ceiling.txt 2>&1 && cat gpurun_out/ceiling.txt &&
timeout -k 10 120 tools/micro/launch_micro.bin > gpurun_out/launch.txt 2>&1 && cat gpurun_out/launch.txt &&
timeout -k 10 300 python tools/micro/step_phases.py > gpurun_out/step_phases.txt 2>&1 && cat gpurun_out/step_phases.txt
