# r03h: drained waves at the lowest issue priority (CRT_DRAIN_PRIO = 8 / 16 / 24 lanes) against the in-tree kernel
set -e
bash tools/gpu_job.sh libs r03h 3 raytracer-cuda_amd/lib_exp/prio8/libcrt_hip.so raytracer-cuda_amd/lib_exp/prio16/libcrt_hip.so raytracer-cuda_amd/lib_exp/prio24/libcrt_hip.so
