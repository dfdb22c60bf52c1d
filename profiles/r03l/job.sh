# r03l: A/B of the current library against the r03f one (before pixel sharding), same box
set -e
bash tools/gpu_job.sh libs r03l 3 raytracer-cuda_amd/lib_exp/prev/libcrt_hip.so
