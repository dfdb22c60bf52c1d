#!/bin/bash
# r03w: is level 2's slowdown the LDS footprint?  t1 (root in LDS, 5952 B) padded to 6144 B and 6464 B (level 2's size).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
unset CRT_HIP_LIB
mkdir -p $R/gpurun_out/r03w
timeout -k 10 180 python3 tools/frame_hash.py > $R/gpurun_out/r03w/hash_intree.txt 2>&1
grep -v amdgpu.ids $R/gpurun_out/r03w/hash_intree.txt
unset CRT_HIP_LIB
bash tools/gpu_job.sh libs r03w 2 raytracer-cuda_amd/lib_exp/t1/libcrt_hip.so raytracer-cuda_amd/lib_exp/t1p192/libcrt_hip.so raytracer-cuda_amd/lib_exp/t1p512/libcrt_hip.so
