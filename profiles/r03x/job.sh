#!/bin/bash
# r03x: level-2 top expansion within the 6144-B LDS budget (10 or 11 LDS stack entries) vs the in-tree level 1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r03x
export CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/t2s10/libcrt_hip.so
timeout -k 10 180 python3 tools/frame_hash.py --big > $R/gpurun_out/r03x/hash_t2s10.txt 2>&1
grep -v amdgpu.ids $R/gpurun_out/r03x/hash_t2s10.txt
unset CRT_HIP_LIB
bash tools/gpu_job.sh libs r03x 2 raytracer-cuda_amd/lib_exp/t1s10/libcrt_hip.so raytracer-cuda_amd/lib_exp/t2s10/libcrt_hip.so raytracer-cuda_amd/lib_exp/t2s11/libcrt_hip.so
