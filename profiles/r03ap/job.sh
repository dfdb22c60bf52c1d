#!/bin/bash
# r03ap: variant 8 at occupancy 8 (64 VGPRs, 21 spilled; LDS 5,024 B fits 32 workgroups per CU) against 7: a throw-away
# build whose occupancy-7 launch runs the <false, 8, 8> instantiation.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03ap; OUT=$R/gpurun_out/$O; mkdir -p $OUT
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o8/libcrt_hip.so timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_o8.txt 2>&1
grep -v amdgpu.ids $OUT/hash_o8.txt | tail -3
bash tools/gpu_job.sh libs $O 2 raytracer-cuda_amd/lib_exp/o8/libcrt_hip.so
