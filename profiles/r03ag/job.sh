#!/bin/bash
# r03ag: the pass's unit-sphere and lens-disk rejection loops fused into one loop per wave (-DCRT_FUSED_DRAWS=1).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03ag; mkdir -p $R/gpurun_out/$O
export CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/fused/libcrt_hip.so
timeout -k 10 180 python3 tools/frame_hash.py --big > $R/gpurun_out/$O/hash_fused.txt 2>&1
grep -v amdgpu.ids $R/gpurun_out/$O/hash_fused.txt
unset CRT_HIP_LIB
bash tools/gpu_job.sh libs $O 2 raytracer-cuda_amd/lib_exp/fused/libcrt_hip.so
