#!/bin/bash
# r03ab: leaf-round marks as 32-bit (owner, primitive base) words, so a pair's primitive loads issue before the owner's
# LDS ray record arrives (-DCRT_MARK32; 11 LDS stack entries to stay inside 6,144 B), and 11 entries alone (s11).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03ac; mkdir -p $R/gpurun_out/$O
export CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/m32/libcrt_hip.so
timeout -k 10 180 python3 tools/frame_hash.py --big > $R/gpurun_out/$O/hash_m32.txt 2>&1
grep -v amdgpu.ids $R/gpurun_out/$O/hash_m32.txt
unset CRT_HIP_LIB
bash tools/gpu_job.sh libs $O 3 raytracer-cuda_amd/lib_exp/m32/libcrt_hip.so
