#!/bin/bash
# r03aa: the trace's shading record loaded at the start of the regeneration pass, ahead of the per-ray sphere test
# (-DCRT_SHADE_EARLY; the two per-ray spheres' records staged in LDS) vs the in-tree build.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03aa; mkdir -p $R/gpurun_out/$O
export CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/se/libcrt_hip.so
timeout -k 10 180 python3 tools/frame_hash.py --big > $R/gpurun_out/$O/hash_se.txt 2>&1
grep -v amdgpu.ids $R/gpurun_out/$O/hash_se.txt
unset CRT_HIP_LIB
bash tools/gpu_job.sh libs $O 3 raytracer-cuda_amd/lib_exp/se/libcrt_hip.so
