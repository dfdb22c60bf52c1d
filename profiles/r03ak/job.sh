#!/bin/bash
# r03ak: at occupancy 7 -- LDS stack entries 8 (in-tree) / 7 / 6 (how often the HBM overflow path runs), overflow slots
# by hardware lane (ovh: -DCRT_OVF_HW, hashes checked), the
# regeneration threshold re-swept, and config B at occupancy 6 against 7.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r03ak
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/ovh/libcrt_hip.so timeout -k 10 180 python3 tools/frame_hash.py --big > $R/gpurun_out/r03ak/hash_ovh.txt 2>&1
grep -v amdgpu.ids $R/gpurun_out/r03ak/hash_ovh.txt
bash tools/gpu_job.sh libs r03ak 2 raytracer-cuda_amd/lib_exp/s7/libcrt_hip.so raytracer-cuda_amd/lib_exp/s6/libcrt_hip.so raytracer-cuda_amd/lib_exp/ovh/libcrt_hip.so
bash tools/gpu_job.sh sweep r03ak_T 2 "T40=--regen-threshold 40" "T48=--regen-threshold 48"
B="--width 1280 --height 720 --spp 256"
bash tools/gpu_job.sh sweep r03ak_B 2 "occ7=$B" "occ6=$B --occupancy 6"
