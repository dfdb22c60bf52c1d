#!/bin/bash
# r03ai: occupancy 7 with 8 LDS stack entries (o7s8) checked bit for bit at occupancy 7, and occupancy 8 for variant 8
# (o8: 64 VGPRs, 21 spilled; a throw-away build whose occupancy-7 launch runs the <false, 8, 8> instantiation).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03ai; OUT=$R/gpurun_out/$O; mkdir -p $OUT
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o7s8/libcrt_hip.so timeout -k 10 180 python3 tools/frame_hash.py --big --occupancy 7 > $OUT/hash_o7s8_occ7.txt 2>&1
grep -v amdgpu.ids $OUT/hash_o7s8_occ7.txt
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2; do
  timeout -k 10 300 $B > $OUT/A_$i.log 2>&1
  CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o7s8/libcrt_hip.so timeout -k 10 300 $B --occupancy 7 > $OUT/o7s8_$i.log 2>&1
  CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o8/libcrt_hip.so timeout -k 10 300 $B --occupancy 7 > $OUT/o8_$i.log 2>&1
  for l in A o7s8 o8; do echo "$l round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/${l}_$i.log)"; done
done
