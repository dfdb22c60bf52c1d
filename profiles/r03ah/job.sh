#!/bin/bash
# r03ah: occupancy 7 for variant 8 (72 VGPRs, 3 spilled) with 11 (in-tree), 9 and 8 LDS stack entries, against
# the default occupancy 6.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03ah; OUT=$R/gpurun_out/$O; mkdir -p $OUT
export CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o7s8/libcrt_hip.so
timeout -k 10 180 python3 tools/frame_hash.py > $OUT/hash_o7s8_occ6.txt 2>&1
unset CRT_HIP_LIB
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2; do
  timeout -k 10 300 $B > $OUT/A_$i.log 2>&1
  timeout -k 10 300 $B --occupancy 7 > $OUT/o7s11_$i.log 2>&1
  CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o7s9/libcrt_hip.so timeout -k 10 300 $B --occupancy 7 > $OUT/o7s9_$i.log 2>&1
  CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/o7s8/libcrt_hip.so timeout -k 10 300 $B --occupancy 7 > $OUT/o7s8_$i.log 2>&1
  for l in A o7s11 o7s9 o7s8; do echo "$l round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/${l}_$i.log) $(grep -o 'crt_render_kernel<[^>]*>' $OUT/${l}_$i.log | tail -1)"; done
done
