#!/bin/bash
# r06s: the in-round row prefetch (r06r) at 4 waves per SIMD against the in-tree library at its own occupancy rule, on
# config C, B, E and the N = 8 rank share, two alternating rounds of bench.py (main kernel only, no profiling code).
# Prediction: B -7 to -9 % (r06r); C and E slower at occupancy 4 (fewer waves to hide the rest of the latency), the N = 8
# share in between.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06s; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
LX=$R/raytracer-cuda_amd/lib_exp
B="python3 bench.py --no-cpu-baseline --no-count --no-parity --steps 3 --warmup 1"
for rep in 1 2; do
  for cfg in "C:" "B:--width 1280 --height 720 --spp 256" "E:--scene cornell_1m --spp 512" "S8:--share 0 8"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 $B $args > $OUT/${name}_A_$rep.log 2>&1
    CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$LX/pf2/libcrt_hip.so timeout -k 10 300 $B $args --occupancy 4 > $OUT/${name}_pf_$rep.log 2>&1
  done
done
echo job done
