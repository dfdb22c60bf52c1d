#!/bin/bash
# r06t: the row prefetch as the shipped occupancy-4 kernel (crt_render_kernel<false, 8, 4>, chosen automatically below
# 4 tiles per wave slot).  The GPU suite (bit-identity of occupancy 4 against 6 and 7, the oracle bands of config B at
# occupancy 4, the checked build's pair checks in the prefetch round), then the rule's crossover: the automatic choice
# against a forced occupancy on frames around it, two alternating rounds.  Prediction: B -8 %; 1280x720 at 64 and 1024 spp
# and 1600x900 at 256 faster at 4 than at 6; 1920x1080 (>= 4 tiles per slot, automatic 7) slower at 4.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06t; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
B="python3 bench.py --no-cpu-baseline --no-count --no-parity --steps 3 --warmup 1"
for rep in 1 2; do
  for cfg in "B:--width 1280 --height 720 --spp 256:6" "B64:--width 1280 --height 720 --spp 64:6" \
             "B1024:--width 1280 --height 720 --spp 1024:6" "W1600:--width 1600 --height 900 --spp 256:6" \
             "W1920:--width 1920 --height 1080 --spp 256:4"; do
    name=${cfg%%:*}; rest=${cfg#*:}; args=${rest%:*}; occ=${rest##*:}
    timeout -k 10 300 $B $args > $OUT/${name}_auto_$rep.log 2>&1
    timeout -k 10 300 $B $args --occupancy $occ > $OUT/${name}_occ${occ}_$rep.log 2>&1
  done
done
echo job done
