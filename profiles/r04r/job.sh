#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04r: experiment, not in the tree: the wave drain's fraction test for any number of live lanes, not only below the
# regeneration threshold (profiles/r04r/wave_drain_any.patch, built as lib_exp/wdall). Bits; C, B and the N = 8 share
# interleaved with the in-tree build, three rounds.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04r; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
E=$R/raytracer-cuda_amd/lib_exp
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so $E/wdall/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$E/wdall/libcrt_hip.so CRT_HOST_LIB=$E/wdall/libcrt_host.so timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_wdall.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_wdall.txt) && echo "wdall identical" || echo "wdall DIFFERS"
BB="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  for v in intree wdall; do
    if [ $v = wdall ]; then L="CRT_HIP_LIB=$E/wdall/libcrt_hip.so CRT_HOST_LIB=$E/wdall/libcrt_host.so"; else L="X=1"; fi
    env $L timeout -k 10 300 $BB --steps 3 > $OUT/C_${v}_$i.log 2>&1
    env $L timeout -k 10 300 $BB --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_${v}_$i.log 2>&1
    env $L timeout -k 10 300 python3 tools/schedule_sweep.py --world 8 --reps 2 --set base: > $OUT/w8_${v}_$i.jsonl 2>&1
    echo "round $i $v: C $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/C_${v}_$i.log | tail -1 | cut -d' ' -f2) B $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/B_${v}_$i.log | tail -1 | cut -d' ' -f2) w8 $(grep -o '"main_median_ms": [0-9.]*' $OUT/w8_${v}_$i.jsonl | cut -d' ' -f2)"
  done
done
echo job done
