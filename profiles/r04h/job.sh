#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04h: (1) the 4-wide kernels keep a ray's o and d in its LDS record only (in-tree) against HEAD's build (base): bits,
# C and E A/B, the interactive loop; (2) the critical tiles' threshold re-swept on B, and C with the best of it.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04h; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/base/libcrt_hip.so > $OUT/sha.txt
BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so
timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$BASE timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_base.txt) && echo "o/d in LDS: hashes identical" || echo "o/d in LDS: HASHES DIFFER"
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
g() { grep -o '"render_ms": [0-9.]*, "probe_sort_ms": [0-9.]*, "main_kernel_ms": [0-9.]*' $1 | tail -1; }
for i in 1 2 3; do
  CRT_HIP_LIB=$BASE timeout -k 10 300 $B > $OUT/C_base_$i.log 2>&1
  timeout -k 10 300 $B > $OUT/C_new_$i.log 2>&1
  for f in C_base C_new; do echo "$f round $i: $(g $OUT/${f}_$i.log)"; done
done
for i in 1 2; do
  CRT_HIP_LIB=$BASE timeout -k 10 300 $B --scene cornell_1m --spp 512 > $OUT/E_base_$i.log 2>&1
  timeout -k 10 300 $B --scene cornell_1m --spp 512 > $OUT/E_new_$i.log 2>&1
  for f in E_base E_new; do echo "$f round $i: $(g $OUT/${f}_$i.log)"; done
done
bash tools/gpu_job.sh viewer $O/viewer
for i in 1 2; do
  for spec in "1024 16" "1024 24" "1024 32" "2048 24" "512 24" "1024 20"; do
    set -- $spec; timeout -k 10 300 $B --width 1280 --height 720 --spp 256 --steps 5 --critical-tiles $1 --critical-lanes $2 > $OUT/B_c$1_l$2_$i.log 2>&1
    echo "B crit $1 lanes $2 round $i: $(g $OUT/B_c$1_l$2_$i.log)"
  done
  for l in 16 24; do
    timeout -k 10 300 $B --critical-tiles 1024 --critical-lanes $l > $OUT/C_l${l}_$i.log 2>&1
    echo "C crit lanes $l round $i: $(g $OUT/C_l${l}_$i.log)"
  done
done
echo job done
