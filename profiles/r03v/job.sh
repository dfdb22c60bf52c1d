#!/bin/bash
# r03v: top-node expansion in the regeneration pass (CRT_TOP_LEVELS 1 / 2) against HEAD: frame hashes, then
# interleaved default benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03v; mkdir -p $OUT
for lib in "" raytracer-cuda_amd/lib_exp/t0/libcrt_hip.so raytracer-cuda_amd/lib_exp/t1/libcrt_hip.so raytracer-cuda_amd/lib_exp/t2/libcrt_hip.so; do
  label=${lib:-head}; label=$(basename $(dirname $label 2>/dev/null) 2>/dev/null || echo head)
  [ -z "$lib" ] && label=head
  if [ -n "$lib" ]; then export CRT_HIP_LIB=$R/$lib; else unset CRT_HIP_LIB; fi
  timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_$label.txt 2>&1
  echo "== $label"; grep -v amdgpu.ids $OUT/hash_$label.txt
done
unset CRT_HIP_LIB
bash tools/gpu_job.sh libs r03v 2 raytracer-cuda_amd/lib_exp/t0/libcrt_hip.so raytracer-cuda_amd/lib_exp/t1/libcrt_hip.so raytracer-cuda_amd/lib_exp/t2/libcrt_hip.so
