#!/bin/bash
# r03ad: finish_ray (the pass's sphere test + shading with the early record load) shared by variants 8 and 7:
# hashes of the in-tree build, A/B against the previous commit (base), the interactive loop (variant 7) for both.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03ad; OUT=$R/gpurun_out/$O; mkdir -p $OUT
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
grep -v amdgpu.ids $OUT/hash_intree.txt
bash tools/gpu_job.sh libs $O 2 raytracer-cuda_amd/lib_exp/base/libcrt_hip.so
F=$(CRT_NO_TORCH=1 python3 -c "import sys; sys.path.insert(0, 'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(map(str, assets.scene_files('cornell_bunny'))))")
for i in 1 2; do
  timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script still -bvh rebuilt $F > $OUT/viewer_A_$i.json
  LD_LIBRARY_PATH=$R/raytracer-cuda_amd/lib_exp/base timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script still -bvh rebuilt $F > $OUT/viewer_base_$i.json
  echo "viewer A: $(grep -o '"fps": [0-9.]*' $OUT/viewer_A_$i.json)  base: $(grep -o '"fps": [0-9.]*' $OUT/viewer_base_$i.json)"
done
