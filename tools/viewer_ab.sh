#!/bin/bash
# A/B of the interactive loop (bin/crt_viewer, 600 frames of 1 spp at 2560x1440, still) over library builds:
#   tools/viewer_ab.sh OUT ROUNDS LIBDIR...   (LIBDIR holds a libcrt_hip.so, e.g. raytracer-cuda_amd/lib_exp/<name>)
# The in-tree library runs first in each round; the others are picked up through LD_LIBRARY_PATH (crt_viewer's
# RUNPATH gives way to it).
set -e
OUT=gpurun_out/$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
F=$(CRT_NO_TORCH=1 python3 -c "import sys; sys.path.insert(0, 'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(map(str, assets.scene_files('cornell_bunny'))))")
for i in $(seq 1 $N); do
  timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script still -bvh rebuilt $F > $R/$OUT/viewer_A_$i.json
  echo "A round $i: $(cat $R/$OUT/viewer_A_$i.json | grep -o '"kernel_ms_mean": [0-9.]*')"
  for d in "$@"; do
    label=$(basename $d)
    LD_LIBRARY_PATH=$R/$d timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script still -bvh rebuilt $F \
        > $R/$OUT/viewer_${label}_$i.json
    echo "$label round $i: $(cat $R/$OUT/viewer_${label}_$i.json | grep -o '"kernel_ms_mean": [0-9.]*')"
  done
done
