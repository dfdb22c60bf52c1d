#!/bin/bash
# r06z6: the default bench line and config B's, with the new render_kernel / render_schedule fields (bench.py only
# changed since r06z3).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06z6; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
timeout -k 10 400 python3 bench.py --width 1280 --height 720 --spp 256 > $OUT/B.log 2>&1
echo job done
