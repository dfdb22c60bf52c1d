#!/bin/bash
# r03am: occupancy for the other launches -- variant 10 (the bit-exact reference-BVH path, config C) at 5 (default) /
# 6 / 7, and variant 7 (1-spp interactive frames at 2560x1440; config A) at 6 (default) / 7.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03am; OUT=$R/gpurun_out/$O; mkdir -p $OUT
CRT_HIP_LIB= timeout -k 10 180 python3 - > $OUT/v10_bits.txt 2>&1 <<'PY'
import sys, numpy as np
sys.path.insert(0, "raytracer-cuda_amd")
import crt_amd
from crt_amd import assets
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
ref = hs.upload(0)
out = []
for occ in (0, 6, 7):
    r = crt_amd.Renderer(320, 180)
    r.set_kernel_variant(10)
    if occ:
        r.set_occupancy_target(occ)
    r.set_camera(crt_amd.camera(64))
    r.init_rand(41)
    r.render(ref, 64, 20)
    r.synchronize()
    out.append((r.last_kernel_name(), r.linear().view(np.uint32).copy(), r.rng_state().copy()))
for k, lin, rng in out:
    print(k, np.array_equal(lin, out[0][1]) and np.array_equal(rng, out[0][2]))
PY
cat $OUT/v10_bits.txt | grep -v amdgpu
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2; do
  for o in 5 6 7; do timeout -k 10 300 $B --bvh reference --steps 2 --occupancy $o > $OUT/v10_o${o}_$i.log 2>&1; done
  for o in 6 7; do timeout -k 10 120 $B --spp 1 --steps 20 --occupancy $o > $OUT/v7_1spp_o${o}_$i.log 2>&1; done
  for o in 6 7; do timeout -k 10 120 $B --scene cornell --width 256 --height 256 --spp 16 --bounces 4 --steps 20 --occupancy $o > $OUT/A_o${o}_$i.log 2>&1; done
  for f in v10_o5 v10_o6 v10_o7 v7_1spp_o6 v7_1spp_o7 A_o6 A_o7; do echo "$f round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/${f}_$i.log)"; done
done
