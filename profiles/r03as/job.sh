#!/bin/bash
# r03as: variant 3 (threaded BVHs below 64 spp: the reference-BVH interactive path) at occupancy 5 (default) against 6,
# with the frame bits compared.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03as; OUT=$R/gpurun_out/$O; mkdir -p $OUT
timeout -k 10 180 python3 - > $OUT/v3_bits.txt 2>&1 <<'PY'
import sys, numpy as np
sys.path.insert(0, "raytracer-cuda_amd")
import crt_amd
from crt_amd import assets
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
ref = hs.upload(0)
out = []
for occ in (0, 6):
    r = crt_amd.Renderer(320, 180)
    if occ:
        r.set_occupancy_target(occ)
    r.set_camera(crt_amd.camera(16))
    r.init_rand(41)
    r.render(ref, 16, 20)
    r.synchronize()
    out.append((r.last_kernel_name(), r.linear().view(np.uint32).copy(), r.rng_state().copy()))
for k, lin, rng in out:
    print(k, np.array_equal(lin, out[0][1]) and np.array_equal(rng, out[0][2]))
PY
grep -v amdgpu $OUT/v3_bits.txt
bash tools/gpu_job.sh sweep $O 2 "o5=--bvh reference --spp 16 --steps 10" "o6=--bvh reference --spp 16 --steps 10 --occupancy 6"
