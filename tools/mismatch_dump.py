"""Dump rays whose closest hit differs between the reference BVH and the rebuilt BVH (GPU), for offline
analysis with tools/mismatch_analyze.py (CPU)."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

out = Path(sys.argv[1])
out.mkdir(parents=True, exist_ok=True)
for scene, w, h, spp in (("cornell_bunny", 1280, 720, 32), ("cornell_1m", 1280, 720, 32)):
    hs = crt_amd.HostScene(assets.scene_files(scene))
    ref = hs.upload(0)
    reb = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2)
    r = crt_amd.Renderer(w, h)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41)
    res, rays = r.compare_dump(ref, reb, spp, 20, 4096)
    print(scene, res, flush=True)
    np.save(out / f"{scene}_mismatch.npy", rays)
