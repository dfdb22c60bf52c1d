import sys, json
from pathlib import Path
import numpy as np
REPO = Path('.').resolve()
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd
from crt_amd import assets
W, H = 2560, 1440
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H)
r.set_camera(crt_amd.camera(2000))
def m(seed, base, spp):
    r.init_rand(seed, base); r.render(sc, spp, 20); r.synchronize()
    lin = r.linear().astype(np.float64).reshape(-1, 3)
    return lin.mean(0) / spp, r.counters()["rays"] / (W * H * spp), r.last_kernel_name()
for spp in (250, 500, 1000, 2000):
    mm, rp, k = m(41, 0, spp)
    print(json.dumps({"family": 0, "spp": spp, "mean_per_sample": mm.round(6).tolist(), "rays_per_path": round(rp, 5), "kernel": k}), flush=True)
for g in (1, 5):
    mm, rp, k = m(41, g * W * H, 250)
    print(json.dumps({"family": g, "spp": 250, "mean_per_sample": mm.round(6).tolist(), "rays_per_path": round(rp, 5), "kernel": k}), flush=True)
# variant 4 (grid, no probe) and variant 10 (reference BVH) at 250 and 2000 spp, family 0
ref = hs.upload(0)
for v, s in ((4, sc), (10, ref)):
    r.set_kernel_variant(v)
    for spp in (250, 2000):
        mm, rp, k = m(41, 0, spp)
        print(json.dumps({"variant": v, "spp": spp, "mean_per_sample": mm.round(6).tolist(), "rays_per_path": round(rp, 5), "kernel": k}), flush=True)
