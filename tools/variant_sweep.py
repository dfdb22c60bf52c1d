"""Render-kernel time of the 4-wide variants (4, 7, 8) at several samples per pixel, interleaved on one box.

    python tools/variant_sweep.py [--spps 1,4,16,64] [--variants 4,7,8] [--reps 5]

Prints one JSON line per (spp, variant): the best of `reps` kernel times (HIP events; includes the cost probe
where the schedule runs one) and Mrays/s.
"""
import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spps", default="1,4,16,64")
ap.add_argument("--variants", default="4,7,8")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene))
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0)
r = crt_amd.Renderer(a.w, a.h)
for spp in (int(x) for x in a.spps.split(",")):
    r.set_camera(crt_amd.camera(spp))
    best = {}
    for _ in range(a.reps):
        for v in (int(x) for x in a.variants.split(",")):
            r.set_kernel_variant(v)
            r.init_rand(41)
            r.render(sc, spp, 20)
            r.synchronize()
            ms = r.last_kernel_ms()
            best[v] = min(best.get(v, 1e30), ms)
            rays = r.counters()["rays"]
    for v, ms in best.items():
        print(json.dumps({"spp": spp, "variant": v, "kernel_ms": round(ms, 3), "mrays_s": round(rays / ms / 1e3, 1)}),
              flush=True)
