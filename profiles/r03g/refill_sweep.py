"""Variant 7 with a refill threshold (crt_renderer_set_refill) against variant 8, interleaved in one process.

    python tools/refill_sweep.py [--w 2560 --h 1440 --spp 2000] [--refill 64,32,16,8] [--reps 2]

Prints the render time (HIP events, probe included) of each configuration and checks every frame equals variant 8's
bit for bit (same per-pixel sample order, so the same frame)."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=2000)
ap.add_argument("--refill", default="64,32,16,8")
ap.add_argument("--thresholds", default="44", help="regeneration thresholds to cross with the refill values")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
configs = [("v8", 8, 64, 44)] + [(f"v7_R{R}_T{T}", 7, int(R), int(T)) for R in a.refill.split(",")
                                  for T in a.thresholds.split(",")]
ref = None
res = {c[0]: [] for c in configs}
for rep in range(a.reps):
    for name, var, R, T in configs:
        r.set_kernel_variant(var)
        r.set_refill(R)
        r.set_regen_threshold(T)
        r.init_rand(41)
        r.render(sc, a.spp, 20)
        r.synchronize()
        t = r.last_timings()
        lin = r.linear()
        if ref is None:
            ref = lin
        same = bool(np.array_equal(lin.view(np.uint32), ref.view(np.uint32)))
        res[name].append(t["render_ms"])
        print(json.dumps({"rep": rep, "config": name, "kernel": r.last_kernel_name(), "same_frame": same, **t}),
              flush=True)
print(json.dumps({k: round(min(v), 2) for k, v in res.items()}))
