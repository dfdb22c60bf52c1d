"""Occupancy A/B of variant 8 in one process (crt_renderer_set_occupancy_target), for one library build: main-kernel ms
per setting, interleaved, and the frame hash (frames must not depend on it).  Used for round 5's cold-path-state
experiment (profiles/r05aa): run once per library (CRT_HIP_LIB / CRT_HOST_LIB).

    python tools/cold_ab.py [--configs C] [--occupancy 7,8] [--reps 2]
"""
import argparse
import hashlib
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

CONFIGS = {"B": ("cornell_bunny", 1280, 720, 256), "C": ("cornell_bunny", 2560, 1440, 2000),
           "E": ("cornell_1m", 2560, 1440, 512), "S": ("cornell_bunny", 640, 360, 64),
           "M": ("cornell_bunny", 1600, 900, 256)}
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C")
ap.add_argument("--occupancy", default="7,8")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--top-levels", default="-1", help="comma list for crt_renderer_set_top_levels, interleaved too")
ap.add_argument("--trees", default="sah", help="comma list of sah / sbvh (spatial splits): interleaved like the occupancies")
a = ap.parse_args()
occs = [int(v) for v in a.occupancy.split(",")]


def frame_hash(r):
    h = hashlib.sha256()
    h.update(r.linear().tobytes())
    h.update(r.rng_state().tobytes())
    return h.hexdigest()[:16]


scenes = {}
for cfg in a.configs.split(","):
    name, W, H, spp = CONFIGS[cfg]
    if name not in scenes:
        hs = crt_amd.HostScene(assets.scene_files(name), build_device=0)
        scenes[name] = {tr: hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0,
                                      gpu_build=(tr == "sah"), spatial_splits=(tr == "sbvh"))
                        for tr in a.trees.split(",")}
    trees = scenes[name]
    r = crt_amd.Renderer(W, H)
    r.set_kernel_variant(8)
    r.set_camera(crt_amd.camera(spp))
    hashes = {}
    settings = [(oc, tr, tl) for oc in occs for tr in trees for tl in (int(v) for v in a.top_levels.split(","))]
    for rep in range(a.reps + 1):
        for oc, tr, tl in (settings if rep % 2 == 0 else settings[::-1]):
            r.set_occupancy_target(oc)
            r.set_top_levels(tl)
            r.init_rand(41)
            r.render(trees[tr], spp, 20)
            r.synchronize()
            ph = r.last_timings()
            hashes.setdefault(f"{oc}/{tr}/{tl}", frame_hash(r))
            print(json.dumps({"config": cfg, "rep": rep, "occ": oc, "tree": tr, "top": tl, "kernel": r.last_kernel_name(),
                              "main_kernel_ms": round(ph["main_kernel_ms"], 3), "rays": r.counters()["rays"]}), flush=True)
    print(json.dumps({"config": cfg, "hashes": {str(k): v for k, v in hashes.items()}}), flush=True)
