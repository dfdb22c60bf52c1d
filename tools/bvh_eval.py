"""Evaluate CRT_BVH_REBUILT against the reference BVH on the GPU.

For each rebuilt configuration (leaf size x layouts):
  * per-ray agreement with the reference BVH (crt_scene_compare: both structures trace the same rays);
  * render speed (variant 3) and work per ray (counting launch);
  * image-level difference of a full frame against the reference-BVH frame (bit-equal pixel fraction,
    per-channel RMS of the resolved linear colour).
Prints one JSON line per configuration.
"""
import argparse
import json
import sys
import time
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
ap.add_argument("--spp", type=int, default=32, help="samples for the timing + image runs")
ap.add_argument("--cmp-spp", type=int, default=8, help="samples for the per-ray comparison")
ap.add_argument("--bounces", type=int, default=20)
ap.add_argument("--configs", default="w4:l4:t1,w4:l8:t2,w2:l16:t6",
                help="comma list of w<width>:l<leaf size>:t<SAH traversal cost>[:L<layouts>][:o<occupancy>]")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--no-compare", action="store_true")
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene))
ref = hs.upload(0)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
scale = crt_amd.pixel_sample_scale(a.spp)


def frame(scene):
    best = None
    for _ in range(a.reps):
        r.init_rand(41)
        r.render(scene, a.spp, a.bounces)
        r.synchronize()
        ms = r.last_kernel_ms()
        best = ms if best is None else min(best, ms)
    rays = r.counters()["rays"]
    return best, rays, r.linear().copy()


def work(scene):
    r.init_rand(41)
    r.render(scene, a.spp, a.bounces, count_work=True)
    r.synchronize()
    c = r.counters()
    return {k: round(c[k] / c["rays"], 3) for k in ("box_tests", "tri_tests", "sphere_tests")}


ms_ref, rays_ref, img_ref = frame(ref)
print(json.dumps({"config": "reference", "scene": a.scene, "stats": ref.stats(), "kernel_ms": round(ms_ref, 2),
                  "mrays_s": round(rays_ref / ms_ref / 1e3, 1), "work_per_ray": work(ref)}), flush=True)
for cfg in a.configs.split(","):
        f = {p[0]: p[1:] for p in cfg.split(":")}
        width, leaf, trav = int(f.get("w", 4)), int(f.get("l", 4)), float(f.get("t", 1))
        layouts, occ = int(f.get("L", 6 if width == 2 else 1)), int(f.get("o", 0))
        r.set_occupancy_target(occ)
        r.set_regen_threshold(int(f.get("T", 24)))
        r.set_kernel_variant(int(f.get("V", 3)))
        r.set_schedule(int(f.get("P", -1)), 64, int(f.get("Y", 2)))
        t = time.time()
        sc = hs.upload(0, bvh="rebuilt", leaf_size=leaf, layouts=layouts, traversal_cost=trav, width=width)
        build_s = time.time() - t
        r.init_rand(41)
        cmp = {"rays": 0, "rank_mismatch": 0} if a.no_compare else r.compare(ref, sc, a.cmp_spp, a.bounces)
        ms, rays, img = frame(sc)
        d = (img - img_ref) * scale
        out = {"config": cfg, "scene": a.scene, "build_upload_s": round(build_s, 3),
               "stats": sc.stats(), "kernel_ms": round(ms, 2), "mrays_s": round(rays / ms / 1e3, 1),
               "speedup_vs_reference": round(ms_ref / ms, 3), "rays_vs_reference": rays / rays_ref,
               "work_per_ray": work(sc), "per_ray": cmp,
               "per_ray_mismatch_rate": cmp["rank_mismatch"] / max(1, cmp["rays"]),
               "image": {"pixels_bit_equal": float(np.mean(np.all(img == img_ref, axis=-1))),
                         "rms_per_channel": [float(x) for x in np.sqrt(np.mean(d.reshape(-1, 3) ** 2, axis=0))]}}
        out["schedule"] = r.schedule_stats()
        prof = r.section_profile()
        tot = max(1, prof["cyc_regen"] + prof["cyc_step"] + prof["cyc_round"])
        out["section_profile"] = dict(prof, frac_regen=round(prof["cyc_regen"] / tot, 3),
                                      frac_step=round(prof["cyc_step"] / tot, 3),
                                      frac_round=round(prof["cyc_round"] / tot, 3))
        print(json.dumps(out), flush=True)
        sc.close()
        r.set_occupancy_target(0)
        r.set_regen_threshold(24)
        r.set_kernel_variant(3)
