"""Frame means by curand subsequence family (diagnostic for profiles/r06k).  For each seed, the frame of `spp` samples
from family g (subsequence g*W*H + pixel) for g = 0 .. G-1; prints each family's mean per sample (float64) and the
scatter of the family means against the independent-pixel noise model (the standard error of one frame's mean).

    python tools/family_means.py [--seeds 41 43] [--families 32] [--spp 250]
"""
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
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=250)
ap.add_argument("--families", type=int, default=32)
ap.add_argument("--seeds", type=int, nargs="+", default=[41, 43])
ap.add_argument("--stride", type=int, default=1, help="family g uses subsequence base g*stride*W*H")
a = ap.parse_args()
W, H = a.w, a.h
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H)
r.set_camera(crt_amd.camera(2000))
for seed in a.seeds:
    means, ses = [], []
    for g in range(a.families):
        r.init_rand(seed, g * a.stride * W * H)
        r.render(sc, a.spp, 20)
        r.synchronize()
        lin = r.linear().astype(np.float64).reshape(-1, 3) / a.spp
        means.append(lin.mean(0))
        ses.append(lin.std(0) / np.sqrt(lin.shape[0]))
    means, ses = np.array(means), np.array(ses)
    scatter = means.std(0, ddof=1)
    print(json.dumps({"seed": seed, "spp": a.spp, "families": a.families,
                      "family_means_R": np.round(means[:, 0], 6).tolist(),
                      "scatter_over_model_se": np.round(scatter / ses.mean(0), 3).tolist(),
                      "family0_minus_rest_in_se": np.round((means[0] - means[1:].mean(0)) / ses.mean(0), 2).tolist()}),
          flush=True)
