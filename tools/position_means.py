"""Frame means by sample position in the pixel streams (diagnostic for profiles/r06k): for each seed and family, the
stream is rendered in consecutive blocks of `spp` samples (init once, then renders that continue the RNG state), and
each block's frame mean per sample is printed.  A position-dependent bias shows as block 0 differing from the later
blocks with the same sign across families.

    python tools/position_means.py [--seeds 41 43] [--families 8] [--blocks 8] [--spp 250]
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
ap.add_argument("--families", type=int, default=8)
ap.add_argument("--blocks", type=int, default=8)
ap.add_argument("--seeds", type=int, nargs="+", default=[41, 43])
a = ap.parse_args()
W, H = a.w, a.h
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H)
r.set_camera(crt_amd.camera(2000))
for seed in a.seeds:
    M = np.zeros((a.families, a.blocks, 3))
    for g in range(a.families):
        r.init_rand(seed, g * W * H)
        for b in range(a.blocks):
            r.render(sc, a.spp, 20)
            r.synchronize()
            M[g, b] = r.linear().astype(np.float64).reshape(-1, 3).mean(0) / a.spp
    print(json.dumps({"seed": seed, "spp_per_block": a.spp, "means_R": np.round(M[:, :, 0], 6).tolist(),
                      "block0_minus_later_R_per_family": np.round(M[:, 0, 0] - M[:, 1:, 0].mean(1), 6).tolist(),
                      "block_means_R_over_families": np.round(M[:, :, 0].mean(0), 6).tolist(),
                      "family_means_R_over_blocks": np.round(M[:, :, 0].mean(1), 6).tolist()}), flush=True)
