"""Bit-identity of a share's frame across kernel variants at full size (diagnostic for the N = 8 statistics, r06k).

    python tools/share_variants.py [--world 8] [--seed 41] [--variants 8,4]

Renders every rank's share of an N-way headline frame (shard_spp samples from family g*W*H) with each variant and
reports, per share, the pixels and 8x8 tiles whose fp32 sums differ from the first variant's; variants 4 and 8 are the
same path program under different schedules (grid vs. cost-ordered tiles), so their frames must agree bit for bit.
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
from crt_amd.dist import shard_spp, subsequence_base  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=2000)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--seed", type=int, default=41)
ap.add_argument("--variants", default="8,4")
ap.add_argument("--ranks", default="")
a = ap.parse_args()
W, H = a.w, a.h
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
variants = [int(v) for v in a.variants.split(",")]
rs = {}
for v in variants:
    rs[v] = crt_amd.Renderer(W, H)
    rs[v].set_kernel_variant(v)
    rs[v].set_camera(crt_amd.camera(a.spp))
ranks = [int(g) for g in a.ranks.split(",")] if a.ranks else list(range(a.world))
for g in ranks:
    frames, names = {}, {}
    for v in variants:
        r = rs[v]
        r.init_rand(a.seed, subsequence_base(g, W, H))
        r.render(sc, shard_spp(a.spp, a.world, g), 20)
        r.synchronize()
        frames[v] = r.linear()
        names[v] = r.last_kernel_name()
    ref = frames[variants[0]]
    for v in variants[1:]:
        diff = np.any(ref.view(np.uint32) != frames[v].view(np.uint32), axis=-1)
        ys, xs = np.nonzero(diff)
        tiles = sorted({(int(y) // 8, int(x) // 8) for y, x in zip(ys, xs)})
        print(json.dumps({"rank": g, "a": names[variants[0]], "b": names[v], "pixels_differing": int(diff.sum()),
                          "tiles_differing": len(tiles), "first_tiles": tiles[:10],
                          "mean_a": ref.reshape(-1, 3).mean(0).round(4).tolist(),
                          "mean_b": frames[v].reshape(-1, 3).mean(0).round(4).tolist()}), flush=True)
