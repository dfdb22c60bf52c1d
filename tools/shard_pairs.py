"""Which comparisons carry the N = 8 frame-mean excess (diagnostic, r06k)?  For one seed on one GPU: F1, F1' (2000 spp,
families 0 and 16), F8 = sum of shares from families 0-7 and F8' = sum of shares from families 8-15 (250 spp each),
and the z of the frame-mean difference (linear, float64) for every pair, plus the RMS ratio against the two-frame noise.

    python tools/shard_pairs.py [--seed 41] [--w 2560 --h 1440]
"""
import argparse
import itertools
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
ap.add_argument("--spp", type=int, default=2000)
ap.add_argument("--seed", type=int, default=41)
ap.add_argument("--n", type=int, default=8)
a = ap.parse_args()
W, H, S, N = a.w, a.h, a.spp, a.n
WH = W * H
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H)
r.set_camera(crt_amd.camera(S))


def frame(base, spp):
    r.init_rand(a.seed, base)
    r.render(sc, spp, 20)
    r.synchronize()
    return r.linear().astype(np.float64).reshape(-1, 3)


F = {"F1": frame(0, S) / S, "F1p": frame(2 * N * WH, S) / S,
     "F8": sum(frame(g * WH, S // N) for g in range(N)) / S,
     "F8p": sum(frame((N + g) * WH, S // N) for g in range(N)) / S}
for x, y in itertools.combinations(F, 2):
    d = F[x] - F[y]
    z = d.mean(0) / (d.std(0) / np.sqrt(d.shape[0]))
    print(json.dumps({"pair": f"{x}-{y}", "z": np.round(z, 2).tolist(), "rms": np.round(np.sqrt((d ** 2).mean(0)), 6).tolist()}),
          flush=True)
