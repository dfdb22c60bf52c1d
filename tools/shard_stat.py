"""Statistical parity of the spp-sharded frame against the 1-GPU frame over several seeds, on ONE GPU.

    python tools/shard_stat.py [--worlds 2 8] [--seeds 41 42 43 44 45] [--w 2560 --h 1440 --spp 2000]

For each seed and world size N, renders the N shares of crt_amd/dist.py's plan one after another (rank g: shard_spp
samples from subsequence family g*W*H), sums them in rank order (what the collective does), and compares the sum
with the 1-GPU frame of the same seed (family 0) and with an independent 1-GPU frame (family N*W*H): the RMS ratio
against sqrt(2) x noise x sqrt(1 - spp_0/spp), and the frame-mean difference in standard errors, on the linear values
and on the displayed ones (writeColor's gamma and clamp).  Over several seeds the z values should look like |N(0,1)|
draws if the sharded estimator is unbiased; a bias shows as the same sign and a growing z on every seed.
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
ap.add_argument("--worlds", type=int, nargs="+", default=[2, 8])
ap.add_argument("--seeds", type=int, nargs="+", default=[41, 42, 43, 44, 45])
a = ap.parse_args()
W, H = a.w, a.h
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H)
r.set_camera(crt_amd.camera(a.spp))
scale = np.float64(crt_amd.pixel_sample_scale(a.spp))


def frame(seed, base, spp):
    r.init_rand(seed, base)
    r.render(sc, spp, 20)
    r.synchronize()
    return r.linear().astype(np.float64).reshape(-1, 3)


def z_of(x, y):
    d = x - y
    return np.abs(d.mean(0)) / (d.std(0) / np.sqrt(d.shape[0])), np.sign(d.mean(0))


shown = lambda f: np.clip(np.sqrt(np.maximum(f, 0.0)), 0.0, 0.999)  # noqa: E731
for seed in a.seeds:
    f1 = frame(seed, 0, a.spp) * scale
    for n in a.worlds:
        fn = np.zeros_like(f1, dtype=np.float32).astype(np.float64)
        acc = np.zeros(f1.shape, np.float32)
        for g in range(n):
            acc = (acc + frame(seed, subsequence_base(g, W, H), shard_spp(a.spp, n, g)).astype(np.float32)).astype(np.float32)
        fn = acc.astype(np.float64) * scale
        f1b = frame(seed, n * W * H, a.spp) * scale
        shared = shard_spp(a.spp, n, 0) / a.spp
        ratio = np.sqrt(((fn - f1) ** 2).mean(0)) / (np.sqrt(((f1b - f1) ** 2).mean(0)) * np.sqrt(1 - shared))
        zl, sl = z_of(fn, f1)
        zc, sc_ = z_of(f1b, f1)
        zd, sd = z_of(shown(fn), shown(f1))
        zdc, _ = z_of(shown(f1b), shown(f1))
        print(json.dumps({"seed": seed, "world": n, "rms_over_expected": np.round(ratio, 4).tolist(),
                          "z_linear": np.round(zl, 2).tolist(), "sign_linear": sl.astype(int).tolist(),
                          "z_linear_control": np.round(zc, 2).tolist(),
                          "z_displayed": np.round(zd, 2).tolist(), "sign_displayed": sd.astype(int).tolist(),
                          "z_displayed_control": np.round(zdc, 2).tolist()}), flush=True)
