"""Per-rank cost of the spp-sharded frame, measured on ONE GPU.

Rank g of N renders shard_spp(spp, N, g) samples of every pixel from the RNG subsequence family pixel + g*W*H
(crt_amd/dist.py), then the framebuffer reduce and rank 0's resolve.  This renders exactly those shares one after
another on one GPU and reports, per (N, g): the end-to-end share (RNG reset + render + resolve, HIP events on the
launch stream), the render alone, its probe + tile-sort phase and the main kernel.  The ideal share is the N = 1 frame
divided by N; the ratio is the strong-scaling efficiency before the collective.

    python tools/rank_share.py [--worlds 1 2 4 8] [--reps 3] [--all-ranks 8]
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import torch  # noqa: E402

import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402
from crt_amd.dist import shard_spp, subsequence_base  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--width", type=int, default=2560)
ap.add_argument("--height", type=int, default=1440)
ap.add_argument("--spp", type=int, default=2000)
ap.add_argument("--bounces", type=int, default=20)
ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--all-ranks", type=int, default=8, help="also time every rank of this world size once")
ap.add_argument("--probe-stride", type=int, default=0, help="variant 8's probe stride (crt_renderer_set_schedule; 0 = auto)")
ap.add_argument("--pixel-groups", type=int, default=1,
                help="P > 1: rank g renders pixel group g %% P (every P-th tile of the cost order, crt_renderer_set_pixel_shard) "
                     "with the spp share g // P of world/P spp groups")
a = ap.parse_args()

W, H = a.width, a.height
hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H, 0)
r.set_camera(crt_amd.camera(a.spp))
if a.probe_stride:
    r.set_schedule(-1, 64, probe_stride=a.probe_stride)
scale = crt_amd.pixel_sample_scale(a.spp)


def share(world: int, g: int) -> dict:
    P = a.pixel_groups if world % a.pixel_groups == 0 and world > 1 else 1
    gs, Q = g // P, world // P
    spp = shard_spp(a.spp, Q, gs)
    base = subsequence_base(gs, W, H)
    r.set_pixel_shard(g % P, P)
    r.init_rand(41, base)        # first init of this (seed, base) runs the jump kernel; the timed ones copy the cache
    r.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    e0.record()
    r.init_rand(41, base)
    r.render(sc, spp, a.bounces)
    r.resolve(scale)
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    ph = r.last_timings()
    r.set_pixel_shard(0, 1)
    return {"world": world, "rank": g, "pixel_groups": P, "spp": spp, "end_to_end_ms": round(e0.elapsed_time(e1), 3),
            "wall_ms": round(wall * 1e3, 3), "render_ms": round(ph["render_ms"], 3),
            "probe_sort_ms": round(ph["probe_sort_ms"], 3), "main_kernel_ms": round(ph["main_kernel_ms"], 3),
            "kernel": r.last_kernel_name(), "rays": r.counters()["rays"]}


share(1, 0)   # warm-up
rows = {}
for world in a.worlds:
    reps = [share(world, 0) for _ in range(a.reps)]
    best = min(reps, key=lambda x: x["end_to_end_ms"])
    best["end_to_end_ms_reps"] = [x["end_to_end_ms"] for x in reps]
    rows[world] = best
    print(json.dumps(best), flush=True)
one = rows.get(1)
if one:
    for world, x in rows.items():
        x["efficiency_vs_n1"] = round(one["end_to_end_ms"] / world / x["end_to_end_ms"], 4)
        x["main_kernel_efficiency_vs_n1"] = round(one["main_kernel_ms"] / world / x["main_kernel_ms"], 4)
summary = {"rank0": list(rows.values())}
if a.all_ranks > 1:
    ranks = [share(a.all_ranks, g) for g in range(a.all_ranks)]
    summary["all_ranks"] = ranks
    summary["all_ranks_max_over_min"] = round(max(x["end_to_end_ms"] for x in ranks)
                                              / min(x["end_to_end_ms"] for x in ranks), 4)
print(json.dumps(summary, indent=1), flush=True)
