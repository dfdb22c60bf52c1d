"""Main-kernel time of variant 8 at forced occupancies, interleaved, for the automatic occupancy rule (r06t, r06u).

    python tools/occ_sweep.py --w 1366 --h 768 --spp 256 --occ 4 6 [--pixel-shard 0 8] [--rounds 2]

Each round renders one warm-up frame and two timed frames per occupancy (0 = the library's automatic choice) and prints
one JSON line per (round, occupancy): the kernel the library launched and its HIP-event time.
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
ap.add_argument("--w", type=int, default=1280)
ap.add_argument("--h", type=int, default=720)
ap.add_argument("--spp", type=int, default=256)
ap.add_argument("--occ", type=int, nargs="+", default=[0, 6])
ap.add_argument("--pixel-shard", type=int, nargs=2, default=None, metavar=("S", "N"))
ap.add_argument("--rounds", type=int, default=2)
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
tiles = ((a.w + 7) // 8) * ((a.h + 7) // 8) // (a.pixel_shard[1] if a.pixel_shard else 1)
for rnd in range(a.rounds):
    for occ in a.occ:
        r = crt_amd.Renderer(a.w, a.h)
        if occ:
            r.set_occupancy_target(occ)
        if a.pixel_shard:
            r.set_pixel_shard(*a.pixel_shard)
        r.set_camera(crt_amd.camera(a.spp))
        ms = []
        for k in range(3):
            r.init_rand(41)
            r.render(sc, a.spp, 20)
            r.synchronize()
            if k:
                ms.append(r.last_kernel_ms())
        print(json.dumps({"round": rnd, "w": a.w, "h": a.h, "spp": a.spp, "pixel_shard": a.pixel_shard, "tiles": tiles,
                          "occupancy": occ, "kernel": r.last_kernel_name(), "main_kernel_ms": round(sum(ms) / len(ms), 3),
                          "schedule": r.last_schedule()}),
              flush=True)
