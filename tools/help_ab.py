"""Helper-lane A/B (round 5, experiment): variant 8 with CRT_HELPER_TILES = each given value, interleaved in one process
(the library reads the variable per render), on configs B / C / E.  Frames, RNG state and ray counts must not depend
on it.

    git apply profiles/r05y/helpers.patch && make -C raytracer-cuda_amd all
    python tools/help_ab.py [--configs B,C] [--values 0,-1,1024] [--reps 3] [--parity]

Measured and not kept (profiles/r05y): without the patch the library ignores CRT_HELPER_TILES.
"""
import argparse
import hashlib
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

CONFIGS = {"B": ("cornell_bunny", 1280, 720, 256), "C": ("cornell_bunny", 2560, 1440, 2000),
           "E": ("cornell_1m", 2560, 1440, 512), "N8": ("cornell_bunny", 2560, 1440, 250)}
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="B,C")
ap.add_argument("--values", default="0,-1,1024")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--parity", action="store_true", help="small frames first, with and without the counting kernel")
a = ap.parse_args()
values = [int(v) for v in a.values.split(",")]


def out(**kw):
    print(json.dumps(kw), flush=True)


def frame_hash(r):
    h = hashlib.sha256()
    h.update(r.linear().tobytes())
    h.update(r.rng_state().tobytes())
    return h.hexdigest()[:16]


scenes = {}


def scene(name):
    if name not in scenes:
        hs = crt_amd.HostScene(assets.scene_files(name), build_device=0)
        scenes[name] = (hs, hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True))
    return scenes[name][1]


if a.parity:
    sc = scene("cornell_bunny")
    bad = 0
    for w, h, spp, count in ((104, 45, 64, False), (104, 45, 64, True), (320, 180, 64, False), (640, 360, 96, True)):
        res = {}
        for v in values:
            os.environ["CRT_HELPER_TILES"] = str(v)
            r = crt_amd.Renderer(w, h)
            r.set_kernel_variant(8)
            r.set_camera(crt_amd.camera(spp))
            r.init_rand(41)
            r.render(sc, spp, 20, count_work=count)
            r.synchronize()
            c = r.counters()
            res[v] = (frame_hash(r), c["rays"], c.get("paths"), c.get("box_tests"), c.get("tri_tests"))
        same = len({x[:3] for x in res.values()}) == 1
        bad += not same
        out(part="parity", frame=f"{w}x{h} {spp}spp count={int(count)}", identical=same, res={str(k): v for k, v in res.items()})
    if bad:
        out(part="parity", error=f"{bad} frames differ")
        sys.exit(1)

for cfg in a.configs.split(","):
    name, W, H, spp = CONFIGS[cfg]
    sc = scene(name)
    r = crt_amd.Renderer(W, H)
    r.set_camera(crt_amd.camera(spp))
    hashes = {}
    for rep in range(a.reps + 1):   # rep 0 is the warm-up
        order = values if rep % 2 == 0 else values[::-1]
        for v in order:
            os.environ["CRT_HELPER_TILES"] = str(v)
            r.init_rand(41)
            r.render(sc, spp, 20)
            r.synchronize()
            ph = r.last_timings()
            hashes.setdefault(v, frame_hash(r))
            out(part="speed", config=cfg, rep=rep, help=v, main_kernel_ms=round(ph["main_kernel_ms"], 3),
                rays=r.counters()["rays"])
    out(part="speed", config=cfg, frames_identical=len(set(hashes.values())) == 1, hashes={str(k): h for k, h in hashes.items()})
