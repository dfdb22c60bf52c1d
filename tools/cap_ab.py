"""The capped unit-sphere loop (crt_renderer_set_sphere_cap) A/B in one process, one library: for each config, the
main-kernel time of every cap setting, interleaved over reps, and the frame hash (linear sums + RNG state + rays), which
must not depend on the cap.  The counting kernel's work counters are compared too.

    python tools/cap_ab.py [--configs C,B,E,N8] [--caps 0,2,3,4] [--reps 3]
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
           "E": ("cornell_1m", 2560, 1440, 512), "N8": ("cornell_bunny", 2560, 1440, 250),
           "S": ("cornell_bunny", 640, 360, 64), "T": ("cornell_bunny", 97, 61, 33), "A": ("cornell", 256, 256, 16)}
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C,B,E,N8")
ap.add_argument("--caps", default="0,2,3,4")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--no-count", action="store_true")
a = ap.parse_args()
caps = [int(v) for v in a.caps.split(",")]


def frame_hash(r):
    h = hashlib.sha256()
    h.update(r.linear().tobytes())
    h.update(r.rng_state().tobytes())
    h.update(str(r.counters()["rays"]).encode())
    return h.hexdigest()[:16]


scenes = {}
for cfg in a.configs.split(","):
    name, W, H, spp = CONFIGS[cfg]
    if name not in scenes:
        hs = crt_amd.HostScene(assets.scene_files(name), build_device=0)
        scenes[name] = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    sc = scenes[name]
    r = crt_amd.Renderer(W, H)
    r.set_camera(crt_amd.camera(spp))
    hashes, counts = {}, {}
    for rep in range(a.reps + 1):
        for cap in (caps if rep % 2 == 0 else caps[::-1]):
            r.set_sphere_cap(cap)
            r.init_rand(41)
            r.render(sc, spp, 20)
            r.synchronize()
            ph = r.last_timings()
            hashes.setdefault(str(cap), frame_hash(r))
            print(json.dumps({"config": cfg, "rep": rep, "cap": cap, "kernel": r.last_kernel_name(),
                              "main_kernel_ms": round(ph["main_kernel_ms"], 3), "rays": r.counters()["rays"]}),
                  flush=True)
    if not a.no_count:
        for cap in caps:
            r.set_sphere_cap(cap)
            r.init_rand(41)
            r.render(sc, spp, 20, count_work=True)
            r.synchronize()
            c = r.counters()
            counts[str(cap)] = [c[k] for k in ("rays", "box_tests", "tri_tests", "sphere_tests", "paths")]
    same = len(set(hashes.values())) == 1 and len({tuple(v) for v in counts.values()}) <= 1
    print(json.dumps({"config": cfg, "hashes": hashes, "counts": counts, "identical": same}), flush=True)
