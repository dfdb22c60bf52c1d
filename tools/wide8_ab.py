"""Round 5's wide-node A/B (round-4 verdict item 4): the 4-wide tree (variant 8) against the 8-wide tree (variant 12,
the same program over two-record nodes), same binary SAH build, same scene, same renderer, interleaved in one process.

    git apply profiles/r05v/wide8.patch && make -C raytracer-cuda_amd lib/libcrt_hip.so
    python tools/wide8_ab.py [--configs C,E] [--reps 3] [--parity-only] [--skip-parity] [--w8-occupancy 6]

The 8-wide kernel was measured and reverted (profiles/r05v): the shipped library rejects width 8, so this
tool needs the patch applied first.

Part 1 (parity): small frames of cornell_bunny on both trees must give bit-identical frames, RNG state and ray counts
(the closest hit does not depend on the tree).  Part 2 (speed): the bench's configs C and E at their full size, main
render kernel ms (HIP events) per width, interleaved.  One JSON line per measurement.
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
           "E": ("cornell_1m", 2560, 1440, 512)}

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C,E")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--parity-only", action="store_true")
ap.add_argument("--w8-occupancy", type=int, default=0, help="occupancy target of the 8-wide renders (0 = the library's)")
ap.add_argument("--skip-parity", action="store_true")
a = ap.parse_args()


def out(**kw):
    print(json.dumps(kw), flush=True)


def frame_hash(r):
    h = hashlib.sha256()
    h.update(r.linear().tobytes())
    h.update(r.rng_state().tobytes())
    return h.hexdigest()[:16]


def upload(hs, width):
    return hs.upload(0, bvh="rebuilt", width=width, leaf_size=4, traversal_cost=2.0, gpu_build=True)


hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
trees = {w: upload(hs, w) for w in (4, 8)}
for w, sc in trees.items():
    out(part="tree", scene="cornell_bunny", width=w, stats={k: v for k, v in sc.stats().items()})
bad = 0
PARITY = ((104, 45, 64, False), (160, 90, 8, False), (96, 54, 4, True), (100, 37, 70, True), (640, 360, 16, False))
for w_px, h_px, spp, count in (() if a.skip_parity else PARITY):
    res = {}
    for w, sc in trees.items():
        r = crt_amd.Renderer(w_px, h_px)
        r.set_camera(crt_amd.camera(spp))
        r.init_rand(41)
        r.render(sc, spp, 20, count_work=count)
        r.synchronize()
        c = r.counters()
        res[w] = (frame_hash(r), c["rays"], c.get("paths"), c.get("box_tests"), c.get("tri_tests"), r.last_kernel_name())
    same = res[4][:3] == res[8][:3]
    bad += not same
    out(part="parity", frame=f"{w_px}x{h_px} {spp}spp count={int(count)}", identical=same,
        w4=res[4], w8=res[8])
if bad:
    out(part="parity", error=f"{bad} frames differ between the 4- and 8-wide trees")
    sys.exit(1)
if a.parity_only:
    sys.exit(0)
del trees, hs

for cfg in a.configs.split(","):
    scene, W, H, spp = CONFIGS[cfg]
    hs = crt_amd.HostScene(assets.scene_files(scene), build_device=0)
    trees = {w: upload(hs, w) for w in (4, 8)}
    r = crt_amd.Renderer(W, H)
    r.set_camera(crt_amd.camera(spp))
    hashes = {}
    for rep in range(a.reps + 1):   # rep 0 is the warm-up
        for w in ((4, 8) if rep % 2 == 0 else (8, 4)):
            r.set_occupancy_target(a.w8_occupancy if w == 8 else 0)
            r.init_rand(41)
            r.render(trees[w], spp, 20)
            r.synchronize()
            ph = r.last_timings()
            hashes.setdefault(w, frame_hash(r))
            out(part="speed", config=cfg, rep=rep, width=w, kernel=r.last_kernel_name(),
                main_kernel_ms=round(ph["main_kernel_ms"], 3), render_ms=round(ph["render_ms"], 3),
                probe_sort_ms=round(ph["probe_sort_ms"], 3), rays=r.counters()["rays"])
    out(part="speed", config=cfg, frames_identical=hashes[4] == hashes[8], hashes=hashes)
    del trees, hs, r
