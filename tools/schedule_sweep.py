"""Variant 8's schedule knobs on one rank share of the spp-sharded frame, interleaved on one GPU.

Rank g of N renders shard_spp(spp, N, g) samples per pixel from subsequence base g*W*H.  For each setting this renders
that share `reps` times, the settings interleaved round by round, and prints per setting the main kernel's HIP-event
time (best and median), the render with the probe and tile sort, and the rays.  Settings are
`name:key=value,key=value` with keys crit (critical tiles, -1 = auto), lanes (their threshold), T (regeneration
threshold), occ (waves per SIMD, 0 = auto), stride (probe stride, 0 = auto), probe (probe spp, -1 = auto), wd (the wave
drain in 64ths, crt_renderer_set_wave_drain).  Results
never depend on them; the ray count is printed so that a setting that changed the work would show.

    python tools/schedule_sweep.py --world 8 --set base: crit0:crit=0 crit2k:crit=2048 T40:T=40 occ6:occ=6
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402
from crt_amd.dist import shard_spp, subsequence_base  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--width", type=int, default=2560)
ap.add_argument("--height", type=int, default=1440)
ap.add_argument("--spp", type=int, default=2000)
ap.add_argument("--bounces", type=int, default=20)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--set", nargs="+", default=["base:"])
a = ap.parse_args()

DEFAULT = {"crit": -1, "lanes": 16, "T": 44, "occ": 0, "stride": 0, "probe": -1, "wd": 48}
settings = []
for s in a.set:
    name, _, kv = s.partition(":")
    d = dict(DEFAULT)
    for item in filter(None, kv.split(",")):
        k, _, v = item.partition("=")
        if k not in d:
            raise SystemExit(f"unknown key {k!r} in {s!r}")
        d[k] = int(v)
    settings.append((name, d))

W, H = a.width, a.height
hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(W, H, 0)
r.set_camera(crt_amd.camera(a.spp))
spp = shard_spp(a.spp, a.world, a.rank)
base = subsequence_base(a.rank, W, H)


def run(d: dict) -> dict:
    r.set_schedule(d["probe"], 64, probe_stride=d["stride"])
    r.set_critical_tiles(d["crit"], d["lanes"])
    r.set_regen_threshold(d["T"])
    r.set_occupancy_target(d["occ"])
    r.set_wave_drain(d["wd"])
    r.init_rand(41, base)
    r.render(sc, spp, a.bounces)
    r.synchronize()
    t = r.last_timings()
    return {"main": t["main_kernel_ms"], "render": t["render_ms"], "probe": t["probe_sort_ms"],
            "rays": r.counters()["rays"], "kernel": r.last_kernel_name()}


run(settings[0][1])   # warm-up (and the RNG jump for this base)
res = {name: [] for name, _ in settings}
for _ in range(a.reps):
    for name, d in settings:
        res[name].append(run(d))
ref_main = None
for name, d in settings:
    xs = res[name]
    mains = [x["main"] for x in xs]
    out = {"name": name, **{k: v for k, v in d.items() if v != DEFAULT[k]}, "world": a.world, "rank": a.rank,
           "spp": spp, "main_best_ms": round(min(mains), 3), "main_median_ms": round(statistics.median(mains), 3),
           "render_best_ms": round(min(x["render"] for x in xs), 3), "probe_ms": round(xs[-1]["probe"], 3),
           "rays": xs[-1]["rays"], "kernel": xs[-1]["kernel"], "main_ms_reps": [round(m, 3) for m in mains]}
    if ref_main is None:
        ref_main = out["main_median_ms"]
    out["vs_first"] = round(out["main_median_ms"] / ref_main - 1, 4)
    print(json.dumps(out), flush=True)
