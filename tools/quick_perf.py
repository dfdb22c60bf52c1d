"""Dev probe: time the render kernel on a config at a given spp (no oracle)."""
import argparse
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--bounces", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--count", action="store_true")
ap.add_argument("--variants", default="0,1,2")
ap.add_argument("--thresholds", default="32")
ap.add_argument("--occupancy", default="1")
a = ap.parse_args()

t = time.time()
hs, sc = crt_amd.load_scene(assets.scene_files(a.scene))
print("scene", a.scene, "load+build+upload %.2fs" % (time.time() - t), sc.stats(), flush=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
variants = [(int(v), int(th), int(oc)) for v in a.variants.split(",")
            for th in (a.thresholds.split(",") if v in ("2", "3") else ["32"])
            for oc in (a.occupancy.split(",") if v in ("2", "3") else ["1"])]
for i in range(a.reps):
    for var, th, oc in variants:          # interleaved A/B in one process
        r.set_kernel_variant(var)
        r.set_regen_threshold(th)
        r.set_occupancy_target(oc)
        r.init_rand(41)
        t = time.time()
        r.render(sc, a.spp, a.bounces)
        r.synchronize()
        dt = time.time() - t
        c = r.counters()
        print(f"rep {i} variant {var} T={th} W={oc}: wall {dt*1e3:.1f} ms kernel {r.last_kernel_ms():.1f} ms rays {c['rays']} "
              f"-> {c['rays']/r.last_kernel_ms()/1e3:.1f} Mrays/s", flush=True)
if a.count:
    r.set_kernel_variant(variants[-1][0])
    r.set_regen_threshold(variants[-1][1])
    r.set_occupancy_target(variants[-1][2])
    r.init_rand(41)
    r.render(sc, a.spp, a.bounces, count_work=True)
    r.synchronize()
    c = r.counters()
    print("counting kernel", r.last_kernel_ms(), "ms", c,
          {k: c[k] / c["rays"] for k in ("box_tests", "tri_tests", "sphere_tests")})
    st = r.schedule_stats()
    print("schedule", st, "step utilisation %.3f" % (c["box_tests"] / max(1, st["step_lane_slots"])),
          "round utilisation %.3f" % (c["tri_tests"] / max(1, st["round_lane_slots"])),
          "rays per wave trace call %.1f" % (c["rays"] / max(1, st["wave_trace_calls"])),
          "steps per wave trace call %.1f" % (st["step_lane_slots"] / 64 / max(1, st["wave_trace_calls"])))
