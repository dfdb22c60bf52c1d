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
a = ap.parse_args()

t = time.time()
hs, sc = crt_amd.load_scene(assets.scene_files(a.scene))
print("scene", a.scene, "load+build+upload %.2fs" % (time.time() - t), sc.stats(), flush=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
for i in range(a.reps):
    r.init_rand(41)
    t = time.time()
    r.render(sc, a.spp, a.bounces)
    r.synchronize()
    dt = time.time() - t
    c = r.counters()
    print(f"rep {i}: wall {dt*1e3:.1f} ms kernel {r.last_kernel_ms():.1f} ms rays {c['rays']} "
          f"-> {c['rays']/r.last_kernel_ms()/1e3:.1f} Mrays/s", flush=True)
if a.count:
    r.init_rand(41)
    r.render(sc, a.spp, a.bounces, count_work=True)
    r.synchronize()
    c = r.counters()
    print("counting kernel", r.last_kernel_ms(), "ms", c,
          {k: c[k] / c["rays"] for k in ("box_tests", "tri_tests", "sphere_tests")})
