"""A/B bit-identity check: hashes of frames, RNG state and work counters for a set of renders.

    CRT_HIP_LIB=<lib> python tools/frame_hash.py [--big]

Run once per library build (tools/build_profile_lib.sh); identical output lines mean identical bits.  The cases
cover the 4-wide kernels (variants 4, 7, 8, with and without the cost probe, the counting kernel) on the rebuilt
BVH and variant 10 on the reference BVH; --big adds a 2560x1440 frame at 16 spp.
"""
import argparse
import hashlib
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--big", action="store_true")
ap.add_argument("--occupancy", type=int, default=0, help="crt_renderer_set_occupancy_target (0 = the library's default)")
ap.add_argument("--xcd-regions", type=int, default=0, help="crt_renderer_set_xcd_regions (variant 8 tile order)")
ap.add_argument("--probe-stride", type=int, default=0, help="variant 8's probe stride (crt_renderer_set_schedule; 0 = auto)")
ap.add_argument("--drain", type=int, default=0, help="variant 7's drain threshold (crt_renderer_set_drain_threshold)")
ap.add_argument("--wave-drain", type=int, default=0, help="variants 4/8 wave drain in 64ths (crt_renderer_set_wave_drain)")
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
wide = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
ref = hs.upload(0)
cases = [("w4", 104, 45, 64, 8, False), ("w4", 104, 45, 64, 4, False), ("w4", 160, 90, 8, 7, False),
         ("w4", 100, 37, 70, 8, False), ("w4", 96, 54, 4, 8, True), ("w4", 96, 54, 4, 4, True),
         ("ref", 96, 64, 64, 10, False)]
if a.big:
    cases.append(("w4", 2560, 1440, 16, 8, False))
for sc_name, w, h, spp, var, count in cases:
    r = crt_amd.Renderer(w, h)
    r.set_kernel_variant(var)
    if a.occupancy:
        r.set_occupancy_target(a.occupancy)
    if a.xcd_regions:
        r.set_xcd_regions(1)
    if a.probe_stride:
        r.set_schedule(-1, 64, probe_stride=a.probe_stride)
    if a.drain:
        r.set_drain_threshold(a.drain)
    if a.wave_drain:
        r.set_wave_drain(a.wave_drain)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41)
    r.render(wide if sc_name == "w4" else ref, spp, 20, count_work=count)
    r.synchronize()
    hsh = hashlib.sha256()
    hsh.update(r.linear().tobytes())
    hsh.update(r.rng_state().tobytes())
    c = r.counters()
    keys = ("rays", "box_tests", "tri_tests", "sphere_tests", "paths") if count else ("rays",)
    print(f"{sc_name} {w}x{h} {spp}spp v{var} count={int(count)}: {hsh.hexdigest()[:16]} "
          + " ".join(f"{k}={c[k]}" for k in keys), flush=True)
