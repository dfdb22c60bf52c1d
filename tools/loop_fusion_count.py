"""The regeneration pass's rejection loops, counted per wave (profiling build only; VERDICT r5 item 2's prediction).

    tools/build_profile_lib.sh loops -DCRT_PROFILE_LOOPS
    CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/loops/libcrt_hip.so python tools/loop_fusion_count.py [--spp 256]

Variant 8's pass runs shade's unit-sphere loop (Utility.cuh:45-53) and next_ray's unit-disk loop (Utility.cuh:55-62)
back to back, so a wave pays max(sphere candidates) + max(disk candidates) over its parked lanes.  One fused loop in
which each lane advances its own phase would pay max(sphere + disk candidates).  The build counts both per pass from
the XORWOW draw counter (crt_hip.hip, CRT_PROFILE_LOOPS); this reports the sums and the predicted VALU saving with the
per-iteration costs of the ISA census (a sphere candidate: 3 draws + length test; a disk candidate: 2 draws + test).
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import _lib, assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=256)
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--base", type=int, default=0)
ap.add_argument("--valu-sphere-iter", type=float, default=40.0, help="VALU per unit-sphere candidate (ISA census)")
ap.add_argument("--valu-disk-iter", type=float, default=26.0, help="VALU per unit-disk candidate (ISA census)")
ap.add_argument("--valu-per-ray", type=float, default=41.16, help="VALU wave-instructions per ray (PMC, r05p)")
a = ap.parse_args()
L = _lib.hip()
L.crt_profile_loop_counts.argtypes = [C.c_void_p, C.c_int]
hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
buf = np.zeros(8, np.uint64)
for k in range(2):
    _lib.check(L.crt_profile_loop_counts(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_loop_counts")
    r.init_rand(41, a.base)
    r.render(sc, a.spp, 20)
    r.synchronize()
_lib.check(L.crt_profile_loop_counts(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_loop_counts")
passes, m1, m2, m12, m1r2, s1, s2, parked = (int(v) for v in buf)
rays = r.counters()["rays"]
# a fused loop pays 3-draw iterations while any lane is still drawing sphere candidates (max k1 of them) and 2-draw
# iterations for the rest of the longest lane's sum; the loops as built pay max k1 sphere and max k2 disk iterations
cur = a.valu_sphere_iter * m1 + a.valu_disk_iter * m2
fused = a.valu_sphere_iter * m1 + a.valu_disk_iter * max(0, m12 - m1)
saved_per_ray = (cur - fused) / rays
print(json.dumps({
    "kernel": r.last_kernel_name(), "w": a.w, "h": a.h, "spp": a.spp, "scene": a.scene, "rays": rays,
    "passes": passes, "parked_lanes_per_pass": round(parked / passes, 2),
    "per_pass": {"max_sphere_candidates": round(m1 / passes, 3), "max_disk_candidates": round(m2 / passes, 3),
                 "max_sphere_plus_disk": round(m12 / passes, 3), "max_sphere_rr_disk": round(m1r2 / passes, 3),
                 "mean_sphere_candidates_per_parked_lane": round(s1 / parked, 3),
                 "mean_disk_candidates_per_parked_lane": round(s2 / parked, 3)},
    "loop_lane_fill": {"sphere": round(s1 / max(1, 64 * m1), 3), "disk": round(s2 / max(1, 64 * m2), 3)},
    "valu_per_ray": {"loops_as_built": round(cur / rays, 3), "fused_loop": round(fused / rays, 3),
                     "saved": round(saved_per_ray, 3),
                     "saved_share_of_kernel": round(saved_per_ray / a.valu_per_ray, 4)},
    "note": "VALU per candidate from the ISA census (next_u32 + uniform + rand_pm1 per draw, length test); a fused "
            "loop also pays the phase bookkeeping and its live state, which this upper bound leaves out"}))
