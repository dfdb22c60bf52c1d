"""Section profile of the TIMED render kernel (profiling build only; VERDICT r5 item 3's dynamic breakdown).

    tools/build_profile_lib.sh pass -DCRT_PROFILE_PASS
    CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/pass/libcrt_hip.so python tools/pass_profile.py [--spp 256]

The counting kernel's section timers (tools/section_profile.py) run in the counting kernel, which is slower and
schedules differently; this build keeps the same s_memtime timers in the timed variant-8 kernel and splits the
regeneration pass into its parts: finish_ray (the per-ray spheres, then shade), next_ray, the new ray's set-up (1/d,
rows, LDS ray record), the LDS root step (top_steps) and the rest (live mask, ray count); plus the loop head (the
parked / live ballots and the drain rule), the node steps and the leaf rounds.  Shares of the wave cycles summed over
waves; the timers add a few instructions per section, so the kernel is somewhat slower than the shipped one.

    tools/build_profile_lib.sh passcrit -DCRT_PROFILE_PASS -DCRT_PROFILE_PASS_FIRST=1

keeps only the first workgroup of the tile order, the most expensive tile: on config B (1280x720, 256 spp) its wave
lasts the whole launch, so its iterations are the frame's critical chain.
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
a = ap.parse_args()
L = _lib.hip()
L.crt_profile_pass_sections.argtypes = [C.c_void_p, C.c_int]
hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
buf = np.zeros(20, np.uint64)
for k in range(2):   # the first frame warms up
    _lib.check(L.crt_profile_pass_sections(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_pass_sections")
    r.init_rand(41, a.base)
    r.render(sc, a.spp, 20)
    r.synchronize()
_lib.check(L.crt_profile_pass_sections(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_pass_sections")
step, rnd, regen, finish, sph, nxt, setup_and_next, top, head, passes, waves, life, n_steps, n_rounds, wrays, \
    row_wait, prim_wait = (int(v) for v in buf[:17])
setup = setup_and_next - nxt
rest = regen - finish - nxt - setup - top
tot = step + rnd + regen + head
rays = r.counters()["rays"]
sh = lambda v: round(v / tot, 4)  # noqa: E731
print(json.dumps({
    "kernel": r.last_kernel_name(), "w": a.w, "h": a.h, "spp": a.spp, "scene": a.scene, "rays": rays,
    "main_kernel_ms": round(r.last_timings()["main_kernel_ms"], 3), "waves_profiled": waves,
    "wave_lifetime_cycles_per_wave": round(life / max(1, waves)), "sections_over_lifetime": round(tot / max(1, life), 4),
    "per_wave": {"iterations (node steps)": round(n_steps / max(1, waves), 1),
                 "leaf rounds": round(n_rounds / max(1, waves), 1), "passes": round(passes / max(1, waves), 1),
                 "rays": round(wrays / max(1, waves), 1)},
    "cycles_per_iteration": round(tot / max(1, n_steps), 1),
    "cycles_per_iteration_by_section": {"node step": round(step / max(1, n_steps), 1),
                                        "leaf rounds": round(rnd / max(1, n_steps), 1),
                                        "loop head": round(head / max(1, n_steps), 1),
                                        "pass": round(regen / max(1, n_steps), 1)},
    "cycles_per_leaf_round": round(rnd / max(1, n_rounds), 1),
    # -DCRT_PROFILE_ROWS builds only (0 otherwise): the loads' issue-to-data cycles, per node step / leaf round
    "row_wait_cycles_per_iteration": round(row_wait / max(1, n_steps), 1),
    "prim_wait_cycles_per_leaf_round": round(prim_wait / max(1, n_rounds), 1),
    "wave_cycles_per_ray": round(tot / rays, 1), "passes_per_wave": round(passes / max(1, waves), 1),
    "share": {"node steps": sh(step), "leaf rounds": sh(rnd), "loop head (ballots, drain rule)": sh(head),
              "pass": sh(regen), "  per-ray spheres": sh(sph), "  shade": sh(finish - sph), "  next_ray": sh(nxt),
              "  new-ray set-up": sh(setup), "  LDS root step": sh(top), "  rest (live mask, ray count)": sh(rest)},
    "wave_cycles_per_pass": {"per-ray spheres": round(sph / passes, 1), "shade": round((finish - sph) / passes, 1),
                             "next_ray": round(nxt / passes, 1), "new-ray set-up": round(setup / passes, 1),
                             "LDS root step": round(top / passes, 1), "rest": round(rest / passes, 1)}}, indent=1))
