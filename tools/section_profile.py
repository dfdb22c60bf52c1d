"""Section profile of the counting render kernel (s_memtime per section, summed over waves; crt_renderer_get_section_profile_ex).

    python tools/section_profile.py [--spp 256] [--w 2560] [--h 1440] [--variant 8]

Prints the share of wave-cycles spent in the regeneration passes (split into the per-ray spheres, shade(), next_ray()
and the rest: ballots, 1/d, LDS ray record), the traversal steps and the leaf rounds, plus the lane-slot fill of the
steps and rounds.  The counting kernel is slower than the timed one (its clock reads and counters), so the shares
are indicative; the timed kernel's totals come from bench.py / rocprofv3.
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
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=256)
ap.add_argument("--bounces", type=int, default=20)
ap.add_argument("--variant", type=int, default=8)
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_kernel_variant(a.variant)
r.set_camera(crt_amd.camera(a.spp))
r.init_rand(41)
r.render(sc, a.spp, a.bounces, count_work=True)
r.synchronize()
c = r.counters()
p = r.section_profile()
s = r.schedule_stats()
tot = p["cyc_regen"] + p["cyc_step"] + p["cyc_round"]
rest = p["cyc_regen"] - p["cyc_shade"] - p["cyc_next"]
out = {
    "config": f"{a.scene} {a.w}x{a.h} {a.spp}spp {a.bounces}b variant {a.variant} (counting kernel {r.last_kernel_name()})",
    "kernel_ms": round(r.last_kernel_ms(), 2), "rays": c["rays"],
    "per_ray": {k: round(c[k] / c["rays"], 3) for k in ("box_tests", "tri_tests", "sphere_tests")},
    "share": {"regen": round(p["cyc_regen"] / tot, 4), "  spheres": round(p["cyc_sph"] / tot, 4),
              "  shade": round((p["cyc_shade"] - p["cyc_sph"]) / tot, 4), "  next_ray": round(p["cyc_next"] / tot, 4),
              "  rest": round(rest / tot, 4), "step": round(p["cyc_step"] / tot, 4),
              "round": round(p["cyc_round"] / tot, 4)},
    "passes_per_wave": round(p["passes"] / max(1, p["waves"]), 1),
    "wave_cycles_per_ray": round(tot / c["rays"], 1),
    "round_fill": round(c["tri_tests"] / max(1, s["round_lane_slots"]), 3),
    "wave_steps_per_ray": round(s["step_lane_slots"] / 64 / c["rays"], 4),
}
print(json.dumps(out, indent=1), flush=True)
