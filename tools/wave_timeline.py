"""Occupancy timeline of one render launch (profiling build with -DCRT_PROFILE_WAVE_TIMES).

Every wave records its start and end (s_memrealtime, 100 MHz).  From them: the launch span, the peak number of
resident waves, and how much of (span x peak) the waves actually occupied.  The shortfall at the end of the
launch is the tail: the last workgroups run while the rest of the chip is idle.

    CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so python tools/wave_timeline.py [--spp 2000]
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
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--w", type=int, default=2560)
ap.add_argument("--h", type=int, default=1440)
ap.add_argument("--spp", type=int, default=2000)
ap.add_argument("--bvh", default="rebuilt")
ap.add_argument("--variant", type=int, default=4)
ap.add_argument("--persistent-waves", type=int, default=256 * 6 * 4, help="variant 7: resident waves launched")
ap.add_argument("--temporal", action="store_true",
                help="variant 7: render a first frame, then time the second with its tiles ordered by the first's "
                     "rays per pixel (crt_renderer_set_temporal_order)")
ap.add_argument("--drain", type=int, default=0, help="variant 7's drain threshold (crt_renderer_set_drain_threshold)")
ap.add_argument("--wave-drain", type=int, default=48, help="variants 4/8 wave drain in 64ths (crt_renderer_set_wave_drain)")
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene))
sc = hs.upload(0, bvh=a.bvh, width=4, leaf_size=4, traversal_cost=2.0) if a.bvh == "rebuilt" else hs.upload(0)
r = crt_amd.Renderer(a.w, a.h)
r.set_kernel_variant(a.variant)
r.set_drain_threshold(a.drain)
r.set_wave_drain(a.wave_drain)
r.set_camera(crt_amd.camera(a.spp))
r.init_rand(41)
if a.temporal:
    r.set_temporal_order(True)
    r.render(sc, a.spp, 20)        # records the rays per pixel the timed frame orders its tiles by
r.render(sc, a.spp, 20)
r.synchronize()
kernel_ms = r.last_kernel_ms()
n_waves = (((a.w + 7) // 8) * ((a.h + 7) // 8) if a.variant == 8 else
           a.persistent_waves if a.variant == 7 else ((a.w + 15) // 16) * ((a.h + 15) // 16) * 4)
L = _lib.hip()
L.crt_profile_wave_times.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros((n_waves, 2), np.uint64)
_lib.check(L.crt_profile_wave_times(buf.ctypes.data_as(C.c_void_p), n_waves), "crt_profile_wave_times")
t = (buf.astype(np.int64) - int(buf[:, 0].min())) / 100.0   # 100 MHz ticks -> microseconds
start, end = t[:, 0], t[:, 1]
span = float(end.max())
ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
active = np.cumsum(ev[:, 1])
peak = int(active.max())
busy = float((end - start).sum())
eff = busy / (span * peak)
# time after which fewer than 95 % of the peak waves are resident, to the end
times = ev[:, 0]
below = np.nonzero(active < 0.95 * peak)[0]
steady_end = float(times[below[below > np.argmax(active)][0]]) if len(below[below > np.argmax(active)]) else span
dur = end - start
# resident waves in 20 equal time bins
bins = np.linspace(0, span, 21)
occ = []
for i in range(20):
    lo, hi = bins[i], bins[i + 1]
    ov = np.clip(np.minimum(end, hi) - np.maximum(start, lo), 0, None).sum() / (hi - lo)
    occ.append(round(float(ov), 1))
out = {"scene": a.scene, "bvh": a.bvh, "variant": a.variant, "temporal": a.temporal, "drain": a.drain, "wave_drain": a.wave_drain, "kernel": r.last_kernel_name(), "spp": a.spp, "kernel_ms": round(kernel_ms, 3), "span_ms": round(span / 1e3, 3),
       "waves": n_waves, "peak_resident_waves": peak, "occupancy_efficiency": round(eff, 4),
       "tail_ms": round((span - steady_end) / 1e3, 3), "tail_fraction": round((span - steady_end) / span, 4),
       "wave_ms": {"min": round(float(dur.min()) / 1e3, 3), "median": round(float(np.median(dur)) / 1e3, 3),
                   "max": round(float(dur.max()) / 1e3, 3)},
       "resident_waves_per_twentieth": occ}
if a.variant == 8:
    # variant 8 runs block b on the b-th tile of the cost order, so the waves' durations in block order show how well
    # the probe ranked the tiles.  Greedy list schedules over `peak` slots (a slot takes the next block when it frees):
    # in block order (checks the model against the measured span) and in the order of the measured durations (the
    # span a perfect cost probe would give).
    import heapq

    def list_schedule(d):
        slots = [0.0] * peak
        for x in d:
            heapq.heapreplace(slots, slots[0] + x)
        return max(slots)

    tail = np.nonzero(end > steady_end)[0]
    out["order"] = {"model_span_ms_block_order": round(list_schedule(dur) / 1e3, 3),
                    "model_span_ms_true_lpt": round(list_schedule(np.sort(dur)[::-1]) / 1e3, 3),
                    "tail_waves": int(len(tail)),
                    "tail_block_quantiles": [round(float(q) / n_waves, 4) for q in
                                             np.quantile(tail, [0.1, 0.5, 0.9])] if len(tail) else [],
                    "tail_wave_ms_median": round(float(np.median(dur[tail])) / 1e3, 3) if len(tail) else 0.0,
                    "last_ending_blocks": [int(b) for b in np.argsort(end)[-8:][::-1]],
                    "wave_ms_by_block_decile": [round(float(np.median(x)) / 1e3, 3) for x in np.array_split(dur, 10)]}
print(json.dumps(out))
