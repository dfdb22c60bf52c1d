"""The critical wave of a few-tiles frame over time (profiling build).

    tools/build_profile_lib.sh crit -DCRT_PROFILE_CRIT_TRACE -DCRT_PROFILE_WAVE_TIMES
    CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/crit/libcrt_hip.so python tools/crit_trace.py [--w 1280 --h 720 --spp 256]

The first workgroup of variant 8's tile order holds the most expensive tile; on config B (1280x720, 256 spp) its wave
lasts the whole launch, so the frame is its chain of loop iterations.  The build logs that wave's s_memrealtime every
16 iterations, and every wave's start, end and hardware slot (HW_ID: SIMD, CU, SH, SE; XCC_ID).  Per tenth of the
critical wave's life: microseconds per iteration, its live lanes, and the waves resident on its SIMD, on its CU and on
the chip.  If the late iterations (an emptied SIMD) are much faster than the early ones, the chain is paced by the
SIMD's other waves (issue and memory sharing); if not, by its own latency.
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
ap.add_argument("--w", type=int, default=1280)
ap.add_argument("--h", type=int, default=720)
ap.add_argument("--spp", type=int, default=256)
ap.add_argument("--bins", type=int, default=10)
ap.add_argument("--occupancy", type=int, default=0, help="crt_renderer_set_occupancy_target (0 = the library's rule)")
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
if a.occupancy:
    r.set_occupancy_target(a.occupancy)
L = _lib.hip()
L.crt_profile_crit_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
L.crt_profile_wave_times.argtypes = [C.c_void_p, C.c_int]
n_waves = ((a.w + 7) // 8) * ((a.h + 7) // 8)
trace = np.zeros((16384, 2), np.uint64)
hw = np.zeros((n_waves, 2), np.uint32)
for k in range(2):   # the first frame warms up; the trace is reset when read
    r.init_rand(41)
    r.render(sc, a.spp, 20)
    r.synchronize()
    _lib.check(L.crt_profile_crit_trace(trace.ctypes.data_as(C.c_void_p), hw.ctypes.data_as(C.c_void_p), n_waves),
               "crt_profile_crit_trace")
kname = r.last_kernel_name()
import hashlib  # noqa: E402
frame_hash = hashlib.sha256(r.linear().tobytes() + r.rng_state().tobytes()).hexdigest()[:16]
assert "8," in kname, kname
wt = np.zeros((n_waves, 2), np.uint64)
_lib.check(L.crt_profile_wave_times(wt.ctypes.data_as(C.c_void_p), n_waves), "crt_profile_wave_times")
t0 = int(wt[:, 0].min())
start = (wt[:, 0].astype(np.int64) - t0) / 100.0      # microseconds
end = (wt[:, 1].astype(np.int64) - t0) / 100.0
span = float(end.max())

# the critical wave = workgroup 0 of the order; its trace rows up to the last written one
rows = trace[trace[:, 0] > 0]
tt = (rows[:, 0].astype(np.int64) - t0) / 100.0
info = rows[:, 1].astype(np.int64)
live, parked, it = info & 0xff, (info >> 8) & 0xff, info >> 16

simd_key = (hw[:, 1].astype(np.int64) << 16) | (hw[:, 0].astype(np.int64) & 0xff30)   # XCC, SE, SH, CU, SIMD
cu_key = (hw[:, 1].astype(np.int64) << 16) | (hw[:, 0].astype(np.int64) & 0xff00)
same_simd = simd_key == simd_key[0]
same_cu = cu_key == cu_key[0]


def resident(mask, lo, hi):
    return float(np.clip(np.minimum(end[mask], hi) - np.maximum(start[mask], lo), 0, None).sum() / (hi - lo))


edges = np.linspace(start[0], end[0], a.bins + 1)
series = []
for i in range(a.bins):
    lo, hi = edges[i], edges[i + 1]
    sel = (tt >= lo) & (tt < hi)
    if sel.sum() < 2:
        continue
    d_it = float(it[sel][-1] - it[sel][0])
    d_t = float(tt[sel][-1] - tt[sel][0])
    series.append({"t_ms": [round(lo / 1e3, 2), round(hi / 1e3, 2)],
                   "us_per_iteration": round(d_t / max(1.0, d_it), 3),
                   "live_lanes": round(float(live[sel].mean()), 1),
                   "waves_on_its_simd": round(resident(same_simd, lo, hi), 2),
                   "waves_on_its_cu": round(resident(same_cu, lo, hi), 2),
                   "waves_on_chip": round(resident(np.ones(n_waves, bool), lo, hi), 1)})
out = {"kernel": kname, "w": a.w, "h": a.h, "spp": a.spp, "kernel_ms": round(r.last_kernel_ms(), 3),
       "span_ms": round(span / 1e3, 3), "critical_wave": {"start_ms": round(start[0] / 1e3, 3),
                                                          "end_ms": round(end[0] / 1e3, 3),
                                                          "iterations": int(it[-1]) if len(it) else 0,
                                                          "longest_wave": bool(np.argmax(end - start) == 0)},
       "waves_sharing_its_simd": int(same_simd.sum()) - 1, "frame_and_rng_sha": frame_hash,
       "longest_waves": [{"block": int(b), "ms": round(float(end[b] - start[b]) / 1e3, 3),
                          "start_ms": round(float(start[b]) / 1e3, 3)} for b in np.argsort(start - end)[:8]],
       "series": series}
print(json.dumps(out, indent=1))
