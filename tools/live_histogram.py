"""Variant 8's wave time by the number of lanes that still have samples (profiling build only).

    tools/build_profile_lib.sh live -DCRT_PROFILE_LIVE
    CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/live/libcrt_hip.so python tools/live_histogram.py [--spp 256] [--w 2560 --h 1440]

Each wave sums the s_memtime cycles of its loop iterations into 9 buckets by its live-lane count (0-7, 8-15, ..., 56-63,
64) and adds them to a device histogram at its end.  The shares say how much of the waves' time is spent draining: a
wave with few live lanes issues the same instructions per iteration as a full one.
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
ap.add_argument("--base", type=int, default=0, help="subsequence base (rank g of N: g*W*H)")
a = ap.parse_args()
L = _lib.hip()
L.crt_profile_live_hist.argtypes = [C.c_void_p, C.c_int]
hs = crt_amd.HostScene(assets.scene_files(a.scene), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
buf = np.zeros(16, np.uint64)
for k in range(2):   # the first frame warms up; the histogram of the second is reported
    _lib.check(L.crt_profile_live_hist(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_live_hist")
    r.init_rand(41, a.base)
    r.render(sc, a.spp, 20)
    r.synchronize()
_lib.check(L.crt_profile_live_hist(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_live_hist")
h = buf[:9].astype(np.float64)
labels = [f"{8 * i}-{8 * i + 7}" for i in range(8)] + ["64"]
print(json.dumps({"kernel": r.last_kernel_name(), "w": a.w, "h": a.h, "spp": a.spp, "scene": a.scene,
                  "main_kernel_ms": round(r.last_timings()["main_kernel_ms"], 3),
                  "wave_cycles": int(h.sum()),
                  "share_by_live_lanes": {labels[i]: round(h[i] / h.sum(), 4) for i in range(9)}}))
