"""Leaf pairs per wave step and lanes per wave step of one headline-geometry frame (profiling build only).

    tools/build_profile_lib.sh pairs -DCRT_PROFILE_PAIRS
    CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/pairs/libcrt_hip.so python tools/pair_histogram.py [--spp 256]

Prints, for the timed kernel (variant 8), the distribution of the leaf pairs a wave step hands to its cooperative
rounds (log2 buckets; 0 = a step without leaves) and of the lanes that step (traversing or holding a leaf span).
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
a = ap.parse_args()
L = _lib.hip()
L.crt_profile_pair_hist.argtypes = [C.c_void_p, C.c_int]
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"), build_device=0)
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(a.w, a.h)
r.set_camera(crt_amd.camera(a.spp))
buf = np.zeros(32, np.uint64)
r.init_rand(41)
r.render(sc, a.spp, 20)
r.synchronize()
_lib.check(L.crt_profile_pair_hist(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_pair_hist")   # includes the probe
buf[:] = 0
r.init_rand(41)
r.render(sc, a.spp, 20)
r.synchronize()
_lib.check(L.crt_profile_pair_hist(buf.ctypes.data_as(C.c_void_p), 1), "crt_profile_pair_hist")
# the second frame still contains its cost-probe launch (4 spp): subtract nothing, report shares
pairs = buf[:16].astype(np.float64)
lanes = buf[16:25].astype(np.float64)
labels = ["0"] + [f"{1 << k}-{(2 << k) - 1}" for k in range(15)]
steps = pairs.sum()
out = {"kernel": r.last_kernel_name(), "steps": int(steps),
       "pairs_per_step_share": {labels[i]: round(pairs[i] / steps, 4) for i in range(16) if pairs[i]},
       "lanes_per_step_share": {f"{8 * i}-{8 * i + 7}" if i < 8 else "64": round(lanes[i] / steps, 4) for i in range(9)}}
print(json.dumps(out, indent=1))
