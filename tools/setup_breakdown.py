"""Where the scene set-up time of bench.py's end_to_end_s goes: each host/device step of loading a
scene, timed twice in one process (the first call pays one-time costs: code-object loading, allocator warm-up).

    python tools/setup_breakdown.py [--scene cornell_bunny] [--device 0]

Prints one JSON line per step and pass.
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--device", type=int, default=0)
ap.add_argument("--torch-first", action="store_true", help="initialise torch's HIP context first, as bench.py does")
a = ap.parse_args()

if a.torch_first:
    import torch
    torch.zeros(1, device=f"cuda:{a.device}")
    torch.cuda.synchronize()

files = assets.scene_files(a.scene)


def timed(label, fn):
    t = time.perf_counter()
    out = fn()
    dt = time.perf_counter() - t
    print(json.dumps({"step": label, "s": round(dt, 4)}), flush=True)
    return out


for p in (1, 2):
    hs = timed(f"pass{p}: load + mesh BVH on the GPU", lambda: crt_amd.HostScene(files, build_device=a.device))
    print(json.dumps({"step": f"pass{p}: mesh BVH device ms", "ms": hs.device_build_ms()}))
    timed(f"pass{p}: load + mesh BVH on the host", lambda: crt_amd.HostScene(files))
    sc = timed(f"pass{p}: rebuilt tree (GPU SAH) + upload",
               lambda: hs.upload(a.device, bvh="rebuilt", gpu_build=True))
    timed(f"pass{p}: rebuilt tree (host SAH) + export", lambda: hs.export(bvh="rebuilt"))
    ref = timed(f"pass{p}: reference-BVH upload", lambda: hs.upload(a.device))
    r = timed(f"pass{p}: Renderer(2560, 1440)", lambda: crt_amd.Renderer(2560, 1440, a.device))
    timed(f"pass{p}: curand_init", lambda: (r.init_rand(41), r.synchronize()))
    del sc, ref, r, hs
