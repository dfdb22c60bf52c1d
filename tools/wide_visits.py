"""Node visits per ray of 4-, 6- and 8-wide collapses of the rebuilt tree, on the CPU ("What the census
says about a wider node"; tools/wide_visits.cpp does the work).

    python tools/wide_visits.py [--scene cornell_bunny] [--paths 200000] [--bounces 6] [--c-node 1.0]

Exports the scene's triangles as the shipped 4-wide tree holds them (crt_scene_export, host only), compiles
wide_visits.cpp with g++, and prints its JSON line.  Nothing runs on a GPU.
"""
import argparse
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_bunny")
ap.add_argument("--paths", type=int, default=200000)
ap.add_argument("--bounces", type=int, default=6)
ap.add_argument("--c-node", type=float, default=1.0, help="node cost of the 6/8-wide collapse (4-wide: 1.0, shipped)")
a = ap.parse_args()

hs = crt_amd.HostScene(assets.scene_files(a.scene))
ex = hs.export(bvh="rebuilt")
n_tri = ex["sphere_first"]
p = ex["prims"][: 3 * n_tri].reshape(n_tri, 12)
tris = np.ascontiguousarray(p[:, :9], dtype=np.float32)   # v0.xyz, e1.xyz, e2.xyz
cam = crt_amd.camera_floats(crt_amd.camera(1))
with tempfile.TemporaryDirectory() as td:
    exe = Path(td) / "wide_visits"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{REPO / 'raytracer-cuda_amd' / 'csrc'}", "-o", str(exe),
                    str(REPO / "tools" / "wide_visits.cpp")], check=True)
    inp = Path(td) / "scene.bin"
    with open(inp, "wb") as f:
        f.write(np.array([n_tri, 2560, 1440], np.int32).tobytes())
        f.write(cam.astype(np.float32).tobytes())
        f.write(tris.tobytes())
    out = subprocess.run([str(exe), str(inp), str(a.paths), str(a.bounces), str(a.c_node)], check=True,
                         capture_output=True, text=True).stdout
print(out.strip().replace('{"triangles"', '{"scene": "%s", "triangles"' % a.scene, 1))
