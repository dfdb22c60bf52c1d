"""Dev probe: one variant-5 frame (for rocprofv3 kernel traces)."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
refill = int(sys.argv[2]) if len(sys.argv) > 2 else 32
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=3)
r = crt_amd.Renderer(2560, 1440)
r.set_camera(crt_amd.camera(spp))
r.set_kernel_variant(5)
r.set_wavefront(refill, 16)
for _ in range(2):
    r.init_rand(41)
    r.render(sc, spp, 20)
    r.synchronize()
    print("v5", r.last_kernel_ms(), "ms", r.counters()["rays"], "rays", r.wavefront_iterations(), "iterations", flush=True)
