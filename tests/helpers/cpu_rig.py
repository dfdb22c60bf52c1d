"""`bench.py --rig cpu_rig`: crt_amd's renderer API over the oracle, so that bench.py's launch, shard, collective and
JSON-line path runs on a machine without a GPU (tests/test_bench_launch.py, gloo ranks).

Test infrastructure, like the oracle it wraps: the scene is loaded by the host library (crt_amd.HostScene, host BVH
builds), each "launch" is oracle/crt_oracle.c rendering the whole frame on the CPU, and the linear framebuffer is the
torch CPU tensor ShardedFrameRenderer attaches.  It measures nothing; bench.py marks its line "rehearsal".
"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd"), str(REPO / "oracle")]
import crt_amd  # noqa: E402
import objload  # noqa: E402
import pyoracle  # noqa: E402

DEVICE_TYPE = "cpu"
camera = crt_amd.camera
camera_floats = crt_amd.camera_floats
pixel_sample_scale = crt_amd.pixel_sample_scale


class RigScene:
    def __init__(self, oracle_scene, counts):
        self.o = oracle_scene
        self._counts = counts

    def stats(self) -> dict:
        return {"device_nodes": 0, "device_bytes": 0}


class HostScene(crt_amd.HostScene):
    """The host half of crt_amd.HostScene (BVHs built on the host whatever build_device asks); upload() hands back the
    oracle's scene of the same OBJ files."""

    def __init__(self, obj_files, build_device=None):
        super().__init__(obj_files, build_device=None)
        self._oracle = pyoracle.OracleScene(objload.load_scene(self.files))

    def upload(self, device: int = 0, **options):
        return RigScene(self._oracle, self.counts())


class Renderer:
    def __init__(self, width: int, height: int, device: int = 0):
        self.width, self.height, self.device = width, height, device
        self._own = np.zeros((height, width, 3), np.float32)
        self._ptr = None
        self._cam = None
        self._seed, self._subseq = 41, 0
        self._counts = {"rays": 0}
        self._ms = 0.0
        self._rgba = np.zeros((height, width, 4), np.uint8)

    def set_camera(self, cam):
        self._cam = camera_floats(cam)

    def init_rand(self, seed: int = 41, subsequence_base: int = 0, stream=None):
        self._seed, self._subseq = int(seed), int(subsequence_base)

    def attach_linear(self, device_ptr):
        self._ptr = device_ptr

    def _view(self) -> np.ndarray:
        if self._ptr is None:
            return self._own
        n = self.width * self.height * 3
        return np.frombuffer((C.c_float * n).from_address(self._ptr), np.float32).reshape(self.height, self.width, 3)

    def render(self, scene, spp: int, max_bounces: int = 20, accumulate=False, count_work=False, stream=None):
        t = time.perf_counter()
        s, _, cnt = scene.o.render(self._cam, self.width, self.height, spp, max_bounces, seed=self._seed,
                                   subseq_base=self._subseq, nthreads=2)
        self._ms = (time.perf_counter() - t) * 1e3
        self._view()[...] = s
        self._counts = cnt

    def resolve(self, scale: float, stream=None):
        """writeColor (Color.cuh) of the linear sums: gamma 2 + clamp, as the oracle's RGBA8."""
        lin = self._view().astype(np.float32) * np.float32(scale)
        c = np.sqrt(np.clip(lin, 0.0, None))
        self._rgba[..., :3] = (256 * np.clip(c, 0.0, 0.999)).astype(np.uint8)
        self._rgba[..., 3] = 255

    def synchronize(self, stream=None):
        pass

    def linear(self) -> np.ndarray:
        return self._view().copy()

    def rgba8(self) -> np.ndarray:
        return self._rgba.copy()

    def counters(self) -> dict:
        return dict(self._counts)

    def last_kernel_name(self) -> str:
        return "oracle (cpu rig)"

    def last_timings(self) -> dict:
        return {"probe_sort_ms": 0.0, "main_kernel_ms": self._ms}

    @staticmethod
    def has_timing_history() -> bool:
        return False

    def last_kernel_ms(self) -> float:
        return self._ms
