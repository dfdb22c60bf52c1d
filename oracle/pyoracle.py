"""ctypes front-end of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# ORACLE_LIB: the sanitizer build (`make -C oracle asan`, tools/run_asan.sh) instead of the in-tree one
LIB_PATH = Path(os.environ["ORACLE_LIB"]) if os.environ.get("ORACLE_LIB") else HERE / "liboracle.so"
_lib = None


def build(force: bool = False) -> Path:
    if os.environ.get("ORACLE_LIB"):
        return LIB_PATH
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "crt_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-B" if force else "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        P, u64, i32, f32p = C.c_void_p, C.c_ulonglong, C.c_int, C.c_void_p
        L.oracle_scene_create.argtypes = [i32, P, u64, P, u64, P, u64, P, i32, P, C.POINTER(C.c_void_p)]
        L.oracle_scene_create.restype = i32
        L.oracle_scene_destroy.argtypes = [P]
        L.oracle_scene_nodes.argtypes = [P, i32, P, P]
        L.oracle_scene_nodes.restype = i32
        L.oracle_scene_mesh_arrays.argtypes = [P, i32, P, P, P]
        L.oracle_camera.argtypes = [C.c_float, C.c_float, P, P, C.c_float, C.c_float, C.c_float, C.c_float, P]
        L.oracle_render.argtypes = [P, P, i32, i32, i32, i32, i32, u64, u64, i32, i32, i32, i32, i32, P, P, P]
        L.oracle_render.restype = i32
        L.oracle_rng_init.argtypes = [u64, u64, P]
        L.oracle_rng_draw.argtypes = [P, i32, P, P]
        L.oracle_seq_matrix.argtypes = [i32, P]
        L.oracle_render_rng.argtypes = [P, P, i32, i32, i32, i32, i32, P, i32, P, P, P]
        L.oracle_render_rng.restype = i32
        L.oracle_camctl_new.argtypes = [C.c_float, C.c_float, P, P, C.c_float, C.c_float]
        L.oracle_camctl_new.restype = P
        L.oracle_camctl_free.argtypes = [P]
        L.oracle_camctl_update.argtypes = [P, C.c_float, i32, i32, C.c_float, C.c_float, i32, C.c_uint, i32]
        L.oracle_camctl_get.argtypes = [P, P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class OracleScene:
    """Reference createRandomWorld + BVH builds over a loaded scene (objload.LoadedScene)."""

    def __init__(self, loaded):
        L = lib()
        self._keep = [np.ascontiguousarray(loaded.positions, np.float32),
                      np.ascontiguousarray(loaded.indices, np.uint32),
                      np.ascontiguousarray(loaded.facemat, np.int32),
                      np.ascontiguousarray(loaded.mesh_info, np.uint32),
                      np.ascontiguousarray(loaded.matdata, np.float32)]
        pos, idx, fm, info, mats = self._keep
        h = C.c_void_p()
        rc = L.oracle_scene_create(len(info), _p(pos), len(pos), _p(idx), len(idx), _p(fm), len(fm),
                                   _p(info), len(mats), _p(mats), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"oracle_scene_create failed rc={rc}")
        self.h = h
        self.n_meshes = len(info)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def nodes(self, which: int):
        L = lib()
        n = L.oracle_scene_nodes(self.h, which, None, None)
        boxes = np.zeros((n, 6), np.float32)
        ints = np.zeros((n, 5), np.int32)
        L.oracle_scene_nodes(self.h, which, _p(boxes), _p(ints))
        return boxes, ints

    def mesh_arrays(self, which: int, n_idx: int):
        idx = np.zeros(n_idx, np.uint32)
        fm = np.zeros(n_idx // 3, np.int32)
        box = np.zeros(6, np.float32)
        lib().oracle_scene_mesh_arrays(self.h, which, _p(idx), _p(fm), _p(box))
        return idx, fm, box

    def render(self, cam19, w, h, spp, max_bounces=20, seed=41, subseq_base=0, rect=None,
               nthreads=None, spp_total=None):
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, w, h)
        rw, rh = x1 - x0, y1 - y0
        s = np.zeros((rh, rw, 3), np.float32)
        rgba = np.zeros((rh, rw, 4), np.uint8)
        cnt = np.zeros(4, np.uint64)
        cam = np.ascontiguousarray(cam19, np.float32)
        nthreads = nthreads or os.cpu_count() or 1
        lib().oracle_render(self.h, _p(cam), w, h, spp, spp_total or spp, max_bounces, seed, subseq_base,
                            x0, y0, x1, y1, nthreads, _p(s), _p(rgba), _p(cnt))
        return s, rgba, {"rays": int(cnt[0]), "box_tests": int(cnt[1]), "tri_tests": int(cnt[2]),
                         "sphere_tests": int(cnt[3])}


    def render_rng(self, cam19, w, h, spp, rng_state, max_bounces=20, nthreads=None, spp_total=None):
        """One frame continuing the per-pixel RNG state (h*w*6 uint32, updated in place), like consecutive
        CUDARenderer::render calls over one curandState array."""
        assert rng_state.dtype == np.uint32 and rng_state.size == w * h * 6 and rng_state.flags.c_contiguous
        s = np.zeros((h, w, 3), np.float32)
        rgba = np.zeros((h, w, 4), np.uint8)
        cnt = np.zeros(4, np.uint64)
        cam = np.ascontiguousarray(cam19, np.float32)
        lib().oracle_render_rng(self.h, _p(cam), w, h, spp, spp_total or spp, max_bounces, _p(rng_state),
                                nthreads or os.cpu_count() or 1, _p(s), _p(rgba), _p(cnt))
        return s, rgba, {"rays": int(cnt[0])}


class CameraController:
    """Camera::updateCamera restated (oracle_camctl_*): input per frame = mouse x/y, right button,
    key bits (W=1 A=2 S=4 D=8 Space=16 LControl=32 F=64), focus steps."""

    def __init__(self, aspect=16.0 / 9.0, vfov=80.0, pos=(0.0, 4.0, 4.0), up=(0.0, 1.0, 0.0), aperture=0.000001,
                 focus=None):
        pos = np.asarray(pos, np.float32)
        if focus is None:
            focus = float(np.sqrt(np.float32(np.dot(pos, pos))))
        self.h = lib().oracle_camctl_new(C.c_float(aspect), C.c_float(vfov), _p(pos),
                                         _p(np.asarray(up, np.float32)), C.c_float(aperture), C.c_float(focus))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_camctl_free(self.h)
            self.h = None

    def update(self, dt, ww, wh, mouse_x=0.0, mouse_y=0.0, right_mouse=False, keys=0, focus_steps=0):
        lib().oracle_camctl_update(self.h, C.c_float(dt), ww, wh, C.c_float(mouse_x), C.c_float(mouse_y),
                                   int(bool(right_mouse)), keys, focus_steps)

    def get(self):
        cam = np.zeros(19, np.float32)
        st = np.zeros(8, np.float32)
        lib().oracle_camctl_get(self.h, _p(cam), _p(st))
        return cam, {"yaw": float(st[0]), "pitch": float(st[1]), "moving": bool(st[2]), "rotating": bool(st[3]),
                     "high_quality": bool(st[4]), "focus": float(st[5]), "spp": int(st[6]), "scale": float(st[7])}


def camera(aspect=16.0 / 9.0, vfov=80.0, pos=(0.0, 0.0, 0.3), up=(0.0, 1.0, 0.0), aperture=0.000001,
           focus=0.3, yaw=-90.0, pitch=0.0) -> np.ndarray:
    out = np.zeros(19, np.float32)
    lib().oracle_camera(C.c_float(aspect), C.c_float(vfov), _p(np.asarray(pos, np.float32)),
                        _p(np.asarray(up, np.float32)), C.c_float(aperture), C.c_float(focus),
                        C.c_float(yaw), C.c_float(pitch), _p(out))
    return out


def rng_init(seed: int, subseq: int) -> np.ndarray:
    st = np.zeros(6, np.uint32)
    lib().oracle_rng_init(seed, subseq, _p(st))
    return st


def rng_draw(state: np.ndarray, n: int):
    u = np.zeros(n, np.uint32)
    f = np.zeros(n, np.float32)
    lib().oracle_rng_draw(_p(state), n, _p(u), _p(f))
    return u, f


def seq_matrix(k: int) -> np.ndarray:
    out = np.zeros(800, np.uint32)
    lib().oracle_seq_matrix(k, _p(out))
    return out


def _kat_lib():
    L = lib()
    if not getattr(L, "_kat_bound", False):
        P, i32 = C.c_void_p, C.c_int
        L.oracle_kat_triangle.argtypes = [P, i32, P]
        L.oracle_kat_box.argtypes = [P, i32, P]
        L.oracle_kat_sphere.argtypes = [P, i32, P]
        L.oracle_kat_get_ray.argtypes = [P, i32, i32, P, P, i32, P]
        L._kat_bound = True
    return L


def kat_triangle(rec: np.ndarray) -> np.ndarray:
    """rayTriangleIntersect on (n, 17) f32 records o3 d3 v0 v1 v2 tmin tmax -> t or -1 (crt_oracle.c)."""
    rec = np.ascontiguousarray(rec, np.float32)
    out = np.zeros(len(rec), np.float32)
    _kat_lib().oracle_kat_triangle(_p(rec), len(rec), _p(out))
    return out


def kat_box(rec: np.ndarray) -> np.ndarray:
    """AABB::hit on (n, 14) f32 records o3 d3 lo3 hi3 tmin tmax -> 1 / 0."""
    rec = np.ascontiguousarray(rec, np.float32)
    out = np.zeros(len(rec), np.int32)
    _kat_lib().oracle_kat_box(_p(rec), len(rec), _p(out))
    return out


def kat_sphere(rec: np.ndarray) -> np.ndarray:
    """Sphere::hit on (n, 12) f32 records o3 d3 centre3 radius tmin tmax -> t or -1."""
    rec = np.ascontiguousarray(rec, np.float32)
    out = np.zeros(len(rec), np.float32)
    _kat_lib().oracle_kat_sphere(_p(rec), len(rec), _p(out))
    return out


def kat_get_ray(cam19: np.ndarray, w: int, h: int, xy: np.ndarray, rng: np.ndarray) -> np.ndarray:
    """Camera::getRay for pixels xy (n, 2); rng (n, 6) u32 is continued in place.  Returns (n, 6) o3 d3."""
    cam19 = np.ascontiguousarray(cam19, np.float32)
    xy = np.ascontiguousarray(xy, np.int32)
    assert rng.dtype == np.uint32 and rng.flags.c_contiguous and rng.shape == (len(xy), 6)
    out = np.zeros((len(xy), 6), np.float32)
    _kat_lib().oracle_kat_get_ray(_p(cam19), w, h, _p(xy), _p(rng), len(xy), _p(out))
    return out
