"""crt_amd — Python front-end of the MI355X path tracer.

Mirrors the reference's host API for the render path (CudaRayTracer/src):
  HostScene      ~ SceneManager host half (OBJ load, normalisation, BVH builds; C++ libcrt_host.so)
  Scene          ~ the device scene (SceneManager::getBVHNodes()/getWorld(); libcrt_hip.so)
  Renderer       ~ CUDARenderer (initialize / updateCamera / render / getImageData)
  camera(...)    ~ CRT::Camera(aspect, fov, position, target, up, aperture, focus)
All compute runs in the HIP library; nothing here computes pixels.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import CameraDesc, CrtError, SceneDesc, SceneStats, WorkCounters, build, check, check_host

RENDER_ACCUMULATE = 1
RENDER_COUNT_WORK = 2

# The screenshot-reproducing bench pose: the reference's default pose
# (Raytracer.h:77-82, pos (0,4,4), target ignored) does not frame the box.
BENCH_CAMERA = dict(aspect=16.0 / 9.0, vfov=80.0, pos=(0.0, 0.0, 0.3), up=(0.0, 1.0, 0.0),
                    aperture=0.000001, focus=0.3, yaw=-90.0, pitch=0.0)


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def camera(spp: int = 1, aspect=16.0 / 9.0, vfov=80.0, pos=(0.0, 0.0, 0.3), up=(0.0, 1.0, 0.0),
           aperture=0.000001, focus=0.3, yaw=-90.0, pitch=0.0) -> CameraDesc:
    """CRT::Camera (Camera.cuh:18-30, :159-182) computed by the C++ host library."""
    d = CameraDesc()
    check_host(_lib.host().crth_camera(C.c_float(aspect), C.c_float(vfov), _p(np.asarray(pos, np.float32)),
                                       _p(np.asarray(up, np.float32)), C.c_float(aperture), C.c_float(focus),
                                       C.c_float(yaw), C.c_float(pitch), int(spp), C.byref(d)), "crth_camera")
    return d


def camera_floats(d: CameraDesc) -> np.ndarray:
    """19-float layout shared with the oracle (origin, llc, horizontal, vertical, right, up, lens_radius)."""
    return np.array(list(d.origin) + list(d.lower_left) + list(d.horizontal) + list(d.vertical) +
                    list(d.right) + list(d.up) + [d.lens_radius], dtype=np.float32)


class HostScene:
    """SceneManager host half: load OBJ files, normalise, build mesh + scene BVHs (C++)."""

    def __init__(self, obj_files, build_device=None):
        """build_device: None = mesh BVHs built by the host restatement; k = on GPU k (crt_build_mesh_bvh,
        same trees)."""
        files = [str(f) for f in obj_files]
        arr = (C.c_char_p * len(files))(*[f.encode() for f in files])
        h = C.c_void_p()
        bd = -1 if build_device is None else int(build_device)
        check_host(_lib.host().crth_scene_load_ex(arr, len(files), bd, C.byref(h)), "crth_scene_load_ex")
        self.h = h
        self.files = files

    def device_build_ms(self) -> float:
        """Device time of the GPU mesh BVH builds of this load (0.0 for host builds)."""
        return float(_lib.host().crth_scene_build_ms(self.h))

    def __del__(self):
        # at interpreter exit the module's globals may already be gone (None); the process frees the scene then
        if getattr(self, "h", None) and _lib is not None:
            _lib.host().crth_scene_destroy(self.h)
            self.h = None

    def counts(self):
        c = np.zeros(5, np.int64)
        check_host(_lib.host().crth_scene_counts(self.h, _p(c)), "crth_scene_counts")
        return dict(n_meshes=int(c[0]), n_slots=int(c[1]), n_indices=int(c[2]), n_faces=int(c[3]),
                    n_materials=int(c[4]))

    def loader_arrays(self):
        c = self.counts()
        pos = np.zeros((c["n_slots"], 3), np.float32)
        idx = np.zeros(c["n_indices"], np.uint32)
        fm = np.zeros(c["n_faces"], np.int32)
        info = np.zeros((c["n_meshes"], 6), np.uint32)
        mats = np.zeros((c["n_materials"], 9), np.float32)
        check_host(_lib.host().crth_scene_loader_arrays(self.h, _p(pos), _p(idx), _p(fm), _p(info), _p(mats)),
                   "crth_scene_loader_arrays")
        return pos, idx, fm, info, mats

    def desc(self) -> SceneDesc:
        d = SceneDesc()
        check_host(_lib.host().crth_scene_desc(self.h, C.byref(d)), "crth_scene_desc")
        return d

    def mesh_bvh(self, i: int):
        """(boxes[n,6], ints[n,5] = left,right,obj_index,obj_count,is_leaf) in builder index order."""
        d = self.desc()
        meshes = C.cast(d.meshes, C.POINTER(_lib.MeshDesc))
        m = meshes[i]
        return _nodes_to_np(m.nodes, m.node_count), np.array(m.aabb, np.float32)

    def scene_bvh(self):
        d = self.desc()
        return _nodes_to_np(d.scene_nodes, d.n_scene_nodes)

    def permuted(self):
        d = self.desc()
        idx = np.ctypeslib.as_array(C.cast(d.indices, C.POINTER(C.c_uint32)), (d.n_indices,)).copy()
        fm = np.ctypeslib.as_array(C.cast(d.face_materials, C.POINTER(C.c_int32)), (d.n_faces,)).copy()
        return idx, fm

    def upload(self, device: int = 0, bvh: str = "reference", leaf_size: int = 0, layouts: int = 0,
               traversal_cost: float = 0.0, width: int = 0, gpu_build: bool = False, stack_cap: int = 0,
               spatial_splits: bool = False, spatial_alpha: float = 0.0, spatial_max_dup: float = 0.0) -> "Scene":
        """Device scene.  bvh="reference": the reference's BVHs, bit-exact (crth_scene_upload);
        bvh="rebuilt": binned-SAH BVH with the reference's hit rule (crt_scene_create_ex)."""
        h = C.c_void_p()
        if (bvh == "reference" and not leaf_size and not layouts and not traversal_cost and not width and not gpu_build
                and not stack_cap and not spatial_splits):
            check_host(_lib.host().crth_scene_upload(self.h, int(device), C.byref(h)), "crth_scene_upload")
            return Scene(h, device)
        o = scene_options(bvh, leaf_size, layouts, traversal_cost, width, gpu_build, stack_cap, spatial_splits,
                          spatial_alpha, spatial_max_dup)
        d = self.desc()
        check(_lib.hip().crt_scene_create_ex(C.byref(d), int(device), C.byref(o), C.byref(h)), "crt_scene_create_ex")
        return Scene(h, device)

    def export(self, bvh: str = "reference", **options) -> dict:
        """The device arrays crt_scene_create_ex would upload (host only, crt_scene_export)."""
        o = scene_options(bvh, **options)
        d = self.desc()
        info = (C.c_int64 * 10)()
        check(_lib.hip().crt_scene_export(C.byref(d), C.byref(o), None, None, None, info), "crt_scene_export")
        nodes = np.zeros((info[0], 4), np.float32)
        prims = np.zeros((info[1], 4), np.float32)
        rank_code = np.zeros(info[2], np.int32)
        check(_lib.hip().crt_scene_export(C.byref(d), C.byref(o), _p(nodes), _p(prims), _p(rank_code), info),
              "crt_scene_export")
        keys = ("node_float4s", "prim_float4s", "ranks", "nodes_per_layout", "layouts", "width", "stack_bound",
                "excluded", "sphere_first", "n_ray_spheres")
        out = dict(zip(keys, (int(v) for v in info)))
        out.update(nodes=nodes, prims=prims, rank_code=rank_code)
        return out


def scene_options(bvh: str = "reference", leaf_size: int = 0, layouts: int = 0, traversal_cost: float = 0.0,
                  width: int = 0, gpu_build: bool = False, stack_cap: int = 0, spatial_splits: bool = False,
                  spatial_alpha: float = 0.0, spatial_max_dup: float = 0.0):
    modes = {"reference": _lib.BVH_REFERENCE, "rebuilt": _lib.BVH_REBUILT}
    if bvh not in modes:
        raise ValueError(f"bvh must be one of {sorted(modes)}")
    o = _lib.SceneOptions()
    o.bvh, o.leaf_size, o.layouts = modes[bvh], int(leaf_size), int(layouts)
    o.traversal_cost = float(traversal_cost)
    o.width = int(width)
    o.gpu_build = int(bool(gpu_build))
    o.stack_cap = int(stack_cap)
    o.spatial_splits = int(bool(spatial_splits))
    o.spatial_alpha = float(spatial_alpha)
    o.spatial_max_dup = float(spatial_max_dup)
    return o


def _nodes_to_np(ptr, n):
    if n == 0:
        return np.zeros((0, 6), np.float32), np.zeros((0, 5), np.int32)
    raw = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), (n * C.sizeof(_lib.BvhNodeDesc),))
    rec = raw.view(np.dtype([("b", "<f4", 6), ("i", "<i4", 5)]))
    return rec["b"].copy(), rec["i"].copy()


class Scene:
    """Device scene handle (crt_scene)."""

    def __init__(self, handle, device):
        self.h = handle
        self.device = device

    def stats(self) -> dict:
        s = SceneStats()
        check(_lib.hip().crt_scene_get_stats(self.h, C.byref(s)), "crt_scene_get_stats")
        return {k: getattr(s, k) for k, _ in SceneStats._fields_}

    def close(self):
        if getattr(self, "h", None) and _lib is not None:   # None: interpreter exit (see HostScene.__del__)
            _lib.hip().crt_scene_destroy(self.h)
            self.h = None

    __del__ = close


def load_scene(obj_files, device: int = 0, **upload_options):
    hs = HostScene(obj_files)
    return hs, hs.upload(device, **upload_options)


class Renderer:
    """CUDARenderer equivalent over crt_renderer (CUDARenderer.cuh:9-60)."""

    def __init__(self, width: int, height: int, device: int = 0):
        h = C.c_void_p()
        check(_lib.hip().crt_renderer_create(int(width), int(height), int(device), C.byref(h)), "crt_renderer_create")
        self.h, self.width, self.height, self.device = h, width, height, device
        self._owned = True

    @classmethod
    def _borrow(cls, handle, width: int, height: int, device: int, owner):
        """A view of a renderer owned by someone else (e.g. a Viewer); never destroys it."""
        r = cls.__new__(cls)
        r.h, r.width, r.height, r.device, r._owned, r._owner = C.c_void_p(handle), width, height, device, False, owner
        return r

    def close(self):
        if getattr(self, "h", None) and _lib is not None:   # None: interpreter exit (see HostScene.__del__)
            if getattr(self, "_owned", True):
                _lib.hip().crt_renderer_destroy(self.h)
            self.h = None

    __del__ = close

    def init_rand(self, seed: int = 41, subsequence_base: int = 0, stream=None):
        check(_lib.hip().crt_renderer_init_rand(self.h, int(seed), int(subsequence_base), stream), "init_rand")

    def set_schedule(self, probe_spp: int = -1, min_spp: int = 64, tile_key: int = 2, probe_stride: int = 0):
        flags = ((int(tile_key) & 0xf) << 16) | ((int(probe_stride) & 0xf) << 20)
        check(_lib.hip().crt_renderer_set_schedule(self.h, int(probe_spp), int(min_spp), flags), "set_schedule")

    def set_critical_tiles(self, tiles: int = -1, lanes: int = 16):
        check(_lib.hip().crt_renderer_set_critical_tiles(self.h, int(tiles), int(lanes)), "set_critical_tiles")

    def set_top_levels(self, levels: int = -1):
        """4-wide kernels: a new ray's first node steps from the LDS copy of the tree's top nodes (-1 = default)."""
        check(_lib.hip().crt_renderer_set_top_levels(self.h, int(levels)), "set_top_levels")

    def set_pixel_shard(self, shard: int = 0, shards: int = 1):
        """Render only every shards-th 8x8 tile (from shard) with all samples; other pixels stay 0 (bit-exact
        multi-GPU mode, crt_renderer_set_pixel_shard)."""
        check(_lib.hip().crt_renderer_set_pixel_shard(self.h, int(shard), int(shards)), "set_pixel_shard")

    def set_kernel_variant(self, variant: int):
        check(_lib.hip().crt_renderer_set_kernel_variant(self.h, int(variant)), "set_kernel_variant")

    def set_occupancy_target(self, waves_per_simd: int):
        check(_lib.hip().crt_renderer_set_occupancy_target(self.h, int(waves_per_simd)), "set_occupancy_target")

    def set_regen_threshold(self, lanes: int):
        check(_lib.hip().crt_renderer_set_regen_threshold(self.h, int(lanes)), "set_regen_threshold")

    def set_stack_lds(self, entries: int):
        check(_lib.hip().crt_renderer_set_stack_lds(self.h, int(entries)), "set_stack_lds")

    def set_camera(self, cam: CameraDesc):
        self._cam = cam
        check(_lib.hip().crt_renderer_set_camera(self.h, C.byref(cam)), "set_camera")

    def render(self, scene: Scene, spp: int, max_bounces: int = 20, accumulate=False, count_work=False, stream=None):
        flags = (RENDER_ACCUMULATE if accumulate else 0) | (RENDER_COUNT_WORK if count_work else 0)
        check(_lib.hip().crt_renderer_render(self.h, scene.h, int(spp), int(max_bounces), flags, stream), "render")

    def resolve(self, scale: float, stream=None):
        check(_lib.hip().crt_renderer_resolve(self.h, C.c_float(scale), stream), "resolve")

    def synchronize(self, stream=None):
        check(_lib.hip().crt_renderer_synchronize(self.h, stream), "synchronize")

    def linear(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 3), np.float32)
        check(_lib.hip().crt_renderer_read_linear(self.h, _p(out)), "read_linear")
        return out

    def write_linear(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr, np.float32)
        check(_lib.hip().crt_renderer_write_linear(self.h, _p(a)), "write_linear")

    def rgba8(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.uint8)
        check(_lib.hip().crt_renderer_read_rgba8(self.h, _p(out)), "read_rgba8")
        return out

    def rng_state(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 6), np.uint32)
        check(_lib.hip().crt_renderer_read_rng(self.h, _p(out)), "read_rng")
        return out

    def counters(self) -> dict:
        w = WorkCounters()
        check(_lib.hip().crt_renderer_get_counters(self.h, C.byref(w)), "get_counters")
        return {k: int(getattr(w, k)) for k, _ in WorkCounters._fields_}

    def schedule_stats(self) -> dict:
        """Lane-slot diagnostics of the last counting render (see crt_renderer_get_schedule_stats)."""
        a = (C.c_ulonglong * 3)()
        check(_lib.hip().crt_renderer_get_schedule_stats(self.h, a), "get_schedule_stats")
        return {"step_lane_slots": int(a[0]), "round_lane_slots": int(a[1]), "wave_trace_calls": int(a[2])}

    def section_profile(self) -> dict:
        """Shader-clock cycles per section of the last counting render (variant 4), summed over waves."""
        a = (C.c_ulonglong * 8)()
        check(_lib.hip().crt_renderer_get_section_profile_ex(self.h, a, 8), "get_section_profile_ex")
        return dict(zip(("cyc_regen", "cyc_step", "cyc_round", "passes", "waves", "cyc_shade", "cyc_next", "cyc_sph"),
                        (int(v) for v in a)))

    def last_kernel_name(self) -> str:
        return (_lib.hip().crt_renderer_last_kernel_name(self.h) or b"").decode()

    def last_schedule(self) -> dict:
        """The last variant-8 render's occupancy choice (crt_renderer_last_schedule): rho = the probe's largest tile work
        over the mean work per occupancy-6 wave slot (0 without the probe-based choice), the occupancy launched, and the
        largest and mean tile works."""
        a = (C.c_float * 4)()
        check(_lib.hip().crt_renderer_last_schedule(self.h, a), "last_schedule")
        return {"rho": a[0], "occupancy": int(a[1]), "max_tile_work": a[2], "mean_tile_work": a[3]}

    def last_timings(self) -> dict:
        """HIP-event ms of the last render: the whole render, the probe + tile sort before the main kernel, and the
        main render kernel alone (crt_renderer_last_timings)."""
        a = (C.c_float * 3)()
        check(_lib.hip().crt_renderer_last_timings(self.h, a), "last_timings")
        return {"render_ms": float(a[0]), "probe_sort_ms": float(a[1]), "main_kernel_ms": float(a[2])}

    def set_temporal_order(self, on: bool):
        """Variant 7: tiles most expensive first by the previous frame's rays per pixel (crt_renderer_set_temporal_order)."""
        check(_lib.hip().crt_renderer_set_temporal_order(self.h, int(bool(on))), "set_temporal_order")

    def set_drain_threshold(self, lanes: int):
        """Variant 7: regeneration threshold once the pixel queue is empty, 0 = unchanged (crt_renderer_set_drain_threshold)."""
        check(_lib.hip().crt_renderer_set_drain_threshold(self.h, int(lanes)), "set_drain_threshold")

    def set_wave_drain(self, sixty_fourths: int):
        """Variants 4/8: a draining wave passes at sixty_fourths/64 of its live lanes (crt_renderer_set_wave_drain)."""
        check(_lib.hip().crt_renderer_set_wave_drain(self.h, int(sixty_fourths)), "set_wave_drain")

    def set_xcd_regions(self, on: bool):
        """Variant 8: XCD groups render equal-cost screen strips (crt_renderer_set_xcd_regions)."""
        check(_lib.hip().crt_renderer_set_xcd_regions(self.h, int(bool(on))), "set_xcd_regions")

    def set_leaf_carry(self, lanes: int, max_pairs: int):
        """Variant 8's leaf-pair carry: measured and removed in round 5; the library reports
        CRT_ERR_UNSUPPORTED, so this raises CrtError (profiles/r04c/leaf_carry.patch restores the kernels)."""
        check(_lib.hip().crt_renderer_set_leaf_carry(self.h, int(lanes), int(max_pairs)), "set_leaf_carry")

    @staticmethod
    def has_timing_history() -> bool:
        """Whether the loaded library exports crt_renderer_timing_history (ABI >= 3; older base builds in A/B runs)."""
        return hasattr(_lib.hip(), "crt_renderer_timing_history")

    def timing_history(self, back: int) -> dict:
        """last_timings() of an earlier render: back = 0 is the last one, up to 31 (crt_renderer_timing_history)."""
        a = (C.c_float * 3)()
        check(_lib.hip().crt_renderer_timing_history(self.h, int(back), a), "timing_history")
        return {"render_ms": float(a[0]), "probe_sort_ms": float(a[1]), "main_kernel_ms": float(a[2])}

    def last_kernel_ms(self) -> float:
        return float(_lib.hip().crt_renderer_last_kernel_ms(self.h))

    def attach_linear(self, device_ptr: int | None):
        """Render into caller-owned device memory (W*H*3 f32), e.g. a torch tensor to RCCL-reduce."""
        check(_lib.hip().crt_renderer_attach_linear(self.h, C.c_void_p(device_ptr) if device_ptr else None),
              "attach_linear")

    def linear_device_ptr(self) -> int:
        return int(_lib.hip().crt_renderer_linear_device_ptr(self.h) or 0)

    def render_frame(self, scene: Scene, spp: int, max_bounces: int = 20, seed: int = 41, subsequence_base: int = 0,
                     stream=None):
        """Fresh RNG (initRandState) + spp samples + writeColor: one reference frame."""
        self.init_rand(seed, subsequence_base, stream)
        self.render(scene, spp, max_bounces, stream=stream)
        self.resolve(pixel_sample_scale(spp), stream)
        self.synchronize(stream)

    def compare(self, scene_a: Scene, scene_b: Scene, spp: int, max_bounces: int = 20) -> dict:
        """Per-ray hit agreement of two device scenes (crt_scene_compare); paths follow scene_a.
        Call init_rand first; the RNG state is consumed."""
        out = (C.c_uint64 * 5)()
        check(_lib.hip().crt_scene_compare(self.h, scene_a.h, scene_b.h, int(spp), int(max_bounces), out),
              "crt_scene_compare")
        keys = ("rays", "rank_mismatch", "t_mismatch", "b_miss", "a_miss")
        return dict(zip(keys, (int(v) for v in out)))

    def compare_dump(self, scene_a: Scene, scene_b: Scene, spp: int, max_bounces: int = 20, max_dump: int = 256):
        """compare() plus the differing rays: array [n, 10] = o.xyz, d.xyz, rank_a, rank_b (int bits), t_a, t_b."""
        out = (C.c_uint64 * 5)()
        buf = np.zeros((max_dump, 10), np.float32)
        check(_lib.hip().crt_scene_compare_dump(self.h, scene_a.h, scene_b.h, int(spp), int(max_bounces), out,
                                                _p(buf), int(max_dump)), "crt_scene_compare_dump")
        keys = ("rays", "rank_mismatch", "t_mismatch", "b_miss", "a_miss")
        res = dict(zip(keys, (int(v) for v in out)))
        return res, buf[:min(max_dump, res["rank_mismatch"])]


def pixel_sample_scale(spp: int) -> float:
    """m_PixelSampleScale = 1.f / m_SamplesPerPixel (Camera.cuh:23), rounded to f32 (spp 0 gives inf, as in C)."""
    with np.errstate(divide="ignore"):
        return float(np.float32(1.0) / np.float32(spp))


def device_count() -> int:
    n = C.c_int(0)
    check(_lib.hip().crt_device_count(C.byref(n)), "device_count")
    return n.value


KEY_W, KEY_A, KEY_S, KEY_D, KEY_SPACE, KEY_LCONTROL, KEY_F = 1, 2, 4, 8, 16, 32, 64


def _input(mouse_x=0.0, mouse_y=0.0, right_mouse=False, keys=0, focus_steps=0) -> _lib.CrthInput:
    return _lib.CrthInput(float(mouse_x), float(mouse_y), int(bool(right_mouse)), int(keys), int(focus_steps))


class CameraController:
    """CRT::Camera + Camera::updateCamera on the host (crth_camera_*; Camera.cuh:46-157). No GPU."""

    def __init__(self, aspect=16.0 / 9.0, vfov=80.0, pos=(0.0, 4.0, 4.0), up=(0.0, 1.0, 0.0), aperture=0.000001,
                 focus=None):
        pos = np.asarray(pos, np.float32)
        if focus is None:
            focus = float(np.sqrt(np.float32(np.dot(pos, pos))))
        h = C.c_void_p()
        check_host(_lib.host().crth_camera_create(aspect, vfov, _p(pos), _p(np.asarray(up, np.float32)), aperture,
                                                  focus, C.byref(h)), "crth_camera_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None) and _lib is not None:   # None: interpreter exit (see HostScene.__del__)
            _lib.host().crth_camera_destroy(self.h)
            self.h = None

    __del__ = close

    def update(self, dt, ww, wh, **inp):
        check_host(_lib.host().crth_camera_update(self.h, dt, ww, wh, C.byref(_input(**inp))), "crth_camera_update")

    def get(self):
        d = CameraDesc()
        st = np.zeros(6, np.float32)
        check_host(_lib.host().crth_camera_get(self.h, C.byref(d), _p(st)), "crth_camera_get")
        return d, {"yaw": float(st[0]), "pitch": float(st[1]), "moving": bool(st[2]), "rotating": bool(st[3]),
                   "high_quality": bool(st[4]), "focus": float(st[5])}


class Viewer:
    """The reference's Raytracer loop, headless (crth_viewer_*; Raytracer.h:52-102): one frame() per
    updateAndRender with the input the window would have delivered."""

    def __init__(self, obj_files, width, height, device=0, bvh="reference", aspect=16.0 / 9.0, vfov=80.0,
                 aperture=0.000001, pos=None, focus=0.0, seed=41, accumulate=False, bvh_width=0, **scene_kw):
        files = [str(f).encode() for f in obj_files]
        arr = (C.c_char_p * len(files))(*files)
        opts = scene_options(bvh, width=bvh_width, **scene_kw)
        pos_a = None if pos is None else np.asarray(pos, np.float32)
        h = C.c_void_p()
        check_host(_lib.host().crth_viewer_create(arr, len(files), device, C.byref(opts), width, height, aspect, vfov,
                                                  aperture, None if pos_a is None else _p(pos_a), focus, seed,
                                                  int(bool(accumulate)), C.byref(h)), "crth_viewer_create")
        self.h, self.width, self.height, self.device = h, width, height, device
        self.renderer = Renderer._borrow(_lib.host().crth_viewer_renderer(h), width, height, device, self)

    def close(self):
        if getattr(self, "h", None) and _lib is not None:   # None: interpreter exit (see HostScene.__del__)
            self.renderer.h = None
            _lib.host().crth_viewer_destroy(self.h)
            self.h = None

    __del__ = close

    def frame(self, dt=1.0 / 60.0, **inp) -> dict:
        fi = _lib.CrthFrameInfo()
        check_host(_lib.host().crth_viewer_frame(self.h, dt, C.byref(_input(**inp)), C.byref(fi)), "crth_viewer_frame")
        return {"frame": fi.frame, "spp": fi.spp, "accumulated": fi.accumulated, "moving": bool(fi.moving),
                "high_quality": bool(fi.high_quality), "kernel_ms": fi.kernel_ms, "frame_ms": fi.frame_ms}

    def camera(self) -> CameraDesc:
        d = CameraDesc()
        check_host(_lib.host().crth_viewer_camera(self.h, C.byref(d)), "crth_viewer_camera")
        return d


IMAGE_FORMATS = {"ppm": 0, "png": 1}


def encode_image(rgba: np.ndarray, fmt: str = "png", flip: bool = True) -> bytes:
    """PNG/PPM bytes of an (H, W, 4) uint8 framebuffer (row 0 = bottom, as the renderer holds it);
    flip=True writes the top row first, like WindowManager::drawFrame (WindowManager.h:79-93)."""
    a = np.ascontiguousarray(rgba, np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise CrtError("rgba must be (H, W, 4) uint8")
    h, w = a.shape[:2]
    n = C.c_uint64(0)
    L = _lib.host()
    check_host(L.crth_encode_image(IMAGE_FORMATS[fmt], _p(a), w, h, int(flip), None, C.byref(n)), "crth_encode_image")
    out = np.empty(n.value, np.uint8)
    check_host(L.crth_encode_image(IMAGE_FORMATS[fmt], _p(a), w, h, int(flip), _p(out), C.byref(n)), "crth_encode_image")
    return out[: n.value].tobytes()


def write_image(path: str, rgba: np.ndarray, flip: bool = True) -> None:
    """Write .png / .ppm by extension (crth_write_image)."""
    a = np.ascontiguousarray(rgba, np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise CrtError("rgba must be (H, W, 4) uint8")
    check_host(_lib.host().crth_write_image(str(path).encode(), _p(a), a.shape[1], a.shape[0], int(flip)),
               "crth_write_image")


NODE_DTYPE = np.dtype([("bmin", "<f4", 3), ("bmax", "<f4", 3), ("left", "<i4"), ("right", "<i4"),
                       ("obj_index", "<i4"), ("obj_count", "<i4"), ("is_leaf", "<i4")])   # crt_bvh_node_desc


def build_mesh_bvh(positions, indices, face_materials, device=None):
    """Mesh::buildBVHMesh + Mesh ctor box (Mesh.cuh:39-47, :121-264) on one mesh.

    device=None: the sequential host restatement (crth_build_mesh_bvh); device=k: the GPU-parallel build
    on device k (crt_build_mesh_bvh).  Returns (nodes [NODE_DTYPE], permuted indices, permuted face
    materials, mesh box (6,), device ms or None).  Raises CrtError; a GPU build that must defer to the
    host builder raises with status CRT_ERR_UNSUPPORTED (-5)."""
    pos = np.ascontiguousarray(positions, np.float32).reshape(-1)
    idx = np.ascontiguousarray(indices, np.uint32).copy()
    fm = np.ascontiguousarray(face_materials, np.int32).copy()
    n_tri = len(idx) // 3
    nodes = np.zeros(max(1, 2 * n_tri - 1), NODE_DTYPE)
    cnt = C.c_int32(0)
    box = np.zeros(6, np.float32)
    if device is None:
        rc = _lib.host().crth_build_mesh_bvh(_p(pos), len(pos) // 3, _p(idx), _p(fm), len(idx), _p(nodes),
                                             C.byref(cnt), _p(box))
        check_host(rc, "crth_build_mesh_bvh")
        ms = None
    else:
        t = C.c_float(0)
        rc = _lib.hip().crt_build_mesh_bvh(int(device), _p(pos), len(pos) // 3, _p(idx), _p(fm), len(idx), _p(nodes),
                                           C.byref(cnt), _p(box), C.byref(t))
        if rc != 0:
            err = CrtError(f"crt_build_mesh_bvh failed (status {rc}): "
                           f"{_lib.hip().crt_last_error().decode(errors='replace')}")
            err.status = rc
            raise err
        ms = t.value
    return nodes[:cnt.value], idx, fm, box, ms
