"""ctypes bindings of the two C ABIs (include/crt_hip.h, include/crt_host.h).

The shared libraries are built in-tree (raytracer-cuda_amd/lib/) by `make`; this
module never falls back to anything else: if libcrt_hip.so is missing or does not
load, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]          # raytracer-cuda_amd/
REPO = PKG_ROOT.parent
LIB_DIR = PKG_ROOT / "lib"
# CRT_HIP_LIB: an alternative build of the same library (A/B profiling builds, tools/); default in-tree
HIP_LIB = Path(os.environ["CRT_HIP_LIB"]) if os.environ.get("CRT_HIP_LIB") else LIB_DIR / "libcrt_hip.so"
# CRT_HOST_LIB: an alternative build of the host library (the sanitizer build, `make asan`, tools/run_asan.sh)
HOST_LIB = Path(os.environ["CRT_HOST_LIB"]) if os.environ.get("CRT_HOST_LIB") else LIB_DIR / "libcrt_host.so"


class CrtError(RuntimeError):
    pass


def build(jobs: int = 8) -> None:
    """Compile libcrt_hip.so (gfx950) + libcrt_host.so + crt_render in-tree."""
    subprocess.run(["make", "-C", str(PKG_ROOT), f"-j{jobs}", "all"], check=True)


class CameraDesc(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("lower_left", C.c_float * 3), ("horizontal", C.c_float * 3),
                ("vertical", C.c_float * 3), ("right", C.c_float * 3), ("up", C.c_float * 3),
                ("lens_radius", C.c_float), ("samples_per_pixel", C.c_int32), ("pixel_sample_scale", C.c_float)]


class CrthInput(C.Structure):        # crt_host.h crth_input
    _fields_ = [("mouse_x", C.c_float), ("mouse_y", C.c_float), ("right_mouse", C.c_int32), ("keys", C.c_uint32),
                ("focus_steps", C.c_int32)]


class CrthFrameInfo(C.Structure):    # crt_host.h crth_frame_info
    _fields_ = [("frame", C.c_int64), ("spp", C.c_int32), ("accumulated", C.c_int32), ("moving", C.c_int32),
                ("high_quality", C.c_int32), ("kernel_ms", C.c_float), ("frame_ms", C.c_double)]


class SceneDesc(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("n_positions", C.c_uint64), ("indices", C.c_void_p),
                ("n_indices", C.c_uint64), ("face_materials", C.c_void_p), ("n_faces", C.c_uint64),
                ("meshes", C.c_void_p), ("n_meshes", C.c_int32), ("spheres", C.c_void_p), ("n_spheres", C.c_int32),
                ("objects", C.c_void_p), ("n_objects", C.c_int32), ("scene_nodes", C.c_void_p),
                ("n_scene_nodes", C.c_int32), ("materials", C.c_void_p), ("n_materials", C.c_int32)]


class BvhNodeDesc(C.Structure):
    _fields_ = [("bmin", C.c_float * 3), ("bmax", C.c_float * 3), ("left", C.c_int32), ("right", C.c_int32),
                ("obj_index", C.c_int32), ("obj_count", C.c_int32), ("is_leaf", C.c_int32)]


class MeshDesc(C.Structure):
    _fields_ = [("vertex_offset", C.c_uint32), ("vertex_count", C.c_uint32), ("index_offset", C.c_uint32),
                ("index_count", C.c_uint32), ("face_offset", C.c_uint32), ("material_id_offset", C.c_uint32),
                ("nodes", C.c_void_p), ("node_count", C.c_int32), ("aabb", C.c_float * 6)]


class MaterialDesc(C.Structure):      # crt_hip.h crt_material_desc
    _fields_ = [("type", C.c_int32), ("albedo", C.c_float * 3), ("emission", C.c_float * 3), ("roughness", C.c_float),
                ("ior", C.c_float)]


class SceneStats(C.Structure):
    _fields_ = [("device_nodes", C.c_int64), ("device_prims", C.c_int64), ("device_bytes", C.c_int64),
                ("max_depth", C.c_int32), ("n_materials", C.c_int32), ("bvh", C.c_int32), ("layouts", C.c_int32),
                ("excluded_prims", C.c_int64), ("width", C.c_int32), ("stack_bound", C.c_int32),
                ("spatial_splits", C.c_int64), ("references", C.c_int64)]


class SceneOptions(C.Structure):
    _fields_ = [("bvh", C.c_int32), ("leaf_size", C.c_int32), ("layouts", C.c_int32),
                ("traversal_cost", C.c_float), ("width", C.c_int32), ("gpu_build", C.c_int32),
                ("stack_cap", C.c_int32), ("spatial_splits", C.c_int32),
                ("spatial_alpha", C.c_float), ("spatial_max_dup", C.c_float)]


BVH_REFERENCE = 0
BVH_REBUILT = 1
ABI_VERSION = 3          # include/crt_hip.h CRT_ABI_VERSION
BUILD_CHECKED = 1        # crt_build_flags(): the -DCRT_CHECKED build


class WorkCounters(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("box_tests", C.c_uint64), ("tri_tests", C.c_uint64),
                ("sphere_tests", C.c_uint64), ("paths", C.c_uint64)]


# exported symbol lists (checked by tests against include/*.h)
HIP_SYMBOLS = [
    "crt_abi_version", "crt_build_flags", "crt_last_error", "crt_device_count", "crt_scene_create", "crt_scene_create_ex", "crt_scene_get_stats", "crt_scene_compare", "crt_scene_compare_dump", "crt_scene_export",
    "crt_renderer_set_stack_lds", "crt_renderer_get_section_profile", "crt_renderer_get_section_profile_ex",
    "crt_scene_destroy", "crt_renderer_create", "crt_renderer_destroy", "crt_renderer_init_rand",
    "crt_renderer_set_camera", "crt_renderer_render", "crt_renderer_resolve", "crt_renderer_render_frame",
    "crt_renderer_synchronize", "crt_renderer_read_linear", "crt_renderer_read_rgba8", "crt_renderer_read_rng",
    "crt_renderer_write_linear", "crt_renderer_get_counters", "crt_renderer_linear_device_ptr",
    "crt_renderer_rgba_device_ptr", "crt_renderer_rng_device_ptr", "crt_renderer_last_kernel_ms",
    "crt_renderer_last_kernel_name", "crt_renderer_last_timings", "crt_renderer_last_schedule", "crt_renderer_timing_history",
    "crt_renderer_set_leaf_carry", "crt_renderer_set_xcd_regions", "crt_renderer_set_temporal_order",
    "crt_renderer_set_drain_threshold", "crt_renderer_set_wave_drain",
    "crt_renderer_attach_linear", "crt_renderer_set_kernel_variant", "crt_renderer_get_schedule_stats",
    "crt_renderer_set_regen_threshold", "crt_renderer_set_occupancy_target",
    "crt_build_mesh_bvh", "crt_renderer_set_schedule", "crt_renderer_set_critical_tiles", "crt_renderer_set_pixel_shard",
    "crt_renderer_set_top_levels",
    "crt_selftest_math", "crt_selftest_rng", "crt_selftest_geometry", "crt_selftest_scan", "crt_selftest_rcp",
    "crt_selftest_uv_div", "crt_selftest_sqrt",
]
HOST_SYMBOLS = [
    "crth_scene_load", "crth_scene_load_ex", "crth_scene_build_ms", "crth_scene_destroy", "crth_scene_desc", "crth_scene_upload", "crth_scene_upload_ex", "crth_scene_counts",
    "crth_scene_loader_arrays", "crth_camera", "crth_last_error", "crth_encode_image", "crth_write_image",
    "crth_build_mesh_bvh", "crth_camera_create", "crth_camera_update", "crth_camera_get", "crth_camera_destroy",
    "crth_viewer_create", "crth_viewer_frame", "crth_viewer_camera", "crth_viewer_renderer", "crth_viewer_destroy",
]

_hip = None
_host = None


def _bind_single_runtime() -> None:
    """Import torch before libcrt_hip.so so the process holds ONE HIP runtime.

    PyTorch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64.so.1; once torch is
    loaded, libcrt_hip.so's DT_NEEDED entries resolve to those same objects by SONAME, so
    torch tensors (RCCL framebuffer reduce) and the crt kernels share one device context.
    Set CRT_NO_TORCH=1 to bind the system ROCm runtime instead (no torch interop)."""
    if os.environ.get("CRT_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def hip():
    global _hip
    if _hip is None:
        _bind_single_runtime()
        if not HIP_LIB.exists():
            raise CrtError(f"{HIP_LIB} not built (run `make -C {PKG_ROOT}` or __graft_entry__.build())")
        L = C.CDLL(str(HIP_LIB), mode=C.RTLD_GLOBAL)
        P, i32, u64, f32 = C.c_void_p, C.c_int, C.c_ulonglong, C.c_float
        sig = {
            "crt_abi_version": ([], i32), "crt_build_flags": ([], i32), "crt_last_error": ([], C.c_char_p),
            "crt_device_count": ([P], i32),
            "crt_scene_create": ([P, i32, P], i32), "crt_scene_create_ex": ([P, i32, P, P], i32),
            "crt_scene_compare": ([P, P, P, i32, i32, P], i32),
            "crt_scene_compare_dump": ([P, P, P, i32, i32, P, P, i32], i32),
            "crt_scene_export": ([P, P, P, P, P, P], i32), "crt_renderer_set_stack_lds": ([P, i32], i32),
            "crt_renderer_get_section_profile": ([P, P], i32),
            "crt_renderer_get_section_profile_ex": ([P, P, i32], i32),
            "crt_scene_get_stats": ([P, P], i32),
            "crt_scene_destroy": ([P], None),
            "crt_renderer_create": ([i32, i32, i32, P], i32), "crt_renderer_destroy": ([P], None),
            "crt_renderer_init_rand": ([P, u64, u64, P], i32), "crt_renderer_set_camera": ([P, P], i32),
            "crt_renderer_render": ([P, P, i32, i32, C.c_uint, P], i32),
            "crt_renderer_resolve": ([P, f32, P], i32), "crt_renderer_render_frame": ([P, P, P], i32),
            "crt_renderer_set_pixel_shard": ([P, i32, i32], i32),
            "crt_renderer_synchronize": ([P, P], i32), "crt_renderer_last_timings": ([P, P], i32), "crt_renderer_last_schedule": ([P, P], i32),
            "crt_renderer_timing_history": ([P, i32, P], i32),
            "crt_renderer_set_leaf_carry": ([P, i32, i32], i32),
            "crt_renderer_set_xcd_regions": ([P, i32], i32),
            "crt_renderer_set_temporal_order": ([P, i32], i32),
            "crt_renderer_set_drain_threshold": ([P, i32], i32),
            "crt_renderer_set_wave_drain": ([P, i32], i32),
            "crt_renderer_read_linear": ([P, P], i32), "crt_renderer_read_rgba8": ([P, P], i32),
            "crt_renderer_read_rng": ([P, P], i32), "crt_renderer_write_linear": ([P, P], i32),
            "crt_renderer_get_counters": ([P, P], i32),
            "crt_renderer_linear_device_ptr": ([P], P), "crt_renderer_rgba_device_ptr": ([P], P),
            "crt_renderer_rng_device_ptr": ([P], P), "crt_renderer_last_kernel_ms": ([P], f32),
            "crt_renderer_last_kernel_name": ([P], C.c_char_p),
            "crt_renderer_attach_linear": ([P, P], i32),
            "crt_renderer_set_kernel_variant": ([P, i32], i32),
            "crt_renderer_get_schedule_stats": ([P, P], i32),
            "crt_renderer_set_regen_threshold": ([P, i32], i32),
            "crt_renderer_set_occupancy_target": ([P, i32], i32),
            "crt_renderer_set_schedule": ([P, i32, i32, i32], i32),
            "crt_renderer_set_critical_tiles": ([P, i32, i32], i32),
            "crt_renderer_set_top_levels": ([P, i32], i32),
            "crt_build_mesh_bvh": ([i32, P, C.c_uint32, P, P, C.c_uint32, P, P, P, P], i32),
            "crt_selftest_math": ([P, P, i32, P, P], i32),
            "crt_selftest_geometry": ([i32, P, i32, P, i32, i32, P, P], i32),
            "crt_selftest_rng": ([u64, P, i32, i32, P, P], i32),
            "crt_selftest_scan": ([P, i32, P], i32),
            "crt_selftest_rcp": ([C.c_uint32, C.c_uint32, P, P], i32),
            "crt_selftest_uv_div": ([i32, P], i32),
            "crt_selftest_sqrt": ([C.c_uint32, C.c_uint32, P, P], i32),
        }
        for name, (args, res) in sig.items():
            if os.environ.get("CRT_SKIP_ABI_CHECK") and not hasattr(L, name):
                continue   # an A/B build of an older revision: self-tests added since then are absent
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        # every library is checked, CRT_HIP_LIB overrides included (a stale build would silently misread newer
        # fields); A/B runs against an older revision's build opt out explicitly with CRT_SKIP_ABI_CHECK=1
        if L.crt_abi_version() != ABI_VERSION and not os.environ.get("CRT_SKIP_ABI_CHECK"):
            raise CrtError(f"{HIP_LIB}: C ABI version {L.crt_abi_version()}, these bindings expect {ABI_VERSION} "
                           "(rebuild the library, or set CRT_SKIP_ABI_CHECK=1 for an A/B run of an older build)")
        _hip = L
    return _hip


def host():
    global _host
    if _host is None:
        hip()   # load libcrt_hip.so first (RTLD_GLOBAL) so libcrt_host resolves against the in-tree copy
        if not HOST_LIB.exists():
            raise CrtError(f"{HOST_LIB} not built")
        L = C.CDLL(str(HOST_LIB))
        P, i32, f32 = C.c_void_p, C.c_int, C.c_float
        sig = {
            "crth_scene_load": ([P, i32, P], i32), "crth_scene_load_ex": ([P, i32, i32, P], i32),
            "crth_scene_build_ms": ([P], C.c_double), "crth_scene_destroy": ([P], None),
            "crth_scene_desc": ([P, P], i32), "crth_scene_upload": ([P, i32, P], i32),
            "crth_scene_upload_ex": ([P, i32, P, P], i32),
            "crth_scene_counts": ([P, P], i32), "crth_scene_loader_arrays": ([P, P, P, P, P, P], i32),
            "crth_camera": ([f32, f32, P, P, f32, f32, f32, f32, i32, P], i32),
            "crth_last_error": ([], C.c_char_p),
            "crth_encode_image": ([i32, P, i32, i32, i32, P, P], i32),
            "crth_write_image": ([C.c_char_p, P, i32, i32, i32], i32),
            "crth_camera_create": ([f32, f32, P, P, f32, f32, P], i32),
            "crth_build_mesh_bvh": ([P, C.c_uint32, P, P, C.c_uint32, P, P, P], i32),
            "crth_camera_update": ([P, f32, i32, i32, P], i32),
            "crth_camera_get": ([P, P, P], i32), "crth_camera_destroy": ([P], None),
            "crth_viewer_create": ([P, i32, i32, P, i32, i32, f32, f32, f32, P, f32, C.c_ulonglong, i32, P], i32),
            "crth_viewer_frame": ([P, f32, P, P], i32), "crth_viewer_camera": ([P, P], i32),
            "crth_viewer_renderer": ([P], P), "crth_viewer_destroy": ([P], None),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _host = L
    return _host


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = hip().crt_last_error().decode(errors="replace")
        raise CrtError(f"{what} failed (status {rc}): {msg}")


def check_host(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = host().crth_last_error().decode(errors="replace")
        raise CrtError(f"{what} failed (status {rc}): {msg}")
