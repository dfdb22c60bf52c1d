"""The C-ABI libraries load and export every symbol include/*.h declares (no GPU needed)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _declared(header: Path, prefix: str):
    txt = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    names = set(re.findall(r"\b(%s\w+)\s*\(" % prefix, txt))
    return sorted(names)


def _exported(lib: Path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


def test_hip_library_exports_header():
    from crt_amd import _lib
    decl = _declared(REPO / "include" / "crt_hip.h", "crt_")
    exp = _exported(_lib.HIP_LIB)
    missing = [d for d in decl if d not in exp]
    assert not missing, missing
    assert sorted(_lib.HIP_SYMBOLS) == decl
    # only the C ABI is exported
    assert all(s.startswith("crt_") for s in exp if not s.startswith("_")), sorted(exp)[:10]


def test_host_library_exports_header():
    from crt_amd import _lib
    decl = _declared(REPO / "include" / "crt_host.h", "crth_")
    assert not [d for d in decl if d not in _exported(_lib.HOST_LIB)]
    assert sorted(_lib.HOST_SYMBOLS) == decl


def test_libraries_load_without_gpu():
    from crt_amd import _lib
    L = _lib.hip()
    assert L.crt_abi_version() == 3
    n = C.c_int(-1)
    assert L.crt_device_count(C.byref(n)) == 0 and n.value >= 0
    _lib.host()


def test_timings_need_a_render():
    from crt_amd import _lib
    ms = (C.c_float * 3)()
    assert _lib.hip().crt_renderer_last_timings(None, ms) == -1
    assert _lib.hip().crt_renderer_timing_history(None, 0, ms) == -1
    assert _lib.hip().crt_build_flags() == 0


def test_errors_are_reported_not_thrown():
    import crt_amd
    from crt_amd import _lib
    h = C.c_void_p()
    rc = _lib.hip().crt_renderer_create(0, 10, 0, C.byref(h))
    assert rc == -1 and b"size" in _lib.hip().crt_last_error()
    assert _lib.hip().crt_scene_create(None, 0, C.byref(h)) == -1
    with pytest.raises(crt_amd.CrtError):
        crt_amd._lib.check(-1, "x")


def test_cli_binary_built():
    assert (REPO / "raytracer-cuda_amd" / "bin" / "crt_render").exists()
