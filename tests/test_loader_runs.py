"""The OBJ parser's runs (host/crt/ObjLoader.cpp): a large file is parsed in up to 16 runs of whole lines at once and
joined in file order.  Whatever the cut, the loaded scene must be the one-run scene: relative face indices that reach
into earlier runs, usemtl / mtllib lines in other runs than their faces, polygons, CRLF, malformed lines and errors.
CPU only; CRT_OBJ_RUN_BYTES sets the run size (read at every load).
"""
import os

import numpy as np
import pytest

import crt_amd
from crt_amd import assets
from test_loader_fuzz import HAND, VALID_MTL, VALID_OBJ, _write


def _load(files, run_bytes):
    old = os.environ.get("CRT_OBJ_RUN_BYTES")
    os.environ["CRT_OBJ_RUN_BYTES"] = str(run_bytes)
    try:
        hs = crt_amd.HostScene(files)
    except crt_amd.CrtError as e:
        return ("rejected", str(e))
    finally:
        if old is None:
            del os.environ["CRT_OBJ_RUN_BYTES"]
        else:
            os.environ["CRT_OBJ_RUN_BYTES"] = old
    return tuple(np.ascontiguousarray(a).tobytes() for a in hs.loader_arrays())


@pytest.mark.parametrize("case", range(len(HAND) + 1))
def test_runs_load_the_one_run_scene(tmp_path, case):
    _write(str(tmp_path), "m.mtl", VALID_MTL)
    obj = _write(str(tmp_path), "s.obj", VALID_OBJ if case == len(HAND) else HAND[case])
    one = _load([obj], 1 << 30)
    for rb in (1, 5, 17, 64):
        assert _load([obj], rb) == one, f"run size {rb}"


def test_runs_on_the_bundled_scenes():
    files = assets.scene_files("cornell_bunny")
    one = _load(files, 1 << 30)
    for rb in (4096, 1 << 16):
        assert _load(files, rb) == one
