"""The oracle itself, pinned against every external anchor available in this image."""
import json
import re
from pathlib import Path

import numpy as np
import pytest

import objload
import pyoracle

GOLDEN = Path(__file__).resolve().parent / "golden"
ROCRAND_TABLE = Path("/opt/rocm/include/rocrand/rocrand_xorwow_precomputed.h")


@pytest.mark.skipif(not ROCRAND_TABLE.exists(), reason="rocRAND headers not present")
def test_xorwow_sequence_jump_matches_rocrand_table():
    """A^(2^67 * 4^k) (curand_init subsequence skip) == rocRAND's published h_xorwow_sequence_jump_matrices."""
    txt = ROCRAND_TABLE.read_text()
    i = txt.index("h_xorwow_sequence_jump_matrices")
    body = txt[i:txt.index("};", i)].split("=", 1)[1]
    nums = [int(x.rstrip("uU"), 0) for x in re.findall(r"0x[0-9a-fA-F]+[uU]?|\b\d+[uU]?\b", body)]
    tab = np.array(nums, dtype=np.uint64).astype(np.uint32).reshape(32, 800)
    for k in range(32):
        assert np.array_equal(pyoracle.seq_matrix(k), tab[k]), f"matrix {k}"


def test_xorwow_recurrence_and_uniform():
    """Marsaglia xorwow step + cuRAND uniform mapping x*2^-32 + 2^-33 on a hand-stepped state."""
    st = pyoracle.rng_init(41, 0)
    v = [int(x) for x in st[:5]]
    d = int(st[5])
    u, f = pyoracle.rng_draw(st.copy(), 5)
    M = 0xFFFFFFFF
    for k in range(5):
        t = (v[0] ^ (v[0] >> 2)) & M
        v = v[1:] + [((v[4] ^ ((v[4] << 4) & M)) ^ (t ^ ((t << 1) & M))) & M]
        d = (d + 362437) & M
        x = (v[4] + d) & M
        assert u[k] == x
        assert f[k] == np.float32(np.float32(x) * np.float32(2.3283064e-10) + np.float32(2.3283064e-10 / 2))
    assert 0.0 < f.min() and f.max() <= 1.0


def test_xorwow_golden_kat():
    for e in json.loads((GOLDEN / "xorwow_kat.json").read_text()):
        st = pyoracle.rng_init(e["seed"], e["subsequence"])
        assert st.tolist() == e["state"]
        u, f = pyoracle.rng_draw(st.copy(), len(e["u32"]))
        assert u.tolist() == e["u32"]
        assert [format(int(x), "08x") for x in f.view(np.uint32)] == e["uniform_hex"]


@pytest.mark.parametrize("bounces,rays", [(4, 3197876), (20, 3420058)])
def test_reference_run_ray_counts(scenes, bounces, rays):
    """Config A (Cornell, 256x256, 16 spp, bench camera): the number of closest-hit queries
    equals the count the survey measured by running the reference's own headers
    (BASELINE.md survey-container table) — a whole-path checksum."""
    S = pyoracle.OracleScene(objload.load_scene(scenes["cornell"]))
    s, rgba, c = S.render(pyoracle.camera(), 256, 256, 16, bounces)
    assert c["rays"] == rays
    g = json.loads((GOLDEN / "frames.json").read_text())[f"configA_256x256_16spp_{bounces}b"]
    import hashlib
    assert hashlib.sha256(s.tobytes()).hexdigest() == g["sum_sha256"]
    assert hashlib.sha256(rgba.tobytes()).hexdigest() == g["rgba_sha256"]


def test_cornell_bunny_golden_frame(oracle_scenes):
    g = np.load(GOLDEN / "cornell_bunny_64x36_16spp.npz")
    s, rgba, c = oracle_scenes["cornell_bunny"].render(pyoracle.camera(), 64, 36, 16, 20)
    assert np.array_equal(s.view(np.uint32), g["sum"].view(np.uint32))
    assert np.array_equal(rgba, g["rgba"])
    meta = json.loads((GOLDEN / "frames.json").read_text())["cornell_bunny_64x36_16spp_20b"]
    assert c["rays"] == meta["rays"] and c["tri_tests"] == meta["tri_tests"]


def test_config_e_slice_golden_frame():
    """Config E's 1M-triangle scene (instanced bunnies) at 64x36, 8 spp: the oracle reproduces the committed
    fixture (sums, RGBA8, ray count); the GPU suite holds both BVH paths to the same file."""
    from crt_amd import assets
    import hashlib
    g = np.load(GOLDEN / "cornell_1m_64x36_8spp.npz")
    S = pyoracle.OracleScene(objload.load_scene(assets.scene_files("cornell_1m")))
    s, rgba, c = S.render(pyoracle.camera(), 64, 36, 8, 20)
    assert np.array_equal(s.view(np.uint32), g["sum"].view(np.uint32))
    assert np.array_equal(rgba, g["rgba"])
    meta = json.loads((GOLDEN / "frames.json").read_text())["cornell_1m_64x36_8spp_20b"]
    assert c["rays"] == int(g["rays"][0]) == meta["rays"]
    assert hashlib.sha256(s.tobytes()).hexdigest() == meta["sum_sha256"]


def test_bvh_golden(scenes, oracle_scenes):
    g = json.loads((GOLDEN / "scene_bvh.json").read_text())
    S = oracle_scenes["cornell"]
    b, i = S.nodes(0)
    assert [format(int(x), "08x") for x in b.view(np.uint32).ravel()] == g["cornell_mesh"]["boxes_hex"]
    assert i.tolist() == g["cornell_mesh"]["ints"]
    b, i = S.nodes(-1)
    assert i.tolist() == g["cornell_scene"]["ints"]
    bb, bi = oracle_scenes["cornell_bunny"].nodes(1)
    assert len(bb) == g["bunny_mesh"]["n_nodes"]


def test_zero_thickness_leaf_is_never_hit():
    """AABB.cuh quirk: an unpadded flat leaf box (computeTrianglesAABB) gives tmax == tmin
    for rays through its plane, so the reference never hits an axis-aligned planar leaf."""
    import ctypes as C
    import tempfile
    import os
    with tempfile.TemporaryDirectory() as d:
        # a single axis-aligned quad (2 triangles < 10 => one leaf, zero thickness in y)
        obj = os.path.join(d, "flat.obj")
        with open(obj, "w") as f:
            f.write("v -1 0 -1\nv 1 0 -1\nv 1 0 1\nv -1 0 1\nf 1 2 3 4\n")
        L = objload.load_scene([obj])
        S = pyoracle.OracleScene(L)
        b, i = S.nodes(0)
        assert len(b) == 1 and i[0, 4] == 1 and b[0, 1] == b[0, 4]    # leaf, min.y == max.y
        cam = pyoracle.camera(pos=(0.0, 0.2, 0.0), yaw=-90.0, pitch=-89.0)
        s, rgba, c = S.render(cam, 8, 8, 1, 1)
        # every ray misses the (invisible) quad; 1-bounce paths end on sky or the ground sphere (returns 0)
        assert c["tri_tests"] == 0
