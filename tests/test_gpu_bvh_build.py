"""GPU-parallel mesh BVH build against the sequential host restatement of the reference's
builder (Mesh::buildBVHMesh, Mesh.cuh:121-264; the host restatement is pinned to the oracle by
test_host_parity.py).

Bar: identical node arrays (structure, leaf ranges, node order) and identical index / face-material
permutations; boxes equal as floats (the GPU's ordered-integer min/max may pick -0 where a sequential
fminf keeps +0, see csrc/crt_bvh_build.hip), bit-identical everywhere else.  Meshes where the reference's
node cap decides the tree must be refused (CRT_ERR_UNSUPPORTED) so callers fall back to the host builder.
"""
import time

import numpy as np
import pytest

import crt_amd

pytestmark = pytest.mark.gpu


def _soup(n_tri, n_vert, seed, quantize=None):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n_vert, 3)).astype(np.float32)
    if quantize:
        v = (np.round(v * quantize) / quantize).astype(np.float32)   # many equal centroids / coordinates
    idx = rng.integers(0, n_vert, 3 * n_tri).astype(np.uint32)
    fm = rng.integers(0, 7, n_tri).astype(np.int32)
    return v, idx, fm


def _assert_same(host, gpu):
    hn, hi, hf, hb, _ = host
    gn, gi, gf, gb, _ = gpu
    assert len(hn) == len(gn)
    for f in ("left", "right", "obj_index", "obj_count", "is_leaf"):
        d = np.nonzero(hn[f] != gn[f])[0]
        assert len(d) == 0, f"{f} differs at nodes {d[:8].tolist()}"
    for f in ("bmin", "bmax"):
        assert np.array_equal(hn[f], gn[f]), f
        bits = hn[f].view(np.uint32) != gn[f].view(np.uint32)
        assert np.all(hn[f][bits] == 0), f"{f}: bit differences other than the sign of zero"
    assert np.array_equal(hi, gi), "index permutation"
    assert np.array_equal(hf, gf), "face-material permutation"
    assert np.array_equal(hb, gb)


def _both(v, idx, fm):
    return crt_amd.build_mesh_bvh(v, idx, fm), crt_amd.build_mesh_bvh(v, idx, fm, device=0)


@pytest.mark.parametrize("n_tri,n_vert,seed,quant", [
    (1, 3, 0, None), (10, 30, 1, None), (11, 33, 2, None), (12, 20, 3, None), (64, 100, 4, None),
    (1000, 700, 5, None), (50_000, 30_000, 6, None), (200_000, 100_000, 7, None),
    (5000, 4000, 8, 4.0), (20_000, 2000, 9, 8.0),
])
def test_random_soups(n_tri, n_vert, seed, quant):
    host, gpu = _both(*_soup(n_tri, n_vert, seed, quant))
    _assert_same(host, gpu)


def test_scene_meshes(scenes):
    """Every mesh of the benchmark scenes: the loader's (unpermuted) arrays through both builders, and the
    GPU result equals the tree the scene pipeline built (SceneManager, host)."""
    for name, files in scenes.items():
        hs = crt_amd.HostScene(files)
        pos, idx, fm, info = hs.loader_arrays()[:4]
        pos = pos.reshape(-1, 3)
        for i, m in enumerate(info):
            vo, vc, io, ic, fo = (int(x) for x in m[:5])
            host, gpu = _both(pos[vo:vo + vc], idx[io:io + ic], fm[fo:fo + ic // 3])
            _assert_same(host, gpu)
            (boxes, ints), aabb = hs.mesh_bvh(i)
            assert np.array_equal(boxes[:, :3], gpu[0]["bmin"]) and np.array_equal(boxes[:, 3:], gpu[0]["bmax"])
            assert np.array_equal(ints[:, 0], gpu[0]["left"]) and np.array_equal(ints[:, 4], gpu[0]["is_leaf"])
            assert np.array_equal(aabb, gpu[3])


def test_million_triangles_speed():
    v, idx, fm = _soup(1_000_000, 500_000, 11)
    t = time.perf_counter()
    host = crt_amd.build_mesh_bvh(v, idx, fm)
    t_host = time.perf_counter() - t
    crt_amd.build_mesh_bvh(v[:1000], idx[:3000] % 1000, fm[:1000], device=0)   # warm up the code object
    t = time.perf_counter()
    gpu = crt_amd.build_mesh_bvh(v, idx, fm, device=0)
    t_gpu = time.perf_counter() - t
    _assert_same(host, gpu)
    print(f"\n1M-triangle mesh BVH: host {t_host * 1e3:.1f} ms, GPU call {t_gpu * 1e3:.1f} ms "
          f"(device {gpu[4]:.1f} ms), {len(gpu[0])} nodes")


def test_degenerate_split_is_refused():
    """All centroids identical: every SAH cost is NaN, the fallback split (axis 0, pos 0) puts everything on
    one side and the reference's node cap ends the recursion.  The GPU build must defer to the host."""
    v = np.array([[1, 1, 1], [2, 1, 1], [1, 2, 1], [0, 1, 1]], np.float32)
    idx = np.tile(np.array([0, 1, 2], np.uint32), 40)
    fm = np.zeros(40, np.int32)
    with pytest.raises(crt_amd.CrtError) as e:
        crt_amd.build_mesh_bvh(v, idx, fm, device=0)
    assert e.value.status == -5
    crt_amd.build_mesh_bvh(v, idx, fm)   # the host builder handles it (node cap)


def test_stack_overflow_matches_host():
    """A coarsely quantized soup (coincident triangles, a tree deeper than the reference's 64-entry stack): the
    host restatement reports the overflow; the GPU build refuses it (degenerate split, status -5: the host builder
    decides, as SceneManager does) or reports the same overflow."""
    v, idx, fm = _soup(20_000, 600, 9, 2.0)
    with pytest.raises(crt_amd.CrtError, match="stack overflow"):
        crt_amd.build_mesh_bvh(v, idx, fm)
    with pytest.raises(crt_amd.CrtError) as e:
        crt_amd.build_mesh_bvh(v, idx, fm, device=0)
    assert e.value.status == -5 or "stack overflow" in str(e.value)


def test_bad_index_is_an_error():
    v = np.zeros((3, 3), np.float32)
    with pytest.raises(crt_amd.CrtError):
        crt_amd.build_mesh_bvh(v, np.array([0, 1, 7] * 12, np.uint32), np.zeros(12, np.int32), device=0)


# ---- the CRT_BVH_REBUILT binned-SAH tree built on the GPU (crt_scene_options.gpu_build) ----

def _export(hs, gpu):
    return hs.export("rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=gpu)


def _leaf_rank_sets(ex):
    """Per 4-wide node: the multiset of primitive ranks under its leaf slots (order inside a leaf is free)."""
    nodes, prims = ex["nodes"].reshape(-1, 8, 4), ex["prims"].reshape(-1, 3, 4)
    out = []
    for n in range(ex["nodes_per_layout"]):
        meta = nodes[n, 6].view(np.int32)
        first, counts = int(meta[2]), int(meta[3])
        total = sum((counts >> (8 * s)) & 0xff for s in range(4))
        out.append(sorted(prims[first:first + total, 2, 2].view(np.int32).tolist()))
    return out


@pytest.mark.parametrize("scene", ["cornell", "cornell_bunny"])
def test_gpu_sah_tree_equals_host(scenes, scene):
    """Bin counts and boxes are order-independent, so the GPU build makes the host's splits: same nodes, same
    boxes, same primitives under every node; only the order inside a leaf may differ (stable partition)."""
    hs = crt_amd.HostScene(scenes[scene])
    h, g = _export(hs, False), _export(hs, True)
    keys = [k for k, v in h.items() if isinstance(v, int)]
    assert {k: h[k] for k in keys} == {k: g[k] for k in keys}
    hn, gn = h["nodes"].reshape(-1, 8, 4), g["nodes"].reshape(-1, 8, 4)
    assert np.array_equal(hn[:, :6], gn[:, :6]), "child boxes"
    assert np.array_equal(hn[:, 6].view(np.int32), gn[:, 6].view(np.int32)), "node meta"
    assert _leaf_rank_sets(h) == _leaf_rank_sets(g)


def test_gpu_sah_scene_renders_identically(scenes):
    """Leaf order does not change any hit (closest t, ties to the higher rank): the frames are bit-identical."""
    hs = crt_amd.HostScene(scenes["cornell_bunny"])
    a = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0)
    b = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    out = []
    for sc in (a, b):
        r = crt_amd.Renderer(160, 90)
        r.set_camera(crt_amd.camera(16))
        r.init_rand(41)
        r.render(sc, 16, 20)
        r.synchronize()
        out.append((r.linear(), r.counters()["rays"]))
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32)) and out[0][1] == out[1][1]


def test_gpu_sah_million_triangles():
    from crt_amd import assets
    hs = crt_amd.HostScene(assets.scene_files("cornell_1m"), build_device=0)
    t = time.perf_counter()
    h = _export(hs, False)
    t_host = time.perf_counter() - t
    _export(hs, True)   # warm-up
    t = time.perf_counter()
    g = _export(hs, True)
    t_gpu = time.perf_counter() - t
    assert h["nodes_per_layout"] == g["nodes_per_layout"] and h["prim_float4s"] == g["prim_float4s"]
    hn, gn = h["nodes"].reshape(-1, 8, 4), g["nodes"].reshape(-1, 8, 4)
    assert np.array_equal(hn[:, :6], gn[:, :6]) and np.array_equal(hn[:, 6].view(np.int32), gn[:, 6].view(np.int32))
    print(f"\n1M-triangle rebuilt-scene export: host SAH {t_host * 1e3:.0f} ms, GPU SAH {t_gpu * 1e3:.0f} ms")
