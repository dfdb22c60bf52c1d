"""Product host pipeline (C++ libcrt_host.so) vs the oracle restatement — CPU only.

Loader (SceneManager.h:198-329 + tinyobj v1.0), mesh/scene BVH builders
(Mesh.cuh:121-264, BVHNode.cuh:21-84) and Camera (Camera.cuh:159-182) must agree
bit-for-bit: the render kernel's traversal quirks depend on the exact tree.
"""
import os

import numpy as np
import pytest

import crt_amd
import objload
import pyoracle


def _compare_scene(files):
    hs = crt_amd.HostScene(files)
    L = objload.load_scene(files)
    pos, idx, fm, info, mats = hs.loader_arrays()
    assert np.array_equal(pos.view(np.uint32), L.positions.view(np.uint32))
    assert np.array_equal(idx, L.indices)
    assert np.array_equal(fm, L.facemat)
    assert np.array_equal(info, L.mesh_info)
    assert np.array_equal(mats.view(np.uint32), L.matdata.view(np.uint32))
    O = pyoracle.OracleScene(L)
    pidx, pfm = hs.permuted()
    for m in range(len(info)):
        (b, i), box = hs.mesh_bvh(m)
        ob, oi = O.nodes(m)
        n_idx = int(info[m, 3])
        oidx, ofm, obox = O.mesh_arrays(m, n_idx)
        assert np.array_equal(box.view(np.uint32), obox.view(np.uint32)), "Mesh::m_BoundingBox"
        if n_idx == 0:
            continue
        leaf = oi[:, 4] == 1
        assert np.array_equal(b.view(np.uint32), ob.view(np.uint32)), f"mesh {m} node boxes"
        assert np.array_equal(i[:, 4], oi[:, 4])
        assert np.array_equal(i[~leaf, :2], oi[~leaf, :2])
        assert np.array_equal(i[leaf, 2:4], oi[leaf, 2:4])
        s0, f0 = int(info[m, 2]), int(info[m, 4])
        assert np.array_equal(pidx[s0:s0 + n_idx], oidx)
        assert np.array_equal(pfm[f0:f0 + n_idx // 3], ofm)
    b, i = hs.scene_bvh()
    ob, oi = O.nodes(-1)
    assert np.array_equal(b.view(np.uint32), ob.view(np.uint32))
    assert np.array_equal(i, oi)
    return hs, L


@pytest.mark.parametrize("name", ["cornell", "cornell_bunny"])
def test_scene_pipeline_matches_oracle(scenes, name):
    _compare_scene(scenes[name])


def test_camera_matches_oracle():
    for kw in [dict(), dict(pos=(0.0, 4.0, 4.0), focus=5.656854, aspect=16 / 9), dict(yaw=-60.0, pitch=12.5, vfov=45.0)]:
        c = crt_amd.camera_floats(crt_amd.camera(7, **kw))
        o = pyoracle.camera(**kw)
        assert np.array_equal(c.view(np.uint32), o.view(np.uint32))
    d = crt_amd.camera(2000)
    assert d.samples_per_pixel == 2000 and d.pixel_sample_scale == np.float32(1.0) / np.float32(2000)


def _write(d, name, text):
    p = os.path.join(d, name)
    with open(p, "w") as f:
        f.write(text)
    return p


def test_loader_edge_cases(tmp_path):
    """tinyobj v1 semantics: fan triangulation of n-gons, negative (relative) indices, v/t/n
    tokens, unknown usemtl (-1 -> clamped to 0), unreferenced vertex slots (stay 0), odd
    float spellings; three files (materialIDOffset = previous mesh only, SceneManager.h:177)."""
    d = str(tmp_path)
    _write(d, "a.mtl", "newmtl red\nKd 0.9 0.1 0.1\nnewmtl mirror\nKd 0.8 0.8 0.8\nKs 1 1 1\nNs 30\n"
                       "newmtl lamp\nKe 4 4 4\nnewmtl glassy\nKd 1 1 1\nTr 0.25\nNi 1.33\n")
    a = _write(d, "a.obj", "mtllib a.mtl\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0.5 1.5 0\nv 9 9 9\n"
                           "usemtl red\nf 1 2 3 4 5\nusemtl nope\nf -6/1/1 -5//2 -4\nusemtl mirror\nf 1 3 5\n"
                           "v +0.25 -0.000 .5\nv 1e-2 2.5E+1 -3.125e0\nv 7 8\nusemtl lamp\nf -3 -2 -1\n"
                           "usemtl glassy\nf 2 3 4\n")
    _write(d, "b.mtl", "newmtl m0\nKd 0.2 0.3 0.4\nnewmtl m1\nKs 0.5 0 0\nPr 0.3\n")
    b = _write(d, "b.obj", "mtllib b.mtl\nv 0 0 1\nv 1 0 1\nv 0 1 1\nv 1 1 1\nusemtl m0\nf 1 2 3\nusemtl m1\nf 2 4 3\n")
    c = _write(d, "c.obj", "v 0 0 2\nv 1 0 2\nv 0 1 2\nf 1 2 3\n")
    hs, L = _compare_scene([a, b, c])
    info = L.mesh_info
    assert info[:, 5].tolist() == [0, 4, 2]          # previous mesh's unique ids: a uses {0,1,2,3}, b {0,1}
    assert L.mesh_info[0, 3] == 3 * (3 + 1 + 1 + 1 + 1)   # pentagon -> 3 triangles
    mt = L.matdata[:, 0].tolist()
    assert mt == [0.0, 1.0, 3.0, 2.0, 0.0, 1.0]       # lambertian, metal, light, dielectric(Tr), lambertian, metal


def test_loader_missing_file_raises(tmp_path):
    with pytest.raises(crt_amd.CrtError):
        crt_amd.HostScene([str(tmp_path / "nope.obj")])


def test_single_triangle_and_planar_mesh(tmp_path):
    d = str(tmp_path)
    one = _write(d, "one.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    _compare_scene([one])
    quad = _write(d, "quad.obj", "v -1 0 -1\nv 1 0 -1\nv 1 0 1\nv -1 0 1\nf 1 2 3 4\n")
    _compare_scene([quad])


def test_large_mesh_bvh_matches_oracle(tmp_path):
    """A 40k-triangle random soup (deep tree, many SAH/partition steps)."""
    rng = np.random.default_rng(3)
    n = 40000
    c = rng.uniform(-1, 1, (n, 3))
    v = (c[:, None, :] + rng.normal(scale=0.02, size=(n, 3, 3))).reshape(-1, 3)
    lines = ["v %.5f %.5f %.5f\n" % tuple(p) for p in v] + ["f %d %d %d\n" % (3 * k + 1, 3 * k + 2, 3 * k + 3) for k in range(n)]
    p = _write(str(tmp_path), "soup.obj", "".join(lines))
    _compare_scene([p])


def test_mesh_builder_abi_matches_scene_pipeline(scenes):
    """crth_build_mesh_bvh (the host restatement of Mesh::buildBVHMesh as a standalone C entry) builds the same
    tree and permutation as the scene pipeline, from the loader's unpermuted arrays."""
    import numpy as np
    import crt_amd
    hs = crt_amd.HostScene(scenes["cornell_bunny"])
    pos, idx, fm, info = hs.loader_arrays()[:4]
    pidx, pfm = hs.permuted()
    for i, m in enumerate(info):
        vo, vc, io, ic, fo = (int(x) for x in m[:5])
        nodes, oidx, ofm, box, _ = crt_amd.build_mesh_bvh(pos.reshape(-1, 3)[vo:vo + vc], idx[io:io + ic],
                                                         fm[fo:fo + ic // 3])
        (boxes, ints), aabb = hs.mesh_bvh(i)
        assert np.array_equal(np.concatenate([nodes["bmin"], nodes["bmax"]], 1).view(np.uint32), boxes.view(np.uint32))
        assert np.array_equal(np.stack([nodes[k] for k in ("left", "right", "obj_index", "obj_count", "is_leaf")], 1),
                              ints)
        assert np.array_equal(oidx, pidx[io:io + ic]) and np.array_equal(ofm, pfm[fo:fo + ic // 3])
        assert np.array_equal(box.view(np.uint32), aabb.view(np.uint32))
