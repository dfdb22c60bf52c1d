"""The reference's rarely-taken paths and config B on the GPU, against the CPU oracle (calls go through the C ABI).

* Config B (BASELINE.json configs[1]): Cornell + bunny proxy, 1280x720, 256 spp, 20 bounces.  The reference-BVH
  frame is checked bit for bit on bands of pixels at the full 256 spp and on the whole frame at 4 spp; the
  benchmarked rebuilt-BVH path (variant 8 at 256 spp) against that frame by the north-star bar.
* Fuzzy Metal (Material.cuh:86-96): MTL materials with Ks > 0 and an Ns- or Pr-derived roughness
  (SceneManager.h:231-237), assets/MetalBlocks.obj.
* Three OBJ files: the per-mesh materialIDOffset is the unique-material count of the PREVIOUS mesh only
  (SceneManager.h:143-145, :177), so the third file's faces index the first file's materials.
* An out-of-range material index (CUDAKernels.h:127): the reference skips scatter and traces the same ray again
  on the next bounce.  The reference's loader cannot produce one; the C ABI can (a caller's materialIDOffset).
* A traversal deeper than the scene's stack bound (forced with the testing override crt_scene_options.stack_cap)
  surfaces as CRT_ERR_HIP at synchronisation, through HIPRenderer::render too (CUDARenderer.cuh:59).

Bar: bit-exact fp32 sums, RGBA8 bytes and ray counts on the reference BVH; <= 1e-4 per-channel RMS and >= 99.9 % of
pixels bit-identical on the rebuilt 4-wide BVH (kernel variants 7 and 8).
"""
import ctypes as C

import numpy as np
import pytest

import crt_amd
import objload
import pyoracle
from crt_amd import _lib, assets

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4
INVALID_OFFSET = 5        # Cornell mesh materialIDOffset: local ids 6, 7 -> 11, 12 >= 11 materials (invalid)


def _render(dev, w, h, spp, bounces=20, variant=None, seed=41):
    r = crt_amd.Renderer(w, h)
    if variant is not None:
        r.set_kernel_variant(variant)
    cam = crt_amd.camera(spp)
    r.set_camera(cam)
    r.init_rand(seed)
    r.render(dev, spp, bounces)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    return r


def _exact(lin, rgba, o_sum, o_rgba):
    diff = np.argwhere(lin.view(np.uint32) != o_sum.view(np.uint32))
    assert len(diff) == 0, f"{len(diff)} fp32 words differ, first at {diff[:5].tolist()}"
    assert np.array_equal(rgba, o_rgba)


def _within(lin, ref, spp, min_equal=0.999):
    rms = np.sqrt(np.mean(((lin - ref) / spp).astype(np.float64) ** 2, axis=(0, 1)))
    assert (rms <= RMS_TOL).all(), f"per-channel RMS {rms}"
    eq = float(np.mean(np.all(lin.view(np.uint32) == ref.view(np.uint32), axis=-1)))
    assert eq >= min_equal, f"only {eq:.6f} of pixels bit-identical"
    return rms, eq


def _cam19(spp):
    return crt_amd.camera_floats(crt_amd.camera(spp))


# ------------------------------------------------------------------------------------------------ config B
@pytest.fixture(scope="module")
def config_b(device_scenes):
    hs, ref = device_scenes["cornell_bunny"]
    fast = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0)
    r = _render(ref, 1280, 720, 256, variant=3)
    return hs, ref, fast, r.linear(), r.rgba8(), r.counters()["rays"]


BANDS_B = [(0, 0, 64, 4), (600, 350, 664, 358), (1248, 716, 1280, 720), (720, 480, 784, 496)]   # last: glass bunny


def test_config_b_reference_bvh_bands_bit_exact(config_b, oracle_scenes):
    """1280x720, 256 spp, 20 bounces through the reference's own BVH: bands (one over the glass bunny) vs oracle."""
    _, _, _, lin, rgba, rays = config_b
    cf = _cam19(256)
    for x0, y0, x1, y1 in BANDS_B:
        o_sum, o_rgba, _ = oracle_scenes["cornell_bunny"].render(cf, 1280, 720, 256, 20, rect=(x0, y0, x1, y1))
        _exact(lin[y0:y1, x0:x1], rgba[y0:y1, x0:x1], o_sum, o_rgba)
    assert rays > 1280 * 720 * 256       # every path traces its camera ray, many bounce


def test_config_b_full_frame_low_spp_bit_exact(device_scenes, oracle_scenes):
    """The whole 1280x720 frame at 4 spp, reference BVH, vs the oracle: every pixel and the ray count."""
    _, ref = device_scenes["cornell_bunny"]
    r = _render(ref, 1280, 720, 4, variant=3)
    o_sum, o_rgba, o_cnt = oracle_scenes["cornell_bunny"].render(_cam19(4), 1280, 720, 4, 20)
    _exact(r.linear(), r.rgba8(), o_sum, o_rgba)
    assert r.counters()["rays"] == o_cnt["rays"]


@pytest.mark.parametrize("variant", [8, 7])
def test_config_b_rebuilt_within_bar(config_b, variant):
    """The benchmarked path (rebuilt 4-wide BVH; 8 = probe-ordered tiles, the default at 256 spp) against the
    reference-BVH frame of the same seeds (== the oracle, previous tests)."""
    _, _, fast, lin_ref, _, rays_ref = config_b
    r = _render(fast, 1280, 720, 256, variant=variant)
    # 2 tiles per wave slot: variant 8 at occupancy 4 with the row prefetch, variant 4 at 6
    assert r.last_kernel_name() == f"crt_render_kernel<false, {variant}, {4 if variant == 8 else 6}>"
    _within(r.linear(), lin_ref, 256)
    assert abs(r.counters()["rays"] - rays_ref) <= 1e-5 * rays_ref


# ------------------------------------------------------------------------------------ loader edge scenes
def _scene_pair(name, mutate_offset=None):
    """(HostScene, reference-BVH device scene, rebuilt device scene, OracleScene); mutate_offset = (mesh, offset)
    replaces that mesh's materialIDOffset on both sides (C-ABI scene description / oracle loader output)."""
    files = assets.scene_files(name)
    hs = crt_amd.HostScene(files)
    loaded = objload.load_scene(files)
    if mutate_offset is None:
        return hs, hs.upload(0), hs.upload(0, bvh="rebuilt", width=4), pyoracle.OracleScene(loaded), None
    mesh, off = mutate_offset
    loaded.mesh_info[mesh, 5] = off
    d = hs.desc()
    meshes = (_lib.MeshDesc * d.n_meshes)()
    C.memmove(meshes, d.meshes, C.sizeof(meshes))
    meshes[mesh].material_id_offset = off
    d.meshes = C.cast(meshes, C.c_void_p)
    out = []
    for o in (crt_amd.scene_options("reference"), crt_amd.scene_options("rebuilt", width=4)):
        h = C.c_void_p()
        crt_amd.check(_lib.hip().crt_scene_create_ex(C.byref(d), 0, C.byref(o), C.byref(h)), "crt_scene_create_ex")
        out.append(crt_amd.Scene(h, 0))
    return hs, out[0], out[1], pyoracle.OracleScene(loaded), meshes


EDGE = {
    "fuzzy_metal": ("cornell_metal", None),
    "three_objs": ("cornell_bunny_metal", None),
    "invalid_material": ("cornell_bunny", (0, INVALID_OFFSET)),
}


@pytest.fixture(scope="module")
def edge_scenes():
    return {k: _scene_pair(*v) for k, v in EDGE.items()}


def test_edge_scenes_exercise_the_paths(edge_scenes):
    """The scenes really hold what the tests are about (loader output of both loaders agrees)."""
    hs, _, _, _, _ = edge_scenes["fuzzy_metal"]
    _, _, fm, info, mats = hs.loader_arrays()
    metal = mats[mats[:, 0] == 1]                        # MaterialType::Metal rows: type, albedo3, emission3, r, ior
    assert np.allclose(np.sort(metal[:, 7]), [0.25, 0.3])   # sqrt(2/(30+2)) and Pr 0.3
    assert info[1, 5] == 8                               # 2 files: offset = Cornell's 8 materials -> the metals
    hs3, _, _, _, _ = edge_scenes["three_objs"]
    _, _, fm3, info3, mats3 = hs3.loader_arrays()
    assert info3[:, 5].tolist() == [0, 8, 1]             # third mesh: offset = the bunny's ONE material
    third = fm3[info3[2, 4]:info3[2, 4] + info3[2, 3] // 3] + info3[2, 5]
    assert set(third.tolist()) == {1, 2}                 # the blocks index Cornell's materials 1, 2 (quirk)
    hsi, _, _, _, meshes = edge_scenes["invalid_material"]
    _, _, fmi, infoi, matsi = hsi.loader_arrays()
    ids = fmi[:infoi[0, 3] // 3] + INVALID_OFFSET
    assert (ids >= len(matsi) + 2).any() and (ids < len(matsi) + 2).any()   # + ground and metal spheres
    assert meshes[0].material_id_offset == INVALID_OFFSET


@pytest.mark.parametrize("case", list(EDGE))
@pytest.mark.parametrize("variant", [0, 3, 10])
def test_edge_scene_reference_bvh_bit_exact(edge_scenes, case, variant):
    _, ref, _, osc, _ = edge_scenes[case]
    w, h, spp = 160, 90, 16
    r = _render(ref, w, h, spp, variant=variant)
    o_sum, o_rgba, o_cnt = osc.render(_cam19(spp), w, h, spp, 20)
    _exact(r.linear(), r.rgba8(), o_sum, o_rgba)
    c = crt_amd.Renderer(w, h)
    c.set_kernel_variant(variant)
    c.set_camera(crt_amd.camera(spp))
    c.init_rand(41)
    c.render(ref, spp, 20, count_work=True)
    cnt = c.counters()
    for k in ("rays", "box_tests", "tri_tests", "sphere_tests"):
        assert cnt[k] == o_cnt[k], (k, cnt[k], o_cnt[k])


@pytest.mark.parametrize("case", list(EDGE))
@pytest.mark.parametrize("variant", [7, 8])
def test_edge_scene_rebuilt_within_bar(edge_scenes, case, variant):
    _, ref, fast, _, _ = edge_scenes[case]
    w, h, spp = 320, 180, 64          # 64 spp: variant 8 runs its cost probe
    a = _render(ref, w, h, spp, variant=3)
    b = _render(fast, w, h, spp, variant=variant)
    _within(b.linear(), a.linear(), spp)


def test_fuzzy_metal_changes_the_image(edge_scenes):
    """The metal blocks are visible and fuzzy: the same frame with fuzz 0 (a 2-file scene whose MTL roughness is
    forced to 0 through the scene description) differs."""
    hs, ref, _, _, _ = edge_scenes["fuzzy_metal"]
    w, h, spp = 160, 90, 16
    base = _render(ref, w, h, spp).linear()
    d = hs.desc()
    mats = (_lib.MaterialDesc * d.n_materials)()
    C.memmove(mats, d.materials, C.sizeof(mats))
    for m in mats:
        if m.type == 1:
            m.roughness = 0.0
    d.materials = C.cast(mats, C.c_void_p)
    hnd = C.c_void_p()
    crt_amd.check(_lib.hip().crt_scene_create_ex(C.byref(d), 0, None, C.byref(hnd)), "crt_scene_create_ex")
    sharp = _render(crt_amd.Scene(hnd, 0), w, h, spp).linear()
    assert not np.array_equal(base, sharp)


# ------------------------------------------------------------------------------ device errors surface
def test_stack_overflow_reported_at_synchronize(device_scenes):
    """A 4-wide scene whose stack bound is overridden below what traversal needs: the kernel drops entries and
    flags it; crt_renderer_synchronize returns CRT_ERR_HIP; the flag is cleared once reported."""
    hs, _ = device_scenes["cornell_bunny"]
    bad = hs.upload(0, bvh="rebuilt", width=4, stack_cap=1)
    good = hs.upload(0, bvh="rebuilt", width=4)
    assert bad.stats()["stack_bound"] == 1 and good.stats()["stack_bound"] > 1
    r = crt_amd.Renderer(96, 54)
    r.set_stack_lds(1)                 # every entry past the first would go to the (now absent) HBM region
    r.set_camera(crt_amd.camera(8))
    r.init_rand(41)
    r.render(bad, 8, 20)
    with pytest.raises(crt_amd.CrtError, match="traversal stack"):
        r.synchronize()
    r.synchronize()                    # reported once
    r.init_rand(41)
    r.render(good, 8, 20)
    r.synchronize()                    # a correct frame reports nothing
    r.render(bad, 8, 20)
    with pytest.raises(crt_amd.CrtError, match="traversal stack"):
        r.counters()


def test_stack_overflow_reported_through_hiprenderer(scenes):
    """The same through the reference-shaped C++ path: Raytracer::updateAndRender -> HIPRenderer::render ->
    crt_renderer_render_frame, whose CRT_CHECK throws like the reference's CUDA_CHECK."""
    v = crt_amd.Viewer(scenes["cornell_bunny"], 96, 54, bvh="rebuilt", bvh_width=4, pos=(0.0, 0.0, 0.3), focus=0.3,
                       stack_cap=1)
    v.renderer.set_stack_lds(1)
    with pytest.raises(crt_amd.CrtError, match="traversal stack"):
        v.frame()
    ok = crt_amd.Viewer(scenes["cornell_bunny"], 96, 54, bvh="rebuilt", bvh_width=4, pos=(0.0, 0.0, 0.3), focus=0.3)
    ok.renderer.set_stack_lds(1)
    assert ok.frame()["frame"] == 1


def test_camera_beyond_slab_bound_rejected():
    """crt_renderer_set_camera refuses an origin the 4-wide slab test cannot take (|o| * 2^64 must stay finite,
    crt_hip.hip box_inv) instead of rendering a frame whose box tests produce NaN."""
    r = crt_amd.Renderer(8, 8)
    cam = crt_amd.camera(1)
    r.set_camera(cam)
    for bad in (float("inf"), float("nan"), 2.0 ** 62):
        c = crt_amd.camera(1)
        c.origin[1] = bad
        with pytest.raises(crt_amd.CrtError, match="beyond 2\\^59"):
            r.set_camera(c)
    c = crt_amd.camera(1)
    c.lens_radius = float("inf")
    with pytest.raises(crt_amd.CrtError, match="beyond 2\\^59"):
        r.set_camera(c)
