"""Device primitives and the config-E scene against committed fixtures (no live oracle).

* tests/golden/primitives.json: crt_selftest_geometry runs the records through the device functions the render
  kernels call (tri_test_rec, ref_scene_box with the exact 1/d, sphere_candidate, next_ray's getRay) and must
  return the oracle's f32 words bit for bit.  Kind 4 checks the per-ray spheres' skip test against the oracle's roots.
* tests/golden/cornell_1m_64x36_8spp.npz: the 1M-triangle scene (config E's, instanced bunnies) rendered by the
  oracle.  The reference-BVH path must match it bit for bit including the ray count; the benchmarked rebuilt
  4-wide path within the north-star RMS.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

import crt_amd
from crt_amd import _lib, assets

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
RMS_TOL = 1e-4


def unhex(words, last):
    a = np.array([int(w, 16) for w in words], np.uint32).view(np.float32)
    return a.reshape(-1, last) if last else a


@pytest.fixture(scope="module")
def kat():
    return json.loads((GOLDEN / "primitives.json").read_text())


def _geometry(kind, rec, cam=None, w=0, h=0, rng=None):
    rec = np.ascontiguousarray(rec)
    n = len(rec)
    out = np.zeros((n, 6 if kind == 3 else 1), np.float32)
    camp = C.byref(cam) if cam is not None else None
    crt_amd.check(_lib.hip().crt_selftest_geometry(kind, rec.ctypes.data_as(C.c_void_p), n, camp, w, h,
                                                   rng.ctypes.data_as(C.c_void_p) if rng is not None else None,
                                                   out.ctypes.data_as(C.c_void_p)))
    return out if kind == 3 else out[:, 0]


def test_device_triangle_kat(kat):
    t = _geometry(0, unhex(kat["triangle"]["in_hex"], 17))
    ref = unhex(kat["triangle"]["t_hex"], 0)
    bad = np.nonzero(t.view(np.uint32) != ref.view(np.uint32))[0]
    assert len(bad) == 0, f"{len(bad)} records differ, first {bad[:5].tolist()}: {t[bad[:5]]} vs {ref[bad[:5]]}"


def test_device_box_kat(kat):
    hit = _geometry(1, unhex(kat["box"]["in_hex"], 14))
    assert (hit == 1).astype(int).tolist() == kat["box"]["hit"]


def test_device_sphere_kat(kat):
    t = _geometry(2, unhex(kat["sphere"]["in_hex"], 12))
    assert np.array_equal(t.view(np.uint32), unhex(kat["sphere"]["t_hex"], 0).view(np.uint32))


def test_device_get_ray_kat(kat):
    g = kat["get_ray"]
    c = unhex(g["camera_hex"], 0)
    cam = _lib.CameraDesc()
    for i, f in enumerate(("origin", "lower_left", "horizontal", "vertical", "right", "up")):
        getattr(cam, f)[:] = c[3 * i:3 * i + 3].tolist()
    cam.lens_radius = float(c[18])
    cam.samples_per_pixel = 1
    cam.pixel_sample_scale = 1.0
    rng = np.array(g["rng_in"], np.uint32)
    xy = np.array(g["xy"], np.int32)
    rays = _geometry(3, xy, cam, g["width"], g["height"], rng)
    assert np.array_equal(rays.view(np.uint32).ravel(), unhex(g["ray_hex"], 0).view(np.uint32))
    assert rng.tolist() == g["rng_out"]


@pytest.fixture(scope="module")
def million():
    hs = crt_amd.HostScene(assets.scene_files("cornell_1m"), build_device=0)
    return hs, hs.upload(0), hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0)


def _frame(dev, variant):
    w, h, spp = 64, 36, 8
    r = crt_amd.Renderer(w, h)
    r.set_kernel_variant(variant)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41)
    r.render(dev, spp, 20)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    return r


def test_config_e_slice_reference_bvh_bit_exact(million):
    g = np.load(GOLDEN / "cornell_1m_64x36_8spp.npz")
    r = _frame(million[1], 3)
    assert np.array_equal(r.linear().view(np.uint32), g["sum"].view(np.uint32))
    assert np.array_equal(r.rgba8(), g["rgba"])
    assert r.counters()["rays"] == int(g["rays"][0])


@pytest.mark.parametrize("variant", [4, 7, 8])
def test_config_e_slice_rebuilt_within_rms(million, variant):
    g = np.load(GOLDEN / "cornell_1m_64x36_8spp.npz")
    lin = _frame(million[2], variant).linear()
    rms = np.sqrt(np.mean(((lin - g["sum"]) / 8).astype(np.float64) ** 2, axis=(0, 1)))
    assert (rms <= RMS_TOL).all(), f"per-channel RMS {rms}"
    eq = np.mean(np.all(lin.view(np.uint32) == g["sum"].view(np.uint32), axis=-1))
    assert eq >= 0.999, f"only {eq:.4f} of pixels bit-identical"


def test_device_sphere_skip_never_drops_a_winner(kat):
    """The per-ray spheres run after the trace and skip the exact root when it is provably beyond the trace's
    closest hit (sphere_beyond).  For closest values at and around each record's exact root (nextafter steps, 1e-6
    and 1e-5 relative, far away), a skipped record's accepted root (oracle, tmax = inf) is strictly beyond closest."""
    import pyoracle
    rec = unhex(kat["sphere"]["in_hex"], 12).copy()
    rec[:, 10], rec[:, 11] = np.float32(0.001), np.float32(np.inf)
    t = pyoracle.kat_sphere(rec)
    hit = rec[t >= 0]
    th = t[t >= 0]
    cands = [th]
    for k in range(1, 9):
        up, dn = th.copy(), th.copy()
        for _ in range(k):
            up = np.nextafter(up, np.float32(np.inf))
            dn = np.nextafter(dn, np.float32(0))
        cands += [up, dn]
    for f in (1 - 1e-5, 1 - 1e-6, 1 + 1e-6, 1 + 1e-5, 1 + 2e-5, 1 + 1e-4, 2.0, 0.5):
        cands.append((th * np.float32(f)).astype(np.float32))
    rows, roots = [], []
    for c in cands:
        r = hit.copy()
        r[:, 10] = c
        rows.append(r)
        roots.append(th)
    rows, roots = np.concatenate(rows), np.concatenate(roots)
    skipped = _geometry(4, rows) == 1
    assert skipped.any() and not skipped.all()
    bad = skipped & ~(roots > rows[:, 10])
    assert not bad.any(), f"{bad.sum()} records skipped with root <= closest"
    # closest = inf (no triangle hit) never skips
    r = hit.copy()
    r[:, 10] = np.inf
    assert not (_geometry(4, r) == 1).any()
