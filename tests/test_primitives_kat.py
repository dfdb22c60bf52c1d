"""Known-answer vectors for the path's primitive functions (tests/golden/primitives.json).

The fixture holds f32 inputs and the oracle's outputs for rayTriangleIntersect (Mesh.cuh:266-308),
AABB::hit (AABB.cuh:123-146), Sphere::hit (Sphere.cuh:27-47) and Camera::getRay (Camera.cuh:32-44),
written by tests/golden/make_golden.py.  Here the oracle must reproduce it bit for bit, and the vectors
are checked on their own terms against a float64 restatement wherever the f32 result is far from a
decision boundary (so the fixture is not only the oracle agreeing with itself).  The GPU half
(tests/test_gpu_primitives.py) runs the same records through the device functions the render kernels use.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import pyoracle

GOLDEN = Path(__file__).resolve().parent / "golden"


def unhex(words, shape_last):
    a = np.array([int(w, 16) for w in words], np.uint32).view(np.float32)
    return a.reshape(-1, shape_last) if shape_last else a


@pytest.fixture(scope="module")
def kat():
    return json.loads((GOLDEN / "primitives.json").read_text())


def test_oracle_reproduces_triangle_kat(kat):
    rec = unhex(kat["triangle"]["in_hex"], 17)
    t = pyoracle.kat_triangle(rec)
    assert np.array_equal(t.view(np.uint32), unhex(kat["triangle"]["t_hex"], 0).view(np.uint32))
    assert int((t >= 0).sum()) == kat["triangle"]["hits"]


def test_oracle_reproduces_box_kat(kat):
    rec = unhex(kat["box"]["in_hex"], 14)
    assert pyoracle.kat_box(rec).tolist() == kat["box"]["hit"]


def test_oracle_reproduces_sphere_kat(kat):
    rec = unhex(kat["sphere"]["in_hex"], 12)
    t = pyoracle.kat_sphere(rec)
    assert np.array_equal(t.view(np.uint32), unhex(kat["sphere"]["t_hex"], 0).view(np.uint32))


def test_oracle_reproduces_get_ray_kat(kat):
    g = kat["get_ray"]
    rng = np.array(g["rng_in"], np.uint32)
    rays = pyoracle.kat_get_ray(unhex(g["camera_hex"], 0), g["width"], g["height"], np.array(g["xy"]), rng)
    assert np.array_equal(rays.view(np.uint32).ravel(), unhex(g["ray_hex"], 0).view(np.uint32))
    assert rng.tolist() == g["rng_out"]


def test_triangle_kat_against_float64(kat):
    """Möller–Trumbore in float64: every record whose u, v, u+v, t and det are clear of the f32 rounding
    agrees on hit/miss, and hits agree on t to f32 precision."""
    rec = unhex(kat["triangle"]["in_hex"], 17).astype(np.float64)
    t32 = unhex(kat["triangle"]["t_hex"], 0)
    o, d, v0, v1, v2, tmin, tmax = rec[:, 0:3], rec[:, 3:6], rec[:, 6:9], rec[:, 9:12], rec[:, 12:15], rec[:, 15], rec[:, 16]
    e1, e2 = v1 - v0, v2 - v0
    h = np.cross(d, e2)
    det = (e1 * h).sum(1)
    with np.errstate(divide="ignore", invalid="ignore"):
        f = 1.0 / det
        s = o - v0
        u = f * (s * h).sum(1)
        q = np.cross(s, e1)
        v = f * (d * q).sum(1)
        t = f * (e2 * q).sum(1)
    scale = np.abs(d).max(1) * np.abs(np.stack([e1, e2], 1)).max((1, 2))
    m = 1e-3
    clear = (np.abs(det) > 1e-3 * scale ** 1.0) & (np.abs(u) > m) & (np.abs(u - 1) > m) & (np.abs(v) > m) \
        & (np.abs(u + v - 1) > m) & (np.abs(t - tmin) > m * (1 + np.abs(t))) & (np.abs(t - tmax) > m * (1 + np.abs(t)))
    hit64 = (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= tmin) & (t <= tmax)
    assert clear.sum() > 300
    assert np.array_equal(hit64[clear], t32[clear] >= 0)
    both = clear & hit64
    assert both.sum() > 100
    assert np.allclose(t32[both], t[both], rtol=1e-4, atol=1e-5)


def test_box_kat_against_float64(kat):
    """Slab test in float64 with the reference's NaN handling (fminf/fmaxf drop a NaN operand); records
    whose entry/exit distances are clear of each other and of tmin agree."""
    rec = unhex(kat["box"]["in_hex"], 14).astype(np.float64)
    hit = np.array(kat["box"]["hit"])
    o, d, lo, hi, tmin, tmax = rec[:, 0:3], rec[:, 3:6], rec[:, 6:9], rec[:, 9:12], rec[:, 12], rec[:, 13]
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0, t1 = (lo - o) * inv, (hi - o) * inv
    near = np.nanmax(np.fmin(t0, t1), axis=1)
    far = np.nanmin(np.fmax(t0, t1), axis=1)
    near = np.fmax(near, tmin)
    far = np.fmin(far, tmax)
    flat = (hi == lo).any(1)
    clear = ~flat & ~np.isnan(t0).any(1) & ~np.isnan(t1).any(1) & (np.abs(far - near) > 1e-4 * (1 + np.abs(near)))
    assert clear.sum() > 50       # three in four records have a zero-thickness axis
    assert np.array_equal(hit[clear] == 1, (far > near)[clear])
    # zero-thickness boxes: a ray not lying in the box's plane never enters (AABB.cuh quirk)
    off_plane = flat & ~np.isnan(t0).any(1) & ~np.isnan(t1).any(1)
    assert off_plane.sum() > 30 and not hit[off_plane].any()


def test_sphere_kat_against_float64(kat):
    rec = unhex(kat["sphere"]["in_hex"], 12).astype(np.float64)
    t32 = unhex(kat["sphere"]["t_hex"], 0)
    o, d, c, r, tmin, tmax = rec[:, 0:3], rec[:, 3:6], rec[:, 6:9], rec[:, 9], rec[:, 10], rec[:, 11]
    oc = o - c
    a = (d * d).sum(1)
    hb = (oc * d).sum(1)
    cc = (oc * oc).sum(1) - r * r
    disc = hb * hb - a * cc
    sq = np.sqrt(np.maximum(disc, 0))
    r0, r1 = (-hb - sq) / a, (-hb + sq) / a
    t64 = np.where((r0 >= tmin) & (r0 <= tmax), r0, np.where((r1 >= tmin) & (r1 <= tmax), r1, -1.0))
    t64[disc < 0] = -1.0
    m = 1e-3
    small = r < 10     # the radius-999 ground sphere is f32-cancellation bound; only the oracle pins it
    clear = small & (np.abs(disc) > m * a * r * r) & (np.abs(r0 - tmin) > m) & (np.abs(r1 - tmin) > m) \
        & (np.abs(r0 - tmax) > m) & (np.abs(r1 - tmax) > m)
    assert clear.sum() > 100
    assert np.array_equal(t32[clear] >= 0, t64[clear] >= 0)
    h = clear & (t64 >= 0)
    assert np.allclose(t32[h], t64[h], rtol=1e-4, atol=1e-4)


def test_get_ray_kat_geometry(kat):
    """The ray leaves the lens (within lens radius of the eye) towards a point of the pixel's square on the
    image plane: u in [x/w, (x+1)/w], v in [y/h, (y+1)/h]; each ray consumed generator output."""
    g = kat["get_ray"]
    cam = unhex(g["camera_hex"], 0).astype(np.float64)
    pos, llc, hor, ver, lens = cam[0:3], cam[3:6], cam[6:9], cam[9:12], cam[18]
    rays = unhex(g["ray_hex"], 6).astype(np.float64)
    w, h = g["width"], g["height"]
    for (x, y), ray in zip(g["xy"], rays):
        o, dvec = ray[:3], ray[3:]
        assert np.linalg.norm(o - pos) <= lens * 1.0001 + 1e-6
        p = o + dvec - llc            # = u*hor + v*ver
        uv, *_ = np.linalg.lstsq(np.stack([hor, ver], 1), p, rcond=None)
        assert x / w - 1e-5 <= uv[0] <= (x + 1) / w + 1e-5
        assert y / h - 1e-5 <= uv[1] <= (y + 1) / h + 1e-5
    assert all(a != b for a, b in zip(g["rng_in"], g["rng_out"]))
