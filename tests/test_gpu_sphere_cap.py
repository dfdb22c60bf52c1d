"""The capped unit-sphere loop (crt_renderer_set_sphere_cap): a lane that has drawn `cap` rejected
candidates in a pass keeps its hit parked and continues the same candidate sequence at the wave's next pass.  Every
lane consumes the same draws in the same order, so the frame, the RNG state left for the next frame, the ray and path
counts and the counting kernel's work counters must not depend on the cap at all (Utility.cuh:45-53,
Material.cuh:66-96).  Checked on the Lambertian / glass scene, the fuzzy-metal scene (metal scatter shares the loop)
and a ragged frame, for variant 8 (>= 64 spp: probe + tile order) and variant 4 (no tiles), and the default cap once
more against the oracle through the reference BVH."""
import hashlib

import numpy as np
import pytest

import crt_amd
from crt_amd import assets

pytestmark = pytest.mark.gpu
CAPS = [0, 1, 2, 3, 5]


@pytest.fixture(scope="module")
def rebuilt():
    out = {}
    for k in ("cornell_bunny", "cornell_metal"):
        hs = crt_amd.HostScene(assets.scene_files(k), build_device=0)
        out[k] = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    return out


def _frame(sc, w, h, spp, cap, variant=None, count=False):
    r = crt_amd.Renderer(w, h)
    if variant is not None:
        r.set_kernel_variant(variant)
    r.set_sphere_cap(cap)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41)
    r.render(sc, spp, 20, count_work=count)
    r.synchronize()
    h_ = hashlib.sha256(r.linear().tobytes() + r.rng_state().tobytes()).hexdigest()
    return h_, r.counters(), r.last_kernel_name()


@pytest.mark.parametrize("scene,w,h,spp,variant", [("cornell_bunny", 97, 61, 64, None),
                                                   ("cornell_bunny", 160, 90, 24, 4),
                                                   ("cornell_metal", 160, 90, 64, 8)])
def test_frames_do_not_depend_on_the_cap(rebuilt, scene, w, h, spp, variant):
    sc = rebuilt[scene]
    base, cnt0, kname = _frame(sc, w, h, spp, 0, variant)
    if variant == 8 or variant is None:
        assert ", 8, " in kname
    for cap in CAPS[1:]:
        hsh, cnt, _ = _frame(sc, w, h, spp, cap, variant)
        assert hsh == base, f"cap {cap}: frame or RNG state differs"
        assert cnt["rays"] == cnt0["rays"] and cnt["paths"] == cnt0["paths"], (cap, cnt, cnt0)
    _, w0, _ = _frame(sc, w, h, spp, 0, variant, count=True)
    for cap in (1, 3):
        _, wc, _ = _frame(sc, w, h, spp, cap, variant, count=True)
        assert wc == w0, (cap, wc, w0)


def test_cap_one_defers_most_lanes_and_still_matches(rebuilt):
    """cap 1: every lane whose first candidate is rejected (about half) defers at least once per Lambertian bounce; the
    full-size-like path (variant 8 at 256 spp on a 320x180 frame) stays identical."""
    sc = rebuilt["cornell_bunny"]
    a, ca, _ = _frame(sc, 320, 180, 256, 0)
    b, cb, _ = _frame(sc, 320, 180, 256, 1)
    assert a == b and ca["rays"] == cb["rays"]


def test_cap_argument_checks():
    r = crt_amd.Renderer(16, 8)
    for bad in (-1, 65):
        with pytest.raises(crt_amd.CrtError):
            r.set_sphere_cap(bad)
    r.set_sphere_cap(64)
    r.set_sphere_cap(0)
