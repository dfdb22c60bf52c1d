"""HIP render path vs the CPU oracle on identical seeds (calls go through the C ABI).

Bar: bit-exact (the kernel repeats the reference's single-precision operation
order with no contraction), asserted as exact equality of the fp32 linear sums
and the RGBA8 bytes; the north-star tolerance (1e-4 per-channel RMS of the
linear colour) is asserted as well so a failure reports the distance.
"""
import numpy as np
import pytest

import crt_amd
import pyoracle

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4


VARIANTS = [0, 1, 2, 3, 10]   # 10: variant 3 over one-wave 8x8 tiles (probe order at spp >= 64)


def _render(dev_scene, w, h, spp, bounces, seed=41, subseq=0, cam=None, variant=2):
    r = crt_amd.Renderer(w, h)
    r.set_kernel_variant(variant)
    r.set_camera(cam or crt_amd.camera(spp))
    r.init_rand(seed, subseq)
    r.render(dev_scene, spp, bounces)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    return r


def _assert_parity(lin, rgba, o_sum, o_rgba, spp):
    rms = np.sqrt(np.mean(((lin - o_sum) / spp).astype(np.float64) ** 2, axis=(0, 1)))
    assert (rms <= RMS_TOL).all(), f"per-channel RMS {rms}"
    diff = np.argwhere(lin.view(np.uint32) != o_sum.view(np.uint32))
    assert len(diff) == 0, f"{len(diff)} fp32 words differ, first at {diff[:5].tolist()}"
    assert np.array_equal(rgba, o_rgba)


def test_selftest_math_ieee():
    rng = np.random.default_rng(7)
    a = np.concatenate([rng.normal(size=20000), rng.uniform(-1e-30, 1e-30, 2000), [0.0, -0.0, 1.0, 3.0]]).astype(np.float32)
    b = np.concatenate([rng.normal(size=20000), rng.uniform(1e-3, 1e3, 2000), [1.0, 3.0, 0.0, 7.0]]).astype(np.float32)
    out = np.zeros((len(a), 4), np.float32)
    out64 = np.zeros((len(a), 2), np.float64)
    import ctypes as C
    from crt_amd import _lib
    crt_amd.check(_lib.hip().crt_selftest_math(a.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p), len(a),
                                               out.ctypes.data_as(C.c_void_p), out64.ctypes.data_as(C.c_void_p)))
    with np.errstate(all="ignore"):
        exp = np.stack([a / b, np.sqrt(np.abs(a)), np.float32(1) / a,
                        np.sqrt(np.abs(a).astype(np.float64)).astype(np.float32)], axis=1)
        dx = np.abs(a.astype(np.float64) * b.astype(np.float64))
        exp64 = np.stack([np.sqrt(dx), 1.0 - dx * dx], axis=1)
    assert np.array_equal(out.view(np.uint32), exp.view(np.uint32))
    assert np.array_equal(out64.view(np.uint64), exp64.view(np.uint64))


def test_fast_reciprocal_exhaustive():
    """rcp_newton(x) == IEEE 1.f/x for EVERY float with 1e-8 <= |x| < 2^126 (both signs); the kernel uses
    it only in that range (crt_device.h::recip_exact), so the MT determinant reciprocal stays exact."""
    import ctypes as C
    from crt_amd import _lib
    lo = int(np.float32(1e-8).view(np.uint32))
    hi = int(np.float32(8.507059e37).view(np.uint32))
    bad, first = C.c_ulonglong(0), C.c_uint32(0)
    crt_amd.check(_lib.hip().crt_selftest_rcp(lo, hi, C.byref(bad), C.byref(first)))
    assert bad.value == 0, f"{bad.value} mismatches, first bits {first.value:#010x}"


def test_fast_sqrt_exhaustive():
    """sqrt_rsq(x) == the correctly rounded sqrtf(x) for EVERY float in [2^-100, FLT_MAX]; the kernels use it only
    when every lane of the wave is in that range (crt_device.h::sqrt_exact_wave)."""
    import ctypes as C
    from crt_amd import _lib
    lo = int(np.float32(2.0 ** -100).view(np.uint32))
    hi = 0x7f800000   # exclusive: up to FLT_MAX
    bad, first = C.c_ulonglong(0), C.c_uint32(0)
    crt_amd.check(_lib.hip().crt_selftest_sqrt(lo, hi, C.byref(bad), C.byref(first)))
    assert bad.value == 0, f"{bad.value} mismatches, first bits {first.value:#010x}"


# frame dimensions of the configs (A 256x256, B 1280x720, C/E 2560x1440), the parity crops and the viewer, plus a
# spread of others (odd, prime, 2^k - 1, 4K)
UV_DIMS = [1, 2, 3, 7, 64, 72, 96, 128, 160, 256, 640, 720, 1000, 1023, 1080, 1280, 1440, 1919, 2160, 2560, 3840, 4093]


def test_uv_division_exhaustive():
    """uv_div(a, dim, RN(1/dim)) == IEEE a / dim for every float a in [2^-33, dim], i.e. every (x + U) next_ray can form
    (crt_device.h::uv_div).  crt_renderer_create runs the same check and divides when it fails; at these sizes it
    never does, so the frames of every parity test run the fast path."""
    import ctypes as C
    from crt_amd import _lib
    for dim in UV_DIMS:
        bad = C.c_ulonglong(0)
        crt_amd.check(_lib.hip().crt_selftest_uv_div(dim, C.byref(bad)))
        assert bad.value == 0, f"dim {dim}: {bad.value} mismatches"


def test_wave_scans():
    import ctypes as C
    from crt_amd import _lib
    rng = np.random.default_rng(1)
    n = 64
    x = rng.integers(-1, 50, size=(n, 64)).astype(np.int32)
    x[0] = 0
    x[1] = -1
    out = np.zeros((n, 64, 3), np.int32)
    crt_amd.check(_lib.hip().crt_selftest_scan(x.ctypes.data_as(C.c_void_p), n, out.ctypes.data_as(C.c_void_p)))
    assert np.array_equal(out[..., 0], np.cumsum(x, axis=1))
    assert np.array_equal(out[..., 1], np.cumsum(x, axis=1))
    assert np.array_equal(out[..., 2], np.maximum.accumulate(x, axis=1))


def test_rng_matches_oracle():
    import ctypes as C
    from crt_amd import _lib
    subs = np.array([0, 1, 2, 3, 4, 1000, 3686399, 2 * 3686400 + 17, 7 * 3686400 + 3686399, 2**40 + 5], np.uint64)
    nd = 32
    st = np.zeros((len(subs), 6), np.uint32)
    u = np.zeros((len(subs), nd), np.float32)
    crt_amd.check(_lib.hip().crt_selftest_rng(41, subs.ctypes.data_as(C.c_void_p), len(subs), nd,
                                              st.ctypes.data_as(C.c_void_p), u.ctypes.data_as(C.c_void_p)))
    for i, s in enumerate(subs):
        o = pyoracle.rng_init(41, int(s))
        assert np.array_equal(st[i], o), f"state mismatch at subsequence {s}"
        _, of = pyoracle.rng_draw(o.copy(), nd)
        assert np.array_equal(u[i].view(np.uint32), of.view(np.uint32))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("bounces", [4, 20])
def test_config_a_full_frame(device_scenes, oracle_scenes, bounces, variant):
    """Config A: Cornell (no bunny) 256x256, 16 spp — whole frame bit-exact vs oracle."""
    w = h = 256
    spp = 16
    _, dev = device_scenes["cornell"]
    cam = crt_amd.camera(spp)
    r = _render(dev, w, h, spp, bounces, cam=cam, variant=variant)
    o_sum, o_rgba, o_cnt = oracle_scenes["cornell"].render(crt_amd.camera_floats(cam), w, h, spp, bounces)
    _assert_parity(r.linear(), r.rgba8(), o_sum, o_rgba, spp)
    assert r.counters()["rays"] == o_cnt["rays"] == {4: 3197876, 20: 3420058}[bounces]


@pytest.mark.parametrize("variant", VARIANTS)
def test_cornell_bunny_crop_parity(device_scenes, oracle_scenes, variant):
    """Cornell + bunny proxy (glass), 128x72 frame, 32 spp, 20 bounces."""
    w, h, spp = 128, 72, 32
    _, dev = device_scenes["cornell_bunny"]
    cam = crt_amd.camera(spp)
    r = _render(dev, w, h, spp, 20, cam=cam, variant=variant)
    o_sum, o_rgba, o_cnt = oracle_scenes["cornell_bunny"].render(crt_amd.camera_floats(cam), w, h, spp, 20)
    _assert_parity(r.linear(), r.rgba8(), o_sum, o_rgba, spp)
    r2 = crt_amd.Renderer(w, h)
    r2.set_kernel_variant(variant)
    r2.set_camera(cam)
    r2.init_rand(41)
    r2.render(dev, spp, 20, count_work=True)
    c = r2.counters()
    for k in ("rays", "box_tests", "tri_tests", "sphere_tests"):
        assert c[k] == o_cnt[k], (k, c[k], o_cnt[k])
    assert c["paths"] == w * h * spp


def test_chunked_accumulate_equals_single(device_scenes):
    """spp split over launches (RNG + sum carried in HBM) is bit-identical to one launch."""
    w, h = 96, 54
    _, dev = device_scenes["cornell_bunny"]
    cam = crt_amd.camera(12)
    a = _render(dev, w, h, 12, 20, cam=cam)
    b = crt_amd.Renderer(w, h)
    b.set_camera(cam)
    b.init_rand(41)
    b.render(dev, 5, 20)
    b.render(dev, 7, 20, accumulate=True)
    b.synchronize()
    assert np.array_equal(a.linear().view(np.uint32), b.linear().view(np.uint32))
    assert np.array_equal(a.rng_state(), b.rng_state())


@pytest.mark.parametrize("variant", VARIANTS)
def test_full_size_frame_sampled_pixels(device_scenes, oracle_scenes, variant):
    """Headline geometry (2560x1440) at reduced spp; a band of pixels checked against the oracle,
    plus size-independent properties (determinism, ray count = counting-kernel count)."""
    w, h, spp = 2560, 1440, 4
    _, dev = device_scenes["cornell_bunny"]
    cam = crt_amd.camera(spp)
    r = _render(dev, w, h, spp, 20, cam=cam, variant=variant)
    lin = r.linear()
    rays = r.counters()["rays"]
    r.init_rand(41)
    r.render(dev, spp, 20)
    r.synchronize()
    assert np.array_equal(lin.view(np.uint32), r.linear().view(np.uint32)), "not deterministic"
    assert r.counters()["rays"] == rays
    cf = crt_amd.camera_floats(cam)
    rgba = r.rgba8()
    for (x0, y0, x1, y1) in [(0, 0, 64, 4), (1200, 700, 1296, 708), (2496, 1436, 2560, 1440), (1700, 900, 1760, 960)]:
        o_sum, o_rgba, _ = oracle_scenes["cornell_bunny"].render(cf, w, h, spp, 20, rect=(x0, y0, x1, y1))
        _assert_parity(lin[y0:y1, x0:x1], rgba[y0:y1, x0:x1], o_sum, o_rgba, spp)


def test_sharded_n1_is_reference_frame_and_shards_sum(device_scenes):
    """ShardedFrameRenderer with world=1 (torch framebuffer, torch stream) == plain render, bit-exact;
    two shards rendered on one GPU and summed == the 2-GPU frame's framebuffer definition."""
    import torch
    from crt_amd.dist import ShardedFrameRenderer
    w, h, spp = 128, 72, 6
    _, dev = device_scenes["cornell_bunny"]
    cam = crt_amd.camera(spp)
    ref = _render(dev, w, h, spp, 20, cam=cam)
    r = crt_amd.Renderer(w, h)
    r.set_camera(cam)
    fr = ShardedFrameRenderer(r, dev, spp, 20, 41, 0, 1)
    fr.render()
    torch.cuda.synchronize()
    assert np.array_equal(fr.linear().view(np.uint32), ref.linear().view(np.uint32))
    assert np.array_equal(r.rgba8(), ref.rgba8())
    # shard g of N renders spp_g samples from subsequences pixel + g*W*H: check against the oracle
    import pyoracle, objload
    from crt_amd import assets
    from crt_amd.dist import shard_plan
    o = pyoracle.OracleScene(objload.load_scene(assets.scene_files("cornell_bunny")))
    for p in shard_plan(spp, 2, w, h):
        rr = crt_amd.Renderer(w, h)
        rr.set_camera(cam)
        rr.init_rand(41, p["subsequence_base"])
        rr.render(dev, p["spp"], 20)
        rr.synchronize()
        o_sum = o.render(crt_amd.camera_floats(cam), w, h, p["spp"], 20, subseq_base=p["subsequence_base"],
                         rect=(0, 0, w, 8))[0]
        assert np.array_equal(rr.linear()[:8].view(np.uint32), o_sum.view(np.uint32))


def test_golden_fixture_frame(device_scenes):
    """HIP output == the committed oracle fixture (tests/golden, make_golden.py), no live oracle."""
    from pathlib import Path
    g = np.load(Path(__file__).resolve().parent / "golden" / "cornell_bunny_64x36_16spp.npz")
    _, dev = device_scenes["cornell_bunny"]
    r = _render(dev, 64, 36, 16, 20, cam=crt_amd.camera(16))
    _assert_parity(r.linear(), r.rgba8(), g["sum"], g["rgba"], 16)


def test_init_rand_cache_returns_the_same_state(device_scenes):
    """crt_renderer_init_rand keeps the last curand_init array and copies it back for a repeated (seed, base):
    the state after any sequence of inits and renders equals a fresh renderer's."""
    w, h = 48, 32
    _, dev = device_scenes["cornell"]
    r = crt_amd.Renderer(w, h)
    r.set_camera(crt_amd.camera(2))
    fresh = {}
    for base in (0, 3 * w * h):
        f = crt_amd.Renderer(w, h)
        f.init_rand(41, base)
        fresh[base] = f.rng_state().copy()
    for base in (0, 0, 3 * w * h, 0, 3 * w * h, 3 * w * h):
        r.init_rand(41, base)
        assert np.array_equal(r.rng_state(), fresh[base]), base
        r.render(dev, 2, 4)          # consumes the stream; the next init must not see it
        r.synchronize()
    r.init_rand(42, 0)
    assert not np.array_equal(r.rng_state(), fresh[0])
