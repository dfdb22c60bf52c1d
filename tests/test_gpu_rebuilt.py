"""CRT_BVH_REBUILT on the GPU vs the reference semantics (oracle / reference-BVH device scene).

The rebuilt BVH keeps the reference's hit rule (closest t, ties to the higher reference DFS rank, primitives
in zero-thickness reference boxes excluded), so almost every ray returns the reference's hit bit for bit.
It can differ only where the reference's unpadded boxes round away a genuine hit; such a ray changes the
rest of its pixel's path.  Bar (north star): per-channel RMS of the resolved linear colour <= 1e-4 against
the oracle, with the per-ray agreement measured by crt_scene_compare (both structures trace the same rays)
and the fraction of bit-identical pixels bounded from below.
"""
import numpy as np
import pytest

import crt_amd

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4

CONFIGS = {"w4": dict(width=4), "w4l8": dict(width=4, leaf_size=8, traversal_cost=2),
           "w2l16": dict(width=2, leaf_size=16, traversal_cost=6),
           "w4sbvh": dict(width=4, spatial_splits=True)}   # spatial splits: triangles referenced from several leaves


@pytest.fixture(scope="module")
def rebuilt(device_scenes):
    out = {}
    for scene in ("cornell", "cornell_bunny"):
        hs, _ = device_scenes[scene]
        for k, opts in CONFIGS.items():
            out[scene, k] = hs.upload(0, bvh="rebuilt", **opts)
    return out


def _frame(dev, w, h, spp, bounces, cam, variant=3, seed=41, stack_lds=16):
    r = crt_amd.Renderer(w, h)
    r.set_kernel_variant(variant)
    r.set_stack_lds(stack_lds)
    r.set_camera(cam)
    r.init_rand(seed)
    r.render(dev, spp, bounces)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    return r


def _compare(lin, o_sum, spp, min_equal):
    rms = np.sqrt(np.mean(((lin - o_sum) / spp).astype(np.float64) ** 2, axis=(0, 1)))
    assert (rms <= RMS_TOL).all(), f"per-channel RMS {rms}"
    eq = np.mean(np.all(lin.view(np.uint32) == o_sum.view(np.uint32), axis=-1))
    assert eq >= min_equal, f"only {eq:.6f} of pixels bit-identical"
    return rms, eq


def test_rebuilt_stats(rebuilt, device_scenes):
    ref = device_scenes["cornell_bunny"][1].stats()
    for k, opts in CONFIGS.items():
        st = rebuilt["cornell_bunny", k].stats()
        assert st["bvh"] == 1 and st["width"] == opts["width"]
        if opts.get("spatial_splits"):   # straddling triangles are referenced from both sides of a spatial split
            plain = rebuilt["cornell_bunny", "w4"].stats()
            assert st["spatial_splits"] > 0 and st["device_prims"] > plain["device_prims"]
            assert st["references"] == st["device_prims"] - 2          # the two per-ray spheres are not in leaves
            continue
        assert st["spatial_splits"] == 0
        assert st["device_prims"] + st["excluded_prims"] == ref["device_prims"]
        if opts["width"] == 4:
            assert st["stack_bound"] > 1


@pytest.mark.parametrize("cfg", list(CONFIGS))
@pytest.mark.parametrize("bounces", [4, 20])
def test_config_a_rebuilt(rebuilt, oracle_scenes, cfg, bounces):
    """Config A (Cornell, 256x256, 16 spp) rendered through the rebuilt BVH vs the oracle."""
    w = h = 256
    spp = 16
    cam = crt_amd.camera(spp)
    r = _frame(rebuilt["cornell", cfg], w, h, spp, bounces, cam)
    o_sum, o_rgba, o_cnt = oracle_scenes["cornell"].render(crt_amd.camera_floats(cam), w, h, spp, bounces)
    _compare(r.linear(), o_sum, spp, 0.999)
    assert abs(r.counters()["rays"] - o_cnt["rays"]) <= 1e-4 * o_cnt["rays"]


@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_cornell_bunny_rebuilt(rebuilt, oracle_scenes, cfg):
    w, h, spp = 128, 72, 32
    cam = crt_amd.camera(spp)
    r = _frame(rebuilt["cornell_bunny", cfg], w, h, spp, 20, cam)
    o_sum, _, _ = oracle_scenes["cornell_bunny"].render(crt_amd.camera_floats(cam), w, h, spp, 20)
    _compare(r.linear(), o_sum, spp, 0.999)
    c = r.counters()
    assert c["rays"] > 0


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_threaded_rebuilt_all_variants_identical(rebuilt, variant):
    """Width-2 rebuilt layouts run on every threaded variant; all give the same frame bit for bit."""
    w, h, spp = 96, 54, 8
    cam = crt_amd.camera(spp)
    base = _frame(rebuilt["cornell_bunny", "w2l16"], w, h, spp, 20, cam, variant=3).linear()
    got = _frame(rebuilt["cornell_bunny", "w2l16"], w, h, spp, 20, cam, variant=variant).linear()
    assert np.array_equal(base.view(np.uint32), got.view(np.uint32))


def test_wide_stack_in_hbm_identical(rebuilt):
    """Variant 4 with 1 LDS stack entry (everything deeper in the HBM overflow region) == 16 entries."""
    w, h, spp = 160, 90, 8
    cam = crt_amd.camera(spp)
    a = _frame(rebuilt["cornell_bunny", "w4"], w, h, spp, 20, cam, stack_lds=16)
    b = _frame(rebuilt["cornell_bunny", "w4"], w, h, spp, 20, cam, stack_lds=1)
    assert np.array_equal(a.linear().view(np.uint32), b.linear().view(np.uint32))
    assert a.counters()["rays"] == b.counters()["rays"]


@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_per_ray_agreement(rebuilt, device_scenes, cfg):
    """Every ray traced through both structures: hit primitive and t agree except at rounding events."""
    r = crt_amd.Renderer(640, 360)
    r.set_camera(crt_amd.camera(4))
    r.init_rand(41)
    c = r.compare(device_scenes["cornell_bunny"][1], rebuilt["cornell_bunny", cfg], 4, 20)
    assert c["rays"] > 2_000_000
    assert c["t_mismatch"] == 0
    assert c["rank_mismatch"] <= 1e-6 * c["rays"], c


def test_full_size_rebuilt_sampled_pixels(rebuilt, oracle_scenes):
    """Headline geometry (2560x1440) through the 4-wide kernel at 4 spp: bands vs the oracle, determinism."""
    w, h, spp = 2560, 1440, 4
    cam = crt_amd.camera(spp)
    dev = rebuilt["cornell_bunny", "w4"]
    r = _frame(dev, w, h, spp, 20, cam)
    lin = r.linear()
    r.init_rand(41)
    r.render(dev, spp, 20)
    r.synchronize()
    assert np.array_equal(lin.view(np.uint32), r.linear().view(np.uint32)), "not deterministic"
    cf = crt_amd.camera_floats(cam)
    for (x0, y0, x1, y1) in [(0, 0, 64, 4), (1200, 700, 1296, 708), (1700, 900, 1760, 960)]:
        o_sum, _, _ = oracle_scenes["cornell_bunny"].render(cf, w, h, spp, 20, rect=(x0, y0, x1, y1))
        _compare(lin[y0:y1, x0:x1], o_sum, spp, 0.99)


def test_golden_fixture_rebuilt(rebuilt):
    from pathlib import Path
    g = np.load(Path(__file__).resolve().parent / "golden" / "cornell_bunny_64x36_16spp.npz")
    r = _frame(rebuilt["cornell_bunny", "w4"], 64, 36, 16, 20, crt_amd.camera(16))
    _compare(r.linear(), g["sum"], 16, 0.99)


@pytest.mark.parametrize("variant", [7, 8])
@pytest.mark.parametrize("w,h,spp", [(160, 90, 8), (100, 37, 70), (64, 36, 0), (1, 1, 64), (9, 1, 65), (1, 17, 3)])
def test_persistent_queue_variant_is_bit_identical(rebuilt, w, h, spp, variant):
    """Variants 7 (lanes take pixels from a global queue in probe-cost order) and 8 (one wave per workgroup, 8x8
    tiles in probe-cost order) trace every pixel with ONE lane, samples in order, from its own RNG stream: the
    frame, the RNG state and the ray count equal variant 4's.  spp 70 >= 64 runs the cost probe and the sorted
    order; 8 uses row-major order; 0 traces nothing.  100x37 has partial 8x8 tiles; 1x1, 9x1 and 1x17 are
    degenerate frames (one partial tile, a partial tile row / column)."""
    dev = rebuilt["cornell_bunny", "w4"]
    cam = crt_amd.camera(max(spp, 1))
    a = _frame(dev, w, h, spp, 20, cam, variant=4)
    b = _frame(dev, w, h, spp, 20, cam, variant=variant)
    assert np.array_equal(a.linear().view(np.uint32), b.linear().view(np.uint32))
    assert np.array_equal(a.rgba8(), b.rgba8())
    assert np.array_equal(a.rng_state(), b.rng_state())
    assert a.counters()["rays"] == b.counters()["rays"]
    # accumulate continues every pixel's sum and stream
    for r in (a, b):
        r.render(dev, 3, 20, accumulate=True)
        r.synchronize()
    assert np.array_equal(a.linear().view(np.uint32), b.linear().view(np.uint32))
    assert np.array_equal(a.rng_state(), b.rng_state())


@pytest.mark.parametrize("variant", [7, 8])
def test_persistent_queue_counting_kernel(rebuilt, variant):
    dev = rebuilt["cornell_bunny", "w4"]
    cam = crt_amd.camera(4)
    a = crt_amd.Renderer(96, 54)
    b = crt_amd.Renderer(96, 54)
    b.set_kernel_variant(variant)
    for r in (a, b):
        r.set_camera(cam)
        r.init_rand(41)
        r.render(dev, 4, 20, count_work=True)
        r.synchronize()
    ca, cb = a.counters(), b.counters()
    for k in ("rays", "box_tests", "tri_tests", "sphere_tests", "paths"):
        assert ca[k] == cb[k], k
    assert np.array_equal(a.linear().view(np.uint32), b.linear().view(np.uint32))
    assert b.last_kernel_name() == f"crt_render_kernel<true, {variant}, 6>"


@pytest.mark.parametrize("probe_spp", [0, 4])
def test_probe_order_is_bit_identical(rebuilt, probe_spp):
    """Variant 8 with and without the cost probe (row order / most expensive tiles first)."""
    _schedule_case(rebuilt, 8, probe_spp)


@pytest.mark.parametrize("key", [1, 2])
def test_tile_key_modes_are_bit_identical(rebuilt, key):
    _schedule_case(rebuilt, 8, 4, tile_key=key)


@pytest.mark.parametrize("tiles,lanes", [(0, 16), (10, 1), (-1, 64), (1000000, 5)])
def test_critical_tiles_are_bit_identical(rebuilt, tiles, lanes):
    """Variant 8's critical tiles (the leading tiles of the cost order regenerate at fewer parked lanes): none, the
    first 10 at every parked lane, the automatic count, every tile."""
    _schedule_case(rebuilt, 8, 4, crit=(tiles, lanes))


def test_critical_tiles_rejects_bad_arguments():
    r = crt_amd.Renderer(16, 16)
    for tiles, lanes in ((-2, 16), (0, 0), (0, 65)):
        with pytest.raises(crt_amd.CrtError):
            r.set_critical_tiles(tiles, lanes)


def _schedule_case(rebuilt, variant, probe_spp, crit=None, **flags):
    """A schedule option, with and without the cost probe: the same frame and RNG state as variant 4."""
    dev = rebuilt["cornell_bunny", "w4"]
    w, h, spp = 104, 45, 64          # 13 x 6 = 78 tiles, the last row partial
    cam = crt_amd.camera(spp)
    a = _frame(dev, w, h, spp, 20, cam, variant=4)
    b = crt_amd.Renderer(w, h)
    b.set_kernel_variant(variant)
    b.set_schedule(probe_spp, 64, **flags)
    if crit is not None:
        b.set_critical_tiles(*crit)
    b.set_camera(cam)
    b.init_rand(41)
    b.render(dev, spp, 20)
    b.synchronize()
    assert np.array_equal(a.linear().view(np.uint32), b.linear().view(np.uint32))
    assert np.array_equal(a.rng_state(), b.rng_state())


@pytest.mark.parametrize("variant,spp,count", [(8, 64, False), (4, 8, False), (7, 8, False), (8, 4, True), (7, 4, True)])
def test_top_levels_are_bit_identical(rebuilt, variant, spp, count):
    """A new ray's first node step from the LDS copy of the root (crt_renderer_set_top_levels, the default) against
    the regular traversal step over the same node: the same frame, RNG state and work counters (box tests included)."""
    dev = rebuilt["cornell_bunny", "w4"]
    w, h = 104, 45
    out = []
    for levels in (0, -1):
        r = crt_amd.Renderer(w, h)
        r.set_kernel_variant(variant)
        r.set_top_levels(levels)
        r.set_camera(crt_amd.camera(spp))
        r.init_rand(41)
        r.render(dev, spp, 20, count_work=count)
        r.synchronize()
        out.append((r.linear().view(np.uint32), r.rng_state(), r.counters()))
    (a_lin, a_rng, a_c), (b_lin, b_rng, b_c) = out
    assert np.array_equal(a_lin, b_lin) and np.array_equal(a_rng, b_rng)
    keys = ("rays", "box_tests", "tri_tests", "sphere_tests", "paths") if count else ("rays",)
    for k in keys:
        assert a_c[k] == b_c[k], k


def test_top_levels_rejects_bad_arguments():
    r = crt_amd.Renderer(16, 16)
    for levels in (-2, 9):
        with pytest.raises(crt_amd.CrtError):
            r.set_top_levels(levels)


def test_occupancy_seven_is_bit_identical_and_automatic(rebuilt):
    """Variant 8 at 7 waves/SIMD (8 LDS stack entries, deeper entries in HBM) and at 4 (16 entries, the next node's rows
    loaded during the leaf round) render the occupancy-6 frame bit for bit; the automatic choice takes 7 for a
    headline-sized frame (>= 4 tiles per wave slot) and 4 for a small one."""
    dev = rebuilt["cornell_bunny", "w4"]
    w, h, spp = 2560, 1440, 64
    out = []
    for occ in (6, 0, 4):
        r = crt_amd.Renderer(w, h)
        if occ:
            r.set_occupancy_target(occ)
        r.set_camera(crt_amd.camera(spp))
        r.init_rand(41)
        r.render(dev, spp, 20)
        r.synchronize()
        out.append((r.last_kernel_name(), r.linear().view(np.uint32), r.rng_state(), r.counters()["rays"]))
    (k6, lin6, rng6, rays6), (k7, lin7, rng7, rays7), (k4, lin4, rng4, rays4) = out
    assert k6 == "crt_render_kernel<false, 8, 6>" and k7 == "crt_render_kernel<false, 8, 7>"
    assert k4 == "crt_render_kernel<false, 8, 4>"
    assert np.array_equal(lin6, lin7) and np.array_equal(rng6, rng7) and rays6 == rays7
    assert np.array_equal(lin6, lin4) and np.array_equal(rng6, rng4) and rays6 == rays4
    small = _frame(dev, 104, 45, 64, 20, crt_amd.camera(64), variant=-1)
    assert small.last_kernel_name() == "crt_render_kernel<false, 8, 4>"


def test_occupancy_choice_follows_the_probe(rebuilt):
    """Below 4 tiles per wave slot the cost probe decides between occupancy 4 (row prefetch) and 6: config B's frame
    (the glass bunny's tiles outlast an even spread of the frame over the wave slots: rho = largest tile work / mean work
    per slot ~ 2) runs at 4, the plain Cornell box at the same size (rho ~ 0.8) at 6; last_schedule reports the choice."""
    got = {}
    for scene in ("cornell_bunny", "cornell"):
        r = crt_amd.Renderer(1280, 720)
        r.set_camera(crt_amd.camera(64))
        r.init_rand(41)
        r.render(rebuilt[scene, "w4"], 64, 20)
        r.synchronize()
        got[scene] = (r.last_kernel_name(), r.last_schedule())
    (kb, sb), (kc, sc) = got["cornell_bunny"], got["cornell"]
    assert kb == "crt_render_kernel<false, 8, 4>" and sb["occupancy"] == 4 and sb["rho"] > 1.6, sb
    assert kc == "crt_render_kernel<false, 8, 6>" and sc["occupancy"] == 6 and 0 < sc["rho"] < 1.6, sc
    assert sb["max_tile_work"] > sb["mean_tile_work"] > 0


@pytest.mark.parametrize("scene,w,h,spp,stack", [("cornell_bunny", 100, 37, 70, 0), ("cornell_bunny", 1280, 720, 64, 0),
                                                 ("cornell_1m", 320, 180, 64, 0), ("cornell_bunny", 160, 90, 64, 1)])
def test_row_prefetch_is_bit_identical(rebuilt, request, scene, w, h, spp, stack):
    """Variant 8 at occupancy 4 loads each lane's next node rows during the step's first leaf round and uses them in the
    next node step (lanes given a new ray in between load their own): frames, RNG state and ray counts equal occupancy
    6's, on a ragged frame, a config-B-sized frame, the deep 1M-triangle tree and with one LDS stack entry (every
    deeper entry pushed to and popped from the HBM overflow region)."""
    dev = request.getfixturevalue("config_e")[0] if scene == "cornell_1m" else rebuilt[scene, "w4"]
    out = []
    for occ in (6, 4):
        r = crt_amd.Renderer(w, h)
        r.set_occupancy_target(occ)
        if stack:
            r.set_stack_lds(stack)
        r.set_camera(crt_amd.camera(spp))
        r.init_rand(41)
        r.render(dev, spp, 20)
        r.synchronize()
        out.append((r.last_kernel_name(), r.linear().view(np.uint32), r.rng_state(), r.counters()["rays"]))
    assert out[0][0].endswith("8, 6>") and out[1][0].endswith("8, 4>")
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2]) and out[0][3] == out[1][3]


def _usable_cores() -> int:
    """The affinity set capped by the cgroup CPU quota (the GPU box: 256 CPUs, a 16-CPU quota)."""
    import os
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def test_shipped_instantiation_against_the_oracle(rebuilt, oracle_scenes):
    """The benchmarked kernel itself against the oracle, with no GPU-vs-GPU link in between: a headline-sized frame
    (2560x1440, so >= 4 tiles per wave slot) at 64 spp through the automatic choice, which runs the cost probe, the tile
    sort and the critical tiles and launches crt_render_kernel<false, 8, 7>.  Four full-width bands, one through the
    glass bunny, are rendered by the oracle (CUDAKernels.h:147-166 restated) from the same RNG streams; each band holds
    the north-star bar (per-channel RMS <= 1e-4) with >= 99.9 % of its pixels bit-identical."""
    dev = rebuilt["cornell_bunny", "w4"]
    w, h, spp = 2560, 1440, 64
    cam = crt_amd.camera(spp)
    r = crt_amd.Renderer(w, h)
    r.set_camera(cam)
    r.init_rand(41)
    r.render(dev, spp, 20)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    assert r.last_kernel_name() == "crt_render_kernel<false, 8, 7>"
    ph = r.last_timings()
    assert ph["probe_sort_ms"] > 0 and ph["main_kernel_ms"] > 0          # the probe and the sort ran before the kernel
    lin, rgba = r.linear(), r.rgba8()
    cf = crt_amd.camera_floats(cam)
    nt = _usable_cores()
    osc = oracle_scenes["cornell_bunny"]
    per_sample = {}
    for y0 in (96, 700, 950, 1360):
        o_sum, o_rgba, o_cnt = osc.render(cf, w, h, spp, 20, rect=(0, y0, w, y0 + 4), nthreads=nt)
        _compare(lin[y0:y0 + 4], o_sum, spp, 0.999)
        assert np.mean(np.all(rgba[y0:y0 + 4] == o_rgba, axis=-1)) >= 0.999
        per_sample[y0] = o_cnt["rays"] / (w * 4 * spp)
    # the y0 = 950 band crosses the glass bunny (x ~1360-1600): its paths there are the frame's longest
    _, _, c = osc.render(cf, w, h, spp, 20, rect=(1360, 950, 1600, 954), nthreads=nt)
    assert c["rays"] / (240 * 4 * spp) > 1.15 * per_sample[950], (c["rays"], per_sample)


def _shipped_frame(dev, w, h, spp, kernel):
    """A frame through the automatic choice (probe, tile sort, critical tiles), asserting the instantiation it ran."""
    cam = crt_amd.camera(spp)
    r = crt_amd.Renderer(w, h)
    r.set_camera(cam)
    r.init_rand(41)
    r.render(dev, spp, 20)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    assert r.last_kernel_name() == kernel
    ph = r.last_timings()
    assert ph["probe_sort_ms"] > 0 and ph["main_kernel_ms"] > 0          # the probe and the sort ran before the kernel
    return r, crt_amd.camera_floats(cam)


@pytest.fixture(scope="module")
def config_e():
    """Config E (BASELINE.json configs[4]): Cornell + one OBJ of ten translated ~100k-triangle glass bunny proxies;
    the device scene as bench.py builds it (GPU mesh BVH, GPU binned-SAH 4-wide tree) and the oracle's own load."""
    import objload
    import pyoracle
    from crt_amd import assets
    files = assets.scene_files("cornell_1m")
    hs = crt_amd.HostScene(files, build_device=0)
    dev = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    return dev, pyoracle.OracleScene(objload.load_scene(files))


# Config E's ten bunnies project onto rows ~80-320 (row 0 = bottom) and columns ~800-1760 of the 2560x1440 frame (their
# vertices through the bench camera); the y0 = 200 band crosses all of them.
BANDS_E = (200, 264, 700, 1300)


def test_config_e_shipped_instantiation_against_the_oracle(config_e):
    """Config E's benchmarked kernel against the oracle directly (the deep-BVH config, Mesh.cuh:55-110): the 1M-triangle
    scene at 2560x1440 and 64 spp through the automatic choice, which runs the cost probe and the tile sort and launches
    crt_render_kernel<false, 8, 7>.  Four full-width 4-row bands, two through the instanced glass bunnies, rendered by
    the oracle (CUDAKernels.h:147-166 restated, the reference's own median-split BVH) from the same RNG streams; each
    band holds the north-star bar (per-channel RMS <= 1e-4) with >= 99.9 % of its pixels bit-identical."""
    dev, osc = config_e
    w, h, spp = 2560, 1440, 64
    r, cf = _shipped_frame(dev, w, h, spp, "crt_render_kernel<false, 8, 7>")
    lin, rgba = r.linear(), r.rgba8()
    nt = _usable_cores()
    for y0 in BANDS_E:
        o_sum, o_rgba, o_cnt = osc.render(cf, w, h, spp, 20, rect=(0, y0, w, y0 + 4), nthreads=nt)
        _compare(lin[y0:y0 + 4], o_sum, spp, 0.999)
        assert np.mean(np.all(rgba[y0:y0 + 4] == o_rgba, axis=-1)) >= 0.999
    # the bunny band really crosses the mesh: its rays descend the reference's mesh BVH much deeper than a wall band's
    # (oracle counters here: 23.7 against 17.3 box tests per ray at 4 spp)
    _, _, c_b = osc.render(cf, w, h, 4, 20, rect=(800, 200, 1760, 204), nthreads=nt)
    _, _, c_w = osc.render(cf, w, h, 4, 20, rect=(0, 1300, 400, 1304), nthreads=nt)
    assert c_b["box_tests"] / c_b["rays"] > 1.2 * c_w["box_tests"] / c_w["rays"], (c_b, c_w)


BANDS_B_FULL = (4, 352, 488, 716)      # full-width 4-row bands of config B; y0 = 488 crosses the glass bunny


def test_config_b_shipped_instantiation_against_the_oracle(rebuilt, oracle_scenes):
    """Config B's benchmarked kernel (1280x720, 256 spp: 2 tiles per wave slot, so crt_render_kernel<false, 8, 4>) against
    the oracle directly, not against the reference-BVH GPU frame: four full-width bands at the full 256 spp, one through
    the glass bunny, each within the north-star bar with >= 99.9 % of its pixels bit-identical."""
    dev = rebuilt["cornell_bunny", "w4"]
    w, h, spp = 1280, 720, 256
    r, cf = _shipped_frame(dev, w, h, spp, "crt_render_kernel<false, 8, 4>")
    lin, rgba = r.linear(), r.rgba8()
    nt = _usable_cores()
    osc = oracle_scenes["cornell_bunny"]
    for y0 in BANDS_B_FULL:
        o_sum, o_rgba, _ = osc.render(cf, w, h, spp, 20, rect=(0, y0, w, y0 + 4), nthreads=nt)
        _compare(lin[y0:y0 + 4], o_sum, spp, 0.999)
        assert np.mean(np.all(rgba[y0:y0 + 4] == o_rgba, axis=-1)) >= 0.999


@pytest.mark.parametrize("w,h,spp", [(640, 360, 64), (100, 37, 70), (2560, 1440, 64)])
def test_xcd_regions_are_bit_identical(rebuilt, w, h, spp):
    """Variant 8 with the XCD-region tile order (crt_renderer_set_xcd_regions: blocks b and b + 8 render one screen
    strip) renders the global-order frame bit for bit: sums, RNG state and ray count; ragged sizes included."""
    dev = rebuilt["cornell_bunny", "w4"]
    out = []
    for on in (0, 1):
        r = crt_amd.Renderer(w, h)
        r.set_xcd_regions(on)
        r.set_camera(crt_amd.camera(spp))
        r.init_rand(41)
        r.render(dev, spp, 20)
        r.synchronize()
        assert r.last_kernel_name().startswith("crt_render_kernel<false, 8,")
        out.append((r.linear().view(np.uint32), r.rng_state(), r.counters()["rays"]))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1]) and out[0][2] == out[1][2]


@pytest.mark.parametrize("stride", [2, 4])
def test_probe_stride_is_bit_identical(rebuilt, stride):
    """Variant 8 with a subsampled cost probe (every 2nd / 4th pixel in x and y): only the tile order changes, so the
    frame, RNG state and ray count equal the full probe's; a ragged size checks the edge tiles."""
    dev = rebuilt["cornell_bunny", "w4"]
    for w, h, spp in ((2560, 1440, 64), (100, 37, 70)):
        out = []
        for s in (1, stride):
            r = crt_amd.Renderer(w, h)
            r.set_schedule(-1, 64, probe_stride=s)
            r.set_camera(crt_amd.camera(spp))
            r.init_rand(41)
            r.render(dev, spp, 20)
            r.synchronize()
            assert r.last_timings()["probe_sort_ms"] > 0
            out.append((r.linear().view(np.uint32), r.rng_state(), r.counters()["rays"]))
        assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1]) and out[0][2] == out[1][2]


def test_wave_drain_is_bit_identical(rebuilt):
    """Variants 8 and 4 with draining waves passing at 16/64 and 48/64 (the default) of their live lanes instead of all
    of them (crt_renderer_set_wave_drain): only when lanes run their shading passes changes, so frames, RNG state and ray
    counts equal those of 64/64, at a ragged size too."""
    dev = rebuilt["cornell_bunny", "w4"]
    for w, h, spp, variant in ((640, 360, 64, 8), (100, 37, 70, 8), (160, 90, 8, 4)):
        out = []
        for wd in (64, 48, 16):
            r = crt_amd.Renderer(w, h)
            r.set_kernel_variant(variant)
            r.set_wave_drain(wd)
            r.set_camera(crt_amd.camera(spp))
            r.init_rand(41)
            r.render(dev, spp, 20)
            r.synchronize()
            assert r.last_kernel_name().startswith(f"crt_render_kernel<false, {variant},")
            out.append((r.linear().view(np.uint32), r.rng_state(), r.counters()["rays"]))
        for o in out[1:]:
            assert np.array_equal(out[0][0], o[0]) and np.array_equal(out[0][1], o[1]) and out[0][2] == o[2]
