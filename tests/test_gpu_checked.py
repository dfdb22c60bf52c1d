"""The checked build and the benchmarked schedule against the oracle (GPU, through the C ABI).

* The checked library (lib/checked/libcrt_hip.so, -DCRT_CHECKED, built by `make all`) re-checks every leaf-round pair
  of the 4-wide kernels: its owner lane, that the pair lies inside the owner's span, and the primitive index
  (crt_hip.hip traverse_step4).  A stale LDS owner mark, the cause of round 2's GPU fault (profiles/r02au), then
  reports through crt_renderer_synchronize instead of loading outside the primitive array.  It runs in a child
  process (one HIP library per process), renders the smoke frame and config-B-shaped crops through variants 4, 7 and 8,
  and must report no error and produce exactly the fast library's frames.
* Variant 8 with its cost probe, tile sort and critical tiles (the configuration bench.py times, spp >= 64) next to
  the oracle directly: the rebuilt-BVH frame against the oracle's (the reference path restated), by the north-star
  bar (<= 1e-4 per-channel RMS) and >= 99.9 % of pixels bit-identical.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import crt_amd
from crt_amd import _lib, assets

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]
CHECKED = REPO / "raytracer-cuda_amd" / "lib" / "checked" / "libcrt_hip.so"
CASES = [(160, 90, 8, 8), (160, 90, 8, 7), (160, 90, 8, 4), (96, 64, 64, 8)]   # (w, h, spp, kernel variant)

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import crt_amd
from crt_amd import _lib, assets
out = {"flags": int(_lib.hip().crt_build_flags()), "frames": []}
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0)
for w, h, spp, var in json.loads(sys.argv[3]):
    r = crt_amd.Renderer(w, h)
    r.set_kernel_variant(var)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41)
    r.render(sc, spp, 20)
    r.synchronize()
    out["frames"].append(r.linear().view(np.uint32).tolist())
json.dump(out, open(sys.argv[2], "w"))
"""


def _fast_frames():
    hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0)
    frames = []
    for w, h, spp, var in CASES:
        r = crt_amd.Renderer(w, h)
        r.set_kernel_variant(var)
        r.set_camera(crt_amd.camera(spp))
        r.init_rand(41)
        r.render(sc, spp, 20)
        r.synchronize()
        frames.append(r.linear().view(np.uint32))
    return frames


def test_checked_build_reports_nothing_and_matches(tmp_path):
    assert CHECKED.exists(), "make all builds lib/checked/libcrt_hip.so"
    assert _lib.hip().crt_build_flags() == 0, "the in-tree library is the fast build"
    res = tmp_path / "checked.json"
    env = dict(os.environ, CRT_HIP_LIB=str(CHECKED))
    p = subprocess.run([sys.executable, "-c", CHILD, str(REPO / "raytracer-cuda_amd"), str(res), json.dumps(CASES)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(res.read_text())
    assert got["flags"] == _lib.BUILD_CHECKED
    for (w, h, spp, var), fast, chk in zip(CASES, _fast_frames(), got["frames"]):
        chk = np.array(chk, np.uint32).reshape(fast.shape)
        assert np.array_equal(chk, fast), f"checked build differs at {w}x{h} {spp}spp variant {var}"


def test_variant8_probe_schedule_against_oracle(oracle_scenes, device_scenes):
    """The benchmarked configuration end to end (rebuilt 4-wide BVH, automatic variant 8 with the 4-spp cost probe,
    the tile sort and critical tiles, spp >= 64) against the oracle frame."""
    hs, _ = device_scenes["cornell_bunny"]
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    w, h, spp = 128, 72, 96
    r = crt_amd.Renderer(w, h)
    cam = crt_amd.camera(spp)
    r.set_camera(cam)
    r.init_rand(41)
    r.render(sc, spp, 20)
    r.synchronize()
    assert r.last_kernel_name() == "crt_render_kernel<false, 8, 4>"
    lin = r.linear()
    o_sum, _, o_cnt = oracle_scenes["cornell_bunny"].render(crt_amd.camera_floats(cam), w, h, spp, 20)
    rms = np.sqrt(np.mean(((lin - o_sum) / spp).astype(np.float64) ** 2, axis=(0, 1)))
    assert (rms <= 1e-4).all(), f"per-channel RMS {rms}"
    eq = float(np.mean(np.all(lin.view(np.uint32) == o_sum.view(np.uint32), axis=-1)))
    assert eq >= 0.999, f"only {eq:.6f} of pixels bit-identical"
    rays = r.counters()["rays"]
    assert abs(rays - o_cnt["rays"]) <= 1e-5 * o_cnt["rays"]


def test_render_phase_timings(device_scenes):
    """crt_renderer_last_timings: the whole render = probe + tile sort + main kernel (HIP events, ms)."""
    hs, _ = device_scenes["cornell_bunny"]
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    r = crt_amd.Renderer(160, 90)
    r.set_camera(crt_amd.camera(64))
    r.init_rand(41)
    r.render(sc, 64, 20)                       # variant 8 with the cost probe
    t = r.last_timings()
    assert t["probe_sort_ms"] > 0 and t["main_kernel_ms"] > 0
    assert abs(t["render_ms"] - (t["probe_sort_ms"] + t["main_kernel_ms"])) < 0.05 * t["render_ms"] + 0.05
    assert abs(t["render_ms"] - r.last_kernel_ms()) < 1e-3
    r.set_kernel_variant(4)
    r.render(sc, 8, 20)                        # no probe: the main kernel is the whole render
    t = r.last_timings()
    # (two back-to-back events on the stream: their gap is launch overhead, measured 0.03-0.055 ms on the pool's boxes)
    assert t["probe_sort_ms"] < 0.25 and abs(t["render_ms"] - t["main_kernel_ms"]) < 0.25


@pytest.mark.parametrize("w,h,spp", [(96, 64, 64), (100, 37, 70), (40, 24, 8)])
def test_variant10_reference_bvh_bit_exact(device_scenes, oracle_scenes, w, h, spp):
    """Variant 10 (variant 3's wave program on the reference's own BVHs, scheduled like variant 8: one 8x8 tile per
    one-wave workgroup, most expensive first by a variant-3 cost probe at spp >= 64) renders the oracle's frame bit for
    bit, ragged sizes included."""
    _, ref = device_scenes["cornell_bunny"]
    r = crt_amd.Renderer(w, h)
    cam = crt_amd.camera(spp)
    r.set_camera(cam)
    r.set_kernel_variant(10)
    r.init_rand(41)
    r.render(ref, spp, 20)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    assert r.last_kernel_name() == "crt_render_kernel<false, 10, 6>"
    assert r.last_timings()["main_kernel_ms"] > 0
    o_sum, o_rgba, o_cnt = oracle_scenes["cornell_bunny"].render(crt_amd.camera_floats(cam), w, h, spp, 20)
    assert np.array_equal(r.linear().view(np.uint32), o_sum.view(np.uint32))
    assert np.array_equal(r.rgba8(), o_rgba)
    assert r.counters()["rays"] == o_cnt["rays"]


@pytest.mark.parametrize("occ", [5, 7])
def test_variant10_other_occupancies_bit_exact(device_scenes, oracle_scenes, occ):
    """Variant 10 at 5 and 7 waves/SIMD (the default is 6) renders the oracle's frame bit for bit too."""
    _, ref = device_scenes["cornell_bunny"]
    w, h, spp = 96, 64, 64
    r = crt_amd.Renderer(w, h)
    cam = crt_amd.camera(spp)
    r.set_camera(cam)
    r.set_kernel_variant(10)
    r.set_occupancy_target(occ)
    r.init_rand(41)
    r.render(ref, spp, 20)
    r.synchronize()
    assert r.last_kernel_name() == f"crt_render_kernel<false, 10, {occ}>"
    o_sum, _, o_cnt = oracle_scenes["cornell_bunny"].render(crt_amd.camera_floats(cam), w, h, spp, 20)
    assert np.array_equal(r.linear().view(np.uint32), o_sum.view(np.uint32))
    assert r.counters()["rays"] == o_cnt["rays"]
