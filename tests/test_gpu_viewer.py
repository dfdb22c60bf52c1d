"""The interactive loop on the GPU: Raytracer::updateAndRender, headless.

Each frame the C++ loop (host/crt/Raytracer.h, C ABI crth_viewer_*) moves the camera, uploads it and
renders with the camera's spp while every pixel's XORWOW state persists across frames (the reference's
curandState array, CUDAKernels.h:151/:165).  The oracle replays the same input through its camera
controller and renders each frame from the RNG state the previous frame left.  Bar: bit-exact fp32 sums,
RGBA8 bytes and RNG state after every frame (reference BVH), and 1e-4 RMS on the rebuilt BVH.
"""
import numpy as np
import pytest

import crt_amd
import pyoracle

pytestmark = pytest.mark.gpu
W, H = 64, 36
BENCH_POS = (0.0, 0.0, 0.3)


def _script():
    k = crt_amd
    return [
        (0.016, {}), (0.016, {}),                                      # idle: 1 spp, RNG continues
        (0.05, {"keys": k.KEY_W}),                                      # walk forward
        (0.016, {"right_mouse": True, "mouse_x": 300.0, "mouse_y": 200.0}),   # press (skipped)
        (0.016, {"right_mouse": True, "mouse_x": 340.0, "mouse_y": 190.0}),   # rotate
        (0.016, {}),
        (0.016, {"keys": k.KEY_F}),                                     # high quality: 2000 spp
        (0.016, {"focus_steps": 1}),                                    # still high quality, new focus
        (0.016, {"keys": k.KEY_D}),                                     # motion: back to 1 spp
    ]


def _oracle_scene(files):
    import objload
    return pyoracle.OracleScene(objload.load_scene(files))


@pytest.mark.parametrize("bvh", ["reference", "rebuilt"])
def test_viewer_frames_match_oracle(scenes, bvh):
    files = scenes["cornell_bunny"]
    kw = {} if bvh == "reference" else {"bvh_width": 4, "leaf_size": 4, "traversal_cost": 2.0}
    v = crt_amd.Viewer(files, W, H, bvh=bvh, pos=BENCH_POS, focus=0.3, seed=41, **kw)
    osc = _oracle_scene(files)
    ctl = pyoracle.CameraController(pos=BENCH_POS, focus=0.3)
    rng = np.stack([pyoracle.rng_init(41, p) for p in range(W * H)]).reshape(H, W, 6)
    assert np.array_equal(v.renderer.rng_state(), rng)
    spps = []
    for i, (dt, inp) in enumerate(_script()):
        info = v.frame(dt, **inp)
        ctl.update(dt, W, H, **inp)
        cam, st = ctl.get()
        assert info["spp"] == st["spp"] and info["frame"] == i + 1
        assert info["moving"] == (st["moving"] or st["rotating"])   # Camera::isCameraInMotion
        assert crt_amd.camera_floats(v.camera()).view(np.uint32).tolist() == cam.view(np.uint32).tolist()
        o_sum, o_rgba, _ = osc.render_rng(cam, W, H, st["spp"], rng)
        lin, rgba = v.renderer.linear(), v.renderer.rgba8()
        spps.append(info["spp"])
        if bvh == "reference":
            assert np.array_equal(lin.view(np.uint32), o_sum.view(np.uint32)), f"frame {i}"
            assert np.array_equal(rgba, o_rgba), f"frame {i}"
            assert np.array_equal(v.renderer.rng_state(), rng), f"frame {i}: RNG state"
        else:
            rms = np.sqrt(np.mean(((lin - o_sum) / st["spp"]).astype(np.float64) ** 2, axis=(0, 1)))
            assert (rms <= 1e-4).all(), (i, rms)
            rng = v.renderer.rng_state().copy()   # continue from the GPU's state (paths may fork on rounding)
    assert spps == [1, 1, 1, 1, 1, 1, 2000, 2000, 1]
    v.close()


def test_accumulate_equals_one_frame_of_k_spp(scenes, oracle_scenes):
    files = scenes["cornell_bunny"]
    v = crt_amd.Viewer(files, W, H, pos=BENCH_POS, focus=0.3, seed=41, accumulate=True)
    k = 6
    for i in range(k):
        info = v.frame(0.016)
        assert info["accumulated"] == i + 1 and info["spp"] == 1
    cam = pyoracle.CameraController(pos=BENCH_POS, focus=0.3)
    cam.update(0.016, W, H)
    o_sum, o_rgba, _ = oracle_scenes["cornell_bunny"].render(cam.get()[0], W, H, k, 20, seed=41)
    assert np.array_equal(v.renderer.linear().view(np.uint32), o_sum.view(np.uint32))
    assert np.array_equal(v.renderer.rgba8(), o_rgba)
    info = v.frame(0.016, keys=crt_amd.KEY_W)        # motion restarts the image
    assert info["accumulated"] == 1 and info["moving"]
    info = v.frame(0.016)
    assert info["accumulated"] == 1
    info = v.frame(0.016)
    assert info["accumulated"] == 2
    v.close()


def test_temporal_order_is_bit_identical(device_scenes):
    """Variant 7 with the temporal tile order (crt_renderer_set_temporal_order): from the second frame on, tiles are
    dispatched by the previous frame's rays per pixel; 1-spp frames accumulated over 4 frames (RNG state continuing) give
    the same sums, RNG state and ray counts as row order, at a ragged size too.  So do drain thresholds
    (crt_renderer_set_drain_threshold: 1 and 8 parked lanes once the pixel queue is empty)."""
    import numpy as np
    import crt_amd
    hs, _ = device_scenes["cornell_bunny"]
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    for w, h in ((640, 360), (100, 37)):
        out = []
        for on, drain in ((False, 0), (True, 0), (True, 1), (False, 8)):
            r = crt_amd.Renderer(w, h)
            r.set_temporal_order(on)
            r.set_drain_threshold(drain)
            r.set_camera(crt_amd.camera(1))
            r.init_rand(41)
            rays = []
            for f in range(4):
                r.render(sc, 1, 20, accumulate=f > 0)
                r.synchronize()
                assert r.last_kernel_name().startswith("crt_render_kernel<false, 7,")
                rays.append(r.counters()["rays"])
            out.append((r.linear().view(np.uint32), r.rng_state(), rays))
        for o in out[1:]:
            assert np.array_equal(out[0][0], o[0]) and np.array_equal(out[0][1], o[1]) and out[0][2] == o[2]
