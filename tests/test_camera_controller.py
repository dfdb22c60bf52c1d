"""Per-frame camera controller: Camera::updateCamera / updateRotation /
updatePosition (Camera.cuh:46-157) driven by a scripted input stream.

The C++ controller (host/crt/Camera.h, C ABI crth_camera_*) is compared bit for bit with the
oracle's C restatement (oracle_camctl_*) on every frame: the 19 camera floats the kernel reads,
yaw / pitch / focus, the motion flags and the spp / scale the frame renders with.
"""
import numpy as np
import pytest

import crt_amd

W_, A_, S_, D_, SP_, LC_, F_ = (crt_amd.KEY_W, crt_amd.KEY_A, crt_amd.KEY_S, crt_amd.KEY_D, crt_amd.KEY_SPACE,
                                crt_amd.KEY_LCONTROL, crt_amd.KEY_F)


def script():
    """(dt, input) per frame: idle, every key, a drag with smoothing, a pitch clamp, F toggles, focus keys."""
    f = []
    f += [(0.016, {})] * 2
    f += [(0.016, {"keys": W_}), (0.033, {"keys": W_ | D_}), (0.020, {"keys": S_ | SP_}), (0.018, {"keys": A_ | LC_})]
    f += [(0.016, {"keys": W_ | S_})]                          # opposite keys: moves and comes back (rounding)
    f += [(0.016, {"right_mouse": True, "mouse_x": 500.0, "mouse_y": 300.0})]   # first press: skipped
    for k in range(6):                                          # drag right and up
        f.append((0.016, {"right_mouse": True, "mouse_x": 500.0 + 37.5 * (k + 1), "mouse_y": 300.0 - 11.25 * k}))
    f += [(0.016, {})]                                          # release
    f += [(0.016, {"right_mouse": True, "mouse_x": 10.0, "mouse_y": 10.0})]
    for k in range(5):                                          # large vertical drag: pitch clamps at +-89
        f.append((0.016, {"right_mouse": True, "mouse_x": 10.0, "mouse_y": 10.0 - 900.0 * (k + 1)}))
    f += [(0.016, {})]
    f += [(0.016, {"keys": F_}), (0.016, {}), (0.016, {})]       # high-quality on: 2000 spp while still
    f += [(0.016, {"keys": F_}), (0.016, {})]                    # off again
    f += [(0.016, {"keys": F_}), (0.016, {"keys": W_}), (0.016, {})]   # motion cancels high quality
    f += [(0.016, {"keys": F_}), (0.016, {"keys": F_})]          # held: toggles every frame
    f += [(0.016, {"focus_steps": 1}), (0.016, {"focus_steps": -3}), (0.016, {"focus_steps": -80})]  # clamp 0.1
    f += [(0.25, {"keys": W_ | A_ | SP_})]
    return f


@pytest.mark.parametrize("pose", [((0.0, 4.0, 4.0), None), ((0.0, 0.0, 0.3), 0.3)])
def test_controller_matches_oracle(pose):
    import pyoracle
    pos, focus = pose
    ww, wh = 1280, 720
    host = crt_amd.CameraController(pos=pos, focus=focus)
    orc = pyoracle.CameraController(pos=pos, focus=focus)
    seen = {"hq": 0, "moving": 0, "rotating": 0, "clamped": 0}
    for i, (dt, inp) in enumerate(script()):
        host.update(dt, ww, wh, **inp)
        orc.update(dt, ww, wh, **inp)
        d, st = host.get()
        cam, ost = orc.get()
        got = crt_amd.camera_floats(d)
        assert got.view(np.uint32).tolist() == cam.view(np.uint32).tolist(), f"frame {i}"
        assert d.samples_per_pixel == ost["spp"] and np.float32(d.pixel_sample_scale) == np.float32(ost["scale"])
        for k in ("yaw", "pitch", "focus"):
            assert np.float32(st[k]).view(np.uint32) == np.float32(ost[k]).view(np.uint32), (i, k)
        for k in ("moving", "rotating", "high_quality"):
            assert st[k] == ost[k], (i, k)
        seen["hq"] += st["high_quality"]
        seen["moving"] += st["moving"]
        seen["rotating"] += st["rotating"]
        seen["clamped"] += abs(st["pitch"]) == 89.0
    # the script exercised every branch
    assert seen["hq"] >= 3 and seen["moving"] >= 5 and seen["rotating"] >= 8 and seen["clamped"] >= 1
    d, st = host.get()
    assert st["focus"] == pytest.approx(0.1)


def test_controller_rules():
    """Reference rules spelled out: idle = 1 spp, F = 2000 spp while still, motion resets to 1."""
    c = crt_amd.CameraController()
    c.update(0.016, 640, 360)
    assert c.get()[0].samples_per_pixel == 1
    c.update(0.016, 640, 360, keys=F_)
    d, st = c.get()
    assert st["high_quality"] and d.samples_per_pixel == 2000 and np.float32(d.pixel_sample_scale) == np.float32(1 / 2000)
    c.update(0.016, 640, 360)
    assert c.get()[0].samples_per_pixel == 2000
    c.update(0.016, 640, 360, keys=S_)
    d, st = c.get()
    assert st["moving"] and not st["high_quality"] and d.samples_per_pixel == 1
