"""Frame output: PNG / PPM encoders of the headless renderer.

The reference shows its RGBA8 framebuffer in a window after `flipVertically`
(WindowManager.h:79-93); row 0 of the framebuffer is the bottom row (Camera.cuh:32-44).
The files must hold exactly those pixels, top row first, alpha dropped.  The checker is an
independent decoder: Python's zlib for the deflate stream plus the PNG filter inversion,
CRC-32 of every chunk recomputed.
"""
import struct
import zlib

import numpy as np
import pytest

import crt_amd


def _decode_png(data: bytes) -> np.ndarray:
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, []
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body), typ
        chunks.append((typ, body))
        pos += 12 + n
    assert [c[0] for c in chunks][0] == b"IHDR" and chunks[-1] == (b"IEND", b"")
    w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", chunks[0][1])
    assert (depth, ctype, comp, filt, inter) == (8, 2, 0, 0, 0)
    raw = zlib.decompress(b"".join(b for t, b in chunks if t == b"IDAT"))
    stride = 3 * w
    assert len(raw) == h * (stride + 1)
    out = np.zeros((h, stride), np.int64)
    prev = np.zeros(stride, np.int64)
    for r in range(h):
        ft = raw[r * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, r * (stride + 1) + 1).astype(np.int64)
        cur = np.zeros(stride, np.int64)
        for i in range(stride):
            a = cur[i - 3] if i >= 3 else 0
            b = prev[i]
            c = prev[i - 3] if i >= 3 else 0
            if ft == 0:
                p = 0
            elif ft == 1:
                p = a
            elif ft == 2:
                p = b
            elif ft == 3:
                p = (a + b) >> 1
            elif ft == 4:
                pp = a + b - c
                pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            else:
                raise AssertionError(f"filter {ft}")
            cur[i] = (line[i] + p) & 255
        out[r] = cur
        prev = cur
    return out.reshape(h, w, 3).astype(np.uint8)


def _frames():
    rng = np.random.default_rng(7)
    noise = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    y, x = np.mgrid[0:48, 0:64]
    smooth = np.stack([x * 4, y * 5, (x + y) * 2, np.full_like(x, 255)], -1).astype(np.uint8)
    flat = np.full((16, 300, 4), 200, np.uint8)       # long runs: matches up to 258 bytes, far distances
    one = np.array([[[1, 2, 3, 255]]], np.uint8)
    return {"noise": noise, "smooth": smooth, "flat": flat, "one": one}


@pytest.mark.parametrize("name", ["noise", "smooth", "flat", "one"])
@pytest.mark.parametrize("flip", [True, False])
def test_png_roundtrip(name, flip):
    img = _frames()[name]
    png = crt_amd.encode_image(img, "png", flip=flip)
    want = img[::-1, :, :3] if flip else img[:, :, :3]
    assert np.array_equal(_decode_png(png), want)


def test_png_compresses_smooth_frames():
    img = _frames()["smooth"]
    png = crt_amd.encode_image(img, "png")
    assert len(png) < 0.25 * img.shape[0] * img.shape[1] * 3


def test_ppm_matches_flipped_rgb():
    img = _frames()["noise"]
    ppm = crt_amd.encode_image(img, "ppm")
    h, w = img.shape[:2]
    head = b"P6\n%d %d\n255\n" % (w, h)
    assert ppm[:len(head)] == head
    assert ppm[len(head):] == img[::-1, :, :3].tobytes()


def test_write_image_by_extension(tmp_path):
    img = _frames()["smooth"]
    crt_amd.write_image(tmp_path / "f.png", img)
    assert np.array_equal(_decode_png((tmp_path / "f.png").read_bytes()), img[::-1, :, :3])
    crt_amd.write_image(tmp_path / "f.ppm", img)
    assert (tmp_path / "f.ppm").read_bytes() == crt_amd.encode_image(img, "ppm")
    with pytest.raises(crt_amd.CrtError):
        crt_amd.write_image(tmp_path / "f.bmp", img)
