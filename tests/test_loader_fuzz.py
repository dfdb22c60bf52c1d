"""Malformed OBJ/MTL input through the host scene pipeline (CPU only).

The loader (host/crt/ObjLoader.cpp, restating SceneManager.h:198-329 and tinyobjloader v1.0's parser) takes untrusted
files.  Every input here must either load into a self-consistent scene or fail with CrtError: no crash, no hang, no
out-of-bounds access.  tools/run_asan.sh runs this file under AddressSanitizer + UndefinedBehaviorSanitizer
(`make asan`), which turns a silent out-of-bounds read into a failure.

Cases: hand-written truncated / garbage lines (the parser's every branch: numbers, faces, v/t/n tokens, relative and
out-of-range indices, mtllib/usemtl/newmtl), then seeded random mutations (byte deletions, insertions, truncation,
line shuffles) of a valid Cornell-like file.  A loaded scene is also pushed through crt_scene_export in both BVH modes
(flattening, the reference builders, the binned SAH and the SBVH builder) on the host.
"""
import os

import numpy as np
import pytest

import crt_amd

VALID_MTL = ("newmtl white\nKd 0.73 0.73 0.73\nnewmtl light\nKe 15 15 15\nKd 1 1 1\n"
             "newmtl glass\nKd 1 1 1\nd 0.1\nNi 1.5\nnewmtl metal\nKd 0.8 0.8 0.8\nKs 1 1 1\nNs 80\n")
VALID_OBJ = ("mtllib m.mtl\n"
             "v -1 -1 -1\nv 1 -1 -1\nv 1 1 -1\nv -1 1 -1\nv -1 -1 1\nv 1 -1 1\nv 1 1 1\nv -1 1 1\n"
             "v -0.2 0.99 -0.2\nv 0.2 0.99 -0.2\nv 0.2 0.99 0.2\nv -0.2 0.99 0.2\n"
             "usemtl white\nf 1 2 3 4\nf 5 6 7 8\nf 1 5 8 4\nusemtl metal\nf 2 6 7 3\n"
             "usemtl light\nf 9 10 11 12\nusemtl glass\nf -4 -3 -2\n")

HAND = [
    "",                                   # empty file
    "v 1\n",                              # too few coordinates
    "v\nv\nv\nf 1 2 3\n",                 # missing coordinates default to 0
    "f\n", "f 1\n", "f 1 2\n",            # faces with < 3 vertices are dropped
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",      # zero index: error
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 99\n",     # past the last vertex
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -99 1 2\n",    # relative index before the first vertex
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1/1/1 2//2 3/3\n",
    "v abc def ghi\nv 1e 1e+ 1e-\nv --1 ++2 .\nf 1 2 3\n",
    "v 1e99999 0 0\nv 0 1 0\nv 0 0 1\nf 1 2 3\n",          # overflow to inf
    "v 1e-99999 0 0\nv 0 1 0\nv 0 0 1\nf 1 2 3\n",
    "v 0 0 0\nv 0 0 0\nv 0 0 0\nf 1 2 3\n",                 # degenerate triangle, zero-size scene
    "v 1 2 3\nv 1 2 3\nv 1 2 3\nv 1 2 3\nf 1 2 3 4\nf 4 3 2 1\n",
    "v 0 0 0\r\nv 1 0 0\r\nv 0 1 0\r\nf 1 2 3\r\n",         # CRLF
    "v\t0\t0\t0\nv\t1\t0\t0\nv\t0\t1\t0\nf\t1\t2\t3",       # tabs, no final newline
    "mtllib\nusemtl\nnewmtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n",
    "mtllib missing.mtl other_missing.mtl\nusemtl nothing\nv 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n",
    "# only a comment\n#\n   \n\t\n",
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3 " + " ".join(["1"] * 300) + "\n",   # a 303-gon
    "v " + "9" * 400 + " 0 0\nv 0 1 0\nv 0 0 1\nf 1 2 3\n",                 # 400-digit mantissa
    "v 0." + "1" * 400 + " 0 0\nv 0 1 0\nv 0 0 1\nf 1 2 3\n",
    "v 1e-2147483648 0 0\nv 1e2147483647 0 0\nv 0 0 1\nf 1 2 3\n",         # exponent overflow
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 2147483647 1 2\nf -2147483648 1 2\n",
    "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 99999999999999999999 1 2\n",
]
HAND_MTL = [
    "newmtl\nKd\nKs 1\nKe\nd\nTr\nNi\nNs\nPr\n",
    "Kd 1 1 1\nnewmtl a\nKd x y z\nKe 1e999 0 0\nnewmtl a\nd -5\nNi 0\n",
    "newmtl a b c\nKs 1 1 1\nNs -2\n",                  # Ns = -2: roughness sqrt(2 / 0)
    "newmtl m\x00\x01\x02\nKd 1 1 1\n",
]


def _write(d, name, data):
    p = os.path.join(d, name)
    with open(p, "wb") as f:
        f.write(data if isinstance(data, bytes) else data.encode("latin-1"))
    return p


def _consistent(hs):
    """The loaded arrays point inside each other."""
    pos, idx, fm, info, mats = hs.loader_arrays()
    c = hs.counts()
    assert len(idx) == c["n_indices"] and len(fm) == c["n_faces"] == len(idx) // 3
    if len(idx):
        assert int(idx.max()) < len(pos)
    if len(fm) and len(mats):
        assert 0 <= int(fm.min()) and int(fm.max()) < len(mats) + int(info[:, 5].max()) + 1


def _exercise(files):
    try:
        hs = crt_amd.HostScene(files)
    except crt_amd.CrtError:
        return "rejected"
    _consistent(hs)
    for opts in (dict(bvh="reference"), dict(bvh="rebuilt", width=4), dict(bvh="rebuilt", width=4, spatial_splits=True),
                 dict(bvh="rebuilt", width=2, layouts=6)):
        try:
            hs.export(**opts)
        except (crt_amd.CrtError, RuntimeError):
            pass
    return "loaded"


@pytest.mark.timeout(120)
def test_hand_written_malformed_objs(tmp_path):
    d = str(tmp_path)
    _write(d, "m.mtl", VALID_MTL)
    seen = set()
    for k, text in enumerate(HAND):
        seen.add(_exercise([_write(d, f"h{k}.obj", "mtllib m.mtl\n" + text)]))
        seen.add(_exercise([_write(d, f"g{k}.obj", text)]))
    assert seen == {"loaded", "rejected"}


@pytest.mark.timeout(120)
def test_hand_written_malformed_mtls(tmp_path):
    d = str(tmp_path)
    for k, text in enumerate(HAND_MTL):
        _write(d, f"m{k}.mtl", text)
        obj = _write(d, f"o{k}.obj", VALID_OBJ.replace("m.mtl", f"m{k}.mtl"))
        assert _exercise([obj]) == "loaded"


def _mutate(rng, data: bytes) -> bytes:
    b = bytearray(data)
    for _ in range(int(rng.integers(1, 6))):
        op = int(rng.integers(0, 5))
        if not b:
            break
        i = int(rng.integers(0, len(b)))
        if op == 0:                                   # delete a run
            del b[i:i + int(rng.integers(1, 8))]
        elif op == 1:                                 # insert bytes from the OBJ alphabet
            alpha = b"0123456789 -+.eE/\nvf#\t\r"
            b[i:i] = bytes(alpha[int(j)] for j in rng.integers(0, len(alpha), int(rng.integers(1, 6))))
        elif op == 2:                                 # truncate
            del b[i:]
        elif op == 3:                                 # random byte
            b[i] = int(rng.integers(0, 256))
        else:                                         # swap two lines
            lines = bytes(b).split(b"\n")
            if len(lines) > 2:
                x, y = rng.integers(0, len(lines), 2)
                lines[x], lines[y] = lines[y], lines[x]
                b = bytearray(b"\n".join(lines))
    return bytes(b)


@pytest.mark.timeout(300)
def test_random_mutations(tmp_path):
    d = str(tmp_path)
    rng = np.random.default_rng(20261017)
    counts = {"loaded": 0, "rejected": 0}
    for k in range(150):
        _write(d, "m.mtl", _mutate(rng, VALID_MTL.encode()) if k % 3 == 0 else VALID_MTL)
        obj = _write(d, f"r{k}.obj", _mutate(rng, VALID_OBJ.encode()))
        counts[_exercise([obj])] += 1
    assert counts["loaded"] > 50 and counts["rejected"] > 0, counts
