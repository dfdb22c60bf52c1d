"""Regenerate tests/golden/* from the CPU oracle (oracle/crt_oracle.c + oracle/objload.py).

    python tests/golden/make_golden.py

Fixtures (small; data only):
  xorwow_kat.json        curand_init(41, subseq) states + first 8 outputs / uniforms
  scene_bvh.json         Cornell mesh BVH + scene BVH node arrays (fp32 as hex), bunny BVH digest
  frames.json            config A (256x256, 16 spp, 4 / 20 bounces) and Cornell+bunny 64x36/16 spp:
                         ray counts, SHA-256 of the fp32 linear sums and RGBA8 bytes, channel means
  cornell_bunny_64x36_16spp.npz   the fp32 linear sum + RGBA8 of that frame
External anchors reproduced (not generated here): the reference-run ray counts recorded in
SURVEY.md/BASELINE.md (3,197,876 and 3,420,058 for config A) and rocRAND's XORWOW
sequence-jump table.
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO / "oracle"), str(REPO / "raytracer-cuda_amd")]
import objload  # noqa: E402
import pyoracle  # noqa: E402
from crt_amd import assets  # noqa: E402

SUBSEQS = [0, 1, 2, 1000, 3686399, 7372800 + 5]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def hexf(a: np.ndarray):
    return [format(int(x), "08x") for x in np.asarray(a, np.float32).view(np.uint32).ravel()]


def xorwow_kat():
    out = []
    for s in SUBSEQS:
        st = pyoracle.rng_init(41, s)
        u, f = pyoracle.rng_draw(st.copy(), 8)
        out.append({"seed": 41, "subsequence": s, "state": [int(x) for x in pyoracle.rng_init(41, s)],
                    "u32": [int(x) for x in u], "uniform_hex": hexf(f)})
    return out


def bvh_fixture():
    L = objload.load_scene(assets.scene_files("cornell"))
    S = pyoracle.OracleScene(L)
    mb, mi = S.nodes(0)
    sb, si = S.nodes(-1)
    LB = objload.load_scene(assets.scene_files("cornell_bunny"))
    SB = pyoracle.OracleScene(LB)
    bb, bi = SB.nodes(1)
    return {"cornell_mesh": {"boxes_hex": hexf(mb), "ints": mi.tolist()},
            "cornell_scene": {"boxes_hex": hexf(sb), "ints": si.tolist()},
            "bunny_mesh": {"n_nodes": int(len(bb)), "boxes_sha256": sha(bb),
                           "leaf_sha256": sha(bi[bi[:, 4] == 1][:, 2:4]), "max_leaf_tris": int(bi[bi[:, 4] == 1][:, 3].max() // 3)}}


def frames():
    cam = pyoracle.camera()
    res = {}
    LA = pyoracle.OracleScene(objload.load_scene(assets.scene_files("cornell")))
    for b in (4, 20):
        s, rgba, c = LA.render(cam, 256, 256, 16, b)
        res[f"configA_256x256_16spp_{b}b"] = {"rays": c["rays"], "box_tests": c["box_tests"], "tri_tests": c["tri_tests"],
                                              "sphere_tests": c["sphere_tests"], "sum_sha256": sha(s),
                                              "rgba_sha256": sha(rgba), "mean_linear": (s.mean((0, 1)) / 16).tolist()}
    LB = pyoracle.OracleScene(objload.load_scene(assets.scene_files("cornell_bunny")))
    s, rgba, c = LB.render(cam, 64, 36, 16, 20)
    res["cornell_bunny_64x36_16spp_20b"] = {"rays": c["rays"], "box_tests": c["box_tests"], "tri_tests": c["tri_tests"],
                                            "sphere_tests": c["sphere_tests"], "sum_sha256": sha(s),
                                            "rgba_sha256": sha(rgba), "mean_linear": (s.mean((0, 1)) / 16).tolist()}
    np.savez_compressed(HERE / "cornell_bunny_64x36_16spp.npz", sum=s, rgba=rgba)
    return res


if __name__ == "__main__":
    (HERE / "xorwow_kat.json").write_text(json.dumps(xorwow_kat(), indent=1))
    (HERE / "scene_bvh.json").write_text(json.dumps(bvh_fixture()))
    (HERE / "frames.json").write_text(json.dumps(frames(), indent=1))
    print("golden fixtures written to", HERE)
