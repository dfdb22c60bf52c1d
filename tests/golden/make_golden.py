"""Regenerate tests/golden/* from the CPU oracle (oracle/crt_oracle.c + oracle/objload.py).

    python tests/golden/make_golden.py

Fixtures (small; data only):
  xorwow_kat.json        curand_init(41, subseq) states + first 8 outputs / uniforms
  scene_bvh.json         Cornell mesh BVH + scene BVH node arrays (fp32 as hex), bunny BVH digest
  frames.json            config A (256x256, 16 spp, 4 / 20 bounces) and Cornell+bunny 64x36/16 spp:
                         ray counts, SHA-256 of the fp32 linear sums and RGBA8 bytes, channel means
  cornell_bunny_64x36_16spp.npz   the fp32 linear sum + RGBA8 of that frame
  cornell_1m_64x36_8spp.npz       config E slice (1,000,032 triangles): fp32 sum + RGBA8 + ray count
  primitives.json        known answers of Moller-Trumbore, AABB::hit, Sphere::hit and Camera::getRay on random
                         and edge-case inputs (zero-thickness boxes, axis-parallel rays, grazing / tangent rays,
                         det ~ 0, origins inside spheres, the radius-999 ground sphere)
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


def config_e_slice():
    """Config E's scene (Cornell + 1M-triangle bunny instancing) through the oracle: 64x36, 8 spp, 20 bounces."""
    cam = pyoracle.camera()
    L = pyoracle.OracleScene(objload.load_scene(assets.scene_files("cornell_1m")))
    s, rgba, c = L.render(cam, 64, 36, 8, 20)
    np.savez_compressed(HERE / "cornell_1m_64x36_8spp.npz", sum=s, rgba=rgba, rays=np.array([c["rays"]], np.int64))
    return {"rays": c["rays"], "sum_sha256": sha(s), "rgba_sha256": sha(rgba)}


def _kat_records():
    rng = np.random.default_rng(2024)
    f = np.float32
    tri, box, sph = [], [], []
    inf = np.inf
    for _ in range(300):   # rays towards random triangles around a point on the ray (hits and near misses)
        o = rng.uniform(-1, 1, 3)
        d = rng.normal(size=3)
        p = o + rng.uniform(0.2, 3.0) * d
        v = p + rng.normal(scale=rng.choice([0.05, 0.3, 1.0]), size=(3, 3))
        tri.append(np.concatenate([o, d, v.ravel(), [0.001, rng.choice([inf, rng.uniform(0.5, 4.0)])]]))
    for _ in range(40):    # edge cases: through a vertex / an edge midpoint, parallel plane, behind, just in front
        v = rng.normal(size=(3, 3))
        o = rng.normal(size=3) * 3
        for target in (v[0], 0.5 * (v[1] + v[2]), (v[0] + v[1] + v[2]) / 3):
            tri.append(np.concatenate([o, target - o, v.ravel(), [0.001, inf]]))
        n = np.cross(v[1] - v[0], v[2] - v[0])
        dpar = np.cross(n, rng.normal(size=3))   # parallel to the plane: det ~ 0
        tri.append(np.concatenate([o, dpar, v.ravel(), [0.001, inf]]))
        tri.append(np.concatenate([v[0] + 1e-4 * n, -n, v.ravel(), [0.001, inf]]))   # t just below 0.001
    for _ in range(300):   # boxes, some with a zero-thickness axis, rays with zero direction components
        lo = rng.uniform(-1, 1, 3)
        hi = lo + rng.uniform(0, 1, 3)
        k = rng.integers(0, 4)
        if k < 3:
            hi[k] = lo[k]                        # zero thickness: the reference never enters it
        o = rng.uniform(-2, 2, 3)
        d = rng.normal(size=3)
        if rng.random() < 0.3:
            d[rng.integers(0, 3)] = 0.0          # 1/d = inf: the NaN-dropping fminf/fmaxf path
        if rng.random() < 0.2:
            o[rng.integers(0, 3)] = lo[rng.integers(0, 3)]
        box.append(np.concatenate([o, d, lo, hi, [0.001, inf]]))
    for _ in range(200):   # spheres: random, tangent, origin inside
        c = rng.uniform(-1, 1, 3)
        r = rng.uniform(0.05, 1.0)
        o = c + rng.normal(size=3) * rng.choice([0.5 * r, 2.0, 5.0])
        d = rng.normal(size=3)
        sph.append(np.concatenate([o, d, c, [r], [0.001, rng.choice([inf, rng.uniform(0.5, 6.0)])]]))
    for _ in range(100):   # the ground sphere of the benchmark scene (catastrophic cancellation in f32)
        o = rng.uniform(-0.3, 0.3, 3)
        o[1] = rng.choice([o[1], -1.0 + rng.uniform(0, 1e-3)])
        d = rng.normal(size=3)
        d[1] = -abs(d[1])
        sph.append(np.concatenate([o, d, [0.0, -1000.0, 0.0], [999.0], [0.001, inf]]))
    return (np.asarray(tri, f), np.asarray(box, f), np.asarray(sph, f))


def primitive_kats():
    import ctypes as C
    L = pyoracle.lib()
    for name, argt in (("oracle_kat_triangle", [C.c_void_p, C.c_int, C.c_void_p]),
                       ("oracle_kat_box", [C.c_void_p, C.c_int, C.c_void_p]),
                       ("oracle_kat_sphere", [C.c_void_p, C.c_int, C.c_void_p]),
                       ("oracle_kat_get_ray", [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                               C.c_void_p])):
        getattr(L, name).argtypes = argt
    tri, box, sph = _kat_records()
    t_out = np.zeros(len(tri), np.float32)
    L.oracle_kat_triangle(tri.ctypes.data, len(tri), t_out.ctypes.data)
    b_out = np.zeros(len(box), np.int32)
    L.oracle_kat_box(box.ctypes.data, len(box), b_out.ctypes.data)
    s_out = np.zeros(len(sph), np.float32)
    L.oracle_kat_sphere(sph.ctypes.data, len(sph), s_out.ctypes.data)
    cam = pyoracle.camera()
    w, h = 2560, 1440
    xy = np.array([[0, 0], [2559, 1439], [1280, 720], [7, 1000], [2000, 3], [640, 360], [1919, 1079], [1, 1438],
                   [100, 200], [300, 400], [500, 600], [700, 800], [900, 1000], [1100, 1200], [1300, 100],
                   [2558, 1]], np.int32)
    rng0 = np.stack([pyoracle.rng_init(41, int(y) * w + int(x)) for x, y in xy]).astype(np.uint32)
    rng1 = rng0.copy()
    rays = np.zeros((len(xy), 6), np.float32)
    L.oracle_kat_get_ray(cam.ctypes.data, w, h, xy.ctypes.data, rng1.ctypes.data, len(xy), rays.ctypes.data)
    return {"triangle": {"in_hex": hexf(tri), "t_hex": hexf(t_out), "hits": int((t_out >= 0).sum())},
            "box": {"in_hex": hexf(box), "hit": b_out.tolist(), "hits": int(b_out.sum())},
            "sphere": {"in_hex": hexf(sph), "t_hex": hexf(s_out), "hits": int((s_out >= 0).sum())},
            "get_ray": {"camera_hex": hexf(cam), "width": w, "height": h, "xy": xy.tolist(),
                        "rng_in": rng0.tolist(), "rng_out": rng1.tolist(), "ray_hex": hexf(rays)}}


if __name__ == "__main__":
    (HERE / "xorwow_kat.json").write_text(json.dumps(xorwow_kat(), indent=1))
    (HERE / "scene_bvh.json").write_text(json.dumps(bvh_fixture()))
    fr = frames()
    fr["cornell_1m_64x36_8spp_20b"] = config_e_slice()
    (HERE / "frames.json").write_text(json.dumps(fr, indent=1))
    (HERE / "primitives.json").write_text(json.dumps(primitive_kats()))
    print("golden fixtures written to", HERE)
