"""Replay rays from tools/mismatch_dump.py through the reference BVH (float32 restatement of AABB::hit with the
reference's intervals) and report which ancestor box of the rebuilt BVH's hit primitive culls it."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "raytracer-cuda_amd")]
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402

F = np.float32
scene = sys.argv[1]
rays = np.load(sys.argv[2])
hs = crt_amd.HostScene(assets.scene_files(scene))
e = hs.export("reference")
nodes = e["nodes"].reshape(-1, 2, 4)
iv = nodes.view(np.int32)
prims = e["prims"].reshape(-1, 3, 4)
rc = e["rank_code"]
n = len(nodes)


def box_test(i, o, inv, tcl):
    A, B = nodes[i]
    lo = np.array([A[0], A[1], A[2]], F)
    hi = np.array([A[3], B[0], B[1]], F)
    with np.errstate(all="ignore"):
        t0 = ((lo - o) * inv).astype(F)
        t1 = ((hi - o) * inv).astype(F)
    tmin = np.fmax(np.fmax(np.fmin(t0[0], t1[0]), np.fmin(t0[1], t1[1])), np.fmin(t0[2], t1[2]))
    tmax = np.fmin(np.fmin(np.fmax(t0[0], t1[0]), np.fmax(t0[1], t1[1])), np.fmax(t0[2], t1[2]))
    tmin = np.fmax(tmin, F(0.001))
    tmax = np.fmin(tmax, tcl)
    return not (tmax <= tmin), float(tmin), float(tmax), lo, hi


for k, r in enumerate(rays):
    o, d = r[0:3].astype(F), r[3:6].astype(F)
    ha, hb = int(r[6:7].view(np.int32)[0]), int(r[7:8].view(np.int32)[0])
    ta, tb = r[8], r[9]
    with np.errstate(all="ignore"):
        inv = (F(1) / d).astype(F)
    p = int(rc[hb]) & ~(1 << 30)
    leaf = [i for i in range(n) if iv[i, 1, 3] >= 0 and iv[i, 1, 3] < (1 << 30) and iv[i, 1, 3] <= p < iv[i, 1, 3] + iv[i, 1, 2]]
    print(f"ray {k}: o={o} d={d} ref hit rank {ha} t={ta}  rebuilt hit rank {hb} t={tb} (prim {p}, leaf {leaf})")
    if not leaf:
        continue
    L = leaf[0]
    anc = [j for j in range(L) if iv[j, 1, 3] < 0 and iv[j, 1, 2] > L]
    for j in anc + [L]:
        scene_level = iv[j, 1, 3] == -3
        ok, tmin, tmax, lo, hi = box_test(j, o, inv, F(np.inf) if scene_level or ha < 0 else F(ta))
        if not ok:
            ext = hi - lo
            print(f"   CULLED by node {j} ({'scene' if scene_level else 'mesh'} level{' leaf' if j == L else ''}): "
                  f"tmin={tmin!r} tmax={tmax!r} box lo={lo} hi={hi} extent={ext}")
    hp = o + F(tb) * d
    print("   hit point", hp)
