"""Oracle OBJ/MTL loader — TEST INFRASTRUCTURE ONLY (see crt_oracle.c header).

Restates, independently of the product's C++ loader:

* ``SceneManager::loadObject`` (reference ``CudaRayTracer/src/SceneManager.h:198-329``):
  MTL classification (:220-247), per-file MeshData with the
  ``vertices.resize(attrib.vertices.size())`` 3x-slot quirk (:253), last-write-wins
  vertex slots (:300), face material clamp against the *global* material count
  (:259-265), and the re-normalisation of *all* meshes loaded so far after each
  file (:307-325);
* ``SceneManager::initMeshes`` (:100-196): concatenation, per-mesh offsets and
  ``materialIDOffset`` = unique face-material ids of the previous mesh only
  (:143-145, :177);
* tinyobjloader v1.0.x (third-party, version unpinned by the reference;
  identified by the 6-argument ``LoadObj`` call at :215): ``tryParseDouble`` float
  parsing, ``fixIndex`` negative indices, polygon fan triangulation, per-face
  material ids, ``LoadMtl`` defaults (dissolve 1, ior 1, shininess 1,
  roughness 0).  Parity against tinyobjloader itself is UNPINNED (not in image).
"""
from __future__ import annotations

import math
import os
import struct
from dataclasses import dataclass, field

import numpy as np

_POW_LUT = [1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001]


def try_parse_double(s: str):
    """tinyobjloader v1.0 tryParseDouble; returns float (double) or None."""
    n = len(s)
    i = 0
    sign = '+'
    if i < n and s[i] in '+-':
        sign = s[i]
        i += 1
    elif i < n and s[i].isdigit():
        pass
    else:
        return None
    mant = 0.0
    read = 0
    while i < n and '0' <= s[i] <= '9':
        mant *= 10
        mant += ord(s[i]) - 48
        i += 1
        read += 1
    if read == 0:
        return None
    exponent = 0
    if i < n:
        if s[i] == '.':
            i += 1
            read = 1
            while i < n and '0' <= s[i] <= '9':
                lut = _POW_LUT[read] if read < len(_POW_LUT) else math.pow(10.0, -read)
                mant += (ord(s[i]) - 48) * lut
                read += 1
                i += 1
        if i < n and s[i] in 'eE':
            i += 1
            esign = '+'
            if i < n and s[i] in '+-':
                esign = s[i]
                i += 1
            elif not (i < n and s[i].isdigit()):
                return None
            read = 0
            while i < n and '0' <= s[i] <= '9':
                exponent = exponent * 10 + (ord(s[i]) - 48)
                i += 1
                read += 1
            if read == 0:
                return None
            if esign == '-':
                exponent = -exponent
    val = math.ldexp(mant * math.pow(5.0, exponent), exponent) if exponent else mant
    return (1 if sign == '+' else -1) * val


def f32(x: float) -> float:
    return struct.unpack('f', struct.pack('f', x))[0]


def parse_real(tok: str, default: float = 0.0) -> float:
    v = try_parse_double(tok) if tok is not None else None
    return f32(default if v is None else v)


@dataclass
class Material:
    name: str = ""
    diffuse: tuple = (0.0, 0.0, 0.0)
    specular: tuple = (0.0, 0.0, 0.0)
    emission: tuple = (0.0, 0.0, 0.0)
    dissolve: float = 1.0
    ior: float = 1.0
    shininess: float = 1.0
    roughness: float = 0.0


def load_mtl(path: str):
    mats, cur = [], None
    with open(path, 'r') as fh:
        for line in fh:
            t = line.strip().split()
            if not t or t[0].startswith('#'):
                continue
            k, a = t[0], t[1:]
            def r3():
                return tuple(parse_real(a[i] if i < len(a) else None) for i in range(3))
            if k == 'newmtl':
                if cur is not None and cur.name:
                    mats.append(cur)
                cur = Material(name=" ".join(a))
            elif cur is None:
                continue
            elif k == 'Kd':
                cur.diffuse = r3()
            elif k == 'Ks':
                cur.specular = r3()
            elif k == 'Ke':
                cur.emission = r3()
            elif k == 'd':
                cur.dissolve = parse_real(a[0] if a else None)
            elif k == 'Tr':
                cur.dissolve = f32(1.0 - parse_real(a[0] if a else None))
            elif k == 'Ni':
                cur.ior = parse_real(a[0] if a else None)
            elif k == 'Ns':
                cur.shininess = parse_real(a[0] if a else None)
            elif k == 'Pr':
                cur.roughness = parse_real(a[0] if a else None)
    if cur is not None and cur.name:
        mats.append(cur)
    return mats


def load_obj_tinyobj(path: str, base_dir: str):
    """Returns (attrib_vertices float32 [3*nv], faces list of (tri vertex_index triple, mat id), materials)."""
    verts = []
    materials, mat_map = [], {}
    cur_mat = -1
    tri_idx, tri_mat = [], []
    with open(path, 'r') as fh:
        for line in fh:
            s = line.strip()
            if not s or s[0] == '#':
                continue
            t = s.split()
            k = t[0]
            if k == 'v':
                for i in range(3):
                    verts.append(parse_real(t[1 + i] if 1 + i < len(t) else None))
            elif k == 'f':
                nv = len(verts) // 3
                face = []
                for tok in t[1:]:
                    vi = int(tok.split('/')[0])
                    if vi > 0:
                        face.append(vi - 1)
                    elif vi < 0:
                        face.append(nv + vi)
                    else:
                        raise ValueError("zero index")
                if len(face) < 3:
                    continue
                i0, i2 = face[0], face[1]
                for kk in range(2, len(face)):
                    i1, i2 = i2, face[kk]
                    tri_idx.extend((i0, i1, i2))
                    tri_mat.append(cur_mat)
            elif k == 'usemtl':
                name = s[7:] if len(s) > 7 else ""
                cur_mat = mat_map.get(name, -1)
            elif k == 'mtllib':
                for fn in t[1:]:
                    mpath = os.path.join(base_dir, fn)
                    if os.path.exists(mpath):
                        for m in load_mtl(mpath):
                            mat_map.setdefault(m.name, len(materials))
                            materials.append(m)
                        break
    return np.asarray(verts, dtype=np.float32), np.asarray(tri_idx, dtype=np.int64), \
        np.asarray(tri_mat, dtype=np.int64), materials


MT_LAMBERTIAN, MT_METAL, MT_DIELECTRIC, MT_LIGHT = 0, 1, 2, 3


@dataclass
class LoadedScene:
    positions: np.ndarray          # float32 [total_slots, 3]
    indices: np.ndarray            # uint32
    facemat: np.ndarray            # int32
    mesh_info: np.ndarray          # uint32 [n_mesh, 6]
    matdata: np.ndarray            # float32 [n_mat, 9]
    meshes: list = field(default_factory=list)


def load_scene(files) -> LoadedScene:
    scene_mats = []      # list of 9-float rows
    mesh_list = []       # per file: [positions float32 (slots,3), indices, facemat]
    for fn in files:
        last = max(fn.rfind('/'), fn.rfind('\\'))
        base_dir = fn[:last + 1] if last >= 0 else "./"
        attrib_v, tri_idx, tri_mat, mats = load_obj_tinyobj(fn, base_dir)
        for m in mats:                                                       # :222-247
            if m.emission[0] > 0 or m.emission[1] > 0 or m.emission[2] > 0:
                mt = MT_LIGHT
            elif m.dissolve < 1.0:
                mt = MT_DIELECTRIC
            elif m.specular[0] > 0:
                mt = MT_METAL
            else:
                mt = MT_LAMBERTIAN
            r = 0.0
            if mt == MT_METAL:
                r = m.roughness if m.roughness > 0 else f32(math.sqrt(f32(2.0 / f32(m.shininess + 2.0))))
            ior = m.ior if mt == MT_DIELECTRIC else 1.0
            scene_mats.append([float(mt), *m.diffuse, *m.emission, r, ior])
        n_slots = len(attrib_v)                                               # :253 resize(attrib.vertices.size())
        pos = np.zeros((n_slots, 3), dtype=np.float32)
        av = attrib_v.reshape(-1, 3)
        if len(tri_idx):
            pos[tri_idx] = av[tri_idx]                                        # :273-300 last write wins (same value)
        fm = tri_mat.copy()
        fm[(fm < 0) | (fm >= len(scene_mats))] = 0                            # :259-265
        mesh_list.append([pos, tri_idx.astype(np.uint32), fm.astype(np.int32)])
        # :307-325 normalise all meshes loaded so far (float32 Vec3 arithmetic)
        allpos = np.concatenate([m[0] for m in mesh_list]) if mesh_list else np.zeros((0, 3), np.float32)
        mn = np.full(3, np.finfo(np.float32).max, dtype=np.float32)
        mx = np.full(3, np.finfo(np.float32).min, dtype=np.float32)
        if len(allpos):
            mn = np.minimum(mn, allpos.min(axis=0))
            mx = np.maximum(mx, allpos.max(axis=0))
        center = ((mn + mx) * np.float32(0.5)).astype(np.float32)
        ext = (mx - mn).astype(np.float32)
        maxc = np.float32(max(ext[0], max(ext[1], ext[2])))
        scale = np.float32(np.float32(0.6) / maxc)
        for m in mesh_list:
            m[0] = ((m[0] - center) * scale).astype(np.float32)
    # initMeshes :125-149
    positions, indices, facemat, info = [], [], [], []
    prev_unique = 0
    vo = io = fo = 0
    for i, (pos, idx, fm) in enumerate(mesh_list):
        info.append([vo, len(pos), io, len(idx), fo, 0 if i == 0 else prev_unique])
        prev_unique = len(set(fm.tolist()))
        positions.append(pos); indices.append(idx); facemat.append(fm)
        vo += len(pos); io += len(idx); fo += len(fm)
    cat = lambda xs, dt, shp: np.concatenate(xs).astype(dt) if xs else np.zeros(shp, dt)
    return LoadedScene(
        positions=cat(positions, np.float32, (0, 3)),
        indices=cat(indices, np.uint32, (0,)),
        facemat=cat(facemat, np.int32, (0,)),
        mesh_info=np.asarray(info, dtype=np.uint32).reshape(-1, 6),
        matdata=np.asarray(scene_mats, dtype=np.float32).reshape(-1, 9),
        meshes=mesh_list,
    )
