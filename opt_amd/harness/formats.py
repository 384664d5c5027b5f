"""Readers / writers for the example data formats.

* PNG: LodePNG::load returns RGBA8 (mLib ColorImageR8G8B8A8); PIL decodes the same pixels.
* `.imagedump`: SimpleBuffer (examples/shape_from_shading/src/SimpleBuffer.cpp:16-59):
  int32 width, height, channelCount, datatype (0 float, 1 uchar), then the pixels;
  float infinities clamped on load (clampInfinity: +inf -> FLT_MAX, -inf -> -10000).
* `.SFSSolverParameters`: TerraSolverParameters (TerraSolverParameters.h:7-45), a raw
  array of floats.
* `.constraints`: image_warping markers (examples/image_warping/src/main.cpp:7-30): a count
  then (x, y, targetX, targetY) integer quadruples.
* `.mrk`: mesh markers (examples/arap_mesh_deformation/src/main.cpp): a count then
  (x, y, z, radius, vertex index) per marker.
* `.ply` (binary little endian or ASCII; float xyz vertices, triangle faces) and `.off`
  (the meshes OpenMesh reads in the graph examples).
"""
from __future__ import annotations

import struct

import numpy as np


def read_png(path) -> np.ndarray:
    """RGBA8 pixels, shape (H, W, 4)."""
    from PIL import Image

    return np.array(Image.open(path).convert("RGBA"))


def write_png(path, rgba: np.ndarray) -> None:
    from PIL import Image

    Image.fromarray(np.ascontiguousarray(rgba.astype(np.uint8))).save(path)


# ---------------------------------------------------------------- SimpleBuffer
def read_imagedump(path, clamp_infinity: bool = True) -> np.ndarray:
    """(H, W) for one channel, (H, W, C) otherwise; float32 or uint8."""
    raw = open(path, "rb").read()
    w, h, ch, dt = struct.unpack("<4i", raw[:16])
    a = np.frombuffer(raw[16:16 + w * h * ch * (4 if dt == 0 else 1)],
                      dtype=np.float32 if dt == 0 else np.uint8).copy()
    if dt == 0 and clamp_infinity:
        a[np.isposinf(a)] = np.finfo(np.float32).max
        a[np.isneginf(a)] = -10000.0
    return a.reshape(h, w) if ch == 1 else a.reshape(h, w, ch)


def write_imagedump(path, a: np.ndarray) -> None:
    a = np.ascontiguousarray(a)
    if a.dtype not in (np.float32, np.uint8):
        a = a.astype(np.float32)
    h, w = a.shape[:2]
    ch = 1 if a.ndim == 2 else a.shape[2]
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", w, h, ch, 0 if a.dtype == np.float32 else 1))
        f.write(a.tobytes())


# ------------------------------------------------------- TerraSolverParameters
SFS_FIELDS = ["weightFitting", "weightRegularizer", "weightPrior", "weightShading", "weightShadingStart",
              "weightShadingIncrement", "weightBoundary", "fx", "fy", "ux", "uy"] + \
             ["deltaTransform_%d" % i for i in range(16)] + ["lighting_%d" % i for i in range(9)]


def read_sfs_parameters(path) -> dict:
    """The float fields of TerraSolverParameters (TerraSolverParameters.h:7-45) by name:
    7 weights, fx, fy, ux, uy, a float4x4 deltaTransform, 9 lighting coefficients."""
    p = np.fromfile(path, dtype=np.float32)
    out = {k: float(p[i]) for i, k in enumerate(SFS_FIELDS) if i < len(p)}
    out["lighting"] = p[27:36].astype(np.float32)
    out["raw"] = p
    return out


# ------------------------------------------------------------------ markers
def read_constraints(path) -> np.ndarray:
    """(n, 4) int32: x, y, target x, target y."""
    tok = open(path).read().split()
    n = int(tok[0])
    return np.array([int(float(t)) for t in tok[1:1 + 4 * n]], np.int32).reshape(n, 4)


def write_constraints(path, c: np.ndarray) -> None:
    with open(path, "w") as f:
        f.write("%d\n" % len(c))
        for row in np.asarray(c, np.int64):
            f.write(" ".join(str(int(v)) for v in row) + "\n")


def read_mrk(path):
    """(positions (n, 3) float32, radius (n,) float32, vertex index (n,) int32)."""
    tok = open(path).read().split()
    n = int(tok[0])
    m = np.array([float(t) for t in tok[1:1 + 5 * n]], np.float64).reshape(n, 5)
    return m[:, :3].astype(np.float32), m[:, 3].astype(np.float32), m[:, 4].astype(np.int32)


def write_mrk(path, pos, radius, idx) -> None:
    with open(path, "w") as f:
        f.write("%d\n" % len(idx))
        for p, r, i in zip(pos, radius, idx):
            f.write("%r %r %r %r %d\n" % (float(p[0]), float(p[1]), float(p[2]), float(r), int(i)))


# -------------------------------------------------------------------- meshes
_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def read_ply(path):
    """(vertices (n, 3) float32, faces (m, k) int32) of a binary-little-endian or ASCII PLY
    whose faces all have the same vertex count. Extra vertex properties are skipped."""
    raw = open(path, "rb").read()
    head, body = raw.split(b"end_header", 1)
    body = body[1:] if body[:1] == b"\n" else body[2:] if body[:2] == b"\r\n" else body
    lines = head.decode("ascii", "replace").splitlines()
    fmt = next(l.split()[1] for l in lines if l.startswith("format"))
    elems = []
    for l in lines:
        t = l.split()
        if not t:
            continue
        if t[0] == "element":
            elems.append([t[1], int(t[2]), []])
        elif t[0] == "property":
            elems[-1][2].append(t[1:])
    verts = faces = None
    if fmt == "ascii":
        toks = body.decode("ascii").split()
        pos = 0
        for name, n, props in elems:
            if name == "vertex":
                k = len(props)
                v = np.array(toks[pos:pos + n * k], np.float64).reshape(n, k)
                names = [p[-1] for p in props]
                verts = v[:, [names.index("x"), names.index("y"), names.index("z")]].astype(np.float32)
                pos += n * k
            elif name == "face":
                fl = []
                for _ in range(n):
                    c = int(toks[pos])
                    fl.append([int(x) for x in toks[pos + 1:pos + 1 + c]])
                    pos += 1 + c
                faces = np.array(fl, np.int32)
            else:
                pos += n * len(props)
        return verts, faces
    if fmt != "binary_little_endian":
        raise ValueError("unsupported PLY format " + fmt)
    off = 0
    for name, n, props in elems:
        if name == "face" or any(p[0] == "list" for p in props):
            lp = props[0]
            ct, it = _PLY_TYPES[lp[1]], _PLY_TYPES[lp[2]]
            c0 = int(np.frombuffer(body, ct, 1, off)[0])
            rec = np.dtype([("n", ct), ("v", "<" + it, (c0,))])
            fr = np.frombuffer(body, rec, n, off)
            if not np.all(fr["n"] == c0):
                raise ValueError("mixed polygon sizes are not supported")
            if name == "face":
                faces = fr["v"].astype(np.int32).copy()
            off += rec.itemsize * n
        else:
            rec = np.dtype([(p[-1], "<" + _PLY_TYPES[p[0]]) for p in props])
            arr = np.frombuffer(body, rec, n, off)
            if name == "vertex":
                verts = np.stack([arr["x"], arr["y"], arr["z"]], 1).astype(np.float32)
            off += rec.itemsize * n
    return verts, faces


def write_ply(path, verts, faces=None) -> None:
    """ASCII PLY (what the examples write for their results, e.g. savePLYMesh)."""
    verts = np.asarray(verts, np.float32).reshape(-1, 3)
    faces = np.zeros((0, 3), np.int32) if faces is None else np.asarray(faces, np.int32)
    with open(path, "w") as f:
        f.write("ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
                "property float z\nelement face %d\nproperty list uchar int vertex_indices\nend_header\n"
                % (len(verts), len(faces)))
        for v in verts:
            f.write("%r %r %r\n" % (float(v[0]), float(v[1]), float(v[2])))
        for fc in faces:
            f.write("%d %s\n" % (len(fc), " ".join(str(int(i)) for i in fc)))


def read_off(path):
    """(vertices (n, 3) float32, faces (m, k) int32) of an OFF file."""
    toks = [t for l in open(path) for t in l.split("#")[0].split()]
    if toks[0].upper() != "OFF":
        raise ValueError("not an OFF file")
    nv, nf = int(toks[1]), int(toks[2])
    pos = 4
    v = np.array(toks[pos:pos + 3 * nv], np.float64).reshape(nv, 3).astype(np.float32)
    pos += 3 * nv
    fl = []
    for _ in range(nf):
        c = int(toks[pos])
        fl.append([int(x) for x in toks[pos + 1:pos + 1 + c]])
        pos += 1 + c
    return v, np.array(fl, np.int32)


def read_obj(path):
    """(vertices (n, 3) float32, faces (m, 3) int32, 0-based) of a triangle OBJ file — the
    'v' and 'f' records OpenMesh's OBJ reader turns into a TriMesh in file order
    (examples/robust_nonrigid_alignment/src/main.cpp: createMesh); f entries may be
    v, v/vt, v/vt/vn or v//vn."""
    v, f = [], []
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            v.append([float(x) for x in t[1:4]])
        elif t[0] == "f":
            f.append([int(x.split("/")[0]) - 1 for x in t[1:4]])
    return np.array(v, np.float64).astype(np.float32), np.array(f, np.int32)


def read_ele(path):
    """Tetrahedra (n, 4) int32 of a TetGen .ele file (count, 4, attrs; then index + 4
    vertex ids per line), as main.cpp: getSourceTetIndices reads them."""
    tok = open(path).read().split()
    n = int(tok[0])
    a = np.array([int(x) for x in tok[3:3 + 5 * n]], np.int64).reshape(n, 5)
    return a[:, 1:].astype(np.int32)
