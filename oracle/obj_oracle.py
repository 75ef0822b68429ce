"""TEST INFRASTRUCTURE ONLY (the checker, never the product path).

An independent restatement, in Python with numpy float32 scalars, of how the
reference turns an OBJ file into triangles: SceneBuilder.loadModel
(SceneBuilder.java:144-183) calls Assimp (LWJGL-assimp 3.3.6, an Assimp 5.x
build) with aiProcess_Triangulate | JoinIdenticalVertices and
keeps every 3-index face.  The Assimp pieces restated from its published
sources, not from this repo's C++ (csrc/scene_build.cpp):

  fast_atoreal_move<float>   code/Common/fast_atof.h (integer digits -> float;
                             up to 15 fraction digits -> double x 10^-n -> float;
                             the two added in float; 'e' exponent x powf(10, e))
  ObjFileParser 'v' lines    the components are the tokens that start like a
                             number (ParsingUtils.h IsNumeric: digit, '-',
                             '+'; or nan / inf): 3, 4 (divided by w) or 6
                             (xyz + colour) read that many words in order;
                             any other count adds no vertex
  TriangulateProcess         quads fanned from the concave corner (acos angle
                             sum > pi, vectors normalised by multiplying with
                             the float reciprocal of the length), else corner 0;
                             larger polygons projected along the Newell
                             normal's largest axis and ear-clipped
                             (PolyTools.h GetArea2D / OnLeftSideOfLine2D /
                             PointInTriangle2D); no ear twice round -> the rest
                             of the polygon is dropped

Parity against a real Assimp run is unpinned: Assimp is not in this image and
the reference holds no triangulated fixtures.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32

_TABLE = [0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
          0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001,
          0.000000000000001]


def _digits(s: str, i: int, cap: int | None):
    """strtoul10_64: (value, next index, digits counted); overflow -> (0, i, 0);
    ValueError (Assimp throws) when no digit starts the string."""
    if not s[i:i + 1].isdigit():
        raise ValueError(f"no digits at {s[i:]!r}")
    j, v, n = i, 0, 0
    while j < len(s) and s[j] in "0123456789":
        nv = (v * 10 + ord(s[j]) - 48) & ((1 << 64) - 1)    # uint64 arithmetic, as Assimp's
        if nv < v:                                          # its overflow test: the value went down
            return 0, i, 0
        v = nv
        j += 1
        n += 1
        if cap is not None and n == cap:
            while j < len(s) and s[j] in "0123456789":
                j += 1
            return v, j, n
    return v, j, n


def fast_atof(tok: str) -> np.float32:
    """fast_atoreal_move<float>; ValueError where Assimp throws."""
    i = 0
    neg = tok[:1] == "-"
    if tok[:1] in "+-" and tok:
        i = 1
    low = tok[i:i + 3].lower()
    if low == "nan":
        return f32("nan")
    if low == "inf":
        return f32(-np.inf) if neg else f32(np.inf)
    c0 = tok[i:i + 1]
    c1 = tok[i + 1:i + 2]
    if not (c0.isdigit() or (c0 in (".", ",") and c0 and c1.isdigit())):
        raise ValueError(f"not a number: {tok!r}")
    f = f32(0.0)
    if c0 not in (".", ","):
        v, i, _ = _digits(tok, i, None)
        f = f32(v)
    if tok[i:i + 1] in (".", ",") and tok[i:i + 1] and tok[i + 1:i + 2].isdigit():
        v, i, n = _digits(tok, i + 1, 15)
        pl = float(v) * _TABLE[n]
        f = f32(f + f32(pl))
    elif tok[i:i + 1] == ".":
        i += 1
    if tok[i:i + 1] in ("e", "E") and tok[i:i + 1]:
        i += 1
        eneg = tok[i:i + 1] == "-"
        if tok[i:i + 1] in ("+", "-") and tok[i:i + 1]:
            i += 1
        v, i, _ = _digits(tok, i, None)
        e = f32(v)
        if eneg:
            e = -e
        f = f32(f * np.power(f32(10.0), e, dtype=np.float32))
    return f32(-f) if neg else f


def _norm(v):
    ln = np.sqrt(_dot3(v, v), dtype=np.float32)
    if ln == f32(0.0):
        return v
    inv = f32(f32(1.0) / ln)
    return (f32(v[0] * inv), f32(v[1] * inv), f32(v[2] * inv))


def _sub3(a, b):
    return (f32(a[0] - b[0]), f32(a[1] - b[1]), f32(a[2] - b[2]))


def _dot3(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def _area2d(v1, v2, v3) -> float:
    x1, y1, x2, y2, x3, y3 = (float(v1[0]), float(v1[1]), float(v2[0]), float(v2[1]), float(v3[0]), float(v3[1]))
    return 0.5 * (x1 * (y3 - y2) + x2 * (y1 - y3) + x3 * (y2 - y1))


def _dot2(a, b) -> float:
    return float(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])))


def _in_triangle(p0, p1, p2, pp) -> bool:
    v0 = (f32(p1[0] - p0[0]), f32(p1[1] - p0[1]))
    v1 = (f32(p2[0] - p0[0]), f32(p2[1] - p0[1]))
    v2 = (f32(pp[0] - p0[0]), f32(pp[1] - p0[1]))
    d00, d11, d01, d02, d12 = _dot2(v0, v0), _dot2(v1, v1), _dot2(v0, v1), _dot2(v0, v2), _dot2(v1, v2)
    den = d00 * d11 - d01 * d01
    if den == 0.0:
        return False
    inv = 1.0 / den
    u = (d11 * d02 - d01 * d12) * inv
    w = (d00 * d12 - d01 * d02) * inv
    return u > 0 and w > 0 and u + w < 1


def triangulate(verts, face):
    """aiProcess_Triangulate for one face (vertex indices): a list of triangles."""
    n = len(face)
    P = [tuple(f32(c) for c in verts[i]) for i in face]
    if n < 3:
        return []
    if n == 3:
        return [tuple(face)]
    if n == 4:
        start = 0
        for i in range(4):
            v = P[i]
            left = _norm(_sub3(P[(i + 3) % 4], v))
            diag = _norm(_sub3(P[(i + 2) % 4], v))
            right = _norm(_sub3(P[(i + 1) % 4], v))
            ang = f32(np.arccos(_dot3(left, diag), dtype=np.float32) + np.arccos(_dot3(right, diag), dtype=np.float32))
            if ang > f32(math.pi):
                start = i
                break
        q = face
        return [(q[start], q[(start + 1) % 4], q[(start + 2) % 4]), (q[start], q[(start + 2) % 4], q[(start + 3) % 4])]
    sxy = syz = szx = f32(0.0)
    for k in range(n):
        a, b, c = P[k], P[(k + 1) % n], P[(k + 2) % n]
        sxy = f32(sxy + f32(b[0] * f32(c[1] - a[1])))
        syz = f32(syz + f32(b[1] * f32(c[2] - a[2])))
        szx = f32(szx + f32(b[2] * f32(c[0] - a[0])))
    nx, ny, nz = syz, szx, sxy
    ax, ay, az = abs(nx), abs(ny), abs(nz)
    ac, bc, inv = 0, 1, nz
    if ax > ay:
        if ax > az:
            ac, bc, inv = 1, 2, nx
    elif ay > az:
        ac, bc, inv = 2, 0, ny
    if inv < 0:
        ac, bc = bc, ac
    tv = [(p[ac], p[bc]) for p in P]
    done = [False] * n
    out = []
    num, ear, prev, nxt = n, 0, n - 1, 0
    while num > 3:
        found = 0
        ear = nxt
        while True:
            nxt = ear + 1
            while True:
                if nxt >= n:
                    nxt = 0
                if not done[nxt]:
                    break
                nxt += 1
            if nxt < ear:
                found += 1
                if found == 2:
                    break
            p0, p1, p2 = tv[prev], tv[ear], tv[nxt]
            ok = _area2d(p0, p1, p2) <= 0               # OnLeftSideOfLine2D(p0, p2, p1) is false
            if ok:
                for q in tv:
                    if q != p1 and q != p2 and q != p0 and _in_triangle(p0, p1, p2, q):
                        ok = False
                        break
            if ok:
                break
            prev, ear = ear, nxt
        if found == 2:
            num = 0
            break
        out.append((prev, ear, nxt))
        done[ear] = True
        num -= 1
    if num > 0:
        rest = [k for k in range(n) if not done[k]]
        out.append(tuple(rest[:3]))
    return [tuple(face[k] for k in t) for t in out]


def load_obj(path: str) -> np.ndarray:
    """(n, 3, 3) float32 triangles in file order; ValueError where the import fails."""
    verts, tris = [], []
    with open(path, "r", errors="replace") as fh:
        for ln in fh:
            s = ln.lstrip(" \t")
            if s[:2] in ("v ", "v\t"):
                tok = s[2:].split()
                n = sum(1 for t in tok if t[0] in "0123456789+-" or t[:3].lower() in ("nan", "inf"))
                if n not in (3, 4, 6):
                    continue                             # Assimp reads no vertex from such a line
                c = [fast_atof(t) for t in tok[:n]]
                if n == 4:
                    if c[3] == 0:
                        raise ValueError("w = 0")
                    c = [f32(c[0] / c[3]), f32(c[1] / c[3]), f32(c[2] / c[3])]
                verts.append(tuple(c[:3]))
            elif s[:2] in ("f ", "f\t"):
                face = []
                for t in s[2:].split():
                    k = int(t.split("/")[0])
                    if k < 0:
                        k = len(verts) + k + 1
                    if not 1 <= k <= len(verts):
                        raise ValueError("bad face")
                    face.append(k - 1)
                tris.extend(triangulate(verts, face))
    out = np.array([[verts[i] for i in t] for t in tris], dtype=np.float32).reshape(-1, 3, 3)
    return out
