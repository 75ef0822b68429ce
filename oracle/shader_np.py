"""shader_np.py — vectorised numpy restatement of shaders/compute_dynamic_ray.comp.

TEST INFRASTRUCTURE ONLY (tests/ imports it to cross-check oracle/rt_oracle.c).

Written independently of rt_oracle.c: all rays of a frame advance together,
each with its own int stack[64] (compute_dynamic_ray.comp:185-210), in numpy
float32 arithmetic (one IEEE operation per ufunc call, no fused multiply-add),
under the same float contract the C oracle states (normalize = v/sqrt(dot),
dot = (x*x'+y*y')+z*z', min/max = fmin/fmax, reflect = I - N*(2*dot(N,I)),
RGBA8 = clamp + round-half-even).  Small frames only (pure numpy, seconds).
"""
from __future__ import annotations

import numpy as np

F = np.float32
T_MIN = F(0.001)                 # :42
T_MAX = F(10000.0)               # :43
MAX_REJECT_TRIPLES = 65536       # see rt_oracle.c header


def _dot(ax, ay, az, bx, by, bz):
    return (ax * bx + ay * by) + az * bz


def _normalize(x, y, z):
    ln = np.sqrt(_dot(x, y, z, x, y, z))
    return x / ln, y / ln, z / ln


def _cross(ax, ay, az, bx, by, bz):
    return ay * bz - az * by, az * bx - ax * bz, ax * by - ay * bx


def pcg(v: np.ndarray) -> np.ndarray:                         # :52-56
    v = v.astype(np.uint32)
    s = v * np.uint32(747796405) + np.uint32(2891336453)
    w = ((s >> ((s >> np.uint32(28)) + np.uint32(4))) ^ s) * np.uint32(277803737)
    return (w >> np.uint32(22)) ^ w


def random_float(seed: np.ndarray):                           # :58-61
    seed = pcg(seed)
    return seed, seed.astype(np.float32) / F(4294967296.0)


def random_in_unit_sphere(seed: np.ndarray):                  # :63-70
    seed = pcg(pcg(pcg(seed)))                                # the discarded temp draws
    n = seed.shape[0]
    px = np.zeros(n, F); py = np.zeros(n, F); pz = np.zeros(n, F)
    todo = np.ones(n, bool)
    for _ in range(MAX_REJECT_TRIPLES):
        if not todo.any():
            break
        s = seed[todo]
        s, a = random_float(s)
        s, b = random_float(s)
        s, c = random_float(s)
        x = a * F(2.0) - F(1.0); y = b * F(2.0) - F(1.0); z = c * F(2.0) - F(1.0)
        ok = _dot(x, y, z, x, y, z) < F(1.0)
        seed[todo] = s
        idx = np.nonzero(todo)[0]
        acc = idx[ok]
        px[acc], py[acc], pz[acc] = x[ok], y[ok], z[ok]
        todo[acc] = False
    return seed, px, py, pz


def render(vertices, materials, nodes, camera_ubo: bytes, width: int, height: int, max_bounces: int,
           rows=None, ext: int = 0, accum=None, spheres=None, on_segment=None):
    """Returns (rgba[len(rows), W, 4], radiance[len(rows), W, 3], counts dict).
    ext / accum / spheres: the non-reference extensions of oracle/rt_oracle.h
    (ORC_EXT_*), restated independently; accum float32[len(rows), W, 3] is
    updated in place; spheres float32[n, 8] = (centre.xyz, radius, albedo.rgb,
    type), hit-tested after the BVH walk with ext bit 8.
    on_segment (analysis aid, tools/): called after every bounce's walks with
    (b, pixel indices, ray origins (n,3), directions (n,3), node visits (n,));
    it changes nothing."""
    V = np.frombuffer(bytes(vertices), np.float32)
    V = V[: (V.size // 12) * 12].reshape(-1, 3, 4)[:, :, :3]    # (the empty scene's 1-float dummy: none)
    M = np.frombuffer(bytes(materials), np.float32)
    M = M[: (M.size // 4) * 4].reshape(-1, 4)
    S = np.asarray(spheres if (spheres is not None and ext & 8) else np.zeros((0, 8)), F).reshape(-1, 8)
    nb = np.frombuffer(bytes(nodes), np.uint8)
    nb = nb[: (nb.size // 48) * 48].reshape(-1, 48)
    BMIN = nb[:, 0:12].copy().view(np.float32).reshape(-1, 3)
    BMAX = nb[:, 16:28].copy().view(np.float32).reshape(-1, 3)
    DATA = nb[:, 32:36].copy().view(np.int32).reshape(-1)
    COUNT = nb[:, 36:40].copy().view(np.int32).reshape(-1)
    cam = np.frombuffer(bytes(camera_ubo), np.float32)[:16].reshape(4, 4)[:, :3]
    frame_count, sky_enabled = (int(x) for x in np.frombuffer(bytes(camera_ubo), np.int32)[16:18])
    org, llc, hor, ver = cam[0], cam[1], cam[2], cam[3]

    rows = np.arange(height) if rows is None else np.asarray(rows)
    ys, xs = np.meshgrid(rows, np.arange(width), indexing="ij")
    ys = ys.reshape(-1).astype(np.int64); xs = xs.reshape(-1).astype(np.int64)
    R = xs.size
    seed = (ys * width + xs).astype(np.uint32)                               # :164
    if ext & 4:                                           # extension: a new sample per frame
        seed = ((seed.astype(np.uint64) + np.uint64(frame_count % 2**32) * np.uint64(width * height))
                % np.uint64(2**32)).astype(np.uint32)
    seed, ru = random_float(seed)
    seed, rv = random_float(seed)
    u = (xs.astype(F) + ru) / F(width)                                        # :167
    v = ((height - 1 - ys).astype(F) + rv) / F(height)                        # :168
    dx = ((llc[0] + hor[0] * u) + ver[0] * v) - org[0]
    dy = ((llc[1] + hor[1] * u) + ver[1] * v) - org[1]
    dz = ((llc[2] + hor[2] * u) + ver[2] * v) - org[2]
    dx, dy, dz = _normalize(dx, dy, dz)                                      # :173
    ox = np.full(R, org[0], F); oy = np.full(R, org[1], F); oz = np.full(R, org[2], F)

    fin = np.zeros((R, 3), F)
    att = np.ones((R, 3), F)
    alive = np.ones(R, bool)
    counts = {"pixels": R, "segments": 0, "node_visits": 0, "tri_tests": 0, "mat_reads": 0}
    n_nodes = BMIN.shape[0]

    for b in range(max_bounces):                                              # :179
        act = np.nonzero(alive)[0]
        if act.size == 0:
            break
        counts["segments"] += act.size
        A = act.size
        closest = np.full(A, T_MAX, F)
        hit = np.full(A, -1, np.int64)
        nx = np.zeros(A, F); ny = np.zeros(A, F); nz = np.zeros(A, F)
        rox, roy, roz = ox[act], oy[act], oz[act]
        rdx, rdy, rdz = dx[act], dy[act], dz[act]
        stack = np.zeros((A, 64), np.int64)
        sp = np.zeros(A, np.int64)
        ray_visits = np.zeros(A, np.int64) if on_segment is not None else None
        if n_nodes > 0:
            sp[:] = 1
        while True:
            w = np.nonzero(sp > 0)[0]
            if w.size == 0:
                break
            sp[w] -= 1
            node = stack[w, sp[w]]
            counts["node_visits"] += w.size
            if ray_visits is not None:
                ray_visits[w] += 1
            with np.errstate(divide="ignore"):                                 # 1/0 = inf, as on the GPU
                ix = F(1.0) / rdx[w]; iy = F(1.0) / rdy[w]; iz = F(1.0) / rdz[w]    # hit_aabb :88-103
            t0x = (BMIN[node, 0] - rox[w]) * ix; t1x = (BMAX[node, 0] - rox[w]) * ix
            t0y = (BMIN[node, 1] - roy[w]) * iy; t1y = (BMAX[node, 1] - roy[w]) * iy
            t0z = (BMIN[node, 2] - roz[w]) * iz; t1z = (BMAX[node, 2] - roz[w]) * iz
            te = np.fmax(np.fmax(np.fmin(t0x, t1x), np.fmin(t0y, t1y)), np.fmin(t0z, t1z))
            tx = np.fmin(np.fmin(np.fmax(t0x, t1x), np.fmax(t0y, t1y)), np.fmax(t0z, t1z))
            hb = (tx > te) & (tx > T_MIN) & (te < closest[w])
            leaf = hb & (COUNT[node] < 0)
            inner = hb & (COUNT[node] >= 0)
            # internal: push right, then left
            wi = w[inner]; ni = node[inner]
            stack[wi, sp[wi]] = COUNT[ni]; sp[wi] += 1
            stack[wi, sp[wi]] = DATA[ni]; sp[wi] += 1
            # leaf: hit_triangle :105-129
            wl = w[leaf]
            if wl.size:
                counts["tri_tests"] += wl.size
                tri = -(DATA[node[leaf]].astype(np.int64) + 1)
                v0 = V[tri, 0]; v1 = V[tri, 1]; v2 = V[tri, 2]
                e1x = v1[:, 0] - v0[:, 0]; e1y = v1[:, 1] - v0[:, 1]; e1z = v1[:, 2] - v0[:, 2]
                e2x = v2[:, 0] - v0[:, 0]; e2y = v2[:, 1] - v0[:, 1]; e2z = v2[:, 2] - v0[:, 2]
                pxx, pxy, pxz = _cross(rdx[wl], rdy[wl], rdz[wl], e2x, e2y, e2z)
                det = _dot(e1x, e1y, e1z, pxx, pxy, pxz)
                ok = ~((det > F(-0.00001)) & (det < F(0.00001)))
                with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                    inv_det = F(1.0) / det
                    sx = rox[wl] - v0[:, 0]; sy = roy[wl] - v0[:, 1]; sz = roz[wl] - v0[:, 2]
                    uu = inv_det * _dot(sx, sy, sz, pxx, pxy, pxz)
                    ok &= ~((uu < F(0.0)) | (uu > F(1.0)))
                    qx, qy, qz = _cross(sx, sy, sz, e1x, e1y, e1z)
                    vv = inv_det * _dot(rdx[wl], rdy[wl], rdz[wl], qx, qy, qz)
                    ok &= ~((vv < F(0.0)) | ((uu + vv) > F(1.0)))
                    t = inv_det * _dot(e2x, e2y, e2z, qx, qy, qz)
                ok &= (t > T_MIN) & (t < closest[wl])
                # a ray tests at most one triangle per step, so updates do not collide
                g = wl[ok]
                closest[g] = t[ok]
                hit[g] = tri[ok]
                cnx, cny, cnz = _cross(e1x[ok], e1y[ok], e1z[ok], e2x[ok], e2y[ok], e2z[ok])
                cnx, cny, cnz = _normalize(cnx, cny, cnz)
                flip = _dot(rdx[g], rdy[g], rdz[g], cnx, cny, cnz) > F(0.0)
                nx[g] = np.where(flip, -cnx, cnx); ny[g] = np.where(flip, -cny, cny); nz[g] = np.where(flip, -cnz, cnz)
            if (sp > 62).any():
                raise RuntimeError("stack overflow (reference int stack[64])")

        # extension: spheres after the BVH walk, in index order; hit = -2 - k
        for k in range(S.shape[0]):
            cx, cy, cz, rad_k = S[k, 0], S[k, 1], S[k, 2], S[k, 3]
            ocx = rox - cx; ocy = roy - cy; ocz = roz - cz
            qa = _dot(rdx, rdy, rdz, rdx, rdy, rdz)
            hb_ = _dot(ocx, ocy, ocz, rdx, rdy, rdz)
            qc = _dot(ocx, ocy, ocz, ocx, ocy, ocz) - rad_k * rad_k
            with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
                disc = hb_ * hb_ - qa * qc
                sq = np.sqrt(np.where(disc >= F(0.0), disc, F(0.0)))
                r1 = (-hb_ - sq) / qa
                r2 = (-hb_ + sq) / qa
            in1 = (r1 > T_MIN) & (r1 < closest)
            in2 = (r2 > T_MIN) & (r2 < closest)
            root = np.where(in1, r1, r2)
            ok = (disc >= F(0.0)) & (in1 | in2)
            g = np.nonzero(ok)[0]
            if g.size == 0:
                continue
            closest[g] = root[g]
            hit[g] = -2 - k
            px_ = rox[g] + rdx[g] * root[g]; py_ = roy[g] + rdy[g] * root[g]; pz_ = roz[g] + rdz[g] * root[g]
            snx = (px_ - cx) / rad_k; sny = (py_ - cy) / rad_k; snz = (pz_ - cz) / rad_k
            flip = _dot(rdx[g], rdy[g], rdz[g], snx, sny, snz) > F(0.0)
            nx[g] = np.where(flip, -snx, snx); ny[g] = np.where(flip, -sny, sny); nz[g] = np.where(flip, -snz, snz)

        if on_segment is not None:
            on_segment(b, act, np.stack([rox, roy, roz], 1), np.stack([rdx, rdy, rdz], 1), ray_visits)
        gh = hit != -1
        # miss: final = att * sky, path ends (:224-227)
        ms = act[~gh]
        if ms.size:
            ux, uy, uz = _normalize(dx[ms], dy[ms], dz[ms])
            t = F(0.5) * (uy + F(1.0))
            omt = F(1.0) - t
            sky = np.stack([omt * F(1.0) + t * F(0.5), omt * F(1.0) + t * F(0.7), omt * F(1.0) + t * F(1.0)], 1)
            fin[ms] = att[ms] * sky
            if (ext & 1) and sky_enabled == 0:            # extension: sky off, a miss is black
                fin[ms] = F(0.0)
            alive[ms] = False
        hs = np.nonzero(gh)[0]
        if hs.size:
            counts["mat_reads"] += hs.size
            ga = act[hs]
            hpx = rox[hs] + rdx[hs] * closest[hs]; hpy = roy[hs] + rdy[hs] * closest[hs]
            hpz = roz[hs] + rdz[hs] * closest[hs]
            hh = hit[hs]
            mat = np.where((hh >= 0)[:, None], M[np.maximum(hh, 0)] if M.shape[0] else F(0.0),
                           S[np.maximum(-2 - hh, 0), 4:8] if S.shape[0] else F(0.0)).astype(F)
            typ = mat[:, 3]
            hnx, hny, hnz = nx[hs], ny[hs], nz[hs]
            ndx = dx[ga].copy(); ndy = dy[ga].copy(); ndz = dz[ga].copy()
            scattered = np.zeros(hs.size, bool)
            lam = typ == F(0.0)                                                # :137-143
            if lam.any():
                sd = seed[ga[lam]]
                sd, px, py, pz = random_in_unit_sphere(sd)
                seed[ga[lam]] = sd
                rx, ry, rz = _normalize(px, py, pz)
                sx = hnx[lam] + rx; sy = hny[lam] + ry; sz = hnz[lam] + rz
                small = np.sqrt(_dot(sx, sy, sz, sx, sy, sz)) < F(0.0001)
                sx = np.where(small, hnx[lam], sx); sy = np.where(small, hny[lam], sy); sz = np.where(small, hnz[lam], sz)
                ndx[lam], ndy[lam], ndz[lam] = _normalize(sx, sy, sz)
                scattered[lam] = True
            met = (typ == F(1.0)) | (typ == F(2.0))                            # :145-151
            if met.any():
                fuzz = np.where(typ[met] == F(2.0), F(0.3), F(0.0)).astype(F)
                ix, iy, iz = _normalize(dx[ga[met]], dy[ga[met]], dz[ga[met]])
                k = F(2.0) * _dot(hnx[met], hny[met], hnz[met], ix, iy, iz)
                rx = ix - hnx[met] * k; ry = iy - hny[met] * k; rz = iz - hnz[met] * k
                sd = seed[ga[met]]
                sd, px, py, pz = random_in_unit_sphere(sd)
                seed[ga[met]] = sd
                qx, qy, qz = _normalize(rx + px * fuzz, ry + py * fuzz, rz + pz * fuzz)
                ndx[met], ndy[met], ndz[met] = qx, qy, qz
                scattered[met] = _dot(qx, qy, qz, hnx[met], hny[met], hnz[met]) > F(0.0)
            if ext & 2:                                   # extension: type 3 emits its albedo
                em = typ == F(3.0)
                fin[ga[em]] = att[ga[em]] * mat[em, :3]
            ok = scattered
            att[ga[ok]] = att[ga[ok]] * mat[ok, :3]
            ox[ga[ok]] = hpx[ok]; oy[ga[ok]] = hpy[ok]; oz[ga[ok]] = hpz[ok]
            dx[ga[ok]] = ndx[ok]; dy[ga[ok]] = ndy[ok]; dz[ga[ok]] = ndz[ok]
            dead = ga[~ok]                                                      # absorbed: black (:220-222)
            att[dead] = F(0.0)
            alive[dead] = False
            if b == max_bounces - 1:                                            # :229-231
                fin[ga[ok]] = F(0.0)
                alive[ga[ok]] = False

    if ext & 4:                                           # extension: running sum, sqrt(mean)
        acc = accum.reshape(-1, 3)
        acc[:] = fin if frame_count == 0 else acc + fin
        fin = acc / F(frame_count + 1)
    rad = np.sqrt(fin).astype(F)                                               # :235
    q = np.where(rad > F(0.0), np.where(rad < F(1.0), np.rint(rad * F(255.0)), F(255.0)), F(0.0)).astype(np.uint8)
    rgba = np.concatenate([q, np.full((R, 1), 255, np.uint8)], 1)
    n_rows = len(rows)
    return rgba.reshape(n_rows, width, 4), rad.reshape(n_rows, width, 3), counts
