#!/usr/bin/env python3
"""Round-trip model of cooperative (one ray per wave) walk schemes on the
heaviest pixels of a config (analysis aid, not part of the product).

From the oracle's exact visit sequence of each segment (orc_trace_pixel):
  lockstep  one dependent load per visit (the per-lane walk)
  window64  the current coop_walk: 64 contiguous preorder nodes per round trip
  frontierK wide DFS: each round tests the first K entries (in preorder) of the
            frontier of subtrees still to visit; a hit internal node is replaced
            by its two children.  Lower bound: only the reference's visited
            nodes are counted (speculation at a stale closest_t can add a few).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT, os.path.dirname(os.path.abspath(__file__))]


def segments(seq):
    segs, cur = [], None
    for v in seq:
        if v < 0:
            cur = []
            segs.append(cur)
        else:
            cur.append(v)
    return segs


def windows(vis, w=64):
    n, k, i = 0, 0, 0
    while i < len(vis):
        n = vis[i]
        k += 1
        while i < len(vis) and vis[i] < n + w:
            i += 1
    return k


def main():
    from rtamd import configs
    from oracle import oracle_lib
    from simd_model import profile
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    npix = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    cfg = configs.get(k)
    b = cfg.build()
    W, H = cfg.width, cfg.height
    nodes = np.frombuffer(b.flat_bvh_data.tobytes(), dtype=np.int32).reshape(-1, 12)
    left = nodes[:, 8]
    right = nodes[:, 9]
    is_leaf = right < 0
    # heaviest pixels from a profile of every 4th row
    visits, _, _ = profile(k, 4, 1)
    tot = visits.astype(np.int64).sum(axis=2)
    order = np.argsort(tot.ravel())[::-1][:npix]
    L = oracle_lib.lib()
    L.orc_trace_pixel.restype = C.c_int
    L.orc_trace_pixel.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    cam = configs.Camera.default(W, H)
    camb = np.frombuffer(cam.ubo_bytes(), np.uint8).copy()
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    buf = np.zeros(1 << 20, dtype=np.int32)
    Ks = (64, 128, 256)
    agg = {"visits": 0, "window64": 0, **{f"frontier{K}": 0 for K in Ks}, "depth": 0}
    for idx in order:
        py, px = divmod(int(idx), W)
        py *= 4
        cnt = L.orc_trace_pixel(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data, n.nbytes,
                                camb.ctypes.data, W, H, cfg.max_bounces, px, py, buf.ctypes.data, buf.size)
        assert cnt > 0
        row = {"visits": 0, "window64": 0, **{f"frontier{K}": 0 for K in Ks}, "depth": 0}
        for vis in segments(buf[:cnt].tolist()):
            if not vis:
                continue
            vs = set(vis)
            row["visits"] += len(vis)
            row["window64"] += windows(vis)
            for K in Ks:
                # frontier of subtree roots in preorder; expand a visited hit internal node
                front = [0]
                rounds = 0
                while front:
                    rounds += 1
                    take, front = front[:K], front[K:]
                    new = []
                    for x in take:
                        if not is_leaf[x] and (x + 1) in vs:      # hit internal: both children visited
                            new += [int(left[x]), int(right[x])]
                    front = sorted(new + front)
                row[f"frontier{K}"] += rounds
        for key in row:
            agg[key] += row[key]
        print(px, py, row, flush=True)
    print("total", agg)


if __name__ == "__main__":
    main()
