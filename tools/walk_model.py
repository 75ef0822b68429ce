#!/usr/bin/env python3
"""Round-trip model of per-lane walk variants (analysis aid, not part of the
product): from the oracle's exact preorder visit sequence of every segment
(orc_trace_pixel), count the dependent memory round trips a lane needs when
one round trip brings the records of a set S of nodes, and the lockstep cost
of 32x2 waves (per bounce the wave runs max-over-lanes round trips).

  A  S = {i}                          the current walk (one node per trip)
  B  S = {i, i+1}                     the node and its preorder successor
  C  S = {i, skip(i)}                 the node and its miss successor
  D  S = {i, i+1, skip(i)}
  E  S = {i, i+1, skip(i), skip(i+1)}
  Wk S = [i, i+k)                     k consecutive preorder nodes
Visits are strictly increasing in preorder, so a trip consumes visits while
the next one is in S.  Usage: walk_model.py [config] [tile-row stride]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    from rtamd import configs
    from oracle import oracle_lib
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    cfg = configs.get(k)
    b = cfg.build()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    nodes = np.frombuffer(b.flat_bvh_data.tobytes(), dtype=np.int32).reshape(-1, 12)
    n_nodes = nodes.shape[0]
    is_leaf = nodes[:, 9] < 0
    # skip(i): first node after i's subtree (leaf: i+1; internal: skip(right))
    skip = np.zeros(n_nodes, np.int64)
    for i in range(n_nodes - 1, -1, -1):
        skip[i] = i + 1 if is_leaf[i] else skip[nodes[i, 9]]
    skip = skip.tolist()
    L = oracle_lib.lib()
    L.orc_trace_pixel.restype = C.c_int
    L.orc_trace_pixel.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    cam = cfg.camera()
    camb = np.frombuffer(cam.ubo_bytes(), np.uint8).copy()
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    buf = np.zeros(1 << 16, dtype=np.int32)

    def sets(i):
        return {
            "A": (i,),
            "B": (i, i + 1),
            "C": (i, skip[i]),
            "D": (i, i + 1, skip[i]),
            "E": (i, i + 1, skip[i], skip[i + 1] if i + 1 < n_nodes else i + 1),
        }

    def trips(vis, policy):
        t, j = 0, 0
        while j < len(vis):
            i = vis[j]
            t += 1
            j += 1
            if policy[0] == "W":
                w = int(policy[1:])
                while j < len(vis) and vis[j] < i + w:
                    j += 1
                continue
            s = set(sets(i)[policy])
            # consume the visits in S; a visit in S brings no new records
            while j < len(vis) and vis[j] in s:
                j += 1
        return t

    policies = ("A", "B", "C", "D", "E", "W2", "W4", "W8")
    lock = {p: 0 for p in policies}
    lane = {p: 0 for p in policies}
    tiles = 0
    for ty in range(0, H // 2, stride):
        for tx in range(W // 32):
            per = {p: np.zeros((64, B), np.int64) for p in policies}
            for q in range(64):
                px, py = tx * 32 + (q & 31), ty * 2 + (q >> 5)
                cnt = L.orc_trace_pixel(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data,
                                        n.nbytes, camb.ctypes.data, W, H, B, px, py, buf.ctypes.data, buf.size)
                seq = buf[:cnt].tolist()
                seg = -1
                cur = []
                segs = []
                for x in seq:
                    if x < 0:
                        cur = []
                        segs.append(cur)
                    else:
                        cur.append(x)
                for sidx, vis in enumerate(segs[:B]):
                    for p in policies:
                        per[p][q, sidx] = trips(vis, p)
            for p in policies:
                lock[p] += int(per[p].max(axis=0).sum())
                lane[p] += int(per[p].sum())
            tiles += 1
    print(f"config {k}: {tiles} 32x2 tiles (tile-row stride {stride})")
    for p in policies:
        print(f"  {p:3s} lane trips {lane[p]:>10d} ({lane[p] / lane['A']:.3f})   "
              f"lockstep wave trips {lock[p]:>9d} ({lock[p] / lock['A']:.3f})")


if __name__ == "__main__":
    main()
