#!/usr/bin/env python3
"""Lockstep load model of the one-node walk (analysis aid, not part of the
product).  From the oracle's exact visit sequences (orc_trace_pixel), replay
32x2 waves in lockstep (per bounce, step k = every walking lane's k-th visit)
and count, per wave step, what the loads need:
  - steps: wave steps (each issues the node loads: 2 vector loads)
  - uniform: steps where every walking lane is at the same node (a scalar
    load could serve the whole wave)
  - leafstep: steps where some walking lane is at a leaf (3 more loads)
  - topK: steps where every walking lane's node has depth < K levels
    (a K-level top tree kept in LDS could serve the whole wave)
  - lines: distinct 64-B node lines per step (mean)
Usage: lockstep_model.py [config] [tile-row stride]
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
    depth = np.zeros(n_nodes, np.int32)
    for i in range(n_nodes):
        if not is_leaf[i]:
            depth[nodes[i, 8]] = depth[i] + 1
            depth[nodes[i, 9]] = depth[i] + 1
    L = oracle_lib.lib()
    L.orc_trace_pixel.restype = C.c_int
    L.orc_trace_pixel.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    cam = cfg.camera()
    camb = np.frombuffer(cam.ubo_bytes(), np.uint8).copy()
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    buf = np.zeros(1 << 16, dtype=np.int32)
    Ks = (6, 8, 10, 12)
    tot = {"steps": 0, "uniform": 0, "leafstep": 0, "lines": 0, "lanes": 0, **{f"top{K}": 0 for K in Ks},
           "path_steps": 0}
    tiles = 0
    for ty in range(0, H // 2, stride):
        for tx in range(W // 32):
            segs = [[None] * 64 for _ in range(B)]
            for q in range(64):
                px, py = tx * 32 + (q & 31), ty * 2 + (q >> 5)
                cnt = L.orc_trace_pixel(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data,
                                        n.nbytes, camb.ctypes.data, W, H, B, px, py, buf.ctypes.data, buf.size)
                seq = buf[:cnt]
                starts = np.flatnonzero(seq < 0)
                for si, st in enumerate(starts[:B]):
                    en = starts[si + 1] if si + 1 < len(starts) else cnt
                    segs[si][q] = seq[st + 1:en]
            # bounce-decoupled lockstep: each lane walks its segments back to back
            tot["path_steps"] += max(sum(len(segs[bb][q]) for bb in range(B) if segs[bb][q] is not None)
                                     for q in range(64))
            for bb in range(B):
                lanes = [s for s in segs[bb] if s is not None and len(s) > 0]
                if not lanes:
                    continue
                mx = max(len(s) for s in lanes)
                for kk in range(mx):
                    cur = np.array([s[kk] for s in lanes if len(s) > kk])
                    tot["steps"] += 1
                    tot["lanes"] += len(cur)
                    u = np.unique(cur)
                    tot["uniform"] += len(u) == 1
                    tot["leafstep"] += bool(is_leaf[cur].any())
                    tot["lines"] += len(np.unique(cur // 2))
                    dmax = depth[cur].max()
                    for K in Ks:
                        tot[f"top{K}"] += dmax < K
            tiles += 1
    s = tot["steps"]
    print(f"config {k}: {tiles} 32x2 tiles (tile-row stride {stride}), {s} wave steps, "
          f"{tot['lanes'] / s:.1f} walking lanes/step, {tot['lines'] / s:.1f} node lines/step")
    print(f"  uniform steps {tot['uniform'] / s:.3f}, steps with a leaf {tot['leafstep'] / s:.3f}")
    print(f"  bounce-decoupled steps (max over lanes of the whole path's visits): {tot['path_steps'] / s:.3f}")
    for K in Ks:
        print(f"  all walking lanes within the top {K} levels ({2 ** K - 1} nodes): {tot[f'top{K}'] / s:.3f}")


if __name__ == "__main__":
    main()
