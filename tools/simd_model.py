#!/usr/bin/env python3
"""SIMD-efficiency model of traversal schedules, from the oracle's per-pixel,
per-bounce node-visit profile (analysis aid, not part of the product).

For a wave of 64 lanes, a schedule's cost is the number of loop iterations
the wave executes; efficiency = useful node visits / (64 x iterations)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def profile(cfg_k=3, row_step=2, scale=1):
    from rtamd import configs
    from oracle import oracle_lib
    cfg = configs.get(cfg_k)
    b = cfg.build()
    W, H = cfg.width // scale, cfg.height // scale
    cam = configs.Camera.default(W, H)
    L = oracle_lib.lib()
    L.orc_render_profile.argtypes = L.orc_render.argtypes + [C.c_void_p]
    rows = (H + row_step - 1) // row_step
    prof = np.zeros((rows, W, cfg.max_bounces), dtype=np.uint32)
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    camb = np.frombuffer(cam.ubo_bytes(), np.uint8).copy()
    c = oracle_lib.Counts()
    rc = L.orc_render_profile(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data, n.nbytes,
                              camb.ctypes.data, W, H, cfg.max_bounces, 0, 0, W, H, row_step, None, None,
                              C.byref(c), 0, prof.ctypes.data)
    assert rc == 0
    return prof & 0xFFFFF, prof >> 20, c.as_dict()


def tiles8(a):
    """(rows, W, B) -> (n_waves, 64, B) grouping 8x8 pixel tiles."""
    r, w, bb = a.shape
    r8, w8 = r // 8 * 8, w // 8 * 8
    a = a[:r8, :w8].reshape(r8 // 8, 8, w8 // 8, 8, bb).transpose(0, 2, 1, 3, 4)
    return a.reshape(-1, 64, bb)


if __name__ == "__main__":
    visits, tris, cnt = profile(int(sys.argv[1]) if len(sys.argv) > 1 else 3, 1, 2)
    print(cnt, "visits/seg", cnt["node_visits"] / cnt["segments"])
    t = tiles8(visits.astype(np.int64))
    useful = t.sum()
    # (1) lockstep per bounce: each bounce costs max over lanes
    it1 = t.max(axis=1).sum()
    print(f"per-pixel lockstep (current kernel): eff {useful / (64 * it1):.3f}")
    # (2) lockstep over the whole path (lanes chain their bounces): cost = max over lanes of total
    it2 = t.sum(axis=2).max(axis=1).sum()
    print(f"per-lane chained bounces, no refill:  eff {useful / (64 * it2):.3f}")
    # (3) ideal refill (persistent lanes pull new paths): bounded by total work / 64
    print(f"ideal refill: eff ~1.0; iterations saved vs (1): {it1 / (useful / 64):.2f}x")
