#!/usr/bin/env python3
"""Secondary-ray grouping model (analysis aid, not part of the product).

From the numpy restatement's per-ray visit counts (oracle/shader_np.py
on_segment hook), for every bounce compare the lockstep steps of 64-ray waves
grouped as 32x2 pixel tiles (the megakernel) with waves of rays sorted by a
coherence key (direction octant, then the Morton code of the origin; or the
direction's cube-map cell, then origin), and with the ideal (rays sorted by
their own walk length).  Usage: sort_model.py [config] [first row] [rows]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def morton3(q):
    """Interleave three 10-bit ints."""
    def spread(x):
        x = x.astype(np.uint64) & 0x3FF
        x = (x | (x << 16)) & 0x30000FF
        x = (x | (x << 8)) & 0x300F00F
        x = (x | (x << 4)) & 0x30C30C3
        x = (x | (x << 2)) & 0x9249249
        return x
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def lockstep(visits, groups):
    """Total wave steps when rays are packed 64 per wave in the given order."""
    v = visits[groups]
    pad = (-len(v)) % 64
    v = np.concatenate([v, np.zeros(pad, v.dtype)]).reshape(-1, 64)
    return int(v.max(axis=1).sum()), float(v.sum() / (64 * max(1, v.max(axis=1).sum())))


def main():
    from rtamd import configs
    from oracle import shader_np
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    y0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ny = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    cfg = configs.get(k)
    b = cfg.build()
    W, H = cfg.width, cfg.height
    rows = np.arange(y0, y0 + ny)
    lo = np.frombuffer(b.model_vertex_data.tobytes(), np.float32).reshape(-1, 3, 4)[:, :, :3].reshape(-1, 3)
    box_lo, box_hi = lo.min(axis=0), lo.max(axis=0)
    rec = []

    def on_segment(bb, act, o, d, vis):
        rec.append((bb, act.copy(), o.copy(), d.copy(), vis.copy()))

    shader_np.render(b.model_vertex_data, b.model_material_data, b.flat_bvh_data, cfg.camera().ubo_bytes(), W, H,
                     cfg.max_bounces, rows=rows, on_segment=on_segment)
    tot = {"tile": 0, "octant_morton": 0, "cube_morton": 0, "coarse_stable": 0, "coarse_random": 0, "ideal": 0}
    for bb, act, o, d, vis in rec:
        # 32x2 tiles: pixel index p -> (row, col) in the rows block
        r, c = act // W, act % W
        tile = (r // 2) * (W // 32 + 1) + c // 32
        order_tile = np.lexsort(((r % 2) * 32 + c % 32, tile))
        # waves = tiles: group by tile id, pad each tile to 64
        ts, first = np.unique(tile[order_tile], return_index=True)
        steps_tile = 0
        for g in np.split(vis[order_tile], first[1:]):
            steps_tile += int(g.max())
        q = np.clip(((o - box_lo) / np.maximum(box_hi - box_lo, 1e-6) * 1023).astype(np.int64), 0, 1023)
        mo = morton3(q)
        octant = ((d[:, 0] < 0).astype(np.uint64) << 2) | ((d[:, 1] < 0).astype(np.uint64) << 1) | (d[:, 2] < 0)
        s1, u1 = lockstep(vis, np.lexsort((mo, octant)))
        ax = np.argmax(np.abs(d), axis=1)
        sg = (d[np.arange(len(d)), ax] < 0).astype(np.int64)
        uv = np.delete(d, ax[:, None] == np.arange(3)[None, :], axis=None).reshape(-1, 2) if False else None
        face = ax * 2 + sg
        a1 = np.take_along_axis(d, ((ax + 1) % 3)[:, None], 1)[:, 0] / np.abs(d[np.arange(len(d)), ax])
        a2 = np.take_along_axis(d, ((ax + 2) % 3)[:, None], 1)[:, 0] / np.abs(d[np.arange(len(d)), ax])
        cell = (face * 64 + np.clip(((a1 + 1) * 4).astype(np.int64), 0, 7) * 8 + np.clip(((a2 + 1) * 4).astype(np.int64), 0, 7))
        s2, u2 = lockstep(vis, np.lexsort((mo, cell)))
        coarse = (mo >> np.uint64(24)).astype(np.int64)
        key = cell * 64 + coarse
        s4, u4 = lockstep(vis, np.lexsort((np.arange(len(key)), key)))          # stable: pixel order in a bucket
        rng = np.random.default_rng(1)
        s5, u5 = lockstep(vis, np.lexsort((rng.permutation(len(key)), key)))    # atomics: random order in a bucket
        s3, u3 = lockstep(vis, np.argsort(vis))
        tot["tile"] += steps_tile
        tot["octant_morton"] += s1
        tot["cube_morton"] += s2
        tot["coarse_stable"] += s4
        tot["coarse_random"] += s5
        tot["ideal"] += s3
        print(f"bounce {bb}: {len(act)} rays, {int(vis.sum())} visits; wave steps: tiles {steps_tile} "
              f"(util {vis.sum() / (64 * steps_tile):.3f}), octant+Morton {s1} ({u1:.3f}), "
              f"cube cell+Morton {s2} ({u2:.3f}), cell+coarse6 stable {s4} ({u4:.3f}), "
              f"cell+coarse6 random {s5} ({u5:.3f}), ideal {s3} ({u3:.3f})", flush=True)
    print("total", tot)


if __name__ == "__main__":
    main()
