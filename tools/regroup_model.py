#!/usr/bin/env python3
"""Segment-boundary regrouping model (analysis aid, not part of the product;
VERDICT r02 "next" item 5).

The lockstep walk keeps a wave on its 64 pixels for their whole paths, so in
later segments many lanes are idle (their path ended in the sky) and the
wave's step count per segment is its longest lane's.  Regrouping at segment
boundaries: a workgroup of M adjacent 8x8 tiles (M waves) compacts its live
rays (in pixel order, so neighbours stay together) into ceil(live / 64)
waves before every segment; surplus waves exit (the live count never grows),
and the block's waves meet at a barrier at every segment boundary, so a
segment holds ceil(live / 64) wave slots for its slowest compacted wave.

From the oracle's exact visit sequences (orc_trace_pixel) this counts, on a
sample of blocks of config 3:
  base   wave-slot steps of one-wave workgroups (today): sum over waves and
         segments of the segment's longest lane
  regroup  sum over blocks and segments of ceil(live / 64) x the longest
         compacted wave's steps in that segment
  bound  the same compaction with no barrier cost (each compacted wave
         frees its slot when its own longest lane ends): an upper bound on
         what regrouping at segment boundaries can save
and the lockstep lane utilisation (walking lanes per wave step) of both.
The VERDICT bar for building it: >= 1.3x fewer wave-slot steps.

Usage: python tools/regroup_model.py [--config 3] [--block 2x2] [--stride 6]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--block", default="2x2,4x4", help="blocks of tiles (tiles across x down), comma list")
    ap.add_argument("--stride", type=int, default=6, help="sample every stride-th block row")
    args = ap.parse_args()
    from rtamd import configs
    from oracle import oracle_lib
    cfg = configs.get(args.config)
    b = cfg.build()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    L = oracle_lib.lib()
    L.orc_trace_pixel.restype = C.c_int
    L.orc_trace_pixel.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    camb = np.frombuffer(cfg.camera().ubo_bytes(), np.uint8).copy()
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    buf = np.zeros(1 << 16, dtype=np.int32)

    def seg_lengths(px, py):
        """Walk steps of each segment of pixel (px, py)'s path."""
        cnt = L.orc_trace_pixel(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data, n.nbytes,
                                camb.ctypes.data, W, H, B, px, py, buf.ctypes.data, buf.size)
        seq = buf[:cnt]
        starts = np.flatnonzero(seq < 0)
        out = []
        for si, st in enumerate(starts[:B]):
            en = starts[si + 1] if si + 1 < len(starts) else cnt
            out.append(int(max(1, en - st - 1)))
        return out

    results = []
    for spec in args.block.split(","):
        bx, by = (int(x) for x in spec.split("x"))
        base = regroup = bound = base_lane = reg_lane = 0
        blocks = 0
        for BY in range(0, H // (8 * by), args.stride):
            for BX in range(W // (8 * bx)):
                # the block's pixels in pixel order within each tile, tiles row-major
                tiles = []
                for ty in range(by):
                    for tx in range(bx):
                        x0, y0 = (BX * bx + tx) * 8, (BY * by + ty) * 8
                        tiles.append([seg_lengths(x0 + (q & 7), y0 + (q >> 3)) for q in range(64)])
                for s in range(B):
                    # base: every tile wave on its own
                    for t in tiles:
                        ls = [p[s] for p in t if len(p) > s]
                        if ls:
                            base += max(ls)
                            base_lane += sum(ls)
                    # regroup: the block's live rays of segment s, compacted in order
                    live = [p[s] for t in tiles for p in t if len(p) > s]
                    if not live:
                        continue
                    waves = [live[i:i + 64] for i in range(0, len(live), 64)]
                    regroup += len(waves) * max(max(w) for w in waves)
                    bound += sum(max(w) for w in waves)
                    reg_lane += sum(live)
                blocks += 1
        r = {"config": args.config, "block": spec, "blocks_sampled": blocks,
             "base_wave_slot_steps": base, "regroup_wave_slot_steps": regroup,
             "ratio": round(base / regroup, 3),
             "bound_wave_slot_steps": bound, "bound_ratio": round(base / bound, 3),
             "base_lanes_per_step": round(base_lane / base, 1),
             "regroup_lanes_per_step": round(reg_lane / regroup, 1)}
        print(json.dumps(r), flush=True)
        results.append(r)


if __name__ == "__main__":
    main()
