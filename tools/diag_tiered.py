#!/usr/bin/env python3
"""Timeline of the tiered schedule (diagnostic build, option diag=1): tier 1's
per-wave span and trace_coop's per-path records (start, end, cooperative
rounds, segments).  Usage: python tools/diag_tiered.py [--opt k=v ...]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[])
    args = ap.parse_args()
    import torch
    import rtamd
    from rtamd import configs
    from rtamd._lib import check
    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    r.set_option("kernel", 3)
    for kv in args.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
    for _ in range(3):
        r.render_tile_device(cam, W, H, B, 0, 0, W, H, out.data_ptr(), None, None)
    r.set_option("diag", 1)
    st = r.render_tile_device(cam, W, H, B, 0, 0, W, H, out.data_ptr(), None, None, stats=True)
    torch.cuda.synchronize()
    L = rtamd.lib()
    n = C.c_size_t(0)
    check(L.rt_diag_copy(r._ctx, None, 0, C.byref(n)))
    buf = np.zeros(n.value, dtype=np.uint64)
    check(L.rt_diag_copy(r._ctx, buf.ctypes.data, n.value, C.byref(n)))
    tw_w, th_w = 8 << r.get_option("wave_tile"), 8 >> r.get_option("wave_tile")
    waves = ((W + 4 * tw_w - 1) // (4 * tw_w)) * ((H + th_w - 1) // th_w) * 4
    w = buf[:waves * 8].reshape(-1, 8).astype(np.int64)
    t0 = w[:, 0].min()
    k1_end = (w[:, 1].max() - t0) / 100.0
    print(f"tier 1: {waves} waves, span {k1_end:.1f} us; handoffs {st['handoffs']}; "
          f"waves ended by 50/90/99/100%: {[round(float(np.percentile(w[:, 1] - t0, q)) / 100, 1) for q in (50, 90, 99, 100)]} us")
    nr = int(st["handoffs"])
    p = buf[waves * 8: waves * 8 + 4 * nr].reshape(-1, 4).astype(np.int64)
    dur = (p[:, 1] - p[:, 0]) / 100.0
    chain = (p[:, 2] >> 16) & 0xFFFF
    rounds = (p[:, 2] & 0xFFFF) + chain
    print(f"  chain rounds: p50 {np.percentile(chain, 50):.0f} max {chain.max()}; "
          f"expansion rounds p50 {np.percentile(rounds - chain, 50):.0f}")
    walk = (p[:, 2] >> 32) / 100.0
    print(f"  time in walks: {walk.sum() / dur.sum():.3f} of path time")
    segs = p[:, 3] & 0xFFFF
    fb = (p[:, 3] >> 16) & 0xFFFF
    r1 = (p[:, 3] >> 32) & 0xFFFFF
    r1 = (r1 >> 16) + (r1 & 0xFFFF)
    t1 = ((p[:, 3] >> 52) & 0xFFF) / 100.0
    walk_all = (p[:, 2] >> 32) / 100.0
    rall = ((p[:, 2] >> 16) & 0xFFFF) + (p[:, 2] & 0xFFFF)
    later = segs_ = (p[:, 3] & 0xFFFF) > 1
    print(f"  first walk: {np.median(t1 / np.maximum(r1, 1)):.2f} us/round (p50 rounds {np.median(r1):.0f}); "
          f"later walks: {np.median((walk_all - t1)[later] / np.maximum(rall - r1, 1)[later]) if later.any() else 0:.2f} us/round "
          f"over {int(later.sum())} paths")
    print(f"  frontier overflows (node_step fallbacks): {int(fb.sum())} in {int((fb > 0).sum())} paths")
    print(f"tier 2: {nr} paths, first start {(p[:, 0].min() - t0) / 100:.1f} us, last end {(p[:, 1].max() - t0) / 100:.1f} us")
    for name, a in (("duration us", dur), ("rounds", rounds), ("segments", segs)):
        print(f"  {name}: p50 {np.percentile(a, 50):.1f} p90 {np.percentile(a, 90):.1f} "
              f"p99 {np.percentile(a, 99):.1f} max {a.max():.1f}")
    per = dur / np.maximum(rounds, 1)
    print(f"  us per round: p50 {np.percentile(per, 50):.2f} p90 {np.percentile(per, 90):.2f}")
    starts = np.sort((p[:, 0] - t0) / 100.0)
    print(f"  starts p0/p50/p100: {starts[0]:.1f} {np.percentile(starts, 50):.1f} {starts[-1]:.1f} us")
    r.close()


if __name__ == "__main__":
    main()
