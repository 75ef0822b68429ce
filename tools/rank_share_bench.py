#!/usr/bin/env python3
"""Strong-scaling model on one GPU: the time of one rank's share of a frame.

bench.py --partition bands (the N > 1 default) gives rank r of N the 16-row
bands b with b mod N = r.  On one GPU this script times every rank's share
alone (rt_render_bands_device, band stride N, offset r, the default schedule
with its learned order and automatic heavy tiles), so max over r of the share
time is the per-frame trace time an N-GPU run would see, before the gather.
Prints one JSON line per N.

Usage: python tools/rank_share_bench.py [--config 3] [--ranks 1,2,4,8] [--frames 50]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--band", type=int, default=16)
    ap.add_argument("--set", default="", help="options name=value,... applied before timing")
    args = ap.parse_args()
    import torch
    import rtamd
    from rtamd import configs
    from rtamd._lib import Stats, check

    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    for kv in filter(None, args.set.split(",")):
        k, v = kv.split("=")
        r.set_option(k, int(v))
    L = rtamd.lib()
    s = torch.cuda.Stream()
    full_segs = None
    for N in (int(x) for x in args.ranks.split(",")):
        band = H if N == 1 else args.band
        per = []
        for rank in range(N):
            rows = L.rt_band_rows(H, band, N, rank)
            out = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda:0")

            def go(st=None):
                check(L.rt_render_bands_device(r._ctx, C.byref(cam.ubo), W, H, B, band, N, rank, out.data_ptr(),
                                               None, s.cuda_stream, C.byref(st) if st is not None else None))

            st = Stats()
            go(st)
            for _ in range(3):          # learn the order, capture the graph
                go()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.frames):
                go()
            e1.record(s)
            torch.cuda.synchronize()
            per.append({"rank": rank, "ms": round(e0.elapsed_time(e1) / args.frames, 4),
                        "segments": st.as_dict()["segments"], "heavy_tiles": r.get_option("heavy_tiles_used")})
        segs = sum(p["segments"] for p in per)
        if N == 1:
            full_segs = segs
        worst = max(p["ms"] for p in per)
        print(json.dumps({"config": cfg.name, "ranks": N, "max_share_ms": worst,
                          "mean_share_ms": round(sum(p["ms"] for p in per) / N, 4),
                          "model_mrays_s": round(segs / (worst * 1e-3) / 1e6, 1), "segments": segs,
                          "per_rank": per}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
