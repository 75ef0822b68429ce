#!/usr/bin/env python3
"""Interleaved A/B timing of trace schedules in ONE process (median of rounds).

Usage: python tools/ab_bench.py [--config 3] [--rounds 7] [--iters 10]
       [--variant kernel=1,shade_min=16 --variant kernel=0 ...]
Each variant is a comma list of rt_set_option name=value pairs.  Prints one
JSON line per variant: median / min kernel ms and Mrays/s.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--bounces", type=int, default=0, help="override the config's max_bounces")
    ap.add_argument("--first", default="", help="options applied before the counting pass")
    args = ap.parse_args()
    variants = args.variant or ["kernel=0", "kernel=1,shade_min=8", "kernel=1,shade_min=16",
                                "kernel=1,shade_min=32"]
    import torch
    import rtamd
    from rtamd import configs
    from rtamd._lib import Stats, check

    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, (args.bounces or cfg.max_bounces)
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    L = rtamd.lib()
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)

    def log(*x):
        print(*x, file=sys.stderr, flush=True)

    def launch(stats=False):
        s = Stats()
        check(L.rt_render_bands_device(r._ctx, C.byref(cam.ubo), W, H, B, H, 1, 0, out.data_ptr(), None,
                                       stream.cuda_stream, C.byref(s) if stats else None))
        return s

    def apply(v):
        for kv in v.split(","):
            k, val = kv.split("=")
            r.set_option(k, int(val))

    if args.first:
        apply(args.first)
    log("counting pass")
    segs = launch(stats=True).segments
    log("segments", segs)
    times = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            log("variant", v)
            apply(v)
            for _ in range(2):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                launch()
            e1.record(stream)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters)
        apply("kernel=0,shade_min=16,blocks_per_cu=0,wave_tile=2,heavy_budget=256,prio_after=0,coop_lanes=2,walk=2,coop_walk=0,block_waves=1,heavy_first=1,heavy_tiles=-1,heavy_stream=1,learn_cost=1,heavy_factor=150")
    for v in variants:
        med = statistics.median(times[v])
        print(json.dumps({"variant": v, "config": cfg.name, "median_ms": round(med, 4),
                          "min_ms": round(min(times[v]), 4), "bounces": B, "mrays_s": round(segs / med / 1e3, 1)}))
    r.close()


if __name__ == "__main__":
    main()
