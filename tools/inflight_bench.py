#!/usr/bin/env python3
"""Frames in flight: K whole frames of a config launched round-robin on S HIP
streams (separate output buffers), so frame k+1's waves can fill the CUs that
frame k's serial tail leaves idle.  Prints one JSON line per S.

Usage: python tools/inflight_bench.py [--config 3] [--frames 40] [--streams 1,2,3,4]
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
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import rtamd  # first: sets GPU_MAX_HW_QUEUES before torch loads HIP
    import torch
    from rtamd import configs
    from rtamd._lib import check

    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    L = rtamd.lib()
    segs = r.render(cam, W, H, B, stats=True)[2]["segments"]
    ref = r.render(cam, W, H, B)[0]
    smax = max(int(s) for s in args.streams.split(","))
    streams = [torch.cuda.Stream() for _ in range(smax)]
    outs = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0") for _ in range(smax)]

    def run(S, n):
        for k in range(n):
            j = k % S
            check(L.rt_render_bands_device(r._ctx, C.byref(cam.ubo), W, H, B, H, 1, 0, outs[j].data_ptr(), None,
                                           streams[j].cuda_stream, None))

    for S in (int(s) for s in args.streams.split(",")):
        best = None
        for _ in range(args.rounds):
            run(S, 2 * S)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(S, args.frames)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        ok = all((o.cpu().numpy() == ref).all() for o in outs[:S])
        print(json.dumps({"streams": S, "config": cfg.name, "frames": args.frames,
                          "ms_per_frame": round(best / args.frames * 1e3, 4),
                          "mrays_s": round(segs * args.frames / best / 1e6, 1), "frames_identical": bool(ok)}),
              flush=True)
    r.close()


if __name__ == "__main__":
    main()
