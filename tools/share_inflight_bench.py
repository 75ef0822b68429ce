#!/usr/bin/env python3
"""Strong-scaling model on one GPU, with frames in flight.

bench.py --partition bands at N > 1 gives rank r the 16-row bands b with
b mod N = r and keeps D frames in flight per rank (step k traces on stream
k mod D).  This script times that trace loop of one rank alone on one GPU
(no gather): K frames of rank r's share, frame k on stream k mod D, and
reports ms per frame.  max over r of that is the per-frame trace rate an
N-GPU run can reach before its gather and host overheads.  Also reports the
host time of issuing one launch (the C-ABI call).

Usage: python tools/share_inflight_bench.py [--config 3] [--ranks 2,4,8]
           [--inflight auto|1,2,4,...] [--frames 200] [--concurrent D|1]
Run it as bench.py runs (GPU_MAX_HW_QUEUES=16: importing bench sets it).
Prints one JSON line per (N, rank, D).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]
import bench  # noqa: E402,F401  (sets GPU_MAX_HW_QUEUES before the GPU is touched)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--which", default="all", help="all | 0 (rank 0 only) | comma list of ranks")
    ap.add_argument("--inflight", default="auto", help="comma list, or auto = bench.py's default_inflight(N)")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--band", type=int, default=16)
    ap.add_argument("--concurrent", default="D", help="concurrent_launches: an int, or 'D' (= frames in flight, "
                                                      "bench.py's setting)")
    ap.add_argument("--set", default="", help="options name=value,... applied before timing")
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
    for kv in filter(None, args.set.split(",")):
        k, v = kv.split("=")
        r.set_option(k, int(v))
    L = rtamd.lib()
    from bench import default_inflight
    Ns = [int(x) for x in args.ranks.split(",")]
    Ds = [int(x) for x in args.inflight.split(",")] if args.inflight != "auto" else None
    n_streams = max(Ds or [default_inflight(n) for n in Ns])
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    for N in Ns:
        ranks = range(N) if args.which == "all" else [int(x) for x in args.which.split(",")]
        for rank in ranks:
            rows = L.rt_band_rows(H, args.band, N, rank)
            bufs = [torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda:0") for _ in range(n_streams)]
            for D in (Ds or [default_inflight(N)]):
                conc = D if args.concurrent == "D" else int(args.concurrent)
                r.set_option("concurrent_launches", conc)

                def go(k):
                    check(L.rt_render_bands_device(r._ctx, C.byref(cam.ubo), W, H, B, args.band, N, rank,
                                                   bufs[k % D].data_ptr(), None,
                                                   streams[k % D].cuda_stream, None))
                go(0)                        # learns this share's order
                torch.cuda.synchronize()
                for k in range(20):
                    go(k)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                host = 0.0
                for k in range(args.frames):
                    h0 = time.perf_counter()
                    go(k)
                    host += time.perf_counter() - h0
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(json.dumps({"config": args.config, "N": N, "rank": rank, "inflight": D,
                                  "concurrent_launches": conc, "ms_per_frame": round(dt * 1e3 / args.frames, 4),
                                  "host_us_per_launch": round(host * 1e6 / args.frames, 1),
                                  "heavy_pixels_used": r.get_option("heavy_pixels_used"),
                                  }), flush=True)


if __name__ == "__main__":
    main()
