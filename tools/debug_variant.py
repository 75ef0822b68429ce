#!/usr/bin/env python3
"""Run one schedule variant a few times on a config, printing each launch's
time as it completes (for finding slow / stuck variants under a timeout).
Usage: python tools/debug_variant.py kernel=3,heavy_budget=128 [--config 3] [--bounces B]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--bounces", type=int, default=0)
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--nostats", action="store_true", help="launch the non-counting kernels")
    args = ap.parse_args()
    import torch
    import rtamd
    from rtamd import configs
    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, (args.bounces or cfg.max_bounces)
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    for kv in args.variant.split(","):
        k, v = kv.split("=")
        r.set_option(k, int(v))
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
    for i in range(args.launches):
        t0 = time.time()
        st = r.render_tile_device(cam, W, H, B, 0, 0, W, H, out.data_ptr(), None, None, stats=not args.nostats)
        if args.nostats:
            torch.cuda.synchronize()
            print(f"{args.variant} launch {i}: {1e3 * (time.time() - t0):.2f} ms wall (no stats)", flush=True)
            continue
        print(f"{args.variant} launch {i}: {1e3 * (time.time() - t0):.2f} ms wall, {st['ms']:.3f} ms events, "
              f"segments {st['segments']} visits {st['node_visits']} handoffs {st['handoffs']}", flush=True)
    r.close()


if __name__ == "__main__":
    main()
