#!/usr/bin/env python3
"""PCIe-inclusive frame rate: synchronous rt_render vs pipelined rt_render_async
(--slots frames in flight, one slot and trace stream each, pinned host frames),
whole frames of a config.

Usage: python tools/pipeline_bench.py [--config 3] [--frames 60]
Prints one JSON line per mode: frames/s, ms/frame, Mrays/s including the
device->host copy of every frame.  (bench.py's `value` never includes PCIe.)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--slots", default="2,4,8", help="rt_render_async frames in flight (async_slots) to time")
    ap.add_argument("--copy-streams", default="1", help="rt option copy_streams values to time (1, 2 or 1,2)")
    ap.add_argument("--depth", default="1", help="host frames pending per slot (1, 2 or 1,2): the caller waits "
                                                  "for its oldest frame once slots x depth are pending")
    args = ap.parse_args()
    import numpy as np
    import rtamd          # sets GPU_MAX_HW_QUEUES, then loads torch's HIP runtime first
    from rtamd import configs
    from rtamd.engine import PinnedFrame

    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    segs = r.render(cam, W, H, B, stats=True)[2]["segments"]
    pageable = np.empty((H, W, 4), np.uint8)
    slots = [int(x) for x in args.slots.split(",")]
    depths = [int(x) for x in args.depth.split(",")]
    frames = [PinnedFrame(H, W) for _ in range(max(slots) * max(depths))]

    def sync_run(n):
        for _ in range(n):
            r.render(cam, W, H, B)

    def async_run(n, d, depth=1):
        r.set_option("async_slots", d)
        pending = []
        for k in range(n):
            pending.append(r.render_async(cam, W, H, B, frames[k % (d * depth)]))
            if len(pending) == d * depth:
                r.wait(pending.pop(0))
        for t in pending:
            r.wait(t)

    modes = [("sync rt_render (pageable copy, fence per frame)", sync_run)]
    def with_copies(c, d, depth):
        def run(n):
            r.set_option("copy_streams", c)
            async_run(n, d, depth)
        return run
    modes += [(f"rt_render_async, {d} in flight, pinned, {c} copy stream(s), {d * depth} host frames pending",
               with_copies(c, d, depth))
              for d in slots for c in [int(x) for x in args.copy_streams.split(",")] for depth in depths]
    for name, fn in modes:
        fn(20)
        t0 = time.perf_counter()
        fn(args.frames)
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": name, "config": cfg.name, "frames": args.frames,
                          "fps": round(args.frames / dt, 1), "ms_per_frame": round(dt / args.frames * 1e3, 3),
                          "mrays_s_incl_pcie": round(segs * args.frames / dt / 1e6, 1)}), flush=True)
    assert np.array_equal(frames[(args.frames - 1) % (slots[-1] * depths[-1])].array, r.render(cam, W, H, B)[0])
    del pageable
    r.close()
    for f in frames:
        f.close()


if __name__ == "__main__":
    main()
