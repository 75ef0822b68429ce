#!/usr/bin/env python3
"""Rank 0 of an N-GPU bench.py run, emulated on one GPU (analysis aid).

bench.py --partition bands at N > 1: rank r traces its 16-row bands of every
frame, D frames in flight (step k on stream k mod D); every G = D frames the
batch is gathered to rank 0 over RCCL and assembled there by one
index_select.  Rank 0 does the most device work: its share of the traces,
the receive of the whole batch and the assembly.  This script runs exactly
that on one GPU: rank 0's share of each frame, and per batch an RCCL gather
(world size 1, so a device copy) of the volume rank 0 receives at N (N x G
packed shares) followed by the assembly of the G frames, with bench.py's
ring of 2G slots and its waits.  Partition blocks (bench.py's default):
rank 0 traces its piece of frame k (rtamd.dist.block_layout, root_share) in
place, and the receive of the other N - 1 pieces of the batch's frames is
emulated by one RCCL gather at world size 1 of that volume, with no assembly
(an RCCL receive is a copy kernel from its staging buffer into the
destination).  --rank r > 0 (blocks only) emulates a sending rank instead: its
piece, and a copy of the volume it sends.  The other ranks' rows are
whatever the buffers hold: the frames are not checked.  Reports ms per frame with and
without the exchange, and with the exchange streams at normal or high
priority (bench.py --exchange-priority).

Usage: python tools/rank0_exchange_bench.py [--ranks 2,4,8] [--frames 240]
Prints one JSON line per (N, exchange, priority).
"""
import argparse
import ctypes as C
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before the GPU is touched)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--frames", type=int, default=240)
    ap.add_argument("--band", type=int, default=16)
    ap.add_argument("--arms", default="bands:0:0,bands:1:1,blocks:0:0,blocks:1:1",
                    help="partition:exchange:priority[:root_share] (root_share: blocks only, default 1)")
    ap.add_argument("--ring", type=int, default=2, help="batches of slots in the ring (bench.py --ring)")
    ap.add_argument("--rank", type=int, default=0, help="blocks: the rank emulated (0 receives, others send)")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import configs
    from rtamd._lib import check
    from rtamd.dist import BatchPlan, block_layout, block_sizes

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    L = rtamd.lib()
    arms = [(a.split(":")[0], int(a.split(":")[1]), int(a.split(":")[2]),
             float(a.split(":")[3]) if len(a.split(":")) > 3 else 1.0) for a in args.arms.split(",")]
    pgs = {}
    for prio in sorted({a[2] for a in arms}):
        from torch.distributed import ProcessGroupNCCL
        opts = ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = bool(prio)
        if not dist.is_initialized():
            store = dist.TCPStore("127.0.0.1", _port(), 1, True)
            dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev, pg_options=opts)
            pgs[prio] = dist.group.WORLD
        else:
            pgs[prio] = dist.new_group([0], pg_options=opts)
    for N in [int(x) for x in args.ranks.split(",")]:
        D = bench.default_inflight(N)
        G = D
        r.set_option("concurrent_launches", D)
        plan = BatchPlan(H, args.band, N, G, rotate=False)
        src = torch.as_tensor(plan.src, device=dev)
        rows = L.rt_band_rows(H, args.band, N, 0)
        # per half: [N * G, max_rows, W, 4]; rank 0's frame f of the batch is block f
        R = args.ring
        slots = torch.zeros((R, N * G, plan.max_rows, W, 4), dtype=torch.uint8, device=dev)
        streams = [torch.cuda.Stream(dev) for _ in range(D)]
        fring = torch.zeros((R * G, H, W, 4), dtype=torch.uint8, device=dev)
        for mode, exch, prio, share in arms:
            main_s = torch.cuda.Stream(dev, priority=-1 if prio else 0)
            gathered = [None] * R
            sizes = block_sizes(H, N, share)
            me = args.rank if mode == "blocks" else 0
            # rows this rank moves per frame: rank 0 receives every other piece, a sender sends its own
            moved = (H - sizes[0]) if me == 0 else sizes[me]
            other = torch.zeros((G, max(1, moved), W, 4), dtype=torch.uint8, device=dev)
            landing = torch.empty_like(other)

            def trace(k):
                s = streams[k % D]
                half = (k // G) % R
                if k % G == 0 and gathered[half] is not None:
                    for t in streams:
                        t.wait_event(gathered[half])
                if mode == "blocks":
                    y0, y1 = block_layout(H, N, k, share)[me]
                    if y1 > y0:
                        check(L.rt_render_tile_device(r._ctx, C.byref(cam.ubo), W, H, B, 0, y0, W, y1 - y0,
                                                      fring[k % (R * G), y0:y1].data_ptr(), None, s.cuda_stream,
                                                      None))
                else:
                    check(L.rt_render_bands_device(r._ctx, C.byref(cam.ubo), W, H, B, args.band, N, 0,
                                                   slots[half, k % G, :rows].data_ptr(), None, s.cuda_stream,
                                                   None))
                if exch and k % G == G - 1:
                    for t in streams:
                        main_s.wait_stream(t)
                    with torch.cuda.stream(main_s):
                        if mode == "blocks":
                            if N > 1 and moved > 0:
                                dist.gather(other, [landing], dst=0, group=pgs[prio])
                        else:
                            stack = torch.empty_like(slots[half])
                            dist.gather(slots[half], [stack], dst=0, group=pgs[prio])
                            out = torch.index_select(stack.reshape(N * G * plan.max_rows, -1), 0, src)
                            out.reshape(G, H, W, 4)
                    ev = torch.cuda.Event()
                    ev.record(main_s)
                    gathered[half] = ev

            for k in range(R * G + 1):                 # learns this share's order; fills the ring
                trace(k)
            torch.cuda.synchronize()
            n = (args.frames // G) * G
            t0 = time.perf_counter()
            for k in range(n):
                trace(k)
            for t in streams:
                main_s.wait_stream(t)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"config": args.config, "N": N, "inflight": D, "ring": R, "partition": mode, "rank": me,
                              "root_share": share if mode == "blocks" else None, "exchange": exch,
                              "exchange_priority": prio, "frames": n,
                              "ms_per_frame": round(dt * 1e3 / n, 4),
                              "gather_MB_per_batch": round(N * G * plan.max_rows * W * 4 / 1e6, 1)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
