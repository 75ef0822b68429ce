#!/usr/bin/env python3
"""One rank of an N-GPU bench.py run (--partition bands), emulated on one GPU.

The driver measures N > 1 on an 8-GPU node; a gpurun box has one GPU and RCCL
refuses two ranks on it.  This runs exactly one rank's device work of
bench.py's bands partition at N: its weighted band share (rtamd.dist
SharePlan) of F frames per launch (rt_render_batch_device), D launches in
flight on their own streams, a ring of R exchange batches of G frames, and
per batch the exchange:

  rank 0  an RCCL gather at world size 1 (a device copy) of the whole batch
          volume it receives at N (N x per_rank rows: its own share and the
          N - 1 others'), then the index_select assembly of the G frames, on
          the high-priority exchange stream (bench.py --exchange-priority 1);
  rank r  an RCCL gather at world size 1 of its own per_rank rows (the send).

The other ranks' rows are whatever the buffers hold: frames are not checked
(bench.py and tests/test_dist.py check them).  max over ranks of ms per frame
is the frame time an N-GPU run can reach; N x that against the one-GPU frame
time is the scaling the driver's SCALE run would see if xGMI transfers cost
rank 0 what the local copy does.

Usage: python tools/rank_emulator.py [--config 3] [--ranks 8] [--which 0,1]
           [--root-weight 0.7,0.8] [--batch 4] [--inflight 4] [--frames 240]
Prints one JSON line per (N, rank, root_weight, batch, inflight), plus the
one-GPU reference (N = 1, bench.py's default) first.
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


def _ints(x):
    return [int(v) for v in str(x).split(",") if v != ""]


def _floats(x):
    return [float(v) for v in str(x).split(",") if v != ""]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ranks", default="8")
    ap.add_argument("--which", default="0,1", help="ranks to emulate (0 receives and assembles, others send)")
    ap.add_argument("--root-weight", default="-1", help="comma list; -1 = bench.default_root_weight(N)")
    ap.add_argument("--batch", default="0", help="frames per launch, comma list; 0 = bench.default_batch(N)")
    ap.add_argument("--inflight", default="0", help="launches in flight, comma list; 0 = bench.default_inflight")
    ap.add_argument("--band", type=int, default=8)
    ap.add_argument("--frames", type=int, default=240)
    ap.add_argument("--exchange", type=int, default=1, help="0: traces only")
    ap.add_argument("--ring", type=int, default=2)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import configs, CameraUBO
    from rtamd._lib import check
    from rtamd.dist import SharePlan
    from torch.distributed import ProcessGroupNCCL

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    L = rtamd.lib()
    opts = ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    store = dist.TCPStore("127.0.0.1", _port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev, pg_options=opts)
    main_s = torch.cuda.Stream(dev, priority=-1)

    def run(N, me, rw, F, D):
        """ms per frame of rank `me` of N (N = 1: whole frames, no exchange)."""
        G = D * F
        R = max(2, args.ring)
        plan = SharePlan(H, args.band, N, G, rw) if N > 1 else None
        bands = np.ascontiguousarray(plan.bands[me]) if plan else None
        rows = plan.counts[me] if plan else H
        per_rank = plan.per_rank if plan else G * H
        slots = torch.zeros((R, per_rank, W, 4), dtype=torch.uint8, device=dev)
        streams = [torch.cuda.Stream(dev) for _ in range(D)]
        r.set_option("concurrent_launches", D)
        src = torch.as_tensor(plan.src, device=dev) if plan else None
        recv = torch.zeros((N * per_rank, W, 4) if me == 0 else (per_rank, W, 4), dtype=torch.uint8, device=dev)
        landing = torch.empty_like(recv)
        gathered = [None] * R
        cams = (CameraUBO * F)(*([cam.ubo] * F))
        bp = bands.ctypes.data_as(C.POINTER(C.c_int32)) if bands is not None else None

        def launch(j):
            k0 = j * F
            s = streams[j % D]
            h = (k0 // G) % R
            if k0 % G == 0 and gathered[h] is not None:
                for t in streams:
                    t.wait_event(gathered[h])
            check(L.rt_render_batch_device(r._ctx, cams, F, W, H, B, args.band if plan else 0, bp,
                                           len(bands) if bands is not None else 0,
                                           slots[h, (k0 % G) * rows].data_ptr(), None, s.cuda_stream, None))
            if args.exchange and N > 1 and (k0 + F) % G == 0:
                for t in streams:
                    main_s.wait_stream(t)
                with torch.cuda.stream(main_s):
                    dist.gather(recv, [landing], dst=0)
                    if me == 0:
                        out = torch.index_select(landing.reshape(N * per_rank, -1), 0, src)
                        out.reshape(G, H, W, 4)
                ev = torch.cuda.Event()
                ev.record(main_s)
                gathered[h] = ev

        n_launch = max(R * D + 1, args.frames // F)
        for j in range(R * D + 1):            # learns the order, fills the ring
            launch(j)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(n_launch):
            launch(j)
        for t in streams:
            main_s.wait_stream(t)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return dt * 1e3 / (n_launch * F), rows, per_rank

    base, _, _ = run(1, 0, 1.0, 1, bench.default_inflight(1))
    print(json.dumps({"config": args.config, "N": 1, "rank": 0, "batch": 1, "inflight": bench.default_inflight(1),
                      "ms_per_frame": round(base, 4), "what": "one GPU, bench.py's N = 1 default"}), flush=True)
    for N in _ints(args.ranks):
        for rw in _floats(args.root_weight):
            rw = bench.default_root_weight(N) if rw < 0 else rw
            for F in _ints(args.batch):
                F = bench.default_batch(N) if F <= 0 else F
                for D in _ints(args.inflight):
                    D = bench.default_inflight(N) if D <= 0 else D
                    for me in _ints(args.which):
                        if me >= N:
                            continue
                        ms, rows, per_rank = run(N, me, rw, F, D)
                        print(json.dumps({"config": args.config, "N": N, "rank": me, "root_weight": rw, "batch": F,
                                          "inflight": D, "exchange": args.exchange, "band_h": args.band,
                                          "rows": rows, "ms_per_frame": round(ms, 4),
                                          "speedup_if_slowest": round(base / ms, 3),
                                          "gather_rows": N * per_rank if me == 0 else per_rank}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
