#!/usr/bin/env python3
"""Benchmark: Mrays/s (ray segments per second) of the path-trace path.

Workload (N = 1): BASELINE config 3 — the 50k-triangle synthetic scene at
1920x1080, 4 bounces, default camera.  One step = one whole
frame traced on the GPU: every pixel's full path, RGBA8 written to HBM.  The
render loop keeps D frames in flight (step k on stream k mod D, each stream
its own hardware queue), as a renderer does to hide each frame's serial tail;
the timed region still covers exactly K frames, synchronised on both sides.
With N > 1 ranks (one process per GPU, torch.distributed over RCCL), default
--partition bands: a step is still ONE frame, tiled over the ranks in
interleaved 16-row bands (rank r traces the bands b with b mod N = r); every
D steps the D frames traced since the last exchange are gathered to rank 0
over xGMI (one dist.gather) and assembled there (one index_select), all
inside the timed region (strong scaling: the work per step is fixed).  The
collective's and the assembly's streams run at high priority
(--exchange-priority), so the traces in flight do not starve them of CU slots.
--partition blocks: one contiguous row piece per rank, the pieces' order
rotated every frame, received by rank 0 straight into the frame (RCCL
send/recv, no assembly); rank 0's piece sized by --root-share.
--partition frames: a step is N frames of the render loop, each frame's bands
rotated over the ranks, so every rank traces one frame's worth of pixels per
step (weak scaling).  Rank 0 checks the assembled frames against a one-GPU
frame afterwards (config.frames_verified) and times the same frames on its
GPU alone (speedup_vs_1gpu).

value = segments of a step x steps / wall time of the timed steps (max over
ranks), in millions.  A segment is one executed bounce-loop iteration
(compute_dynamic_ray.comp:179-232); its count per frame is deterministic and is
taken from a counting pass outside the timed region.

roofline: the walk is bound by the issue of its vector memory
instructions (the texture addresser / data path), not by HBM
bandwidth (the 8-MB scene stays in L2 / MALL).  bound "vmem_issue":
achieved = SQ_INSTS_VMEM_RD per launch (PMC, tools/pmc.sh, committed in
profiles/pmc_latest.json for this config) / frame_ms_device, the device time
per launch of the running loop (HIP events around the timed region on the
main stream after joining every launch stream, divided by the launches); peak
= CUs / TA_NS_PER_VMEM, the measured floor of one wave-level
global_load_dwordx4 per CU (tools/ubench/ta_cost.hip,
profiles/r02/walks/ubench_ta_cost.txt:1); frac = achieved / peak.  Beside it:
"hbm" = the PMC HBM bytes per launch (FETCH_SIZE, corrected) over the same
time against 8 TB/s, and "algorithmic" = the contract's algorithmic bytes
(32 B per BVH node visit + 36 B per triangle test + 16 B per material read +
4 B per pixel) over that time against 8 TB/s, which can exceed 1 because
those bytes are cache hits.  kernel_ms is the mean duration of one launch
(HIP events on its own stream; what rocprofv3 reports per kernel); with D
frames in flight launches overlap, and kernel_ms / frame_ms_device is the
average number running at once.
cpu_baseline: the CPU oracle (oracle/rt_oracle.c, OpenMP) on a bounded row
sample of the same frame, rank 0 at N = 1 only (the reference has no CPU
render path: BVHNode.hit throws, BVHNode.java:35-41).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E, MI355X_MICROARCH.md chip table
# ns of the vector memory pipeline per wave-level global_load_dwordx4 per CU
# when every lane reads one address: the cheapest form a walk step's loads take
# (tools/ubench/ta_cost.hip; profiles/r02/walks/ubench_ta_cost.txt:1, 7.39 ns
# = 17.7 cycles at 2.4 GHz)
TA_NS_PER_VMEM = 7.39
TA_NS_SOURCE = "profiles/r02/walks/ubench_ta_cost.txt:1 (tools/ubench/ta_cost.hip: width 16 B, stride 0, 64 lanes)"
BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Frames in flight need one hardware queue per stream to run concurrently; the
# HIP default (4 queues per process) puts several streams on one queue and
# serialises their launches (config 3, a rank's 1/8 share with 8 frames in
# flight: 0.118 ms per frame on 4 queues, 0.057 on 16; profiles/r02/inflight16).
# Read by the HIP runtime at initialisation, so set before torch touches the GPU.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"


def default_inflight(world: int) -> int:
    """Frames in flight per rank (bands partition), measured best for config 3
    (tools/share_inflight_bench.py on one MI355X, 16 queues, the default
    schedule; profiles/r02/inflight16/share4_q16.jsonl): N = 1: 4 (0.338 ms
    per frame); N = 2: 8 (0.175 ms per half frame); N = 4, 8: 12 (0.092 /
    0.050 ms per share vs 0.104 / 0.077 at 4).  At most 12: with the main
    stream, the collective's and the runtime's own, 16 queues stay one per
    stream."""
    return 4 if world == 1 else (8 if world == 2 else 12)


def default_root_share(world: int) -> float:
    """blocks partition: rank 0's piece in units of H / N rows.  Rank 0 also
    receives the other N - 1 pieces of every frame into place, which costs it
    device time the other ranks do not spend; balancing trace + exchange time
    per frame, rank 0's share is 1 - X (N - 1) / T (X: its exchange time per
    frame, T: N x a share's trace time).  The one-GPU emulation of rank 0
    (tools/rank0_exchange_bench.py, profiles/r02/rccl/) puts X at ~0.019 ms
    per frame at N = 8 and ~0.01 at N = 4 for config 3."""
    return 1.0 if world <= 2 else (0.9 if world <= 4 else 0.6)


def file_sha16(path: str) -> str:
    import hashlib
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 frames of config 3 are ~70 ms: with 4-12 frames in flight, 20 steps
    # would spend a fifth of the timed region filling and draining the pipeline.
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, help="BASELINE config index (3 = headline)")
    ap.add_argument("--band", type=int, default=16, help="band height for N > 1")
    ap.add_argument("--partition", choices=("bands", "blocks", "frames"), default="bands",
                    help="N > 1: bands = one frame per step in interleaved --band-row bands, gathered and "
                         "assembled on rank 0 (strong scaling, default); blocks = one frame per step in N "
                         "contiguous row pieces laid out in an order rotated every frame, received by rank 0 "
                         "straight into the frame (strong; emulated slower on the sending ranks, "
                         "profiles/r02/rccl/README.md); frames = N frames per step, bands rotated over ranks (weak)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight per rank (bands partition): each step's trace goes on the next of this "
                         "many streams, so frames overlap each other's serial tails and the gathers "
                         "(0 = auto, default_inflight(): 4 at N = 1, 8 at N = 2, 12 at N > 2)")
    ap.add_argument("--drain", type=int, default=0,
                    help="1: the last frames of a run of steps plan their heavy pixels for the frames still in "
                         "flight beside them (concurrent_launches min(D, frames left)); 0 (default): every frame "
                         "for D.  Measured slower at 20 steps (0.329-0.332 vs 0.309-0.312 ms/frame, "
                         "profiles/r02/drain)")
    ap.add_argument("--set", default="", help="schedule options name=value,... (rt_set_option) before timing")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single", action="store_true", help="N > 1: skip rank 0's one-GPU timing")
    ap.add_argument("--ring", type=int, default=2,
                    help="N > 1 (blocks, bands): batches of frame slots in the ring (>= 2); the traces of a batch "
                         "wait for the exchange of the batch that used its slots, ring - 1 batches back")
    ap.add_argument("--root-share", type=float, default=-1.0,
                    help="blocks: rank 0's piece in units of H / N rows (it also receives every other piece); "
                         "-1 = default_root_share(N)")
    ap.add_argument("--exchange-priority", type=int, default=1,
                    help="N > 1: 1 = the collective's stream and the assembly stream at high priority, so the "
                         "exchange is not starved of workgroup slots by the traces in flight")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample time")
    ap.add_argument("--settle-s", type=float, default=0.2,
                    help="untimed frames before the warmup steps: this many seconds of counting-pass time "
                         "(5-100 frames; steady clocks and caches)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC per launch of each config (tools/pmc_traffic.py: SQ_INSTS_VMEM_RD, HBM bytes) for "
                         "the roofline")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import configs

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    # BENCH_FORCE_DIST=1 (rehearsal only): the N > 1 code path at any world size,
    # so one GPU runs the bands partition, its RCCL gather and the rank-0 checks.
    dist_on = world > 1 or os.environ.get("BENCH_FORCE_DIST") == "1"
    # BENCH_SHARE_GPU=1 (rehearsal only): ranks share the visible GPUs round-robin.
    dev_index = local_rank % torch.cuda.device_count() if os.environ.get("BENCH_SHARE_GPU") else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    local_rank = dev_index
    backend = None
    if dist_on:
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")     # nccl = RCCL over xGMI
        pg_options = None
        if backend == "nccl" and args.exchange_priority:
            # RCCL's internal stream at high priority: with D traces in flight
            # every CU slot is taken, and a normal-priority collective gets
            # slots only as trace waves end
            from torch.distributed import ProcessGroupNCCL
            pg_options = ProcessGroupNCCL.Options()
            pg_options.is_high_priority_stream = True
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None, pg_options=pg_options)

    cfg = configs.get(args.config)
    t0 = time.time()
    built = cfg.build()
    cam = cfg.camera()
    log(f"[rank {rank}] built {cfg.name}: {built.triangle_count} flat tris, {built.n_nodes} nodes "
        f"in {time.time() - t0:.2f}s")
    W, H, B = cfg.width, cfg.height, cfg.max_bounces

    renderer = rtamd.Renderer((local_rank,))
    renderer.upload_scene(built)
    for kv in filter(None, args.set.split(",")):
        k, v = kv.split("=")
        renderer.set_option(k.strip(), int(v))
    L = rtamd.lib()
    from rtamd.dist import (BatchPlan, batch_band_offset, block_layout, block_sizes, exchange_blocks, gather_batch,
                            gather_frames)

    # Partition.  bands (default): one frame per step tiled over the ranks in
    # interleaved band_h-row bands (strong scaling; a frame lasts as long as
    # its slowest wave).  frames: a step renders N frames of the
    # render loop (the reference re-renders the current camera every loop
    # iteration, VulkanEngine.java:240-276), each tiled over all ranks in
    # rotating bands, so every rank traces one frame's worth of pixels per
    # step (weak scaling).  At N = 1 both are one whole frame per step.
    frames_mode = args.partition == "frames" and world > 1
    blocks_mode = args.partition == "blocks" and dist_on
    F = world if frames_mode else 1
    band_h = H if (not dist_on or blocks_mode) else args.band
    offsets = [batch_band_offset(f, world, rank) if frames_mode else rank for f in range(F)]
    plan = BatchPlan(H, band_h, world, F) if frames_mode else None
    rows_f = [L.rt_band_rows(H, band_h, world, off) for off in offsets]
    max_rows = plan.max_rows if plan else max(L.rt_band_rows(H, band_h, world, r) for r in range(world))
    # blocks: rank 0's piece is root_share x H / N rows (it also receives the
    # other pieces of every frame), the other ranks split the rest
    share = (args.root_share if args.root_share >= 0 else default_root_share(world)) if blocks_mode else 1.0
    if blocks_mode:
        max_rows = max(block_sizes(H, world, share))
    # Frames in flight (bands partition): step k traces on stream k mod D.  A
    # frame's own time is bounded by its slowest pixel's dependent chain
    # (DESIGN.md §7), so the render loop keeps D frames on the device at once
    # (each stream its own hardware queue, GPU_MAX_HW_QUEUES above) and a
    # rank's 1/N share of a frame fills the GPU only with several in flight
    # (tools/share_inflight_bench.py, profiles/r02/inflight16/).
    D = 1 if frames_mode else (args.inflight if args.inflight > 0 else default_inflight(world))
    # The heavy-pixel bar counts every launch of similar work on the device at
    # once (option concurrent_launches): a frame batch's F launches, or the D
    # frames in flight.
    renderer.set_option("concurrent_launches", F * D)
    # Exchange (N > 1, blocks / bands): every G = D steps the G frames traced
    # since the last exchange go to rank 0 in one RCCL group (blocks: sends /
    # receives straight into rank 0's frames; bands: one gather and one
    # index_select, dist.gather_frames), so the host cost of the exchange is
    # paid once per G frames.  R x G frame slots: batches are traced while
    # earlier ones are exchanged; a slot is retraced only after the exchange
    # that used it.  N = 1: one slot per stream.  frames partition: one gather
    # per step of F frames, D + 1 buffers.
    G = D if (dist_on and not frames_mode) else 1
    # R batches of slots in the ring: a batch's slots are retraced only after
    # the exchange R - 1 batches back has finished.  The exchange kernels get
    # workgroup slots only as trace waves end, so a deep ring keeps a late
    # exchange from stalling the traces.
    R = max(2, args.ring)
    if frames_mode:
        n_slots = D + 1
    elif dist_on:
        n_slots = R * G
    else:
        n_slots = D
    d_bufs = [torch.empty((F, max_rows, W, 4), dtype=torch.uint8, device=dev) for _ in range(n_slots)] \
        if frames_mode else None
    slots = torch.empty((n_slots, max_rows, W, 4), dtype=torch.uint8, device=dev) if not frames_mode else None
    # blocks: rank 0 traces its block of frame k in place in fring[k mod n_slots]
    # and receives the other blocks there
    fring = torch.empty((n_slots, H, W, 4), dtype=torch.uint8, device=dev) if (blocks_mode and rank == 0) else None
    gathered = [None] * (n_slots if frames_mode else R)   # event: the last exchange that used a buffer / batch slot
    # One stream per launch in flight (launches and their events on the same
    # queue); the gathers run on main_stream.
    streams = [torch.cuda.Stream(dev) for _ in range(min(F * D, 12))]
    hi = -1 if (dist_on and args.exchange_priority) else 0   # the assembly (index_select) at high priority
    main_stream = torch.cuda.Stream(dev, priority=hi) if (dist_on or len(streams) > 1) else streams[0]
    torch.cuda.set_stream(main_stream)
    src_index = torch.as_tensor(plan.src, device=dev) if (plan and dist_on) else None

    import ctypes as C
    from rtamd._lib import Stats, check

    def trace(f, stats: bool = False, ev=None, out=None, si=0, rect=None):
        s = streams[si % len(streams)]
        st = Stats()
        if ev is not None:          # recorded after the stream's wait for the gather: the trace only
            ev[0].record(s)
        if rect is not None:        # blocks: frame rows [y0, y1), packed into out
            if rect[1] > rect[0]:
                check(L.rt_render_tile_device(renderer._ctx, C.byref(cam.ubo), W, H, B, 0, rect[0], W,
                                              rect[1] - rect[0], out.data_ptr(), None, s.cuda_stream,
                                              C.byref(st) if stats else None))
        else:
            check(L.rt_render_bands_device(renderer._ctx, C.byref(cam.ubo), W, H, B, band_h, world, offsets[f],
                                           out.data_ptr(), None, s.cuda_stream, C.byref(st) if stats else None))
        if ev is not None:
            ev[1].record(s)
        return st.as_dict() if stats else None

    k_step = [0]
    last = [None]

    def flush():
        """Bands, N > 1: gather the frames of the current batch traced so far
        (a whole batch from step(), the rest at the end of a phase)."""
        k = k_step[0]
        n = k % G if k % G else (G if k else 0)
        if n == 0:
            return None
        half = ((k - 1) // G) % R
        for s in streams:
            main_stream.wait_stream(s)
        if blocks_mode:         # RCCL sends / receives straight into rank 0's frames
            base = half * G
            exchange_blocks(fring[base: base + n] if rank == 0 else None, slots[base: base + n],
                            list(range(k - n, k)), H, share)
            out = fring[base: base + n] if rank == 0 else None
        else:
            out = gather_frames(slots[half * G: half * G + n], H, band_h)   # RCCL gather + rank-0 assembly
        gathered[half] = torch.cuda.Event()
        gathered[half].record(main_stream)
        k_step[0] = ((k + G - 1) // G) * G       # the next phase starts a fresh batch
        last[0] = out
        return out

    def step(evs=None):
        k = k_step[0]
        k_step[0] += 1
        if frames_mode:
            b = k % n_slots
            mine = [streams[(k * F + f) % len(streams)] for f in range(F)]
            for s in mine:                             # the gather that last read this buffer is done
                if gathered[b] is not None:
                    s.wait_event(gathered[b])
            for f in range(F):
                trace(f, ev=evs[f] if evs is not None else None, out=d_bufs[b][f], si=k * F + f)
            for s in mine:
                if s is not main_stream:
                    main_stream.wait_stream(s)
            last[0] = gather_batch(d_bufs[b], plan, src_index=src_index)
            gathered[b] = torch.cuda.Event()
            gathered[b].record(main_stream)
            return
        s = streams[k % len(streams)]
        if blocks_mode:
            half = (k // G) % R
            if k % G == 0 and gathered[half] is not None:
                for t in streams:                      # the exchange that last used this half is done
                    t.wait_event(gathered[half])
            y0, y1 = block_layout(H, world, k, share)[rank]
            out = fring[k % n_slots, y0:y1] if rank == 0 else slots[k % n_slots, : y1 - y0]
            trace(0, ev=evs[0] if evs is not None else None, out=out, si=k, rect=(y0, y1))
            if k % G == G - 1:
                flush()
        elif dist_on:
            half = (k // G) % R
            if k % G == 0 and gathered[half] is not None:
                for t in streams:                      # the gather that last read this half is done
                    t.wait_event(gathered[half])
            trace(0, ev=evs[0] if evs is not None else None, out=slots[k % n_slots, :rows_f[0]], si=k)
            if k % G == G - 1:
                flush()
        else:
            trace(0, ev=evs[0] if evs is not None else None, out=slots[k % n_slots, :rows_f[0]], si=k)

    # Counting pass (untimed): this rank's work, then the job totals.
    count_out = torch.empty((max_rows, W, 4), dtype=torch.uint8, device=dev)
    per = [trace(f, stats=True, out=count_out, rect=block_layout(H, world, 0, share)[rank] if blocks_mode else None)
           for f in range(F)]
    torch.cuda.synchronize(dev)
    counts = torch.tensor([sum(p[k] for p in per) for k in ("pixels", "segments", "node_visits", "tri_tests",
                                                             "mat_reads")], dtype=torch.float64, device=dev)
    local = counts.clone()
    if dist_on:
        dist.all_reduce(counts)
    pixels, segments, node_visits, tri_tests, mat_reads = [float(x) for x in counts.tolist()]
    # per launch (blocks: the mean over the ranks' blocks, which differ in cost)
    per_launch = (counts / world) if blocks_mode else local
    l_pix, l_seg, l_nodes, l_tris, l_mats = [float(x) / F for x in per_launch.tolist()]
    log(f"[rank {rank}] step: {F} frame(s), {segments:.0f} segments ({segments / pixels:.3f}/px), "
        f"{node_visits / segments:.2f} node visits/seg, {tri_tests / segments:.3f} tri tests/seg; "
        f"{D} frame(s) in flight, exchange every {G} step(s)")

    # Drain (option --drain, off by default: measured slower): a launch's heavy-pixel bar counts
    # the launches that will run beside it, and at the end of a run of frames
    # fewer do: step j of n has min(D, n - j) frames in flight from its launch
    # on, so the last frames split their slowest pixels into one-pixel waves
    # as a lone frame does, instead of leaving the run's end to one frame's
    # serial tail.  Pixels and results do not change.
    conc_now = [F * D]

    def set_conc(c):
        if c != conc_now[0]:
            renderer.set_option("concurrent_launches", c)
            conc_now[0] = c

    def phase(n, evs=None):
        for j in range(n):
            if args.drain:
                set_conc(F * min(D, n - j))
            step(evs[j] if evs is not None else None)
        set_conc(F * D)
        if dist_on and not frames_mode:
            flush()

    # Settle (untimed): 5-100 frames, about settle_s / (the counting pass's
    # device time; a counting launch runs ~4x a plain one), so the timed steps
    # see the steady state of a running render loop (the first frames after
    # start-up run 3-4% slower: profiles/r02/warmup), then the W warmup steps
    # of the contract.
    # The count is fixed up front (from the counting pass's device time) and
    # agreed over the ranks, so every rank runs the same collectives.
    est_ms = max(0.05, float(per[0].get("ms", 1.0)))
    # at least 2D: the drain's launch keys (concurrency 1..D) learn their
    # orders here, not in the timed region
    n_settle = torch.tensor([max(5, 2 * D, min(100, int(args.settle_s * 1e3 / est_ms)))], dtype=torch.int64,
                            device=dev)
    if dist_on:
        dist.all_reduce(n_settle, op=dist.ReduceOp.MIN)
    phase(int(n_settle.item()))
    torch.cuda.synchronize(dev)
    phase(args.warmup)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)

    # HIP events: around every launch on its own stream (the launch's device
    # duration; with D in flight the launches overlap), and around the whole
    # timed region on main_stream after joining every stream (the device time
    # per frame of the running loop).
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(F)]
           for _ in range(args.steps)]
    reg = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t_start = time.perf_counter()
    reg[0].record(main_stream)
    for s in streams:
        if s is not main_stream:
            s.wait_stream(main_stream)
    phase(args.steps, evs)
    for s in streams:
        if s is not main_stream:
            main_stream.wait_stream(s)
    reg[1].record(main_stream)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    launch_ms = float(np.mean([a.elapsed_time(b) for e in evs for a, b in e]))
    region_ms = reg[0].elapsed_time(reg[1])
    frame_ms = region_ms / (args.steps * F)            # device time per launch of the running loop
    out = last[0]

    heavy_used = renderer.get_option("heavy_tiles_used")   # of the last timed launch
    verified = None
    single = None
    if dist_on and rank == 0:
        # the assembled frames equal the 1-GPU frame
        full = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
        check(L.rt_render_bands_device(renderer._ctx, C.byref(cam.ubo), W, H, B, H, 1, 0, full.data_ptr(), None,
                                       main_stream.cuda_stream, None))
        torch.cuda.synchronize(dev)
        frames = out if out.dim() == 4 else out[None]
        verified = bool(all(torch.equal(frames[f], full) for f in range(frames.shape[0])))
        if not args.no_single:
            # The same frames on this GPU alone: whole frames, one per launch,
            # with the one-GPU default frames in flight, for the speedup of
            # this partition.
            D1 = default_inflight(1)
            renderer.set_option("concurrent_launches", D1)
            fulls = [full] + [torch.empty_like(full) for _ in range(D1 - 1)]
            sstreams = streams[:D1] + [torch.cuda.Stream(dev) for _ in range(D1 - len(streams))]

            def one(j):
                check(L.rt_render_bands_device(renderer._ctx, C.byref(cam.ubo), W, H, B, H, 1, 0,
                                               fulls[j % D1].data_ptr(), None, sstreams[j % D1].cuda_stream, None))
            one(0)                                    # learns the whole-frame order
            torch.cuda.synchronize(dev)
            for j in range(4 * D1):
                one(j)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for j in range(args.steps * F):
                one(j)
            torch.cuda.synchronize(dev)
            single = time.perf_counter() - t1

    t = torch.tensor([elapsed, launch_ms, frame_ms], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, launch_ms_max, frame_ms_max = float(t[0]), float(t[1]), float(t[2])

    value = segments * args.steps / elapsed / 1e6
    alg_bytes = 32.0 * l_nodes + 36.0 * l_tris + 16.0 * l_mats + 4.0 * l_pix
    ref_layout_bytes = 48.0 * l_nodes + 48.0 * l_tris + 16.0 * l_mats + 4.0 * l_pix
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    pmc = load_pmc(args.pmc_json, cfg.name) if (world == 1 and F == 1) else None
    roof = roofline(pmc, alg_bytes, ref_layout_bytes, l_seg, frame_ms, n_cu)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(built, cam, W, H, B, segments, args.cpu_seconds)

    if rank == 0:
        gather_kind = "RCCL" if backend == "nccl" else (backend or "none")
        shared = " (ranks share one GPU: rehearsal)" if os.environ.get("BENCH_SHARE_GPU") else ""
        out = {
            "metric": BASELINE["metric"],
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if frames_mode else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"{'reference asset' if args.config == 6 else 'synthetic'} "
                    f"({cfg.note}; default camera)",
            "config": {
                "workload": cfg.name,
                "width": W, "height": H, "max_bounces": B,
                "triangles_flat": built.triangle_count, "bvh_nodes": built.n_nodes,
                "segments_per_frame": int(segments / F),
                "node_visits_per_segment": round(node_visits / segments, 3),
                "tri_tests_per_segment": round(tri_tests / segments, 4),
                "partition": f"one whole frame per step, {D} frames in flight" if not dist_on else
                             (f"{F} frames per step, {band_h}-row bands rotated over {world} ranks "
                              f"(rank r traces bands (r+f) mod {world} of frame f), {gather_kind} gather + rank-0 "
                              f"assembly{shared}"
                              if frames_mode else
                              f"one frame per step in {world} contiguous row pieces (rows per rank "
                              f"{block_sizes(H, world, share)}, root_share {share}) laid out in an order rotated "
                              f"every frame, {D} frames in flight per rank, {gather_kind} sends / receives of every "
                              f"{G} frames straight into rank 0's frames{shared}"
                              if blocks_mode else
                              f"one frame per step, interleaved {band_h}-row bands over {world} ranks, "
                              f"{D} frames in flight per rank, {gather_kind} gather of every {G} frames + rank-0 "
                              f"assembly{shared}"),
                "frames_per_step": F,
                "frames_in_flight": D,
                "frames_verified": verified,
                "parallelism": f"tile{world}",
                "schedule": {**{k: renderer.get_option(k) for k in ("kernel", "walk", "wave_tile", "coop_lanes",
                                                                      "heavy_first", "heavy_tiles", "heavy_factor",
                                                                      "heavy_stream", "heavy_pixels",
                                                                      "heavy_pixel_factor", "heavy_cap", "graph")},
                             "concurrent_launches": renderer.get_option("concurrent_launches"),
                             "drain": args.drain,
                             "heavy_tiles_used": heavy_used,
                             "heavy_pixels_used": renderer.get_option("heavy_pixels_used")},
                "launches_per_step": F * (2 if heavy_used > 0 and renderer.get_option("heavy_stream") != 2 else 1),
            },
            "roofline": {
                **roof,
                "kernel": ("trace_simple" if renderer.get_option("kernel") == 0 else "trace_*") + (
                    f" (one launch per frame: the {renderer.get_option('heavy_pixels_used')} heaviest pixels one per "
                    f"wave first, then every {8 << renderer.get_option('wave_tile')}x"
                    f"{8 >> renderer.get_option('wave_tile')} tile without them)"
                    if renderer.get_option("heavy_pixels_used") > 0
                    else f" (one launch per frame: the {heavy_used} heaviest tiles one pixel per wave first)"
                    if heavy_used > 0 and renderer.get_option("heavy_stream") == 2
                    else f" (frame = the {heavy_used} heaviest tiles' one-pixel-wave launch concurrent with the "
                         f"other tiles' launch; kernel_ms spans both)" if heavy_used > 0 else ""),
                "kernel_ms": round(launch_ms, 4),
                "kernel_ms_max_over_ranks": round(launch_ms_max, 4) if dist_on else None,
                "frame_ms_device": round(frame_ms, 4),
                "frame_ms_device_max_over_ranks": round(frame_ms_max, 4) if dist_on else None,
                "launches_in_flight_avg": round(launch_ms / frame_ms, 2),
                "events": "kernel_ms: each launch's own stream, around every launch (after its wait for the "
                          "gather); frame_ms_device: main stream around the timed region after joining every "
                          "launch stream, / launches",
            },
            "primary_mrays_s": round(pixels * args.steps / elapsed / 1e6, 2),
            "cpu_baseline": cpu,
            "bench_sha16": file_sha16(os.path.abspath(__file__)),
        }
        if single is not None:
            sv = segments * args.steps / single / 1e6
            out["single_gpu"] = {"value": round(sv, 2), "ms_per_frame": round(single / (args.steps * F) * 1e3, 4),
                                 "what": f"the same frames traced whole on rank 0's GPU alone, one per launch, "
                                         f"{D} in flight"}
            out["speedup_vs_1gpu"] = round(value / sv, 3)
        print(json.dumps(out), flush=True)
    renderer.close()
    if dist_on:
        dist.destroy_process_group()


def load_pmc(path, config_name):
    """PMC per launch for config_name from profiles/pmc_latest.json
    (tools/pmc_traffic.py), or None."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        tj = json.load(fh)
    return tj.get("configs", {}).get(config_name)


def roofline(pmc, alg_bytes, ref_layout_bytes, l_seg, frame_ms, n_cu):
    """The roofline object of the JSON line (module docstring): the vector
    memory issue bound from PMC, with the HBM and algorithmic figures."""
    t = frame_ms * 1e-3                                     # s per launch of the running loop
    vmem = pmc.get("SQ_INSTS_VMEM_RD") if pmc else None
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    peak = n_cu / TA_NS_PER_VMEM                            # G wave-instructions / s
    achieved = vmem / t / 1e9 if vmem else None
    hbm = traffic / t / 1e9 if traffic else None
    alg = alg_bytes / t / 1e9
    return {
        "bound": "vmem_issue",
        "achieved": round(achieved, 3) if achieved else None,
        "peak": round(peak, 3),
        "unit": "G wave-level vector-memory instructions/s",
        "frac": round(achieved / peak, 4) if achieved else None,
        "traffic": traffic,
        "basis": f"achieved = SQ_INSTS_VMEM_RD per launch ({vmem}, PMC) / frame_ms_device; peak = {n_cu} CUs / "
                 f"{TA_NS_PER_VMEM} ns per wave-level global_load_dwordx4 per CU ({TA_NS_SOURCE}); traffic = PMC "
                 f"HBM bytes per launch (FETCH_SIZE x 1024 x 2). null without a PMC record of this config "
                 f"(profiles/pmc_latest.json) or for N > 1 shares",
        "pmc_source": pmc.get("source") if pmc else None,
        "vmem_rd_per_launch": vmem,
        "vmem_rd_per_segment": round(vmem / l_seg, 3) if vmem else None,
        "hbm": {"achieved": round(hbm, 1) if hbm else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hbm / HBM_PEAK_GBS, 4) if hbm else None},
        "algorithmic": {"bytes_per_launch": int(alg_bytes), "bytes_per_segment": round(alg_bytes / l_seg, 1),
                        "achieved": round(alg, 1), "unit": "GB/s",
                        "alg_throughput_frac": round(alg / HBM_PEAK_GBS, 4),
                        "reference_layout_frac": round(ref_layout_bytes / t / 1e9 / HBM_PEAK_GBS, 4),
                        "note": "the reference's visit counts x record sizes (SURVEY.md §8d) over the launch time; "
                                "mostly L2/MALL hits, so it can exceed the HBM peak"},
    }


def host_cpu():
    """CPU model, the host's logical CPUs and the ones this process may use."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), None)
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or 1, usable


def cpu_baseline(built, cam, W, H, B, frame_segments, target_s):
    """The oracle on every k-th row of the same frame, all host threads we may use."""
    from oracle import oracle_lib
    model, nproc, usable = host_cpu()
    # A GPU box gives one GPU's job a share of 16 of the host's CPUs (the pool's
    # rule; os.cpu_count() reports the whole host), and sets OMP_NUM_THREADS to it
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    threads = max(1, min(share, usable))
    args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), W, H, B)
    # probe on every 64th row, then size the sample to ~target_s: every k-th
    # row if the frame takes longer than that, else the whole frame repeated.
    t0 = time.perf_counter()
    _, _, c = oracle_lib.render(*args, row_step=64, radiance=False, n_threads=threads)
    probe = time.perf_counter() - t0
    rate = c["segments"] / max(probe, 1e-6)
    frame_s = frame_segments / rate
    step, reps = 1, 1
    if frame_s > target_s:
        step = next((s for s in (2, 4, 8, 16, 32, 64) if frame_s / s <= target_s), 64)
    else:
        reps = max(1, min(100, int(round(target_s / frame_s))))
    # the probe under-estimates the steady rate (thread start-up on a small
    # sample), so repeat until the sample really lasts ~target_s
    segs = 0
    px = 0
    n = 0
    t0 = time.perf_counter()
    while n < reps or (time.perf_counter() - t0 < target_s and n < 100):
        _, _, c = oracle_lib.render(*args, row_step=step, radiance=False, n_threads=threads)
        segs += c["segments"]
        px += c["pixels"]
        n += 1
    dt = time.perf_counter() - t0
    what = (f"every {step}th row of the frame" + (f" x {n}" if n > 1 else "")) if step > 1 \
        else f"the whole frame x {n}"
    return {
        "value": round(segs / dt / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{what} ({px} px, {segs} segments, {dt:.2f} s, OpenMP threads {threads})",
        "cpu_model": model,
        "nproc": nproc,
        "cpus_usable": usable,
        "threads_why": f"the job's CPU share: OMP_NUM_THREADS / 16 per GPU on the GPU pool (of {nproc} logical "
                       f"CPUs on the host, {usable} in this process's affinity mask)",
        "what": "oracle/rt_oracle.c (a line-by-line C restatement of compute_dynamic_ray.comp, the parity "
                "checker) with OpenMP over rows: the reference has no CPU render path (BVHNode.hit throws "
                "UnsupportedOperationException, BVHNode.java:35-41), so no 'reference' CPU baseline exists",
    }


if __name__ == "__main__":
    main()
