#!/usr/bin/env python3
"""Benchmark: Mrays/s (ray segments per second) of the path-trace path.

Workload (N = 1): BASELINE config 3 — the 50k-triangle synthetic scene at
1920x1080, 4 bounces, default camera.  One step = one whole
frame traced on the GPU: every pixel's full path, RGBA8 written to HBM.  The
render loop keeps D launches in flight (launch j on stream j mod D, each
stream its own hardware queue), as a renderer does to hide each frame's
serial tail; a launch traces F frames (rt_render_batch_device; F = 4 at
N = 1 when the timed frames are whole quadruples, default_batch).  The timed region covers exactly K frames, synchronised on both
sides.

With N > 1 ranks (one process per GPU, torch.distributed over RCCL), every
frame is tiled over ALL ranks and its rows sent to rank 0 over xGMI inside
the timed region.
--scaling weak (default): a step is N frames of the render loop (every rank
  traces one frame's worth of pixels per step, the per-GPU work of N = 1).
  --scaling strong: a step is ONE frame.
--partition spans (default): an exchange batch of G frames is one column of
  G x H rows cut into N contiguous spans of band_h-row bands, rank 0's
  --root-weight times the others' (it also receives every span).  A rank
  traces its span one frame per launch (whole frames, a band run at either
  end; rtamd.dist.SpanPlan / SpanTracer), D launches in flight; rank 0 traces
  its span in place in the batch's frames and receives the others' straight
  into them (one group of RCCL point-to-point receives per batch), so there
  is no assembly pass.  The exchange is ordered by the host, one batch
  behind, and the launch streams never wait on a device event.
--partition bands: interleaved band_h-row bands dealt out by a weighted round
  robin (rank 0 weighted --root-weight: it also receives and assembles every
  frame; rtamd.dist.band_owners).  A rank traces its bands of F frames per
  launch (rt_render_batch_device; weak: F = N, the step), D launches in
  flight; heavy-first order with option order_split 15; one dist.gather per
  exchange batch and one index_select assembly on rank 0.  Where that deal
  gives the other ranks unequal bands (N = 8), the deal runs on over the N
  frames of a launch instead (--deal, rtamd.dist.dealt_bands; one band list
  per frame, rt_render_batch_lists_device).
--partition pieces: N contiguous row pieces, rank r tracing position
  (r + f) mod N of frame f, all N pieces of a launch from different frames
  (rt_render_batch_lists_device); gathered and assembled as the bands.
--partition tiles: the screen tiled gx x gy over the ranks (2 x 2 at N = 4,
  BASELINE config 4), one tile per rank, gathered and assembled likewise.
--gather radiance: the float radiance (the sqrt'd colour before
  quantisation) is gathered beside the RGBA8 frame.
Afterwards rank 0 checks the last assembled frames (and radiance) against
the same frames traced on its GPU alone (config.frames_verified) and times
those (single_gpu, speedup_vs_1gpu); every rank reports its trace and
exchange device time (per_rank).

--camera-path orbit: every frame has its own camera (the default camera's
origin orbiting the look-at point, 0.5 degrees per frame, as the app's
camera moves between frames, VulkanApp.java:726-770); segments are counted
per camera.  After the timed frames the camera stops and the first frames
at rest (the learning frame of the heavy-first order among them) are timed
one by one (camera_stop).

value = segments of the K timed frames / wall time of the timed steps (max
over ranks), in millions.  A segment is one executed bounce-loop iteration
(compute_dynamic_ray.comp:179-232); its count per frame is deterministic and is
taken from a counting pass outside the timed region.

roofline, the frame kernel trace_simple: bound "hbm",
achieved = the algorithmic bytes of one launch (32 B per BVH
node visit + 36 B per triangle test + 16 B per material read + 4 B per pixel,
from the reference's own visit counts) / kernel_ms, the mean duration of one
launch (HIP events around every timed launch on the stream it runs on; what
rocprofv3 reports per kernel); peak = 8 TB/s; traffic = the PMC HBM bytes per
launch (FETCH_SIZE x 1024 x 2, tools/pmc.sh, profiles/pmc_latest.json) when
a PMC record of this config AND camera path exists, else null.  With D
launches in flight the launches overlap (kernel_ms / frame_ms_device is the
average number running at once), so "views" restates the same bytes over
frame_ms_device, the device time per launch of the running loop, against the
HBM and the L2 peaks (the scene stays in L2 / MALL: those bytes are mostly
cache hits), the measured HBM rate (PMC bytes / frame_ms_device), the
vector-memory issue rate (SQ_INSTS_VMEM_RD against a floor measured by
tools/ubench/ta_cost.hip, a builder's microbenchmark, not a guide figure) and
the lockstep walk's lane utilisation (a diagnostic launch outside the timed
region: the lanes' own walk steps / (64 x the waves' lockstep steps)).
cpu_baseline: the CPU oracle (oracle/rt_oracle.c, OpenMP) on a bounded row
sample of the same frame, rank 0 at N = 1 only (the reference has no CPU
render path: BVHNode.hit throws, BVHNode.java:35-41).
pcie (N = 1): rt_render_async with 4 frames in flight into pinned host
frames, every frame read back over PCIe (the rate a host that displays the
frames sees; never `value`).
"""
from __future__ import annotations

import argparse
import ctypes as C
import gc
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E, MI355X_MICROARCH.md chip table
L2_PEAK_GBS = 34500.0      # the 8 XCDs' L2 together, MI355X_MICROARCH.md § L2 (per XCD): ≈34.5 TB/s
# ns of the vector memory pipeline per wave-level global_load_dwordx4 per CU
# when every lane reads one address: the cheapest form a walk step's loads take
# (tools/ubench/ta_cost.hip; profiles/r02/walks/ubench_ta_cost.txt:1, 7.39 ns
# = 17.7 cycles at 2.4 GHz)
TA_NS_PER_VMEM = 7.39
TA_NS_SOURCE = "profiles/r02/walks/ubench_ta_cost.txt:1 (tools/ubench/ta_cost.hip: width 16 B, stride 0, 64 lanes)"
BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Launches in flight need one hardware queue per stream to run concurrently;
# the HIP default (4 queues per process) puts several streams on one queue and
# serialises their launches (config 3, a rank's 1/8 share with 8 frames in
# flight: 0.118 ms per frame on 4 queues, 0.057 on 16; profiles/r02/inflight16).
# Read by the HIP runtime at initialisation, so set before torch touches the GPU.
def _queues() -> None:
    raw = os.environ.get("GPU_MAX_HW_QUEUES", "")
    try:
        have = int(raw) if raw.strip() else 4
    except ValueError:
        have = 4
    if have < 16:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"


_queues()


def default_inflight(world: int) -> int:
    """Launches in flight per rank.  N = 1: 4 whole frames (0.338 ms per
    frame vs 0.343 at 6-12, profiles/r02/inflight16/share4_q16.jsonl).  N > 1:
    4 batched launches (default_batch frames each): a rank's share of one
    frame is too small a launch to fill the GPU past its own tail (DESIGN.md
    §6)."""
    return 4


def default_batch(world: int, weak: bool = False, steps: int = 0) -> int:
    """Frames per launch.  N = 1: 4 when the timed frames are whole
    quadruples (steps a multiple of 4, or steps not given), else 2 for whole
    pairs, else 1: a launch of several frames runs past the other launches'
    tails with one learned order for all (round 5, 2 against 1, A/B on one
    box: config 3 0.1190-0.1200 ms per frame against 0.1214-0.1222, config 5
    1.156-1.164 against 1.174, config 6 0.1223-0.1239 against 0.1234-0.1239;
    profiles/r05/r5ar, r5as.  Round 6, 4 against 2 on the final walk: config
    3 at the driver's 20 steps 0.1172 against 0.1214 ms (4 runs each), at 200
    steps 0.1141 against 0.1148, config 5 1.127 against 1.143 and 1.127
    against 1.140; profiles/r06/r6ag, r6af); a frame count that is not a
    multiple would end on a smaller launch of a new launch key.  N > 1, weak scaling: N (a launch is a step, this
    rank's share of the step's N frames: one frame of work, the shape of an
    N = 1 launch).  N > 1, strong scaling: N / 2 (about half a frame of work
    per launch): a rank's 1/8 share of one frame is too small a launch to
    run past its own tail (rank emulation at N = 8, 200 steps:
    profiles/r03/evidence_r3c/emu.jsonl, 3.9x with 1 frame per launch
    against 6.3-7.7x with 4).  At most 16."""
    if world == 1:
        return 4 if steps % 4 == 0 else (2 if steps % 2 == 0 else 1)
    return max(1, min(16, world if weak else world // 2))


def default_root_weight(world: int) -> float:
    """bands: rank 0's weight in the band deal (the others weigh 1).  Rank 0
    also receives the other ranks' shares of every frame and assembles the
    frame, device work the other ranks do not do (at the
    driver's 20 steps rank 0 weighted 0.7 of 8 finished 10% before the
    others, 1.0 of 2 5% after: profiles/r03/batch/r3s)."""
    if world == 1:
        return 1.0
    return 0.9 if world == 2 else (0.85 if world <= 4 else 0.8)


# N > 1: only the tiles costing at least this percentage of the costliest go
# first in the heavy-first order, the rest keep their raster order (rt option
# order_split; a rank's batched launch of band shares runs faster with the
# waves at once on neighbouring tiles; neutral at N = 1)
ORDER_SPLIT_N_GT_1 = 15


def default_span_weight(world: int) -> float:
    """spans: rank 0's span relative to the others' (it also receives every
    other span of the batch).  Emulated at the driver's 20 steps
    (profiles/r05/r5v, r5w): N = 2 1.0 (0.1437 ms per step, both ranks even;
    0.9 leaves rank 1 the slower), N = 4 0.9 (0.162 vs 0.171 at 1.0), N = 8
    0.8 (0.163 vs 0.171 at 0.9)."""
    return 1.0 if world <= 2 else (0.9 if world <= 4 else 0.8)


def default_span_batch(world: int) -> int:
    """spans: frames per exchange batch (bench.py fits it to divide the timed
    frames).  Fewer, larger batches cost the launch streams less host order
    (N = 8 at 200 steps: 64 frames 0.143 ms per step, 32 0.146; r5v), but the
    batch exchanged after the last trace is exposed: 32 at N = 2 and 8, 16 at
    N = 4 (0.162 vs 0.170 ms per step at 20 steps, r5w)."""
    return 16 if world == 4 else 32


def default_piece_weight(world: int) -> float:
    """pieces: rank 0's piece relative to the others' (its receive and
    assembly of every frame are work the other ranks do not do)."""
    return 1.0


def camera_path(cfg, kind: str, n: int, first: int = 0):
    """The cameras of frames first .. first + n - 1."""
    from rtamd import configs
    if kind == "static":
        cam = cfg.camera()
        return [cam] * n
    out = []
    ox, oy, oz = -25.0, 30.0, 140.0                 # VulkanApp.java:132-138
    rad = math.hypot(ox, oz)
    a0 = math.atan2(oz, ox)
    for k in range(first, first + n):
        a = a0 + math.radians(0.5) * k
        out.append(configs.Camera((rad * math.cos(a), oy, rad * math.sin(a)), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0),
                                  20.0, cfg.width / cfg.height))
    return out


def file_sha16(path: str) -> str:
    import hashlib
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


# ---- rank launcher -----------------------------------------------------------
# `python bench.py --gpus N` with no launcher (WORLD_SIZE unset) starts its own
# N ranks: N fresh child processes of this script, one per GPU, each with
# RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as
# torch.distributed.run sets them.  The parent never touches the GPU (it does
# not import torch): it only relays rank 0's stdout (the JSON line), passes
# every rank's stderr through, and exits with the first failing rank's status,
# ending the other ranks when one fails or the whole job outlives
# --launch-timeout.  Under torch.distributed.run (WORLD_SIZE set) bench.py runs
# as that rank directly.


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_plan(argv, n: int, port: int, base_env=None, script: str = None):
    """The N child processes of a self-launched run: (command, env) per rank."""
    base = dict(os.environ if base_env is None else base_env)
    cmd = [sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv)
    plan = []
    for r in range(n):
        env = dict(base)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_LAUNCHED="1")
        plan.append((cmd, env))
    return plan


def launch_ranks(plan, timeout_s: float, out=None, poll_s: float = 0.2) -> int:
    """Run the ranks of `plan` (spawn_plan) to completion: rank 0's JSON line is
    relayed to `out` (default sys.stdout); its other stdout lines and the other
    ranks' stdout go to stderr.  Returns 0 when every rank exits 0; otherwise the first
    failing rank's exit status (124 on timeout), after ending the others."""
    import signal
    import subprocess
    import threading
    out = out or sys.stdout
    procs = []
    for r, (cmd, env) in enumerate(plan):
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr,
                                      start_new_session=True))

    def relay():
        # rank 0's JSON line to stdout; anything else it prints there (gloo's
        # connection notes) to stderr, so stdout holds the one JSON line
        for line in iter(procs[0].stdout.readline, b""):
            text = line.decode(errors="replace")
            dst = out if text.lstrip().startswith("{") else sys.stderr
            dst.write(text)
            dst.flush()

    th = threading.Thread(target=relay, daemon=True)
    th.start()
    t_end = time.monotonic() + timeout_s
    status = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            r, c = bad[0]
            log(f"launcher: rank {r} exited with status {c}; ending the other ranks")
            status = c if c > 0 else 128 - c           # a signal -s reads as 128 + s, like a shell
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > t_end:
            log(f"launcher: ranks still running after {timeout_s:.0f} s; ending them")
            status = 124
            break
        time.sleep(poll_s)
    for p in procs:                                    # end what is left: SIGTERM, then SIGKILL
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.monotonic() + 10.0
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
    th.join(timeout=5.0)
    return status


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 frames of config 3 are ~60 ms: with 4 launches in flight, 20 steps
    # spend a fifth of the timed region filling and draining the pipeline.
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, help="BASELINE config index (3 = headline)")
    ap.add_argument("--partition", choices=("bands", "tiles", "pieces", "spans"), default="spans",
                    help="N > 1: how a frame is tiled over the ranks: bands = weighted interleaved row bands; tiles = gx x gy rectangles (2 x 2 at N = 4); pieces = N contiguous row "
                         "pieces rotated frame by frame (a launch of N frames holds every piece once); spans = "
                         "one contiguous span of each exchange batch's rows per rank (whole frames, a run of "
                         "bands at its ends), received by rank 0 straight into the frames (no assembly; the default)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="N > 1: weak = a step is N frames of the render loop, each tiled over all ranks and "
                         "gathered (every rank traces one frame's worth per step; default); strong = a step is "
                         "one frame tiled over all ranks")
    ap.add_argument("--band", type=int, default=8, help="band height (rows) for N > 1 (8 = one wave-tile row)")
    ap.add_argument("--deal", choices=("auto", "rotate", "fixed"), default="auto",
                    help="bands: rotate = the weighted deal runs on over N frames (one band list per frame, "
                         "rtamd.dist.dealt_bands), so a launch of N frames gives every rank other than 0 the "
                         "same rows to a band; fixed = the same bands in every frame; auto = rotate where the "
                         "fixed deal gives the ranks other than 0 unequal bands (N = 8 at 1080 rows: 18 / 17; "
                         "emulated 6.69-6.83x rotate vs 5.90-5.91x fixed, profiles/r03/emulation/r3dl)")
    ap.add_argument("--root-weight", type=float, default=-1.0,
                    help="bands: rank 0's weight in the band deal, the others weigh 1 (-1 = default_root_weight)")
    ap.add_argument("--inflight", type=int, default=0, help="launches in flight per rank (0 = default_inflight)")
    ap.add_argument("--batch", type=int, default=0, help="frames per launch (whole / bands; 0 = default_batch)")
    ap.add_argument("--exchange-every", type=int, default=0,
                    help="N > 1: frames per exchange batch (a multiple of --batch; 0 = default_span_batch for "
                         "spans, launches in flight x batch otherwise; spans fit it to divide the timed frames)")
    ap.add_argument("--send-lag", type=int, default=1,
                    help="spans: a sender sends each batch's span this many batches after queueing it (the host "
                         "waits for the batch's launches to end then; the ring grows to lag + 2 slots)")
    ap.add_argument("--ring", type=int, default=2,
                    help="N > 1: exchange batches of slots in the ring (>= 2); a batch's slots are retraced only "
                         "after the exchange ring - 1 batches back")
    ap.add_argument("--wire", choices=("rgb", "rgba"), default="rgba",
                    help="spans: rgb = the RGBA8 rows travel as RGB (the alpha byte is always 255, "
                         "compute_dynamic_ray.comp:235), 3/4 of the bytes over each xGMI link, packed and "
                         "unpacked by rt_pack_rgb / rt_unpack_rgb (emulated 5%% slower at N = 8, profiles/r05/"
                         "emulation/r5ap; it pays only where a link is the bound, DESIGN.md §6)")
    ap.add_argument("--span-launch-frames", type=int, default=2,
                    help="spans: consecutive frames of a rank's span per launch (1..16; rt_render_batch_runs_device; "
                         "2, the default: two frames of work per launch as at N = 1, and a span-end run goes with "
                         "its neighbouring whole frame. Emulated on config 3 at 20 steps, slowest rank against 1 "
                         "frame per launch: N = 2 0.158 vs 0.169 ms per step, N = 4 0.1626 vs 0.1643, N = 8 "
                         "0.170 vs 0.169; profiles/r06/r6g, r6i)")
    ap.add_argument("--span-cut", choices=("frames", "bands"), default="bands",
                    help="spans: frames = cut each exchange batch at frame boundaries (every launch a whole "
                         "frame; rank 0 its weighted share rounded, the others' extra frames rotating from batch "
                         "to batch); bands = cut at band boundaries, exactly weighted (a band run at a span's ends)")
    ap.add_argument("--last-pieces", choices=("on", "off"), default="on",
                    help="spans: the last exchange batch of a phase travels launch by launch (each "
                         "launch's rows sent as it ends), so only the last launch's transfer is left "
                         "after the traces (DESIGN.md §6)")
    ap.add_argument("--piece-wait", choices=("host", "device"), default="host",
                    help="spans, --last-pieces: each piece's send waits for its launch on the host, or on the "
                         "device (the exchange stream waits for the launch's event; the host queues every piece)")
    ap.add_argument("--gather", choices=("rgba", "radiance"), default="rgba",
                    help="N > 1: radiance = gather the float radiance beside the RGBA8 frame")
    ap.add_argument("--camera-path", choices=("static", "orbit"), default="static")
    ap.add_argument("--exchange-priority", type=int, default=1, choices=(0, 1, 2),
                    help="N > 1: 1 = the collective's stream and the assembly stream at high priority, so the "
                         "exchange is not starved of workgroup slots by the traces in flight; 2 = on rank 0 only "
                         "(the senders' copies wait for slots); 0 = normal priority")
    ap.add_argument("--assembly-priority", choices=("high", "normal"), default="high",
                    help="N > 1, bands / pieces: the rank-0 assembly (index_select) on the exchange stream at high "
                         "priority, or on a normal-priority stream of its own that a ring slot's reuse does not wait "
                         "for")
    ap.add_argument("--bracket", choices=("lean", "join"), default="lean",
                    help="timed region: lean = the launch streams start right after the device synchronisation "
                         "and the closing device synchronisation joins them; join = they also wait on / are joined "
                         "into the main stream around the region (two cross-queue hops)")
    ap.add_argument("--set", default="", help="schedule options name=value,... (rt_set_option) before timing")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lanes", action="store_true", help="skip the lane-utilisation diagnostic launch")
    ap.add_argument("--no-single", action="store_true", help="N > 1: skip rank 0's one-GPU timing")
    ap.add_argument("--no-pcie", action="store_true", help="N = 1: skip the PCIe-inclusive rt_render_async rate")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample time")
    ap.add_argument("--settle-max", type=int, default=3000, help="at most this many settle launches")
    ap.add_argument("--pcie-warm", type=int, default=200,
                    help="untimed frames before the PCIe-inclusive rate (8: 0.41 ms per frame, 200: 0.345; r3z)")
    ap.add_argument("--settle-s", type=float, default=3.0,
                    help="untimed frames before the warmup steps: this many seconds of counting-pass time "
                         "(5 to --settle-max launches; a GPU that has idled runs its first launches slower: "
                         "N = 1 at 20 steps 0.1240-0.1256 ms per frame against 0.1253-0.1292 with 0.4 s and "
                         "100 launches, profiles/r05/r5bn; N > 1 keeps 0.4 s and 100)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC per launch of each config (tools/pmc_traffic.py: SQ_INSTS_VMEM_RD, HBM bytes) for "
                         "the roofline")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N > 1 without a launcher: the spawned ranks are ended after this many seconds")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, before anything touches the GPU
        plan = spawn_plan(sys.argv[1:], args.gpus, free_port())
        log(f"launcher: starting {args.gpus} ranks (one process per GPU, MASTER_ADDR 127.0.0.1 port "
            f"{plan[0][1]['MASTER_PORT']})")
        sys.exit(launch_ranks(plan, args.launch_timeout))

    import numpy as np
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import configs
    from rtamd._lib import CameraUBO, Stats, check
    from rtamd import dist as rdist
    from rtamd.dist import (SharePlan, ShareTracer, SpanPlan, SpanTracer, TilePlan, assemble_shares, assemble_tiles,
                            band_list,
                            gather_stack, gather_tiles)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    n_visible = torch.cuda.device_count()             # counts devices without initialising HIP
    if not os.environ.get("BENCH_SHARE_GPU") and local_rank >= n_visible:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but only {n_visible} GPU(s) visible; one process "
                         f"per GPU needs --gpus <= the GPUs of the node (BENCH_SHARE_GPU=1 shares them: rehearsal)")
    # BENCH_FORCE_DIST=1 (rehearsal only): the N > 1 code path at any world size,
    # so one GPU runs the partition, its RCCL gather and the rank-0 checks.
    # BENCH_EMULATE=N:r (analysis only, run under torchrun at world size 1):
    # rank r of an N-rank run on this one GPU, its share and its exchange
    # volume (rank 0: the whole batch into a stack + the assembly; rank r > 0:
    # its own rows), the collective an RCCL gather at world size 1 (a device
    # copy).  Frames are not checked; value is the job's rate if every rank
    # ran at this rank's pace.
    emu = os.environ.get("BENCH_EMULATE", "")
    dist_on = world > 1 or os.environ.get("BENCH_FORCE_DIST") == "1" or bool(emu)
    # BENCH_SHARE_GPU=1 (rehearsal only): ranks share the visible GPUs round-robin.
    dev_index = local_rank % torch.cuda.device_count() if os.environ.get("BENCH_SHARE_GPU") else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    backend = None
    if dist_on:
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")     # nccl = RCCL over xGMI
        pg_options = None
        prio_rank = int(emu.split(":")[1]) if emu else rank     # the (emulated) rank
        if backend == "nccl" and (args.exchange_priority == 1 or (args.exchange_priority == 2 and prio_rank == 0)):
            # RCCL's internal stream at high priority: with traces in flight
            # every CU slot is taken, and a normal-priority collective gets
            # slots only as trace waves end
            from torch.distributed import ProcessGroupNCCL
            pg_options = ProcessGroupNCCL.Options()
            pg_options.is_high_priority_stream = True
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None, pg_options=pg_options)

    if emu:
        world, rank = (int(x) for x in emu.split(":"))
    cfg = configs.get(args.config)
    t0 = time.time()
    built = cfg.build()
    log(f"[rank {rank}] built {cfg.name}: {built.triangle_count} flat tris, {built.n_nodes} nodes "
        f"in {time.time() - t0:.2f}s")
    W, H, B = cfg.width, cfg.height, cfg.max_bounces

    renderer = rtamd.Renderer((dev_index,))
    if dist_on:
        renderer.set_option("order_split", ORDER_SPLIT_N_GT_1)
    # --set before the upload: some options shape the uploaded records (leaf_align)
    for kv in filter(None, args.set.split(",")):
        k, v = kv.split("=")
        renderer.set_option(k.strip(), int(v))
    renderer.upload_scene(built)
    L = rtamd.lib()
    ctx = renderer._ctx
    # The PCIe-inclusive rate first, before this process creates its own
    # streams: HIP deals its hardware queues out to streams in creation order,
    # and rt_render_async's slot streams must not share queues with bench's
    # (in the middle of bench.py they did: 0.49 vs 0.36 ms per frame,
    # profiles/r03/emulation/r3l pipeline.jsonl vs bench20_pcie.json).
    pcie = None
    if rank == 0 and not dist_on and args.camera_path == "static" and not args.no_pcie:
        pcie = pcie_rate(renderer, cfg.camera(), W, H, B, warm=args.pcie_warm)

    # ---- partition -------------------------------------------------------
    mode = args.partition if dist_on else "whole"
    weak = dist_on and args.scaling == "weak"
    step_frames = world if weak else 1                         # frames per step (weak scaling: N)
    D = args.inflight if args.inflight > 0 else default_inflight(world)
    F = args.batch if args.batch > 0 else default_batch(world, weak, args.steps)
    F = min(F, 16)
    if mode in ("bands", "pieces", "spans"):
        # one exchange per D launches: every exchange costs the host a
        # collective and an assembly and the streams a join, so fewer, larger
        # ones (one per launch measured 0.426 vs 0.348 ms per step at N = 8,
        # emulated: profiles/r03/evidence_r3h)
        G = args.exchange_every if args.exchange_every > 0 else \
            (default_span_batch(world) if mode == "spans" else D * F)
        G = max(F, (G + F - 1) // F * F)                       # whole launches per exchange batch
        if mode == "spans":
            # a span covers a whole batch: the timed frames are whole batches
            while G > F and (args.steps * step_frames) % G:
                G -= F
    elif mode == "tiles":
        # F frames' tiles per launch (rt_render_batch_rect_device): a rank's
        # launch is a frame's worth of pixels at weak scaling; one quarter-
        # frame launch per frame ran 3-5x slower per pixel (profiles/r06/r6e)
        G = args.exchange_every if args.exchange_every > 0 else D * F
        G = max(F, (G + F - 1) // F * F)
    else:
        G = D * F                                              # N = 1: the slot ring
    # ring of exchange batches: enough for the D launches in flight plus the
    # batch being exchanged
    # spans: a sender sends a batch --send-lag batches after tracing it
    lag = max(1, args.send_lag)
    R = max(lag + 2 if mode == "spans" else 2, args.ring, -(-D * F // G) + 1)
    rad_on = dist_on and args.gather == "radiance"
    band_h = args.band
    plan = tplan = None
    src_index = None
    wire_rgb = False                                  # spans: RGB rows on the wire (below)
    if mode in ("bands", "pieces"):
        rw = args.root_weight if args.root_weight >= 0 else default_root_weight(world)
        deal = args.deal
        if deal == "auto":
            # per-frame band lists (the rotating deal) pack whole bands: only
            # where band_h divides the height
            fixed = [len(band_list(H, band_h, world, r, rw)) for r in range(1, world)]
            deal = "rotate" if fixed and max(fixed) > min(fixed) and H % band_h == 0 else "fixed"
        if (mode == "pieces" or deal == "rotate") and H % band_h:
            raise SystemExit(f"--partition {mode} --deal {deal}: per-frame band lists need --band ({band_h}) to "
                             f"divide the height ({H})")
        plan = SharePlan(H, band_h, world, G, rw, layout="dealt" if deal == "rotate" else "interleave") \
            if mode == "bands" else \
            SharePlan(H, band_h, world, G, rw if args.root_weight >= 0 else default_piece_weight(world),
                      layout="pieces")
        src_index = torch.as_tensor(plan.src, device=dev)
        rgba_slots = torch.empty((R, plan.per_rank, W, 4), dtype=torch.uint8, device=dev)
        rad_slots = torch.empty((R, plan.per_rank, W, 3), dtype=torch.float32, device=dev) if rad_on else None
        px_per_frame = plan.counts[rank] * W
    elif mode == "spans":
        if H % band_h:
            raise SystemExit(f"--partition spans: --band ({band_h}) must divide the height ({H})")
        plan = SpanPlan(H, band_h, world, G, args.root_weight if args.root_weight >= 0 else default_span_weight(world),
                        whole_frames=args.span_cut == "frames", launch_frames=args.span_launch_frames)
        # rank 0: the batch's frames (its own span traced in place, the others
        # received into them); rank r: its span
        rows = G * H if rank == 0 else plan.per_rank
        rgba_slots = torch.empty((R, rows, W, 4), dtype=torch.uint8, device=dev)
        wire_rgb = args.wire == "rgb" and world > 1
        if wire_rgb:
            # RGB on the wire: a sender packs its span, rank 0 receives into a
            # packed landing and writes the RGB bytes into its frames, whose
            # alpha bytes (255, as the kernel writes them) are set here once
            rgb_slots = torch.empty((R, rows, W, 3), dtype=torch.uint8, device=dev)
            if rank == 0:
                rgba_slots.fill_(255)
        rad_slots = torch.empty((R, rows, W, 3), dtype=torch.float32, device=dev) if rad_on else None
        px_per_frame = int(np.mean([plan.batch(b).rows[rank] for b in range(max(1, world - 1))])) * W // G
    elif mode == "tiles":
        tplan = TilePlan(W, H, world, G)
        src_index = torch.as_tensor(tplan.src, device=dev)
        rect = tplan.rects[rank]
        rgba_slots = torch.empty((R, G, tplan.tile_px, 4), dtype=torch.uint8, device=dev)
        rad_slots = torch.empty((R, G, tplan.tile_px, 3), dtype=torch.float32, device=dev) if rad_on else None
        px_per_frame = rect[2] * rect[3]
    else:
        rgba_slots = torch.empty((D, F * H, W, 4), dtype=torch.uint8, device=dev)
        rad_slots = None
        px_per_frame = W * H
    if emu and mode == "spans":
        # rank 0: the others' spans land in its frames (a device copy per span,
        # the bytes RCCL's receives write); rank r: its span read once (the send)
        emu_buf = torch.zeros((plan.per_rank, W, 3 if wire_rgb else 4), dtype=torch.uint8, device=dev)
        emu_land = torch.empty_like(emu_buf)
    elif emu and mode == "tiles":
        # rank 0: the other ranks' tiles land in a stack (the bytes RCCL's gather
        # writes), then the assembly; rank r: its tiles read once (the send)
        emu_t = torch.empty_like(rgba_slots[0])
        emu_tr = torch.empty_like(rad_slots[0]) if rad_on else None
    elif emu:
        if mode not in ("bands", "pieces"):
            raise SystemExit("BENCH_EMULATE emulates --partition bands / pieces / spans / tiles")
        emu_buf = torch.zeros((world * plan.per_rank, W, 4) if rank == 0 else (1,), dtype=torch.uint8, device=dev)
        emu_land = torch.empty_like(emu_buf if rank == 0 else rgba_slots[0])
    streams = [torch.cuda.Stream(dev) for _ in range(D)]
    # the exchange's own stream (and rank 0's assembly) at high priority
    hi = -1 if (dist_on and (args.exchange_priority == 1 or (args.exchange_priority == 2 and rank == 0))) else 0
    main_stream = torch.cuda.Stream(dev, priority=hi)
    torch.cuda.set_stream(main_stream)
    asm_stream = torch.cuda.Stream(dev) if args.assembly_priority == "normal" else main_stream
    # The heavy-pixel bar counts the launches of similar work on the device at
    # once: the D launches in flight.
    renderer.set_option("concurrent_launches", D)

    cam_cache = {}
    cam_arrays = {}

    def cam_of(k):
        if args.camera_path == "static":
            k = 0
        c = cam_cache.get(k)
        if c is None:
            c = cam_cache[k] = camera_path(cfg, args.camera_path, 1, k)[0]
        return c

    span_tracers = {}

    def view_of(k0):
        """spans: the plan of the batch that starts at frame k0 (SpanPlan.batch)."""
        return plan.batch(k0 // G)

    def tracer_of(v):
        """spans: the SpanTracer of batch plan v, and every launch's pointers per
        ring slot, made once per plan (no tensor indexing on the host between
        launches)."""
        t = span_tracers.get(id(v))
        if t is None:
            tr = SpanTracer(ctx, W, H, B, v, rank)
            t = span_tracers[id(v)] = (tr, [[span_ptrs(h, tr.group_row(j)) for j in range(len(tr.groups))]
                                            for h in range(R)])
        return t

    tracer = None if mode == "spans" else \
        ShareTracer(ctx, W, H, B, mode, rank, plan=plan, tplan=tplan, band_h=band_h, batch=G)

    def trace(k0, n, s, rgba_ptr, rad_ptr, stats=False):
        """Frames k0 .. k0 + n - 1 (one exchange batch) in one launch on stream s
        (rtamd.dist.ShareTracer: the tests replay the same launches)."""
        st = Stats() if stats else None
        ck = (0, n) if args.camera_path == "static" else (k0, n)
        cams = cam_arrays.get(ck)
        if cams is None:                              # built once per (frames, count): no host work per launch
            cams = cam_arrays[ck] = (CameraUBO * n)(*[cam_of(k).ubo for k in range(k0, k0 + n)])
        tracer.launch(cams, k0, n, s.cuda_stream, rgba_ptr, rad_ptr, st)
        return st.as_dict() if stats else None

    def trace_span(k0, jl, s, rgba_ptr, rad_ptr, stats=False, one=False):
        """Launch (group) jl of this rank's span of the batch that starts at
        frame k0 (rtamd.dist.SpanTracer); one: entry jl of its frames alone
        (the counting pass)."""
        st_ = Stats() if stats else None
        tr = tracer_of(view_of(k0))[0]
        if one:
            tr.launch(cam_of(k0 + tr.launches[jl][0]).ubo, jl, s.cuda_stream, rgba_ptr, rad_ptr, st_)
            return st_.as_dict() if stats else None
        fs = tr.group_frames(jl)
        ck = (0, len(fs)) if args.camera_path == "static" else (k0 + fs[0], len(fs))
        cams = cam_arrays.get(ck)
        if cams is None:                              # the group's frames are consecutive
            cams = cam_arrays[ck] = (CameraUBO * len(fs))(*[cam_of(k0 + f).ubo for f in fs])
        tr.launch_group(cams, jl, s.cuda_stream, rgba_ptr, rad_ptr, st_)
        return st_.as_dict() if stats else None

    def span_ptrs(h, out_row):
        """Where a span launch writes: row out_row of the span (rank 0: of its
        span inside the batch's frames) in ring slot h."""
        y = out_row + (plan.row0[0] if rank == 0 else 0)
        return rgba_slots[h, y].data_ptr(), (rad_slots[h, y].data_ptr() if rad_on else None)


    def out_ptrs(k0, j):
        """Where launch j (frames k0 ...) writes: its slot of the ring."""
        if mode == "whole":
            return rgba_slots[j % D].data_ptr(), None
        h = (k0 // G) % R
        if mode == "tiles":
            f = k0 % G
            return (rgba_slots[h, f].data_ptr(), rad_slots[h, f].data_ptr() if rad_on else None)
        off = plan.off[rank][k0 % G]
        return (rgba_slots[h, off].data_ptr() if off < plan.per_rank else rgba_slots[h].data_ptr(),
                (rad_slots[h, off].data_ptr() if off < plan.per_rank else rad_slots[h].data_ptr()) if rad_on else None)

    st = {"k": 0, "j": 0}
    slot_last = {}         # N = 1: slot -> (first frame, frames) of its last launch
    batch_streams = []     # streams that traced part of the current exchange batch
    gathered = [None] * R
    last = {"rgba": None, "rad": None, "frames": []}
    ex_evs = []            # (start, end) events of the timed region's exchanges
    ev_pool = []           # timing events created (and their HIP events made) before the timed region

    def timing_event():
        return ev_pool.pop() if ev_pool else torch.cuda.Event(enable_timing=True)

    def assemble(stack, n):
        """Rank 0's frames from a gathered stack, on the assembly stream."""
        if stack is None:
            return None
        if asm_stream is main_stream:
            return assemble_shares(stack, plan, src_index, n)
        asm_stream.wait_stream(main_stream)
        stack.record_stream(asm_stream)
        with torch.cuda.stream(asm_stream):
            return assemble_shares(stack, plan, src_index, n)

    def flush(timed=False):
        """Exchange the frames of the current batch traced so far (N > 1)."""
        k = st["k"]
        n = k % G if k % G else (G if k else 0)
        if not dist_on or n == 0:
            return
        h = ((k - 1) // G) % R
        for s in batch_streams:                       # only the streams that traced this batch
            main_stream.wait_stream(s)
        batch_streams.clear()
        e0 = e1 = None
        if timed:
            e0, e1 = timing_event(), timing_event()
            e0.record(main_stream)
        if emu and mode in ("bands", "pieces"):
            # the exchange volume of rank `rank` of `world`, through a world-size-1 gather
            # (BENCH_EMULATE_NOX=1: no exchange at all, the traces alone)
            if os.environ.get("BENCH_EMULATE_NOX") == "1":
                out = None
            elif rank == 0:
                dist.gather(emu_buf, [emu_land])
                out = assemble(emu_land.reshape(world, plan.per_rank, -1), n)
            else:
                dist.gather(rgba_slots[h], [emu_land])
                out = None
            rad = None
        elif emu and mode == "tiles":
            out = rad = None
            if os.environ.get("BENCH_EMULATE_NOX") == "1":
                pass
            elif rank == 0:
                def land(local):
                    stk = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
                    for r in range(world):                 # its own tiles and the (world - 1) received ones
                        stk[r].copy_(local)
                    return assemble_tiles(stk, tplan, src_index)[:n]
                out = land(rgba_slots[h])
                rad = land(rad_slots[h]) if rad_on else None
            else:
                emu_t.copy_(rgba_slots[h])
                if rad_on:
                    emu_tr.copy_(rad_slots[h])
        elif mode == "tiles":
            out = gather_tiles(rgba_slots[h], tplan, src_index=src_index)
            rad = gather_tiles(rad_slots[h], tplan, src_index=src_index) if rad_on else None
            if out is not None:
                out, rad = out[:n], (rad[:n] if rad is not None else None)
        else:
            stk = gather_stack(rgba_slots[h], plan)
            stk_r = gather_stack(rad_slots[h], plan) if rad_on else None
            out = assemble(stk, n)
            rad = assemble(stk_r, n)
        if timed:
            e1.record(main_stream)
            ex_evs.append((e0, e1))
        ev = torch.cuda.Event()
        ev.record(main_stream)                        # the slots are free once the gather has read them
        gathered[h] = ev
        last["rgba"], last["rad"] = out, rad
        last["frames"] = list(range(k - n, k))
        st["k"] = ((k + G - 1) // G) * G            # the next phase starts a fresh batch

    # ---- spans: the exchange in host order ------------------------------------
    # A wait packet in a launch stream's queue (hipStreamWaitEvent) slows every
    # trace in flight: the dist path at world size 1 ran 0.145 ms per frame with
    # the slot ring's device-side waits against 0.126 host-ordered and 0.124 for
    # N = 1 (profiles/r05/r5q, r5r).  So the launch streams never wait: the host
    # orders the exchange.  A rank r > 0 sends its span of batch b (one
    # batch_isend_irecv, one RCCL group) once the host has seen batch b's
    # launches end, which it checks after queueing batch b + 1 (one batch
    # behind: the GPU always has a batch of traces queued).  Rank 0 posts batch
    # b's receives (one per rank, straight into the batch's frames) before it
    # traces its own span of batch b.  A ring slot is traced into again only
    # after the host has seen its last exchange complete (ring R >= 3 leaves a
    # batch of slack).  Sending each launch's rows as it ended instead (smaller
    # last exchange) ran the senders 25% slower in the emulation (r5t, r5u).
    span_sent = [None] * R     # r > 0: event after the last send out of slot h
    span_recv = [None] * R     # rank 0: (works, landings, k_end, e0) of slot h's pending receive group
    send_q = []                # r > 0: (launch end events, slot, out_row, rows) of traced batches not yet sent

    def span_send(timed):
        e_ends, h, orow, nr, pieces, v = send_q.pop(0)
        if pieces is None:
            for e_end in e_ends:
                e_end.synchronize()                    # host: the batch's launches have ended
            pieces = [(None, orow, nr)]
        e0 = e1 = None
        if timed:
            e0, e1 = timing_event(), timing_event()
            e0.record(main_stream)
        for e_end, y, n in pieces:                     # the last batch of a phase: launch by launch
            if e_end is not None:
                if args.piece_wait == "device":
                    main_stream.wait_event(e_end)      # the send's stream: after this launch
                else:
                    e_end.synchronize()                # host: this launch has ended
            if emu:
                src = rgba_slots[h][y:y + n]
                if wire_rgb:
                    rdist.wire_copy(src, rgb_slots[h][y:y + n], pack=True)   # the alpha byte stays home
                    src = rgb_slots[h][y:y + n]
                if os.environ.get("BENCH_EMULATE_NOX") != "1":
                    emu_land[:n].copy_(src)            # the send's read of the rows
            else:
                rows = (y, n) if e_end is not None else None
                for w in rdist.span_send(rgba_slots[h], v, rgb=rgb_slots[h] if wire_rgb else None,
                                         rad=rad_slots[h] if rad_on else None, rows=rows):
                    w.wait()                           # NCCL: main_stream waits for the send (host free)
        if timed:
            e1.record(main_stream)
            ex_evs.append((e0, e1))
        ev = torch.cuda.Event()
        ev.record(main_stream)
        span_sent[h] = ev

    def span_post_recvs(k0, h, timed, pieces=False):
        """Rank 0: batch k0's receives of every other span, into slot h's
        frames (pieces: one receive per launch of each span)."""
        e0 = None
        if timed:
            e0 = timing_event()
            e0.record(main_stream)
        works, landings = [], []
        v = view_of(k0)
        if emu:
            col = rgb_slots[h] if wire_rgb else rgba_slots[h]
            if os.environ.get("BENCH_EMULATE_NOX") != "1":
                for _, y0, nr in v.recv_slices():      # the bytes the receives write
                    col[y0:y0 + nr].copy_(emu_buf[:nr])
        else:
            works, landings = rdist.span_post_recvs(rgba_slots[h], v, rgb=rgb_slots[h] if wire_rgb else None,
                                                    rad=rad_slots[h] if rad_on else None, pieces=pieces)
        span_recv[h] = (works, landings, k0 + G, e0, v)

    def span_complete_recvs(h, timed):
        works, landings, k_end, e0, v = span_recv[h]
        span_recv[h] = None
        # NCCL: main_stream waits (gloo: the host); the RGB rows into the frames
        rdist.span_finish_recvs(works, landings, rgba_slots[h], v, rgb=rgb_slots[h] if wire_rgb else None)
        if timed and e0 is not None:
            e1 = timing_event()
            e1.record(main_stream)
            ex_evs.append((e0, e1))
        ev = torch.cuda.Event()
        ev.record(main_stream)
        gathered[h] = ev
        if not emu:
            last["rgba"] = rgba_slots[h][:G * H].view(G, H, W, 4)
            last["rad"] = rad_slots[h][:G * H].view(G, H, W, 3) if rad_on else None
            last["frames"] = list(range(k_end - G, k_end))


    def phase_spans(n_frames, evs=None):
        """n_frames frames in whole exchange batches: per batch this rank's
        span launches, round robin over the D streams, the exchange streamed
        behind them in host order (above)."""
        timed = evs is not None
        end = st["k"] + n_frames
        while st["k"] < end:
            k0 = st["k"]
            h = (k0 // G) % R
            # the phase's last batch: its exchange is the one no later trace
            # overlaps, so its spans travel launch by launch (--last-pieces)
            pieces = args.last_pieces == "on" and k0 + G >= end
            if rank == 0:
                if span_recv[h] is not None:           # the slot's last batch: its receives complete
                    span_complete_recvs(h, timed)
                if gathered[h] is not None:
                    gathered[h].synchronize()
                span_post_recvs(k0, h, timed, pieces)
            else:
                while any(q[1] == h for q in send_q):  # the slot's last batch: every launch sent
                    span_send(timed)
                if span_sent[h] is not None:
                    span_sent[h].synchronize()
            used = []
            piece_q = [] if (pieces and rank) else None
            v = view_of(k0)
            tr, tab = tracer_of(v)
            for jl in range(len(tr.groups)):
                j = st["j"]
                s = streams[j % D]
                rp, dp = tab[h][jl]
                if timed:
                    e = (timing_event(), timing_event())
                    e[0].record(s)
                trace_span(k0, jl, s, rp, dp)
                if timed:
                    e[1].record(s)
                    evs.append((e, 1))
                if piece_q is not None:
                    ev = torch.cuda.Event()
                    ev.record(s)
                    orow, n = v.pieces(rank)[jl]
                    if n:
                        piece_q.append((ev, orow, n))
                if s not in used:
                    used.append(s)
                st["j"] = j + 1
            st["k"] = k0 + G
            if rank and v.rows[rank]:
                ends = []
                for s in used:
                    ev = torch.cuda.Event()
                    ev.record(s)
                    ends.append(ev)
                send_q.append((ends, h, 0, v.rows[rank], piece_q, v))
                while len(send_q) > lag:               # the batch before: sent once its launches end
                    span_send(timed)
        # the phase's exchanges complete before it ends
        while send_q:
            span_send(timed)
        if rank == 0:
            k_ends = sorted((span_recv[h][2], h) for h in range(R) if span_recv[h] is not None)
            for _, h in k_ends:
                span_complete_recvs(h, timed)

    def phase(n_frames, evs=None):
        """n_frames frames: launches of up to F frames, never across an exchange batch."""
        if mode == "spans":
            return phase_spans(n_frames, evs)
        end = st["k"] + n_frames
        while st["k"] < end:
            k0 = st["k"]
            n = min(F, end - k0, G - k0 % G)
            j = st["j"]
            s = streams[j % D]
            if dist_on and gathered[(k0 // G) % R] is not None:
                s.wait_event(gathered[(k0 // G) % R])  # the exchange that last read this batch's slots is done
            if dist_on and s not in batch_streams:
                batch_streams.append(s)
            rp, dp = out_ptrs(k0, j)
            if evs is not None:
                e = (timing_event(), timing_event())
                e[0].record(s)
            trace(k0, n, s, rp, dp)
            if evs is not None:
                e[1].record(s)
                evs.append((e, n))
            if mode == "whole":
                slot_last[j % D] = (k0, n)            # the frames slot j mod D now holds
            st["k"] = k0 + n
            st["j"] = j + 1
            if dist_on and st["k"] % G == 0:
                flush(timed=evs is not None)
        if dist_on:
            flush(timed=evs is not None)
        elif F > 1:
            st["k"] = ((st["k"] + G - 1) // G) * G           # the next phase starts a whole slot ring

    # ---- frame indices of the phases (fixed up front, so the counting pass
    # counts exactly the timed frames' cameras): a phase of n frames from
    # frame k ends at k + n, rounded up to a whole exchange batch at N > 1
    def after(k, n):
        # phases start on a whole exchange batch (N > 1) or a whole slot ring
        # (N = 1 with several frames per launch), so every timed launch has
        # the same frame count and launch key (a new key learns, with a
        # stream synchronisation)
        k += n
        return ((k + G - 1) // G) * G if (dist_on or F > 1) else k

    # ---- counting pass (untimed): the timed frames' work ------------------
    K = args.steps * step_frames                       # timed frames
    W_fr = args.warmup * step_frames
    count_rgba = torch.empty((max(rgba_slots[0].numel() // 4, 1), 4), dtype=torch.uint8, device=dev)

    def count_frames(ks):
        """This rank's work in frames ks (counting launches, one frame each);
        spans: in the batches that start at frames ks, one span launch each."""
        tot = {k2: 0.0 for k2 in ("pixels", "segments", "node_visits", "tri_tests", "mat_reads")}
        ms = []
        if mode == "spans":
            for k in ks:
                for jl, (_, _, _, orow) in enumerate(tracer_of(view_of(k))[0].launches):
                    d = trace_span(k, jl, main_stream, count_rgba[orow * W].data_ptr(), None, stats=True, one=True)
                    for k2 in tot:
                        tot[k2] += d[k2]
                    ms.append(d["ms"])
            return tot, ms
        for k in ks:
            d = trace(k, 1, main_stream, count_rgba.data_ptr(), None, stats=True)
            for k2 in tot:
                tot[k2] += d[k2]
            ms.append(d["ms"])
        return tot, ms

    # settle: 5 to --settle-max launches, about settle_s / (the counting
    # launch's device time; a counting launch runs ~4x a plain one), so the
    # timed steps see the steady state of a running render loop (a GPU takes
    # ~0.1 s of load to settle: --settle-s), then the W warmup steps.  Agreed
    # over the ranks, so every rank runs the same collectives.  N > 1 settles
    # as round 4 did, 0.4 s and at most 100 launches: longer settles measured
    # no better in the spans emulation at N = 2 and 8 (profiles/r05/emulation/
    # r5bm, r5bp).
    settle_s, settle_max = args.settle_s, args.settle_max
    if dist_on:
        settle_s, settle_max = min(settle_s, 0.4), min(settle_max, 100)
    _, ms0 = count_frames([0])
    est_ms = max(0.05, float(ms0[0]) * F)                  # a launch's counting time
    n_settle = torch.tensor([max(5, 2 * D, min(settle_max, int(settle_s * 1e3 / est_ms)))], dtype=torch.int64,
                            device=dev)
    if dist_on:
        dist.all_reduce(n_settle, op=dist.ReduceOp.MIN)
    n_settle = int(n_settle.item()) * F
    k_t0 = after(after(0, n_settle), W_fr)
    if mode == "spans":
        if args.camera_path == "static" and plan.batch(1) is plan:   # every batch the same span
            one = count_frames([k_t0])[0]
            loc = {k2: v * (K // G) for k2, v in one.items()}
        else:
            loc, _ = count_frames(range(k_t0, k_t0 + K, G))
    elif args.camera_path == "static":
        one = count_frames([k_t0])[0]
        loc = {k2: v * K for k2, v in one.items()}
    else:
        loc, _ = count_frames(range(k_t0, k_t0 + K))
    torch.cuda.synchronize(dev)
    counts = torch.tensor([loc[k2] for k2 in ("pixels", "segments", "node_visits", "tri_tests", "mat_reads")],
                          dtype=torch.float64, device=dev)
    local = counts.clone()
    if emu:
        # the job's work: whole frames of the timed frames' cameras
        tot = {k2: 0.0 for k2 in ("pixels", "segments", "node_visits", "tri_tests", "mat_reads")}
        whole = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
        for k in ([k_t0] if args.camera_path == "static" else range(k_t0, k_t0 + K)):
            sw = Stats()
            check(L.rt_render_tile_device(ctx, C.byref(cam_of(k).ubo), W, H, B, 0, 0, W, H, whole.data_ptr(), None,
                                          main_stream.cuda_stream, C.byref(sw)))
            for k2 in tot:
                tot[k2] += getattr(sw, k2) * (K if args.camera_path == "static" else 1)
        counts = torch.tensor([tot[k2] for k2 in ("pixels", "segments", "node_visits", "tri_tests", "mat_reads")],
                              dtype=torch.float64, device=dev)
    elif dist_on:
        dist.all_reduce(counts)
    pixels, segments, node_visits, tri_tests, mat_reads = [float(x) for x in counts.tolist()]
    log(f"[rank {rank}] {mode}: {K} timed frames, {segments / K:.0f} segments per frame ({segments / pixels:.3f}/px), "
        f"{node_visits / segments:.2f} node visits/seg; {D} launches in flight x {F} frames, exchange every "
        f"{G if dist_on else '-'} frames")

    # ---- settle, warmup, timed ---------------------------------------------
    # the timed launches' and exchanges' events, created and recorded once here:
    # torch makes the HIP event at its first record, which would otherwise be
    # host time between the timed region's first launches
    for _ in range(2 * (K // F + 2) + (2 * (K // G + 2) if dist_on else 0) + D + 2):
        e = torch.cuda.Event(enable_timing=True)
        e.record(main_stream)
        ev_pool.append(e)
    reg = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    reg[0].record(main_stream)
    reg[1].record(main_stream)
    # Settle, then warm up, then time with no host work in between: the GPU's
    # launches slow down after it idles (a frame's kernel ran 1.35 ms at the
    # start of the settle, 1.16-1.20 ms after ~50 launches, and 1.29-1.31 ms
    # again after a 69 ms host pause before the timed region:
    # profiles/r03/r3f/prof3, kernel trace)
    phase(n_settle)
    torch.cuda.synchronize(dev)
    phase(W_fr)
    torch.cuda.synchronize(dev)
    assert st["k"] == k_t0, (st["k"], k_t0)
    evs = []
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    lean = args.bracket == "lean"
    pk_start = renderer.get_option("plain_kernels")
    gc.disable()                                       # no collector pause between the timed launches
    t_start = time.perf_counter()
    if lean:
        # the device is idle: the first launch's stream starts the region, and
        # every stream's last event (launches, exchanges, assembly) ends it
        reg[0].record(streams[0])
    else:
        reg[0].record(main_stream)
        for s in streams:
            s.wait_stream(main_stream)
    phase(K, evs)
    host_ms = (time.perf_counter() - t_start) * 1e3      # the host's enqueue time of the timed launches
    if lean:
        ends = [timing_event() for _ in streams] + ([timing_event()] if asm_stream is not main_stream else [])
        for e, s in zip(ends, streams + ([asm_stream] if asm_stream is not main_stream else [])):
            e.record(s)
        ends.append(timing_event())
        ends[-1].record(main_stream)
    else:
        for s in streams:
            main_stream.wait_stream(s)
        if asm_stream is not main_stream:
            main_stream.wait_stream(asm_stream)
        reg[1].record(main_stream)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    gc.enable()
    pk_timed = renderer.get_option("plain_kernels")
    n_launch = len(evs)
    launch_ms = float(np.mean([a.elapsed_time(b) for (a, b), _ in evs]))
    region_ms = (max(reg[0].elapsed_time(e) for e in ends) if lean else reg[0].elapsed_time(reg[1]))
    frame_ms = region_ms / n_launch                    # device time per launch of the running loop
    ivs = sorted((reg[0].elapsed_time(a), reg[0].elapsed_time(b)) for (a, b), _ in evs)
    busy, cs, ce = 0.0, None, None
    for a0, b0 in ivs:                                 # union of the launches' intervals
        if ce is None or a0 > ce:
            busy += (ce - cs) if ce is not None else 0.0
            cs, ce = a0, b0
        else:
            ce = max(ce, b0)
    busy += (ce - cs) if ce is not None else 0.0
    exchange_ms = float(sum(a.elapsed_time(b) for a, b in ex_evs))
    mine = torch.tensor([rank, px_per_frame, launch_ms, region_ms / K, busy / K, exchange_ms / K, host_ms / K],
                        dtype=torch.float64, device=dev)
    if dist_on and not emu:
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
    else:
        allr = [mine]
    per_rank = [{"rank": int(x[0]), "pixels_per_frame": int(x[1]), "kernel_ms": round(float(x[2]), 4),
                 "device_ms_per_frame": round(float(x[3]), 4), "trace_busy_ms_per_frame": round(float(x[4]), 4),
                 "exchange_ms_per_frame": round(float(x[5]), 4),
                 "host_enqueue_ms_per_frame": round(float(x[6]), 4)} for x in (t.tolist() for t in allr)]

    heavy_used = renderer.get_option("heavy_tiles_used")   # of the last timed launch
    heavy_px_used = renderer.get_option("heavy_pixels_used")
    lanes = lane_utilisation(renderer, L, ctx, lambda: trace(k_t0, 1, main_stream, count_rgba.data_ptr(), None),
                             dev) if not (args.no_lanes or mode == "spans") else None
    verified = None
    single = None
    if dist_on and not emu and rank == 0 and last["rgba"] is not None:
        # the assembled frames (and radiance) equal the frames traced whole on one GPU
        ok = True
        full = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
        fullr = torch.empty((H, W, 3), dtype=torch.float32, device=dev) if rad_on else None
        for i, k in enumerate(last["frames"]):
            c = cam_of(k)
            check(L.rt_render_tile_device(ctx, C.byref(c.ubo), W, H, B, 0, 0, W, H, full.data_ptr(),
                                          fullr.data_ptr() if rad_on else None, main_stream.cuda_stream, None))
            torch.cuda.synchronize(dev)
            ok = ok and torch.equal(last["rgba"][i], full)
            if rad_on:
                ok = ok and torch.equal(last["rad"][i].view(torch.int32), fullr.view(torch.int32))
        verified = bool(ok)
        if not args.no_single:
            # The same frames on this GPU alone: whole frames with the one-GPU
            # defaults (default_batch(1) frames per launch, default_inflight(1)
            # launches in flight), for the speedup of this partition.
            D1 = default_inflight(1)
            F1 = default_batch(1, steps=K)
            renderer.set_option("concurrent_launches", D1)
            fulls = [torch.empty((F1 * H, W, 4), dtype=torch.uint8, device=dev) for _ in range(D1)]

            def one(j, k):
                ubos = (CameraUBO * F1)(*[cam_of(k + f).ubo for f in range(F1)])
                check(L.rt_render_batch_device(ctx, ubos, F1, W, H, B, 0, None, 0, fulls[j % D1].data_ptr(), None,
                                               streams[j % D].cuda_stream, None))
            one(0, k_t0)                              # learns the whole-frame order
            torch.cuda.synchronize(dev)
            for j in range(max(4 * D1, 100)):         # an idle GPU runs its first launches slower (r3g)
                one(j, k_t0 + (j * F1) % K)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for j in range(K // F1):
                one(j, k_t0 + j * F1)
            torch.cuda.synchronize(dev)
            single = time.perf_counter() - t1
            renderer.set_option("concurrent_launches", D)

    gpu_frame = None
    if mode == "whole" and rank == 0:
        # N = 1: the frames the timed loop left in its slots (the last launch of
        # every stream) equal the same frames traced whole, one launch at a time
        # on one stream (rt_render_tile_device)
        ok = bool(slot_last)
        full = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
        for j_slot, (k0, n) in sorted(slot_last.items()):
            for f in range(n):
                check(L.rt_render_tile_device(ctx, C.byref(cam_of(k0 + f).ubo), W, H, B, 0, 0, W, H, full.data_ptr(),
                                              None, main_stream.cuda_stream, None))
                torch.cuda.synchronize(dev)
                ok = ok and torch.equal(rgba_slots[j_slot][f * H:(f + 1) * H], full)
        verified = bool(ok)
        if args.camera_path == "static":
            gpu_frame = full.cpu().numpy()

    # the camera stops (orbit): the first frames at rest, timed one by one (the
    # first repeat of a camera learns its own heavy-first order)
    stop = None
    if args.camera_path != "static" and mode != "spans":
        k_last = k_t0 + K - 1
        ms = []
        for i in range(8):
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            rp, dp = out_ptrs(k_last, 0) if mode != "whole" else (rgba_slots[0].data_ptr(), None)
            trace(k_last, 1, streams[0], rp, dp)
            torch.cuda.synchronize(dev)
            ms.append(round((time.perf_counter() - t1) * 1e3, 4))
        stop = {"ms_per_frame": ms,
                "what": "the camera of the last timed frame traced 8 more times one at a time (launch to "
                        "completion, host clock): the first repeat of a camera is its learning launch (the "
                        "diagnostic build in the reused order, the order then computed on the device with no "
                        "synchronisation, rt_learn.hip), later ones run its own learned order"}

    t = torch.tensor([elapsed, launch_ms, frame_ms], dtype=torch.float64, device=dev)
    if dist_on and not emu:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, launch_ms_max, frame_ms_max = float(t[0]), float(t[1]), float(t[2])

    value = segments / elapsed / 1e6
    # this rank's work per launch of the timed region
    l_seg, l_nodes, l_tris, l_mats, l_pix = [float(x) / n_launch for x in
                                            (local[1], local[2], local[3], local[4], local[0])]
    alg_bytes = 32.0 * l_nodes + 36.0 * l_tris + 16.0 * l_mats + 4.0 * l_pix
    ref_layout_bytes = 48.0 * l_nodes + 48.0 * l_tris + 16.0 * l_mats + 4.0 * l_pix
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    # PMC only from a record of this config and camera path (pmc_key)
    pmc = load_pmc(args.pmc_json, pmc_key(cfg.name, args.camera_path, renderer.get_option("accel_used"),
                                         renderer.get_option("accel_half_used"), F,
                                         renderer.get_option("accel_wide_used"))) \
        if mode == "whole" else None
    walk_mb = round(renderer.walk_bytes() / 2**20, 2)
    roof = roofline(pmc, alg_bytes, ref_layout_bytes, l_seg, launch_ms, frame_ms, n_cu, lanes, walk_mb)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(built, cam_of(k_t0), W, H, B, segments / K, args.cpu_seconds, gpu_frame)

    # production kernels enqueued after the timed region (verification, camera
    # stop): tools/rocprof_union.py cuts them off the end of a kernel trace
    pk_after = renderer.get_option("plain_kernels") - pk_timed
    if rank == 0 or emu:
        gather_kind = "RCCL" if backend == "nccl" else (backend or "none")
        shared = " (ranks share one GPU: rehearsal)" if os.environ.get("BENCH_SHARE_GPU") else ""
        if mode == "whole":
            part = f"one whole frame per step, {D} launches in flight, {F} frame(s) per launch"
        elif mode == "bands":
            part = (f"one frame per step in {band_h}-row bands dealt to {world} ranks by a weighted round robin "
                    f"{'run on over ' + str(world) + ' frames (one band list per frame) ' if plan.lists else ''}"
                    f"(rank 0 weight {plan.root_weight}, rows per rank {plan.counts}), {D} launches in flight x "
                    f"{F} frames per launch, {gather_kind} gather of every {G} frames + rank-0 assembly{shared}")
        elif mode == "pieces":
            part = (f"every frame cut into {world} contiguous pieces of {band_h}-row bands (rows {plan.counts}, "
                    f"rank 0 weight {plan.root_weight}), rank r tracing position (r + f) mod {world} of frame f, {D} "
                    f"launches in flight x {F} frames per "
                    f"launch (one band list per frame), {gather_kind} gather of every {G} frames + rank-0 "
                    f"assembly{shared}")
        elif mode == "spans":
            if plan.whole_frames:
                cut = (f"cut at frame boundaries into {world} contiguous spans of whole frames (rank 0 weight "
                       f"{plan.root_weight}: frames per rank {plan.frame_counts(0)}, the others' extra frames "
                       f"rotating from batch to batch), one launch per frame")
            else:
                cut = (f"cut into {world} contiguous spans of {band_h}-row bands (rank 0 weight {plan.root_weight}, "
                       f"rows per rank {plan.rows}), one launch per frame of a span (whole frames, a band run at "
                       f"either end)")
            part = (f"every batch of {G} frames {cut}, {D} launches in flight, {gather_kind} point-to-point "
                    f"receives of every span straight into rank 0's frames (no assembly){shared}")
        elif mode == "tiles":
            part = (f"one frame per step tiled {tplan.gx} x {tplan.gy} over {world} ranks (tiles "
                    f"{tplan.rects}), {D} frames in flight, {gather_kind} gather of every {G} frames + rank-0 "
                    f"assembly{shared}")
        out = {
            "metric": BASELINE["metric"],
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            # the series this run belongs to (at N = 1 weak and strong are the same work)
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"{'reference asset' if args.config == 6 else 'synthetic'} "
                    f"({cfg.note}; {'default camera' if args.camera_path == 'static' else 'orbiting camera'})",
            "config": {
                "workload": cfg.name,
                "width": W, "height": H, "max_bounces": B,
                "triangles_flat": built.triangle_count, "bvh_nodes": built.n_nodes,
                "segments_per_frame": int(round(segments / K)),
                "node_visits_per_segment": round(node_visits / segments, 3),
                "tri_tests_per_segment": round(tri_tests / segments, 4),
                "camera_path": args.camera_path,
                "partition": part,
                "frames_per_step": step_frames,
                "frames_per_launch": F,
                "launches_in_flight": D,
                "exchange_every_frames": G if dist_on else None,
                "band_h": band_h if mode in ("bands", "pieces", "spans") else None,
                "root_weight": plan.root_weight if plan is not None else None,
                "deal": (("rotate" if plan.lists else "fixed") if mode == "bands" else None),
                "gather": ((("rgb8 on the wire (alpha 255 set on rank 0)" if wire_rgb else "rgba8") +
                            (" + float radiance" if rad_on else "")) if dist_on else None),
                "frames_verified": verified,
                "parallelism": f"{mode}{world}",
                "schedule": {**{k: renderer.get_option(k) for k in ("walk", "wave_tile", "coop_lanes",
                                                                      "heavy_first", "heavy_tiles", "heavy_factor",
                                                                      "heavy_stream", "heavy_pixels",
                                                                      "heavy_pixel_factor", "heavy_cap", "graph",
                                                                      "reuse_order", "order_split", "hw_queues",
                                                                      "coop_window", "coop_window_used",
                                                                      "leaf_align", "leaf_align_used",
                                                                      "accel", "accel_used", "accel_half",
                                                                      "accel_half_used", "accel_wide",
                                                                      "accel_wide_used", "split_bounce",
                                                                      "wave_tile_used")},
                             "concurrent_launches": renderer.get_option("concurrent_launches"),
                             "heavy_tiles_used": heavy_used,
                             "heavy_pixels_used": heavy_px_used},
            },
            "roofline": {
                **roof,
                "kernel": "trace_simple" + (
                    f" (one launch per {F} frame(s): the {heavy_px_used} heaviest pixels one per wave first, then "
                    f"every {8 << renderer.get_option('wave_tile_used')}x{8 >> renderer.get_option('wave_tile_used')} tile "
                    f"without them)" if heavy_px_used > 0 else
                    f" (one launch per {F} frame(s): the {heavy_used} heaviest tiles one pixel per wave first)"
                    if heavy_used > 0 else f" (one launch per {F} frame(s), tiles in the learned order)"),
                "kernel_ms": round(launch_ms, 4),
                "kernel_ms_max_over_ranks": round(launch_ms_max, 4) if dist_on else None,
                "frame_ms_device": round(frame_ms, 4),
                "frame_ms_device_max_over_ranks": round(frame_ms_max, 4) if dist_on else None,
                "launches_in_flight_avg": round(launch_ms / frame_ms, 2),
                "events": "kernel_ms: each launch's own stream, around every launch (after its wait for the "
                          "exchange); frame_ms_device: from an event before the first launch to the last event of "
                          "every stream (bracket lean) or main stream around the region after joining every launch "
                          "stream (bracket join), / launches",
                "bracket": args.bracket,
                "plain_kernels_timed": pk_timed - pk_start,
                "plain_kernels_after_timed": pk_after,
            },
            "per_rank": per_rank,
            "primary_mrays_s": round(pixels / elapsed / 1e6, 2),
            "cpu_baseline": cpu,
            "pcie": pcie,
            "camera_stop": stop,
            "bench_sha16": file_sha16(os.path.abspath(__file__)),
        }
        if emu:
            out["emulated"] = {"world": world, "rank": rank,
                               "what": "EMULATION on one GPU (BENCH_EMULATE): this rank's share and exchange volume "
                                       "only; value = the job's rate if every rank ran at this rank's pace; not a "
                                       "measurement of N GPUs"}
        if single is not None:
            sv = segments / single / 1e6
            out["single_gpu"] = {"value": round(sv, 2), "ms_per_frame": round(single / K * 1e3, 4),
                                 "what": f"the same frames traced whole on rank 0's GPU alone, "
                                         f"{default_batch(1, steps=K)} per launch, {default_inflight(1)} launches "
                                         f"in flight"}
            out["speedup_vs_1gpu"] = round(value / sv, 3)
        print(json.dumps(out), flush=True)
    renderer.close()
    if dist_on:
        dist.destroy_process_group()


def pcie_rate(renderer, cam, W, H, B, n=200, warm=8):
    """rt_render_async: 4 frames in flight into pinned host frames, every frame
    read back over PCIe (tools/pipeline_bench.py's async mode)."""
    from rtamd.engine import PinnedFrame
    S = 4
    frame_segments = renderer.render(cam, W, H, B, stats=True)[2]["segments"]
    renderer.set_option("async_slots", S)
    frames = [PinnedFrame(H, W) for _ in range(S)]
    try:
        pend = []
        for j in range(max(2 * S, warm)):            # learns / warms up
            pend.append(renderer.render_async(cam, W, H, B, frames[j % S]))
            if len(pend) == S:
                renderer.wait(pend.pop(0))
        while pend:
            renderer.wait(pend.pop(0))
        t0 = time.perf_counter()
        for j in range(n):
            pend.append(renderer.render_async(cam, W, H, B, frames[j % S]))
            if len(pend) == S:
                renderer.wait(pend.pop(0))
        while pend:
            renderer.wait(pend.pop(0))
        dt = time.perf_counter() - t0
    finally:
        for f in frames:
            f.close()
    return {"value": round(frame_segments * n / dt / 1e6, 2), "unit": "Mrays/s",
            "ms_per_frame": round(dt / n * 1e3, 4), "frames": n,
            "what": f"rt_render_async, {S} frames in flight, every frame's RGBA8 read back into pinned host memory "
                    f"(readback overlapped with later traces); the rate a host displaying the frames sees"}


def lane_utilisation(renderer, L, ctx, launch, dev):
    """One diagnostic launch of the first timed frame (option diag; outside the
    timed region): per wave, its lockstep steps (diag word 4), cooperative
    windows (5) and its lanes' own steps summed (7).  Lane utilisation = lane
    steps / (64 x wave steps), over the tile waves (the heavy pixels' one-pixel
    waves record zeros)."""
    import numpy as np
    import torch
    from rtamd._lib import check
    renderer.set_option("diag", 1)
    try:
        launch()
        torch.cuda.synchronize(dev)
        n = C.c_size_t()
        check(L.rt_diag_copy(ctx, None, 0, C.byref(n)))
        buf = np.zeros(max(8, n.value), np.uint64)
        check(L.rt_diag_copy(ctx, buf.ctypes.data, n.value, C.byref(n)))
    finally:
        renderer.set_option("diag", 0)
    rec = buf[: n.value // 8 * 8].reshape(-1, 8).astype(np.float64)
    steps, lane_steps, wins = rec[:, 4].sum(), rec[:, 7].sum(), rec[:, 5].sum()
    tile = rec[:, 4] > 0
    return {"lockstep_lane_utilisation": round(lane_steps / (64.0 * steps), 4) if steps else None,
            "lane_steps": int(lane_steps), "wave_steps": int(steps), "coop_windows": int(wins),
            "tile_waves_walking": int(tile.sum()),
            "what": "a diagnostic launch of the first timed frame in the learned order (heavy pixels split out): "
                    "the lanes' own lockstep walk steps / (64 x the waves' lockstep steps), tile waves only; "
                    "coop_windows = 64-node windows of the cooperative tail"}


def pmc_key(config_name: str, camera_path: str, accel: int = 0, half: int = 0, frames: int = 1,
            wide: int = 0) -> str:
    """The key of a PMC record in profiles/pmc_latest.json: the config, the
    camera path unless it is the static default camera, the accel layouts
    unless the scene runs the reference's own tree (accel 0; round 4's
    records), with "h" for option accel_half's records and "w" for option
    accel_wide's, and "@f<F>" for launches of F > 1 frames (a record is per
    launch)."""
    k = config_name if camera_path == "static" else f"{config_name}@{camera_path}"
    k = f"{k}@accel{accel}{'h' if half else ''}{'w' if wide else ''}" if accel else k
    return f"{k}@f{frames}" if frames > 1 else k


def load_pmc(path, config_name):
    """PMC per launch for config_name from profiles/pmc_latest.json
    (tools/pmc_traffic.py), or None."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        tj = json.load(fh)
    return tj.get("configs", {}).get(config_name)


def roofline(pmc, alg_bytes, ref_layout_bytes, l_seg, kernel_ms, frame_ms, n_cu, lanes=None, walk_mb=None):
    """The roofline object of the JSON line (module docstring).

    Headline (round 5): the algorithmic bytes of one launch
    over frame_ms_device, the device time per launch of the running loop (the
    launches' union), so the fraction does not move with the number of launches
    in flight, against the resource that binds: the L2 (34.5 TB/s) when the
    scene is cache-resident (the PMC HBM bytes are a small part of the
    algorithmic bytes, or without PMC: the records one ray walks fit the 8
    XCDs' L2s), else HBM (8 TB/s) with the PMC-measured HBM bytes.  The
    contract's per-launch form (bytes / the mean launch duration, which counts
    the overlap of the launches in flight) is the view "per_launch"."""
    tk = kernel_ms * 1e-3                                   # s per launch (its own duration)
    tf = frame_ms * 1e-3                                    # s per launch of the running loop
    vmem = pmc.get("SQ_INSTS_VMEM_RD") if pmc else None
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    alg_dev = alg_bytes / tf / 1e9
    l2_frac = alg_dev / L2_PEAK_GBS
    hbm_meas = traffic / tf / 1e9 if traffic else None
    if traffic:
        bound = "hbm" if hbm_meas / HBM_PEAK_GBS > l2_frac else "l2"
        why = (f"PMC: HBM {hbm_meas / HBM_PEAK_GBS:.3f} of 8 TB/s against algorithmic bytes "
               f"{l2_frac:.3f} of the L2's 34.5 TB/s over frame_ms_device; the larger binds")
    else:
        bound = "l2" if (walk_mb is not None and walk_mb <= 32.0) else "hbm"
        why = (f"no PMC record of this config: the records one ray walks ({walk_mb} MB) "
               f"{'fit' if bound == 'l2' else 'exceed'} the 8 XCDs' L2s (32 MB)")
    if bound == "l2":
        achieved, peak = alg_dev, L2_PEAK_GBS
        basis = ("achieved = algorithmic bytes per launch (SURVEY.md §8d: 32 B per BVH node visit + 36 B per "
                 "triangle test + 16 B per material read + 4 B per pixel, counted on this walk by a counting launch) "
                 "/ frame_ms_device (the device time per launch of the running loop: the union of the launches in "
                 "flight); peak = the L2 of the 8 XCDs, 34.5 TB/s (MI355X_MICROARCH.md § L2); traffic = PMC HBM "
                 "bytes per launch (FETCH_SIZE x 1024 x 2, tools/pmc.sh), null without a PMC record")
    else:
        achieved = hbm_meas if hbm_meas else alg_dev
        peak = HBM_PEAK_GBS
        basis = ("achieved = " + ("PMC HBM bytes per launch (FETCH_SIZE x 1024 x 2, tools/pmc.sh)" if hbm_meas else
                                  "algorithmic bytes per launch (SURVEY.md §8d)") +
                 " / frame_ms_device (the device time per launch of the running loop); peak = 8 TB/s HBM "
                 "(MI355X_MICROARCH.md)")
    issue_peak = n_cu / TA_NS_PER_VMEM                      # G wave-instructions / s
    issue = vmem / tf / 1e9 if vmem else None
    return {
        "bound": bound,
        "achieved": round(achieved, 1),
        "peak": peak,
        "unit": "GB/s",
        "frac": round(achieved / peak, 4),
        "traffic": traffic,
        "bound_why": why,
        "basis": basis,
        "pmc_source": pmc.get("source") if pmc else None,
        "alg_bytes_per_launch": int(alg_bytes),
        "alg_bytes_per_segment": round(alg_bytes / l_seg, 1),
        "reference_layout_bytes_per_launch": int(ref_layout_bytes),
        "traffic_over_alg": round(traffic / alg_bytes, 4) if traffic else None,
        "views": {
            "per_launch": {
                "what": "SURVEY.md §8(d)'s form: the algorithmic bytes of one launch / kernel_ms, the mean duration "
                        "of one launch (HIP events on its own stream; what rocprofv3 averages), against 8 TB/s HBM. "
                        "With launches in flight kernel_ms spans the overlap, so this fraction falls as more "
                        "launches run at once",
                "achieved": round(alg_bytes / tk / 1e9, 1), "unit": "GB/s",
                "frac": round(alg_bytes / tk / 1e9 / HBM_PEAK_GBS, 4),
            },
            "device_time": {
                "what": "the same algorithmic bytes over frame_ms_device, against the HBM and the L2 peaks",
                "achieved": round(alg_dev, 1), "unit": "GB/s",
                "hbm_frac": round(alg_dev / HBM_PEAK_GBS, 4),
                "l2_peak": L2_PEAK_GBS, "l2_frac": round(l2_frac, 4),
                "reference_layout_hbm_frac": round(ref_layout_bytes / tf / 1e9 / HBM_PEAK_GBS, 4),
            },
            "hbm_measured": {
                "what": "PMC HBM bytes per launch over frame_ms_device: the HBM rate the running loop draws",
                "achieved": round(hbm_meas, 1) if hbm_meas else None, "unit": "GB/s",
                "frac": round(hbm_meas / HBM_PEAK_GBS, 4) if hbm_meas else None,
            },
            "vmem_issue": {
                "what": f"SQ_INSTS_VMEM_RD per launch (PMC) over frame_ms_device against {n_cu} CUs / "
                        f"{TA_NS_PER_VMEM} ns per wave-level global_load_dwordx4 per CU (a builder-measured floor, "
                        f"{TA_NS_SOURCE}; not a guide figure)",
                "achieved": round(issue, 3) if issue else None, "peak": round(issue_peak, 3),
                "unit": "G wave-level vector-memory instructions/s",
                "frac": round(issue / issue_peak, 4) if issue else None,
                "vmem_rd_per_launch": vmem,
                "vmem_rd_per_segment": round(vmem / l_seg, 3) if vmem else None,
            },
            "lane_utilisation": lanes,
        },
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


def cpu_baseline(built, cam, W, H, B, frame_segments, target_s, gpu_frame=None):
    """The oracle on every k-th row of the same frame, all host threads we may use.
    gpu_frame (the timed loop's frame, host RGBA8): the oracle's rows of the
    sample are compared with it (gpu_rows_match), the oracle as the checker."""
    import numpy as np
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
    match = None
    if gpu_frame is not None:
        rgba = oracle_lib.render(*args, row_step=step, radiance=False, n_threads=threads)[0]
        match = bool(np.array_equal(rgba, gpu_frame[::step]))
    what = (f"every {step}th row of the frame" + (f" x {n}" if n > 1 else "")) if step > 1 \
        else f"the whole frame x {n}"
    return {
        "value": round(segs / dt / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{what} ({px} px, {segs} segments, {dt:.2f} s, OpenMP threads {threads})",
        "gpu_rows_match": match,
        "gpu_rows_match_what": "the sample's oracle rows (RGBA8) equal the same rows of the timed loop's frame "
                               "(checked outside the timed CPU sample)" if match is not None else None,
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
