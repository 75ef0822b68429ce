"""bench.py's N > 1 exchange on the GPU, with device tensors.

A gpurun box has one GPU and RCCL refuses two ranks on one GPU, so:

* every rank's share of an exchange batch is traced on this GPU with the
  launches bench.py issues at N > 1 (rtamd.dist.ShareTracer: the band lists of
  SharePlan's "interleave", "dealt" and "pieces" layouts, one list for every
  frame of a launch or one per frame, F = N frames per launch; TilePlan's
  rectangles), into the ranks' exchange buffers at the plan's offsets, RGBA8
  and float radiance;
* the ranks' buffers are stacked as the gather to rank 0 stacks them, and
  rank 0's assembly (assemble_shares / assemble_tiles, one index_select) runs
  on that stack;
* the collective itself, gather_stack / gather_tile_stack, runs over RCCL
  (backend "nccl") at world size 1 on the same buffers.

Every assembled frame (RGBA8 and radiance bits) equals the frame traced whole
on the GPU.  The multi-process collective at world sizes 2-8 runs over gloo on
the CPU (test_dist.py) and in the self-launched one-GPU rehearsal
(`BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo python bench.py --gpus N`).
"""
import ctypes as C
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def rccl_group():
    import torch
    import torch.distributed as dist
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield dist.group.WORLD
    finally:
        dist.destroy_process_group()


def _orbit_cams(W, H, n):
    import math
    from rtamd import configs
    ox, oy, oz = -25.0, 30.0, 140.0
    rad, a0 = math.hypot(ox, oz), math.atan2(oz, ox)
    return [configs.Camera((rad * math.cos(a0 + math.radians(3.0) * k), oy, rad * math.sin(a0 + math.radians(3.0) * k)),
                           (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H) for k in range(n)]


def _whole(renderer, cams, W, H, B):
    """Reference frames: each traced whole on the GPU (RGBA8, radiance)."""
    import torch
    from rtamd import lib
    from rtamd._lib import check
    s = torch.cuda.current_stream()
    out = []
    for c in cams:
        rgba = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
        rad = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
        check(lib().rt_render_tile_device(renderer._ctx, C.byref(c.ubo), W, H, B, 0, 0, W, H, rgba.data_ptr(),
                                          rad.data_ptr(), s.cuda_stream, None))
        out.append((rgba, rad))
    torch.cuda.synchronize()
    return out


def _check(frames, rads, whole, what):
    import torch
    for f, (rgba, rad) in enumerate(whole):
        if not torch.equal(frames[f], rgba):
            bad = torch.nonzero((frames[f] != rgba).any(-1)).cpu().tolist()
            raise AssertionError(f"{what}: frame {f} RGBA8: {len(bad)} pixels differ, first {bad[:8]}")
        assert torch.equal(rads[f].view(torch.int32), rad.view(torch.int32)), f"{what}: frame {f} radiance"


@pytest.mark.parametrize("layout,world,rw", [("interleave", 1, 1.0), ("interleave", 2, 0.9), ("interleave", 4, 0.85),
                                             ("dealt", 8, 0.8), ("dealt", 4, 1.0), ("pieces", 4, 1.0),
                                             ("pieces", 8, 0.7)])
@pytest.mark.parametrize("accel", [0, 8])
def test_share_exchange_bit_exact(renderer, rccl_group, layout, world, rw, accel):
    import torch
    from rtamd import configs
    from rtamd._lib import CameraUBO
    from rtamd.dist import SharePlan, ShareTracer, assemble_shares, gather_stack
    cfg = configs.config2()
    renderer.set_option("accel", accel)
    renderer.upload_scene(cfg.build())
    renderer.set_option("accel", 0)
    W, H, B, band_h = 320, 184, 3, 8          # 23 bands of 8 rows
    F = world                                  # frames per launch (weak scaling: a launch is a step)
    G = 2 * F                                  # frames per exchange batch
    cams = _orbit_cams(W, H, G)
    whole = _whole(renderer, cams, W, H, B)
    plan = SharePlan(H, band_h, world, G, rw, layout=layout)
    src = torch.as_tensor(plan.src, device="cuda:0")
    streams = [torch.cuda.Stream() for _ in range(2)]
    bufs, rbufs = [], []
    for rank in range(world):
        tracer = ShareTracer(renderer._ctx, W, H, B, "bands", rank, plan=plan, band_h=band_h, batch=G)
        rgba = torch.full((plan.per_rank, W, 4), 7, dtype=torch.uint8, device="cuda:0")
        rad = torch.zeros((plan.per_rank, W, 3), dtype=torch.float32, device="cuda:0")
        # the fills above run on the current stream: the launch streams wait
        # for them (without this a fast trace can land before its buffer's fill)
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        for j, k0 in enumerate(range(0, G, F)):
            off = tracer.offset_rows(k0)
            rp = rgba[off].data_ptr() if off < plan.per_rank else rgba.data_ptr()
            dp = rad[off].data_ptr() if off < plan.per_rank else rad.data_ptr()
            ubos = (CameraUBO * F)(*[c.ubo for c in cams[k0:k0 + F]])
            tracer.launch(ubos, k0, F, streams[j % 2].cuda_stream, rp, dp)
        bufs.append(rgba)
        rbufs.append(rad)
    torch.cuda.synchronize()
    frames = assemble_shares(torch.stack(bufs), plan, src)
    rads = assemble_shares(torch.stack(rbufs), plan, src)
    torch.cuda.synchronize()
    _check(frames, rads, whole, f"{layout} N={world}")
    if world == 1:
        # the collective half over RCCL at world size 1, on the same buffers
        stk = gather_stack(bufs[0], plan)
        stk_r = gather_stack(rbufs[0], plan)
        _check(assemble_shares(stk, plan, src), assemble_shares(stk_r, plan, src), whole, "RCCL gather_stack")


@pytest.mark.parametrize("world,rw,lf", [(1, 1.0, 1), (2, 0.9, 1), (4, 0.8, 1), (8, 0.55, 1), (8, 1.0, 1),
                                         (2, 0.9, 2), (4, 0.8, 2), (8, 0.55, 3)])
@pytest.mark.parametrize("accel", [0, 8])
def test_span_exchange_bit_exact(renderer, world, rw, accel, lf):
    """bench.py --partition spans: every rank's span of an exchange batch
    traced with SpanTracer's launch groups (lf frames' band runs each,
    rt_render_batch_runs_device packing them back to back) on 4 streams,
    rank 0's in place in the batch's frames, the others' into span buffers
    that land in rank 0's frames at the plan's rows (what the point-to-point
    receives write; exchange_spans itself runs over gloo in test_dist.py).
    Every frame and its radiance equal the frame traced whole."""
    import torch
    from rtamd import configs
    from rtamd._lib import CameraUBO
    from rtamd.dist import SpanPlan, SpanTracer
    cfg = configs.config2()
    renderer.set_option("accel", accel)
    renderer.upload_scene(cfg.build())
    renderer.set_option("accel", 0)
    W, H, B, band_h = 320, 184, 3, 8          # 23 bands of 8 rows
    G = 4 * world if world > 1 else 4
    cams = _orbit_cams(W, H, G)
    whole = _whole(renderer, cams, W, H, B)
    plan = SpanPlan(H, band_h, world, G, rw, launch_frames=lf)
    col = torch.full((G * H, W, 4), 7, dtype=torch.uint8, device="cuda:0")
    colr = torch.zeros((G * H, W, 3), dtype=torch.float32, device="cuda:0")
    streams = [torch.cuda.Stream() for _ in range(4)]
    spans = []
    j = 0
    for rank in range(world):
        tracer = SpanTracer(renderer._ctx, W, H, B, plan, rank)
        if rank == 0:
            buf, rbuf, base = col, colr, plan.row0[0]
        else:
            buf = torch.full((plan.per_rank, W, 4), 7, dtype=torch.uint8, device="cuda:0")
            rbuf = torch.zeros((plan.per_rank, W, 3), dtype=torch.float32, device="cuda:0")
            base = 0
            spans.append((rank, buf, rbuf))
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        for jl in range(len(tracer.groups)):
            fs = tracer.group_frames(jl)
            orow = tracer.group_row(jl)
            tracer.launch_group((CameraUBO * len(fs))(*[cams[f].ubo for f in fs]), jl, streams[j % 4].cuda_stream,
                                buf[base + orow].data_ptr(), rbuf[base + orow].data_ptr())
            j += 1
    torch.cuda.synchronize()
    for rank, buf, rbuf in spans:
        y0, n = plan.row0[rank], plan.rows[rank]
        col[y0:y0 + n].copy_(buf[:n])
        colr[y0:y0 + n].copy_(rbuf[:n])
    torch.cuda.synchronize()
    _check(col.view(G, H, W, 4), colr.view(G, H, W, 3), whole, f"spans N={world} rw={rw}")


@pytest.mark.parametrize("accel", [0, 8])
@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("size,per_launch", [((322, 181), 1), ((322, 181), 3), ((320, 180), 3)])
def test_tile_exchange_bit_exact(renderer, rccl_group, world, accel, size, per_launch):
    """BASELINE config 4's tile grid (2 x 2 at N = 4): every rank's rectangle
    of every frame of a batch, stacked and assembled; at world size 1 the
    gather runs over RCCL.  per_launch 3: the batch's tiles in one launch
    (rt_render_batch_rect_device, bench.py's tiles mode; odd sizes: uneven
    tiles, one launch per frame at the plan's tile pitch)."""
    import torch
    from rtamd import configs
    from rtamd._lib import CameraUBO
    from rtamd.dist import ShareTracer, TilePlan, assemble_tiles, gather_tile_stack, gather_tiles
    cfg = configs.config2()
    renderer.set_option("accel", accel)
    renderer.upload_scene(cfg.build())
    renderer.set_option("accel", 0)
    (W, H), B, G = size, 3, 3                 # odd sizes: uneven tiles, padded to the largest
    cams = _orbit_cams(W, H, G)
    whole = _whole(renderer, cams, W, H, B)
    plan = TilePlan(W, H, world, G)
    src = torch.as_tensor(plan.src, device="cuda:0")
    s = torch.cuda.current_stream()
    bufs, rbufs = [], []
    for rank in range(world):
        tracer = ShareTracer(renderer._ctx, W, H, B, "tiles", rank, tplan=plan, batch=G)
        rgba = torch.zeros((G, plan.tile_px, 4), dtype=torch.uint8, device="cuda:0")
        rad = torch.zeros((G, plan.tile_px, 3), dtype=torch.float32, device="cuda:0")
        if per_launch == 1:
            for f in range(G):
                tracer.launch((CameraUBO * 1)(cams[f].ubo), f, 1, s.cuda_stream, rgba[f].data_ptr(),
                              rad[f].data_ptr())
        else:
            tracer.launch((CameraUBO * G)(*[c.ubo for c in cams[:G]]), 0, G, s.cuda_stream, rgba[0].data_ptr(),
                          rad[0].data_ptr())
        bufs.append(rgba)
        rbufs.append(rad)
    torch.cuda.synchronize()
    _check(assemble_tiles(torch.stack(bufs), plan, src), assemble_tiles(torch.stack(rbufs), plan, src), whole,
           f"tiles N={world}")
    if world == 1:
        _check(gather_tiles(bufs[0], plan, src_index=src), gather_tiles(rbufs[0], plan, src_index=src), whole,
               "RCCL gather_tiles")
        assert torch.equal(gather_tile_stack(bufs[0], plan)[0], bufs[0])


@pytest.mark.parametrize("band_h,n_frames", [(16, 4), (7, 3)])
def test_rccl_gather_frames_bit_exact(renderer, rccl_group, band_h, n_frames):
    """gather_frames / DistRenderer (the plain interleave of rtamd.dist) over RCCL."""
    import torch
    from rtamd import configs, lib
    from rtamd._lib import check
    from rtamd.dist import DistRenderer, band_row_count, gather_frames
    cfg = configs.config2()
    W, H, B = 320, 180, cfg.max_bounces
    cam = configs.Camera.default(W, H)
    renderer.upload_scene(cfg.build())
    full = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream()
    check(lib().rt_render_bands_device(renderer._ctx, C.byref(cam.ubo), W, H, B, H, 1, 0, full.data_ptr(), None,
                                       s.cuda_stream, None))
    rows = band_row_count(H, band_h, 1, 0)
    slots = torch.zeros((2 * n_frames, rows, W, 4), dtype=torch.uint8, device="cuda:0")
    for k in range(n_frames):
        check(lib().rt_render_bands_device(renderer._ctx, C.byref(cam.ubo), W, H, B, band_h, 1, 0,
                                           slots[n_frames + k].data_ptr(), None, s.cuda_stream, None))
    frames = gather_frames(slots[n_frames:], H, band_h)
    torch.cuda.synchronize()
    assert frames.shape == (n_frames, H, W, 4)
    for k in range(n_frames):
        assert torch.equal(frames[k], full), k
    one = DistRenderer(renderer, band_h=band_h).render(cam, W, H, B)
    torch.cuda.synchronize()
    assert torch.equal(one, full)


@pytest.mark.parametrize("n_px", [1, 3, 4, 1920 * 7, 1920 * 7 + 3])
def test_wire_rgb_round_trip(n_px):
    """The RGB wire (rt_pack_rgb / rt_unpack_rgb, rtamd.dist.wire_copy): RGBA8
    pixels packed to 3 bytes and written back with alpha 255 give the frame's
    pixels back (their alpha is always 255), including the n % 4 tail; the
    packed bytes are the RGB channels in order."""
    import torch
    from rtamd.dist import wire_copy
    g = torch.Generator(device="cpu").manual_seed(n_px)
    src = torch.randint(0, 256, (1, n_px, 4), dtype=torch.uint8, generator=g)
    src[..., 3] = 255
    d = src.to("cuda:0")
    rgb = torch.full((1, n_px, 3), 7, dtype=torch.uint8, device="cuda:0")
    wire_copy(d, rgb, pack=True)
    back = torch.zeros((1, n_px, 4), dtype=torch.uint8, device="cuda:0")
    wire_copy(back, rgb, pack=False)
    torch.cuda.synchronize()
    assert torch.equal(rgb.cpu(), src[..., :3])
    assert torch.equal(back.cpu(), src)


def test_wire_rgb_rejects_misaligned():
    import ctypes as C
    import torch
    from rtamd import lib
    from rtamd._lib import RtError, check
    a = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(RtError):
        check(lib().rt_pack_rgb(a.data_ptr() + 4, a.data_ptr(), 4, None))
    with pytest.raises(RtError):
        check(lib().rt_unpack_rgb(a.data_ptr() + 1, a.data_ptr(), 4, None))
