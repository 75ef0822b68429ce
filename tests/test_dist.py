"""Multi-process frame tiling on CPU (gloo, world_size 2 and 3): the
interleaved-band partition plus the gather to rank 0 reassembles the one-GPU
frame exactly.  The band tracer here is the CPU oracle (the check runs the
same partition / gather / scatter code the GPU path uses)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, band_h, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]
    import torch
    import torch.distributed as dist
    from oracle import oracle_lib
    from rtamd import configs
    from rtamd.dist import band_rows, gather_frame
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = configs.config2()
        built = cfg.build()
        W, H, B = 160, 90, 3
        cam = configs.Camera.default(W, H)
        rows = band_rows(H, band_h, world, rank)
        parts = []
        for y in rows:        # this rank's bands, packed in the kernels' order
            rgba, _, _ = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                           cam.ubo_bytes(), W, H, B, tile=(0, int(y), W, 1), n_threads=1)
            parts.append(rgba)
        local = torch.from_numpy(np.concatenate(parts) if parts else np.zeros((0, W, 4), np.uint8))
        frame = gather_frame(local, H, band_h)
        if rank == 0:
            q.put(frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band_h", [(2, 16), (3, 8)])
def test_band_gather_reassembles_frame(world, band_h):
    from oracle import oracle_lib
    from rtamd import configs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_h, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    built = configs.config2().build()
    cam = configs.Camera.default(160, 90)
    ref, _, _ = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                  cam.ubo_bytes(), 160, 90, 3)
    assert np.array_equal(frame, ref)


def _batch_worker(rank, world, port, band_h, q, rotate=True):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]
    import torch
    import torch.distributed as dist
    from oracle import oracle_lib
    from rtamd import configs
    from rtamd.dist import BatchPlan, batch_band_offset, band_rows, gather_batch, gather_frames
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = configs.config2()
        built = cfg.build()
        W, H, B = 96, 53, 3
        F = world if rotate else 3
        plan = BatchPlan(H, band_h, world, F, rotate)
        local = torch.zeros((F, plan.max_rows, W, 4), dtype=torch.uint8)
        traced = 0
        for f in range(F):
            cam = configs.Camera((-25.0 + 5 * f, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
            rows = band_rows(H, band_h, world, batch_band_offset(f, world, rank) if rotate else rank)
            assert len(rows) == plan.local_rows(rank, f)
            for k, y in enumerate(rows):
                rgba, _, _ = oracle_lib.render(built.model_vertex_data, built.model_material_data,
                                               built.flat_bvh_data, cam.ubo_bytes(), W, H, B,
                                               tile=(0, int(y), W, 1), n_threads=1)
                local[f, k] = torch.from_numpy(rgba[0])
            traced += len(rows)
        q.put(("traced", rank, traced))
        frames = gather_batch(local, plan) if rotate else gather_frames(local, H, band_h)
        if rank == 0:
            q.put(("frames", frames.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band_h", [(2, 16), (3, 8)])
def test_batch_gather_reassembles_frames(world, band_h):
    """Weak-scaling batches: frame f's bands rotate over the ranks, every rank
    traces one frame's worth of rows, and rank 0 reassembles all frames."""
    from oracle import oracle_lib
    from rtamd import configs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, band_h, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    traced = {}
    for _ in range(world + 1):
        item = q.get(timeout=300)
        if item[0] == "traced":
            traced[item[1]] = item[2]
        else:
            got["frames"] = item[1]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    cfg = configs.config2()
    built = cfg.build()
    W, H, B = 96, 53, 3
    assert set(traced.values()) == {H}                       # one frame's rows per rank
    for f in range(world):
        cam = configs.Camera((-25.0 + 5 * f, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
        ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                cam.ubo_bytes(), W, H, B)[0]
        assert np.array_equal(got["frames"][f], ref), f


@pytest.mark.parametrize("world,band_h", [(2, 16), (3, 8)])
def test_bands_steps_gathered_in_one_batch(world, band_h):
    """Strong scaling with the exchange batched: three consecutive one-frame
    steps (rank r traces the bands r of each) gathered by one collective
    (gather_frames, as bench.py does every few steps) give the three frames."""
    from oracle import oracle_lib
    from rtamd import configs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, band_h, q, False)) for r in range(world)]
    for p in procs:
        p.start()
    got = None
    for _ in range(world + 1):
        item = q.get(timeout=300)
        if item[0] == "frames":
            got = item[1]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    built = configs.config2().build()
    W, H, B = 96, 53, 3
    assert got.shape == (3, H, W, 4)
    for f in range(3):
        cam = configs.Camera((-25.0 + 5 * f, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
        ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                cam.ubo_bytes(), W, H, B)[0]
        assert np.array_equal(got[f], ref), f


def _blocks_worker(rank, world, port, q, first_frame, share):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]
    import torch
    import torch.distributed as dist
    from oracle import oracle_lib
    from rtamd import configs
    from rtamd.dist import block_layout, block_sizes, exchange_blocks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = configs.config2()
        built = cfg.build()
        W, H, B = 96, 53, 3
        ids = list(range(first_frame, first_frame + 4))           # one batch of 4 consecutive steps
        bh = max(block_sizes(H, world, share))
        local = torch.zeros((len(ids), bh, W, 4), dtype=torch.uint8)
        frames = torch.zeros((len(ids), H, W, 4), dtype=torch.uint8) if rank == 0 else None
        traced = []
        for i, f in enumerate(ids):
            cam = configs.Camera((-25.0 + 5 * f, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
            lay = block_layout(H, world, f, share)
            assert sorted(lay) == [(a, b) for a, b in zip([0] + [y for _, y in sorted(lay)][:-1],
                                                          [y for _, y in sorted(lay)])]   # tiles the frame
            y0, y1 = lay[rank]
            if y1 > y0:
                rgba, _, _ = oracle_lib.render(built.model_vertex_data, built.model_material_data,
                                               built.flat_bvh_data, cam.ubo_bytes(), W, H, B,
                                               tile=(0, y0, W, y1 - y0), n_threads=1)
                (frames[i, y0:y1] if rank == 0 else local[i, : y1 - y0]).copy_(torch.from_numpy(rgba))
            traced.append(y0)
        q.put(("traced", rank, traced))
        exchange_blocks(frames, local, ids, H, share)
        if rank == 0:
            q.put(("frames", frames.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,first,share", [(2, 0, 1.0), (3, 5, 1.0), (4, 2, 0.6), (3, 1, 0.0)])
def test_blocks_exchange_assembles_frames(world, first, share):
    """Rotating row blocks exchanged point to point (rtamd.dist.exchange_blocks,
    an option of the library; bench.py's partitions gather instead): frame k
    lays the ranks' pieces out in the rotated order k, k+1, ...; rank 0 traces its piece (of
    root_share x H / N rows, 0 to a full share) in place and receives every
    other rank's piece straight into the frame (one batch of point-to-point
    receives).  53 rows over 3 / 4 ranks leaves unequal pieces.  Every frame of
    the batch equals the oracle's frame."""
    from oracle import oracle_lib
    from rtamd import configs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_blocks_worker, args=(r, world, port, q, first, share)) for r in range(world)]
    for p in procs:
        p.start()
    got, traced = None, {}
    for _ in range(world + 1):
        item = q.get(timeout=300)
        if item[0] == "frames":
            got = item[1]
        else:
            traced[item[1]] = item[2]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for i in range(4):                                    # each frame's pieces start at different rows
        assert len({traced[r][i] for r in range(world)}) == world or share == 0.0
    built = configs.config2().build()
    W, H, B = 96, 53, 3
    for i, f in enumerate(range(first, first + 4)):
        cam = configs.Camera((-25.0 + 5 * f, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
        ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                cam.ubo_bytes(), W, H, B)[0]
        assert np.array_equal(got[i], ref), f


# --- weighted bands, batches of frames, tile grids, radiance (bench.py's N > 1) ---

def _cams(n, W, H):
    from rtamd import configs
    return [configs.Camera((-25.0 + 7 * f, 30.0 - 2 * f, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
            for f in range(n)]


def _share_worker(rank, world, port, q, kind, arg, n_frames, W, H, B):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]
    import torch
    import torch.distributed as dist
    from oracle import oracle_lib
    from rtamd import configs
    from rtamd.dist import SharePlan, SpanPlan, TilePlan, exchange_spans, gather_shares, gather_tiles
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        built = configs.config2().build()
        args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data)
        cams = _cams(n_frames, W, H)
        traced = 0
        if kind == "spans":
            # bench.py --partition spans: rank 0 traces its span in place in
            # the batch's frames, the others into a span buffer; one group of
            # point-to-point receives lands every span in rank 0's frames
            band_h, rw, wire, pieces, whole_b = arg[:5]
            lf = arg[5] if len(arg) > 5 else 1
            # whole_b >= 0: cut at frame boundaries, batch whole_b's plan (its
            # extra frames on its own ranks); lf: frames per launch group (the
            # pieces follow the groups)
            plan = SpanPlan(H, band_h, world, n_frames, rw, whole_frames=whole_b >= 0,
                            launch_frames=lf).batch(max(0, whole_b))
            col = torch.zeros((n_frames * H, W, 4), dtype=torch.uint8) if rank == 0 else None
            rgb = None
            if wire == "rgb":
                # the RGB wire: rank 0's frames get their alpha bytes once, the rows travel as RGB
                rgb = torch.zeros(((n_frames * H) if rank == 0 else plan.per_rank, W, 3), dtype=torch.uint8)
                if rank == 0:
                    col[:, :, 3] = 255
            colr = torch.zeros((n_frames * H, W, 3), dtype=torch.float32) if rank == 0 else None
            span = torch.zeros((plan.per_rank, W, 4), dtype=torch.uint8) if rank else None
            spanr = torch.zeros((plan.per_rank, W, 3), dtype=torch.float32) if rank else None
            base = plan.row0[0] if rank == 0 else 0
            for f, lo, hi, orow in plan.launches[rank]:
                a, r, _ = oracle_lib.render(*args, cams[f].ubo_bytes(), W, H, B,
                                            tile=(0, lo * band_h, W, (hi - lo) * band_h), n_threads=1)
                o = base + orow
                n = (hi - lo) * band_h
                (col if rank == 0 else span)[o:o + n] = torch.from_numpy(a)
                (colr if rank == 0 else spanr)[o:o + n] = torch.from_numpy(r)
                traced += W * n
            exchange_spans(col, span, plan, rgb=rgb, pieces=pieces)
            exchange_spans(colr, spanr, plan, pieces=pieces)
            out = col.view(n_frames, H, W, 4) if rank == 0 else None
            outr = colr.view(n_frames, H, W, 3) if rank == 0 else None
        elif kind == "tiles":
            plan = TilePlan(W, H, world, n_frames)
            x0, y0, w, h = plan.rects[rank]
            rgba = torch.zeros((n_frames, plan.tile_px, 4), dtype=torch.uint8)
            rad = torch.zeros((n_frames, plan.tile_px, 3), dtype=torch.float32)
            for f in range(n_frames):
                if w * h:
                    a, r, _ = oracle_lib.render(*args, cams[f].ubo_bytes(), W, H, B, tile=(x0, y0, w, h), n_threads=1)
                    rgba[f, : w * h] = torch.from_numpy(a.reshape(-1, 4))
                    rad[f, : w * h] = torch.from_numpy(r.reshape(-1, 3))
                    traced += w * h
            out = gather_tiles(rgba, plan)
            outr = gather_tiles(rad, plan)
        elif kind in ("pieces", "dealt"):
            # rt_render_batch_lists_device's packing: one launch of all the
            # batch's frames, list position k of frame f at rows off + k * band_h
            band_h, rw = arg
            plan = SharePlan(H, band_h, world, n_frames, rw, layout=kind)
            rgba = torch.zeros((plan.per_rank, W, 4), dtype=torch.uint8)
            rad = torch.zeros((plan.per_rank, W, 3), dtype=torch.float32)
            lists = plan.launch_lists(rank, 0, n_frames)
            for f in range(n_frames):
                for k, b in enumerate(lists[f]):
                    if b < 0:
                        continue
                    a, r, _ = oracle_lib.render(*args, cams[f].ubo_bytes(), W, H, B, tile=(0, int(b) * band_h, W, band_h),
                                                n_threads=1)
                    o = plan.off[rank][f] + k * band_h
                    rgba[o: o + band_h] = torch.from_numpy(a)
                    rad[o: o + band_h] = torch.from_numpy(r)
                    traced += W * band_h
            out = gather_shares(rgba, plan)
            outr = gather_shares(rad, plan)
        else:
            band_h, rw, rotate = arg
            plan = SharePlan(H, band_h, world, n_frames, rw, rotate=rotate)
            rgba = torch.zeros((plan.per_rank, W, 4), dtype=torch.uint8)
            rad = torch.zeros((plan.per_rank, W, 3), dtype=torch.float32)
            for f in range(n_frames):
                for i, y in enumerate(plan.frame_rows(rank, f)):   # this rank's rows, packed as the kernel packs them
                    a, r, _ = oracle_lib.render(*args, cams[f].ubo_bytes(), W, H, B, tile=(0, int(y), W, 1),
                                                n_threads=1)
                    rgba[plan.off[rank][f] + i] = torch.from_numpy(a[0])
                    rad[plan.off[rank][f] + i] = torch.from_numpy(r[0])
                    traced += W
            out = gather_shares(rgba, plan)
            outr = gather_shares(rad, plan)
        q.put(("traced", rank, traced))
        if rank == 0:
            q.put(("frames", out.numpy(), outr.numpy()))
    finally:
        dist.destroy_process_group()


def _run_share(world, kind, arg, n_frames=3, W=96, H=53, B=3):
    from oracle import oracle_lib
    from rtamd import configs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_share_worker, args=(r, world, port, q, kind, arg, n_frames, W, H, B))
             for r in range(world)]
    for p in procs:
        p.start()
    got, traced = None, {}
    for _ in range(world + 1):
        item = q.get(timeout=600)
        if item[0] == "frames":
            got = item[1:]
        else:
            traced[item[1]] = item[2]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    built = configs.config2().build()
    for f, cam in enumerate(_cams(n_frames, W, H)):
        ref, rad, _ = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                        cam.ubo_bytes(), W, H, B)
        assert np.array_equal(got[0][f], ref), f
        assert np.array_equal(got[1][f].view(np.uint32), rad.view(np.uint32)), f
    return traced


@pytest.mark.parametrize("world,band_h,root_weight", [(4, 8, 0.6), (4, 4, 1.0), (8, 4, 0.7)])
def test_weighted_bands_batch_reassembles_frames_and_radiance(world, band_h, root_weight):
    """bench.py's N > 1 default: a weighted band deal (rank 0 lighter), each
    rank's shares of a batch of 3 frames (different cameras) packed back to
    back as rt_render_batch_device writes them, one gather of the RGBA8 and
    one of the float radiance to rank 0, one index_select each: every frame
    and its radiance equal the oracle's, bit for bit, and rank 0 traced fewer
    pixels than the others when its weight is below 1."""
    traced = _run_share(world, "bands", (band_h, root_weight, False))
    assert sum(traced.values()) == 3 * 96 * 53
    if root_weight < 1.0:
        assert traced[0] <= min(traced[r] for r in range(1, world))


@pytest.mark.parametrize("world", [4, 2])
def test_tile_grid_reassembles_frames_and_radiance(world):
    """--partition tiles: the screen tiled 2 x 2 over 4 ranks (BASELINE config 4)
    or 2 x 1; 96 x 53 leaves unequal tiles.  Tiles and radiance gathered and
    assembled equal the oracle's frames."""
    traced = _run_share(world, "tiles", None, n_frames=2)
    assert sum(traced.values()) == 2 * 96 * 53


def test_rotating_bands_weak_scaling_8_ranks():
    """--partition frames at 8 ranks: in frame f rank r traces the bands of
    position (r + f) mod 8, so over 8 frames every rank traces one frame's
    worth of rows; the 8 frames reassemble."""
    traced = _run_share(8, "bands", (4, 1.0, True), n_frames=8, W=48, H=40, B=2)
    assert set(traced.values()) == {48 * 40}


@pytest.mark.parametrize("world,n_frames,band_h,rw", [(8, 8, 4, 1.0), (3, 6, 4, 1.0), (2, 2, 8, 1.0),
                                                      (4, 8, 2, 0.7), (8, 8, 2, 0.85)])
def test_rotating_pieces_weak_scaling(world, n_frames, band_h, rw):
    """--partition pieces (bench.py's weak-scaling option): every frame cut
    into world contiguous pieces of whole bands (sizes differ by a band), rank
    r tracing piece (r + f) mod world of frame f, all the batch's frames in
    one launch with one band list per frame (-1 padded to the longest piece,
    rt_render_batch_lists_device's packing); one gather and one index_select:
    every frame and its radiance equal the oracle's, and over world frames
    every rank traced exactly one frame's worth of rows; with a root weight
    below 1 (rank 0's piece smaller, the cut points moving with it) rank 0
    traced less than every other rank."""
    W, H = 48, 40
    traced = _run_share(world, "pieces", (band_h, rw), n_frames=n_frames, W=W, H=H, B=2)
    assert sum(traced.values()) == n_frames * W * H
    if rw == 1.0:
        assert set(traced.values()) == {n_frames // world * W * H}
    else:
        assert traced[0] < min(traced[r] for r in range(1, world))


@pytest.mark.parametrize("world,n_frames,band_h,rw", [(8, 8, 2, 0.8), (4, 8, 2, 0.85), (3, 3, 4, 1.0)])
def test_dealt_bands_weak_scaling(world, n_frames, band_h, rw):
    """bench.py --partition bands --deal rotate: the weighted band deal runs
    on over world frames (rtamd.dist.dealt_bands), one band list per frame
    packed as rt_render_batch_lists_device writes them; one gather and one
    index_select give every frame and its radiance bit for bit, and over world
    frames the ranks other than 0 traced the same rows to within one band."""
    W, H = 48, 40
    traced = _run_share(world, "dealt", (band_h, rw), n_frames=n_frames, W=W, H=H, B=2)
    assert sum(traced.values()) == n_frames * W * H
    others = [traced[r] for r in range(1, world)]
    assert max(others) - min(others) <= band_h * W * (n_frames // world)
    if rw < 1.0:
        assert traced[0] < min(others)


def test_dealt_bands_balance_1080p():
    """At 1080 rows in 8-row bands, N = 8, root weight 0.8: a fixed deal gives
    ranks 1-2 18 bands a frame and ranks 3-7 17; dealt over 8 frames every rank
    other than 0 gets 138-139 bands per 8 frames, and each frame's bands are
    every band exactly once."""
    from rtamd.dist import SharePlan, band_list
    fixed = [len(band_list(1080, 8, 8, r, 0.8)) for r in range(8)]
    assert max(fixed[1:]) == 18 and min(fixed[1:]) == 17
    plan = SharePlan(1080, 8, 8, 32, 0.8, layout="dealt")
    tot = [sum(len(plan.frame_bands(r, f)) for f in range(8)) for r in range(8)]
    assert max(tot[1:]) - min(tot[1:]) <= 1 and max(tot[1:]) <= 139
    for f in range(8):
        allb = np.sort(np.concatenate([plan.frame_bands(r, f) for r in range(8)]))
        assert np.array_equal(allb, np.arange(135))


def test_share_tracer_rejects_uneven_lists():
    """Per-frame band lists (dealt / pieces, rt_render_batch_lists_device) pack
    whole bands: a band height that does not divide the frame is refused up
    front, as bench.py's --deal auto avoids choosing it."""
    from rtamd.dist import SharePlan, ShareTracer, TilePlan
    plan = SharePlan(1080, 16, 8, 8, 0.8, layout="dealt")
    with pytest.raises(ValueError, match="divide the height"):
        ShareTracer(None, 1920, 1080, 4, "bands", 1, plan=plan, band_h=16, batch=8)
    ok = SharePlan(1080, 8, 8, 8, 0.8, layout="dealt")
    t = ShareTracer(None, 1920, 1080, 4, "bands", 1, plan=ok, band_h=8, batch=8)
    assert [len(b) for b in t.my_bands] == [len(ok.frame_bands(1, f)) for f in range(8)]
    assert t.offset_rows(3) == ok.off[1][3]
    with pytest.raises(ValueError):
        ShareTracer(None, 1920, 1080, 4, "tiles", 0)
    tt = ShareTracer(None, 1920, 1080, 4, "tiles", 3, tplan=TilePlan(1920, 1080, 4, 2), batch=2)
    assert tt.rect == (960, 540, 960, 540)


@pytest.mark.parametrize("world,n_frames,band_h,rw,wire,pieces,whole_b,lf", [(2, 3, 4, 1.0, "rgba", False, -1, 1),
                                                                          (4, 4, 4, 0.6, "rgb", False, -1, 1),
                                                                          (8, 8, 2, 0.8, "rgb", False, -1, 1),
                                                                          (3, 2, 8, 0.0, "rgba", False, -1, 1),
                                                                          (3, 2, 8, 0.5, "rgb", False, -1, 1),
                                                                          (4, 4, 4, 0.6, "rgb", True, -1, 1),
                                                                          (3, 3, 4, 0.8, "rgba", True, -1, 1),
                                                                          (8, 11, 4, 0.8, "rgba", True, 3, 1),
                                                                          (4, 6, 4, 0.6, "rgb", False, 1, 1),
                                                                          (4, 8, 4, 0.6, "rgb", True, -1, 2),
                                                                          (3, 5, 4, 0.8, "rgba", True, -1, 3)])
def test_spans_weak_scaling(world, n_frames, band_h, rw, wire, pieces, whole_b, lf):
    """bench.py --partition spans: each rank traces one contiguous span of the
    batch's rows (whole frames, a run of bands at either end; rank 0's span
    rw times the others'), rank 0 in place in the batch's frames, and one
    group of point-to-point receives lands every other span straight in them
    (wire "rgb": the rows travel as RGB and rank 0 writes them into its RGBA8
    frames, whose alpha bytes it set once; pieces: the spans travel launch by
    launch, one receive per piece, as bench.py's last batch of a phase;
    whole_b >= 0: spans cut at frame boundaries, the plan of batch whole_b):
    every frame and its radiance equal the oracle's, bit for bit."""
    W, H = 48, 40
    traced = _run_share(world, "spans", (band_h, rw, wire, pieces, whole_b, lf), n_frames=n_frames, W=W, H=H, B=2)
    assert sum(traced.values()) == n_frames * W * H
    if 0 < rw < 1.0:
        assert traced[0] < min(traced[r] for r in range(1, world)) or \
            (whole_b >= 0 and traced[0] <= min(traced[r] for r in range(1, world)))   # whole frames: rounded
    if rw == 0.0:
        assert traced[0] == 0


def test_span_plan_1080p():
    """The N = 8 batch of bench.py (32 frames of 1080 rows in 8-row bands,
    rank 0 weight 0.8): the spans tile the batch column in rank order, the
    ranks other than 0 get the same rows to within one band, every launch is
    one frame's band run (a whole frame or an end piece), and the launches of
    a span pack its rows back to back."""
    from rtamd.dist import SpanPlan, SpanTracer
    plan = SpanPlan(1080, 8, 8, 32, 0.8)
    assert plan.row0[0] == 0 and plan.row0[1:] == [plan.row0[r] + plan.rows[r] for r in range(7)]
    assert plan.row0[7] + plan.rows[7] == 32 * 1080
    others = plan.rows[1:]
    assert max(others) - min(others) <= 8 and plan.rows[0] < min(others)
    for r in range(8):
        out_row = 0
        for f, lo, hi, orow in plan.launches[r]:
            assert 0 <= lo < hi <= 135 and orow == out_row
            assert plan.row0[r] + orow == f * 1080 + lo * 8           # the span is the batch column
            out_row += (hi - lo) * 8
        assert out_row == plan.rows[r]
        t = SpanTracer(None, 1920, 1080, 4, plan, r)
        assert sum(1 for b in t._lists if b is None) >= 2             # mostly whole frames
    assert plan.recv_slices() == [(r, plan.row0[r], plan.rows[r]) for r in range(1, 8)]
    # the pieces (one per launch) tile each span in order
    for r in range(1, 8):
        ps = [(y, n) for rr, y, n in plan.recv_pieces() if rr == r]
        assert ps[0][0] == plan.row0[r] and sum(n for _, n in ps) == plan.rows[r]
        assert all(ps[i][0] + ps[i][1] == ps[i + 1][0] for i in range(len(ps) - 1))
        assert [(plan.row0[r] + o, n) for o, n in plan.pieces(r)] == ps
    # cut at frame boundaries (--span-cut frames): whole-frame launches only, rank 0
    # 3 frames, the others 4 and one extra frame rotating over them batch by batch
    wp = SpanPlan(1080, 8, 8, 32, 0.8, whole_frames=True)
    extra = []
    for b in range(14):
        v = wp.batch(b)
        c = v.frame_counts(b)
        assert c[0] == 3 and sum(c) == 32 and sorted(c[1:]) == [4] * 6 + [5]
        assert v.rows == [n * 1080 for n in c] and all((lo, hi) == (0, 135) for r in range(8)
                                                       for _, lo, hi, _ in v.launches[r])
        assert v.per_rank == 5 * 1080 and v is wp.batch(b + 7)
        extra.append(c.index(5))
    assert extra[:7] == list(range(1, 8))
    assert SpanPlan(1080, 8, 4, 16, 0.9, whole_frames=True).frame_counts(0) == [4, 4, 4, 4]
    with pytest.raises(ValueError, match="divide the height"):
        SpanPlan(1080, 16, 8, 32, 0.8)
    # launch groups (--span-launch-frames 2): runs of two consecutive entries,
    # the span-end runs with their neighbours; the pieces follow the groups and
    # still tile each span in order
    gp = SpanPlan(1080, 8, 8, 32, 0.8, launch_frames=2)
    for r in range(8):
        ls, gs = gp.launches[r], gp.groups[r]
        assert [i for g, n in gs for i in range(g, g + n)] == list(range(len(ls)))
        assert all(n == 2 for _, n in gs[:-1]) and 1 <= gs[-1][1] <= 2
        t = SpanTracer(None, 1920, 1080, 4, gp, r)
        for j, (g, n) in enumerate(gs):
            assert t.group_frames(j) == [ls[g + i][0] for i in range(n)]
            assert t.group_frames(j) == list(range(ls[g][0], ls[g][0] + n))   # consecutive frames
            assert t.group_row(j) == ls[g][3]
        ps = gp.pieces(r)
        assert len(ps) == len(gs) and ps[0][0] == 0 and sum(n for _, n in ps) == gp.rows[r]
        assert all(ps[i][0] + ps[i][1] == ps[i + 1][0] for i in range(len(ps) - 1))
    with pytest.raises(ValueError, match="launch_frames"):
        SpanPlan(1080, 8, 8, 32, 0.8, launch_frames=0)
