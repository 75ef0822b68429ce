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
    """Rotating row pieces (bench.py's N > 1 default): frame k lays the ranks'
    pieces out in the rotated order k, k+1, ...; rank 0 traces its piece (of
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
