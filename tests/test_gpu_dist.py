"""The exchange on the GPU over RCCL (backend "nccl"): one process, world size 1.

The multi-GPU runs are the driver's; this runs the same calls bench.py makes
at N > 1 (rtamd/dist.py: gather_frames of a batch of frame slots, gather_frame,
DistRenderer) through RCCL with device tensors, and checks that the assembled
frames equal the whole frame traced on one GPU bit for bit.  The partition and
assembly logic at world sizes 2 and 3 is covered on CPU (test_dist.py, gloo).
"""
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


@pytest.mark.parametrize("band_h,n_frames", [(16, 4), (7, 3)])
def test_rccl_gather_frames_bit_exact(renderer, rccl_group, band_h, n_frames):
    import ctypes as C
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
    # bench.py's N > 1 exchange: frame slots traced as bands, one gather per batch
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
