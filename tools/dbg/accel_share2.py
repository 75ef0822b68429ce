"""Debug: the test_gpu_dist sequence on one renderer, every launch checked
right after it (synchronised) against the whole frames."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import configs  # noqa: E402
from rtamd._lib import CameraUBO  # noqa: E402
from rtamd.dist import SharePlan, ShareTracer  # noqa: E402
from test_gpu_dist import _orbit_cams, _whole  # noqa: E402

cfg = configs.config2()
built = cfg.build()
W, H, B, band_h = 320, 184, 3, 8
cases = [("interleave", 1, 1.0), ("interleave", 2, 0.9), ("interleave", 4, 0.85), ("dealt", 8, 0.8),
         ("dealt", 4, 1.0), ("pieces", 4, 1.0), ("pieces", 8, 0.7)]
sync_each = len(sys.argv) > 1 and sys.argv[1] == "sync"
r = rtamd.Renderer((0,))
for accel in (0, 8):
    for layout, world, rw in cases:
        r.set_option("accel", accel)
        r.upload_scene(built)
        r.set_option("accel", 0)
        F, G = world, 2 * world
        cams = _orbit_cams(W, H, G)
        whole = _whole(r, cams, W, H, B)
        plan = SharePlan(H, band_h, world, G, rw, layout=layout)
        streams = [torch.cuda.Stream() for _ in range(2)]
        for rank in range(world):
            tracer = ShareTracer(r._ctx, W, H, B, "bands", rank, plan=plan, band_h=band_h, batch=G)
            rgba = torch.full((plan.per_rank, W, 4), 7, dtype=torch.uint8, device="cuda:0")
            for j, k0 in enumerate(range(0, G, F)):
                print(f"--- accel {accel} {layout} N={world} rank {rank} launch {j}", file=sys.stderr, flush=True)
                off = tracer.offset_rows(k0)
                rp = rgba[off].data_ptr() if off < plan.per_rank else rgba.data_ptr()
                ubos = (CameraUBO * F)(*[c.ubo for c in cams[k0:k0 + F]])
                tracer.launch(ubos, k0, F, streams[j % 2].cuda_stream, rp, None)
                if sync_each:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            miss = []
            for f in range(G):
                o, nrow = plan.off[rank][f], len(plan.frame_rows(rank, f))
                u = int((rgba[o:o + nrow] == 7).all(-1).sum())
                if u:
                    miss.append((f, u))
            print(f"accel {accel} {layout} N={world} rank {rank}: untraced (frame, px) {miss}", flush=True)
r.close()
