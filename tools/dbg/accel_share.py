"""Debug: test_share_exchange_bit_exact with accel 8 under option variants,
reporting untraced (fill value 7) and wrong pixels of every assembled frame."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import configs  # noqa: E402
from rtamd._lib import CameraUBO  # noqa: E402
from rtamd.dist import SharePlan, ShareTracer, assemble_shares  # noqa: E402
from test_gpu_dist import _orbit_cams, _whole  # noqa: E402
from test_gpu_parity import DEFAULT_OPTS  # noqa: E402

cfg = configs.config2()
built = cfg.build()
W, H, B, band_h = 320, 184, 3, 8
cases = [("interleave", 1, 1.0), ("interleave", 2, 0.9), ("interleave", 4, 0.85), ("dealt", 8, 0.8),
         ("dealt", 4, 1.0), ("pieces", 4, 1.0), ("pieces", 8, 0.7)]
r = rtamd.Renderer((0,))                     # one renderer for every case, as the session fixture
if len(sys.argv) > 1:
    for kv in sys.argv[1].split(","):
        k, v = kv.split("=")
        r.set_option(k, int(v))
for accel in (0, 8):
    for layout, world, rw in cases:
        print(f"=== accel {accel} {layout} {world}", file=sys.stderr, flush=True)
        r.set_option("accel", accel)
        r.upload_scene(built)
        r.set_option("accel", 0)
        F, G = world, 2 * world
        cams = _orbit_cams(W, H, G)
        whole = _whole(r, cams, W, H, B)
        plan = SharePlan(H, band_h, world, G, rw, layout=layout)
        src = torch.as_tensor(plan.src, device="cuda:0")
        streams = [torch.cuda.Stream() for _ in range(2)]
        bufs = []
        for rank in range(world):
            tracer = ShareTracer(r._ctx, W, H, B, "bands", rank, plan=plan, band_h=band_h, batch=G)
            rgba = torch.full((plan.per_rank, W, 4), 7, dtype=torch.uint8, device="cuda:0")
            for j, k0 in enumerate(range(0, G, F)):
                off = tracer.offset_rows(k0)
                rp = rgba[off].data_ptr() if off < plan.per_rank else rgba.data_ptr()
                ubos = (CameraUBO * F)(*[c.ubo for c in cams[k0:k0 + F]])
                tracer.launch(ubos, k0, F, streams[j % 2].cuda_stream, rp, None)
            bufs.append(rgba)
        torch.cuda.synchronize()
        frames = assemble_shares(torch.stack(bufs), plan, src)
        torch.cuda.synchronize()
        msg = []
        for f in range(G):
            diff = (frames[f] != whole[f][0]).any(-1)
            seven = (frames[f] == 7).all(-1)
            if diff.any():
                rows = torch.nonzero(diff.any(-1)).flatten().tolist()
                # which frame's camera do the wrong rows show?
                other = [g for g in range(G) if g != f and bool((frames[f][diff] == whole[g][0][diff]).all())]
                msg.append(f"f{f}: {int(diff.sum())} differ ({int((diff & seven).sum())} untraced), rows "
                           f"{rows[:12]} ({len(rows)}), equal to frame {other}")
        print(f"accel {accel} {layout} N={world}: {'OK' if not msg else '; '.join(msg)}  "
              f"heavy_px_used {r.get_option('heavy_pixels_used')}", flush=True)
r.close()
