"""Debug: accel frames through rt_render_tile_device and batched band lists
against the oracle (config 2 scene, orbiting cameras), per accel / coop_lanes."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtamd  # noqa: E402
from oracle import oracle_lib  # noqa: E402
from rtamd import configs, lib  # noqa: E402
from rtamd._lib import CameraUBO, check  # noqa: E402
from rtamd.dist import SharePlan, ShareTracer, assemble_shares  # noqa: E402
from test_gpu_dist import _orbit_cams  # noqa: E402

cfg = configs.config2()
built = cfg.build()
W, H, B, band_h = 320, 184, 3, 8
for accel in (8, 1):
    for coop in (1, 0):
        r = rtamd.Renderer((0,))
        r.set_option("accel", accel)
        r.set_option("coop_lanes", coop)
        r.set_option("concurrent_launches", 1)
        r.upload_scene(built)
        world, rw, layout = 2, 0.9, "interleave"
        F, G = world, 2 * world
        cams = _orbit_cams(W, H, G)
        refs = [oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                  c.ubo_bytes(), W, H, B, radiance=False)[0] for c in cams]
        s = torch.cuda.current_stream()
        for f, c in enumerate(cams):
            rgba = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
            check(lib().rt_render_tile_device(r._ctx, C.byref(c.ubo), W, H, B, 0, 0, W, H, rgba.data_ptr(), None,
                                              s.cuda_stream, None))
            torch.cuda.synchronize()
            bad = np.argwhere((rgba.cpu().numpy() != refs[f]).any(-1))
            print(f"accel {accel} coop {coop} whole frame {f}: {len(bad)} px differ {bad[:6].tolist()}", flush=True)
        plan = SharePlan(H, band_h, world, G, rw, layout=layout)
        src = torch.as_tensor(plan.src, device="cuda:0")
        bufs = []
        streams = [torch.cuda.Stream() for _ in range(2)]
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
        frames = assemble_shares(torch.stack(bufs), plan, src).cpu().numpy()
        for f in range(G):
            bad = np.argwhere((frames[f] != refs[f]).any(-1))
            print(f"accel {accel} coop {coop} batched frame {f}: {len(bad)} px differ {bad[:6].tolist()}", flush=True)
        r.close()
