"""Debug: the accumulation extension on a two-device context (0, 0) with host
learning (the learned tile order from frame 1 on): which device-local tiles
differ, and whether a differing pixel holds a stale or a twice-accumulated
value."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import rtamd
from rtamd import configs
from oracle import oracle_lib
from test_oracle_kat import _ext_scene

built = _ext_scene()
w, h, b = 150, 97, 4


def oracle(cam, ext, acc):
    return oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                             cam.ubo_bytes(), w, h, b, ext=ext, accum=acc)


for name, opts, devs, ext in [("host2_ext7", {"learn_device": 0}, (0, 0), 7),
                              ("host2_ext1", {"learn_device": 0}, (0, 0), 1),
                              ("host2_ext7_nocoop", {"learn_device": 0, "coop_lanes": 0}, (0, 0), 7),
                              ("host2_ext7_cost0", {"learn_device": 0, "learn_cost": 0}, (0, 0), 7),
                              ("host1_ext7", {"learn_device": 0}, (0,), 7),
                              ("host2_ext7_noreuse", {"learn_device": 0, "reuse_order": 0}, (0, 0), 7)]:
    r = rtamd.Renderer(devs)
    r.upload_scene(built)
    r.set_option("extensions", ext)
    for k, v in opts.items():
        r.set_option(k, v)
    cam = configs.Camera.default(w, h)
    acc = np.zeros((h, w, 3), np.float32)
    prev = None
    for f in range(3):
        cam.ubo.frame_count = f
        rgba, rad, _ = r.render(cam, w, h, b, radiance=True)
        ref = oracle(cam, ext, acc)
        bad = np.any(rgba != ref[0], axis=-1)
        ys, xs = np.nonzero(bad)
        line = f"{name} f{f}: {int(bad.sum())} px"
        if len(ys):
            dev = (ys // 16) % len(devs)
            ly = (ys // 16 // len(devs)) * 16 + ys % 16
            tiles = sorted(set(zip((ly // 8).tolist(), (xs // 8).tolist())))
            stale = prev is not None and bool(np.all(rgba[bad] == prev[bad]))
            line += (f", devices {sorted(set(dev.tolist()))}, local tiles ({len(tiles)}) {tiles[:12]}, "
                     f"stale(prev frame) {stale}, max |d rad| {float(np.abs(rad[bad] - ref[1][bad]).max()):.4g}")
        print(line, flush=True)
        prev = ref[0]
    r.close()
