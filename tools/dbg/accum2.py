"""Debug: the accumulation extension on a two-device context (0, 0) under
schedule variations; prints which frames / rows differ from the oracle."""
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
for name, opts, devs in [("default", {}, (0, 0)), ("learn_host", {"learn_device": 0}, (0, 0)),
                         ("no_heavy_first", {"heavy_first": 0}, (0, 0)), ("no_coop", {"coop_lanes": 0}, (0, 0)),
                         ("walk0", {"walk": 0}, (0, 0)), ("one_dev", {}, (0,)),
                         ("no_ext_2dev", {"_noext": 1}, (0, 0))]:
    r = rtamd.Renderer(devs)
    r.upload_scene(built)
    ext = 0 if opts.get("_noext") else 7
    r.set_option("extensions", ext)
    for k, v in opts.items():
        if not k.startswith("_"):
            r.set_option(k, v)
    cam = configs.Camera.default(w, h)
    acc = np.zeros((h, w, 3), np.float32)
    out = []
    for f in range(4):
        cam.ubo.frame_count = f
        rgba, rad, _ = r.render(cam, w, h, b, radiance=True)
        ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                cam.ubo_bytes(), w, h, b, ext=ext, accum=acc if ext else None)[0]
        bad = np.any(rgba != ref, axis=-1)
        rows = np.flatnonzero(bad.any(axis=1))
        out.append(f"f{f}: {int(bad.sum())} px, rows {rows[:6].tolist()}{'...' if len(rows) > 6 else ''}")
    print(name, "|", "; ".join(out), flush=True)
    r.close()
