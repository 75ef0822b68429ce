#!/usr/bin/env python3
"""Generate tests/golden/golden.json — the committed known-answer fixtures.

No reference fixture exists for this path (the reference has no tests and
cannot run here: SURVEY.md §8c), so the fixtures are produced by this repo's
restatements and cross-checked at generation time:
  * PCG / randomFloat KATs: a pure-Python big-integer restatement of
    compute_dynamic_ray.comp:52-61 (checked against the C oracle), including
    a seed found by inverting pcg whose randomFloat() is exactly 1.0;
  * frames: the C oracle (oracle/rt_oracle.c) — each also checked against the
    independent numpy restatement (oracle/shader_np.py) before it is written;
    stored as SHA-256 of the RGBA8 / float radiance bytes + work counters;
  * scene buffers: SHA-256 of the product builder's three buffers for the
    BASELINE configs (checked against oracle/scene_oracle.py for the small ones).
Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]

M32 = 0xFFFFFFFF


def pcg_py(v):
    s = (v * 747796405 + 2891336453) & M32
    w = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & M32
    return ((w >> 22) ^ w) & M32


def pcg_inverse(out):
    w = out ^ (out >> 22)
    x = (w * pow(277803737, -1, 1 << 32)) & M32
    k = (x >> 28) + 4
    s = x
    for _ in range(10):
        s = x ^ (s >> k)
    v = ((s - 2891336453) * pow(747796405, -1, 1 << 32)) & M32
    assert pcg_py(v) == out
    return v


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


FRAMES = [  # (name, config, width, height, max_bounces)
    ("cfg1_640x480_b1", 1, 640, 480, 1),
    ("cfg2_320x180_b2", 2, 320, 180, 2),
    ("cfg2_128x72_b10", 2, 128, 72, 10),
    ("cfg3_192x108_b4", 3, 192, 108, 4),
    ("cfg3_96x54_b8", 3, 96, 54, 8),
]


def main():
    warnings.filterwarnings("ignore")
    from oracle import oracle_lib, scene_oracle, shader_np
    from rtamd import configs, triangles_of

    L = oracle_lib.lib()
    kat = {"pcg": {}, "random_float_seq": {}}
    for v in [0, 1, 2, 3, 42, 12345, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF]:
        assert L.orc_pcg(v) == pcg_py(v)
        kat["pcg"][str(v)] = pcg_py(v)
    import ctypes as C
    for s0 in [0, 1, 921599, 2073599]:
        seed = C.c_uint32(s0)
        kat["random_float_seq"][str(s0)] = [float(L.orc_random_float(C.byref(seed))) for _ in range(8)]
    one = pcg_inverse(0xFFFFFFFF)
    seed = C.c_uint32(one)
    assert L.orc_random_float(C.byref(seed)) == 1.0
    kat["random_float_one_seed"] = one
    kat["random_float_below_one_seed"] = pcg_inverse(0xFFFFFF7F)

    frames = {}
    for name, k, w, h, b in FRAMES:
        cfg = configs.get(k)
        built = cfg.build()
        cam = configs.Camera.default(w, h)
        rgba, rad, cnt = oracle_lib.render(built.model_vertex_data, built.model_material_data,
                                           built.flat_bvh_data, cam.ubo_bytes(), w, h, b)
        r2 = shader_np.render(built.model_vertex_data.tobytes(), built.model_material_data.tobytes(),
                              built.flat_bvh_data.tobytes(), cam.ubo_bytes(), w, h, b)
        assert np.array_equal(rgba, r2[0]) and np.array_equal(rad.view(np.uint32), r2[1].view(np.uint32))
        assert cnt == r2[2], (cnt, r2[2])
        ys, xs = np.nonzero(np.any(rgba[..., :3] != rgba[0, 0, :3], axis=-1))
        pick = np.linspace(0, len(ys) - 1, 8).astype(int) if len(ys) else []
        frames[name] = {"config": k, "width": w, "height": h, "max_bounces": b,
                        "rgba_sha256": sha(rgba), "radiance_sha256": sha(rad), "counts": cnt,
                        "samples": [[int(xs[i]), int(ys[i]), rgba[ys[i], xs[i]].tolist(),
                                     rad[ys[i], xs[i]].tolist()] for i in pick]}
        print("frame", name, cnt)

    scenes = {}
    for k in (1, 2, 3, 5):
        cfg = configs.get(k)
        built = cfg.build()
        cam = cfg.camera()
        if k in (1, 2):
            verts, mats = triangles_of(cfg.scene)
            tris = [(tuple(v[0:3]), tuple(v[3:6]), tuple(v[6:9]), tuple(m))
                    for v, m in zip(verts.tolist(), mats.tolist())]
            vb, mb, bb, nf = scene_oracle.build_scene(tris, 1)
            assert vb == built.model_vertex_data.tobytes() and bb == built.flat_bvh_data.tobytes()
        scenes[cfg.name] = {"flat_triangles": built.triangle_count, "nodes": built.n_nodes,
                            "vertices_sha256": sha(built.model_vertex_data),
                            "materials_sha256": sha(built.model_material_data),
                            "nodes_sha256": sha(built.flat_bvh_data),
                            "camera_ubo_hex": cam.ubo_bytes().hex()}
        print("scene", cfg.name, built.triangle_count, built.n_nodes)

    out = {"generator": "tests/golden/make_golden.py", "axis_seed": 1, "kat": kat, "frames": frames,
           "scenes": scenes}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote golden.json")


if __name__ == "__main__":
    main()
