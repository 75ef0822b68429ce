"""Option accel's exactness margin under adversarial geometry (verdict r05,
next #2): a CPU study, no GPU.

The accel walk returns the reference's closest hit when the
reference's candidate i* (the lowest (t, flattened index) over the triangles
whose own leaf box the ray's line crosses in front) satisfies
te* <= t* (1 + 2^-10) + 2^-10, te* being the t_enter of i*'s leaf box; a hit
before its box takes the fallback to the reference's order.  Nothing in the
BASELINE configs comes near that margin (round 5: 0 of 10.5 M pixels).  Here
the geometry is built to approach it:

  slivers      needle triangles 5-15 long and 1e-5 - 1e-3 wide in random
               orientations around the cube of config 2, camera close;
  fine_mesh    a 200k-triangle closed shell 2 units across: most primary hits
               have |det| in (1e-5, 1e-4] (the shader's cut is 1e-5,
               compute_dynamic_ray.comp:110), where Moeller-Trumbore's t error
               is largest;
  grazing      a tilted (no flat axis, so no 1e-4 box padding), finely
               tessellated 300-unit ground with the camera 1e-2 above it,
               looking along it, plus the cube with the camera in the plane of
               its top face;
  far_origin   config 2's cube and plane and a procedural shell translated to
               +-1e4 (coordinates whose float ulp is 2^-10, the margin's
               absolute part), camera translated with them, near and far;
  near_camera  small triangles 1e-3 - 1e-2 in front of the camera (t at
               T_MIN = 0.001, where the absolute part of the margin dominates).

Each scene is built with the reference builder at axis seeds 1, 2 and 3 and
rendered by the reference-order oracle (oracle/rt_oracle.c) and by the accel
walk's model (oracle/rt_accel_model.c, 1 and 8 layouts) with the margin audit
on (orc_accel_audit): pixels that differ (RGBA8 or radiance bits) from the
seed-1 oracle, differences between the reference's own seeds (the reference
tree is random per build, BVHBuilder.java:53), and the audit's counts.

Output: tests/golden/accel_adversarial.json (tests/test_accel_model.py
re-checks a small version of every scene; DESIGN.md §4a cites it).

    python tools/accel_adversarial.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd")]

import numpy as np  # noqa: E402

from oracle import oracle_lib as O  # noqa: E402
from rtamd import _lib, build_buffers, configs, triangles_of  # noqa: E402
from rtamd.scene import Mesh  # noqa: E402


def _mats(n, rng, types=(0, 1, 2)):
    return np.concatenate([rng.uniform(0.2, 0.95, (n, 3)), rng.choice(types, (n, 1))], 1).astype(np.float32)


def scene_slivers(scale=1.0, seed=11):
    rng = np.random.default_rng(seed)
    v0, m0 = triangles_of(configs.config2().scene)
    n = int(3000 * scale)
    c = rng.uniform(-15.0, 15.0, (n, 3)) + np.array([0.0, 2.0, 0.0])
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    p = rng.normal(size=(n, 3))
    p -= (p * u).sum(1, keepdims=True) * u
    p /= np.linalg.norm(p, axis=1, keepdims=True)
    length = rng.uniform(5.0, 15.0, (n, 1))
    width = 10.0 ** rng.uniform(-5.0, -3.0, (n, 1))
    a, b = c - 0.5 * length * u, c + 0.5 * length * u
    tip = c + width * p + rng.uniform(-0.4, 0.4, (n, 1)) * length * u
    verts = np.concatenate([v0, np.stack([a, b, tip], 1).reshape(n, 9)])
    mats = np.concatenate([m0, _mats(n, rng)])
    cam = ((6.0, 9.0, 34.0), (0.0, 0.0, 0.0))
    return verts, mats, cam, 40.0


def scene_fine_mesh(scale=1.0, seed=12):
    rng = np.random.default_rng(seed)
    n = int(200_000 * scale) // 2 * 2
    m = Mesh.procedural(n, 0xF1E, (-1.0, -1.0, -1.0), (1.0, 1.0, 1.0)).tris.astype(np.float64).reshape(n, 9)
    mats = _mats(n, rng, (0, 1))
    ground = np.array([[-50, -1.2, -50, 50, -1.2, -50, 50, -1.2, 50], [-50, -1.2, -50, 50, -1.2, 50, -50, -1.2, 50]],
                      np.float64)
    verts = np.concatenate([m, ground])
    mats = np.concatenate([mats, np.array([[0.5, 0.5, 0.5, 0.0]] * 2, np.float32)])
    return verts, mats, ((0.6, 0.9, 3.2), (0.0, 0.0, 0.0)), 45.0


def _grid(n, size, y0, tilt, seed):
    """n x n quads (2n^2 triangles) over [-size, size]^2, height y0 + tilt . (x, z)
    plus a small seeded jitter: no axis is flat, so no box padding."""
    rng = np.random.default_rng(seed)
    xs = np.linspace(-size, size, n + 1)
    X, Z = np.meshgrid(xs, xs, indexing="ij")
    Y = y0 + tilt[0] * X + tilt[1] * Z + rng.uniform(-1e-3, 1e-3, X.shape)
    P = np.stack([X, Y, Z], -1)
    a, b, c, d = P[:-1, :-1], P[1:, :-1], P[1:, 1:], P[:-1, 1:]
    t1 = np.stack([a, b, c], -2).reshape(-1, 9)
    t2 = np.stack([a, c, d], -2).reshape(-1, 9)
    return np.concatenate([t1, t2])


def scene_grazing(scale=1.0, seed=13):
    rng = np.random.default_rng(seed)
    v0, m0 = triangles_of(configs.config2().scene)
    cube = v0[2:]                                          # the config-2 cube (the first 2 are the plane)
    g = _grid(max(8, int(150 * np.sqrt(scale))), 150.0, -10.0, (1.3e-3, -0.7e-3), seed)
    verts = np.concatenate([g, cube])
    mats = np.concatenate([_mats(len(g), rng, (0, 1)), m0[2:]])
    # camera 1e-2 above the ground's height at its position, looking along it
    # towards the cube; the cube's top face (y = 0) sits at the eye's height
    return verts, mats, ((-120.0, -10.0 + 1.3e-3 * -120.0 + 1e-2, 0.0), (0.0, 0.0, 0.0)), 30.0


def scene_grazing_cube(scale=1.0, seed=14):
    v0, m0 = triangles_of(configs.config2().scene)
    # the eye in the plane of the cube's top face (y = 0), rays skimming it
    return v0, m0, ((-60.0, 0.0, 13.0), (0.0, 0.0, 0.0)), 25.0


def scene_far_origin(scale=1.0, seed=15, offset=(1.0e4, -1.0e4, 1.0e4), near=True):
    rng = np.random.default_rng(seed)
    v0, m0 = triangles_of(configs.config2().scene)
    n = int(20_000 * scale) // 2 * 2
    sh = Mesh.procedural(n, 0xFA2, (-8.0, -10.0, -8.0), (8.0, 6.0, 8.0)).tris.astype(np.float64).reshape(n, 9)
    sh += np.array([25.0, 0.0, 0.0] * 3)
    verts = np.concatenate([v0, sh]) + np.array(list(offset) * 3)
    mats = np.concatenate([m0, _mats(n, rng)])
    o = np.array(offset)
    eye = (-4.0, 6.0, 14.0) if near else (-25.0, 30.0, 140.0)
    return verts, mats, (tuple(o + eye), tuple(o)), 60.0 if near else 30.0


def scene_near_camera(scale=1.0, seed=16):
    rng = np.random.default_rng(seed)
    v0, m0 = triangles_of(configs.config2().scene)
    eye = np.array([0.0, 5.0, 40.0])
    n = int(400 * scale)
    fwd = np.array([0.0, -5.0, -40.0]) / np.linalg.norm([0.0, -5.0, -40.0])
    d = 10.0 ** rng.uniform(-3.0, -2.0, (n, 1))              # 1e-3 .. 1e-2 ahead of the eye
    c = eye + d * fwd + rng.uniform(-1.0, 1.0, (n, 3)) * d * 0.6
    tris = c[:, None, :] + rng.uniform(-1.0, 1.0, (n, 3, 3)) * d[:, :, None] * 0.25
    verts = np.concatenate([v0, tris.reshape(n, 9)])
    mats = np.concatenate([m0, _mats(n, rng)])
    return verts, mats, (tuple(eye), (0.0, 0.0, 0.0)), 50.0


SCENES = {
    "slivers": scene_slivers,
    "fine_mesh": scene_fine_mesh,
    "grazing": scene_grazing,
    "grazing_cube": scene_grazing_cube,
    "far_origin_near": lambda scale=1.0: scene_far_origin(scale, near=True),
    "far_origin_far": lambda scale=1.0: scene_far_origin(scale, near=False),
    "far_origin_neg": lambda scale=1.0: scene_far_origin(scale, offset=(-1.0e4, 1.0e4, -1.0e4), near=True),
    "near_camera": scene_near_camera,
}


def run_scene(name: str, w: int, h: int, b: int, scale: float = 1.0, seeds=(1, 2, 3), layouts=(1, 8)) -> dict:
    verts, mats, (eye, at), vfov = SCENES[name](scale)
    cam = configs.Camera(eye, at, (0.0, 1.0, 0.0), vfov, w / h)
    out = {"scene": name, "triangles": int(len(verts)), "width": w, "height": h, "max_bounces": b, "seeds": {}}
    base = None
    for seed in seeds:
        built = build_buffers(verts, mats, seed)
        args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), w, h, b)
        ref = O.render(*args)
        if base is None:
            base = ref
        e = {"segments": ref[2]["segments"], "mat_reads": ref[2]["mat_reads"],
             "reference_vs_seed1_px": int(((ref[0] != base[0]).any(-1) |
                                           (ref[1].view(np.uint32) != base[1].view(np.uint32)).any(-1)).sum())}
        for nl in layouts:
            rec, info = _lib.accel_records(built, nl)
            O.accel_audit(True)
            acc = O.render_accel(*args, rec, info)
            aud = O.accel_audit_result()
            O.accel_audit(False)
            e[f"layouts{nl}"] = {
                "rgba_px": int((acc[0] != ref[0]).any(-1).sum()),
                "radiance_px": int((acc[1].view(np.uint32) != ref[1].view(np.uint32)).any(-1).sum()),
                "segments_equal": acc[2]["segments"] == ref[2]["segments"],
                "mat_reads_equal": acc[2]["mat_reads"] == ref[2]["mat_reads"],
                "fallback_segments": acc[2]["fallbacks"],
                "audit": aud,
            }
        out["seeds"][str(seed)] = e
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="small frames and scenes (a test-sized run)")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "accel_adversarial.json"))
    a = ap.parse_args()
    w, h, b, scale = (160, 90, 4, 0.1) if a.quick else (960, 540, 4, 1.0)
    cases = []
    for name in SCENES:
        t0 = time.time()
        c = run_scene(name, w, h, b, scale)
        c["seconds"] = round(time.time() - t0, 1)
        cases.append(c)
        s1 = c["seeds"]["1"]
        print(name, c["triangles"], {k: (v["rgba_px"], v["radiance_px"], v["audit"]) for k, v in s1.items()
                                     if k.startswith("layouts")}, c["seconds"], "s", flush=True)
    res = {"tool": "tools/accel_adversarial.py", "quick": a.quick,
           "margin": "t_enter <= closest_t * (1 + 2^-10) + 2^-10 (rt_trace.hip accel_enter)",
           "headroom": "(te* - t*) / (t* 2^-10 + 2^-10) of the reference's candidate hit i*: > 1 = unsafe",
           "cases": cases}
    if not a.quick:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        print("wrote", a.out)


if __name__ == "__main__":
    main()
