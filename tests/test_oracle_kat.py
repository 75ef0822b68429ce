"""The oracle, pinned: known-answer tests, SPIR-V facts, two independent
restatements agreeing, and the committed golden frames (CPU only)."""
import ctypes as C
import json
import os
import struct
import warnings

import numpy as np
import pytest


def _load_json(path):
    with open(path) as f:
        return json.load(f)


HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = _load_json(os.path.join(HERE, "golden", "golden.json"))
SPIRV = _load_json(os.path.join(HERE, "golden", "spirv_facts.json"))
M32 = 0xFFFFFFFF


def L():
    from oracle import oracle_lib
    return oracle_lib.lib()


def f3(*v):
    return (C.c_float * 3)(*v)


def pcg_py(v):
    s = (v * 747796405 + 2891336453) & M32
    w = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & M32
    return ((w >> 22) ^ w) & M32


def test_pcg_kat():
    for v, expect in GOLDEN["kat"]["pcg"].items():
        assert L().orc_pcg(int(v)) == expect == pcg_py(int(v))
    for v in range(0, 1 << 32, 9_999_991):
        assert L().orc_pcg(v) == pcg_py(v)


def test_pcg_is_a_bijection_sample():
    from oracle.shader_np import pcg
    v = np.arange(1 << 20, dtype=np.uint32)
    assert np.unique(pcg(v)).size == v.size


def test_random_float_sequences_and_one():
    from oracle.shader_np import random_float
    for s0, seq in GOLDEN["kat"]["random_float_seq"].items():
        seed = C.c_uint32(int(s0))
        got = [float(L().orc_random_float(C.byref(seed))) for _ in range(len(seq))]
        assert got == seq
        s = np.array([int(s0)], np.uint32)
        for x in seq:
            s, f = random_float(s)
            assert float(f[0]) == x
    # float(0xFFFFFFFFu) rounds to 2^32, so randomFloat() can return exactly 1.0
    seed = C.c_uint32(GOLDEN["kat"]["random_float_one_seed"])
    assert L().orc_random_float(C.byref(seed)) == 1.0
    seed = C.c_uint32(GOLDEN["kat"]["random_float_below_one_seed"])
    assert L().orc_random_float(C.byref(seed)) < 1.0


def test_spirv_constants_are_the_oracles():
    """Every constant of the executed SPIR-V that the path uses appears in the
    oracle with the same float32 bits."""
    floats = {c["bits"] for c in SPIRV["constants"] if c["type"] == "float"}
    uints = {c["value"] for c in SPIRV["constants"] if c["type"] == "uint"}
    ints = {c["value"] for c in SPIRV["constants"] if c["type"] == "int"}
    bits = lambda x: "%08x" % struct.unpack("<I", struct.pack("<f", x))[0]
    for x in (4294967296.0, 2.0, 1.0, 0.5, 0.7, -0.00001, 0.00001, 0.0, 0.001, 0.0001, 0.3, 10000.0):
        assert bits(x) in floats, x
    assert {747796405, 2891336453, 28, 4, 277803737, 22, 64} <= uints
    assert {10, 9, -1} <= ints             # MAX_BOUNCES, MAX_BOUNCES-1, "no hit"
    src = open(os.path.join(HERE, "..", "oracle", "rt_oracle.c")).read()
    for lit in ("747796405u", "2891336453u", "277803737u", "0.001f", "10000.0f", "0.00001f", "0.0001f",
                "0.3f", "0.7f", "STACK_SIZE 64"):
        assert lit in src, lit


def test_spirv_call_structure():
    """The executed shader's call graph: two AA draws in main, three temp
    draws + 3 per rejection try in randomVec3InUnitSphere, metal always
    draws (scatter calls randomVec3InUnitSphere directly)."""
    calls = SPIRV["calls"]
    assert calls["main"][:2] == ["randomFloat", "randomFloat"]
    assert calls["randomVec3InUnitSphere"] == ["randomFloat"] * 6
    assert calls["scatter"] == ["randomUnitVector", "randomVec3InUnitSphere"]
    ops = {(e["function"], e["glsl_std_450"]) for e in SPIRV["glsl_std_450_ops"]}
    assert ("hit_aabb", 37) in ops and ("hit_aabb", 40) in ops      # FMin / FMax
    assert ("scatter", 71) in ops                                   # Reflect
    assert ("main", 31) in ops                                      # Sqrt (gamma)


def test_hit_aabb_kat():
    t = L().orc_hit_aabb
    lo, hi = f3(-1, -1, -1), f3(1, 1, 1)
    assert t(f3(0, 0, -5), f3(0, 0, 1), lo, hi, 0.001, 10000.0) == 1
    assert t(f3(0, 0, -5), f3(0, 0, -1), lo, hi, 0.001, 10000.0) == 0          # behind
    assert t(f3(0, 0, 0), f3(0, 0, 1), lo, hi, 0.001, 10000.0) == 1            # from inside
    assert t(f3(0, 0, -5), f3(0, 0, 1), lo, hi, 0.001, 3.0) == 0               # t_enter 4 >= t_max
    assert t(f3(2, 0, -5), f3(0, 0, 1), lo, hi, 0.001, 10000.0) == 0           # parallel, outside
    # zero direction components: 1/0 = inf; inside the x slab the x terms are -inf / +inf
    assert t(f3(0.5, 0, -5), f3(0, 0, 1), lo, hi, 0.001, 10000.0) == 1
    # exactly in the face plane: (1 - 1) * inf = NaN, fmaxf(-inf, NaN) = -inf -> miss
    # (GLSL leaves min/max of NaN undefined; the oracle and the kernel both use fminf/fmaxf)
    assert t(f3(1, 0, -5), f3(0, 0, 1), lo, hi, 0.001, 10000.0) == 0
    assert t(f3(0, 0, -5), f3(0, 0, 1), f3(-1, -1, 0), f3(1, 1, 0), 0.001, 10000.0) == 0  # flat box: t_exit == t_enter


def test_hit_triangle_kat():
    t = L().orc_hit_triangle
    v0, v1, v2 = f3(-1, -1, 0), f3(1, -1, 0), f3(-1, 1, 0)
    c = C.c_float(10000.0)
    n = (C.c_float * 3)()
    assert t(f3(-0.5, -0.5, -5), f3(0, 0, 1), v0, v1, v2, C.byref(c), n) == 1
    assert c.value == 5.0 and list(n) == [0.0, 0.0, -1.0]                       # flipped to face the ray
    c = C.c_float(10000.0)
    assert t(f3(-0.5, -0.5, 5), f3(0, 0, -1), v0, v1, v2, C.byref(c), n) == 1 and list(n) == [0.0, 0.0, 1.0]
    c = C.c_float(4.0)
    assert t(f3(-0.5, -0.5, -5), f3(0, 0, 1), v0, v1, v2, C.byref(c), n) == 0   # t >= closest
    c = C.c_float(10000.0)
    assert t(f3(0.6, 0.6, -5), f3(0, 0, 1), v0, v1, v2, C.byref(c), n) == 0     # u + v > 1
    assert t(f3(-0.5, -0.5, -5), f3(1, 0, 0), v0, v1, v2, C.byref(c), n) == 0   # parallel: det ~ 0
    assert t(f3(-0.5, -0.5, -0.0005), f3(0, 0, 1), v0, v1, v2, C.byref(c), n) == 0  # t <= T_MIN
    c = C.c_float(5.0)
    assert t(f3(-0.5, -0.5, -5), f3(0, 0, 1), v0, v1, v2, C.byref(c), n) == 0   # tie keeps the first hit


def test_scatter_kat():
    s = L().orc_scatter
    att, out = (C.c_float * 3)(), (C.c_float * 3)()
    seed = C.c_uint32(7)
    mat = (C.c_float * 4)(0.6, 0.7, 0.1, 1.0)                                   # metal, fuzz 0
    ok = s(mat, C.byref(seed), f3(0, -1, 0), f3(0, 0, 0), f3(0, 1, 0), att, out)
    assert ok == 1 and list(out) == [0.0, 1.0, 0.0] and [round(x, 6) for x in att] == [0.6, 0.7, 0.1]
    assert seed.value != 7                                                      # metal always draws
    seed = C.c_uint32(7)
    mat = (C.c_float * 4)(0.5, 0.5, 0.5, 3.0)                                   # "emissive": absorbed
    assert s(mat, C.byref(seed), f3(0, -1, 0), f3(0, 0, 0), f3(0, 1, 0), att, out) == 0
    assert seed.value == 7                                                      # no draws
    seed = C.c_uint32(7)
    mat = (C.c_float * 4)(0.5, 0.5, 0.5, 0.0)                                   # Lambertian
    assert s(mat, C.byref(seed), f3(0, -1, 0), f3(0, 0, 0), f3(0, 1, 0), att, out) == 1
    assert abs(sum(x * x for x in out) - 1.0) < 1e-6


@pytest.mark.parametrize("name", list(GOLDEN["frames"]))
def test_golden_frames(name):
    """The C oracle reproduces the committed frames (hash + counters)."""
    from oracle import oracle_lib
    from rtamd import configs
    import hashlib
    g = GOLDEN["frames"][name]
    built = configs.get(g["config"]).build()
    cam = configs.Camera.default(g["width"], g["height"])
    rgba, rad, cnt = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                       cam.ubo_bytes(), g["width"], g["height"], g["max_bounces"])
    assert hashlib.sha256(rgba.tobytes()).hexdigest() == g["rgba_sha256"]
    assert hashlib.sha256(rad.tobytes()).hexdigest() == g["radiance_sha256"]
    assert cnt == g["counts"]
    for x, y, px, rd in g["samples"]:
        assert rgba[y, x].tolist() == px and rad[y, x].tolist() == rd


@pytest.mark.parametrize("k,w,h,b", [(2, 96, 54, 3), (3, 64, 36, 4), (1, 48, 36, 1)])
def test_numpy_restatement_agrees(k, w, h, b):
    """Two independent restatements (C scalar, numpy vectorised) agree bit for bit."""
    from oracle import oracle_lib, shader_np
    from rtamd import configs
    warnings.filterwarnings("ignore")
    built = configs.get(k).build()
    cam = configs.Camera.default(w, h)
    a = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                          cam.ubo_bytes(), w, h, b)
    n = shader_np.render(built.model_vertex_data.tobytes(), built.model_material_data.tobytes(),
                         built.flat_bvh_data.tobytes(), cam.ubo_bytes(), w, h, b)
    assert np.array_equal(a[0], n[0])
    assert np.array_equal(a[1].view(np.uint32), n[1].view(np.uint32))
    assert a[2] == n[2]


def test_row_subsets_and_tiles_compose():
    """Oracle tiles / row subsets equal the corresponding parts of the full frame."""
    from oracle import oracle_lib
    from rtamd import configs
    built = configs.config2().build()
    cam = configs.Camera.default(200, 120)
    args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), 200, 120, 3)
    full, _, cf = oracle_lib.render(*args)
    sub, _, _ = oracle_lib.render(*args, tile=(0, 3, 200, 117), row_step=5)
    assert np.array_equal(sub, full[3::5])
    t, _, _ = oracle_lib.render(*args, tile=(17, 9, 50, 40))
    assert np.array_equal(t, full[9:49, 17:67])


def _ext_scene():
    """Cube + plane with the cube emissive (type 3, colour 4,4,4), as the UI's
    "Emissive (Light)" material (VulkanApp.java:487)."""
    from rtamd import build_buffers, configs, triangles_of
    verts, mats = triangles_of(configs.config2().scene)
    mats = mats.copy()
    cube = mats[:, 0] == np.float32(0.6)
    mats[cube] = (4.0, 4.0, 4.0, 3.0)
    return build_buffers(verts, mats)


@pytest.mark.parametrize("ext,sky", [(1, 0), (1, 1), (2, 1), (3, 0)])
def test_extensions_c_vs_numpy(ext, sky):
    """The non-reference extensions (ORC_EXT_*) agree bit for bit between the C
    oracle and the independent numpy restatement (parity vs the reference is
    not defined: the reference has none of them)."""
    from oracle import oracle_lib, shader_np
    from rtamd import configs
    built = _ext_scene()
    w, h = 96, 54
    cam = configs.Camera.default(w, h)
    cam.ubo.sky_enabled = sky
    args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), w, h, 5)
    rgba_c, rad_c, cnt_c = oracle_lib.render(*args, ext=ext)
    rgba_n, rad_n, cnt_n = shader_np.render(*args, ext=ext)
    assert np.array_equal(rgba_c, rgba_n)
    assert np.array_equal(rad_c.view(np.uint32), rad_n.view(np.uint32))
    assert cnt_c == cnt_n
    base = oracle_lib.render(*args)[0]
    if ext & 2:
        assert (rgba_c != base).any()           # the emitter lights the frame
    if ext == 1 and sky == 1:
        assert np.array_equal(rgba_c, base)     # sky on: the reference frame


def test_accumulation_c_vs_numpy():
    from oracle import oracle_lib, shader_np
    from rtamd import configs
    built = _ext_scene()
    w, h = 64, 40
    cam = configs.Camera.default(w, h)
    acc_c = np.zeros((h, w, 3), np.float32)
    acc_n = np.zeros((h, w, 3), np.float32)
    frames = []
    for f in range(3):
        cam.ubo.frame_count = f
        args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), w, h, 4)
        rgba_c, rad_c, _ = oracle_lib.render(*args, ext=4, accum=acc_c)
        rgba_n, rad_n, _ = shader_np.render(*args, ext=4, accum=acc_n)
        assert np.array_equal(rad_c.view(np.uint32), rad_n.view(np.uint32)), f
        assert np.array_equal(acc_c.view(np.uint32), acc_n.view(np.uint32)), f
        frames.append(rgba_c)
    cam.ubo.frame_count = 0
    ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                            cam.ubo_bytes(), w, h, 4)[0]
    assert np.array_equal(frames[0], ref)       # frame 0 is the reference's frame
    assert (frames[1] != frames[0]).any()


# ---- extension ORC_EXT_SPHERES (no reference counterpart) -------------------

SPHERES = np.array([
    (-14.0, -4.0, 4.0, 6.0, 0.8, 0.3, 0.3, 0.0),    # Lambert, resting on the ground plane
    (14.0, -5.0, -6.0, 5.0, 0.9, 0.9, 0.9, 1.0),    # mirror
    (0.0, 10.0, -12.0, 4.0, 0.7, 0.8, 0.3, 2.0),    # fuzzy metal
    (7.0, -8.0, 14.0, 2.0, 6.0, 6.0, 6.0, 3.0),     # type 3 (an emitter with EXT_EMISSIVE)
    (-3.0, 3.0, 3.0, 3.0, 0.2, 0.4, 0.9, 0.0),      # cuts a corner of the cube
], np.float32)


def _f3(*v):
    import ctypes as C
    return (C.c_float * len(v))(*v)


def test_hit_sphere_kat():
    import ctypes as C
    from oracle import oracle_lib
    L = oracle_lib.lib()
    t = C.c_float(10000.0)
    n = _f3(0, 0, 0)
    # from outside, head on: the nearer root, t = 4, normal +z
    assert L.orc_hit_sphere(_f3(0, 0, 5), _f3(0, 0, -1), _f3(0, 0, 0, 1), C.byref(t), n) == 1
    assert t.value == 4.0 and list(n) == [0.0, 0.0, 1.0]
    # from inside: the far root; the normal is turned to face the ray
    t = C.c_float(10000.0)
    assert L.orc_hit_sphere(_f3(0, 0, 0), _f3(0, 0, -1), _f3(0, 0, 0, 2), C.byref(t), n) == 1
    assert t.value == 2.0 and list(n) == [0.0, 0.0, 1.0]
    # closest_t bounds both roots; a miss leaves closest_t alone
    t = C.c_float(3.5)
    assert L.orc_hit_sphere(_f3(0, 0, 5), _f3(0, 0, -1), _f3(0, 0, 0, 1), C.byref(t), n) == 0
    assert t.value == np.float32(3.5)
    t = C.c_float(10000.0)
    assert L.orc_hit_sphere(_f3(0, 3, 5), _f3(0, 0, -1), _f3(0, 0, 0, 1), C.byref(t), n) == 0
    # behind the origin: both roots <= T_MIN
    assert L.orc_hit_sphere(_f3(0, 0, -5), _f3(0, 0, -1), _f3(0, 0, 0, 1), C.byref(t), n) == 0
    # grazing: disc == 0 hits at the tangent point
    t = C.c_float(10000.0)
    assert L.orc_hit_sphere(_f3(1, 0, 5), _f3(0, 0, -1), _f3(0, 0, 0, 1), C.byref(t), n) == 1
    assert t.value == 5.0


@pytest.mark.parametrize("ext,sky", [(8, 1), (10, 1), (9, 0), (8 | 2 | 1, 0)])
def test_spheres_c_vs_numpy(ext, sky):
    """Spheres after the BVH walk agree bit for bit between the C oracle and
    the numpy restatement; primary-segment BVH counts are unchanged by them."""
    from oracle import oracle_lib, shader_np
    from rtamd import build_buffers, configs, triangles_of
    verts, mats = triangles_of(configs.config2().scene)
    built = build_buffers(verts, mats)
    w, h = 96, 54
    cam = configs.Camera.default(w, h)
    cam.ubo.sky_enabled = sky
    args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), w, h, 5)
    rgba_c, rad_c, cnt_c = oracle_lib.render(*args, ext=ext, spheres=SPHERES)
    rgba_n, rad_n, cnt_n = shader_np.render(*args, ext=ext, spheres=SPHERES)
    assert np.array_equal(rgba_c, rgba_n)
    assert np.array_equal(rad_c.view(np.uint32), rad_n.view(np.uint32))
    assert cnt_c == cnt_n
    base, _, cnt_b = oracle_lib.render(*args, ext=ext & ~8)
    if sky or ext & 2:                          # (sky off and no emitter: all black)
        assert (rgba_c != base).any()
    # spheres passed without the bit are ignored
    assert np.array_equal(oracle_lib.render(*args, ext=ext & ~8, spheres=SPHERES)[0], base)
    # one bounce: the same BVH walk; mat_reads grows by the sphere hits
    one = args[:-1] + (1,)
    _, _, c1 = oracle_lib.render(*one, ext=ext, spheres=SPHERES)
    _, _, b1 = oracle_lib.render(*one, ext=ext & ~8)
    assert (c1["node_visits"], c1["tri_tests"]) == (b1["node_visits"], b1["tri_tests"])
    assert c1["mat_reads"] > b1["mat_reads"]


def test_spheres_only_scene():
    """Spheres with the reference's empty-scene dummies (no triangles)."""
    from oracle import oracle_lib, shader_np
    from rtamd import build_buffers, configs, triangles_of
    verts, mats = triangles_of(configs.config2().scene)
    built = build_buffers(verts[:0], mats[:0])
    w, h = 64, 36
    cam = configs.Camera.default(w, h)
    args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), w, h, 4)
    rgba_c, rad_c, cnt_c = oracle_lib.render(*args, ext=8 | 2, spheres=SPHERES)
    rgba_n, rad_n, cnt_n = shader_np.render(*args, ext=8 | 2, spheres=SPHERES)
    assert np.array_equal(rad_c.view(np.uint32), rad_n.view(np.uint32)) and cnt_c == cnt_n
    assert cnt_c["node_visits"] == 0 and cnt_c["mat_reads"] > 0
