"""Host scene pipeline (CPU): the product's C++ builder vs the Python
restatement of the Java code (oracle/scene_oracle.py), byte for byte."""
import json
import os
import random

import numpy as np
import pytest

from conftest import reference_path


def _load_json(path):
    with open(path) as f:
        return json.load(f)


HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = _load_json(os.path.join(HERE, "golden", "golden.json"))


def _oracle_build(verts, mats, seed):
    from oracle import scene_oracle
    tris = [(tuple(v[0:3]), tuple(v[3:6]), tuple(v[6:9]), tuple(m)) for v, m in zip(verts.tolist(), mats.tolist())]
    return scene_oracle.build_scene(tris, seed)


def _same(built, ref):
    vb, mb, bb, nf = ref
    assert built.triangle_count == nf
    assert built.model_vertex_data.tobytes() == vb
    assert built.model_material_data.tobytes() == mb
    assert built.flat_bvh_data.tobytes() == bb


def test_layout_sizes():
    from oracle import scene_oracle
    import ctypes as C
    from rtamd import lib
    for n in list(range(0, 300)) + [1000, 4097, 50_000, 1_000_000]:
        nn, nf = C.c_size_t(), C.c_size_t()
        assert lib().rt_bvh_layout_size(n, C.byref(nn), C.byref(nf)) == 0
        assert (nn.value, nf.value) == scene_oracle.layout_size(n)
        if n:
            assert nn.value == 2 * nf.value - 1          # full binary tree


@pytest.mark.parametrize("k", [1, 2])
def test_config_scenes_match_restatement(k):
    from rtamd import configs, build_buffers, triangles_of
    cfg = configs.get(k)
    verts, mats = triangles_of(cfg.scene)
    for seed in (1, 2, 12345):
        _same(build_buffers(verts, mats, seed), _oracle_build(verts, mats, seed))


def _random_tris(n, rng, grid=False):
    if grid:   # many exactly tied centroids, flat (axis-aligned) triangles, negative zeros
        pts = rng.integers(-3, 4, size=(n, 3, 3)).astype(np.float64)
        pts[rng.random((n, 3, 3)) < 0.1] = -0.0
        pts[rng.random(n) < 0.3, :, 1] = 0.0
    else:
        pts = rng.normal(size=(n, 3, 3)) * rng.uniform(0.1, 10, size=(n, 1, 1))
    mats = rng.random((n, 4)).astype(np.float32)
    mats[:, 3] = rng.integers(0, 4, n)
    return pts.reshape(n, 9), mats


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 16, 17, 100, 257, 1500])
@pytest.mark.parametrize("grid", [False, True])
def test_random_scenes_match_restatement(n, grid):
    from rtamd import build_buffers
    rng = np.random.default_rng(n * 7 + grid)
    verts, mats = _random_tris(n, rng, grid)
    seed = int(rng.integers(0, 1 << 62))
    _same(build_buffers(verts, mats, seed), _oracle_build(verts, mats, seed))


def test_thread_count_does_not_change_output():
    from rtamd import build_buffers
    rng = np.random.default_rng(5)
    verts, mats = _random_tris(120_000, rng)
    a = build_buffers(verts, mats, 3, n_threads=1)
    b = build_buffers(verts, mats, 3, n_threads=8)
    for x, y in ((a.model_vertex_data, b.model_vertex_data), (a.model_material_data, b.model_material_data),
                 (a.flat_bvh_data, b.flat_bvh_data)):
        assert np.array_equal(x, y)


def test_built_buffers_validate_and_are_preorder():
    import ctypes as C
    from rtamd import lib, configs
    for k in (1, 2, 3):
        b = configs.get(k).build()
        nn, depth = C.c_size_t(), C.c_int()
        assert lib().rt_scene_validate(b.model_vertex_data.ctypes.data, b.model_vertex_data.nbytes,
                                       b.model_material_data.ctypes.data, b.model_material_data.nbytes,
                                       b.flat_bvh_data.ctypes.data, b.flat_bvh_data.nbytes,
                                       C.byref(nn), C.byref(depth)) == 0
        assert nn.value == b.n_nodes


@pytest.mark.parametrize("name", list(GOLDEN["scenes"]))
def test_config_buffers_golden(name):
    import hashlib
    from rtamd import configs
    k = int(name[3])
    cfg = configs.get(k)
    b = cfg.build()
    g = GOLDEN["scenes"][name]
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert (b.triangle_count, b.n_nodes) == (g["flat_triangles"], g["nodes"])
    assert sha(b.model_vertex_data) == g["vertices_sha256"]
    assert sha(b.model_material_data) == g["materials_sha256"]
    assert sha(b.flat_bvh_data) == g["nodes_sha256"]
    assert cfg.camera().ubo_bytes().hex() == g["camera_ubo_hex"]


def test_camera_matches_restatement():
    from oracle import scene_oracle
    from rtamd import Camera
    rng = random.Random(3)
    cams = [((-25, 30, 140), (0, 0, 0), (0, 1, 0), 20.0, 1280 / 720)]
    for _ in range(50):
        o = tuple(rng.uniform(-200, 200) for _ in range(3))
        la = tuple(rng.uniform(-20, 20) for _ in range(3))
        cams.append((o, la, (0.0, 1.0, 0.0), rng.uniform(5, 120), rng.uniform(0.3, 4.0)))
    for o, la, up, fov, asp in cams:
        c = Camera(o, la, up, fov, asp)
        assert c.ubo_bytes() == scene_oracle.camera_ubo(tuple(map(float, o)), tuple(map(float, la)),
                                                        up, fov, asp)


def test_camera_move_recomputes_viewport():
    from rtamd import Camera
    c = Camera.default(1280, 720)
    before = c.ubo_bytes()
    c.set_origin((-25 + 5.5, 30, 140))          # VulkanApp 'D' key, VulkanApp.java:765
    assert c.ubo_bytes() != before and c.get_origin() == (-19.5, 30.0, 140.0)


def test_procedural_mesh():
    from rtamd import Mesh
    from rtamd.configs import FINAL_BASE_MESH_BMAX, FINAL_BASE_MESH_BMIN
    for n in (8, 1000, 50_000, 200_002):
        m = Mesh.procedural(n, 0x5EED, FINAL_BASE_MESH_BMIN, FINAL_BASE_MESH_BMAX)
        assert len(m) == n
        assert (m.tris.min(axis=(0, 1)) >= np.float32(FINAL_BASE_MESH_BMIN) - 1e-3).all()
        assert (m.tris.max(axis=(0, 1)) <= np.float32(FINAL_BASE_MESH_BMAX) + 1e-3).all()
    # closed: every undirected edge is shared by exactly two triangles
    m = Mesh.procedural(1000, 1, (-1, -1, -1), (1, 1, 1))
    v = m.tris.reshape(-1, 3)
    _, idx = np.unique(v, axis=0, return_inverse=True)
    t = idx.reshape(-1, 3)
    edges = np.sort(np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [2, 0]]]), axis=1)
    _, cnt = np.unique(edges, axis=0, return_counts=True)
    assert (cnt == 2).all()
    a = Mesh.procedural(5000, 9, (-1, -1, -1), (1, 1, 1)).tris
    b = Mesh.procedural(5000, 9, (-1, -1, -1), (1, 1, 1)).tris
    assert np.array_equal(a, b)


def test_obj_loader_on_reference_assets():
    """SceneBuilder.loadModel inputs: the reference's own OBJ files (read when
    the reference checkout is present; the configs embed the same triangles)."""
    from rtamd import Mesh
    from rtamd.configs import cube_mesh, plane_mesh
    assert np.array_equal(Mesh.load_obj(reference_path("objects", "cube.obj")).tris, cube_mesh().tris)
    assert np.array_equal(Mesh.load_obj(reference_path("objects", "ground_plane.obj")).tris, plane_mesh().tris)
    fbm = Mesh.load_obj(reference_path("objects", "FinalBaseMesh.obj"))
    assert len(fbm) == 48_918                   # 24,459 quads -> 2 triangles each
    lo, hi = fbm.tris.min(axis=(0, 1)), fbm.tris.max(axis=(0, 1))
    assert np.allclose(lo, [-5.8425, -0.0566, -1.8531]) and np.allclose(hi, [5.8425, 20.6841, 1.9170])


def test_obj_loader_formats(tmp_path):
    from rtamd import Mesh, RtError
    p = tmp_path / "m.obj"
    p.write_text("# c\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\n"
                 "f 1/1/1 2/2/1 3/3/1 4/4/1\nf -4 -2 -1\nl 1 2\n")
    m = Mesh.load_obj(str(p))
    assert len(m) == 3                          # quad -> 2, triangle with relative indices -> 1
    assert m.tris[2].tolist() == [[0, 0, 0], [1, 1, 0], [0, 1, 0]]
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(RtError, match="IO"):
        Mesh.load_obj(str(bad))
    with pytest.raises(RtError, match="IO"):
        Mesh.load_obj(str(tmp_path / "missing.obj"))


def test_scene_builder_skips_unloadable_models(tmp_path):
    """SceneBuilder.java:55-58: a model that fails to load is skipped."""
    from rtamd import ModelInstance, Scene, SceneBuilder
    from rtamd.configs import ground_plane_instance
    s = Scene()
    s.add_instance(ModelInstance(str(tmp_path / "nope.obj"), "missing"))
    s.add_instance(ground_plane_instance())
    b = SceneBuilder().build_scene(s)
    assert b.triangle_count == 2                # 2 plane triangles -> one node with 2 leaves
    empty = SceneBuilder().build_scene(Scene())
    assert empty.triangle_count == 0 and empty.flat_bvh_data.size == 1   # the 1-byte dummy


def test_final_base_mesh_fixture():
    """Config 6 renders the reference's own objects/FinalBaseMesh.obj from the
    gzip'd fixture (tests/golden/FinalBaseMesh.obj.gz): the OBJ loader gives
    48,918 triangles (24,459 quads), and with the plane and the cube the
    reference builder's split rule gives 2·flat − 1 nodes."""
    from rtamd import configs
    m = configs.final_base_mesh()
    assert len(m) == 48_918
    lo, hi = m.tris.min(axis=(0, 1)), m.tris.max(axis=(0, 1))
    assert np.allclose(lo, configs.FINAL_BASE_MESH_BMIN, atol=1e-4)
    assert np.allclose(hi, configs.FINAL_BASE_MESH_BMAX, atol=1e-4)
    built = configs.get(6).build()
    flat = built.triangle_count
    assert flat == 65_096
    assert built.flat_bvh_data.nbytes == 48 * (2 * flat - 1)
    from conftest import REFERENCE
    src = os.path.join(REFERENCE, "objects", "FinalBaseMesh.obj")
    if os.path.exists(src):                     # the fixture is the reference's file, unchanged
        from rtamd import Mesh
        assert np.array_equal(Mesh.load_obj(src).tris, m.tris)


def _obj_text(rng, n_polys=60):
    """Random OBJ: star-shaped and comb-shaped (concave) polygons of 3-14
    corners in random planes, coordinates written with 1-18 fraction digits,
    exponents, '+' signs and leading dots, plus one self-intersecting face."""
    lines, nv = [], 0

    def num(x):
        k = int(rng.integers(0, 6))
        if k == 0:
            return f"{x:.{int(rng.integers(1, 19))}f}"
        if k == 1:
            return f"{x:.{int(rng.integers(1, 9))}e}"
        if k == 2:
            return ("+" if x >= 0 else "") + f"{x:.6f}"
        if k == 3 and abs(x) < 1:
            return ("-" if x < 0 else "+") + f"{abs(x):.7f}"[1:]      # "+.1234567" (a bare "." does not count)
        return repr(float(np.float32(x)))

    for pi in range(n_polys):
        n = int(rng.integers(3, 15))
        ang = np.sort(rng.uniform(0, 2 * np.pi, n))
        if pi % 3 == 0:                                          # comb: alternating radii
            rad = np.where(np.arange(n) % 2 == 0, 1.0, rng.uniform(0.05, 0.5, n))
        else:
            rad = rng.uniform(0.2, 1.5, n)
        if pi % 5 == 4:
            ang = ang[::-1]                                      # clockwise winding
        pts2 = np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)
        u, v = rng.normal(size=3), rng.normal(size=3)
        if pi % 4 == 1:                                          # axis-aligned planes, both signs
            ax = int(rng.integers(0, 3))
            u = np.eye(3)[(ax + 1) % 3] * rng.choice([-1, 1])
            v = np.eye(3)[(ax + 2) % 3]
        o = rng.normal(size=3) * 5
        for p in pts2:
            x = o + p[0] * u + p[1] * v
            lines.append("v " + " ".join(num(c) for c in x))
        lines.append("f " + " ".join(str(nv + k + 1) for k in range(n)))
        nv += n
    # a self-intersecting hexagon (figure eight): no ear is found twice round
    for x, y in ((0, 0), (2, 2), (4, 0), (4, 2), (2, 0), (0, 2)):
        lines.append(f"v {x} {y} 0")
    lines.append("f " + " ".join(str(nv + k + 1) for k in range(6)))
    return "\n".join(lines) + "\n"


def test_obj_loader_matches_assimp_restatement(tmp_path):
    """rt_mesh_load_obj vs oracle/obj_oracle.py (an independent restatement of
    Assimp's fast_atof, OBJ 'v' lines and aiProcess_Triangulate): bit-exact
    triangles, in order, on random concave / convex / clockwise polygons of
    3-14 corners in random and axis-aligned planes, numbers written in many
    forms.  Parity vs a real Assimp run is unpinned."""
    from oracle import obj_oracle as oo
    from rtamd import Mesh
    for seed in range(6):
        p = tmp_path / f"poly{seed}.obj"
        p.write_text(_obj_text(np.random.default_rng(seed)))
        got = Mesh.load_obj(str(p)).tris
        want = oo.load_obj(str(p)) + np.float32(0)       # the loader's x*1 + 0 turns -0 into +0
        assert got.shape == want.shape, (seed, got.shape, want.shape)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), seed


def test_obj_ear_clipping_properties(tmp_path):
    """Every simple polygon of n corners gives n - 2 triangles covering its
    area, each wound like the polygon (ear clipping, not a fan: a fan from
    corner 0 of a comb polygon leaves it and overlaps itself)."""
    from rtamd import Mesh
    rng = np.random.default_rng(7)
    for trial in range(40):
        n = int(rng.integers(5, 16))
        ang = (np.arange(n) + rng.uniform(0.1, 0.9, n)) * (2 * np.pi / n)   # star-shaped around 0: simple
        rad = np.where(np.arange(n) % 2 == 0, 1.0, rng.uniform(0.05, 0.6, n))
        pts = np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1).astype(np.float32)
        p = tmp_path / f"comb{trial}.obj"
        p.write_text("".join(f"v {float(x)!r} {float(y)!r} 0\n" for x, y in pts)
                     + "f " + " ".join(str(k + 1) for k in range(n)) + "\n")
        t = Mesh.load_obj(str(p)).tris.astype(np.float64)[:, :, :2]
        assert len(t) == n - 2
        area = 0.5 * ((t[:, 1, 0] - t[:, 0, 0]) * (t[:, 2, 1] - t[:, 0, 1])
                      - (t[:, 2, 0] - t[:, 0, 0]) * (t[:, 1, 1] - t[:, 0, 1]))
        x, y = pts[:, 0].astype(np.float64), pts[:, 1].astype(np.float64)
        poly = 0.5 * np.sum(x * np.roll(y, -1) - np.roll(x, -1) * y)
        assert (area > -1e-9).all(), trial                # every triangle counter-clockwise like the polygon
        assert abs(area.sum() - poly) < 1e-5 * max(1.0, abs(poly)), (trial, area.sum(), poly)


def test_obj_numbers_are_assimp_fast_atof(tmp_path):
    """Assimp parses OBJ numbers with fast_atof, not a correctly rounded
    strtof: FinalBaseMesh's coordinates (4 decimals) differ from strtof in
    about 5% of cases, and the loader follows Assimp."""
    import gzip
    from oracle import obj_oracle as oo
    vals = []
    with gzip.open(os.path.join(os.path.dirname(__file__), "golden", "FinalBaseMesh.obj.gz"), "rt") as fh:
        for ln in fh:
            if ln.startswith("v "):
                vals.extend(ln.split()[1:4])
    vals = vals[:6000]
    fa = np.array([oo.fast_atof(t) for t in vals], dtype=np.float32)
    st = np.array([float(t) for t in vals], dtype=np.float32)
    assert 0.01 < np.mean(fa != st) < 0.2
    assert np.all(np.abs(fa.astype(np.float64) - st) <= np.spacing(np.abs(st)))   # one ulp at most
    p = tmp_path / "nums.obj"
    toks = ["1.5", "-0.25", "+3", "+.5", "-.75", "1e3", "2.5E-2", "7.", "1,5", "123456789012.123456789012345678",
            "0.1234567890123456789", "-1.000000000000000001"]
    body = "".join(f"v {toks[k]} {toks[(k + 1) % len(toks)]} {toks[(k + 2) % len(toks)]}\n" for k in range(len(toks)))
    body += "".join(f"f {k + 1} {(k + 1) % len(toks) + 1} {(k + 2) % len(toks) + 1}\n" for k in range(len(toks)))
    p.write_text(body)
    from rtamd import Mesh
    got = Mesh.load_obj(str(p)).tris
    want = oo.load_obj(str(p)) + np.float32(0)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert got[0, 0].tolist() == [1.5, -0.25, 3.0]


def test_obj_vertex_component_rule(tmp_path):
    """ObjFileParser counts a 'v' line's components as the tokens that start
    like a number (a digit, '-', '+', nan / inf): a trailing comment does not
    count; a count other than 3, 4 or 6 adds no vertex (later indices shift);
    6 is xyz + a colour.  "1e" (no exponent digits) fails the import, as
    Assimp's strtoul10_64 throws.  Both restatements agree."""
    from oracle import obj_oracle as oo
    from rtamd import Mesh, RtError
    p = tmp_path / "rule.obj"
    p.write_text("v 1 2 3 # a note\n"          # 3 components: (1, 2, 3)
                 "v .5 1 2\n"                  # '.5' does not count: 2 -> no vertex
                 "v 4 5 6 7 8\n"               # 5 -> no vertex
                 "v 0 1 0 0.5 0.25 1\n"        # 6: xyz + colour
                 "v 2 4 6 2\n"                 # 4: divided by w
                 "v -1 -2 -3\n"
                 "v 99999999999999999999 1 2\n"   # integer overflow: Assimp's 0, with a warning
                 "f 1 2 3\nf 2 3 4\nf 1 4 5\n")
    got = Mesh.load_obj(str(p)).tris
    want = oo.load_obj(str(p)) + np.float32(0)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert got[0].tolist() == [[1, 2, 3], [0, 1, 0], [1, 2, 3]]
    assert got[1].tolist() == [[0, 1, 0], [1, 2, 3], [-1, -2, -3]]
    assert got[2, 2, 0] == oo.fast_atof("99999999999999999999")
    bad = tmp_path / "exp.obj"
    bad.write_text("v 1e 2 3\nv 0 0 0\nv 1 0 0\nf 1 2 3\n")
    with pytest.raises(RtError, match="IO"):
        Mesh.load_obj(str(bad))
    with pytest.raises(ValueError):
        oo.load_obj(str(bad))
