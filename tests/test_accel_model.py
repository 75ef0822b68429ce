"""Option accel on the CPU: the records rt_accel_records builds
and the accel walk's CPU model (oracle/rt_accel_model.c) against the
reference-order oracle (oracle/rt_oracle.c).

The accel walk visits a binned-SAH tree near child first, enters a box when
t_enter <= closest_t and takes a triangle on t < closest_t or on a tie with a
lower flattened index.  The claim: its frames are the reference's, bit for
bit, while its node visits differ by design.  tools/accel_study.py measured
whole frames of configs 1-6 (tests/golden/accel_study.json); these tests
re-check small cases, tie-heavy scenes and the record format."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _records(built, n_layouts, half=False):
    """half: True = option accel_half's format, "wide" = option accel_wide's."""
    from rtamd import _lib
    return _lib.accel_records(built, n_layouts, half is True, half == "wide")


def _frames(built, cam, w, h, b, n_layouts, tile=None, row_step=1, half=False):
    from oracle import oracle_lib as O
    args = (built.model_vertex_data, built.model_material_data, built.flat_bvh_data, cam.ubo_bytes(), w, h, b)
    ref = O.render(*args, tile=tile, row_step=row_step)
    rec, info = _records(built, n_layouts, half)
    acc = O.render_accel(*args, rec, info, tile=tile, row_step=row_step)
    return ref, acc


def _assert_frames_equal(ref, acc, what=""):
    (r_rgba, r_rad, r_c), (a_rgba, a_rad, a_c) = ref, acc
    bad = (r_rgba != a_rgba).any(-1) | (r_rad.view(np.uint32) != a_rad.view(np.uint32)).any(-1)
    assert not bad.any(), f"{what}: {int(bad.sum())} pixels differ, first at {np.argwhere(bad)[0]}"
    # the path of every pixel is the reference's: same segments and hits
    assert a_c["segments"] == r_c["segments"] and a_c["mat_reads"] == r_c["mat_reads"], what


def _walk_all(rec, info, o):
    """Every slot of layout o in walk order with every box entered: the walk
    must reach each leaf exactly once and end at the layout's end."""
    s = info["slots"]
    n, end, leaf = o * s, (o + 1) * s, bool(info["root_leaf"])
    tris, steps = [], 0
    while n < end:
        aw, bw = int(rec[8 * n + 3]), int(rec[8 * n + 7])
        assert bool((aw >> 30) & 1) == leaf, f"slot {n}: bit 30 disagrees with the L bit that led here"
        if leaf:
            tris.append(aw & 0x1FFFFFFF)
            n, leaf = n + 2, bool(aw >> 31)
        else:
            skip = aw & 0x1FFFFFFF
            assert n < skip <= end
            n, leaf = n + 1, bool(bw >> 31)
        steps += 1
        assert steps <= s
    assert n == end
    return tris


def _walk_all_half(rec, info, o):
    """_walk_all over format 1 (option accel_half): 16-B slots, a leaf four."""
    s = info["slots"]
    n, end, leaf = o * s, (o + 1) * s, bool(info["root_leaf"])
    tris, steps = [], 0
    while n < end:
        aw = int(rec[4 * n + 3])
        if leaf:
            assert (aw >> 30) & 1, f"slot {n}: a leaf without its marker"
            tris.append(aw & 0x1FFFFFFF)
            n, leaf = n + 4, bool(aw >> 31)
        else:
            skip = aw & 0x3FFFFFFF
            assert n < skip <= end
            n, leaf = n + 1, bool((aw >> 30) & 1)
        steps += 1
        assert steps <= s
    assert n == end
    return tris


def _half(bits):
    return np.array(bits, dtype=np.uint16).view(np.float16).astype(np.float32)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_record_layouts_half(k):
    """Option accel_half's records: 5m - 1 16-B slots per layout, the same
    triangles in the same walk order as format 0, every leaf's 64 bytes equal
    to format 0's, and every internal box the format-0 box rounded outward to
    the nearest halves (lo down, hi up)."""
    from rtamd import configs
    built = configs.get(k).build()
    for nl in (1, 8):
        r0, i0 = _records(built, nl)
        r1, i1 = _records(built, nl, half=True)
        m = i0["n_prims"]
        assert i1["slots"] == 5 * m - 1 and r1.size == 4 * nl * i1["slots"] + 16
        for o in range(nl):
            assert _walk_all_half(r1, i1, o) == _walk_all(r0, i0, o)
            # walk both layouts in step, every box entered: the same nodes
            a, b = o * i0["slots"], o * i1["slots"]
            leaf = bool(i0["root_leaf"])
            while a < (o + 1) * i0["slots"]:
                w0, w1 = r0[8 * a: 8 * a + 16], r1[4 * b: 4 * b + 16]
                if leaf:
                    assert np.array_equal(w0, w1)
                    leaf = bool(int(w0[3]) >> 31)
                    a, b = a + 2, b + 4
                else:
                    lo0, hi0 = w0[0:3].view(np.float32), w0[4:7].view(np.float32)
                    h = w1[0:3].astype(np.uint32)
                    lo1 = _half([h[0] & 0xFFFF, h[0] >> 16, h[1] & 0xFFFF])
                    hi1 = _half([h[1] >> 16, h[2] & 0xFFFF, h[2] >> 16])
                    assert (lo1 <= lo0).all() and (hi1 >= hi0).all()
                    # the nearest halves outward: one step further in would cut the box
                    lo_in = np.nextafter(lo1.astype(np.float16), np.float16(np.inf)).astype(np.float32)
                    hi_in = np.nextafter(hi1.astype(np.float16), np.float16(-np.inf)).astype(np.float32)
                    assert ((lo_in > lo0) | ~np.isfinite(lo1)).all() and ((hi_in < hi0) | ~np.isfinite(hi1)).all()
                    leaf = bool(int(w0[7]) >> 31)
                    assert leaf == bool((int(w1[3]) >> 30) & 1)
                    a, b = a + 1, b + 1


@pytest.mark.parametrize("k", [1, 2, 3])
def test_record_layouts(k):
    from rtamd import configs
    built = configs.get(k).build()
    for nl in (1, 8):
        rec, info = _records(built, nl)
        assert rec.size == 8 * (nl * info["slots"] + 2)
        assert info["slots"] == 3 * info["n_prims"] - 1
        first = None
        for o in range(nl):
            tris = _walk_all(rec, info, o)
            assert len(tris) == info["n_prims"] == len(set(tris))
            if first is None:
                first = sorted(tris)
            assert sorted(tris) == first            # every layout holds the same triangles
        # a flattened triangle dropped as a duplicate is byte-identical to a kept one
        vb = built.model_vertex_data.view(np.uint8).reshape(-1, 48)
        kept = {vb[t].tobytes() for t in first}
        for t in range(built.triangle_count):
            assert vb[t].tobytes() in kept


def test_duplicates_dropped():
    from rtamd import configs
    built = configs.config3().build()
    _, info = _records(built, 1)
    # 50,000 triangles + plane (2) + cube (12); the reference's one-triangle
    # nodes flatten to two copies (BVHBuilder.java:60-62): 65,536 leaves
    assert info["n_inputs"] == 65536 and info["n_prims"] == 50014


@pytest.mark.parametrize("nl,half", [(1, False), (8, False), (8, True), (8, "wide")])
@pytest.mark.parametrize("k,b,tile,row_step", [(1, 1, None, 1), (2, 2, None, 2), (2, 10, (400, 200, 480, 320), 1),
                                                 (3, 4, None, 24), (6, 4, None, 40)])
def test_model_matches_oracle(k, b, tile, row_step, nl, half):
    from rtamd import configs
    cfg = configs.get(k)
    built = cfg.build()
    ref, acc = _frames(built, cfg.camera(), cfg.width, cfg.height, b, nl, tile=tile, row_step=row_step, half=half)
    _assert_frames_equal(ref, acc, f"config {k} half {half}")
    # far fewer box tests than the reference's walk (3: 36.8 vs 8.2 per segment)
    if k >= 3:
        assert acc[2]["node_visits"] < 0.4 * ref[2]["node_visits"]


def random_scene(seed):
    """A random triangle soup: well-shaped triangles, needles (one edge 1e-4 -
    1e-2 of the other) and tiny ones, in a box of random size and offset, every
    material type."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(20, 600))
    scale = float(10.0 ** rng.uniform(-1, 2))
    off = rng.uniform(-1, 1, 3) * float(10.0 ** rng.uniform(0, 3))
    c = rng.uniform(-1, 1, (n, 3)) * scale + off
    e1 = rng.normal(size=(n, 3)) * scale * 0.4
    e2 = rng.normal(size=(n, 3)) * scale * 0.4
    kind = rng.integers(0, 3, n)
    needle = kind == 1
    e2[needle] = e1[needle] * (1.0 + rng.uniform(-1, 1, (int(needle.sum()), 1)) * 1e-3) + \
        rng.normal(size=(int(needle.sum()), 3)) * scale * 10.0 ** rng.uniform(-6, -3, (int(needle.sum()), 1))
    tiny = kind == 2
    e1[tiny] *= 1e-3
    e2[tiny] *= 1e-3
    verts = np.stack([c, c + e1, c + e2], 1).astype(np.float32)
    mats = np.concatenate([rng.uniform(0.1, 0.95, (n, 3)), rng.integers(0, 3, (n, 1))], 1).astype(np.float32)
    eye = off + rng.uniform(-1, 1, 3) * scale * 3.0
    return verts, mats, (tuple(eye.tolist()), tuple(off.tolist())), float(rng.uniform(20, 90))


@pytest.mark.parametrize("nl", [1, 8])
def test_model_random_scenes(nl):
    """random_scene's 24 soups (tests/test_gpu_accel.py runs them on the GPU):
    the model's frames equal the oracle's."""
    from rtamd import build_buffers, configs
    for seed in range(24):
        verts, mats, (eye, at), vfov = random_scene(seed)
        w, h, b = 64, 48, 3
        cam = configs.Camera(eye, at, (0.0, 1.0, 0.0), vfov, w / h)
        built = build_buffers(verts, mats, 1 + seed % 3)
        ref, acc = _frames(built, cam, w, h, b, nl)
        _assert_frames_equal(ref, acc, f"random scene {seed}")


def _tie_scenes():
    from rtamd import build_buffers, configs, triangles_of
    verts, mats = triangles_of(configs.config2().scene)
    rng = np.random.default_rng(7)
    out = {}
    # twins: every triangle twice, the copy in another colour: equal t on every
    # hit, the lower flattened index must win (the reference's first found)
    m2 = mats.copy()
    m2[:, :3] = 1.0 - m2[:, :3]
    out["twins"] = build_buffers(np.concatenate([verts, verts]), np.concatenate([mats, m2]), 1)
    out["twins_rev"] = build_buffers(np.concatenate([verts, verts]), np.concatenate([m2, mats]), 3)
    # an integer grid: coplanar, coincident and axis-aligned faces, shared edges
    g = rng.integers(-3, 4, size=(300, 3, 3)).astype(np.float64) * 4.0
    gm = np.concatenate([rng.random((300, 3)), rng.integers(0, 4, (300, 1))], 1).astype(np.float32)
    out["grid"] = build_buffers(g.reshape(300, 9), gm, 5)
    # the cube's faces also split along their other diagonal, in other
    # colours: coincident triangles that cross, ties on half of each face
    q = verts[2:].reshape(-1, 2, 3, 3)     # face k: triangles (a, b, c) and (a, c, d)
    a, b, c, d = q[:, 0, 0], q[:, 0, 1], q[:, 0, 2], q[:, 1, 2]
    other = np.stack([np.stack([a, b, d], 1), np.stack([b, c, d], 1)], 1).reshape(-1, 9)
    out["cube_both_diagonals"] = build_buffers(np.concatenate([verts, other]),
                                               np.concatenate([mats, m2[2:]]), 2)
    return out


@pytest.mark.parametrize("nl,half", [(1, False), (8, False), (8, True), (8, "wide")])
def test_model_ties(nl, half):
    from rtamd import configs
    for name, built in _tie_scenes().items():
        for (w, h, b) in [(160, 90, 3), (97, 61, 10)]:
            cam = configs.Camera.default(w, h)
            ref, acc = _frames(built, cam, w, h, b, nl, half=half)
            _assert_frames_equal(ref, acc, f"{name} {w}x{h}x{b} half {half}")


def test_model_tree_independent():
    """The reference's frame does not depend on its random tree (SURVEY.md §0
    fact 9), and the accel walk's does not depend on which reference tree its
    primitives came from."""
    from rtamd import configs
    from oracle import oracle_lib as O
    cfg = configs.config2()
    cam = cfg.camera()
    frames = []
    for seed in (1, 2, 3):
        built = cfg.build(axis_seed=seed)
        ref, acc = _frames(built, cam, cfg.width, cfg.height, 2, 1, row_step=3)
        _assert_frames_equal(ref, acc, f"seed {seed}")
        frames.append(acc[0])
    assert all(np.array_equal(frames[0], f) for f in frames[1:])


def test_study_claims():
    with open(os.path.join(HERE, "golden", "accel_study.json")) as f:
        d = json.load(f)
    names = {c["config"] for c in d["cases"]}
    assert {"cfg2_cube_plane_1280x720_b2", "cfg3_50k_1920x1080_b4", "cfg6_fbm_1920x1080_b4",
            "cfg5_1M_3840x2160_b8"} <= names
    for c in d["cases"]:
        for k, e in c["accel"].items():
            assert e["rgba_px"] == 0 and e["radiance_px"] == 0, (c["config"], k)
            if k in ("layouts1", "layouts8"):
                assert e["segments_equal"] and e["mat_reads_equal"]
                # rare: hits on a face that lies on its box's entry plane (the
                # cube of configs 1-2 is a large share of those frames)
                assert e["fallback_segments"] < (1e-2 if c["config"].startswith(("cfg1", "cfg2")) else 1e-3) * \
                    e["segments"]
        if c["config"].startswith(("cfg3", "cfg5", "cfg6")):
            ref = c["reference_seed1"]["visits_per_segment"]
            assert c["accel"]["layouts1"]["visits_per_segment"] < ref / 3.0


@pytest.mark.parametrize("k", [3])
def test_forced_records(k):
    """Format 0's thin-triangle rule (accel_build.h kAccelForce): bit 29 of a
    record's word 3 is set exactly when its subtree holds a triangle of shape
    class >= 7 (a leaf: its own), in every layout; internal word 7 is L(first
    child) << 31 only."""
    from rtamd import configs
    built = configs.get(k).build()
    rec, info = _records(built, 8)
    s = info["slots"]
    w = rec[: 8 * 8 * s].reshape(-1, 8)
    v = built.model_vertex_data.view(np.float32).reshape(-1, 12)
    e1, e2 = (v[:, 4:7] - v[:, 0:3]).astype(np.float64), (v[:, 8:11] - v[:, 0:3]).astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        sn = np.linalg.norm(np.cross(e1, e2), axis=1) / (np.linalg.norm(e1, axis=1) * np.linalg.norm(e2, axis=1))
        thin_tri = ~(sn > 0.0) | (np.floor(-np.log2(sn)) >= 7)

    def thin(tri):
        return bool(thin_tri[tri])

    n_thin, n_forced = 0, 0
    for o in range(8):
        n, end, leaf = o * s, (o + 1) * s, bool(info["root_leaf"])
        stack = []                       # (end of subtree, index of its record)
        forced_below = {}
        while n < end:
            while stack and n >= stack[-1][0]:
                stack.pop()
            aw = int(w[n, 3])
            if leaf:
                t = thin(aw & 0x1FFFFFFF)
                assert bool(aw & (1 << 29)) == t, (o, n)
                if t:
                    n_thin += o == 0
                    for _, i in stack:
                        forced_below[i] = True
                n, leaf = n + 2, bool(aw >> 31)
            else:
                assert int(w[n, 7]) in (0, 1 << 31)
                sk = aw & 0x1FFFFFFF
                # L(skip): the record the skip lands on is a leaf (its bit 30)
                assert bool(aw >> 31) == (sk < end and bool((int(w[sk, 3]) >> 30) & 1)), (o, n)
                stack.append((sk, n))
                forced_below.setdefault(n, False)
                n, leaf = n + 1, bool(int(w[n, 7]) >> 31)
        for i, f in forced_below.items():
            assert bool(int(w[i, 3]) & (1 << 29)) == f, (o, i)
            n_forced += f
    assert n_thin == info["n_thin"] > 0 and n_forced > 0


def test_trailing_subtree_not_a_primitive():
    """A valid upload may hold nodes past the root's subtree (a second tree
    appended after it): the reference's DFS never reaches them, so the accel
    records must not hold their triangles.  The combined buffers give exactly
    the first scene's records, and the model's frame is the oracle's (advisor
    finding, round 5)."""
    from raw_bvh import raw_bvh_scene, trailing_subtree_scene
    from rtamd import configs
    first = configs.config2().build()
    second = raw_bvh_scene(40, "random", seed=3)        # triangles in front of the default camera
    both = trailing_subtree_scene(first, second)
    for nl in (1, 8):
        r0, i0 = _records(first, nl)
        r1, i1 = _records(both, nl)
        assert i1 == i0 and np.array_equal(r1, r0)
    w, h, b = 160, 90, 4
    cam = configs.Camera.default(w, h)
    ref, acc = _frames(both, cam, w, h, b, 8)
    _assert_frames_equal(ref, acc, "trailing subtree")
    # the appended triangles are in view: walking them would change the frame
    from oracle import oracle_lib as O
    alone = O.render(second.model_vertex_data, second.model_material_data, second.flat_bvh_data,
                     cam.ubo_bytes(), w, h, b)
    assert (alone[0] != ref[0]).any()


def _coincident(n, nested=False):
    """n triangles about one centre, each its own colour (no byte-identical
    copies to drop): identical (nested=False) or scaled copies of one
    triangle (nested boxes, one centroid)."""
    from rtamd import build_buffers
    base = np.array([[-2.0, -1.0, 0.0], [2.0, -1.0, 0.5], [0.0, 2.0, -0.5]])
    s = (1.0 + np.arange(n) / n)[:, None, None] if nested else np.ones((n, 1, 1))
    verts = (base[None] * s).reshape(n, 9)
    mats = np.stack([np.arange(n) / n, (np.arange(n) % 97) / 97.0, np.full(n, 0.5),
                     np.arange(n) % 3], 1).astype(np.float32)
    return build_buffers(verts, mats, 1)


@pytest.mark.parametrize("nested", [False, True])
def test_coincident_triangles_build_bounded(nested):
    """~100k triangles whose boxes or centroids coincide: every SAH split ties
    (or peels the largest box off), which once built a tree 100k deep in
    O(n^2) on every upload (advisor finding, round 5).  Ties now keep the
    split nearest the middle and below depth 64 nodes split at the median,
    so the tree stays shallow and the build quick."""
    import time
    built = _coincident(100_000, nested)
    t0 = time.time()
    _, info = _records(built, 1)
    dt = time.time() - t0
    assert info["n_prims"] == 100_000
    assert info["depth"] <= 64 + 18, info
    assert dt < 30.0, dt


def test_coincident_triangles_frames():
    """Coincident triangles in different colours: every hit ties, the lowest
    flattened index wins (the reference's first found); the model's frame is
    the oracle's with the bounded build."""
    from rtamd import configs
    for nested in (False, True):
        built = _coincident(3000, nested)
        w, h, b = 97, 61, 4
        cam = configs.Camera((0.0, 0.5, 12.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 30.0, w / h)
        for nl in (1, 8):
            ref, acc = _frames(built, cam, w, h, b, nl)
            _assert_frames_equal(ref, acc, f"coincident nested={nested} layouts {nl}")
            assert ref[2]["mat_reads"] > 0


def test_capacity_fallback(monkeypatch):
    """Past the records' slot cap, 8 layouts fall back to 1 and a scene too
    large for one layout gets no accel records (rt_upload_scene then walks
    the reference's own tree): a scene the reference tree accepts is never
    refused by default (verdict r05, next #4).  Driven here through
    rt_accel_records with a test-only lowered cap (RTAMD_ACCEL_CAP_SLOTS)."""
    from rtamd import configs
    built = configs.config2().build()
    full, info = _records(built, 8)
    slots = info["slots"]
    monkeypatch.setenv("RTAMD_ACCEL_CAP_SLOTS", str(8 * slots + 8))      # exactly fits
    rec, i8 = _records(built, 8)
    assert i8["n_layouts"] == 8 and np.array_equal(rec, full)
    monkeypatch.setenv("RTAMD_ACCEL_CAP_SLOTS", str(8 * slots + 7))      # 8 layouts do not fit: 1
    rec, i1 = _records(built, 8)
    one, ione = _records(built, 1)
    assert i1["n_layouts"] == 1 and i1 == {**ione, "format": 0} and np.array_equal(rec, one)
    monkeypatch.setenv("RTAMD_ACCEL_CAP_SLOTS", str(slots + 7))          # not even one: the reference's tree
    rec, i0 = _records(built, 8)
    assert rec.size == 0 and i0["n_layouts"] == 0 and i0["slots"] == 0


def _adversarial():
    tools = os.path.join(os.path.dirname(HERE), "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    import accel_adversarial
    return accel_adversarial


@pytest.mark.parametrize("name", ["slivers", "fine_mesh", "grazing", "grazing_cube", "far_origin_near",
                                  "far_origin_far", "far_origin_neg", "near_camera"])
def test_adversarial_scenes(name):
    """Geometry built to approach the accel walk's exactness margin (verdict
    r05, next #2; tools/accel_adversarial.py): needle slivers, a fine mesh
    whose hits have |det| near the shader's 1e-5 cut, grazing rays on a
    tilted ground and along the cube's faces, meshes at +-1e4, triangles
    1e-3 from the eye.  Small versions: the model's frame equals the
    oracle's, and the audit finds no segment outside the margin the walk
    applies (thin triangles' boxes carry wider ones: accel_build.h
    accel_relax), with headroom to spare (< 0.25 of it)."""
    A = _adversarial()
    c = A.run_scene(name, 160, 90, 4, scale=0.1, seeds=(1,), layouts=(8,))
    e = c["seeds"]["1"]["layouts8"]
    assert e["rgba_px"] == 0 and e["radiance_px"] == 0, e
    assert e["segments_equal"] and e["mat_reads_equal"]
    a = e["audit"]
    assert a["hits"] > 0 and a["unsafe"] == 0 and a["max_headroom_class"] < 0.25, a


def test_adversarial_study_claims():
    """tests/golden/accel_adversarial.json (the full-size study): every scene,
    seed and layout count bit-exact against the seed-1 oracle, no segment
    outside the margin the walk applies (< 0.25 of it), the fine mesh's
    near-degenerate hits present, and the needles' hits that lie more than
    the default 2^-10 margin before their box (the case the class margins
    exist for) found."""
    with open(os.path.join(HERE, "golden", "accel_adversarial.json")) as f:
        d = json.load(f)
    assert not d["quick"]
    names = {c["scene"] for c in d["cases"]}
    assert names == set(_adversarial().SCENES)
    slivers, worst = 0, 0.0
    for c in d["cases"]:
        for seed, e in c["seeds"].items():
            for k in ("layouts1", "layouts8"):
                a = e[k]
                assert a["rgba_px"] == 0 and a["radiance_px"] == 0, (c["scene"], seed, k)
                assert a["audit"]["unsafe"] == 0 and a["audit"]["max_headroom_class"] < 0.25, (c["scene"], seed, k)
                slivers += a["audit"]["sliver_hits"]
                if c["scene"] == "slivers":
                    worst = max(worst, a["audit"]["max_headroom"])
    assert slivers > 1000
    assert worst > 1.0


@pytest.mark.parametrize("k", [1, 2, 3, 6])
def test_wide_records(k):
    """Option accel_wide's records (accel_build.h format 2): every child box,
    decoded exactly as the kernel decodes it (origin + q 2^e in float),
    holds the child's own box (a leaf's exact box, or the union of the
    grandchildren's decoded boxes' true extents); children are contiguous
    blocks; every primitive is reached exactly once."""
    from rtamd import configs
    built = configs.get(k).build()
    rec, info = _records(built, 8, "wide")
    w = rec.reshape(-1, 16)
    n_rec = info["slots"]
    assert info["n_layouts"] == 1 and w.shape[0] == n_rec + 1
    f32 = lambda x: np.array(x, np.uint32).view(np.float32)   # noqa: E731

    seen = []

    def visit(i, leaf, lo_bound, hi_bound):
        if leaf:
            lo, hi = f32(w[i, [7, 11, 12]]), f32(w[i, 13:16])
            assert (lo >= lo_bound).all() and (hi <= hi_bound).all(), (i, lo, lo_bound, hi, hi_bound)
            seen.append(int(w[i, 0]) & 0x1FFFFFFF)
            assert (int(w[i, 0]) >> 30) & 1
            return
        n = int(w[i, 3]) >> 24 & 7
        assert 2 <= n <= 4
        org = f32(w[i, 0:3])
        assert (org >= lo_bound).all(), (i, org, lo_bound)      # the node's true lo inside its decoded box
        e = [np.int8(np.uint8((int(w[i, 3]) >> (8 * q)) & 0xFF)) for q in range(3)]
        sc = np.array([np.ldexp(np.float32(1.0), int(x)) for x in e], np.float32)
        base = int(w[i, 10]) & 0x07FFFFFF
        for c in range(n):
            ql = np.array([(int(w[i, 4 + q]) >> (8 * c)) & 0xFF for q in range(3)], np.float32)
            qh = np.array([(int(w[i, 7 + q]) >> (8 * c)) & 0xFF for q in range(3)], np.float32)
            lo = (org + ql * sc).astype(np.float32)
            hi = (org + qh * sc).astype(np.float32)
            f = (int(w[i, 11]) >> (8 * c)) & 0xFF
            visit(base + c, bool(f & 1), lo, hi)

    root_leaf = bool(info["root_leaf"])
    visit(0, root_leaf, np.full(3, -np.inf, np.float32), np.full(3, np.inf, np.float32))
    assert len(seen) == info["n_prims"] == len(set(seen))
