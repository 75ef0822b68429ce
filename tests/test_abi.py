"""The C ABI library (no GPU needed): it loads, exports every symbol
include/rtamd.h declares, validates scenes and reports errors."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import has_gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtamd.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", src))


def test_library_exports_every_header_symbol():
    from rtamd import LIB_PATH, lib
    lib()
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rt_[a-z_0-9]+)$", out, flags=re.M))
    syms = header_symbols()
    assert len(syms) >= 20
    assert syms <= exported, syms - exported
    from rtamd._lib import EXPORTED
    assert set(EXPORTED) == syms


def test_library_is_gfx950_code_object():
    from rtamd import LIB_PATH
    data = open(LIB_PATH, "rb").read()
    assert b"gfx950" in data and b"trace_simple" in data
    assert b"trace_persistent" not in data and b"trace_coop" not in data   # archived in round 3


def test_structs_match_reference_bytes():
    from rtamd import CameraUBO, Stats
    assert C.sizeof(CameraUBO) == 80              # VulkanEngine.java createCameraUbo: 80 bytes
    assert CameraUBO.vertical.offset == 48 and CameraUBO.frame_count.offset == 64
    assert CameraUBO.sky_enabled.offset == 68
    # {segments, node_visits, tri_tests, mat_reads; double ms}, then pixels
    assert [f for f, _ in Stats._fields_] == ["segments", "node_visits", "tri_tests", "mat_reads", "ms", "pixels"]
    assert Stats.ms.offset == 32 and Stats.pixels.offset == 40 and C.sizeof(Stats) == 48


@pytest.mark.skipif(has_gpu(), reason="only meaningful without a GPU")
def test_no_cpu_fallback():
    from rtamd import Renderer, RtError
    with pytest.raises(RtError, match="NO_DEVICE|HIP"):
        Renderer((0,))
    with pytest.raises(RtError, match="INVALID_ARG"):
        Renderer(())


def _validate(v, m, n):
    from rtamd import lib
    from rtamd._lib import check
    nn, d = C.c_size_t(), C.c_int()
    v, m, n = (np.ascontiguousarray(x) for x in (v, m, n))
    check(lib().rt_scene_validate(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data, n.nbytes,
                                  C.byref(nn), C.byref(d)))
    return nn.value, d.value


def test_scene_validation():
    from rtamd import RtError, configs
    b = configs.config2().build()
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    assert _validate(v, m, n) == (31, 4)
    # the reference's empty-scene dummies (SceneBuilder.java:61-70) are an empty scene
    assert _validate(np.zeros(1, np.float32), np.zeros(1, np.float32), np.zeros(1, np.uint8))[0] == 0
    bad = n.copy().view(np.int32).reshape(-1, 12)
    bad[0, 8] = 3                                  # left child must be i+1
    with pytest.raises(RtError, match="BAD_SCENE.*preorder"):
        _validate(v, m, bad)
    bad = n.copy().view(np.int32).reshape(-1, 12)
    leaf = np.nonzero(bad[:, 9] < 0)[0][0]
    bad[leaf, 8] = -(1000 + 1)                     # triangle 1000 does not exist
    with pytest.raises(RtError, match="BAD_SCENE.*triangle 1000"):
        _validate(v, m, bad)
    with pytest.raises(RtError, match="BAD_SCENE.*material|BAD_SCENE.*outside"):
        _validate(v, m[:4], n)                     # materials shorter than the triangles used
    with pytest.raises(RtError, match="multiple of 48"):
        _validate(v, m, n[:-8])


def test_band_rows():
    from rtamd import lib
    from rtamd.dist import band_rows
    for h in (1, 7, 16, 720, 1080, 2160):
        for bh in (1, 16, 64):
            for world in (1, 2, 3, 4, 8):
                rows = [lib().rt_band_rows(h, bh, world, r) for r in range(world)]
                assert sum(rows) == h
                for r in range(world):
                    assert len(band_rows(h, bh, world, r)) == rows[r]
    assert lib().rt_band_rows(10, 0, 1, 0) == -1
    assert lib().rt_band_rows(10, 4, 2, 2) == -1


def test_error_message_is_thread_local():
    import threading
    from rtamd import lib
    L = lib()
    L.rt_set_option(None, b"kernel", 0)
    msg = L.rt_last_error()
    seen = []
    t = threading.Thread(target=lambda: seen.append(L.rt_last_error()))
    t.start()
    t.join()
    assert b"null" in msg and seen == [b""]


def test_unbalanced_bvh_validates():
    """Left-/right-deep chains and random splits are valid preorder uploads."""
    from raw_bvh import raw_bvh_scene
    for shape, n, depth in (("left", 50, 49), ("right", 200, 199), ("random", 300, None)):
        b = raw_bvh_scene(n, shape, seed=n)
        nn, md = _validate(b.model_vertex_data, b.model_material_data, b.flat_bvh_data)
        assert nn == 2 * n - 1
        if depth is not None:
            assert md == depth


def test_band_list_rows_and_weighted_deal():
    """rt_band_list_rows (the C ABI's row count of a band list) against the
    Python deal (rtamd.dist.band_owners): every band has exactly one owner,
    the counts follow the weights, weight 1 is the plain interleave."""
    import ctypes as C
    from rtamd import lib
    from rtamd.dist import SharePlan, band_owners, list_rows
    L = lib()

    def rows(h, bh, bands):
        arr = (C.c_int32 * max(1, len(bands)))(*bands)
        return L.rt_band_list_rows(h, bh, arr, len(bands))
    for h, bh, world, rw in [(1080, 8, 8, 0.7), (1080, 16, 8, 0.6), (2160, 8, 4, 0.85), (53, 4, 3, 0.5),
                             (720, 8, 2, 1.0), (7, 8, 4, 1.0)]:
        own = band_owners(h, bh, world, rw)
        assert len(own) == (h + bh - 1) // bh
        total = 0
        for r in range(world):
            b = np.flatnonzero(own == r).astype(np.int32)
            n = rows(h, bh, list(b))
            assert n == len(list_rows(h, bh, b))
            total += n
        assert total == h
        if rw == 1.0:
            assert (own == np.arange(len(own)) % world).all()
        else:
            c = np.bincount(own, minlength=world)
            assert c[0] <= c[1:].min() and abs(c[0] / c[1:].mean() - rw) < 0.2
        plan = SharePlan(h, bh, world, 2, rw)
        assert sorted(plan.src.tolist()) == sorted(set(plan.src.tolist()))     # every row from one place
    assert rows(10, 4, [1, 0]) == -1          # not increasing
    assert rows(10, 4, [3]) == -1             # past the frame

    def lrows(h, bh, lists):
        flat = [b for lst in lists for b in lst]
        arr = (C.c_int32 * len(flat))(*flat)
        return L.rt_band_lists_rows(h, bh, arr, len(lists), len(lists[0]))
    # rt_band_lists_rows: per-frame lists, -1 padding at the end only, band_h | height
    assert lrows(48, 4, [[0, 1, 2], [3, 4, -1]]) == 12
    assert lrows(48, 4, [[0, -1, 2]]) == -1
    assert lrows(48, 4, [[2, 1, -1]]) == -1
    assert lrows(48, 4, [[12, -1]]) == -1     # past the frame
    assert lrows(50, 4, [[0, 1]]) == -1       # band_h must divide the height
    for world in (2, 3, 8):
        plan = SharePlan(1080, 8, world, world, layout="pieces")
        lists = plan.launch_lists(1, 0, world)
        assert lrows(1080, 8, lists.tolist()) == plan.max_rows == plan.n_per * 8
        assert sorted(int(b) for b in lists.reshape(-1) if b >= 0) == list(range(135))   # every band once
    assert rows(10, 4, []) == 0
    assert rows(10, 4, [2]) == 2              # the partial last band


def test_jni_shim_matches_java_and_header():
    """jni/: every native method HipNative.java declares has its
    Java_dev_demir_vulkan_engine_HipNative_* function in HipNative.c and back,
    and every rt_* call in the shim is declared in include/rtamd.h (the shim
    cannot be compiled here: no JDK / jni.h)."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c_src = open(os.path.join(root, "jni", "HipNative.c")).read()
    j_src = open(os.path.join(root, "jni", "dev", "demir", "vulkan", "engine", "HipNative.java")).read()
    hdr = open(os.path.join(root, "include", "rtamd.h")).read()
    natives = set(re.findall(r"static native \w+ (\w+)\(", j_src))
    jni_fns = set(re.findall(r"Java_dev_demir_vulkan_engine_HipNative_(\w+)\(", c_src))
    assert natives and natives == jni_fns
    calls = set(re.findall(r"\b(rt_\w+)\(", c_src))
    declared = set(re.findall(r"\b(rt_\w+)\(", hdr))
    assert calls <= declared, calls - declared


def test_every_option_is_documented():
    """Every option name rt_set_option / rt_get_option accepts
    (csrc/rt_runtime.hip) is documented in include/rtamd.h."""
    import re
    src = open(os.path.join(ROOT, "3d-ray-tracer-vulkan_amd", "csrc", "rt_runtime.hip")).read()
    hdr = open(os.path.join(ROOT, "include", "rtamd.h")).read()
    names = set(re.findall(r'std::strcmp\(name, "([a-z0-9_]+)"\)', src))
    assert len(names) > 20
    missing = sorted(n for n in names if f'"{n}"' not in hdr)
    assert not missing, missing
