"""GPU parity of option accel: the binned-SAH tree walked near
child first through the C ABI, against the reference-order CPU oracle
(oracle/rt_oracle.c).

Bar: bit-exact RGBA8 and float radiance, and the same segments and material
reads as the oracle (every path is the reference's); node visits and
triangle tests equal the accel walk's CPU model (oracle/rt_accel_model.c),
which walks the same records with the same rules and fallback."""
import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def acc():
    if not has_gpu():
        pytest.skip("no GPU")
    import rtamd
    r = rtamd.Renderer((0,))
    yield r
    r.close()


def _oracle(built, cam, w, h, b, **kw):
    from oracle import oracle_lib
    return oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                             cam.ubo_bytes(), w, h, b, **kw)


# A layout spec: 1 or 8 layouts; 108 = 8 layouts in option accel_half's format;
# 208 = option accel_wide's 4-wide tree (one layout).
HALF8 = 108
WIDE = 208


def _model(built, cam, w, h, b, nl, **kw):
    from oracle import oracle_lib
    from rtamd import _lib
    rec, info = _lib.accel_records(built, nl % 100, 100 <= nl < 200, nl >= 200)
    return oracle_lib.render_accel(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                   cam.ubo_bytes(), w, h, b, rec, info, **kw)


def _check(rgba, rad, st, ref, model=None, what=""):
    r_rgba, r_rad, r_c = ref
    bad = (rgba != r_rgba).any(-1) | (rad.view(np.uint32) != r_rad.view(np.uint32)).any(-1)
    assert not bad.any(), f"{what}: {int(bad.sum())} pixels differ from the oracle, first {np.argwhere(bad)[:4].tolist()}"
    if st is not None:
        assert st["segments"] == r_c["segments"] and st["mat_reads"] == r_c["mat_reads"], (what, st, r_c)
        if model is not None:
            m = model[2]
            assert (st["node_visits"], st["tri_tests"]) == (m["node_visits"], m["tri_tests"]), (what, st, m)


def _upload(r, built, nl):
    r.set_option("accel", nl % 100)
    r.set_option("accel_half", 1 if 100 <= nl < 200 else 0)
    r.set_option("accel_wide", 1 if nl >= 200 else 0)
    try:
        r.upload_scene(built)
    finally:
        r.set_option("accel_half", 0)
        r.set_option("accel_wide", 0)
    assert r.get_option("accel_used") == (1 if nl >= 200 else nl % 100)
    assert r.get_option("accel_half_used") == (1 if 100 <= nl < 200 else 0)
    assert r.get_option("accel_wide_used") == (1 if nl >= 200 else 0)


@pytest.mark.parametrize("nl", [1, 8, HALF8, WIDE])
@pytest.mark.parametrize("k,b", [(1, 1), (2, 2), (2, 10), (3, 4), (6, 4)])
def test_accel_full_frame(acc, k, b, nl):
    """Whole frames of configs 1, 2, 3 and 6: frames equal the oracle's, the
    counters the accel model's."""
    from rtamd import configs
    cfg = configs.get(k)
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, nl)
    ref = _oracle(built, cam, cfg.width, cfg.height, b)
    model = _model(built, cam, cfg.width, cfg.height, b, nl)
    for stats in (False, True, False):         # learning, counting, then the production build
        rgba, rad, st = acc.render(cam, cfg.width, cfg.height, b, radiance=True, stats=stats)
        _check(rgba, rad, st, ref, model, f"config {k} b{b} layouts {nl}")


@pytest.mark.parametrize("nl", [1, 8, HALF8, WIDE])
def test_accel_config5_strips(acc, nl):
    """Config 5 (1M triangles, 3840x2160, 8 bounces, all material types):
    three 64-row strips through rt_render_tile_device."""
    import torch
    from rtamd import configs
    cfg = configs.config5()
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, nl)
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    for y0 in (0, 1000, 1800):
        tile = (0, y0, W, 64)
        d_rgba = torch.empty((64, W, 4), dtype=torch.uint8, device="cuda:0")
        d_rad = torch.empty((64, W, 3), dtype=torch.float32, device="cuda:0")
        st = acc.render_tile_device(cam, W, H, B, *tile, d_rgba.data_ptr(), d_rad.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream, stats=True)
        torch.cuda.synchronize()
        ref = _oracle(built, cam, W, H, B, tile=tile)
        model = _model(built, cam, W, H, B, nl, tile=tile)
        _check(d_rgba.cpu().numpy(), d_rad.cpu().numpy(), st, ref, model, f"config 5 rows {y0}+64")


def _tie_scenes():
    import test_accel_model as M
    return M._tie_scenes()


@pytest.mark.parametrize("band", [2, 1000])
def test_accel_xcd_order(acc, band):
    """Option xcd_order (rt_learn.hip xcd_keys / xcd_place): the device-learned
    order regrouped so that XCD c's workgroups take one class of row bands;
    every tile still traced once, so frames and counters are unchanged
    (config 3, 120 x 270 wave tiles, a multiple of 8)."""
    from rtamd import configs
    cfg = configs.config3()
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, 8)
    ref = _oracle(built, cam, cfg.width, cfg.height, 4)
    model = _model(built, cam, cfg.width, cfg.height, 4, 8)
    acc.set_option("xcd_order", band)
    try:
        assert acc.get_option("xcd_order") == band
        for stats in (False, False, True, False):    # learning, then launches in the regrouped order
            rgba, rad, st = acc.render(cam, cfg.width, cfg.height, 4, radiance=True, stats=stats)
            _check(rgba, rad, st, ref, model, f"xcd_order {band}")
    finally:
        acc.set_option("xcd_order", 0)


@pytest.mark.parametrize("mask", [5, 0])
def test_accel_octants(acc, mask):
    """Option accel_octants: rays walk layout (octant & mask) of the 8 (fewer
    layouts touched, a worse child order on the dropped axes); frames equal
    the oracle's, counters the model's with the same mask
    (orc_accel_octants)."""
    from oracle import oracle_lib
    from rtamd import configs
    cfg = configs.config3()
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, 8)
    ref = _oracle(built, cam, cfg.width, cfg.height, 4)
    L = oracle_lib.lib(accel=True)
    L.orc_accel_octants(mask)
    try:
        model = _model(built, cam, cfg.width, cfg.height, 4, 8)
    finally:
        L.orc_accel_octants(7)
    acc.set_option("accel_octants", mask)
    try:
        assert acc.get_option("accel_octants") == mask
        for stats in (False, True, False):
            rgba, rad, st = acc.render(cam, cfg.width, cfg.height, 4, radiance=True, stats=stats)
            _check(rgba, rad, st, ref, model, f"accel_octants {mask}")
    finally:
        acc.set_option("accel_octants", 7)


@pytest.mark.parametrize("nl", [1, 8])
def test_accel_random_scenes(acc, nl):
    """Random triangle soups (sizes, offsets, needles, tiny triangles), 24
    scenes: frames equal the oracle's, counters the accel model's."""
    import test_accel_model as M
    from rtamd import build_buffers, configs
    for seed in range(24):
        verts, mats, (eye, at), vfov = M.random_scene(seed)
        w, h, b = 64, 48, 3
        cam = configs.Camera(eye, at, (0.0, 1.0, 0.0), vfov, w / h)
        built = build_buffers(verts, mats, 1 + seed % 3)
        _upload(acc, built, nl)
        ref = _oracle(built, cam, w, h, b)
        model = _model(built, cam, w, h, b, nl)
        rgba, rad, st = acc.render(cam, w, h, b, radiance=True, stats=True)
        _check(rgba, rad, st, ref, model, f"random scene {seed} layouts {nl}")


def _adversarial():
    import os
    import sys
    tools = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    import accel_adversarial
    return accel_adversarial


@pytest.mark.parametrize("nl", [1, 8, HALF8, WIDE])
@pytest.mark.parametrize("name", ["slivers", "fine_mesh", "grazing", "grazing_cube", "far_origin_near",
                                  "far_origin_far", "far_origin_neg", "near_camera"])
def test_accel_adversarial_scenes(acc, name, nl):
    """The adversarial scenes of the margin audit (tools/accel_adversarial.py,
    DESIGN.md §4a) on the GPU: needles whose rounded t lies up to 17 margins
    before their box (the forced records of accel_build.h kAccelForce), a fine
    shell with |det| near the shader's 1e-5 cut, grazing rays, meshes at
    +-1e4, triangles 1e-3 from the eye.  Small versions (scale 0.3, 240 x 135,
    4 bounces): frames equal the oracle's, counters the accel model's."""
    from rtamd import build_buffers, configs
    A = _adversarial()
    verts, mats, (eye, at), vfov = A.SCENES[name](0.3)
    w, h, b = 240, 135, 4
    cam = configs.Camera(eye, at, (0.0, 1.0, 0.0), vfov, w / h)
    built = build_buffers(verts, mats, 1)
    _upload(acc, built, nl)
    ref = _oracle(built, cam, w, h, b)
    model = _model(built, cam, w, h, b, nl)
    for stats in (False, True, False):
        rgba, rad, st = acc.render(cam, w, h, b, radiance=True, stats=stats)
        _check(rgba, rad, st, ref, model, f"{name} layouts {nl}")


@pytest.mark.parametrize("nl", [1, 8, HALF8, WIDE])
def test_accel_ties_and_fallback(acc, nl):
    """Scenes built to tie: every triangle twice in two colours, an integer
    grid of coplanar and coincident faces, the cube's faces split both ways.
    Hits on a face whose box starts at the face (rounding puts t before the
    box's t_enter) take the fallback to the reference's order."""
    from rtamd import configs
    for name, built in _tie_scenes().items():
        _upload(acc, built, nl)
        for (w, h, b) in [(160, 90, 3), (97, 61, 10)]:
            cam = configs.Camera.default(w, h)
            ref = _oracle(built, cam, w, h, b)
            model = _model(built, cam, w, h, b, nl)
            rgba, rad, st = acc.render(cam, w, h, b, radiance=True, stats=True)
            _check(rgba, rad, st, ref, model, f"{name} {w}x{h}x{b}")


@pytest.mark.parametrize("opts", [{"coop_lanes": 0}, {"coop_lanes": 8}, {"heavy_first": 0},
                                  {"wave_tile": 1}, {"wave_tile": 3}, {"coop_window": 32},
                                  {"block_waves": 4}])
def test_accel_schedules(acc, opts):
    """Schedule options change which wave traces a pixel and when, never what
    it computes."""
    from rtamd import configs
    cfg = configs.config3()
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, 1)
    ref = _oracle(built, cam, cfg.width, cfg.height, cfg.max_bounces, row_step=8)
    old = {k: acc.get_option(k) for k in opts}
    try:
        for k, v in opts.items():
            acc.set_option(k, v)
        for _ in range(2):                         # a learning launch, then the learned order
            rgba, rad, _ = acc.render(cam, cfg.width, cfg.height, cfg.max_bounces, radiance=True)
            _check(rgba[::8], rad[::8], None, ref, None, str(opts))
    finally:
        for k, v in old.items():
            acc.set_option(k, v)


def test_accel_empty_and_tiny_scenes(acc):
    from rtamd import build_buffers, configs, triangles_of
    verts, mats = triangles_of(configs.config2().scene)
    for n in (0, 1, 2, 3):
        built = build_buffers(verts[:n], mats[:n])
        for nl in (1, 8, HALF8, WIDE):
            _upload(acc, built, nl)
            for (w, h, b) in [(37, 23, 3), (1, 1, 1)]:
                cam = configs.Camera.default(w, h)
                ref = _oracle(built, cam, w, h, b)
                rgba, rad, st = acc.render(cam, w, h, b, radiance=True, stats=True)
                _check(rgba, rad, st, ref, _model(built, cam, w, h, b, nl), f"{n} triangles")


@pytest.mark.parametrize("nl", [1, HALF8, WIDE])
def test_accel_extensions(acc, nl):
    """The non-reference extensions run over the accel walk too (sky toggle,
    emissive, spheres); frames equal the oracle's extension build."""
    from oracle import oracle_lib
    from rtamd import configs
    cfg = configs.config3()
    built = cfg.build()
    _upload(acc, built, nl)
    w, h, b = 320, 180, 4
    cam = configs.Camera.default(w, h)
    spheres = np.array([[0.0, 5.0, 20.0, 6.0, 0.9, 0.9, 0.9, 1.0],
                        [-15.0, 2.0, 0.0, 4.0, 5.0, 5.0, 5.0, 3.0]], np.float32)
    acc.upload_spheres(spheres)
    ext = oracle_lib.EXT_SKY_TOGGLE | oracle_lib.EXT_EMISSIVE | oracle_lib.EXT_SPHERES
    try:
        acc.set_option("extensions", ext)
        rgba, rad, _ = acc.render(cam, w, h, b, radiance=True)
        ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                cam.ubo_bytes(), w, h, b, ext=ext, spheres=spheres)
        _check(rgba, rad, None, ref, None, "extensions")
    finally:
        acc.set_option("extensions", 0)
        acc.upload_spheres(np.zeros((0, 8), np.float32))


@pytest.mark.parametrize("nl", [8, HALF8, WIDE])
@pytest.mark.parametrize("cfg_k", [3, 4, 5, 6])
def test_accel_bench_setting_whole_frame(acc, cfg_k, nl):
    """BASELINE configs 3, 4, 5 (1M triangles, 3840x2160, 8 bounces) and 6 as
    whole frames under bench.py's N = 1 setting with the default options
    (accel 8, 4 launches in flight counted): the learning launch, the
    production kernel in the learned order, then a counting launch.  Frames
    equal the oracle's; the counters equal the accel model's."""
    from rtamd import configs
    from test_gpu_parity import _bands_device
    cfg = configs.get(cfg_k)
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, nl)
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    ref = _oracle(built, cam, W, H, B)
    model = _model(built, cam, W, H, B, nl)
    try:
        acc.set_option("concurrent_launches", 4)
        for stats in (False, False, True):
            rgba, rad, st = _bands_device(acc, cam, W, H, B, H, 1, 0, stats=stats)
            _check(rgba, rad, st if stats else None, ref, model, f"config {cfg_k} whole frame")
        assert st["pixels"] == W * H
    finally:
        acc.set_option("concurrent_launches", 1)


def test_accel_is_the_default():
    """A context that is not told otherwise walks the accel tree in 8 octant
    layouts; RTAMD_ACCEL only overrides it (the legacy suites
    pin 0, conftest.py)."""
    import os
    import rtamd
    from rtamd import configs
    old = os.environ.pop("RTAMD_ACCEL", None)
    try:
        with rtamd.Renderer((0,)) as r:
            assert r.get_option("accel") == 8 and r.get_option("coop_lanes") == -1
            r.upload_scene(configs.config2().build())
            assert r.get_option("accel_used") == 8
    finally:
        if old is not None:
            os.environ["RTAMD_ACCEL"] = old


@pytest.mark.parametrize("split", [1, 2, 3])
@pytest.mark.parametrize("k,b", [(2, 10), (3, 4), (6, 4)])
def test_accel_split_launch(acc, k, b, split):
    """Option split_bounce: kernel 1 to bounce split, each
    wave's surviving paths packed into its ray slots, a scan, kernel 2 for the
    rest, 64 paths per wave in slot order.  Same frames (RGBA8 and radiance)
    as the oracle, in the learned order and on 4 streams."""
    from rtamd import configs
    from test_gpu_parity import _bands_device
    cfg = configs.get(k)
    built = cfg.build()
    cam = cfg.camera()
    _upload(acc, built, 8)
    W, H = cfg.width, cfg.height
    ref = _oracle(built, cam, W, H, b)
    old = acc.get_option("split_bounce")
    try:
        acc.set_option("split_bounce", split)
        acc.set_option("concurrent_launches", 4)
        for _ in range(3):                         # the learning launch, then the learned order
            rgba, rad, _ = _bands_device(acc, cam, W, H, b, H, 1, 0, stats=False)
            _check(rgba, rad, None, ref, None, f"config {k} b{b} split {split}")
        rgba, rad, _ = acc.render(cam, W, H, b, radiance=True)
        _check(rgba, rad, None, ref, None, f"config {k} b{b} split {split} (rt_render)")
    finally:
        acc.set_option("split_bounce", old)
        acc.set_option("concurrent_launches", 1)

