"""GPU: the frames a pipelined caller gets (bench.py's timed loop, HipEngine's
frames in flight) and the runtime's synchronisation around them.

* bench.py's N = 1 trace() shape: rt_render_batch_device, one or two whole
  frames (the N = 1 default) and no band list per launch, 4 launches at once
  on 4 streams (ShareTracer, the class bench.py launches through), config 3:
  every frame equals the oracle's.
* A scene swap between rt_render_async submits, as HipEngine.java does with
  4 frames in flight (VulkanEngine.internalSwapScene drains the device first,
  VulkanEngine.java:321): every frame equals the oracle frame of the scene it
  was submitted with.
* rt_render_wait on a split readback (copy_streams 2) waits for its own frame,
  not for the newest frame in flight (rt_render_poll says the newer one is
  still running).
"""
import ctypes as C

import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu


def _oracle(built, cam_bytes, w, h, b, **kw):
    from oracle import oracle_lib
    return oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                             cam_bytes, w, h, b, **kw)


def _orbit(cfg, k):
    import math
    from rtamd import configs
    ox, oy, oz = -25.0, 30.0, 140.0
    rad, a0 = math.hypot(ox, oz), math.atan2(oz, ox)
    a = a0 + math.radians(0.5) * k
    return configs.Camera((rad * math.cos(a), oy, rad * math.sin(a)), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0,
                          cfg.width / cfg.height)


@pytest.mark.parametrize("accel,F", [(0, 1), (8, 1), (8, 2)])
@pytest.mark.parametrize("camera", ["static", "orbit"])
def test_bench_trace_shape_frames(renderer, camera, accel, F):
    """Config 3 through bench.py's N = 1 launches: D = 4 launches in flight on
    4 streams (concurrent_launches 4), each F whole frames into its slot
    (F = 2: bench.default_batch at N = 1), three rounds (the learning launch,
    then the learned order with heavy pixels).  Every frame of every round
    equals the oracle's."""
    import torch
    from rtamd import configs
    from rtamd._lib import CameraUBO
    from rtamd.dist import ShareTracer
    cfg = configs.get(3)
    built = cfg.build()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    D = 4
    try:
        renderer.set_option("accel", accel)       # accel 8: the default walk
        renderer.upload_scene(built)
        renderer.set_option("concurrent_launches", D)
        cams = [cfg.camera() if camera == "static" else _orbit(cfg, k) for k in range(D * F)]
        refs = {}
        for k in range(D * F if camera == "orbit" else 1):
            refs[k] = _oracle(built, cams[k].ubo_bytes(), W, H, B, radiance=False)[0]
        tracer = ShareTracer(renderer._ctx, W, H, B, "whole")
        slots = torch.zeros((D, F * H, W, 4), dtype=torch.uint8, device="cuda:0")
        streams = [torch.cuda.Stream() for _ in range(D)]
        ubos = [(CameraUBO * F)(*[c.ubo for c in cams[j * F:(j + 1) * F]]) for j in range(D)]
        for rnd in range(3):
            torch.cuda.synchronize()
            slots.zero_()
            torch.cuda.synchronize()
            for j in range(D):
                tracer.launch(ubos[j], j * F, F, streams[j].cuda_stream, slots[j].data_ptr(), None)
            torch.cuda.synchronize()
            got = slots.cpu().numpy()
            for j in range(D):
                for f in range(F):
                    ref = refs[j * F + f if camera == "orbit" else 0]
                    fr = got[j][f * H:(f + 1) * H]
                    if not np.array_equal(fr, ref):
                        n = int(np.any(fr != ref, axis=-1).sum())
                        raise AssertionError(f"round {rnd}, stream {j}, frame {f}: {n} pixels differ")
        assert renderer.get_option("heavy_pixels_used") > 0 or camera == "orbit" or accel
    finally:
        renderer.set_option("concurrent_launches", 1)
        renderer.set_option("accel", 0)


@pytest.mark.parametrize("accel", [0, 8])
def test_scene_swap_with_frames_in_flight(accel):
    """HipEngine.java's loop: 4 frames in flight through rt_render_async and a
    scene upload between two submits (the old scene's frames still tracing);
    then frames of the new scene.  Every frame equals the oracle frame of the
    scene it was submitted with."""
    if not has_gpu():
        pytest.skip("no GPU")
    import rtamd
    from rtamd import configs
    from rtamd.engine import PinnedFrame
    w, h, b = 480, 272, 4
    scenes = [configs.get(3).build(), configs.config2().build(), configs.get(3).build()]
    cam = configs.Camera.default(w, h)
    refs = [_oracle(s, cam.ubo_bytes(), w, h, b, radiance=False)[0] for s in scenes]
    S = 4
    r = rtamd.Renderer((0,))
    frames = [PinnedFrame(h, w) for _ in range(S)]
    try:
        r.set_option("async_slots", S)
        r.set_option("accel", accel)
        order = [0] * 6 + [1] * 6 + [2] * 6          # a swap after every 6 submits
        pending = []
        cur = None
        for k, sc in enumerate(order):
            if sc != cur:
                r.upload_scene(scenes[sc])            # frames of the previous scene are in flight here
                cur = sc
            if len(pending) == S:
                t, j, s0 = pending.pop(0)
                r.wait(t)
                assert np.array_equal(frames[j % S].array, refs[s0]), f"frame {j} (scene {s0})"
            pending.append((r.render_async(cam, w, h, b, frames[k % S]), k, sc))
        while pending:
            t, j, s0 = pending.pop(0)
            r.wait(t)
            assert np.array_equal(frames[j % S].array, refs[s0]), f"frame {j} (scene {s0})"
    finally:
        r.close()
        for f in frames:
            f.close()


def test_split_wait_covers_only_its_frame():
    """copy_streams 2 (every one-device frame splits its readback): a wait on
    an older frame returns once that frame is read back, while a newer, much
    longer frame is still tracing (rt_render_poll: not done); the newer frame's
    own wait then completes it.  Both frames equal rt_render's."""
    if not has_gpu():
        pytest.skip("no GPU")
    import time
    import rtamd
    from rtamd import configs
    from rtamd.engine import PinnedFrame
    cfg = configs.get(3)
    built = cfg.build()
    small = (64, 48, 2)
    big = (3840, 2160, 10)                        # tens of ms per frame alone
    cam_s = configs.Camera.default(small[0], small[1])
    cam_b = configs.Camera.default(big[0], big[1])
    r = rtamd.Renderer((0,))
    fs = PinnedFrame(small[1], small[0])
    fb = PinnedFrame(big[1], big[0])
    try:
        r.upload_scene(built)
        r.set_option("copy_streams", 2)
        ref_s = r.render(cam_s, *small)[0]
        ref_b = r.render(cam_b, *big)[0]
        # warm both launch keys (learning launches synchronise) and the ring size
        for _ in range(2):
            r.wait(r.render_async(cam_b, *big, fb))
            r.wait(r.render_async(cam_s, *small, fs))
        ts = r.render_async(cam_s, *small, fs)
        tb = r.render_async(cam_b, *big, fb)
        r.wait(ts)
        still_running = not r.poll(tb)
        assert np.array_equal(fs.array, ref_s)
        t0 = time.time()
        while not r.poll(tb):
            assert time.time() - t0 < 60
            time.sleep(0.001)
        r.wait(tb)
        assert np.array_equal(fb.array, ref_b)
        assert r.poll(ts) and r.poll(tb)
        assert still_running, "waiting on the older split frame waited for the newest frame too"
        with pytest.raises(rtamd.RtError, match="INVALID_ARG"):
            r.poll(tb + 1)
    finally:
        r.close()
        fs.close()
        fb.close()


def test_async_poll_then_wait_matches_sync(renderer):
    """rt_render_poll never blocks and turns true for every ticket; the
    frames it reports done equal rt_render's."""
    import time
    import rtamd
    from rtamd import configs
    from rtamd.engine import PinnedFrame
    cfg = configs.config2()
    built = cfg.build()
    w, h, b = 320, 180, 3
    cams = [rtamd.Camera((-25.0 + 5 * k, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, w / h)
            for k in range(6)]
    renderer.upload_scene(built)
    refs = [renderer.render(c, w, h, b)[0] for c in cams]
    frames = [PinnedFrame(h, w) for _ in cams]
    try:
        tickets = [renderer.render_async(c, w, h, b, f) for c, f in zip(cams, frames)]
        for t, f, ref in zip(tickets, frames, refs):
            t0 = time.time()
            while not renderer.poll(t):
                assert time.time() - t0 < 60
                time.sleep(0.0005)
            assert np.array_equal(f.array, ref)
    finally:
        renderer.wait(tickets[-1])
        for f in frames:
            f.close()


def test_stats_struct_order(renderer):
    """rt_stats is SURVEY.md §8(b)'s {segments, node_visits, tri_tests,
    mat_reads, ms} followed by pixels."""
    from rtamd import configs
    from rtamd._lib import Stats
    assert [f for f, _ in Stats._fields_] == ["segments", "node_visits", "tri_tests", "mat_reads", "ms", "pixels"]
    assert C.sizeof(Stats) == 48
    cfg = configs.config2()
    renderer.upload_scene(cfg.build())
    _, _, st = renderer.render(configs.Camera.default(64, 36), 64, 36, 2, stats=True)
    assert st["pixels"] == 64 * 36 and st["segments"] >= 64 * 36 and st["ms"] > 0


@pytest.mark.parametrize("cfg_k", [3, 6])
def test_device_learning_matches_host_learning(renderer, cfg_k):
    """The order learned on the device (rt_learn.hip) picks the heavy pixels the
    host path picks from the same kind of learning launch (learn_cost 0: the
    lockstep steps, a deterministic cost), and every frame stays the oracle's."""
    from rtamd import configs
    cfg = configs.get(cfg_k)
    built = cfg.build()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    cam = configs.Camera((-25.0, 30.0, 141.5), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H)
    ref = _oracle(built, cam.ubo_bytes(), W, H, B, row_step=9, radiance=False)[0]
    used = {}
    try:
        renderer.set_option("learn_cost", 0)
        for dev in (1, 0):
            renderer.set_option("learn_device", dev)
            renderer.upload_scene(built)                 # a new scene generation: nothing learned yet
            for launch in range(3):                      # the learning launch, then the learned order
                rgba = renderer.render(cam, W, H, B)[0]
                assert np.array_equal(rgba[::9], ref), (dev, launch)
            used[dev] = renderer.get_option("heavy_pixels_used")
    finally:
        renderer.set_option("learn_cost", 1)
        renderer.set_option("learn_device", 1)
    assert used[1] > 0 and used[1] == used[0], used


@pytest.mark.parametrize("align", [0, 1])
@pytest.mark.parametrize("cfg_k", [3, 6, 2])
def test_leaf_align_bit_exact(renderer, cfg_k, align):
    """Option leaf_align both ways (1: walk records with a pad slot before any
    leaf that would straddle a 128-B line, the predecessor's pad bit stepping
    over it, run by the kFeatPad kernels; 0: packed): frames and counters equal
    the oracle's, in the lockstep walk, the cooperative windows (coop_lanes 64:
    every walk) and the learned order."""
    from rtamd import configs
    cfg = configs.get(cfg_k)
    built = cfg.build()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    cam = cfg.camera()
    ref = _oracle(built, cam.ubo_bytes(), W, H, B, row_step=7)
    try:
        renderer.set_option("leaf_align", align)
        renderer.upload_scene(built)
        assert renderer.get_option("leaf_align_used") == align
        for coop in (1, 64):
            renderer.set_option("coop_lanes", coop)
            for launch in range(2):
                rgba, rad, st = renderer.render(cam, W, H, B, radiance=True, stats=launch == 1)
                assert np.array_equal(rgba[::7], ref[0]), (coop, launch)
                assert np.array_equal(rad[::7].view(np.uint32), ref[1].view(np.uint32)), (coop, launch)
        full = _oracle(built, cam.ubo_bytes(), W, H, B, radiance=False)[2]
        for k in ("segments", "node_visits", "tri_tests", "mat_reads"):
            assert st[k] == full[k], k
    finally:
        renderer.set_option("leaf_align", 2)
        renderer.set_option("coop_lanes", 1)
        renderer.upload_scene(built)


@pytest.mark.parametrize("win", [32, 64])
@pytest.mark.parametrize("cfg_k", [3, 6])
def test_coop_window_bit_exact(renderer, cfg_k, win):
    """Option coop_window (the cooperative tail's window: 32 or 64 slots):
    frames and counters equal the oracle's, in the learned order with heavy
    pixels and with every walk cooperative (coop_lanes 64)."""
    from rtamd import configs
    cfg = configs.get(cfg_k)
    built = cfg.build()
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    cam = cfg.camera()
    ref = _oracle(built, cam.ubo_bytes(), W, H, B, row_step=11)
    try:
        renderer.upload_scene(built)
        assert renderer.get_option("coop_window_used") == 64    # L2-sized scenes: 64-slot windows
        assert renderer.get_option("leaf_align_used") == 0      # and packed records
        renderer.set_option("coop_window", win)
        assert renderer.get_option("coop_window") == win
        for coop in (1, 64):
            renderer.set_option("coop_lanes", coop)
            for launch in range(3):
                rgba, rad, st = renderer.render(cam, W, H, B, radiance=True, stats=launch == 2)
                assert np.array_equal(rgba[::11], ref[0]), (coop, launch)
                assert np.array_equal(rad[::11].view(np.uint32), ref[1].view(np.uint32)), (coop, launch)
        full = _oracle(built, cam.ubo_bytes(), W, H, B, radiance=False)[2]
        for k in ("segments", "node_visits", "tri_tests", "mat_reads"):
            assert st[k] == full[k], k
    finally:
        renderer.set_option("coop_window", 0)
        renderer.set_option("coop_lanes", 1)
