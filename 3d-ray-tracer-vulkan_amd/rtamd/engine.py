"""Render side of the host API.

Renderer   — a synchronous wrapper of one rt_ctx (the C ABI).
HipEngine  — a mirror of the reference's VulkanEngine public API
             (src/dev/demir/vulkan/engine/VulkanEngine.java:120-185): a render
             thread fed through queues that are drained to their latest value
             (handleCommands :277-313), rendering frames as long as a scene and
             a camera are present (mainLoop :244-271) and publishing each one to
             an AtomicReference-like slot (:264).
FrameData  — FrameData.java:9-16 (+ the render statistics its TODO asks for).
"""
from __future__ import annotations

import ctypes as C
import queue
import threading
import time
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple, Union

import numpy as np

from ._lib import CameraUBO, RtError, Stats, check, lib
from .scene import BuiltCpuData, Camera

REFERENCE_WIDTH = 1280          # VulkanEngine.java:45
REFERENCE_HEIGHT = 720          # VulkanEngine.java:46
REFERENCE_MAX_BOUNCES = 10      # compute_dynamic_ray.comp:44


def _ubo(cam: Union[Camera, CameraUBO, bytes]) -> CameraUBO:
    if isinstance(cam, Camera):
        return cam.ubo
    if isinstance(cam, CameraUBO):
        return cam
    if isinstance(cam, (bytes, bytearray)) and len(cam) == 80:
        return CameraUBO.from_buffer_copy(cam)
    raise TypeError("camera must be a Camera, a CameraUBO or 80 UBO bytes")


class Renderer:
    """One context on one or more HIP devices (rt_create / rt_destroy)."""

    def __init__(self, device_ids: Sequence[int] = (0,)):
        ids = (C.c_int * len(device_ids))(*device_ids)
        self._ctx = C.c_void_p()
        check(lib().rt_create(ids, len(device_ids), C.byref(self._ctx)))
        self.device_ids = tuple(device_ids)

    def close(self) -> None:
        if self._ctx:
            lib().rt_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, name: str, value: int) -> None:
        """Schedule options (rt_set_option; the list is in include/rtamd.h):
        "walk", "coop_lanes", "heavy_first", "concurrent_launches", ...
        Results do not depend on them."""
        check(lib().rt_set_option(self._ctx, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        check(lib().rt_get_option(self._ctx, name.encode(), C.byref(v)))
        return v.value

    def walk_bytes(self) -> int:
        """Bytes of the records one ray walks (option walk_bytes)."""
        return self.get_option("walk_bytes")

    def upload_scene(self, data: BuiltCpuData) -> None:
        """internalSwapScene (VulkanEngine.java:318-373); deep copy."""
        v = np.ascontiguousarray(data.model_vertex_data, dtype=np.float32)
        m = np.ascontiguousarray(data.model_material_data, dtype=np.float32)
        b = np.ascontiguousarray(data.flat_bvh_data, dtype=np.uint8)
        check(lib().rt_upload_scene(self._ctx, v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes,
                                    b.ctypes.data, b.nbytes))

    def upload_spheres(self, spheres) -> None:
        """Extension (option "extensions" bit 8; no reference counterpart):
        float32[n, 8] = (centre.xyz, radius, albedo.rgb, type); n = 0 removes
        them.  Deep copy; independent of upload_scene."""
        s = np.ascontiguousarray(np.asarray(spheres, dtype=np.float32).reshape(-1, 8))
        check(lib().rt_upload_spheres(self._ctx, s.ctypes.data if len(s) else None, len(s)))

    def upload_raw(self, vertices: bytes, materials: bytes, nodes: bytes) -> None:
        check(lib().rt_upload_scene(self._ctx, vertices, len(vertices), materials, len(materials),
                                    nodes, len(nodes)))

    def scene_info(self) -> dict:
        nn, nt, d = C.c_size_t(), C.c_size_t(), C.c_int()
        check(lib().rt_scene_info(self._ctx, C.byref(nn), C.byref(nt), C.byref(d)))
        return {"n_nodes": nn.value, "n_tris": nt.value, "max_depth": d.value}

    def render(self, camera, width: int, height: int, max_bounces: int = REFERENCE_MAX_BOUNCES,
               radiance: bool = False, stats: bool = False):
        """renderFrame (VulkanEngine.java:401-431).  Returns (rgba[H,W,4] uint8,
        radiance[H,W,3] float32 or None, stats dict or None)."""
        rgba = np.empty((height, width, 4), dtype=np.uint8)
        rad = np.empty((height, width, 3), dtype=np.float32) if radiance else None
        st = Stats() if stats else None
        check(lib().rt_render(self._ctx, C.byref(_ubo(camera)), width, height, max_bounces,
                              rgba.ctypes.data, rad.ctypes.data if rad is not None else None,
                              C.byref(st) if st is not None else None))
        return rgba, rad, (st.as_dict() if st is not None else None)

    def render_async(self, camera, width: int, height: int, max_bounces: int, out: "PinnedFrame") -> int:
        """Enqueue a whole frame into a pinned host frame and return its ticket
        (rt_render_async); the frame is complete after wait(ticket)."""
        if out.shape != (height, width, 4):
            raise ValueError(f"frame buffer is {out.shape}, need {(height, width, 4)}")
        t = C.c_uint64()
        check(lib().rt_render_async(self._ctx, C.byref(_ubo(camera)), width, height, max_bounces,
                                    out.ptr, C.byref(t)))
        return t.value

    def wait(self, ticket: int) -> None:
        check(lib().rt_render_wait(self._ctx, ticket))

    def poll(self, ticket: int) -> bool:
        """True when the frame of `ticket` is complete (rt_render_poll; never blocks)."""
        done = C.c_int32()
        check(lib().rt_render_poll(self._ctx, ticket, C.byref(done)))
        return bool(done.value)

    def render_tile_device(self, camera, width: int, height: int, max_bounces: int,
                           x0: int, y0: int, tile_w: int, tile_h: int,
                           d_rgba: Optional[int], d_radiance: Optional[int] = None,
                           stream: Optional[int] = None, stats: bool = False):
        """Enqueue one tile into device buffers (raw device pointers, e.g.
        torch tensor data_ptr()) on a HIP stream handle."""
        st = Stats() if stats else None
        check(lib().rt_render_tile_device(self._ctx, C.byref(_ubo(camera)), width, height, max_bounces,
                                          x0, y0, tile_w, tile_h, d_rgba, d_radiance, stream,
                                          C.byref(st) if st is not None else None))
        return st.as_dict() if st is not None else None


class PinnedFrame:
    """An RGBA8 frame in pinned host memory (rt_host_alloc), as a numpy view."""

    def __init__(self, height: int, width: int):
        n = height * width * 4
        self.ptr = lib().rt_host_alloc(n)
        if not self.ptr:
            raise RtError(-6, lib().rt_last_error().decode())   # RT_ERR_OOM
        self.array = np.ctypeslib.as_array((C.c_uint8 * n).from_address(self.ptr)).reshape(height, width, 4)
        self.shape = self.array.shape

    def close(self) -> None:
        if self.ptr:
            self.array = None
            lib().rt_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.close()


@dataclass
class FrameData:
    """FrameData.java: RGBA8 pixels of one frame, row 0 = top."""
    pixel_data: np.ndarray
    stats: Optional[dict] = None


class AtomicReference:
    """The java.util.concurrent.atomic.AtomicReference the UI shares with the engine."""

    def __init__(self, value=None):
        self._v = value
        self._lock = threading.Lock()

    def set(self, v) -> None:
        with self._lock:
            self._v = v

    def get(self):
        with self._lock:
            return self._v

    def get_and_set(self, v):
        with self._lock:
            old, self._v = self._v, v
            return old


class HipEngine:
    """Drop-in for VulkanEngine: same public methods, a render thread that owns
    the rt_ctx (single-thread affinity, VulkanEngine.java:194-206)."""

    def __init__(self, frame_queue: AtomicReference, width: int = REFERENCE_WIDTH,
                 height: int = REFERENCE_HEIGHT, max_bounces: int = REFERENCE_MAX_BOUNCES,
                 device_ids: Sequence[int] = (0,), collect_stats: bool = False, pipelined: bool = True,
                 inflight: int = 4):
        self.frame_queue = frame_queue
        # pipelined: `inflight` frames in flight (rt_render_async, one slot and
        # trace stream each), so the frames' traces overlap each other and
        # their readbacks; the reference waits for each frame
        # (VulkanEngine.java:410-429).  Stats need the synchronous path.
        self.pipelined = pipelined and not collect_stats
        self.inflight = max(1, min(8, int(inflight)))
        self.width, self.height, self.max_bounces = width, height, max_bounces
        self.device_ids = tuple(device_ids)
        self.collect_stats = collect_stats
        self._scene_q: "queue.Queue[BuiltCpuData]" = queue.Queue()
        self._camera_q: "queue.Queue[Camera]" = queue.Queue()
        self._sky_q: "queue.Queue[bool]" = queue.Queue()
        self._running = False
        self._thread = threading.Thread(target=self._run, name="HIP-Engine-Thread", daemon=True)
        self.is_sky_enabled = 1
        self.frames_rendered = 0
        self.frames_submitted = 0
        self.error: Optional[BaseException] = None

    # --- public API (UI thread) ---
    def start(self) -> None:
        self._running = True
        self._thread.start()

    def stop(self) -> None:
        self._running = False
        self._thread.join(5.0)          # 5 s graceful window, VulkanEngine.java:145

    def submit_scene(self, scene_data: BuiltCpuData) -> None:
        self._scene_q.put(scene_data)

    def submit_camera_update(self, camera: Camera) -> None:
        self._camera_q.put(camera)

    def submit_sky_toggle(self, is_sky_on: bool) -> None:
        self._sky_q.put(bool(is_sky_on))

    # --- render thread ---
    def _run(self) -> None:
        renderer = None
        slots, pending = None, []
        try:
            renderer = Renderer(self.device_ids)
            renderer.set_option("async_slots", self.inflight)
            have_scene, camera = False, None
            while self._running:
                try:                                        # one scene per pass (:281-285)
                    scene = self._scene_q.get_nowait()
                    while pending:                          # frames of the old scene first
                        self._finish(renderer, slots, pending.pop(0))
                    renderer.upload_scene(scene)
                    have_scene = True
                except queue.Empty:
                    pass
                while True:                                 # drain to the latest camera (:288-298)
                    try:
                        camera = self._camera_q.get_nowait()
                    except queue.Empty:
                        break
                while True:                                 # latest sky state (:300-312)
                    try:
                        self.is_sky_enabled = 1 if self._sky_q.get_nowait() else 0
                    except queue.Empty:
                        break
                if not have_scene or camera is None:
                    time.sleep(0.016)
                    continue
                ubo = CameraUBO.from_buffer_copy(bytes(camera.ubo))
                ubo.sky_enabled = self.is_sky_enabled        # written, ignored by the shader
                if not self.pipelined:
                    rgba, _, st = renderer.render(ubo, self.width, self.height, self.max_bounces,
                                                  stats=self.collect_stats)
                    self._publish(FrameData(rgba, st))
                    continue
                if slots is None:
                    slots = [PinnedFrame(self.height, self.width) for _ in range(self.inflight)]
                k = self.frames_submitted % self.inflight
                pending.append((renderer.render_async(ubo, self.width, self.height, self.max_bounces, slots[k]), k))
                self.frames_submitted += 1
                if len(pending) == self.inflight:
                    self._finish(renderer, slots, pending.pop(0))
            while pending:                                  # drain on stop
                self._finish(renderer, slots, pending.pop(0))
        except BaseException as e:                          # FATAL (VRT) path, :197-201
            self.error = e
            self._running = False
        finally:
            if renderer is not None:
                renderer.close()
            for f in slots or ():
                f.close()

    def _finish(self, renderer, slots, item) -> None:
        ticket, k = item
        renderer.wait(ticket)
        # a fresh buffer per frame, as the reference publishes (:416-429)
        self._publish(FrameData(slots[k].array.copy()))

    def _publish(self, frame: "FrameData") -> None:
        self.frame_queue.set(frame)
        self.frames_rendered += 1
