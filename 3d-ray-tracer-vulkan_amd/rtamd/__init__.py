"""rtamd — MI355X (gfx950) backend for the per-pixel path-trace path of
this-Demir/3D-Ray-Tracer-Vulkan.

The product is the native library lib/librtamd.so (HIP kernels + C ABI,
include/rtamd.h); this package is the Python host side over that ABI:
scene model and builder (scene.py), renderer and a VulkanEngine-shaped engine
(engine.py), the benchmark configurations (configs.py) and multi-GPU tiling
(dist.py).
"""
import os as _os
import sys as _sys
import warnings as _warnings

# Frames in flight (rt_render_async slots, a caller's streams) run at once
# only on hardware queues of their own.  HIP's default is 4 per process and is
# read once, when the HIP runtime initialises, so this only helps if nothing
# in the process has initialised HIP yet (bench.py sets it at its top as
# well).  A host that starts HIP first (or a JVM) must set
# GPU_MAX_HW_QUEUES >= frames in flight + 2 itself; rt_get_option("hw_queues")
# and "queues_short" report what the library saw.
_HW_QUEUES = 16


def _want_queues() -> None:
    raw = _os.environ.get("GPU_MAX_HW_QUEUES", "")
    try:
        have = int(raw) if raw.strip() else 4
    except ValueError:
        _warnings.warn(f"GPU_MAX_HW_QUEUES={raw!r} is not an integer; leaving it alone", RuntimeWarning)
        return
    if have >= _HW_QUEUES:
        return
    torch = _sys.modules.get("torch")
    try:
        started = torch is not None and torch.cuda.is_initialized()
    except Exception:
        started = False
    if started:
        _warnings.warn(f"HIP is already initialised with GPU_MAX_HW_QUEUES={have}: frames in flight on more "
                       f"than {max(1, have - 2)} streams will share hardware queues", RuntimeWarning)
        return
    _os.environ["GPU_MAX_HW_QUEUES"] = str(_HW_QUEUES)


_want_queues()

from ._lib import LIB_PATH, RtError, CameraUBO, Stats, lib  # noqa: E402
from .scene import (BuiltCpuData, Camera, Mesh, ModelInstance, Scene, SceneBuilder,
                    build_buffers, triangles_of)
from .engine import AtomicReference, FrameData, HipEngine, Renderer

__all__ = [
    "LIB_PATH", "RtError", "CameraUBO", "Stats", "lib",
    "BuiltCpuData", "Camera", "Mesh", "ModelInstance", "Scene", "SceneBuilder",
    "build_buffers", "triangles_of",
    "AtomicReference", "FrameData", "HipEngine", "Renderer",
]
