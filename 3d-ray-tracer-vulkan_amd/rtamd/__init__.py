"""rtamd — MI355X (gfx950) backend for the per-pixel path-trace path of
this-Demir/3D-Ray-Tracer-Vulkan.

The product is the native library lib/librtamd.so (HIP kernels + C ABI,
include/rtamd.h); this package is the Python host side over that ABI:
scene model and builder (scene.py), renderer and a VulkanEngine-shaped engine
(engine.py), the benchmark configurations (configs.py) and multi-GPU tiling
(dist.py).
"""
import os as _os

# Frames in flight (rt_render_async slots, a caller's streams) run at once
# only on hardware queues of their own; HIP's default is 4 per process and is
# fixed when the HIP runtime loads, so the variable must be set before the
# first import of torch or of the library (bench.py sets it likewise).
if int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    _os.environ["GPU_MAX_HW_QUEUES"] = "16"

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
