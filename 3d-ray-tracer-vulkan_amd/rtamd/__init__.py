"""rtamd — MI355X (gfx950) backend for the per-pixel path-trace path of
this-Demir/3D-Ray-Tracer-Vulkan.

The product is the native library lib/librtamd.so (HIP kernels + C ABI,
include/rtamd.h); this package is the Python host side over that ABI:
scene model and builder (scene.py), renderer and a VulkanEngine-shaped engine
(engine.py), the benchmark configurations (configs.py) and multi-GPU tiling
(dist.py).
"""
from ._lib import LIB_PATH, RtError, CameraUBO, Stats, lib
from .scene import (BuiltCpuData, Camera, Mesh, ModelInstance, Scene, SceneBuilder,
                    build_buffers, triangles_of)
from .engine import AtomicReference, FrameData, HipEngine, Renderer

__all__ = [
    "LIB_PATH", "RtError", "CameraUBO", "Stats", "lib",
    "BuiltCpuData", "Camera", "Mesh", "ModelInstance", "Scene", "SceneBuilder",
    "build_buffers", "triangles_of",
    "AtomicReference", "FrameData", "HipEngine", "Renderer",
]
