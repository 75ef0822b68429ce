"""Scene side of the host API: a Python mirror of the reference's scene model and
SceneBuilder, producing the three buffers the render path consumes.

Mirrors (names, argument meaning, error behaviour):
  ModelInstance      src/dev/demir/vulkan/scene/ModelInstance.java:11-68 (defaults :34-43)
  Scene              src/dev/demir/vulkan/scene/Scene.java:17-69
  Camera             src/dev/demir/vulkan/scene/Camera.java:11-118
  SceneBuilder       src/dev/demir/vulkan/renderer/SceneBuilder.java:38-191
  BuiltCpuData       src/dev/demir/vulkan/renderer/BuiltCpuData.java:10-22

The heavy lifting (OBJ parse, median-split BVH, preorder flatten, packing,
camera basis) is native C++ behind the C ABI (csrc/scene_build.cpp).
"""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import CameraUBO, check, lib

Vec3 = Tuple[float, float, float]

DEFAULT_AXIS_SEED = 1


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Mesh:
    """Model-space triangles as float32 (n, 3, 3) — what Assimp hands the
    reference (aiVector3D is float)."""

    def __init__(self, tris: np.ndarray, name: str = "mesh"):
        tris = np.ascontiguousarray(tris, dtype=np.float32)
        if tris.ndim != 3 or tris.shape[1:] != (3, 3):
            raise ValueError("mesh triangles must have shape (n, 3, 3)")
        self.tris = tris
        self.name = name

    def __len__(self) -> int:
        return self.tris.shape[0]

    @staticmethod
    def load_obj(path: str) -> "Mesh":
        """aiImportFile(path, Triangulate | JoinIdenticalVertices) (SceneBuilder.java:144)."""
        L = lib()
        h = C.c_void_p()
        check(L.rt_mesh_load_obj(path.encode(), C.byref(h)))
        try:
            n = L.rt_mesh_tri_count(h)
            out = np.empty((n, 3, 3), dtype=np.float64)
            one = np.ones(3)
            zero = np.zeros(3)
            if n:
                check(L.rt_mesh_transform(h, _dptr(one), _dptr(zero), _dptr(out)))
        finally:
            L.rt_mesh_free(h)
        return Mesh(out.astype(np.float32), name=path)

    @staticmethod
    def procedural(n_tris: int, seed: int, bmin: Vec3, bmax: Vec3) -> "Mesh":
        """Seeded closed shell with exactly n_tris triangles inside [bmin, bmax]."""
        out = np.empty((n_tris, 3, 3), dtype=np.float64)
        check(lib().rt_mesh_procedural(n_tris, seed, _dptr(np.asarray(bmin, dtype=np.float64)),
                                       _dptr(np.asarray(bmax, dtype=np.float64)), _dptr(out)))
        return Mesh(out.astype(np.float32), name=f"procedural(n={n_tris}, seed={seed:#x})")


_mesh_cache: dict = {}


class ModelInstance:
    """One placed model: path (or mesh), position, scale, color, material type.
    Defaults as ModelInstance.java:34-43: pos (0,0,0), scale (1,1,1), color
    (0.8,0.8,0.8), type 0.0 (Lambertian)."""

    def __init__(self, model_path: str, display_name: str, mesh: Optional[Mesh] = None):
        self.model_path = model_path
        self.display_name = display_name
        self.position: Vec3 = (0.0, 0.0, 0.0)
        self.scale: Vec3 = (1.0, 1.0, 1.0)
        self.color: Vec3 = (0.8, 0.8, 0.8)
        self.material_type: float = 0.0
        self._mesh = mesh

    # Java-style accessors (ModelInstance.java:46-59)
    def get_model_path(self): return self.model_path
    def get_display_name(self): return self.display_name
    def get_position(self): return self.position
    def set_position(self, p: Vec3): self.position = tuple(map(float, p))
    def get_scale(self): return self.scale
    def set_scale(self, s: Vec3): self.scale = tuple(map(float, s))
    def get_color(self): return self.color
    def set_color(self, c: Vec3): self.color = tuple(map(float, c))
    def get_material_type(self): return self.material_type
    def set_material_type(self, t: float): self.material_type = float(np.float32(t))

    def mesh(self) -> Mesh:
        if self._mesh is None:
            m = _mesh_cache.get(self.model_path)
            if m is None:
                m = Mesh.load_obj(self.model_path)
                _mesh_cache[self.model_path] = m
            self._mesh = m
        return self._mesh

    def __str__(self) -> str:
        return self.display_name


class Scene:
    """Thread-safe instance list (Scene.java:17-69)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._instances: List[ModelInstance] = []

    def add_instance(self, inst: ModelInstance) -> None:
        with self._lock:
            self._instances.append(inst)

    def remove_instance(self, inst: ModelInstance) -> None:
        with self._lock:
            self._instances.remove(inst)

    def get_instances(self) -> List[ModelInstance]:
        with self._lock:
            return list(self._instances)

    def create_snapshot(self) -> "Scene":
        s = Scene()
        for i in self.get_instances():
            s.add_instance(i)
        return s


class Camera:
    """Camera.java: origin/lookAt/vUp/vfov/aspect; the viewport vectors are
    computed natively in double and stored as the 80-B UBO (floats)."""

    def __init__(self, origin: Vec3, look_at: Vec3, v_up: Vec3, vfov: float, aspect_ratio: float):
        self.origin = tuple(map(float, origin))
        self.look_at = tuple(map(float, look_at))
        self.v_up = tuple(map(float, v_up))
        self.vfov = float(vfov)
        self.aspect_ratio = float(aspect_ratio)
        self.frame_count = 0
        self.ubo = CameraUBO()
        self._recalculate()

    def _recalculate(self) -> None:
        check(lib().rt_camera_from_lookat(_dptr(np.asarray(self.origin)), _dptr(np.asarray(self.look_at)),
                                          _dptr(np.asarray(self.v_up)), self.vfov, self.aspect_ratio,
                                          C.byref(self.ubo)))
        self.ubo.frame_count = self.frame_count

    def get_origin(self) -> Vec3: return self.origin

    def set_origin(self, origin: Vec3) -> None:
        self.origin = tuple(map(float, origin))
        self._recalculate()

    def get_lower_left(self): return tuple(self.ubo.lower_left[:3])
    def get_horizontal(self): return tuple(self.ubo.horizontal[:3])
    def get_vertical(self): return tuple(self.ubo.vertical[:3])
    def reset_accumulation(self): self.frame_count = 0; self.ubo.frame_count = 0
    def increment_frame_count(self): self.frame_count += 1; self.ubo.frame_count = self.frame_count
    def get_frame_count(self): return self.frame_count

    def ubo_bytes(self) -> bytes:
        return bytes(self.ubo)

    @staticmethod
    def default(width: int, height: int) -> "Camera":
        """The app's default camera (VulkanApp.java:132-138)."""
        return Camera((-25.0, 30.0, 140.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, float(width) / float(height))


@dataclass
class BuiltCpuData:
    """BuiltCpuData.java: the three buffers + flattened triangle count."""
    model_vertex_data: np.ndarray     # float32, 12 per flattened triangle
    model_material_data: np.ndarray   # float32, 4 per flattened triangle
    flat_bvh_data: np.ndarray         # uint8, 48 per node
    triangle_count: int

    @property
    def n_nodes(self) -> int:
        return self.flat_bvh_data.size // 48


def triangles_of(scene: Scene) -> Tuple[np.ndarray, np.ndarray]:
    """loadModel for every instance (SceneBuilder.java:47-59, 129-191): returns
    post-transform double vertices (n,9) and float materials (n,4)."""
    verts, mats = [], []
    for inst in scene.get_instances():
        try:
            m = inst.mesh()
        except Exception as e:  # SceneBuilder.java:55-58: skip the model, keep going
            print(f"WARN (SRT): Failed to load model {inst.model_path}: {e}")
            continue
        v = m.tris.astype(np.float64) * np.asarray(inst.scale, dtype=np.float64) + np.asarray(inst.position, dtype=np.float64)
        verts.append(v.reshape(-1, 9))
        mat = np.empty((len(m), 4), dtype=np.float32)
        mat[:, :3] = np.asarray(inst.color, dtype=np.float64).astype(np.float32)
        mat[:, 3] = np.float32(inst.material_type)
        mats.append(mat)
    if not verts:
        return np.zeros((0, 9)), np.zeros((0, 4), dtype=np.float32)
    return np.concatenate(verts), np.concatenate(mats)


def build_buffers(tri_verts: np.ndarray, tri_mats: np.ndarray, axis_seed: int = DEFAULT_AXIS_SEED,
                  n_threads: int = 0) -> BuiltCpuData:
    """BVHBuilder.build + BVHFlattener.flatten + packing (SceneBuilder.java:75-117)."""
    L = lib()
    tri_verts = np.ascontiguousarray(tri_verts, dtype=np.float64).reshape(-1, 9)
    tri_mats = np.ascontiguousarray(tri_mats, dtype=np.float32).reshape(-1, 4)
    n = tri_verts.shape[0]
    if n == 0:
        # SceneBuilder.java:61-70: 1-float / 1-byte dummies, triangleCount 0.
        return BuiltCpuData(np.zeros(1, np.float32), np.zeros(1, np.float32), np.zeros(1, np.uint8), 0)
    nn, nf = C.c_size_t(), C.c_size_t()
    check(L.rt_bvh_layout_size(n, C.byref(nn), C.byref(nf)))
    v = np.empty(nf.value * 12, dtype=np.float32)
    m = np.empty(nf.value * 4, dtype=np.float32)
    b = np.empty(nn.value * 48, dtype=np.uint8)
    check(L.rt_build_scene(_dptr(tri_verts), _fptr(tri_mats), n, axis_seed, n_threads,
                           _fptr(v), _fptr(m), b.ctypes.data_as(C.c_void_p)))
    return BuiltCpuData(v, m, b, nf.value)


class SceneBuilder:
    """SceneBuilder.buildScene(Scene) -> BuiltCpuData (SceneBuilder.java:38-118)."""

    def __init__(self, axis_seed: int = DEFAULT_AXIS_SEED, n_threads: int = 0):
        self.axis_seed = axis_seed
        self.n_threads = n_threads

    def build_scene(self, scene: Scene) -> BuiltCpuData:
        verts, mats = triangles_of(scene)
        return build_buffers(verts, mats, self.axis_seed, self.n_threads)
