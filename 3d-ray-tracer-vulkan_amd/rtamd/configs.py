"""The BASELINE.json configurations as concrete scenes.

All use the app's default camera (VulkanApp.java:132-138) with aspect W/H.
cube / ground_plane geometry is built in code (the triangles of the
reference's objects/cube.obj and objects/ground_plane.obj: unit cube centred
at the origin, 12 triangles; 2-triangle XZ plane of half-size 1), so that the
GPU box, which has no /root/reference, can build every config; tests check
these against the OBJ files themselves when the reference is present.
"""
from __future__ import annotations

import gzip
import os
import tempfile

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .scene import Camera, Mesh, ModelInstance, Scene, SceneBuilder, BuiltCpuData

# FinalBaseMesh.obj's bounding box (objects/FinalBaseMesh.obj, 24,461 vertices).
FINAL_BASE_MESH_BMIN = (-5.8425, -0.0566, -1.8531)
FINAL_BASE_MESH_BMAX = (5.8425, 20.6841, 1.9170)

_CUBE_V = np.array([(-0.5, -0.5, 0.5), (0.5, -0.5, 0.5), (-0.5, 0.5, 0.5), (0.5, 0.5, 0.5),
                    (-0.5, 0.5, -0.5), (0.5, 0.5, -0.5), (-0.5, -0.5, -0.5), (0.5, -0.5, -0.5)],
                   dtype=np.float32)
_CUBE_F = np.array([(1, 2, 4), (1, 4, 3), (3, 4, 6), (3, 6, 5), (5, 6, 8), (5, 8, 7),
                    (7, 8, 2), (7, 2, 1), (2, 8, 6), (2, 6, 4), (7, 1, 3), (7, 3, 5)]) - 1
_PLANE_V = np.array([(-1.0, 0.0, 1.0), (1.0, 0.0, 1.0), (1.0, 0.0, -1.0), (-1.0, 0.0, -1.0)],
                    dtype=np.float32)
_PLANE_F = np.array([(1, 2, 3), (1, 3, 4)]) - 1


def cube_mesh() -> Mesh:
    return Mesh(_CUBE_V[_CUBE_F], name="cube")


def plane_mesh() -> Mesh:
    return Mesh(_PLANE_V[_PLANE_F], name="ground_plane")


def ground_plane_instance() -> ModelInstance:
    """VulkanApp.java:313-317: pos (0,-10,0), scale (150,1,150), grey 0.5, Lambertian."""
    p = ModelInstance("./objects/ground_plane.obj", "Ground Plane", mesh=plane_mesh())
    p.set_position((0.0, -10.0, 0.0))
    p.set_scale((150.0, 1.0, 150.0))
    p.set_color((0.5, 0.5, 0.5))
    p.set_material_type(0.0)
    return p


@dataclass
class RenderConfig:
    name: str
    scene: Scene
    width: int
    height: int
    max_bounces: int
    note: str = ""

    def camera(self) -> Camera:
        return Camera.default(self.width, self.height)

    def build(self, axis_seed: int = 1, n_threads: int = 0) -> BuiltCpuData:
        return SceneBuilder(axis_seed, n_threads).build_scene(self.scene)


def config1() -> RenderConfig:
    s = Scene()
    c = ModelInstance("./objects/cube.obj", "Cube", mesh=cube_mesh())
    c.set_scale((20.0, 20.0, 20.0))
    c.set_color((0.5, 0.5, 0.5))
    c.set_material_type(0.0)
    s.add_instance(c)
    return RenderConfig("cfg1_cube_640x480_b1", s, 640, 480, 1, "cube only, Lambertian; 1 bounce")


def config2() -> RenderConfig:
    s = Scene()
    s.add_instance(ground_plane_instance())
    c = ModelInstance("./objects/cube.obj", "Cube", mesh=cube_mesh())
    c.set_position((0.0, -5.0, 0.0))          # resting on the plane (y = -10)
    c.set_scale((10.0, 10.0, 10.0))
    c.set_color((0.6, 0.7, 0.1))         # the car's colour/material, VulkanApp.java:322-326
    c.set_material_type(1.0)
    s.add_instance(c)
    return RenderConfig("cfg2_cube_plane_1280x720_b2", s, 1280, 720, 2, "cube (metal) + ground plane")


def synthetic_scene(n_tris: int, seed: int = 0x5EED, all_types: bool = False) -> Scene:
    """Config 3/4 (50k) and 5 (1M): a procedural FinalBaseMesh-sized shell on the
    ground plane plus a small type-3 ("emissive") cube that renders black
    (compute_dynamic_ray.comp:153).  all_types: four shells of types 0/1/2/3."""
    s = Scene()
    s.add_instance(ground_plane_instance())
    if not all_types:
        m = ModelInstance("procedural://shell", "Synthetic mesh",
                          mesh=Mesh.procedural(n_tris, seed, FINAL_BASE_MESH_BMIN, FINAL_BASE_MESH_BMAX))
        m.set_position((0.0, -10.0, 0.0))
        m.set_color((0.8, 0.8, 0.8))
        m.set_material_type(1.0)
        s.add_instance(m)
    else:
        per = n_tris // 4
        per -= per % 2
        colors = [(0.8, 0.3, 0.3), (0.8, 0.8, 0.8), (0.3, 0.6, 0.9), (4.0, 4.0, 4.0)]
        for k in range(4):
            m = ModelInstance(f"procedural://shell{k}", f"Synthetic mesh {k}",
                              mesh=Mesh.procedural(per, seed + k, FINAL_BASE_MESH_BMIN, FINAL_BASE_MESH_BMAX))
            m.set_position((-21.0 + 14.0 * k, -10.0, 0.0))
            m.set_color(colors[k])
            m.set_material_type(float(k))
            s.add_instance(m)
    light = ModelInstance("./objects/cube.obj", "Light Source", mesh=cube_mesh())
    light.set_position((0.0, 40.0, 0.0))
    light.set_scale((5.0, 5.0, 5.0))
    light.set_color((4.0, 4.0, 4.0))
    light.set_material_type(3.0)
    s.add_instance(light)
    return s


def config3() -> RenderConfig:
    return RenderConfig("cfg3_50k_1920x1080_b4", synthetic_scene(50_000), 1920, 1080, 4,
                        "50k-triangle procedural shell (metal) + plane + type-3 cube")


def config4() -> RenderConfig:
    return RenderConfig("cfg4_50k_1920x1080_b8", synthetic_scene(50_000), 1920, 1080, 8,
                        "config 3 scene at 8 bounces (tiled over GPUs)")


def config5() -> RenderConfig:
    return RenderConfig("cfg5_1M_3840x2160_b8", synthetic_scene(1_000_000, all_types=True), 3840, 2160, 8,
                        "1M triangles, material types 0/1/2/3")


# The reference's own objects/FinalBaseMesh.obj (24,459 quads), committed
# gzip'd as a data fixture so that the GPU box, which has no /root/reference,
# can render the real mesh ("also run FinalBaseMesh itself").
FINAL_BASE_MESH_GZ = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                  "tests", "golden", "FinalBaseMesh.obj.gz")


def final_base_mesh() -> Mesh:
    """objects/FinalBaseMesh.obj through the OBJ loader (SceneBuilder.loadModel,
    SceneBuilder.java:129-191; Assimp's quad rule): 48,918 triangles."""
    with gzip.open(FINAL_BASE_MESH_GZ, "rb") as f:
        data = f.read()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "FinalBaseMesh.obj")
        with open(path, "wb") as g:
            g.write(data)
        return Mesh.load_obj(path)


def config6() -> RenderConfig:
    """Config 3's placement and material with the real FinalBaseMesh in place of
    the procedural shell: the SURVEY's probe scene (mesh + plane + type-3 cube)."""
    s = Scene()
    s.add_instance(ground_plane_instance())
    m = ModelInstance("./objects/FinalBaseMesh.obj", "FinalBaseMesh", mesh=final_base_mesh())
    m.set_position((0.0, -10.0, 0.0))
    m.set_color((0.8, 0.8, 0.8))
    m.set_material_type(1.0)
    s.add_instance(m)
    light = ModelInstance("./objects/cube.obj", "Light Source", mesh=cube_mesh())
    light.set_position((0.0, 40.0, 0.0))
    light.set_scale((5.0, 5.0, 5.0))
    light.set_color((4.0, 4.0, 4.0))
    light.set_material_type(3.0)
    s.add_instance(light)
    return RenderConfig("cfg6_fbm_1920x1080_b4", s, 1920, 1080, 4,
                        "the reference's FinalBaseMesh.obj (metal) + plane + type-3 cube")


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5, 6: config6}


def get(k: int) -> RenderConfig:
    return CONFIGS[k]()
