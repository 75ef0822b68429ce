"""ctypes wrapper of oracle/liboracle.so (rt_oracle.c).  TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
ENV_LIB = os.path.join(HERE, "liboracle_env.so")     # rt_envelope.c: the Vulkan-envelope study
ACCEL_LIB = os.path.join(HERE, "liboracle_accel.so") # rt_accel_model.c: option accel's walk on the CPU
ENV_FMA, ENV_RSQ, ENV_RCP, ENV_ULP, ENV_FTZ = 1, 2, 4, 8, 16   # rt_oracle.c ENV_* bits
ENV_ULP2, ENV_SQRT_RCP, ENV_SQRT_MUL = 32, 64, 128


class Counts(C.Structure):
    _fields_ = [("pixels", C.c_uint64), ("segments", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("mat_reads", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None
_env_lib = None
_accel_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(envelope: bool = False, accel: bool = False) -> C.CDLL:
    """liboracle.so (the contract), or with envelope=True liboracle_env.so
    (the same oracle with orc_env_set_variant), or with accel=True
    liboracle_accel.so (the oracle walking option accel's records)."""
    global _lib, _env_lib, _accel_lib
    if accel:
        if _accel_lib is None:
            if not os.path.exists(ACCEL_LIB):
                build()
            _accel_lib = _bind(C.CDLL(ACCEL_LIB))
            _accel_lib.orc_accel_set.restype = C.c_int
            _accel_lib.orc_accel_set.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
            _accel_lib.orc_accel_format.argtypes = [C.c_int]
            _accel_lib.orc_accel_fallbacks.restype = C.c_uint64
            _accel_lib.orc_accel_margin.argtypes = [C.c_float, C.c_float]
            _accel_lib.orc_accel_audit.argtypes = [C.c_int]
            _accel_lib.orc_accel_audit_get.argtypes = [C.POINTER(C.c_double)]
            _accel_lib.orc_accel_relax_half.argtypes = [C.c_float]
            _accel_lib.orc_accel_overflows.restype = C.c_uint64
            _accel_lib.orc_accel_stack.argtypes = [C.c_int]
            _accel_lib.orc_accel_count_steps.argtypes = [C.c_int]
            _accel_lib.orc_accel_audit_bins.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double),
                                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        return _accel_lib
    if envelope:
        if _env_lib is None:
            if not os.path.exists(ENV_LIB):
                build()
            _env_lib = _bind(C.CDLL(ENV_LIB))
            _env_lib.orc_env_set_variant.restype = C.c_int
            _env_lib.orc_env_set_variant.argtypes = [C.c_int]
        return _env_lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = _bind(C.CDLL(LIB))
    return _lib


def _bind(L: C.CDLL) -> C.CDLL:
    f3 = C.POINTER(C.c_float)
    L.orc_pcg.restype = C.c_uint32
    L.orc_pcg.argtypes = [C.c_uint32]
    L.orc_random_float.restype = C.c_float
    L.orc_random_float.argtypes = [C.POINTER(C.c_uint32)]
    L.orc_random_in_unit_sphere.argtypes = [C.POINTER(C.c_uint32), f3]
    L.orc_hit_aabb.argtypes = [f3, f3, f3, f3, C.c_float, C.c_float]
    L.orc_hit_triangle.argtypes = [f3, f3, f3, f3, f3, f3, f3]
    L.orc_hit_sphere.argtypes = [f3, f3, f3, f3, f3]
    L.orc_scatter.argtypes = [f3, C.POINTER(C.c_uint32), f3, f3, f3, f3, f3]
    L.orc_render.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                             C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                             C.c_int, C.c_void_p, C.c_void_p, C.POINTER(Counts), C.c_int]
    L.orc_render_ext.argtypes = L.orc_render.argtypes + [C.c_int, C.c_void_p]
    L.orc_render_profile.argtypes = L.orc_render.argtypes + [C.c_void_p]
    L.orc_render_spheres.argtypes = L.orc_render_ext.argtypes + [C.c_void_p, C.c_int]
    return L


def _buf(x):
    a = np.ascontiguousarray(np.frombuffer(x, dtype=np.uint8) if isinstance(x, (bytes, bytearray)) else x)
    return a, a.ctypes.data, a.nbytes


EXT_SKY_TOGGLE, EXT_EMISSIVE, EXT_ACCUMULATE, EXT_SPHERES = 1, 2, 4, 8   # rt_oracle.h ORC_EXT_*


def render(vertices, materials, nodes, camera_ubo: bytes, width: int, height: int, max_bounces: int,
           tile=None, row_step: int = 1, radiance: bool = True, n_threads: int = 0, ext: int = 0,
           accum: "np.ndarray | None" = None, spheres: "np.ndarray | None" = None, variant: "int | None" = None):
    """Returns (rgba[rows, w, 4], radiance[rows, w, 3] or None, counts dict).
    ext: ORC_EXT_* bits (non-reference extensions); accum: float32[rows, w, 3],
    updated in place, required with EXT_ACCUMULATE; spheres: float32[n, 8]
    (centre.xyz, radius, albedo.rgb, type), tested with EXT_SPHERES.
    variant: ENV_* bits: render with liboracle_env.so (the Vulkan-envelope
    study) instead of the contract's liboracle.so."""
    x0, y0, tw, th = tile if tile is not None else (0, 0, width, height)
    rows = (th + row_step - 1) // row_step
    v, vp, vn = _buf(vertices)
    m, mp, mn = _buf(materials)
    b, bp, bn = _buf(nodes)
    cam = np.frombuffer(bytes(camera_ubo), dtype=np.uint8).copy()
    rgba = np.empty((rows, tw, 4), dtype=np.uint8)
    rad = np.empty((rows, tw, 3), dtype=np.float32) if radiance else None
    c = Counts()
    if accum is not None:
        assert accum.dtype == np.float32 and accum.shape == (rows, tw, 3) and accum.flags.c_contiguous
    sph = np.ascontiguousarray(spheres if spheres is not None else np.zeros((0, 8)), dtype=np.float32)
    assert sph.ndim == 2 and sph.shape[1] == 8
    L = lib()
    if variant is not None:                 # the envelope build, with these ENV_* bits
        L = lib(envelope=True)
        L.orc_env_set_variant(int(variant))
    rc = L.orc_render_spheres(vp, vn, mp, mn, bp, bn, cam.ctypes.data, width, height, max_bounces,
                                  x0, y0, tw, th, row_step, rgba.ctypes.data,
                                  rad.ctypes.data if rad is not None else None, C.byref(c), n_threads,
                                  ext, accum.ctypes.data if accum is not None else None,
                                  sph.ctypes.data if len(sph) else None, len(sph))
    if rc != 0:
        raise RuntimeError(f"orc_render failed ({rc})")
    return rgba, rad, c.as_dict()


def accel_relax(cls: int) -> float:
    """accel_build.h accel_relax: the margin factor of shape class cls."""
    one = np.float32(1.0)
    return float(one + np.float32(2.0 ** -10)) if cls < 7 else float(one + np.float32(2.0 ** (cls - 16)))


def render_accel(vertices, materials, nodes, camera_ubo: bytes, width: int, height: int, max_bounces: int,
                 records: np.ndarray, info: dict, tile=None, row_step: int = 1, n_threads: int = 0,
                 profile: bool = False):
    """The same frame through option accel's walk (rt_accel_model.c) over
    `records` / `info` (rtamd._lib.accel_records).  Returns (rgba, radiance,
    counts[, profile uint32[rows, w, max_bounces]: node visits | tri tests << 20
    per bounce])."""
    x0, y0, tw, th = tile if tile is not None else (0, 0, width, height)
    rows = (th + row_step - 1) // row_step
    v, vp, vn = _buf(vertices)
    m, mp, mn = _buf(materials)
    b, bp, bn = _buf(nodes)
    rec = np.ascontiguousarray(records, dtype=np.uint32)
    cam = np.frombuffer(bytes(camera_ubo), dtype=np.uint8).copy()
    rgba = np.empty((rows, tw, 4), dtype=np.uint8)
    rad = np.empty((rows, tw, 3), dtype=np.float32)
    prof = np.zeros((rows, tw, max_bounces), dtype=np.uint32) if profile else None
    c = Counts()
    L = lib(accel=True)
    if L.orc_accel_format(int(info.get("format", 0))) != 0:
        raise RuntimeError("orc_accel_format failed")
    L.orc_accel_relax_half(accel_relax(int(info.get("max_class", 0))))
    if L.orc_accel_set(rec.ctypes.data, int(info["n_layouts"]), int(info["slots"]), int(info["root_leaf"])) != 0:
        raise RuntimeError("orc_accel_set failed")
    rc = L.orc_render_profile(vp, vn, mp, mn, bp, bn, cam.ctypes.data, width, height, max_bounces,
                              x0, y0, tw, th, row_step, rgba.ctypes.data, rad.ctypes.data, C.byref(c), n_threads,
                              prof.ctypes.data if prof is not None else None)
    if rc != 0:
        raise RuntimeError(f"orc_render_profile (accel) failed ({rc})")
    cd = c.as_dict()
    cd["fallbacks"] = int(L.orc_accel_fallbacks())
    cd["overflows"] = int(L.orc_accel_overflows())
    if profile:
        return rgba, rad, cd, prof
    return rgba, rad, cd


def accel_audit(on: bool = True) -> None:
    """Starts (or stops) the accel model's margin audit (rt_accel_model.c
    orc_accel_audit): every following render_accel segment is first walked
    exhaustively for the reference's candidate hit i* and its box."""
    lib(accel=True).orc_accel_audit(1 if on else 0)


def accel_audit_result() -> dict:
    """The audit since accel_audit(): segments with a hit, of them hits before
    their own box's t_enter, headroom > 0.5 of the margin, unsafe (the margin
    test with i*'s class factor fails: the exactness argument does not cover
    the segment), the largest headroom (te* - t*) / (t* 2^-10 + 2^-10) and the
    same against i*'s class margin (max_headroom_class), and the hits on
    near-degenerate triangles (|det| <= 1e-4, compute_dynamic_ray.comp:110 cuts
    at 1e-5) with their largest headroom."""
    out = (C.c_double * 8)()
    lib(accel=True).orc_accel_audit_get(out)
    sh, gr = (C.c_double * 32)(), (C.c_double * 32)()
    shn, grn = (C.c_uint64 * 32)(), (C.c_uint64 * 32)()
    lib(accel=True).orc_accel_audit_bins(sh, gr, shn, grn)

    def bins(mx, n):      # bin k: x in (2^-(k+1), 2^-k]; only the bins with hits
        return {str(k): [int(n[k]), float(mx[k])] for k in range(32) if n[k]}
    return {"hits": int(out[0]), "before_box": int(out[1]), "over_half": int(out[2]), "unsafe": int(out[3]),
            "max_headroom": float(out[4]), "sliver_hits": int(out[5]), "sliver_max_headroom": float(out[6]),
            "max_headroom_class": float(out[7]),
            "by_shape": bins(sh, shn), "by_grazing": bins(gr, grn)}


def render_profile(vertices, materials, nodes, camera_ubo: bytes, width: int, height: int, max_bounces: int,
                   tile=None, row_step: int = 1, n_threads: int = 0):
    """orc_render_profile of the contract oracle: (rgba, radiance, counts, profile)."""
    x0, y0, tw, th = tile if tile is not None else (0, 0, width, height)
    rows = (th + row_step - 1) // row_step
    v, vp, vn = _buf(vertices)
    m, mp, mn = _buf(materials)
    b, bp, bn = _buf(nodes)
    cam = np.frombuffer(bytes(camera_ubo), dtype=np.uint8).copy()
    rgba = np.empty((rows, tw, 4), dtype=np.uint8)
    rad = np.empty((rows, tw, 3), dtype=np.float32)
    prof = np.zeros((rows, tw, max_bounces), dtype=np.uint32)
    c = Counts()
    rc = lib().orc_render_profile(vp, vn, mp, mn, bp, bn, cam.ctypes.data, width, height, max_bounces,
                                  x0, y0, tw, th, row_step, rgba.ctypes.data, rad.ctypes.data, C.byref(c),
                                  n_threads, prof.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orc_render_profile failed ({rc})")
    return rgba, rad, c.as_dict(), prof
