"""ctypes binding of the C ABI (include/rtamd.h) — the Python stand-in for the
JNI shim a Java host would use.

The library is the in-tree lib/librtamd.so built by __graft_entry__.build()
(or `make -C 3d-ray-tracer-vulkan_amd`).  There is no fallback: if it is
missing or fails to load, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RTAMD_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "librtamd.so")   # override: experiments

RT_OK = 0
RT_ERR = {
    -1: "RT_ERR_INVALID_ARG",
    -2: "RT_ERR_NO_DEVICE",
    -3: "RT_ERR_HIP",
    -4: "RT_ERR_BAD_SCENE",
    -5: "RT_ERR_NO_SCENE",
    -6: "RT_ERR_OOM",
    -7: "RT_ERR_IO",
}

# Every symbol include/rtamd.h declares (checked by tests/test_abi.py).
ABI_VERSION = 6           # include/rtamd.h RT_ABI_VERSION

EXPORTED = (
    "rt_create", "rt_upload_scene", "rt_render", "rt_render_tile_device", "rt_destroy",
    "rt_last_error", "rt_scene_info", "rt_bvh_layout_size", "rt_build_scene",
    "rt_camera_from_lookat", "rt_mesh_load_obj", "rt_mesh_tri_count", "rt_mesh_transform",
    "rt_mesh_free", "rt_mesh_procedural", "rt_render_bands_device", "rt_band_rows",
    "rt_scene_validate", "rt_set_option", "rt_get_option", "rt_diag_copy",
    "rt_host_alloc", "rt_host_free", "rt_render_async", "rt_render_wait", "rt_upload_spheres",
    "rt_render_batch_device", "rt_band_list_rows", "rt_render_batch_lists_device", "rt_band_lists_rows",
    "rt_render_poll", "rt_accel_records", "rt_abi_version", "rt_pack_rgb", "rt_unpack_rgb",
    "rt_build_id", "rt_render_batch_rect_device", "rt_render_batch_runs_device",
)

# The library's sources in the Makefile's SRC_ALL order: rt_build_id's
# "src=" field is the first 16 hex digits of SHA-256 over them concatenated.
BUILD_SOURCES = ("csrc/rt_trace.hip", "csrc/rt_runtime.hip", "csrc/rt_learn.hip", "csrc/rt_wire.hip",
                 "csrc/scene_build.cpp", "csrc/accel_build.cpp", "csrc/rt_internal.h", "csrc/accel_build.h",
                 "../include/rtamd.h")


def source_hash() -> str:
    """SHA-256 (16 hex digits) of the library's sources as they are in this tree."""
    import hashlib
    h = hashlib.sha256()
    for f in BUILD_SOURCES:
        with open(os.path.join(PKG_ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def file_build_id(path: str = LIB_PATH) -> str | None:
    """The build id embedded in a built library, read from the file (no load)."""
    import re
    try:
        with open(path, "rb") as fh:
            m = re.search(rb"RTAMD_BUILD_ID:(src=[0-9a-f]{16} git=[0-9a-z]+)", fh.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def build_matches_tree(path: str = LIB_PATH) -> bool:
    """True when the library at path was built from this tree's sources."""
    bid = file_build_id(path)
    return bid is not None and bid.startswith(f"src={source_hash()} ")


class RtError(RuntimeError):
    """A non-zero status from the C ABI (the JNI shim throws RuntimeException)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"{RT_ERR.get(code, code)}: {message}")
        self.code = code


class CameraUBO(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 4),
        ("lower_left", C.c_float * 4),
        ("horizontal", C.c_float * 4),
        ("vertical", C.c_float * 4),
        ("frame_count", C.c_int32),
        ("sky_enabled", C.c_int32),
        ("pad", C.c_int32 * 2),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("segments", C.c_uint64),
        ("node_visits", C.c_uint64),
        ("tri_tests", C.c_uint64),
        ("mat_reads", C.c_uint64),
        ("ms", C.c_double),
        ("pixels", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


assert C.sizeof(CameraUBO) == 80

_lock = threading.Lock()
_lib = None


def lib() -> C.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RtError(-3, f"{LIB_PATH} is missing: run __graft_entry__.build() "
                                  "(there is no non-HIP fallback)")
            # torch bundles its own libamdhip64.so.7 (same soname as ROCm's).  The
            # first one loaded serves the whole process, and torch only works
            # with its own; load it first so torch tensors and this library
            # share one HIP runtime.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            L = C.CDLL(LIB_PATH)
            vp, sz, i32, u64, dp, fp = C.c_void_p, C.c_size_t, C.c_int, C.c_uint64, C.POINTER(C.c_double), C.POINTER(C.c_float)
            sig = {
                "rt_create": (i32, [C.POINTER(C.c_int), i32, C.POINTER(vp)]),
                "rt_upload_scene": (i32, [vp, vp, sz, vp, sz, vp, sz]),
                "rt_upload_spheres": (i32, [vp, vp, i32]),
                "rt_render": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, vp, vp, C.POINTER(Stats)]),
                "rt_render_tile_device": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, i32, i32, i32, i32,
                                                vp, vp, vp, C.POINTER(Stats)]),
                "rt_destroy": (i32, [vp]),
                "rt_last_error": (C.c_char_p, []),
                "rt_scene_info": (i32, [vp, C.POINTER(sz), C.POINTER(sz), C.POINTER(i32)]),
                "rt_bvh_layout_size": (i32, [sz, C.POINTER(sz), C.POINTER(sz)]),
                "rt_build_scene": (i32, [dp, fp, sz, u64, i32, fp, fp, vp]),
                "rt_camera_from_lookat": (i32, [dp, dp, dp, C.c_double, C.c_double, C.POINTER(CameraUBO)]),
                "rt_mesh_load_obj": (i32, [C.c_char_p, C.POINTER(vp)]),
                "rt_mesh_tri_count": (sz, [vp]),
                "rt_mesh_transform": (i32, [vp, dp, dp, dp]),
                "rt_mesh_free": (i32, [vp]),
                "rt_mesh_procedural": (i32, [sz, u64, dp, dp, dp]),
                "rt_render_bands_device": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, i32, i32, i32,
                                                 vp, vp, vp, C.POINTER(Stats)]),
                "rt_band_rows": (i32, [i32, i32, i32, i32]),
                "rt_render_batch_device": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, i32, i32,
                                                 C.POINTER(C.c_int32), i32, vp, vp, vp, C.POINTER(Stats)]),
                "rt_band_list_rows": (i32, [i32, i32, C.POINTER(C.c_int32), i32]),
                "rt_render_batch_lists_device": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, i32, i32,
                                                       C.POINTER(C.c_int32), i32, vp, vp, vp, C.POINTER(Stats)]),
                "rt_band_lists_rows": (i32, [i32, i32, C.POINTER(C.c_int32), i32, i32]),
                "rt_render_batch_rect_device": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, i32, i32, i32, i32,
                                                      i32, vp, vp, vp, C.POINTER(Stats)]),
                "rt_render_batch_runs_device": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, i32, i32,
                                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32), vp, vp, vp,
                                                      C.POINTER(Stats)]),
                "rt_scene_validate": (i32, [vp, sz, vp, sz, vp, sz, C.POINTER(sz), C.POINTER(i32)]),
                "rt_set_option": (i32, [vp, C.c_char_p, C.c_int64]),
                "rt_get_option": (i32, [vp, C.c_char_p, C.POINTER(C.c_int64)]),
                "rt_diag_copy": (i32, [vp, vp, sz, C.POINTER(sz)]),
                "rt_host_alloc": (vp, [sz]),
                "rt_host_free": (None, [vp]),
                "rt_render_async": (i32, [vp, C.POINTER(CameraUBO), i32, i32, i32, vp, C.POINTER(u64)]),
                "rt_render_wait": (i32, [vp, u64]),
                "rt_render_poll": (i32, [vp, u64, C.POINTER(i32)]),
                "rt_accel_records": (i32, [vp, sz, vp, sz, vp, sz, i32, C.POINTER(C.c_uint32), sz, C.POINTER(sz),
                                           C.POINTER(C.c_int32)]),
                "rt_abi_version": (i32, [C.POINTER(sz), C.POINTER(sz)]),
                "rt_build_id": (C.c_char_p, []),
                "rt_pack_rgb": (i32, [vp, vp, sz, vp]),
                "rt_unpack_rgb": (i32, [vp, vp, sz, vp]),
            }
            for name, (res, args) in sig.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            # the structs this binding lays out must be the library's
            sb, cb = C.c_size_t(), C.c_size_t()
            ver = L.rt_abi_version(C.byref(sb), C.byref(cb))
            if ver != ABI_VERSION or sb.value != C.sizeof(Stats) or cb.value != C.sizeof(CameraUBO):
                raise RtError(-1, f"{LIB_PATH}: ABI version {ver} (rt_stats {sb.value} B, camera {cb.value} B); "
                                  f"this binding expects {ABI_VERSION} ({C.sizeof(Stats)} B, {C.sizeof(CameraUBO)} B)")
            _lib = L
        return _lib


def check(rc: int) -> None:
    if rc != RT_OK:
        msg = lib().rt_last_error()
        raise RtError(rc, msg.decode() if msg else "")


RT_ACCEL_FORMAT_HALF = 0x100
RT_ACCEL_FORMAT_WIDE = 0x200


def accel_records(built, n_layouts: int = 8, half: bool = False, wide: bool = False):
    """Option accel's records for a BuiltCpuData (rt_accel_records): returns
    (uint32[slots_total * 8] (half: * 4, option accel_half's format; wide: *
    16, option accel_wide's 64-B records), info dict).  Host-only; no device
    needed."""
    import numpy as np
    L = lib()
    bufs = [np.ascontiguousarray(np.frombuffer(bytes(x), dtype=np.uint8)) if isinstance(x, (bytes, bytearray))
            else np.ascontiguousarray(x) for x in (built.model_vertex_data, built.model_material_data,
                                                   built.flat_bvh_data)]
    args = []
    for b in bufs:
        args += [b.ctypes.data, b.nbytes]
    n = C.c_size_t(0)
    info = (C.c_int32 * 8)()
    nl = n_layouts | (RT_ACCEL_FORMAT_HALF if half else 0) | (RT_ACCEL_FORMAT_WIDE if wide else 0)
    check(L.rt_accel_records(*args, nl, None, 0, C.byref(n), info))
    out = np.zeros(n.value, dtype=np.uint32)
    check(L.rt_accel_records(*args, nl, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size, C.byref(n), info))
    keys = ("n_layouts", "slots", "root_leaf", "n_prims", "n_inputs", "depth", "max_class", "n_thin")
    d = dict(zip(keys, list(info)))
    d["format"] = 1 if half else (2 if wide else 0)
    return out, d
