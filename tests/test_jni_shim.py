"""jni/HipNative.c executed: the JNI shim HipEngine.java calls, compiled against
a mock JNIEnv (tests/jni_mock: the JNI function table laid out by the
specification's indices, no JVM in this image) and driven through ctypes the
way the JVM drives it (VulkanEngine.java:120-185, 318-431 is what it
replaces).

CPU: create() on a machine without a GPU throws RuntimeException carrying
rt_last_error(); an error status from any call becomes a RuntimeException;
every Get*Elements / GetStringUTFChars is released.
GPU: uploadScene + render, renderAsync / pollFrame / waitFrame into a pinned
frame from allocFrame, setOption / getOption, uploadSpheres, through the shim
on config 2: bit-exact against the oracle.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT, has_gpu

MOCK = os.path.join(ROOT, "jni", "build", "libhipnative_mock.so")
PREFIX = "Java_dev_demir_vulkan_engine_HipNative_"


class JavaException(Exception):
    def __init__(self, cls, msg):
        super().__init__(f"{cls}: {msg}")
        self.cls, self.msg = cls, msg


class Jvm:
    """Calls HipNative's static natives as the JVM would: (JNIEnv*, jclass, args...)."""

    def __init__(self):
        import rtamd
        from rtamd._lib import LIB_PATH
        rtamd.lib()                                     # torch's HIP runtime first, then librtamd
        C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)            # the shim's rt_* symbols resolve against it
        if not os.path.exists(MOCK):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "jni"), "mock"], check=True)
        L = C.CDLL(MOCK)
        vp = C.c_void_p
        L.mock_env.restype = vp
        for name, args in (("mock_direct_buffer", [vp, C.c_int64]), ("mock_int_array", [vp, C.c_int32]),
                           ("mock_float_array", [vp, C.c_int32]), ("mock_string", [C.c_char_p]),
                           ("mock_heap_buffer", [])):
            getattr(L, name).restype = vp
            getattr(L, name).argtypes = args
        L.mock_buffer_address.restype = vp
        L.mock_buffer_address.argtypes = [vp]
        L.mock_buffer_capacity.restype = C.c_int64
        L.mock_buffer_capacity.argtypes = [vp]
        L.mock_take_exception.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        sig = {"create": (C.c_int64, [vp]), "uploadScene": (None, [C.c_int64, vp, C.c_int64, vp, C.c_int64, vp,
                                                                   C.c_int64]),
               "render": (None, [C.c_int64, vp, C.c_int32, C.c_int32, C.c_int32, vp]),
               "allocFrame": (vp, [C.c_int64]), "freeFrame": (None, [vp]),
               "renderAsync": (C.c_int64, [C.c_int64, vp, C.c_int32, C.c_int32, C.c_int32, vp]),
               "waitFrame": (None, [C.c_int64, C.c_int64]), "pollFrame": (C.c_uint8, [C.c_int64, C.c_int64]),
               "uploadSpheres": (None, [C.c_int64, vp]), "setOption": (None, [C.c_int64, vp, C.c_int64]),
               "getOption": (C.c_int64, [C.c_int64, vp]), "destroy": (None, [C.c_int64])}
        self.fn = {}
        for k, (res, args) in sig.items():
            f = getattr(L, PREFIX + k)
            f.restype = res
            f.argtypes = [vp, vp] + args
            self.fn[k] = f
        self.L = L
        self.env = L.mock_env()
        self._keep = []

    def call(self, name, *args):
        r = self.fn[name](self.env, None, *args)
        cls, msg = C.create_string_buffer(256), C.create_string_buffer(2048)
        if self.L.mock_take_exception(cls, 256, msg, 2048):
            raise JavaException(cls.value.decode(), msg.value.decode())
        return r

    # Java-side objects
    def direct(self, arr):
        self._keep.append(arr)
        return self.L.mock_direct_buffer(arr.ctypes.data, arr.nbytes)

    def ints(self, values):
        a = np.ascontiguousarray(values, dtype=np.int32)
        self._keep.append(a)
        return self.L.mock_int_array(a.ctypes.data, len(a))

    def floats(self, values):
        a = np.ascontiguousarray(values, dtype=np.float32).reshape(-1)
        self._keep.append(a)
        return self.L.mock_float_array(a.ctypes.data, len(a))

    def string(self, s):
        return self.L.mock_string(s.encode())


def test_mock_table_matches_jni_indices():
    """The mock header's typed entries sit at the JNI specification's indices
    (also asserted at compile time in jni_mock.c)."""
    import re
    text = open(os.path.join(ROOT, "tests", "jni_mock", "jni.h")).read()
    body = text[text.index("struct JNINativeInterface_ {"):]
    entries = re.findall(r"^\s+(.*?);", body, re.M)
    want = {"FindClass": 6, "ThrowNew": 14, "GetStringUTFChars": 169, "ReleaseStringUTFChars": 170,
            "GetArrayLength": 171, "GetIntArrayElements": 187, "GetFloatArrayElements": 189,
            "ReleaseIntArrayElements": 195, "ReleaseFloatArrayElements": 197, "NewDirectByteBuffer": 229,
            "GetDirectBufferAddress": 230}
    for name, idx in want.items():
        assert f"*{name})" in entries[idx], (name, idx, entries[idx])
    assert len(entries) == 233


@pytest.mark.skipif(has_gpu(), reason="the no-device path needs a machine without a GPU")
def test_create_without_device_throws_runtime_exception():
    from rtamd import lib
    jvm = Jvm()
    with pytest.raises(JavaException) as ei:
        jvm.call("create", jvm.ints([0]))
    assert ei.value.cls == "java/lang/RuntimeException"
    assert "rtamd error -2" in ei.value.msg
    assert lib().rt_last_error().decode() in ei.value.msg        # carries rt_last_error()
    assert "no HIP device" in ei.value.msg
    assert jvm.L.mock_outstanding() == 0                           # ReleaseIntArrayElements was called


def test_error_status_becomes_runtime_exception():
    """Every call with a bad context reports through RuntimeException, with the
    string and array elements released."""
    jvm = Jvm()
    with pytest.raises(JavaException, match="rtamd error -1: rt_get_option: null argument"):
        jvm.call("getOption", 0, jvm.string("walk"))
    with pytest.raises(JavaException, match="rt_set_option: null argument"):
        jvm.call("setOption", 0, jvm.string("walk"), 2)
    with pytest.raises(JavaException, match="rt_upload_spheres: null context"):
        jvm.call("uploadSpheres", 0, jvm.floats(np.zeros(8)))
    with pytest.raises(JavaException, match="rt_render_wait: null context"):
        jvm.call("waitFrame", 0, 1)
    with pytest.raises(JavaException, match="rt_render_poll: null argument"):
        jvm.call("pollFrame", 0, 1)
    with pytest.raises(JavaException, match="rt_upload_scene: null context"):
        jvm.call("uploadScene", 0, None, 0, None, 0, None, 0)
    assert jvm.L.mock_outstanding() == 0
    jvm.call("destroy", 0)                                         # destroy(0) is a no-op


@pytest.mark.gpu
@pytest.mark.parametrize("accel", [0, 8])
def test_shim_renders_config2_bit_exact(accel):
    if not has_gpu():
        pytest.skip("no GPU")
    from oracle import oracle_lib
    from rtamd import configs
    jvm = Jvm()
    cfg = configs.config2()
    built = cfg.build()
    W, H, B = 320, 180, cfg.max_bounces
    cam = configs.Camera.default(W, H)
    ref = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                            cam.ubo_bytes(), W, H, B, radiance=False)[0]
    ctx = jvm.call("create", jvm.ints([0]))
    assert ctx != 0
    try:
        v = np.ascontiguousarray(built.model_vertex_data, dtype=np.float32)
        m = np.ascontiguousarray(built.model_material_data, dtype=np.float32)
        b = np.ascontiguousarray(built.flat_bvh_data, dtype=np.uint8)
        jvm.call("setOption", ctx, jvm.string("accel"), accel)   # at the upload below
        # byte counts as VulkanEngine.java:337,345,353 computes them (remaining() * 4 / remaining())
        jvm.call("uploadScene", ctx, jvm.direct(v), v.size * 4, jvm.direct(m), m.size * 4, jvm.direct(b), b.size)
        ubo = np.frombuffer(cam.ubo_bytes(), dtype=np.uint8).copy()
        out = np.zeros((H, W, 4), np.uint8)
        jvm.call("render", ctx, jvm.direct(ubo), W, H, B, jvm.direct(out))
        assert np.array_equal(out, ref)
        # pipelined frames into pinned frames, as HipEngine.java's loop does
        assert jvm.call("getOption", ctx, jvm.string("async_slots")) == 4
        frames = [jvm.call("allocFrame", W * H * 4) for _ in range(4)]
        assert all(jvm.L.mock_buffer_capacity(f) == W * H * 4 for f in frames)
        views = [np.ctypeslib.as_array((C.c_uint8 * (W * H * 4)).from_address(jvm.L.mock_buffer_address(f)))
                 .reshape(H, W, 4) for f in frames]
        tickets = [jvm.call("renderAsync", ctx, jvm.direct(ubo), W, H, B, f) for f in frames]
        for t, view in zip(tickets, views):
            while not jvm.call("pollFrame", ctx, t):
                pass
            jvm.call("waitFrame", ctx, t)
            assert np.array_equal(view, ref)
        for f in frames:
            jvm.call("freeFrame", f)
        # a bad option value and a non-direct buffer surface as RuntimeException
        with pytest.raises(JavaException, match="unknown option or bad value"):
            jvm.call("setOption", ctx, jvm.string("async_slots"), 99)
        with pytest.raises(JavaException, match="rt_render: out_rgba is required"):
            jvm.call("render", ctx, jvm.direct(ubo), W, H, B, jvm.L.mock_heap_buffer())
        # the spheres extension through the shim
        jvm.call("uploadSpheres", ctx, jvm.floats([0.0, 5.0, 0.0, 4.0, 0.9, 0.2, 0.2, 0.0]))
        jvm.call("setOption", ctx, jvm.string("extensions"), 8)
        assert jvm.call("getOption", ctx, jvm.string("extensions")) == 8
        jvm.call("render", ctx, jvm.direct(ubo), W, H, B, jvm.direct(out))
        sph = np.array([[0.0, 5.0, 0.0, 4.0, 0.9, 0.2, 0.2, 0.0]], np.float32)
        ref_s = oracle_lib.render(built.model_vertex_data, built.model_material_data, built.flat_bvh_data,
                                  cam.ubo_bytes(), W, H, B, radiance=False, ext=oracle_lib.EXT_SPHERES,
                                  spheres=sph)[0]
        assert np.array_equal(out, ref_s)
        assert jvm.L.mock_outstanding() == 0
    finally:
        jvm.call("destroy", ctx)
