import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "3d-ray-tracer-vulkan_amd")
for p in (PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"

# A Renderer that does not choose otherwise walks the reference's own tree
# (option accel 0, whose work counters are the oracle's own; rt_create reads
# RTAMD_ACCEL).  The default accel walk (SAH tree) runs in
# test_gpu_accel.py, in every test of test_gpu_parity.py (its module fixture
# runs each test on accel 8 and on accel 0) and in the tests of
# test_gpu_pipeline / test_gpu_dist / test_jni_shim parametrized over accel.
os.environ["RTAMD_ACCEL"] = "0"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """The native library under test is this tree's: its embedded build id
    (rt_build_id, read from the file) must carry the SHA-256 of the sources
    as they are here.  A library that is missing or built from other sources
    is rebuilt first (make is incremental); the oracle is built if missing."""
    import fcntl
    import subprocess
    from rtamd import _lib
    # one builder at a time (pytest -n: every worker runs this fixture; a
    # worker must not load a library another one is still writing)
    with open(os.path.join(ROOT, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not _lib.build_matches_tree() and "RTAMD_LIB_PATH" not in os.environ:
            subprocess.run(["make", "-j8", "-C", PKG_DIR], check=True)
        if "RTAMD_LIB_PATH" not in os.environ:
            assert _lib.build_matches_tree(), (f"{_lib.LIB_PATH}: build id {_lib.file_build_id()} does not "
                                               f"match the tree's sources (src={_lib.source_hash()})")
        # the oracle (test infrastructure) follows its sources (incremental)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
        # the JNI shim against the mock JNIEnv follows include/rtamd.h (incremental)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "jni"), "mock"], check=True,
                       stdout=subprocess.DEVNULL)
    print(f"\nlibrtamd build id: {_lib.file_build_id()} (tree src={_lib.source_hash()})")
    yield


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def renderer():
    if not has_gpu():
        pytest.skip("no GPU")
    import rtamd
    r = rtamd.Renderer((0,))
    yield r
    r.close()


def reference_path(*parts):
    p = os.path.join(REFERENCE, *parts)
    if not os.path.exists(p):
        pytest.skip("reference checkout not present")
    return p
