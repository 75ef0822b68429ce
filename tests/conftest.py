import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "3d-ray-tracer-vulkan_amd")
for p in (PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"

# The GPU suites test_gpu_parity / test_gpu_pipeline / test_gpu_dist / test_jni_shim
# pin the reference-order walk (option accel 0), whose work counters are the
# oracle's own, on every Renderer that does not choose otherwise (rt_create
# reads RTAMD_ACCEL).  The default accel walk (binned-SAH tree, DESIGN.md
# §4a) is tested by test_gpu_accel.py and by the tests below that set option
# accel themselves, against the same oracle frames.
os.environ["RTAMD_ACCEL"] = "0"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the native library and the oracle once (no GPU needed)."""
    import subprocess
    lib = os.path.join(PKG_DIR, "lib", "librtamd.so")
    olib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-j8", "-C", PKG_DIR], check=True)
    if not os.path.exists(olib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
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
